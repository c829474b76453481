#!/bin/bash
# The round's bench lines on one GPU (each step under its own time limit):
#   default (bench.py with no flags: P = 512, B = 128, CPU baseline leg included),
#   P = 64 (split decode), B = 64 at P = 512 and P = 64 (64-row slabs), 'bu' features, greedy_linprob,
#   and the per-GPU shapes of configs[3] (P = 256) and configs[4] (P = 64, bu).
# usage (on the GPU box): bash scripts/bench_set.sh TAG
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-benchset}
mkdir -p $O
timeout -k 10 400 python3 -u bench.py > $O/bench_default.json 2> $O/bench_default.err
timeout -k 10 200 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --pop-per-gpu 64 > $O/bench_p64.json 2> $O/bench_p64.err
timeout -k 10 200 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --batch 64 > $O/bench_b64.json 2> $O/bench_b64.err
timeout -k 10 200 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --pop-per-gpu 64 --batch 64 > $O/bench_p64_b64.json 2> $O/bench_p64_b64.err
timeout -k 10 200 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --bu > $O/bench_bu.json 2> $O/bench_bu.err
timeout -k 10 200 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --fitness greedy_linprob > $O/bench_linprob.json 2> $O/bench_linprob.err
# per-GPU shapes of the multi-GPU configs: configs[3] pop=2048 / 8 GPUs, configs[4] bu pop=512 / 8 GPUs
timeout -k 10 200 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --pop-per-gpu 256 > $O/bench_p256.json 2> $O/bench_p256.err
timeout -k 10 200 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --pop-per-gpu 64 --bu > $O/bench_p64_bu.json 2> $O/bench_p64_bu.err
# peaked, trained-like logits (theta gain 4, bias std 0.1): the adaptive bounded-lse policy
timeout -k 10 200 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --theta-gain 4 --bias-std 0.1 > $O/bench_trained_like_theta.json 2> $O/bench_trained_like_theta.err
# single_batch: false (mscoco_nes.json's default): 64 distinct batches, member i on batch i mod 64
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --batches 64 > $O/bench_batches64.json 2> $O/bench_batches64.err
echo done
