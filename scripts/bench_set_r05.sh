#!/bin/bash
# The round's bench lines on one GPU (each step under its own time limit): the default line (the metric's
# pop=512 on one GPU, CPU baseline leg included), the per-GPU shapes of the metric at 2/4/8 GPUs
# (--population 256/128/64: what one rank of a strong-scaled run evaluates), configs[1] (pop=64),
# configs[3] and configs[4] (their whole populations on one GPU), B = 64 (mscoco_nes.json's batch_size)
# at P = 512 and 64, greedy_linprob, trained-like theta, 64 batches per iteration, SM-G-SUM / SM-PROPORTIONAL
# and the sampled fitness modes.
# usage (on the GPU box): bash scripts/bench_set_r05.sh TAG
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-benchset_r05}
mkdir -p $O
B="python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline"
timeout -k 10 400 python3 -u bench.py > $O/bench_default.json 2> $O/bench_default.err
for P in 256 128 64; do
  timeout -k 10 200 $B --population $P > $O/bench_pop$P.json 2> $O/bench_pop$P.err
done
timeout -k 10 300 $B --preset configs3 > $O/bench_configs3.json 2> $O/bench_configs3.err
timeout -k 10 200 $B --preset configs4 > $O/bench_configs4.json 2> $O/bench_configs4.err
timeout -k 10 200 $B --preset configs4 --population 64 > $O/bench_configs4_per_gpu.json 2> $O/bench_configs4_per_gpu.err
timeout -k 10 200 $B --batch 64 > $O/bench_b64.json 2> $O/bench_b64.err
timeout -k 10 200 $B --batch 64 --population 64 > $O/bench_p64_b64.json 2> $O/bench_p64_b64.err
timeout -k 10 200 $B --fitness greedy_linprob > $O/bench_linprob.json 2> $O/bench_linprob.err
timeout -k 10 200 $B --theta-gain 4 --bias-std 0.1 > $O/bench_trained_like_theta.json 2> $O/bench_trained_like_theta.err
timeout -k 10 300 $B --batches 64 > $O/bench_batches64.json 2> $O/bench_batches64.err
timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --mutation SM-G-SUM > $O/bench_smgsum.json 2> $O/bench_smgsum.err
for F in sample self_critical sc_loss; do
  timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --fitness $F > $O/bench_fitness_$F.json 2> $O/bench_fitness_$F.err
done
timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --fitness sample --theta-gain 4 --bias-std 0.1 > $O/bench_sample_trained_like.json 2> $O/bench_sample_trained_like.err
timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --mutation SM-PROPORTIONAL > $O/bench_smprop.json 2> $O/bench_smprop.err
echo done
