#!/bin/bash
# One parameterised driver for the GPU-box runs (replaces round 5's scripts/gpu_r05_*.sh one-offs). Every GPU step
# runs under its own time limit and the script stops at the first failure (set -e), so a faulted or hung step
# ends the call. Output goes to gpurun_out/TAG/.
#
# usage (on the GPU box): bash scripts/gpu.sh TAG ACTION [args...]
#   tests   [FILES|all]             the GPU suite (or the named files) in one pytest process -> tests.log
#   bench   [bench.py args...]      one bench line -> bench.json / bench.err
#   rehearse                        the launcher's own 2-rank line, both ranks time-sharing cuda:0 over gloo
#   benchset                        the round's set of bench lines (the metric, the per-GPU shares, configs, modes)
#   ab      "SHAPES" [EXACT] [R]    one-process A/B of the decode builds in ablate_libs/ (scripts/ablate.py) per shape:
#                                   512 512b64 64 128 64b64 512s
#   libstats "VARIANTS" [POP] [R] [bench args]   rocprofv3 kernel stats of the bench with each ablate_libs/ library
#   benchab "VARIANTS" R NAME [bench args]   bench lines with each ablate_libs/ library, R interleaved rounds
#   prof    "POPS" [bench args]     kernel-trace stats + PMC passes (scripts/profile.sh)
#   stats   NAME [bench args]       one rocprofv3 --kernel-trace --stats pass of a bench line
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:?TAG}
ACT=${2:?ACTION}
shift 2
O=gpurun_out/$TAG
mkdir -p $O
B="python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline"
case $ACT in
  tests)
    T=${1:-all}
    if [ "$T" = all ]; then T=tests; fi
    timeout -k 10 1100 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread $T > $O/tests.log 2>&1 ;;
  bench)
    timeout -k 10 400 python3 -u bench.py "$@" > $O/bench.json 2> $O/bench.err ;;
  rehearse)
    NICNES_BENCH_SHARE_GPU=1 NICNES_BENCH_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 2 --steps 10 \
      --warmup 2 > $O/bench_2rank_shared.json 2> $O/bench_2rank_shared.err ;;
  benchset)
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
    timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --mutation SM-G-SUM > $O/bench_smgsum.json 2> $O/bench_smgsum.err
    timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --mutation SM-PROPORTIONAL > $O/bench_smprop.json 2> $O/bench_smprop.err
    for F in sample self_critical sc_loss; do
      timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --fitness $F > $O/bench_fitness_$F.json 2> $O/bench_fitness_$F.err
    done
    timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --fitness sample --theta-gain 4 \
      --bias-std 0.1 > $O/bench_sample_trained_like.json 2> $O/bench_sample_trained_like.err ;;
  ab)
    export ABLATE_DIR=ablate_libs EXACT=${2:-}
    R=${3:-7}
    for sh in ${1:-512}; do
      case $sh in
        512)    POP=512 ROUNDS=$R timeout -k 10 300 python -u scripts/ablate.py > $O/p512.log 2>&1 ;;
        512b64) POP=512 BATCH=64 ROUNDS=$R timeout -k 10 300 python -u scripts/ablate.py > $O/p512_b64.log 2>&1 ;;
        64)     POP=64 ROUNDS=$((R + 4)) timeout -k 10 300 python -u scripts/ablate.py > $O/p64.log 2>&1 ;;
        128)    POP=128 ROUNDS=$((R + 2)) timeout -k 10 300 python -u scripts/ablate.py > $O/p128.log 2>&1 ;;
        64b64)  POP=64 BATCH=64 ROUNDS=$((R + 4)) timeout -k 10 300 python -u scripts/ablate.py > $O/p64_b64.log 2>&1 ;;
        512s)   POP=512 FITNESS=sample ROUNDS=3 timeout -k 10 400 python -u scripts/ablate.py > $O/p512_sample.log 2>&1 ;;
        *) echo "unknown shape $sh"; exit 2 ;;
      esac
    done ;;
  libstats)
    LIB=nes-img-captioning_amd/nicnes/libnicnes.so
    V=${1:-base}; POP=${2:-512}; R=${3:-2}; shift 3 || shift $#
    for r in $(seq 1 $R); do
      for v in $V; do
        cp ablate_libs/libnicnes_$v.so $LIB
        timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${v}_$r -o run --output-format csv -- \
          python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --population $POP "$@" > $O/${v}_$r.log 2>&1
      done
    done ;;
  prof)
    POPS=${1:?POPS}; shift
    bash scripts/profile.sh $TAG "$POPS" "$@" ;;
  benchab)
    # bench lines of each ablate_libs/ library in turn, R interleaved rounds; NAME tags the workload
    LIB=nes-img-captioning_amd/nicnes/libnicnes.so
    V=${1:?VARIANTS}; R=${2:-2}; N=${3:?NAME}; shift 3
    cp $LIB $O/product_lib.so
    for r in $(seq 1 $R); do
      for v in $V; do
        cp ablate_libs/libnicnes_$v.so $LIB
        timeout -k 10 200 $B "$@" > $O/${N}_${v}_$r.json 2> $O/${N}_${v}_$r.err
      done
    done
    cp $O/product_lib.so $LIB && rm $O/product_lib.so ;;
  stats)
    N=${1:?NAME}; shift
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$N -o run --output-format csv -- \
      python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline "$@" > $O/$N.json 2> $O/$N.err ;;
  *) echo "unknown action $ACT"; exit 2 ;;
esac
echo ok
