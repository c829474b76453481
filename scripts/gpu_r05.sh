#!/bin/bash
# Round-5 GPU check (on the GPU box): the GPU tests (all, or the named files) in one pytest process, then
# the default bench line and the launcher's own 2-rank line (both ranks time-sharing cuda:0 over gloo).
# usage: bash scripts/gpu_r05.sh TAG ["tests/test_a.py ..." | all | none] [bench|nobench]
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05}
mkdir -p $O
T=${2:-all}
if [ "$T" = all ]; then T=tests; fi
if [ "$T" != none ]; then
  timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread $T > $O/tests.log 2>&1
fi
if [ "${3:-bench}" = bench ]; then
  timeout -k 10 300 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err
  NICNES_BENCH_SHARE_GPU=1 NICNES_BENCH_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 2 --steps 10 \
    --warmup 2 > $O/bench_2rank_shared.json 2> $O/bench_2rank_shared.err
fi
echo ok
