#!/bin/bash
# Round-5 check of the per-iteration small kernels (on the GPU box): the update/rank GPU tests, then a
# kernel-trace profile of the P = 64 and P = 512 benches (per-kernel averages under rocprofv3 --stats).
# usage: bash scripts/gpu_r05_small.sh TAG ["tests/test_a.py ..." | none]
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05small}
mkdir -p $O
T=${2:-"tests/test_gpu_parity.py tests/test_gpu_master.py tests/test_gpu_faults.py tests/test_gpu_reference.py"}
if [ "$T" != none ]; then
  timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread $T > $O/tests.log 2>&1
fi
for P in 64 512; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p$P -o run -- python3 bench.py --population $P --steps 10 \
    --warmup 2 --no-cpu-baseline > $O/bench_p$P.json 2> $O/bench_p$P.err
done
echo ok
