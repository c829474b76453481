#!/bin/bash
# Round-3 quick GPU check: the named test files (one pytest process), then bench lines at the given
# populations (strong scaling shapes on one GPU). Each step has its own time limit.
# usage (on the GPU box): bash scripts/gpu_r03_quick.sh TAG "tests/test_a.py tests/test_b.py" "64 128"
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-quick}
mkdir -p $O
if [ -n "$2" ]; then
  timeout -k 10 600 python -u -m pytest -m gpu -x -v --timeout 120 --timeout-method thread $2 > $O/tests.log 2>&1
fi
for P in $3; do
  timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --population $P > $O/bench_pop$P.json 2> $O/bench_pop$P.err
done
echo ok
