#!/bin/bash
# Round-4 GPU check: the named test files (one pytest process), then an optional A/B of an engine env switch
# on bench lines at one population (alternating, two reps).
# usage (on the GPU box): bash scripts/gpu_r04.sh TAG "tests/test_a.py ..." [VAR "valA valB" POP]
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r04}
mkdir -p $O
if [ -n "$2" ]; then
  timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread $2 > $O/tests.log 2>&1
fi
if [ -n "$3" ]; then
  for rep in 1 2; do
    for v in $4; do
      env $3=$v timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --population ${5:-512} \
        > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err
    done
  done
fi
echo ok
