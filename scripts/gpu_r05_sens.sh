#!/bin/bash
# Round-5 SM-G-SUM check (on the GPU box): the mutation GPU tests, then bench lines with --mutation SM-G-SUM,
# alternating an env switch (two settings, two reps) and a rocprofv3 kernel-trace of the default setting.
# usage: bash scripts/gpu_r05_sens.sh TAG [VAR "valA valB"]
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05sens}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests/test_gpu_mutations.py > $O/tests.log 2>&1
if [ -n "$2" ]; then
  for rep in 1 2; do
    for v in $3; do
      env $2=$v timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --mutation SM-G-SUM \
        > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err
    done
  done
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- \
  python3 bench.py --steps 6 --warmup 1 --no-cpu-baseline --mutation SM-G-SUM > $O/stats.log 2>&1
echo ok
