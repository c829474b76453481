#!/bin/bash
# A/B of an engine env switch on the bench workload: the -m gpu suite (optional), then bench lines
# alternating the two settings. usage: bash scripts/gpu_ab.sh TAG VAR "valA valB" [tests|notests] [POP]
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-ab}
mkdir -p $O
if [ "${4:-tests}" = tests ]; then
  timeout -k 10 600 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests/ > $O/tests.log 2>&1
fi
P=${5:-512}
for rep in 1 2; do
  for v in $3; do
    env $2=$v timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --population $P \
      > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err
  done
done
echo ok
