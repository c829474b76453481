#!/bin/bash
# Round-5 end check (on the GPU box): the whole GPU suite in one pytest process, then the default bench line.
# usage: bash scripts/gpu_r05_end.sh TAG
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05end}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread tests > $O/tests.log 2>&1
timeout -k 10 300 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err
echo ok
