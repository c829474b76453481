#!/bin/bash
# dev: GPU suite + smoke + the P = 512 and P = 64 bench lines (each step under its own limit)
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-quick}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/ > $O/tests.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench512.json 2> $O/bench512.err
timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --pop-per-gpu 64 > $O/bench64.json 2> $O/bench64.err
echo ok
