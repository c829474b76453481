#!/bin/bash
# Round-5 check of the final decode sources (on the GPU box): the whole GPU suite in one pytest process, then the
# default bench line and the bench at B = 64 (mscoco_nes.json's batch size, steps2) and at 64 members per GPU.
# usage: bash scripts/gpu_r05_final.sh TAG
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05final}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests > $O/tests.log 2>&1
timeout -k 10 300 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err
timeout -k 10 300 python -u bench.py --batch 64 --no-cpu-baseline > $O/bench_b64.json 2> $O/bench_b64.err
timeout -k 10 300 python -u bench.py --population 64 --no-cpu-baseline > $O/bench_p64.json 2> $O/bench_p64.err
echo ok
