#!/bin/bash
# Round-5 one-process A/B of the decode builds in ablate_libs/ at the greedy shapes (P = 512 and B = 64).
# usage: bash scripts/gpu_r05_ab.sh TAG [EXACT variants] [ROUNDS]
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05ab}
mkdir -p $O
export ABLATE_DIR=ablate_libs EXACT=${2:-}
POP=512 ROUNDS=${3:-7} timeout -k 10 300 python -u scripts/ablate.py > $O/p512.log 2>&1
POP=512 BATCH=64 ROUNDS=${3:-7} timeout -k 10 300 python -u scripts/ablate.py > $O/p512_b64.log 2>&1
echo ok
