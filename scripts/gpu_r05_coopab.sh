#!/bin/bash
# Round-5 one-process A/B of the decode builds in ablate_libs/ at the coop shapes (P = 64, 128) and the split
# path (P = 64, B = 64). usage: bash scripts/gpu_r05_coopab.sh TAG [EXACT variants]
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05coopab}
mkdir -p $O
export ABLATE_DIR=ablate_libs EXACT=${2:-}
POP=64 ROUNDS=11 timeout -k 10 300 python -u scripts/ablate.py > $O/p64.log 2>&1
POP=128 ROUNDS=9 timeout -k 10 300 python -u scripts/ablate.py > $O/p128.log 2>&1
POP=64 BATCH=64 ROUNDS=11 timeout -k 10 300 python -u scripts/ablate.py > $O/p64_b64.log 2>&1
echo ok
