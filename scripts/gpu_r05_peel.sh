#!/bin/bash
# Round-5 A/B of two decode builds (base vs the others in ablate_libs/) over the bench shapes: P = 512 greedy,
# P = 512 sampled, B = 64 (steps2) and P = 64 (coop); timing-only harness scripts/ablate.py, one process each.
# usage: bash scripts/gpu_r05_peel.sh TAG [EXACT variants]
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05peel}
mkdir -p $O
export ABLATE_DIR=ablate_libs EXACT=${2:-}
POP=512 ROUNDS=5 timeout -k 10 300 python -u scripts/ablate.py > $O/p512.log 2>&1
POP=512 BATCH=64 ROUNDS=5 timeout -k 10 300 python -u scripts/ablate.py > $O/p512_b64.log 2>&1
POP=64 ROUNDS=7 timeout -k 10 300 python -u scripts/ablate.py > $O/p64.log 2>&1
POP=512 FITNESS=sample ROUNDS=3 timeout -k 10 400 python -u scripts/ablate.py > $O/p512_sample.log 2>&1
echo ok
