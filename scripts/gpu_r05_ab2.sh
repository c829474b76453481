#!/bin/bash
# Round-5 one-process A/B of the decode builds in ablate_libs/ at the coop shapes (P = 64, 128) and the sampled
# decode (P = 512). usage: bash scripts/gpu_r05_ab2.sh TAG [EXACT variants]
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05ab2}
mkdir -p $O
export ABLATE_DIR=ablate_libs EXACT=${2:-}
POP=64 ROUNDS=9 timeout -k 10 300 python -u scripts/ablate.py > $O/p64.log 2>&1
POP=128 ROUNDS=7 timeout -k 10 300 python -u scripts/ablate.py > $O/p128.log 2>&1
POP=512 FITNESS=sample ROUNDS=3 timeout -k 10 400 python -u scripts/ablate.py > $O/p512_sample.log 2>&1
echo ok
