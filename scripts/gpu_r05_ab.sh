#!/bin/bash
# Round-5 one-process A/B of the decode builds in ablate_libs/ (make -C nes-img-captioning_amd ablate ABL=..., then
# copied there; base first) over the named shapes, one scripts/ablate.py process per shape:
#   512 (P = 512 greedy, the steps kernel)   512b64 (P = 512, B = 64: steps2)   64 / 128 (the coop kernel)
#   64b64 (the split path)                   512s (P = 512 sampled)
# usage (on the GPU box): bash scripts/gpu_r05_ab.sh TAG "SHAPES" [EXACT variants] [ROUNDS]
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05ab}
mkdir -p $O
export ABLATE_DIR=ablate_libs EXACT=${3:-}
R=${4:-7}
for sh in ${2:-512}; do
  case $sh in
    512)    POP=512 ROUNDS=$R timeout -k 10 300 python -u scripts/ablate.py > $O/p512.log 2>&1 ;;
    512b64) POP=512 BATCH=64 ROUNDS=$R timeout -k 10 300 python -u scripts/ablate.py > $O/p512_b64.log 2>&1 ;;
    64)     POP=64 ROUNDS=$((R + 4)) timeout -k 10 300 python -u scripts/ablate.py > $O/p64.log 2>&1 ;;
    128)    POP=128 ROUNDS=$((R + 2)) timeout -k 10 300 python -u scripts/ablate.py > $O/p128.log 2>&1 ;;
    64b64)  POP=64 BATCH=64 ROUNDS=$((R + 4)) timeout -k 10 300 python -u scripts/ablate.py > $O/p64_b64.log 2>&1 ;;
    512s)   POP=512 FITNESS=sample ROUNDS=3 timeout -k 10 400 python -u scripts/ablate.py > $O/p512_sample.log 2>&1 ;;
    *) echo "unknown shape $sh"; exit 2 ;;
  esac
done
echo ok
