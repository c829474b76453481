#!/bin/bash
# Round-5 decode ablation (on the GPU box): timing-only builds of the decode kernel (make -C nes-img-captioning_amd
# ablate ABL=..., copied to ablate_libs/) interleaved in one process by scripts/ablate.py.
# usage: bash scripts/gpu_r05_abl.sh TAG POP [EXACT variants] [ROUNDS]
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05abl}
mkdir -p $O
ABLATE_DIR=ablate_libs POP=${2:-64} EXACT=${3:-} ROUNDS=${4:-5} timeout -k 10 600 python -u scripts/ablate.py > $O/ablate.log 2>&1
echo ok
