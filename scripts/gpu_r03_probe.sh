#!/bin/bash
# Build and run the stage probe (scripts/stage_probe.hip) on the GPU box: the decode's 64-row stage
# structure alone, in its register-staged and LDS-DMA-staged forms.
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-probe}
mkdir -p $O
hipcc --offload-arch=gfx950 -O3 -w scripts/stage_probe.hip -o /tmp/stage_probe
timeout -k 10 90 /tmp/stage_probe > $O/probe.txt 2>&1
