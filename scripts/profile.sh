#!/bin/bash
# Profile set of one GPU call: rocprofv3 kernel-trace stats of the bench at each population on one GPU
# (the strong-scaling shapes: P = 512 fused steps kernel, P = 128 / 64 coop kernel), then per P four PMC
# passes (each within the per-pass slot limits of MI355X_MICROARCH.md: <= 8 SQ, <= 2 GRBM, FETCH_SIZE /
# WRITE_SIZE alone). Raw CSVs go to gpurun_out/<TAG>/; scripts/make_profiles.py post-processes them.
# usage (on the GPU box): bash scripts/profile.sh TAG "512 128 64" [extra bench args]
set -eo pipefail
TAG=${1:-r03}
PS=${2:-"512 128 64"}
shift 2 || true
EXTRA="$*"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
for P in $PS; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats$P -o run --output-format csv -- \
      python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --population $P $EXTRA > $O/stats$P.log 2>&1
  i=0
  for C in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
    timeout -s KILL 120 rocprofv3 --pmc $C -d $O/pmc${P}_$i -o run --output-format csv -- \
        python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline --population $P $EXTRA > $O/pmc${P}_$i.log 2>&1
    i=$((i+1))
  done
done
echo done
