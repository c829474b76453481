#!/bin/bash
# quick GPU check: parity tests (split + fused), bench P=512 and P=64, one SQ instruction-count pass
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-quick}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_split.py tests/test_gpu_parity.py tests/test_gpu_reference.py > $O/tests.log 2>&1
timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench512.json 2> $O/bench512.err
timeout -k 10 200 python -u bench.py --steps 20 --warmup 2 --pop-per-gpu 64 --no-cpu-baseline > $O/bench64.json 2> $O/bench64.err
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d $O/pmc -o run --output-format csv -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline > $O/pmc.log 2>&1
echo ok
