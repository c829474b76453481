set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/sensdbg3; mkdir -p $O
for c in 5 4 2 0; do NICNES_SENS_CELL=$c timeout -k 10 400 python -u scripts/dev/debug_sens2.py 41 > $O/r41_c$c.log 2>&1; done
echo ok
