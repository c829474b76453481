set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/cider; mkdir -p $O
timeout -k 10 300 python -u scripts/dev/cider_ab.py ablate_libs 512 8 > $O/p512.log 2>&1
timeout -k 10 300 python -u scripts/dev/cider_ab.py ablate_libs 64 8 > $O/p64.log 2>&1
echo ok
