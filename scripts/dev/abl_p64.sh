set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/abl64; mkdir -p $O
ABLATE_DIR=ablate_libs FITNESS=greedy POP=64 ROUNDS=6 timeout -k 10 300 python -u scripts/ablate.py > $O/p64.log 2>&1
ABLATE_DIR=ablate_libs FITNESS=greedy POP=512 ROUNDS=3 timeout -k 10 300 python -u scripts/ablate.py > $O/p512.log 2>&1
echo ok
