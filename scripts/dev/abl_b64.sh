set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ablb64; mkdir -p $O
ABLATE_DIR=ablate_libs FITNESS=greedy POP=512 BATCH=64 ROUNDS=4 timeout -k 10 300 python -u scripts/ablate.py > $O/b64.log 2>&1
echo ok
