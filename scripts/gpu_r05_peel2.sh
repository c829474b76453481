set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05peel2; mkdir -p $O
export ABLATE_DIR=ablate_libs EXACT=peel2
POP=512 ROUNDS=7 timeout -k 10 300 python -u scripts/ablate.py > $O/p512.log 2>&1
POP=512 BATCH=64 ROUNDS=7 timeout -k 10 300 python -u scripts/ablate.py > $O/p512_b64.log 2>&1
echo ok
