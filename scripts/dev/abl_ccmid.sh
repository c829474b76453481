set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ccmid; mkdir -p $O
EXACT=ccmid ABLATE_DIR=ablate_libs FITNESS=greedy POP=64 ROUNDS=10 timeout -k 10 300 python -u scripts/ablate.py > $O/p64.log 2>&1
EXACT=ccmid ABLATE_DIR=ablate_libs FITNESS=greedy POP=128 ROUNDS=10 timeout -k 10 300 python -u scripts/ablate.py > $O/p128.log 2>&1
echo ok
