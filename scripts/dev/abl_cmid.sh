set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/cmid; mkdir -p $O
EXACT=cmid ABLATE_DIR=ablate_libs FITNESS=greedy POP=512 ROUNDS=5 timeout -k 10 300 python -u scripts/ablate.py > $O/g512.log 2>&1
EXACT=cmid ABLATE_DIR=ablate_libs FITNESS=sample POP=512 ROUNDS=3 timeout -k 10 400 python -u scripts/ablate.py > $O/s512.log 2>&1
echo ok
