set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/cmid2; mkdir -p $O
EXACT=cmid ABLATE_DIR=ablate_libs FITNESS=greedy POP=512 ROUNDS=10 timeout -k 10 300 python -u scripts/ablate.py > $O/g512.log 2>&1
EXACT=cmid ABLATE_DIR=ablate_libs FITNESS=greedy POP=256 ROUNDS=10 timeout -k 10 300 python -u scripts/ablate.py > $O/g256.log 2>&1
EXACT=cmid ABLATE_DIR=ablate_libs FITNESS=greedy_linprob POP=512 ROUNDS=6 timeout -k 10 300 python -u scripts/ablate.py > $O/lp512.log 2>&1
echo ok
