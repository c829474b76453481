set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; mkdir -p $O
ABLATE_DIR=ablate_libs FITNESS=sample POP=512 ROUNDS=2 timeout -k 10 600 python -u scripts/ablate.py > $O/sample.log 2>&1
ABLATE_DIR=ablate_libs FITNESS=greedy POP=512 ROUNDS=2 timeout -k 10 600 python -u scripts/ablate.py > $O/greedy.log 2>&1
echo ok
