set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; mkdir -p $O
EXACT=${EXACT:-} ABLATE_DIR=ablate_libs FITNESS=${2:-greedy} POP=${3:-512} ROUNDS=${4:-3} timeout -k 10 300 python -u scripts/ablate.py > $O/ablate.log 2>&1
echo ok
