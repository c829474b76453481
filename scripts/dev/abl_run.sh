set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$1
EXACT=${EXACT:-} ABLATE_DIR=ablate_libs FITNESS=${2:-sample} POP=${3:-512} ROUNDS=${4:-3} timeout -k 10 600 python -u scripts/ablate.py > gpurun_out/$1/ablate.log 2>&1
echo ok
