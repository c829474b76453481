# dev: GPU suite on the default build, then the ablation builds timed in one process
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-exp}
mkdir -p $O
if [ "${SKIP_TESTS:-0}" != 1 ]; then
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/ > $O/tests.log 2>&1
fi
EXACT=${EXACT:-} ROUNDS=${ROUNDS:-5} timeout -k 10 500 python -u scripts/ablate.py > $O/ablate.log 2>&1
echo done
