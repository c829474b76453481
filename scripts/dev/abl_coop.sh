set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/abl_coop; mkdir -p $O
EXACT=nohalf ABLATE_DIR=ablate_libs FITNESS=greedy POP=64 ROUNDS=6 timeout -k 10 300 python -u scripts/ablate.py > $O/p64.log 2>&1
EXACT=nohalf ABLATE_DIR=ablate_libs FITNESS=greedy POP=128 ROUNDS=6 timeout -k 10 300 python -u scripts/ablate.py > $O/p128.log 2>&1
timeout -k 10 400 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/test_gpu_coop.py tests/test_gpu_reference.py > $O/tests.log 2>&1
echo ok
