set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ldsl1; mkdir -p $O
timeout -k 10 300 python -u scripts/dev/debug_sample_fb.py 512 > $O/fb.log 2>&1
timeout -k 10 400 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/test_gpu_sample.py tests/test_gpu_faults.py > $O/tests.log 2>&1
ABLATE_DIR=ablate_libs FITNESS=sample POP=512 ROUNDS=4 timeout -k 10 600 python -u scripts/ablate.py > $O/ablate.log 2>&1
echo ok
