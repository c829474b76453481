set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/stage1
timeout -k 10 300 python -u scripts/dev/debug_sample_stage.py > gpurun_out/stage1/debug.log 2>&1
timeout -k 10 600 python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread tests/test_gpu_sample.py > gpurun_out/stage1/tests.log 2>&1
echo done
