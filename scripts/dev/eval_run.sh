set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/evalt; mkdir -p $O
timeout -k 10 400 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests/test_gpu_eval_theta.py tests/test_gpu_faults.py tests/test_gpu_sample.py > $O/tests.log 2>&1
echo ok
