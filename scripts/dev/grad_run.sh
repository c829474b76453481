set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/grad; mkdir -p $O
timeout -k 10 400 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_faults.py tests/test_gpu_mutations.py tests/test_gpu_reference.py tests/test_gpu_fullsize.py tests/test_gpu_properties.py tests/test_gpu_master.py > $O/tests.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/st -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench.json 2> $O/bench.err
echo ok
