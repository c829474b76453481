set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/smg2; mkdir -p $O
timeout -k 10 400 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests/test_gpu_mutations.py > $O/tests.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/st -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --mutation SM-G-SUM > $O/bench.json 2> $O/bench.err
echo ok
