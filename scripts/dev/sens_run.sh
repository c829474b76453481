set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 300 python -u scripts/dev/debug_sens.py 41 > $O/dbg41.log 2>&1
timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests/test_gpu_mutations.py tests/test_gpu_sample.py tests/test_gpu_faults.py > $O/tests.log 2>&1
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --mutation SM-G-SUM > $O/bench_smgsum.json 2> $O/bench_smgsum.err
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --fitness sample > $O/bench_sample.json 2> $O/bench_sample.err
echo ok
