set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 300 python -u scripts/dev/debug_sens.py 41 > $O/dbg41.log 2>&1
timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests/test_gpu_mutations.py tests/test_gpu_split.py tests/test_gpu_coop.py > $O/tests.log 2>&1
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --mutation SM-G-SUM > $O/bench_smgsum.json 2> $O/bench_smgsum.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --mutation SM-G-SUM > $O/stats.log 2>&1
timeout -k 10 400 python -u scripts/dev/debug_sample_fb.py 512 > $O/fb512.log 2>&1
echo ok
