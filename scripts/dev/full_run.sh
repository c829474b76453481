set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/full1; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_default.json 2> $O/bench_default.err
timeout -k 10 200 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --fitness sample > $O/bench_sample.json 2> $O/bench_sample.err
timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --mutation SM-G-SUM > $O/bench_smg.json 2> $O/bench_smg.err
echo ok
