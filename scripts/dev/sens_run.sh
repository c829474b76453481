set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests/test_gpu_mutations.py > $O/tests.log 2>&1
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --mutation SM-G-SUM > $O/bench_smgsum.json 2> $O/bench_smgsum.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --mutation SM-G-SUM > $O/stats.log 2>&1
EXACT=nt,sc1,ntsc1 ABLATE_DIR=ablate_libs FITNESS=sample POP=512 ROUNDS=3 timeout -k 10 600 python -u scripts/ablate.py > $O/ablate.log 2>&1
echo ok
