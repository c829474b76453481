set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/smgprof; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/st -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --mutation SM-G-SUM > $O/run.log 2>&1
echo ok
