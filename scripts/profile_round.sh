#!/bin/bash
# One GPU call: bench line + rocprofv3 kernel-trace stats of the same command + the two PMC
# passes (FETCH_SIZE, WRITE_SIZE) for the dominant (stage) kernel's HBM traffic, post-processed. Outputs under gpurun_out/.
# usage (on the GPU box): bash scripts/profile_round.sh TAG
set -eo pipefail
TAG=${1:-r01}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -rf gpurun_out/prof_stats_$TAG gpurun_out/prof_fetch_$TAG gpurun_out/prof_write_$TAG
timeout -k 10 400 python bench.py --steps 10 --warmup 2 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_stats_$TAG -o run --output-format csv -- \
    python3 bench.py --steps 10 --warmup 2 > gpurun_out/prof_stats_$TAG.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_fetch_$TAG -o run --output-format csv -- \
    python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline > gpurun_out/prof_fetch_$TAG.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_write_$TAG -o run --output-format csv -- \
    python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline > gpurun_out/prof_write_$TAG.log 2>&1
python scripts/trace_summary.py --trace gpurun_out/prof_stats_$TAG --command "python3 bench.py --steps 10 --warmup 2" \
    --out gpurun_out/decode_launches_$TAG.json > /dev/null
python scripts/pmc_traffic.py --fetch gpurun_out/prof_fetch_$TAG --write gpurun_out/prof_write_$TAG \
    --kernel nicnes_decode_step_kernel --out gpurun_out/decode_pmc_$TAG.json > /dev/null
echo done
