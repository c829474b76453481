set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/stage2
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --fitness sample > gpurun_out/stage2/bench_sample.json 2> gpurun_out/stage2/bench_sample.err
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --fitness sample --theta-gain 4 --bias-std 0.1 > gpurun_out/stage2/bench_sample_peaked.json 2> gpurun_out/stage2/bench_sample_peaked.err
bash scripts/profile_r03.sh stage2 "512" --fitness sample
echo ok
