set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_split.py > gpurun_out/split_tests.log 2>&1 && \
timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench512.json 2> gpurun_out/bench512.err && \
timeout -k 10 200 python -u bench.py --steps 20 --warmup 2 --pop-per-gpu 64 --no-cpu-baseline > gpurun_out/bench64.json 2> gpurun_out/bench64.err && \
timeout -k 10 200 python -u bench.py --steps 20 --warmup 2 --pop-per-gpu 64 --batch 64 --no-cpu-baseline > gpurun_out/bench64_b64.json 2> gpurun_out/bench64_b64.err && \
timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --batch 64 --no-cpu-baseline > gpurun_out/bench512_b64.json 2> gpurun_out/bench512_b64.err
