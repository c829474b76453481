#!/bin/bash
# Round-3 GPU run: the -m gpu suite, smoke, and the strong-scaling bench shapes on one GPU
# (P = 512 split over N = 1/2/4/8 GPUs gives 512/256/128/64 members per GPU), then a 2-rank
# torchrun rehearsal of the N > 1 path (gloo, both ranks on cuda:0). Each step has its own limit.
# usage (on the GPU box): bash scripts/gpu_r03.sh TAG [tests|notests]
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r03}
mkdir -p $O
if [ "${2:-tests}" = tests ]; then
  timeout -k 10 600 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests/ > $O/tests.log 2>&1
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
fi
for P in 512 256 128 64; do
  timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --population $P > $O/bench_pop$P.json 2> $O/bench_pop$P.err
done
timeout -k 10 200 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --preset configs3 > $O/bench_configs3.json 2> $O/bench_configs3.err
NICNES_BENCH_BACKEND=gloo NICNES_BENCH_SHARE_GPU=1 timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 5 --warmup 1 \
  --no-cpu-baseline > $O/bench_2rank_shared.json 2> $O/bench_2rank_shared.err
echo ok
