#!/bin/bash
# Round-5 kernel-time A/B of whole libraries (for kernels outside the decode, which scripts/ablate.py does not time):
# rocprofv3 kernel-trace stats of the bench with each library in ablate_libs/ copied over the product library
# in turn (this box's copy of the tree only), alternating A B A B.
# usage (on the GPU box): bash scripts/gpu_r05_libstats.sh TAG "base nopar" [POP] [ROUNDS] [extra bench args]
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05ls}
mkdir -p $O
LIB=nes-img-captioning_amd/nicnes/libnicnes.so
for r in $(seq 1 ${4:-2}); do
  for v in ${2:-base}; do
    cp ablate_libs/libnicnes_$v.so $LIB
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${v}_$r -o run --output-format csv -- \
        python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --population ${3:-512} ${5:-} > $O/${v}_$r.log 2>&1
  done
done
echo ok
