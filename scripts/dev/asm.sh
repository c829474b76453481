#!/bin/bash
# dev: device assembly of the decode kernels (in-tree sources) -> $1 (default /tmp/decode.s)
OUT=${1:-/tmp/decode.s}
cd "$(dirname "$0")/../../nes-img-captioning_amd" && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 \
  -ffp-contract=off -x hip -c csrc/decode_kernel.hip --cuda-device-only -S -o "$OUT" ${EXTRA_FLAGS}
