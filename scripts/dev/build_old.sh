#!/bin/bash
# Builds build/ablate/libnicnes_old.so from the committed (HEAD or $1) decode kernel + math header,
# linked with the current non-decode objects, for interleaved A/B timing with scripts/ablate.py.
set -e
REV=${1:-HEAD}
cd "$(dirname "$0")/../nes-img-captioning_amd"
mkdir -p build/ablate/x/y build/ablate/include
git show $REV:nes-img-captioning_amd/csrc/decode_kernel.hip > build/ablate/x/y/decode_old.hip
git show $REV:nes-img-captioning_amd/csrc/decode_kernel.h > build/ablate/x/y/decode_kernel.h
git show $REV:include/nicnes_math.h > build/ablate/include/nicnes_math.h
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -x hip -c build/ablate/x/y/decode_old.hip -o build/ablate/decode_old.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o build/ablate/libnicnes_old.so build/ablate/decode_old.o build/cider_kernel.hip.o build/update_kernels.hip.o build/engine.cpp.o
