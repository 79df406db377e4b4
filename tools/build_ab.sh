#!/bin/bash
# Build one A/B variant of the library: engine.hip recompiled with extra
# compiler flags (e.g. -DLDPC_AB_V2C_ST=16), linked with the in-tree objects of
# the other sources, into ab_lib/libldpc_amd_<name>.so (git-ignored) for
# tools/gpu_ab_lib.sh.  Run `make -C dna-ldpc-codes_amd` first.
#   usage: tools/build_ab.sh <name> [hipcc flags...]
set -euo pipefail
name=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
P=$R/dna-ldpc-codes_amd
mkdir -p "$R/build_ab/$name" "$R/ab_lib"
HIPFLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -Wall -Wno-unused-function -Wno-unused-result -Wno-unused-value"
/opt/rocm/bin/hipcc $HIPFLAGS "$@" -c -o "$R/build_ab/$name/engine.o" "$P/csrc/engine.hip"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$R/ab_lib/libldpc_amd_$name.so" "$R/build_ab/$name/engine.o" \
    "$P/build/capi.o" "$P/build/graph.o" "$P/build/dna.o" "$P/build/dna_io.o" "$P/build/host_simd.o" -lpthread
echo "ab_lib/libldpc_amd_$name.so"
