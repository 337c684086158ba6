#!/bin/bash
# the host permutation on the box's CPU: AVX-512 vs scalar (equality + time), the
# library's absorb rate both ways, then a fold() trace on the scalar-valued CCS
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
/opt/rocm/bin/hipcc -O3 -std=c++17 -x hip --offload-arch=gfx950 --offload-host-only tools/exp/p2_avx_test.cpp \
  -o /tmp/p2avx -Llatticeum_amd -llatticeum_amd -Wl,-rpath,$GRAFT_REPO_ROOT/latticeum_amd && /tmp/p2avx
echo "library, AVX-512:"; python3 tools/exp/p2_absorb.py
echo "library, scalar:"; LATTICEUM_AMD_P2_SCALAR=1 python3 tools/exp/p2_absorb.py
