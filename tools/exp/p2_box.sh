#!/bin/bash
# host Poseidon2 permutation variants timed on the GPU box's CPU (no GPU use)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
lscpu | grep -E "Model name|^CPU\(s\)|MHz|Flags" | cut -c1-300 > gpurun_out/lscpu.txt
/opt/rocm/bin/hipcc -O3 -std=c++17 -Ilatticeum_amd/csrc tools/exp/p2_variants.cpp -o /tmp/p2v 2>/dev/null && /tmp/p2v
/opt/rocm/bin/hipcc -O3 -march=native -std=c++17 -Ilatticeum_amd/csrc tools/exp/p2_variants.cpp -o /tmp/p2n 2>/dev/null && echo native && /tmp/p2n
cat gpurun_out/lscpu.txt
python3 tools/exp/p2_absorb.py
