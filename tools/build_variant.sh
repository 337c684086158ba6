#!/bin/bash
# Build a variant of the library with extra compile flags into abl/lib<name>.so
# (timing experiments, A/B runs through LATTICEUM_AMD_LIB): tools/build_variant.sh name -DFLAG ...
set -e
NAME=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
SRC=$ROOT/latticeum_amd/csrc
OUT=/tmp/lf_variant_$NAME
mkdir -p "$OUT" "$ROOT/abv"
SRCS="kernels.hip kernels_n32.hip kernels_n4k.hip ajtai_mfma.hip fold_coeff.hip sumcheck.hip mz.hip merkle.hip fold_prove.hip lf_api.hip transcript.cpp serialize.cpp replay.cpp"
pids=()
for f in $SRCS; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-pass-failed -Wno-unused-function "$@" \
    -c "$SRC/$f" -o "$OUT/$f.o" &
  pids+=($!)
done
for p in "${pids[@]}"; do wait "$p"; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$ROOT/abv/lib$NAME.so" "$OUT"/*.o
echo "abv/lib$NAME.so"
