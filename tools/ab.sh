#!/bin/bash
# A/B timing on one box: alternate bench runs of ab/lib*.so builds (names as args)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-}
for rep in 1 2; do
  for v in "$@"; do
    LATTICEUM_AMD_LIB=ab/lib$v.so timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/ab_${TAG}${v}_$rep.log 2>&1 || exit 1
  done
done
