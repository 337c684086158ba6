#!/bin/bash
# Timing experiments: the headline bench line with each abl/lib<name>.so (names as
# args), twice alternating; prints value and the per-phase launch times
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-var}
for rep in 1 2; do
  for v in "$@"; do
    LATTICEUM_AMD_LIB=abl/lib$v.so timeout -k 10 300 python -u bench.py --no-small-shape --no-cpu-baseline \
      --steps 8 --warmup 4 ${BENCH_ARGS} --detail gpurun_out/var_${TAG}_${v}_$rep.json > gpurun_out/var_${TAG}_${v}_$rep.log 2>&1 || exit 1
    python3 -c "
import json; d=json.load(open('gpurun_out/var_${TAG}_${v}_$rep.json'))
print('$v', $rep, round(d['value'],2), round(d['ms_per_step'],3), {k: round(p['avg_launch_ms'],3) for k,p in d['phases'].items()})"
  done
done
