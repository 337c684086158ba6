#!/bin/bash
# A/B timing on one box: alternate headline bench runs of abv/lib<name>.so builds
# (tools/build_variant.sh), REPS rounds; every run under its own time limit, and
# the first failure ends the script. BENCH_ARGS adds bench.py flags.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-ab}
REPS=${REPS:-2}
for rep in $(seq 1 $REPS); do
  for v in "$@"; do
    LATTICEUM_AMD_LIB=abv/lib$v.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-small-shape \
      --detail gpurun_out/${TAG}_${v}_$rep.json ${BENCH_ARGS} > gpurun_out/${TAG}_${v}_$rep.log 2>&1 || exit 1
    python3 -c "
import json,sys
d=json.load(open('gpurun_out/${TAG}_${v}_$rep.json'))
ph=d.get('phases',{})
print('$v', $rep, round(d['value'],2), round(d['ms_per_step'],3), {k: round(p['ms_per_step'],3) for k,p in ph.items()})
" | tee -a gpurun_out/${TAG}_summary.txt
  done
done
