#!/bin/bash
# the Phi72 contraction's register-A depth (LATTICEUM_AMD_AJTAI_RA) on the reference-ring line
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp; mkdir -p gpurun_out
for REP in 1 2; do
for R in 4 3 5 0; do
  export LATTICEUM_AMD_AJTAI_RA=$R
  for S in 1 4; do
  timeout -k 10 120 python3 -u bench.py --d 24 --w 19763 --streams $S --steps 384 --warmup 12 --no-small-shape --no-cpu-baseline > gpurun_out/p24ra.log 2>&1 || exit 1
  python3 -c "import json; j=json.loads(open('gpurun_out/p24ra.log').read().strip().splitlines()[-1]); print('ra', $R, 'streams', $S, round(j['value'],1), 'ajtai', round(j['phases']['ajtai']['avg_launch_ms'],4))"
  done
done
done
