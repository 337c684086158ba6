#!/bin/bash
# coefficient-form fold split over witnesses at few elements (LATTICEUM_AMD_FOLD_SPLIT=0 turns it off): the W=464 line
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp; mkdir -p gpurun_out
for REP in 1 2 3; do
for V in 1 0; do
  export LATTICEUM_AMD_FOLD_SPLIT=$V
  for S in 1 4; do
  timeout -k 10 120 python3 -u bench.py --w 464 --streams $S --steps 768 --warmup 24 --no-small-shape --no-cpu-baseline > gpurun_out/fs.log 2>&1 || exit 1
  python3 -c "
import json; j=json.loads(open('gpurun_out/fs.log').read().strip().splitlines()[-1])
print('split', $V, 'streams', $S, round(j['value'],1), ' '.join(f\"{k} {v['avg_launch_ms']:.3f}\" for k, v in j['phases'].items()))"
  done
done
done
