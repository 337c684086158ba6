#!/bin/bash
# W = 464 streams x batch sweep (the bench's main path at --w 464), two
# alternations: prints value and ms per step for each (streams, batch)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
CFGS=${CFGS:-4:2 4:4 8:4 8:8}
for rep in 1 2; do
  for sb in $CFGS; do
    s=${sb%%:*}; b=${sb#*:}
    timeout -k 10 300 python -u bench.py --w 464 --streams $s --batch $b --steps 256 --warmup 32 --no-small-shape \
      --no-cpu-baseline --detail gpurun_out/w464b_${s}_${b}_$rep.json > gpurun_out/w464b_${s}_${b}_$rep.log 2>&1 || exit 1
    python3 -c "
import json; d=json.load(open('gpurun_out/w464b_${s}_${b}_$rep.json'))
print('streams $s batch $b rep $rep', round(d['value'],1), round(d['ms_per_step'],4), {k: round(p['ms_per_step'],4) for k,p in d['phases'].items()})"
  done
done
