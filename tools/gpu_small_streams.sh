#!/bin/bash
# the W = 464 shape at 2..6 step streams
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp; mkdir -p gpurun_out
for REP in 1 2; do
for S in 3 4 5 6; do
  timeout -k 10 120 python3 -u bench.py --w 464 --streams $S --steps 768 --warmup 24 --no-small-shape --no-cpu-baseline > gpurun_out/ss.log 2>&1 || exit 1
  python3 -c "import json; j=json.loads(open('gpurun_out/ss.log').read().strip().splitlines()[-1]); print('streams', $S, round(j['value'],1))"
done
done
