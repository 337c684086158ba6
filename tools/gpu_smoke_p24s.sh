#!/bin/bash
# smoke() on the box, then the reference ring at 3..8 step streams
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
for REP in 1 2; do
for S in 3 4 6 8; do
  timeout -k 10 120 python3 -u bench.py --d 24 --w 19763 --streams $S --steps 384 --warmup 12 --no-small-shape --no-cpu-baseline > gpurun_out/p24s.log 2>&1 || exit 1
  python3 -c "import json; j=json.loads(open('gpurun_out/p24s.log').read().strip().splitlines()[-1]); print('streams', $S, round(j['value'],1))"
done
done
