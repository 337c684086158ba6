#!/bin/bash
# Phi72 decomposition streaming-store mask (3: rows, 7: rows + operand rows) with the coefficient-form fold
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp; mkdir -p gpurun_out
for REP in 1 2 3; do
for M in 3 7; do
  export LATTICEUM_AMD_DEC24_NT=$M
  timeout -k 10 120 python3 -u bench.py --d 24 --w 19763 --streams 4 --steps 384 --warmup 12 --no-small-shape --no-cpu-baseline > gpurun_out/p24nt.log 2>&1 || exit 1
  python3 -c "import json; j=json.loads(open('gpurun_out/p24nt.log').read().strip().splitlines()[-1]); print('mask', $M, round(j['value'],1), ' '.join(f\"{k} {v['avg_launch_ms']:.4f}\" for k, v in j['phases'].items()))"
done
done
