#!/bin/bash
# fused decompositions with streaming stores below 4 GiB of outputs (LATTICEUM_AMD_DEC_NT=1) vs cached (0)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp; mkdir -p gpurun_out
for REP in 1 2; do
for V in 0 1; do
  export LATTICEUM_AMD_DEC_NT=$V
  timeout -k 10 120 python3 -u bench.py --w 464 --streams 4 --steps 768 --warmup 24 --no-small-shape --no-cpu-baseline > gpurun_out/dnt.log 2>&1 || exit 1
  python3 -c "import json; j=json.loads(open('gpurun_out/dnt.log').read().strip().splitlines()[-1]); print('W464 nt', $V, round(j['value'],1), ' '.join(f\"{k} {v['avg_launch_ms']:.3f}\" for k, v in j['phases'].items()))"
done
done
