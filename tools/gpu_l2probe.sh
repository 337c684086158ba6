#!/bin/bash
# contraction timing with L2-resident operands (a -DLF_AJ_L2PROBE build; results wrong, timing only)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for a in "--streams 1" "--streams 2 --batch 2"; do
  timeout -k 10 300 python -u bench.py --no-small-shape --no-cpu-baseline --steps 6 --warmup 2 $a > gpurun_out/probe_l2.log 2>&1 || exit 1
  python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/probe_l2.log') if l.startswith('{')][-1])
print('$a', round(d['value'],2), {k: round(v['avg_launch_ms'],3) for k,v in d['phases'].items()})"
done
