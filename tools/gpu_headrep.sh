#!/bin/bash
# the default headline (no side lines) several times on one box: run-to-run spread
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2 3 4; do
  timeout -k 10 300 python -u bench.py --no-small-shape --no-cpu-baseline > gpurun_out/bench_hr_$rep.log 2>&1 || exit 1
  python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/bench_hr_$rep.log') if l.startswith('{')][-1])
print('$rep', round(d['value'],2), round(d['ms_per_step'],3), d['steps'], d['warmup'])"
done
