#!/bin/bash
# W = 464: 4 streams in pairs vs one batch of 4, alternating
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # name, args
  timeout -k 10 300 python -u bench.py --no-small-shape --no-cpu-baseline $2 > gpurun_out/bench_wb_$1.log 2>&1 || return 1
  python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/bench_wb_$1.log') if l.startswith('{')][-1])
print('$1', round(d['value'],2), round(d['ms_per_step'],3))"
}
S="--w 464 --steps 256 --warmup 16"
for rep in 1 2 3; do
  run b2_$rep "$S --streams 4 --batch 2" && run b4_$rep "$S --streams 4 --batch 4" && run s8b4_$rep "$S --streams 8 --batch 4" || exit 1
done
