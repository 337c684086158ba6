#!/bin/bash
# configs[4] (d = 4096, kappa = 64, W = 1024): one stream against two batched streams
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-c4}
run() {  # name, args
  timeout -k 10 300 python -u bench.py --no-small-shape --no-cpu-baseline $2 > gpurun_out/bench_${TAG}_$1.log 2>&1 || return 1
  python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/bench_${TAG}_$1.log') if l.startswith('{')][-1])
print('$1', round(d['value'],2), round(d['ms_per_step'],3), {k: round(v['avg_launch_ms'],3) for k,v in d['phases'].items()})"
}
A="--d 4096 --w 1024 --kappa 64"
run s1 "$A --streams 1 --steps 20 --warmup 3" && run s2b2 "$A --streams 2 --batch 2 --steps 20 --warmup 4" && \
run s4b4 "$A --streams 4 --batch 4 --steps 20 --warmup 4" && run s1r "$A --streams 1 --steps 20 --warmup 3" && \
run s2b2r "$A --streams 2 --batch 2 --steps 20 --warmup 4"
