#!/bin/bash
# the four bench lines (headline, reference ring, W = 464, configs[4]) twice, with their phase times
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-ln}
run() {  # name, args
  timeout -k 10 300 python -u bench.py --no-small-shape --no-cpu-baseline $2 > gpurun_out/bench_${TAG}_$1.log 2>&1 || return 1
  python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/bench_${TAG}_$1.log') if l.startswith('{')][-1])
print('$1', round(d['value'],2), round(d['ms_per_step'],3), {k: round(v['avg_launch_ms'],3) for k,v in d['phases'].items()})"
}
for rep in 1 2; do
  run head$rep "" && run d24_$rep "--d 24 --w 19763 --streams 4 --batch 4 --steps 128 --warmup 8" && \
  run w464_$rep "--w 464 --streams 4 --batch 2 --steps 256 --warmup 16" && \
  run c4_$rep "--d 4096 --w 1024 --kappa 64 --streams 2 --batch 2 --steps 20 --warmup 4" || exit 1
done
