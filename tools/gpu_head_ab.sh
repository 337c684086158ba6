#!/bin/bash
# headline stream / batch-group A/B on one box
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-hab}
run() {  # name, args
  timeout -k 10 300 python -u bench.py --no-small-shape --no-cpu-baseline $2 > gpurun_out/bench_${TAG}_$1.log 2>&1 || return 1
  python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/bench_${TAG}_$1.log') if l.startswith('{')][-1])
print('$1', round(d['value'],2), round(d['ms_per_step'],3), {k: round(v['avg_launch_ms'],3) for k,v in d['phases'].items()})"
}
run s1 "--steps 6 --warmup 2" && run s2b2 "--streams 2 --batch 2 --steps 8 --warmup 2" && \
run s4g2 "--streams 4 --batch 2 --steps 8 --warmup 4" && run s3b3 "--streams 3 --batch 3 --steps 9 --warmup 3" && \
run s2b2r "--streams 2 --batch 2 --steps 8 --warmup 2" && run s4g2r "--streams 4 --batch 2 --steps 8 --warmup 4" && \
run d24b4 "--d 24 --w 19763 --streams 4 --batch 4 --steps 128 --warmup 8" && \
run d24g2 "--d 24 --w 19763 --streams 4 --batch 2 --steps 128 --warmup 8"
