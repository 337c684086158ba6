#!/bin/bash
# stream / batch count A/B on the reference ring, W = 464 and the headline
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-st}
run() {  # name, args
  timeout -k 10 300 python -u bench.py --no-small-shape --no-cpu-baseline $2 > gpurun_out/bench_${TAG}_$1.log 2>&1 || return 1
  python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/bench_${TAG}_$1.log') if l.startswith('{')][-1])
print('$1', round(d['value'],2), round(d['ms_per_step'],3))"
}
R="--d 24 --w 19763 --steps 128 --warmup 8"
S="--w 464 --steps 256 --warmup 16"
run d24_s4b4 "$R --streams 4 --batch 4" && run d24_s8b4 "$R --streams 8 --batch 4" && run d24_s4b4r "$R --streams 4 --batch 4" && \
run d24_s8b4r "$R --streams 8 --batch 4" && run w_s4b2 "$S --streams 4 --batch 2" && run w_s8b2 "$S --streams 8 --batch 2" && \
run w_s6b2 "$S --streams 6 --batch 2" && run w_s4b2r "$S --streams 4 --batch 2" && \
run h_s2b2 "--steps 8 --warmup 2 --streams 2 --batch 2" && run h_s4b4 "--steps 8 --warmup 2 --streams 4 --batch 4" && \
run h_s4b2 "--steps 8 --warmup 2 --streams 4 --batch 2"
