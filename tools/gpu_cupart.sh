#!/bin/bash
# d=1024 W=2^14: step streams with and without a CU partition (lf_stream_create_cu_mask)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-cup}
for REP in 1 2; do
for V in "1" "2" "2 --cu-partition" "3 --cu-partition" "4 --cu-partition"; do
  timeout -k 10 200 python3 -u bench.py --streams $V --steps 12 --warmup 4 --no-small-shape --no-cpu-baseline > gpurun_out/${TAG}.log 2>&1 || exit 1
  python3 - "gpurun_out/${TAG}.log" "$V" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        j = json.loads(line)
        print("streams", sys.argv[2], round(j["value"], 2), round(j["ms_per_step"], 2))
PY
done
done
