#!/bin/bash
# the byte-equivalent small shape (d=1024, W=464): stream counts and fold variants
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-small}
for V in ${VARS:-coeff slot}; do
  for S in ${STREAMS:-4 8}; do
    if [ $V = slot ]; then export LATTICEUM_AMD_FOLD=slot; else unset LATTICEUM_AMD_FOLD; fi
    timeout -k 10 120 python3 -u bench.py --w 464 --streams $S --steps 512 --warmup 16 --no-small-shape --no-cpu-baseline > gpurun_out/${TAG}_${V}_$S.log 2>&1 || exit 1
    python3 - "gpurun_out/${TAG}_${V}_$S.log" $V $S <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        j = json.loads(line); ph = j["phases"]
        print(sys.argv[2], "streams", sys.argv[3], round(j["value"], 1), " ".join(f"{k} {v['avg_launch_ms']:.3f}" for k, v in ph.items()))
PY
  done
done
