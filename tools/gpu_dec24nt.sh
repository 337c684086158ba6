#!/bin/bash
# d = 24 decomposition A/B: streaming-store variants (LATTICEUM_AMD_DEC24_NT bit mask; "b" = the block-wide kernel)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-nt}
for REP in 1 2; do
for M in ${MASKS:-b 0 3 5 6 7}; do
  if [ $M = b ]; then export LATTICEUM_AMD_DEC24=block LATTICEUM_AMD_DEC24_NT=0; else export LATTICEUM_AMD_DEC24=wave LATTICEUM_AMD_DEC24_NT=$M; fi
  for S in ${STREAMS:-1 4}; do
    timeout -k 10 120 python3 -u bench.py --d 24 --w 19763 --kappa 32 --streams $S --steps 256 --warmup 8 --no-small-shape --no-cpu-baseline > gpurun_out/${TAG}_${M}_$S.log 2>&1 || exit 1
    python3 - "gpurun_out/${TAG}_${M}_$S.log" $M $S <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        j = json.loads(line); ph = j["phases"]
        print("mask", sys.argv[2], "streams", sys.argv[3], round(j["value"], 1), "dec", round(ph["decompose"]["avg_launch_ms"], 4), "ajtai", round(ph["ajtai"]["avg_launch_ms"], 4), "fold", round(ph["fold"]["avg_launch_ms"], 4))
PY
  done
done
done
