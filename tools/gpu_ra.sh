#!/bin/bash
# contraction with A in registers (LATTICEUM_AMD_AJTAI_RA = chunks in flight): parity, then the d=1024 step
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-ra}
for R in ${RAS:-4}; do
  LATTICEUM_AMD_AJTAI_RA=$R timeout -k 10 300 python -u -m pytest tests -m gpu -k "ajtai or dev_fold_step_matches or bench_shape_d1024 or configs4" -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_${TAG}_$R.log 2>&1
  rc=$?; echo "pytest RA=$R rc=$rc"; tail -2 gpurun_out/pytest_${TAG}_$R.log; [ $rc -eq 0 ] || exit $rc
done
for REP in 1 2; do
for R in 0 ${RAS:-4}; do
  LATTICEUM_AMD_AJTAI_RA=$R timeout -k 10 200 python3 -u bench.py --steps 10 --warmup 2 --no-small-shape --no-cpu-baseline > gpurun_out/bench_${TAG}_$R.log 2>&1 || exit 1
  python3 - "gpurun_out/bench_${TAG}_$R.log" $R <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        j = json.loads(line); ph = j["phases"]
        print("RA", sys.argv[2], round(j["value"], 2), round(j["ms_per_step"], 2), "ajtai", round(ph["ajtai"]["avg_launch_ms"], 3), "dec", round(ph["decompose"]["avg_launch_ms"], 3))
PY
done
done
