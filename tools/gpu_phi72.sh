#!/bin/bash
# Phi_72 (the reference ring): its parity tests, then the reference-ring bench line
# (new wave-local decomposition, then the block-wide one for comparison)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-phi72}
timeout -k 10 600 python -u -m pytest tests -m gpu -k "24 or phi72 or Phi72" -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
for V in wave block; do
  if [ $V = block ]; then export LATTICEUM_AMD_DEC24=block; fi
  timeout -k 10 300 python3 -u bench.py --d 24 --w 19763 --kappa 32 --streams 4 --steps 128 --warmup 8 --no-small-shape --no-cpu-baseline > gpurun_out/bench_${TAG}_$V.log 2>&1
  rc=$?; echo "bench $V rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 - "gpurun_out/bench_${TAG}_$V.log" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        j = json.loads(line); print(j["value"], j["ms_per_step"])
        for k, v in j.get("phases", {}).items():
            print(k, v["kernel"], round(v["avg_launch_ms"], 4), v["launches_per_step"], round(v["frac_hbm"], 3))
PY
done
