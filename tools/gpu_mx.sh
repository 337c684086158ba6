#!/bin/bash
# the fused d = 1024 decomposition with stage 1 on the matrix cores (default) vs
# the VALU network (LATTICEUM_AMD_DEC_MX=0): GPU suite, then the bench line of each
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-mx}
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
for V in 0 1; do
  LATTICEUM_AMD_DEC_MX=$V timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/bench_${TAG}_$V.log 2>&1
  rc=$?; echo "bench MX=$V rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 - gpurun_out/bench_${TAG}_$V.log <<'PY'
import json, sys
j = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print("value", round(j["value"], 2), {k: round(v["avg_launch_ms"], 3) for k, v in j["phases"].items()},
      "W464", round(j["small_shape"]["value"]), j["small_shape"]["phases"]["decompose"]["avg_launch_ms"],
      "d4096", round(j["configs4_d4096_kappa64"]["value"], 1))
PY
done
