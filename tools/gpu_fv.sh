#!/bin/bash
# F-from-vectors contraction: Ajtai / fold-step parity and bench-size tests, then the d=1024 main line
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-fv}
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --no-small-shape --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/bench_$TAG.log 2>&1
rc=$?; echo "bench rc=$rc"; python3 - "$TAG" <<'PY'
import json, sys
for line in open(f"gpurun_out/bench_{sys.argv[1]}.log"):
    if line.startswith("{"):
        j = json.loads(line); print("main", round(j["value"], 2), round(j["ms_per_step"], 2))
        for k, v in j.get("phases", {}).items():
            print(" ", k, v["kernel"], round(v["avg_launch_ms"], 3), v["launches_per_step"], round(v["frac_hbm"], 3))
PY
exit $rc
