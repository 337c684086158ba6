#!/bin/bash
# Phi_72 coefficient-form fold: parity, then the reference-ring line with it and with the NTT-form fold
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-p24f}
[ -n "$SKIP_TESTS" ] || timeout -k 10 600 python -u -m pytest tests -m gpu -k "24 or phi72 or Phi72 or cu_masked or montgomery or lcccs or sharded or reference_ring" -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; [ -n "$SKIP_TESTS" ] || { echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc; }
for REP in 1 2; do
for V in coeff slot; do
  if [ $V = slot ]; then export LATTICEUM_AMD_FOLD=slot; else unset LATTICEUM_AMD_FOLD; fi
  for S in 1 4; do
    timeout -k 10 120 python3 -u bench.py --d 24 --w 19763 --streams $S --steps 256 --warmup 8 --no-small-shape --no-cpu-baseline > gpurun_out/${TAG}_${V}_$S.log 2>&1 || exit 1
    python3 - gpurun_out/${TAG}_${V}_$S.log "$V streams=$S" <<'PY'
import json, sys
j = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(j["value"], 1), " ".join(f"{k} {v['avg_launch_ms']:.4f}" for k, v in j["phases"].items()))
PY
  done
done
done
