cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp; mkdir -p gpurun_out
for REP in 1 2; do
for WV in 2048 1024 4096 8192; do
  export LATTICEUM_AMD_AJTAI_WAVES=$WV
  for S in 1 4; do
  timeout -k 10 120 python3 -u bench.py --d 24 --w 19763 --streams $S --steps 256 --warmup 8 --no-small-shape --no-cpu-baseline > gpurun_out/p24w.log 2>&1 || exit 1
  python3 - gpurun_out/p24w.log "waves=$WV streams=$S" <<'PY'
import json, sys
j = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(j["value"], 1), " ".join(f"{k} {v['avg_launch_ms']:.4f}" for k, v in j["phases"].items()))
PY
  done
done
done
