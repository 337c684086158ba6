cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 120 python3 bench.py --w 464 --streams 4 --steps 256 --warmup 16 --no-small-shape --no-cpu-baseline > gpurun_out/so1.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/so2.log 2>&1 || exit 1
timeout -k 10 120 python3 bench.py --w 464 --streams 4 --steps 256 --warmup 16 --no-small-shape --no-cpu-baseline > gpurun_out/so3.log 2>&1 || exit 1
python3 - <<'PY'
import json
for f in ("so1", "so2", "so3"):
    j = json.loads(open(f"gpurun_out/{f}.log").read().strip().splitlines()[-1])
    print(f, round(j["value"], 1), "small", round(j["small_shape"]["value"], 1) if "small_shape" in j else "", "ref", round(j["reference_ring"]["value"], 1) if "reference_ring" in j else "")
PY
