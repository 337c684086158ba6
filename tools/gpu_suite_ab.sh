#!/bin/bash
# full GPU suite, then bench lines: W = 464 (4 streams), the reference ring
# (4 streams, unbatched and batched in one group of 4) and the headline (1 stream,
# 2 streams batched)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-suite}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
run() {  # name, args
  timeout -k 10 300 python -u bench.py --no-small-shape --no-cpu-baseline $2 > gpurun_out/bench_${TAG}_$1.log 2>&1
  local rc=$?
  python3 - "$1" "gpurun_out/bench_${TAG}_$1.log" <<'PY'
import json, sys
try:
    d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
except Exception as e:
    print(sys.argv[1], "no line", e); sys.exit(0)
ph = " ".join(f"{k}={v['avg_launch_ms']:.3f}" for k, v in d["phases"].items())
print(f"{sys.argv[1]:14s} {d['value']:9.1f} steps/s  {d['ms_per_step']:.3f} ms  {ph}")
PY
  return $rc
}
run w464 "--w 464 --streams 4 --steps 256 --warmup 16" && \
run d24_b0 "--d 24 --w 19763 --streams 4 --steps 128 --warmup 8" && \
run d24_b4 "--d 24 --w 19763 --streams 4 --batch 4 --steps 128 --warmup 8" && \
run head_s1 "--steps 6 --warmup 2" && \
run head_s2b "--streams 2 --batch 2 --steps 6 --warmup 2"
