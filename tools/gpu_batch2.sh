#!/bin/bash
# batch-group A/B: W = 464, the reference ring and the headline with the step
# streams batched in groups (bench.py --batch G), plus rocprof stats of W = 464
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-batch2}
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
run w464_b0 "--w 464 --streams 4 --steps 256 --warmup 16" && \
run w464_g2 "--w 464 --streams 4 --batch 2 --steps 256 --warmup 16" && \
run d24_g2 "--d 24 --w 19763 --streams 4 --batch 2 --steps 128 --warmup 8" && \
run d24_g4 "--d 24 --w 19763 --streams 4 --batch 4 --steps 128 --warmup 8" && \
run head_s2 "--streams 2 --steps 6 --warmup 2" && \
run head_s2b "--streams 2 --batch 2 --steps 6 --warmup 2" && \
run head_s3b "--streams 3 --batch 3 --steps 6 --warmup 3" && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_w464 -o run --output-format csv -- \
  python bench.py --no-cpu-baseline --no-small-shape --w 464 --streams 4 --steps 64 --warmup 8 > gpurun_out/benchprof_${TAG}_w464.log 2>&1 && \
python tools/prof_summary.py stats gpurun_out/prof_${TAG}_w464 gpurun_out/stats_${TAG}_w464.md > /dev/null; echo "prof rc=$?"
