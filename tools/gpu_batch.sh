#!/bin/bash
# batched fold steps (lf_dev_fold_step_batch): parity tests, then A/B bench lines
# of the W = 464 shape, the reference ring and the headline, unbatched vs batched
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-batch}
timeout -k 10 600 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider \
  --timeout 300 --timeout-method thread -k "batch or fold_step or rho" > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
run() {  # name, args
  timeout -k 10 300 python -u bench.py --no-small-shape --no-cpu-baseline $2 > gpurun_out/bench_${TAG}_$1.log 2>&1
  local rc=$?
  python3 - "$1" "gpurun_out/bench_${TAG}_$1.log" <<'EOF'
import json, sys
try:
    d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
except Exception as e:
    print(sys.argv[1], "no line", e); sys.exit(0)
ph = " ".join(f"{k}={v['avg_launch_ms']:.3f}" for k, v in d["phases"].items())
print(f"{sys.argv[1]:14s} {d['value']:9.1f} steps/s  {d['ms_per_step']:.3f} ms  {ph}")
EOF
  return $rc
}
run w464_b0 "--w 464 --streams 4 --steps 256 --warmup 16" && \
run w464_b1 "--w 464 --streams 4 --batch 1 --steps 256 --warmup 16" && \
run d24_b0 "--d 24 --w 19763 --streams 4 --steps 128 --warmup 8" && \
run d24_b1 "--d 24 --w 19763 --streams 4 --batch 1 --steps 128 --warmup 8" && \
run head_s1 "--steps 6 --warmup 2" && \
run head_s2b "--streams 2 --batch 1 --steps 6 --warmup 2"
