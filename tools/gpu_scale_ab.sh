#!/bin/bash
# the bench-scale parity tests (incl. the batched ones), then stream-group A/B
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-sab}
timeout -k 10 900 python -u -m pytest tests/test_gpu_scale.py -m gpu -x -v -p no:cacheprovider --timeout 600 --timeout-method thread \
  > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|passed|failed" gpurun_out/pytest_$TAG.log | tail -12; [ $rc -eq 0 ] || exit $rc
run() {  # name, args
  timeout -k 10 300 python -u bench.py --no-small-shape --no-cpu-baseline $2 > gpurun_out/bench_${TAG}_$1.log 2>&1 || return 1
  python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/bench_${TAG}_$1.log') if l.startswith('{')][-1])
print('$1', round(d['value'],2), round(d['ms_per_step'],3), {k: round(v['avg_launch_ms'],3) for k,v in d['phases'].items()})"
}
run s2b2 "--streams 2 --batch 2 --steps 8 --warmup 2" && run s4g2 "--streams 4 --batch 2 --steps 8 --warmup 4" && \
run s4g4 "--streams 4 --batch 4 --steps 8 --warmup 4" && run s2b2r "--streams 2 --batch 2 --steps 8 --warmup 2" && \
run s4g2r "--streams 4 --batch 2 --steps 8 --warmup 4" && \
run d24g4 "--d 24 --w 19763 --streams 4 --batch 4 --steps 128 --warmup 8" && \
run d24g2 "--d 24 --w 19763 --streams 4 --batch 2 --steps 128 --warmup 8" && \
run w464g2 "--w 464 --streams 4 --batch 2 --steps 256 --warmup 16" && \
run w464b0 "--w 464 --streams 4 --batch 0 --steps 256 --warmup 16"
