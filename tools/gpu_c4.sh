#!/bin/bash
# configs[4] (d = 4096, kappa = 64, W = 1024): packed planes vs u64 rows, 2 or 4 streams
# per batch; first the d = 4096 parity tests
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-c4}
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  tests/test_gpu_batch.py tests/test_gpu_scale.py -k "4096 or configs4" > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
fi
run() {  # name, args
  timeout -k 10 300 python -u bench.py --no-small-shape --no-cpu-baseline $2 > gpurun_out/bench_${TAG}_$1.log 2>&1 || return 1
  python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/bench_${TAG}_$1.log') if l.startswith('{')][-1])
print('$1', round(d['value'],2), round(d['ms_per_step'],3), {k: round(v['avg_launch_ms'],3) for k,v in d['phases'].items()})"
}
A="--d 4096 --w 1024 --kappa 64"
run p1s2 "$A --streams 2 --batch 2 --steps 20 --warmup 4" && run p0s2 "$A --packed 0 --streams 2 --batch 2 --steps 20 --warmup 4" && \
run p1s4 "$A --streams 4 --batch 4 --steps 20 --warmup 4" && run p0s4 "$A --packed 0 --streams 4 --batch 4 --steps 20 --warmup 4" && \
run p1s4b2 "$A --streams 4 --batch 2 --steps 20 --warmup 4"
