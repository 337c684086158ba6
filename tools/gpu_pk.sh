#!/bin/bash
# round 3: packed planes at d = 1024 -- parity tests, then the default workload with and without them
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-pk}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multi.py tests/test_gpu_fold_prove.py -m gpu -x -q \
  -p no:cacheprovider --timeout 300 --timeout-method thread -k "packed or fold_step or planes or sharded or multi or fold_prove or poseidon2" \
  > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
for p in 0 1 0 1; do
  timeout -k 10 300 python bench.py --packed $p --no-small-shape --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/bench_${TAG}_$p.log 2>&1
  rc=$?; [ $rc -eq 0 ] || exit $rc
  python3 -c "
import json; d=json.loads(open('gpurun_out/bench_${TAG}_$p.log').read().strip().splitlines()[-1])
print('packed $p value', round(d['value'],2), {k: round(v['avg_launch_ms'],3) for k,v in d['phases'].items()})"
done
