#!/bin/bash
# round 3: Phi72 packed digit planes -- the fold-step parity tests, then the
# reference-ring line (4 step streams)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-packed}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_merkle.py -m gpu -x -q -p no:cacheprovider \
  --timeout 300 --timeout-method thread -k "phi72 or packed or reference_ring or without_fk or fold_step or merkle" > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --d 24 --w 19763 --streams 4 --steps 128 --warmup 8 --no-cpu-baseline --no-small-shape \
  > gpurun_out/bench_$TAG.log 2>&1
rc=$?; python3 -c "
import json; d=json.loads(open('gpurun_out/bench_$TAG.log').read().strip().splitlines()[-1])
print('value', round(d['value'],1)); [print(k, round(v['avg_launch_ms'],4)) for k,v in d['phases'].items()]"
exit $rc
