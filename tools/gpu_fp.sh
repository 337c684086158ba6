#!/bin/bash
# round 3: lf_fold_prove -- its GPU tests (oracle parity, zkvm dimensions), then the bench's next_rows lines
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-fp}
timeout -k 10 600 python -u -m pytest tests/test_gpu_fold_prove.py -m gpu -x -v -p no:cacheprovider --timeout 400 \
  --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -c "
import json, torch, bench, latticeum_amd as LA
torch.cuda.set_device(0)
print(json.dumps(bench.next_rows(LA, torch, 0, None)))" > gpurun_out/next_$TAG.log 2>&1
rc=$?; tail -c 1500 gpurun_out/next_$TAG.log; exit $rc
