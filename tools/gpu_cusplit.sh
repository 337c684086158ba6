#!/bin/bash
# CU-split A/B: the batch tests with the contraction on a
# CU-masked stream of its own, then the headline with each group's contraction
# on the last N CUs beside the step streams (bench.py --cu-split N) against the
# default one-group-of-4 line, on one box.
#   tools/gpu_cusplit.sh TAG "ARGS_A" "ARGS_B" ...
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; shift
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py -x -q -p no:cacheprovider --timeout 120 \
  --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
i=0
for A in "$@"; do
  i=$((i+1))
  timeout -k 10 300 python -u bench.py --no-small-shape --no-cpu-baseline --steps 16 --warmup 4 $A \
    --detail gpurun_out/cs_${TAG}_$i.json > gpurun_out/cs_${TAG}_$i.log 2>&1 || exit 1
  python3 -c "
import json; d=json.load(open('gpurun_out/cs_${TAG}_$i.json'))
print('$A', round(d['value'],2), round(d['ms_per_step'],3), {k: round(p['ms_per_step'],3) for k,p in d['phases'].items()})"
done
