#!/bin/bash
# quick iteration: GPU parity tests, kernel micro-bench, default bench without side workloads
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-quick}
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/kbench.py > gpurun_out/kb_$TAG.json 2>&1; rc=$?; tail -1 gpurun_out/kb_$TAG.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-small-shape --no-cpu-baseline > gpurun_out/bench_$TAG.log 2>&1; rc=$?
python3 -c "
import json,sys; d=json.loads(open('gpurun_out/bench_$TAG.log').read().strip().splitlines()[-1])
print('value', round(d['value'],2), 'ms', round(d['ms_per_step'],2)); [print(k, round(v['avg_launch_ms'],3), round(v['frac_hbm'],3)) for k,v in d['phases'].items()]"
exit $rc
