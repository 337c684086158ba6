#!/bin/bash
# fold() end to end: its GPU tests, then the default bench line's fold_prove / replay timings
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-fp}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fold_prove.py \
  tests/test_gpu_sumcheck.py tests/test_replay.py tests/test_abi.py > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/bench_$TAG.log 2>&1 || exit 1
python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/bench_$TAG.log') if l.startswith('{')][-1]); f=d['next_rows']['fold_prove']
n=d['next_rows']
print(round(d['value'],2), round(f['ms_per_fold_prove'],2), round(f['ms_per_replay'],2), {k: round(v,2) for k,v in f['span_ms'].items()})
print('lin', round(n['linearization_sumcheck']['ms_per_prove'],2), 'fold_sc', round(n['folding_sumcheck']['ms_per_prove'],2))"
