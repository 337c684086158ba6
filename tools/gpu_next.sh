#!/bin/bash
# 8(f) kernels: their GPU tests, then one profiled run of bench.next_rows
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-next}
timeout -k 10 600 python -u -m pytest tests/test_gpu_sumcheck.py tests/test_gpu_mz.py tests/test_merkle.py tests/test_wire.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 tools/prof_next.py > gpurun_out/prof_$TAG.log 2>&1
rc=$?; echo "prof rc=$rc"; grep -h '^{' gpurun_out/prof_$TAG.log | tail -1; exit $rc
