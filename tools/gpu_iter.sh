#!/bin/bash
# iteration loop on the GPU box: parity tests, then full bench + rocprof kernel stats
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-iter}
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py ${BENCH_ARGS} > gpurun_out/bench_$TAG.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/kbench.py > gpurun_out/kb_$TAG.json 2>&1
rc=$?; echo "kbench rc=$rc"; tail -1 gpurun_out/kb_$TAG.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- \
  python bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/benchprof_$TAG.log 2>&1
echo "prof rc=$?"
