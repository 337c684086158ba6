#!/bin/bash
# One GPU-box check of the tree as it is: the -m gpu suite, smoke(), then the
# default bench line (compact line on stdout, the full record in
# gpurun_out/bench_detail_$TAG.json). Stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-check}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke_$TAG.log; [ $rc -eq 0 ] || exit $rc
[ -n "$SKIP_BENCH" ] && exit 0
timeout -k 10 600 python bench.py --detail gpurun_out/bench_detail_$TAG.json > gpurun_out/bench_$TAG.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 2500 gpurun_out/bench_$TAG.log; exit $rc
