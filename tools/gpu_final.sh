#!/bin/bash
# end-of-round check of HEAD on the GPU box: the whole -m gpu suite, smoke(), the default
# bench line and a rocprofv3 kernel-trace --stats run of the default workload
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-final}
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_$TAG.log 2>&1
rc=$?; tail -1 gpurun_out/smoke_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.log 2>&1
rc=$?; tail -c 400 gpurun_out/bench_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- \
  python bench.py --no-cpu-baseline --no-small-shape > gpurun_out/benchprof_$TAG.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python tools/prof_summary.py stats gpurun_out/prof_$TAG gpurun_out/stats_${TAG}_d1024_W16384.md > /dev/null
