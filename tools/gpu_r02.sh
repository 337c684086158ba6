#!/bin/bash
# round-2 iteration: GPU parity suite, then the full bench line
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r02}
SEL=${2:-}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread $SEL > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/pytest_$TAG.log | tail -3; [ $rc -eq 0 ] || exit $rc
[ -n "$NOBENCH" ] && exit 0
timeout -k 10 500 python -u bench.py > gpurun_out/bench_$TAG.log 2>&1; rc=$?
tail -c 600 gpurun_out/bench_$TAG.log; exit $rc
