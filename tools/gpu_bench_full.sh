#!/bin/bash
# full-size default bench (d=1024, W=2^14) + rocprof kernel stats of the same command
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r01}
timeout -k 10 400 python bench.py > gpurun_out/bench_full_$TAG.log 2>&1
echo "bench rc=$?"
tail -2 gpurun_out/bench_full_$TAG.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_full_$TAG -o run --output-format csv -- \
  python bench.py --no-cpu-baseline > gpurun_out/bench_full_prof_$TAG.log 2>&1
echo "prof rc=$?"
tail -1 gpurun_out/bench_full_prof_$TAG.log
