#!/bin/bash
# rocprofv3 kernel-trace --stats of one bench.py invocation: bash tools/gpu_prof.sh TAG [bench args]
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; shift
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- \
  python bench.py --no-cpu-baseline --no-small-shape "$@" > gpurun_out/bench_$TAG.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -c 400 gpurun_out/bench_$TAG.log
python tools/prof_summary.py stats gpurun_out/prof_$TAG gpurun_out/stats_$TAG.md > /dev/null && cat gpurun_out/stats_$TAG.md
exit $rc
