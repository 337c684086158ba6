#!/bin/bash
# rocprofv3 kernel stats of the default bench line (its next_rows: linearization / folding sumchecks, Mz, fold_prove)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-pn}
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run -- python3 bench.py --no-cpu-baseline \
  > gpurun_out/profnext_$TAG.log 2>&1 || exit 1
f=$(ls gpurun_out/prof_$TAG/*/run_kernel_stats.csv 2>/dev/null | head -1)
[ -n "$f" ] || f=$(find gpurun_out/prof_$TAG -name "*kernel_stats.csv" | head -1)
head -30 "$f"
