#!/bin/bash
# A/B timing of library builds: kernel micro-bench + default bench summary per library.
# usage: bash tools/gpu_ab.sh TAG LIB1 [LIB2 ...]   ("default" = the in-tree build)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; shift
for lib in "$@"; do
  name=$(basename "$lib" .so)
  if [ "$lib" = default ]; then unset LATTICEUM_AMD_LIB; else export LATTICEUM_AMD_LIB="$PWD/$lib"; fi
  echo "== $name"
  timeout -k 10 120 python tools/kbench.py > gpurun_out/kb_${TAG}_$name.json 2>&1; rc=$?; tail -1 gpurun_out/kb_${TAG}_$name.json; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python bench.py --no-small-shape --no-cpu-baseline > gpurun_out/bench_${TAG}_$name.log 2>&1; rc=$?; [ $rc -eq 0 ] || exit $rc
  python3 -c "
import json; d=json.loads(open('gpurun_out/bench_${TAG}_$name.log').read().strip().splitlines()[-1])
print('value', round(d['value'],2), 'ms', round(d['ms_per_step'],2)); [print(' ', k, round(v['avg_launch_ms'],3)) for k,v in d['phases'].items()]"
  if [ -n "$D24" ]; then timeout -k 10 120 python tools/streams_sweep.py 24 19763 32 1,4 64 || exit 1; fi
done
