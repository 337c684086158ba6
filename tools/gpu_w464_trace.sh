#!/bin/bash
# W = 464 timed steps under a kernel trace, summarised by tools/trace_busy.py
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-w464}; shift
timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace -d gpurun_out/tr_$TAG -o run --output-format csv -- \
  python tools/w464_trace.py "$@" > gpurun_out/tr_$TAG.log 2>&1
rc=$?; echo "trace rc=$rc"; grep steps/s gpurun_out/tr_$TAG.log; [ $rc -eq 0 ] || exit $rc
python3 tools/trace_busy.py gpurun_out/tr_$TAG > gpurun_out/tr_$TAG.txt 2>&1; cat gpurun_out/tr_$TAG.txt
