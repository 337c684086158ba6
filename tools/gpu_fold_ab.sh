#!/bin/bash
# A/B of library variants (abv/lib<v>.so) on fold(): the mz/fold GPU tests, then per
# variant a kernel trace of tools/fold_prof.py $FOLD_ARGS (default --scalar; gpurun_out/fab_<v>/)
# and its line
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for v in "$@"; do
  LATTICEUM_AMD_LIB=$R/abv/lib$v.so timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread \
    $R/tests/test_gpu_mz.py > $R/gpurun_out/fab_$v.test.log 2>&1 || { echo "$v tests failed"; exit 1; }
  LATTICEUM_AMD_LIB=$R/abv/lib$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $R/gpurun_out/fab_$v -o run -- python $R/tools/fold_prof.py ${FOLD_ARGS---scalar} > $R/gpurun_out/fab_$v.log 2>&1 || { echo "$v prof failed"; exit 1; }
  echo "$v ok"
done
