#!/bin/bash
# a short GPU pass while iterating: selected -m gpu test files ($TESTS), then a kernel
# trace of fold() at the zkvm shape (tools/fold_prof.py)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-quick}
TESTS=${TESTS:-tests/test_gpu_sumcheck.py tests/test_gpu_fold_prove.py}
timeout -k 10 600 python -u -m pytest $TESTS -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/proffold_$TAG -o run --output-format csv -- \
  python tools/fold_prof.py $FOLD_ARGS > gpurun_out/fold_prof_$TAG.log 2>&1
rc=$?; echo "fold prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/fold_prof_$TAG.log') if l.startswith('{')][-1])
print({k: (round(v,2) if isinstance(v,float) else v) for k,v in d.items() if k.startswith('ms') or k.startswith('vars')})
print({k: round(v,2) for k,v in d['span_ms'].items()})"
python tools/prof_summary.py stats gpurun_out/proffold_$TAG gpurun_out/stats_fold_$TAG.md > /dev/null
head -14 gpurun_out/stats_fold_$TAG.md
if [ -n "$P2" ]; then bash tools/exp/p2_box.sh; fi
