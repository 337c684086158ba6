#!/bin/bash
# fold() at the zkvm shape under a HIP API + kernel trace (host enqueue costs), after
# the selected -m gpu tests ($TESTS)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-trace}
TESTS=${TESTS:-tests/test_gpu_mz.py tests/test_gpu_sumcheck.py tests/test_gpu_fold_prove.py}
timeout -k 10 600 python -u -m pytest $TESTS -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace -d gpurun_out/proftrace_$TAG -o run --output-format csv -- \
  python tools/fold_prof.py > gpurun_out/fold_prof_$TAG.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/fold_prof_$TAG.log') if l.startswith('{')][-1])
print({k: (round(v,2) if isinstance(v,float) else v) for k,v in d.items() if k.startswith('ms') or k.startswith('vars')})
print({k: round(v,2) for k,v in d['span_ms'].items()})"
