#!/bin/bash
# one GPU pass over the round's work: the -m gpu suite, the default bench line, and a
# kernel-trace of fold() at the zkvm shape (tools/fold_prof.py)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-check}
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
fi
if [ -z "$SKIP_BENCH" ]; then
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.log 2>&1
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
python - <<PY
import json
b=json.loads([l for l in open('gpurun_out/bench_$TAG.log') if l.startswith('{')][-1])
print('value', round(b['value'],2), 'ms', round(b['ms_per_step'],3))
for k in ('reference_ring','small_shape','configs4_d4096_kappa64'): print(k, round(b[k]['value'],1))
fp=b['next_rows']['fold_prove']; print('fold', {k: round(v,2) if isinstance(v,float) else v for k,v in fp.items() if k.startswith('ms') or k.startswith('vars')})
print('spans', {k: round(v,2) for k,v in fp['span_ms'].items()})
fs=b['next_rows'].get('fold_prove_scalar')
if fs:
    print('fold scalar CCS', {k: round(v,2) if isinstance(v,float) else v for k,v in fs.items() if k.startswith('ms') or k.startswith('vars')})
    print('spans scalar', {k: round(v,2) for k,v in fs['span_ms'].items()})
    print('mz', b['next_rows']['mz_products'].get('challenged_mle_ms'), b['next_rows']['mz_products'].get('etas_ms'),
          'scalar', b['next_rows']['mz_products_scalar'])
ch=b['next_rows']['zkvm_chain']; print('chain', {k: (round(v,2) if isinstance(v,float) else v) for k,v in ch.items() if k not in ('workload','span_ms_per_step')})
print('chain spans', {k: round(v,2) for k,v in ch['span_ms_per_step'].items()})
print('cpu', b['cpu_baseline']['sample'], b['reference_ring']['cpu_baseline']['sample'])
PY
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/proffold_$TAG -o run --output-format csv -- \
  python tools/fold_prof.py > gpurun_out/fold_prof_$TAG.log 2>&1
rc=$?; echo "fold prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python tools/prof_summary.py stats gpurun_out/proffold_$TAG gpurun_out/stats_fold_$TAG.md > /dev/null
head -30 gpurun_out/stats_fold_$TAG.md
