#!/bin/bash
# Same-box A/B of an environment switch: the -m gpu suite with the switch set
# (parity), then the headline bench line alternating without / with it.
#   tools/gpu_ab_env.sh TAG VAR=value
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; SW=$2
if [ -z "$SKIP_TESTS" ]; then
env $SW timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest ($SW) rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
fi
for rep in 1 2; do
  for arm in off on; do
    E=""; [ $arm = on ] && E=$SW
    env $E timeout -k 10 300 python -u bench.py --no-small-shape --no-cpu-baseline --steps 16 --warmup 4 ${BENCH_ARGS} \
      --detail gpurun_out/ab_${TAG}_${arm}_$rep.json > gpurun_out/ab_${TAG}_${arm}_$rep.log 2>&1 || exit 1
    python3 -c "
import json; d=json.load(open('gpurun_out/ab_${TAG}_${arm}_$rep.json'))
print('$arm', $rep, round(d['value'],2), round(d['ms_per_step'],3), {k: round(p['avg_launch_ms'],3) for k,p in d['phases'].items()})"
  done
done
