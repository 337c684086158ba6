#!/bin/bash
# same-box A/B of two library builds (abl/libold.so, abl/libnew.so): the reference ring and the headline, alternating
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-ab2}
run() {  # name, lib, args
  LATTICEUM_AMD_LIB=abl/lib$2.so timeout -k 10 300 python -u bench.py --no-small-shape --no-cpu-baseline $3 \
    > gpurun_out/bench_${TAG}_$1.log 2>&1 || return 1
  python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/bench_${TAG}_$1.log') if l.startswith('{')][-1])
print('$1', round(d['value'],2), round(d['ms_per_step'],3), {k: round(v['avg_launch_ms'],3) for k,v in d['phases'].items()})"
}
R="--d 24 --w 19763 --streams 4 --batch 4 --steps 128 --warmup 8"
for rep in 1 2; do
  run d24_old$rep old "$R" && run d24_new$rep new "$R" || exit 1
done
for rep in 1 2; do
  run head_old$rep old "" && run head_new$rep new "" || exit 1
done
