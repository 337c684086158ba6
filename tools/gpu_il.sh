#!/bin/bash
# k_ajtai_mfma_ra with the operand copies interleaved with the products against in front of them (LATTICEUM_AMD_AJTAI_IL=0):
# parity of the layouts and batched steps, then bench A/B pairs
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-il}
SKIP_TESTS=${SKIP_TESTS:-0}
if [ "$SKIP_TESTS" != 1 ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_batch.py \
    tests/test_gpu_parity.py -k "ajtai or fold_step or commit or frag or batch or phi72 or d4096 or n4k" \
    > gpurun_out/pytest_$TAG.log 2>&1
  rc=$?; tail -5 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
fi
run() {  # name, env, args
  env $2 timeout -k 10 300 python -u bench.py --no-small-shape --no-cpu-baseline $3 > gpurun_out/bench_${TAG}_$1.log 2>&1 || return 1
  python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/bench_${TAG}_$1.log') if l.startswith('{')][-1])
print('$1', round(d['value'],2), round(d['ms_per_step'],3), {k: round(v['avg_launch_ms'],3) for k,v in d['phases'].items()})"
}
H="--steps 8 --warmup 2"
run pair "X=1" "$H" && run ra "LATTICEUM_AMD_AJTAI_IL=0" "$H" && run pair2 "X=1" "$H" && run ra2 "LATTICEUM_AMD_AJTAI_IL=0" "$H" && \
run w464p "X=1" "--w 464 --streams 4 --batch 2 --steps 256 --warmup 16" && \
run w464r "LATTICEUM_AMD_AJTAI_IL=0" "--w 464 --streams 4 --batch 2 --steps 256 --warmup 16" && \
run d24p "X=1" "--d 24 --w 19763 --streams 4 --batch 4 --steps 128 --warmup 8" && \
run d24r "LATTICEUM_AMD_AJTAI_IL=0" "--d 24 --w 19763 --streams 4 --batch 4 --steps 128 --warmup 8" && \
run c4p "X=1" "--d 4096 --w 1024 --kappa 64 --streams 2 --batch 2 --steps 20 --warmup 4" && \
run c4r "LATTICEUM_AMD_AJTAI_IL=0" "--d 4096 --w 1024 --kappa 64 --streams 2 --batch 2 --steps 20 --warmup 4"
