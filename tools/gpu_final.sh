#!/bin/bash
# round close-out on one box: the fold-split A/B on the W = 464 line, then the full evidence run
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp; mkdir -p gpurun_out
TAG=${1:-final}
for V in 1 0 1 0; do
  export LATTICEUM_AMD_FOLD_SPLIT=$V
  timeout -k 10 120 python3 -u bench.py --w 464 --streams 4 --steps 768 --warmup 24 --no-small-shape --no-cpu-baseline > gpurun_out/fs.log 2>&1 || exit 1
  python3 -c "
import json; j=json.loads(open('gpurun_out/fs.log').read().strip().splitlines()[-1])
print('split', $V, round(j['value'],1), ' '.join(f\"{k} {v['avg_launch_ms']:.3f}\" for k, v in j['phases'].items()))" | tee -a gpurun_out/fsplit_$TAG.txt
done
unset LATTICEUM_AMD_FOLD_SPLIT
bash tools/gpu_evidence.sh $TAG
