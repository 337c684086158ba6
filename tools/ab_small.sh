#!/bin/bash
# A/B of the byte-equivalent small shape and the reference ring: old tree (ab/old) vs this one, same box
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for side in old new new old; do
  if [ $side = old ]; then dir=ab/old; else dir=.; fi
  (cd $dir && timeout -k 10 200 python -c "
import sys, json; sys.path.insert(0, '.')
import torch, bench, latticeum_amd as LA
from latticeum_amd import dist as LD
r = bench.extra_shape(LA, torch, LD, None, 0, 0, 1, 1024, 464, 32, 4, 256, 16, 'small')
r2 = bench.extra_shape(LA, torch, LD, None, 0, 0, 1, 24, 19763, 32, 4, 128, 8, 'phi72')
print('$side', round(r['value'], 1), round(r2['value'], 1))
") || exit 1
done
