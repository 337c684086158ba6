#!/bin/bash
# L2 hit / miss counters of the batched headline step (one --pmc pass)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-tcc}
timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc_$TAG -o run --output-format csv -- \
  python bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-small-shape > gpurun_out/pmc_$TAG.log 2>&1
rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/pmc_table.py gpurun_out/pmc_$TAG 2>&1 | head -30
