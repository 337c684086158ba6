#!/bin/bash
# SQ issue/stall counters for every kernel of a short default-workload bench run (one --pmc pass).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-sq}
mkdir -p gpurun_out
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU \
  SQ_ACTIVE_INST_ANY SQ_WAVES GRBM_GUI_ACTIVE -d gpurun_out/pmc_sq_$TAG -o run --output-format csv -- \
  python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-small-shape ${BENCH_ARGS} > gpurun_out/pmc_sq_$TAG.log 2>&1
echo "rc=$?"
