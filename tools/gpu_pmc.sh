#!/bin/bash
# PMC passes on the GPU box (MI355X_MICROARCH.md §HBM / §rocprofv3 PMC slots):
# FETCH_SIZE and WRITE_SIZE in separate passes, then SQ issue counters.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-pmc}
ARGS="--steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS}"
mkdir -p gpurun_out
rocprofv3 -L > gpurun_out/counters_$TAG.txt 2>&1 || true
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_$TAG -o run --output-format csv -- \
  python bench.py $ARGS > gpurun_out/pmc_fetch_$TAG.log 2>&1 && echo fetch ok &&
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_$TAG -o run --output-format csv -- \
  python bench.py $ARGS > gpurun_out/pmc_write_$TAG.log 2>&1 && echo write ok &&
timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  -d gpurun_out/pmc_sq_$TAG -o run --output-format csv -- \
  python bench.py $ARGS > gpurun_out/pmc_sq_$TAG.log 2>&1 && echo sq ok
