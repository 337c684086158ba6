#!/bin/bash
# PMC passes over the d = 24 step (one stream): SQ issue/wait counters and the
# TCP/TCC request counters, for the wave-local and the block-wide decomposition
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-p24}
mkdir -p gpurun_out
ARGS="--d 24 --w 19763 --kappa 32 --streams 1 --steps 6 --warmup 2 --no-small-shape --no-cpu-baseline"
for V in wave block; do
  if [ $V = block ]; then export LATTICEUM_AMD_DEC24=block; fi
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_INSTS_LDS SQ_BUSY_CYCLES \
    -d gpurun_out/${TAG}_sq_$V -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/${TAG}_sq_$V.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc TCP_TCC_WRITE_REQ_sum TCP_TCC_READ_REQ_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE \
    -d gpurun_out/${TAG}_tc_$V -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/${TAG}_tc_$V.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_kt_$V -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/${TAG}_kt_$V.log 2>&1 || exit 1
done
echo done
