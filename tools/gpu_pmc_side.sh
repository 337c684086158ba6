#!/bin/bash
# PMC passes on the side ops alone (tools/side_ops_run.py): FETCH_SIZE and
# WRITE_SIZE in passes of their own, then one SQ pass; summarised into
# gpurun_out/pmc_side/pmc_{traffic,sq}_side_ops.json and profiles/ (bench.side_ops reads
# them back while the kernel sources still hash the same)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/pmc_side
rm -rf $O && mkdir -p $O
CFG='{"side_ops": true}'
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python3 tools/side_ops_run.py \
  > $O/fetch.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- python3 tools/side_ops_run.py \
  > $O/write.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
  SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -d $O/sq -o run --output-format csv -- \
  python3 tools/side_ops_run.py > $O/sq.log 2>&1 || exit 1
python3 tools/prof_summary.py traffic $O/fetch $O/write $O/pmc_traffic_side_ops.json --config "$CFG" > $O/traffic_summary.log 2>&1 &&
python3 tools/prof_summary.py sq $O/sq $O/pmc_sq_side_ops.json --config "$CFG" > $O/sq_summary.log 2>&1 &&
cp $O/pmc_traffic_side_ops.json $O/pmc_sq_side_ops.json profiles/ || exit 1
rm -rf $O/fetch $O/write $O/sq
echo "side-op PMC rc=0"
