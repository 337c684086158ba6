#!/bin/bash
# exploration: VALU probe, new-kernel parity, NTT / decomposition A/B, side configs
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-explore}
timeout -k 10 120 ./tools/probe/probe_valu > gpurun_out/probe_valu_$TAG.txt 2>&1
rc=$?; echo "probe rc=$rc"; cat gpurun_out/probe_valu_$TAG.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread \
  -k "o4 or variants or fold_step or transform" > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/kbench.py > gpurun_out/kb_default_$TAG.json 2>&1; rc=$?; tail -1 gpurun_out/kb_default_$TAG.json; [ $rc -eq 0 ] || exit $rc
LATTICEUM_AMD_NTT=o4 timeout -k 10 120 python tools/kbench.py > gpurun_out/kb_o4_$TAG.json 2>&1; rc=$?; tail -1 gpurun_out/kb_o4_$TAG.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-small-shape --no-cpu-baseline > gpurun_out/bench_v2_$TAG.log 2>&1; rc=$?; tail -c 1500 gpurun_out/bench_v2_$TAG.log; [ $rc -eq 0 ] || exit $rc
LATTICEUM_AMD_DEC=v1 timeout -k 10 300 python bench.py --no-small-shape --no-cpu-baseline > gpurun_out/bench_v1_$TAG.log 2>&1; rc=$?; tail -c 1500 gpurun_out/bench_v1_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/configs_bench.py > gpurun_out/configs_$TAG.json 2> gpurun_out/configs_$TAG.err
rc=$?; echo "configs rc=$rc"; cat gpurun_out/configs_$TAG.json; tail -5 gpurun_out/configs_$TAG.err
