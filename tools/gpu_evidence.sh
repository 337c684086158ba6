#!/bin/bash
# Round evidence on the GPU box, for the four bench lines (headline d=1024 W=2^14,
# reference ring d=24 W=19763, W=464, configs[4] d=4096 kappa=64):
#   1. (unless SKIP_TESTS) the -m gpu suite
#   2. per line: PMC passes FETCH_SIZE, WRITE_SIZE (separately, MI355X_MICROARCH.md §HBM)
#      and the SQ issue counters, over the same workload the bench line runs ->
#      gpurun_out/pmc_{traffic,sq}_d<d>_W<W>_k<kappa>.json (collect_evidence.sh copies
#      them to profiles/, where bench.py reads them)
#   3. (unless SKIP_BENCH) the default bench line, reading those files
#   4. rocprofv3 --kernel-trace --marker-trace --stats of the default bench command:
#      bench.py wraps every workload's serialized phase pass in a roctx range, and
#      prof_summary.py stats keeps the kernels inside each range (the launches the
#      line's per-phase HIP-event averages come from)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-evidence}
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
fi
Q="--no-cpu-baseline --no-small-shape"
CFGS=${CFGS:-"1024:16384:32:--steps 8 --warmup 4
24:19763:32:--d 24 --w 19763 --kappa 32 --streams 4 --batch 4 --steps 16 --warmup 4
1024:464:32:--w 464 --streams 4 --batch 2 --steps 32 --warmup 8
4096:1024:64:--d 4096 --w 1024 --kappa 64 --streams 2 --batch 2 --steps 8 --warmup 2"}
if [ -z "$SKIP_PMC" ]; then
while IFS= read -r cfg; do
  d=${cfg%%:*}; r=${cfg#*:}; W=${r%%:*}; r=${r#*:}; k=${r%%:*}; args=${r#*:}
  n=d${d}_W${W}_k${k}
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcf_${TAG}_$n -o run --output-format csv -- \
    python bench.py $Q $args > gpurun_out/pmcf_${TAG}_$n.log 2>&1
  rc=$?; echo "fetch $n rc=$rc"; [ $rc -eq 0 ] || exit $rc
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcw_${TAG}_$n -o run --output-format csv -- \
    python bench.py $Q $args > gpurun_out/pmcw_${TAG}_$n.log 2>&1
  rc=$?; echo "write $n rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python tools/prof_summary.py traffic gpurun_out/pmcf_${TAG}_$n gpurun_out/pmcw_${TAG}_$n \
    gpurun_out/pmc_traffic_$n.json $d $W $k > /dev/null || exit 1
  timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
    SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -d gpurun_out/pmcs_${TAG}_$n -o run --output-format csv -- \
    python bench.py $Q $args > gpurun_out/pmcs_${TAG}_$n.log 2>&1
  rc=$?; echo "sq $n rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python tools/prof_summary.py sq gpurun_out/pmcs_${TAG}_$n gpurun_out/pmc_sq_$n.json $d $W $k > /dev/null || exit 1
  cp gpurun_out/pmc_traffic_$n.json gpurun_out/pmc_sq_$n.json profiles/
  rm -rf gpurun_out/pmcf_${TAG}_$n gpurun_out/pmcw_${TAG}_$n gpurun_out/pmcs_${TAG}_$n
done <<< "$CFGS"
# the side ops (configs[1]'s 2^16 NTT / INTT, the 2^20-state Poseidon2 batch) at their own sizes
tools/gpu_pmc_side.sh || exit 1
fi
if [ -z "$SKIP_BENCH" ]; then
timeout -k 10 600 python bench.py --detail gpurun_out/bench_detail_$TAG.json > gpurun_out/bench_$TAG.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 300 gpurun_out/bench_$TAG.log; [ $rc -eq 0 ] || exit $rc
fi
[ -n "$SKIP_PROF" ] && exit 0
timeout -k 10 600 rocprofv3 --kernel-trace --marker-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- \
  python bench.py --detail gpurun_out/benchprof_detail_$TAG.json > gpurun_out/benchprof_$TAG.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python tools/prof_summary.py stats gpurun_out/prof_$TAG gpurun_out/stats_$TAG.md > /dev/null || exit 1
python tools/check_profile.py gpurun_out/benchprof_$TAG.log gpurun_out/stats_$TAG.windows.json > gpurun_out/check_$TAG.txt 2>&1
echo "check rc=$?"; tail -20 gpurun_out/check_$TAG.txt
rm -rf gpurun_out/prof_$TAG/*/*.csv.bak 2>/dev/null
exit 0
