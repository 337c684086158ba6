#!/bin/bash
# Round evidence on the GPU box: parity tests, PMC traffic passes (FETCH_SIZE /
# WRITE_SIZE separately, MI355X_MICROARCH.md §HBM) of the default workload, the
# bench line (which reads the traffic file), and rocprofv3 kernel-trace --stats
# runs of the default workload, the W=464 shape and the d=24 reference ring.
# Everything lands in gpurun_out/; tools/collect_evidence.sh copies it to profiles/.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-evidence}
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
fi
ARGS="--steps 8 --warmup 4 --no-cpu-baseline --no-small-shape"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_$TAG -o run --output-format csv -- \
  python bench.py $ARGS > gpurun_out/pmc_fetch_$TAG.log 2>&1
rc=$?; echo "fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_$TAG -o run --output-format csv -- \
  python bench.py $ARGS > gpurun_out/pmc_write_$TAG.log 2>&1
rc=$?; echo "write rc=$rc"; [ $rc -eq 0 ] || exit $rc
python tools/prof_summary.py traffic gpurun_out/pmc_fetch_$TAG gpurun_out/pmc_write_$TAG \
  gpurun_out/pmc_traffic_$TAG.json 1024 16384 32 > /dev/null && cp gpurun_out/pmc_traffic_$TAG.json profiles/pmc_traffic.json
# the reference ring (d = 24 at the zkvm shape, one stream): its own traffic file
A24="--d 24 --w 19763 --kappa 32 --streams 4 --batch 4 --steps 16 --warmup 4 --no-cpu-baseline --no-small-shape"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc24_fetch_$TAG -o run --output-format csv -- \
  python bench.py $A24 > gpurun_out/pmc24_fetch_$TAG.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc24_write_$TAG -o run --output-format csv -- \
  python bench.py $A24 > gpurun_out/pmc24_write_$TAG.log 2>&1 && \
python tools/prof_summary.py traffic gpurun_out/pmc24_fetch_$TAG gpurun_out/pmc24_write_$TAG \
  gpurun_out/pmc_traffic_d24_$TAG.json 24 19763 32 > /dev/null && cp gpurun_out/pmc_traffic_d24_$TAG.json profiles/pmc_traffic_d24.json
rc=$?; echo "d24 traffic rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
  SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_WAVES GRBM_GUI_ACTIVE -d gpurun_out/pmc_sq_$TAG -o run --output-format csv -- \
  python bench.py $ARGS > gpurun_out/pmc_sq_$TAG.log 2>&1
rc=$?; echo "sq rc=$rc"; [ $rc -eq 0 ] || exit $rc
python tools/prof_summary.py sq gpurun_out/pmc_sq_$TAG gpurun_out/pmc_sq_$TAG.json 1024 16384 32 > /dev/null && \
  cp gpurun_out/pmc_sq_$TAG.json profiles/pmc_sq.json
# the same SQ pass over the reference ring's step (d = 24 at the zkvm shape, one stream)
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
  SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_WAVES GRBM_GUI_ACTIVE -d gpurun_out/pmc24_sq_$TAG -o run --output-format csv -- \
  python bench.py $A24 > gpurun_out/pmc24_sq_$TAG.log 2>&1
rc=$?; echo "sq24 rc=$rc"; [ $rc -eq 0 ] || exit $rc
python tools/prof_summary.py sq gpurun_out/pmc24_sq_$TAG gpurun_out/pmc_sq_d24_$TAG.json 24 19763 32 > /dev/null && \
  cp gpurun_out/pmc_sq_d24_$TAG.json profiles/pmc_sq_d24.json
if [ -z "$SKIP_BENCH" ]; then
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 300 gpurun_out/bench_$TAG.log; [ $rc -eq 0 ] || exit $rc
fi
for cfg in "d1024_W16384:" "d1024_W464:--w 464 --streams 1 --steps 64 --warmup 8" "d24_W19763:--d 24 --w 19763 --streams 4 --batch 4 --steps 32 --warmup 4" \
           "d4096_W1024:--d 4096 --w 1024 --kappa 64 --streams 2 --batch 2 --steps 10 --warmup 2"; do
  name=${cfg%%:*}; args=${cfg#*:}
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_$name -o run --output-format csv -- \
    python bench.py --no-cpu-baseline --no-small-shape $args > gpurun_out/benchprof_${TAG}_$name.log 2>&1
  rc=$?; echo "prof $name rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python tools/prof_summary.py stats gpurun_out/prof_${TAG}_$name gpurun_out/stats_${TAG}_$name.md > /dev/null
done
