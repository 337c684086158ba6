#!/bin/bash
# d = 4096 register-transform kernels: their parity tests, then a d = 4096 bench line
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-n4k}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -k "4096" -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --d 4096 --w 1024 --kappa 64 --no-small-shape --no-cpu-baseline --steps 20 --warmup 3 > gpurun_out/bench_$TAG.log 2>&1
rc=$?; echo "bench rc=$rc"; grep -h '^{' gpurun_out/bench_$TAG.log | tail -1 | cut -c1-600; exit $rc
