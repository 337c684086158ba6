#!/bin/bash
# GPU validation: parity tests, then (only if no crash) a small bench + rocprof kernel stats
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -25 gpurun_out/pytest_gpu.log
if [ $rc -le 1 ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_small -o run --output-format csv -- \
    python bench.py --w 1024 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_small.log 2>&1
  echo "bench rc=$?"
  tail -3 gpurun_out/bench_small.log
  find gpurun_out/prof_small -name "*kernel_stats.csv" | head -1 | xargs -r cat | cut -d, -f1-8 | head -30
fi
