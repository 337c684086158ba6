#!/bin/bash
# GPU suite, the W = 464 line (4 streams), and kernel stats of W = 464 on one
# stream (each kernel's own duration, no overlap)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-w464}
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
fi
for i in 1 2; do
timeout -k 10 300 python -u bench.py --no-small-shape --no-cpu-baseline --w 464 --streams 4 --batch 0 --steps 256 --warmup 16 \
  > gpurun_out/bench_${TAG}_$i.log 2>&1 || exit 1
python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/bench_${TAG}_$i.log') if l.startswith('{')][-1])
print(round(d['value'],1), round(d['ms_per_step'],3), {k: round(v['avg_launch_ms'],3) for k,v in d['phases'].items()})"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_1s -o run --output-format csv -- \
  python bench.py --no-cpu-baseline --no-small-shape --w 464 --streams 1 --steps 64 --warmup 8 > gpurun_out/benchprof_${TAG}_1s.log 2>&1 && \
python tools/prof_summary.py stats gpurun_out/prof_${TAG}_1s gpurun_out/stats_${TAG}_1s.md > /dev/null; echo "prof rc=$?"
head -24 gpurun_out/stats_${TAG}_1s.md
