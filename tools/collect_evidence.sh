#!/bin/bash
# copy a gpu_evidence.sh run's summaries from gpurun_out/ into profiles/ (committed):
# the per-line PMC files bench.py reads, the bench line, the rocprof kernel-trace
# summary with its roctx windows, and the line-vs-trace check
TAG=${1:?tag}; R=${2:-r06}
cd "$(dirname "$0")/.." || exit 1
cp gpurun_out/pmc_traffic_d*_W*_k*.json gpurun_out/pmc_sq_d*_W*_k*.json profiles/ 2>/dev/null
# (tools/gpu_pmc_side.sh writes profiles/pmc_{traffic,sq}_side_ops.json on the box: merged back by gpurun_out only)
cp gpurun_out/pmc_side/pmc_*_side_ops.json profiles/ 2>/dev/null
grep "^{" gpurun_out/bench_$TAG.log | tail -1 > profiles/${R}_bench.json
grep "^{" gpurun_out/benchprof_$TAG.log | tail -1 > profiles/${R}_benchprof.json
cp gpurun_out/bench_detail_$TAG.json profiles/${R}_bench_detail.json
cp gpurun_out/benchprof_detail_$TAG.json profiles/${R}_benchprof_detail.json
cp gpurun_out/stats_$TAG.md profiles/${R}_rocprof_stats_windows.md
cp gpurun_out/stats_$TAG.windows.json profiles/${R}_rocprof_stats_windows.json
python tools/check_profile.py gpurun_out/benchprof_$TAG.log gpurun_out/stats_$TAG.windows.json > profiles/${R}_check_profile.txt
python tools/check_profile.py gpurun_out/bench_$TAG.log gpurun_out/stats_$TAG.windows.json > profiles/${R}_check_bench_vs_trace.txt
exit 0
