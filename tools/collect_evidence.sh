#!/bin/bash
# copy a gpu_evidence.sh run's summaries from gpurun_out/ into profiles/ (committed)
TAG=${1:?tag}; R=${2:-r01}
cd "$(dirname "$0")/.." || exit 1
cp gpurun_out/pmc_traffic_$TAG.json profiles/pmc_traffic.json
[ -f gpurun_out/pmc_sq_$TAG.json ] && cp gpurun_out/pmc_sq_$TAG.json profiles/pmc_sq.json
[ -f gpurun_out/pmc_traffic_d24_$TAG.json ] && cp gpurun_out/pmc_traffic_d24_$TAG.json profiles/pmc_traffic_d24.json
[ -f gpurun_out/pmc_sq_d24_$TAG.json ] && cp gpurun_out/pmc_sq_d24_$TAG.json profiles/pmc_sq_d24.json
grep "^{" gpurun_out/bench_${BENCH_TAG:-$TAG}.log | tail -1 > profiles/${R}_bench.json
for name in d1024_W16384 d1024_W464 d24_W19763 d4096_W1024; do
  cp gpurun_out/stats_${TAG}_$name.md profiles/${R}_rocprof_stats_$name.md
  grep "^{" gpurun_out/benchprof_${TAG}_$name.log | tail -1 > profiles/${R}_benchprof_$name.json
done
