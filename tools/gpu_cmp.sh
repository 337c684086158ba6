#!/bin/bash
# side workloads A/B: the reference ring (4 streams) and the small shape, with the
# register-A contraction on (default) and off (LATTICEUM_AMD_AJTAI_RA=0), plus fold variants
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-cmp}
show() {
  python3 - "$1" "$2" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        j = json.loads(line); ph = j["phases"]
        print(sys.argv[2], round(j["value"], 1), " ".join(f"{k} {v['avg_launch_ms']:.3f}" for k, v in ph.items()))
PY
}
for REP in 1 2; do
for RA in 4 0; do
  export LATTICEUM_AMD_AJTAI_RA=$RA
  timeout -k 10 120 python3 -u bench.py --d 24 --w 19763 --streams 4 --steps 256 --warmup 8 --no-small-shape --no-cpu-baseline > gpurun_out/${TAG}_p24_$RA.log 2>&1 || exit 1
  show gpurun_out/${TAG}_p24_$RA.log "phi72 RA=$RA"
  for FV in coeff slot; do
    if [ $FV = slot ]; then export LATTICEUM_AMD_FOLD=slot; else unset LATTICEUM_AMD_FOLD; fi
    for S in 4 8; do
      timeout -k 10 120 python3 -u bench.py --w 464 --streams $S --steps 512 --warmup 16 --no-small-shape --no-cpu-baseline > gpurun_out/${TAG}_small_${RA}_${FV}_$S.log 2>&1 || exit 1
      show gpurun_out/${TAG}_small_${RA}_${FV}_$S.log "small RA=$RA fold=$FV streams=$S"
    done
  done
  unset LATTICEUM_AMD_FOLD
done
done
