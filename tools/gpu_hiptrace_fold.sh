#!/bin/bash
# host-side HIP API time inside fold() (tools/fold_prof.py --scalar): which runtime calls
# the host thread spends its time in between transcript work
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-hiptrace}
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace -d gpurun_out/ht_$TAG -o run --output-format csv -- \
  python tools/fold_prof.py --scalar > gpurun_out/ht_$TAG.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 - <<PY > gpurun_out/ht_${TAG}_summary.txt
import csv, glob, collections
f=glob.glob('gpurun_out/ht_$TAG/**/*hip_api_trace.csv', recursive=True)[0]
k=glob.glob('gpurun_out/ht_$TAG/**/*kernel_trace.csv', recursive=True)[0]
ks=sorted(int(r['Start_Timestamp']) for r in csv.DictReader(open(k)) if 'k_decompose_phi72_w' in r['Kernel_Name'])
a,b=ks[2],ks[3]
tot=collections.defaultdict(float); cnt=collections.Counter()
for r in csv.DictReader(open(f)):
    s,e=int(r['Start_Timestamp']),int(r['End_Timestamp'])
    if a<=s<b:
        tot[r['Function']]+=(e-s)/1e6; cnt[r['Function']]+=1
print('fold window ms', (b-a)/1e6)
for n,v in sorted(tot.items(), key=lambda x:-x[1])[:25]: print(f"{n:40s} {cnt[n]:6d} {v:8.3f} ms")
PY
cat gpurun_out/ht_${TAG}_summary.txt
