#!/bin/bash
# SQ counters of fold() at the zkvm shape (tools/fold_prof.py), one --pmc pass
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-pmcfold}
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
  SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_WAVES GRBM_GUI_ACTIVE -d gpurun_out/pmcs_$TAG -o run --output-format csv -- \
  python tools/fold_prof.py $FOLD_ARGS > gpurun_out/pmcs_$TAG.log 2>&1
rc=$?; echo "pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 - <<PY
import csv, glob, collections, re
f=glob.glob('gpurun_out/pmcs_$TAG/**/*counter_collection.csv', recursive=True)[0]
rows=list(csv.DictReader(open(f)))
agg=collections.defaultdict(lambda: collections.defaultdict(float)); cnt=collections.Counter()
for r in rows:
    m=re.search(r'k_\w+(<[^>]*>)?', r['Kernel_Name']); k=m.group(0) if m else r['Kernel_Name'][:30]
    agg[k][r['Counter_Name']]+=float(r['Counter_Value'])
for k,v in sorted(agg.items(), key=lambda x:-x[1].get('GRBM_GUI_ACTIVE',0))[:12]:
    g=v.get('GRBM_GUI_ACTIVE',1)
    print(f"{k[:32]:32s} gui {g:12.0f} valu_inst {v.get('SQ_INSTS_VALU',0):14.0f} active_valu/gui {4*v.get('SQ_ACTIVE_INST_VALU',0)/(1024*g/8 if g else 1):6.3f} wave_cyc {v.get('SQ_WAVE_CYCLES',0):14.0f} wait_any {v.get('SQ_WAIT_ANY',0):14.0f} waves {v.get('SQ_WAVES',0):10.0f}")
PY
