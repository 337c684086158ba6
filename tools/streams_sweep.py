"""Diagnostic: commit+fold steps/s vs concurrent step streams per GPU.
usage: python tools/streams_sweep.py D W KAPPA S1,S2,... [STEPS]"""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
sys.path.insert(0, str(Path(__file__).resolve().parent))
import configs_bench as CB  # noqa: E402

d, W, kappa = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
steps = int(sys.argv[5]) if len(sys.argv) > 5 else 256
out = {}
for S in (int(x) for x in sys.argv[4].split(",")):
    out[S] = CB.fold_steps(d, W, kappa, S, steps, max(2, steps // 16))["steps_per_s"]
    print(json.dumps(out), flush=True)
