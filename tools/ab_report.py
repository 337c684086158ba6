"""Summarise tools/ab.sh output: per variant, steps/s and per-phase ms of each run."""
import json, sys, glob, os
tag = os.environ.get("TAG", "")
for v in sys.argv[1:]:
    for f in sorted(glob.glob(f"gpurun_out/ab_{tag}{v}_*.log")):
        j = json.loads(open(f).read().strip().splitlines()[-1])
        ph = {k: round(p["avg_launch_ms"], 3) for k, p in j["phases"].items()}
        print(f"{v:>8s} {os.path.basename(f)[-5]} {j['value']:.2f}", ph)
