"""A/B of the fold-step phases (diagnostic): one bench workload, the phase
times of a few steps under each value of an environment variable read per call.
usage: python tools/fold_ab.py VAR v1 v2 ... [--d 1024 --w 16384 --kappa 32 --steps 3]"""
import argparse
import json
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

import bench  # noqa: E402
import latticeum_amd as LA  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("var")
    ap.add_argument("values", nargs="+")
    ap.add_argument("--d", type=int, default=1024)
    ap.add_argument("--w", type=int, default=1 << 14)
    ap.add_argument("--kappa", type=int, default=32)
    ap.add_argument("--steps", type=int, default=3)
    a = ap.parse_args()
    wl = bench.Workload(LA, torch, 0, 0, a.d, a.w, a.kappa, 1)
    c = wl.ctxs[0]
    wl.run(1)
    wl.sync()
    for v in a.values:
        os.environ[a.var] = v
        wl.run(1)  # warm
        wl.sync()
        c.kernel_timing(True)
        before = {p: c.phase_stats(p) for p in c.PHASES}
        wl.run(a.steps)
        wl.sync()
        res = {a.var: v}
        for p in c.PHASES:
            ms, cnt = c.phase_stats(p)
            dms, dc = ms - before[p][0], cnt - before[p][1]
            if dc:
                res[p] = round(dms / a.steps, 3)
        c.kernel_timing(False)
        print(json.dumps(res), flush=True)
    wl.close()


if __name__ == "__main__":
    main()
