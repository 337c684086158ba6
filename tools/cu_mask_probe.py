"""Phase times of the d=1024 W=2^14 step on a stream restricted to n CUs
(lf_stream_create_cu_mask), for n in a list, and two concurrent step streams on
complementary masks -- how far the phases scale with CUs.
usage: python tools/cu_mask_probe.py [--w 16384] [--cus 256,192,160,128,96,64] [--pattern spread|block]"""
import argparse
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

import bench  # noqa: E402
import latticeum_amd as LA  # noqa: E402


def cu_set(n, pattern, total=256, offset=0):
    if pattern == "block":
        return [(offset + i) % total for i in range(n)]
    # spread: n CUs evenly over the index space
    return sorted({(offset + (i * total) // n) % total for i in range(n)})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--w", type=int, default=1 << 14)
    ap.add_argument("--cus", default="256,192,160,128,96,64")
    ap.add_argument("--pattern", default="spread")
    ap.add_argument("--steps", type=int, default=4)
    a = ap.parse_args()
    wl = bench.Workload(LA, torch, 0, 0, 1024, a.w, 32, 2)
    out = {}
    for n in [int(x) for x in a.cus.split(",")]:
        c = wl.ctxs[0]
        st = c.use_cu_mask(cu_set(n, a.pattern))
        wl.run(1, streams=1)
        wl.sync()
        c.kernel_timing(True)
        t0 = time.perf_counter()
        wl.run(a.steps, streams=1)
        wl.sync()
        dt = (time.perf_counter() - t0) / a.steps * 1e3
        tot = wl.phase_totals()
        wl.timing(False)
        out[n] = {"ms_per_step": dt, **{k: v[0] / max(1, v[1]) for k, v in tot.items() if v[1]}}
        print(json.dumps({"cus": n, **{k: round(v, 3) for k, v in out[n].items()}}), flush=True)
        c.set_stream(torch.cuda.current_stream().cuda_stream)
        c.lib.lf_stream_destroy(st)
        c._masked.remove(st)
    wl.close()


if __name__ == "__main__":
    main()
