"""The W = 464 line's timed steps under a kernel trace: the bench workload (4 step
streams, contractions batched in pairs), warmed up, then STEPS steps inside one
roctx range `timed_steps` (rocprofv3 --kernel-trace --marker-trace keeps the
range); tools/trace_busy.py reads the trace.
usage: rocprofv3 --kernel-trace --marker-trace -d DIR -o run --output-format csv -- \
       python tools/w464_trace.py [--w 464] [--streams 4] [--batch 2] [--steps 128]"""
import argparse
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

import bench  # noqa: E402
import latticeum_amd as LA  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--w", type=int, default=464)
    ap.add_argument("--d", type=int, default=1024)
    ap.add_argument("--kappa", type=int, default=32)
    ap.add_argument("--streams", type=int, default=4)
    ap.add_argument("--batch", type=int, default=2)
    ap.add_argument("--steps", type=int, default=128)
    a = ap.parse_args()
    wl = bench.Workload(LA, torch, 0, 0, a.d, a.w, a.kappa, a.streams, batch=a.batch)
    wl.run(4 * max(1, wl.group))
    wl.sync()
    torch.cuda.synchronize()
    bench.ROCTX.push("timed_steps")
    t0 = time.perf_counter()
    wl.run(a.steps)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    bench.ROCTX.pop()
    print(f"{a.steps} steps in {dt * 1e3:.2f} ms: {a.steps / dt:.1f} steps/s", flush=True)
    wl.close()


if __name__ == "__main__":
    main()
