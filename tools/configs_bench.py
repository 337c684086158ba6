"""Side measurements for the other BASELINE.json configs (diagnostic; bench.py
reports the headline). usage: python tools/configs_bench.py [--what ntt,phi72,d24,d4096,p2]"""
import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402

import bench  # noqa: E402
import latticeum_amd as LA  # noqa: E402


def ev_time(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def transforms(ctx, d, n, seed, reps=10):
    x = torch.empty(n * d, dtype=torch.int64, device="cuda")
    ctx.dev_fill_uniform(x, seed)
    f = ev_time(lambda: ctx.dev_crt(x, d), reps)
    i = ev_time(lambda: ctx.dev_icrt(x, d), reps)
    by = 2 * n * d * 8
    return {"d": d, "npoly": n, "fwd_ms": f, "inv_ms": i, "fwd_GBs": by / f / 1e6, "inv_GBs": by / i / 1e6,
            "frac_hbm_fwd": by / f / 1e6 / bench.HBM_PEAK_GBS, "polys_per_s_fwd": n / f * 1e3}


def fold_steps(d, W, kappa, streams, steps, warmup):
    wl = bench.Workload(LA, torch, 0, 0, d, W, kappa, streams)
    wl.run(warmup)
    wl.sync()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    wl.run(steps)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    wl.close()
    step_bytes, _ = bench.algorithmic_bytes(d, W, kappa)
    v = steps / dt
    return {"d": d, "W": W, "kappa": kappa, "streams": streams, "steps_per_s": v, "ms_per_step": dt / steps * 1e3,
            "GBs_algorithmic": step_bytes * v / 1e9}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--what", default="ntt,phi72,d24,d4096,p2")
    a = ap.parse_args()
    what = a.what.split(",")
    ctx = LA.Context(0)
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    out = {}
    if "ntt" in what:
        out["ntt_d1024"] = transforms(ctx, 1024, 1 << 16, bench.SEED_W - 2)
    if "phi72" in what:
        out["crt_phi72"] = transforms(ctx, 24, 1 << 22, bench.SEED_W - 1)
    if "p2" in what:
        n = 1 << 20
        s = torch.empty(16 * n, dtype=torch.int64, device="cuda")
        ctx.dev_fill_uniform(s, 0x4C460007)
        ms = ev_time(lambda: ctx.dev_poseidon2_permute(s), 10)
        out["poseidon2_w16"] = {"states": n, "ms": ms, "perms_per_s": n / ms * 1e3}
    ctx.sync()
    torch.cuda.empty_cache()
    print(json.dumps(out), flush=True)
    if "d24" in what:
        for S in (1, 4):
            out[f"d24_real_W19763_s{S}"] = fold_steps(24, 19763, 32, S, 64, 8)
            torch.cuda.empty_cache()
            print(json.dumps(out), flush=True)
    if "d4096" in what:
        out["d4096_k64_W1024"] = fold_steps(4096, 1024, 64, 1, 3, 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
