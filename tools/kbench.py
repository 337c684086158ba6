"""Kernel micro-benchmarks (diagnostic): time individual device ops on synthetic data.
usage: python tools/kbench.py [--n 81920]"""
import argparse
import json
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

import latticeum_amd as LA  # noqa: E402


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=81920)
    ap.add_argument("--d", type=int, default=1024)
    a = ap.parse_args()
    ctx = LA.Context(0)
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    d, n = a.d, a.n
    pr = LA.goldilocks_dp(d)
    x = torch.empty(n * d, dtype=torch.int64, device="cuda")
    ctx.dev_fill_uniform(x, 1)
    res = {"variant": os.environ.get("LATTICEUM_AMD_NTT", "default"), "d": d, "n": n}
    res["crt_ms"] = timeit(lambda: ctx.dev_crt(x, d))
    res["icrt_ms"] = timeit(lambda: ctx.dev_icrt(x, d))
    W = n // pr.L
    w = torch.empty(W * d, dtype=torch.int64, device="cuda")
    ctx.dev_fill_uniform(w, 2)
    fc, f = torch.empty(n * d, dtype=torch.int64, device="cuda"), torch.empty(n * d, dtype=torch.int64, device="cuda")
    C = LA._lib.C
    res["from_w_ccs_ms"] = timeit(lambda: ctx.check(ctx.lib.lf_dev_witness_from_w_ccs(
        ctx.h, C.byref(pr), w.data_ptr(), W, fc.data_ptr(), f.data_ptr())))
    K = pr.K
    fck, fk = torch.empty(K * n * d, dtype=torch.int64, device="cuda"), torch.empty(K * n * d, dtype=torch.int64, device="cuda")
    wk = torch.empty(K * W * d, dtype=torch.int64, device="cuda")
    res["decompose_ms"] = timeit(lambda: ctx.check(ctx.lib.lf_dev_decompose_witness(
        ctx.h, C.byref(pr), fc.data_ptr(), n, fck.data_ptr(), fk.data_ptr(), wk.data_ptr())), reps=3)
    res["from_f_ms"] = timeit(lambda: ctx.check(ctx.lib.lf_dev_witness_from_f(
        ctx.h, C.byref(pr), f.data_ptr(), n, fc.data_ptr(), w.data_ptr())))
    ctx.sync()
    bytes_xf = 2 * n * d * 8
    res["crt_GBs"] = bytes_xf / res["crt_ms"] / 1e6
    res["ntt_per_s_crt"] = n / res["crt_ms"] * 1e3
    print(json.dumps(res))


if __name__ == "__main__":
    main()
