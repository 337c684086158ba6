"""Probe (diagnostic only): fold-step throughput at a small W with S step streams
(one lf context + HIP stream + buffer set each, sharing the Ajtai scheme)."""
import sys, time
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import numpy as np
import torch
import latticeum_amd as LA

W = int(sys.argv[1]) if len(sys.argv) > 1 else 464
STEPS = 64
d, kappa = 1024, 32
pr = LA.goldilocks_dp(d)
K, L = pr.K, pr.L
N = W * L
i64 = dict(dtype=torch.int64, device="cuda:0")
z = lambda n: torch.empty(n, **i64)
ctx0 = LA.Context(0)
A = z(kappa * N * d)
ctx0.dev_fill_uniform(A, 1)
sch = LA.AjtaiCommitmentScheme(ctx0, device_tensor=A, kappa=kappa, ncols=N, d=d)
del A


def make(ctx, seed):
    keep = {"w_ccs": z(W * d), "acc_cm": z(kappa * d), "acc_f_coeff": z(N * d), "rho": z(2 * K * d),
            "f_coeff": z(N * d), "f": z(N * d), "cm": z(kappa * d),
            "fk_coeff": [z(K * N * d) for _ in range(2)], "fk": [z(K * N * d) for _ in range(2)],
            "wk": [z(K * W * d) for _ in range(2)], "y": [z(K * kappa * d) for _ in range(2)],
            "f0": z(N * d), "f0_coeff": z(N * d), "w_ccs0": z(W * d), "cm0": z(kappa * d)}
    ctx.dev_fill_uniform(keep["w_ccs"], seed)
    ctx.dev_fill_uniform(keep["acc_cm"], seed + 1)
    # small-digit accumulator coefficients and short rho: any values decompose
    keep["acc_f_coeff"].copy_(torch.randint(-3000, 3000, (N * d,), **i64) % ((1 << 64) - (1 << 32) + 1) if False else torch.randint(0, 3000, (N * d,), **i64))
    keep["rho"].copy_(torch.randint(0, 64, (2 * K * d,), **i64))
    bufs = LA.LfFoldStepBufs()
    for k, v in keep.items():
        if isinstance(v, list):
            for s in range(2):
                getattr(bufs, k)[s] = v[s].data_ptr()
        else:
            setattr(bufs, k, v.data_ptr())
    ctx.reserve(kappa, N, d, 2 * (K - 1) + 1)
    return keep, bufs


for S in (1, 2, 4, 8):
    ctxs, streams, sets = [], [], []
    for i in range(S):
        c = ctx0 if i == 0 else LA.Context(0)
        st = torch.cuda.Stream()
        c.set_stream(st.cuda_stream)
        ctxs.append(c); streams.append(st); sets.append(make(c, 100 + i))
    for i in range(S):
        for _ in range(2):
            ctxs[i].dev_fold_step(sch, pr, W, sets[i][1])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for it in range(STEPS):
        i = it % S
        ctxs[i].dev_fold_step(sch, pr, W, sets[i][1])
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"W={W} streams={S}: {STEPS / dt:.1f} steps/s ({dt / STEPS * 1e3:.3f} ms/step)", flush=True)
    for c in ctxs:
        c.sync()
    del ctxs[1:], sets
