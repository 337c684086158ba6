"""fold() at the zkvm's shape (bench.py next_rows' CCS and fold_prove_line) on its
own, for rocprofv3 kernel traces of lf_fold_prove: `python tools/fold_prof.py [--scalar]`
prints the line bench.py reports as next_rows.fold_prove (with --scalar:
next_rows.fold_prove_scalar, the same rows with scalar values as the zkvm's)."""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402


def main():
    import torch
    import latticeum_amd as LA
    torch.cuda.set_device(0)
    ctx = LA.Context(0)
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    d, nv, t, mm, nn = 24, 17, 125, 1 << 17, 19768
    i64 = dict(dtype=torch.int64, device="cuda:0")
    rng = np.random.default_rng(0x4C460014)
    S = [list(rng.integers(0, 125, 7)) for _ in range(16)] + [list(rng.integers(0, 125, 1 + (i % 2))) for i in range(36)]
    S = [[int(j) for j in x] for x in S]
    rng = np.random.default_rng(0x4C460012)
    mats, nnz = [], 0
    for j in range(t):
        cnt = rng.integers(0, 3, mm)
        rp = np.concatenate([[0], np.cumsum(cnt)]).astype(np.uint64)
        mats.append([rp, rng.integers(0, nn, int(rp[-1])).astype(np.uint32), None])
        nnz += int(rp[-1])
    if "--scalar" in sys.argv:
        sv = torch.empty(nnz, **i64)
        ctx.dev_fill_uniform(sv, 0x4C460019)
        hv = np.zeros((nnz, d), np.uint64)
        hv[:, ::3] = sv.cpu().numpy().view(np.uint64)[:, None]
        hv = hv.ravel()
    else:
        vals = torch.empty(nnz * d, **i64)
        ctx.dev_fill_uniform(vals, 0x4C460013)
        hv = vals.cpu().numpy().view(np.uint64)
    off = 0
    for mt in mats:
        k = int(mt[0][-1])
        mt[2] = hv[off * d:(off + k) * d]
        off += k
    M = LA.CCSMatrices(ctx, d, mm, nn, mats)
    out = bench.fold_prove_line(LA, torch, ctx, M, S, d, nn, t, mm)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
