"""Debug aid: one batch of Ajtai commitments (lf_dev_ajtai_commit) on fixed seeded
inputs, saved to gpurun_out/ajdump_<tag>.npy; with two tags, prints where they differ
(how an opt-in contraction variant was checked against the default one).
usage: python tools/exp/ajtai_dump.py TAG d ncols [REFTAG]"""
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import latticeum_amd as LA  # noqa: E402

tag = sys.argv[1]
d, kappa, ncols, nvec = int(sys.argv[2]), 32, int(sys.argv[3]), 29
ctx = LA.Context(0)
ctx.set_stream(torch.cuda.current_stream().cuda_stream)
A = torch.empty(kappa * ncols * d, dtype=torch.int64, device="cuda")
ctx.dev_fill_uniform(A, 5)
sch = LA.AjtaiCommitmentScheme(ctx, device_tensor=A, kappa=kappa, ncols=ncols, d=d)
vecs = [torch.empty(ncols * d, dtype=torch.int64, device="cuda") for _ in range(nvec)]
for i, v in enumerate(vecs):
    ctx.dev_fill_uniform(v, 100 + i)
cm = torch.empty(nvec * kappa * d, dtype=torch.int64, device="cuda")
ctx.dev_ajtai_commit(sch, vecs, cm)
ctx.sync()
out = cm.cpu().numpy().view(np.uint64).reshape(nvec, kappa, d)
np.save(f"gpurun_out/ajdump_{tag}.npy", out)
if len(sys.argv) > 4:
    ref = np.load(f"gpurun_out/ajdump_{sys.argv[4]}.npy")
    bad = ref != out
    print("mismatch", bad.sum(), "of", bad.size)
    if bad.any():
        v, r, s = np.nonzero(bad)
        print("vectors", np.unique(v)[:40])
        print("rows", np.unique(r)[:40])
        print("slots", np.unique(s)[:40], "count", len(np.unique(s)))
        print("first", v[0], r[0], s[0], hex(int(ref[v[0], r[0], s[0]])), hex(int(out[v[0], r[0], s[0]])))
