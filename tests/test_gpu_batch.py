"""GPU parity of lf_dev_fold_step_batch: several independent commit+fold steps
(each its own context, stream and buffers, one Ajtai scheme) whose commitment
contractions share one launch -- every step's outputs equal the oracle's step,
as lf_dev_fold_step's do (tests/test_gpu_parity.py::check_dev_fold_step)."""
import numpy as np
import pytest

import latticeum_amd as LA
import oracle as O
from test_gpu_parity import check_fold_outputs, make_rho, params, rand, valid_f_coeff

pytestmark = pytest.mark.gpu


def planes_u64(d, K, N):
    """u64 words of one side's packed planes (lf.h lf_fold_step_bufs.planes)"""
    return K * N if d == 24 else N * 256 if d == 1024 else N * K * 128


def make_step(torch, A, kappa, d, W, seed, packed, keep_fk=True, rho=None, zero_w=False):
    pr = params(d)
    K, L = pr.K, pr.L
    N = W * L
    dev = lambda x: torch.from_numpy(np.ascontiguousarray(x).view(np.int64)).cuda()
    z = lambda n: torch.zeros(n, dtype=torch.int64, device="cuda")
    # zero_w: a zero witness, so every digit plane of the step's new side is zero
    # (all its operand units dead: never written, read as the offset form of 0)
    w_ccs = np.zeros(W * d, np.uint64) if zero_w else rand(W * d, seed)
    acc_fc, acc_f = valid_f_coeff(d, W, seed + 1)
    acc_cm = O.ajtai_commit(A, kappa, N, d, acc_f)
    if rho is None:
        rho = make_rho(d, K, seed + 2)
    keep = {
        "w_ccs": dev(w_ccs), "acc_cm": dev(acc_cm), "acc_f_coeff": dev(acc_fc), "rho": dev(rho),
        "f_coeff": z(N * d), "f": z(N * d), "cm": z(kappa * d),
        "fk_coeff": [z(K * N * d) for _ in range(2)] if not packed else [None, None],
        "fk": [z(K * N * d) for _ in range(2)] if keep_fk and not packed else [None, None],
        "wk": [z(K * W * d) for _ in range(2)], "y": [z(K * kappa * d) for _ in range(2)],
        "f0": z(N * d), "f0_coeff": z(N * d), "w_ccs0": z(W * d), "cm0": z(kappa * d),
        "planes": [z(planes_u64(d, K, N)) for _ in range(2)] if packed else [None, None],
    }
    b = LA.LfFoldStepBufs()
    for k, v in keep.items():
        if isinstance(v, list):
            for s in range(2):
                getattr(b, k)[s] = v[s].data_ptr() if v[s] is not None else None
        else:
            setattr(b, k, v.data_ptr())
    return {"keep": keep, "b": b, "w_ccs": w_ccs, "acc_cm": acc_cm, "acc_fc": acc_fc, "rho": rho}


def expand(ctx, torch, pr, keep, N, d):
    """the packed planes as the u64 rows the oracle returns (lf_dev_expand_planes)"""
    K = pr.K
    for s in range(2):
        fck = torch.zeros(K * N * d, dtype=torch.int64, device="cuda")
        fk = torch.zeros(K * N * d, dtype=torch.int64, device="cuda")
        torch.cuda.synchronize()  # torch's fills before the context's own stream writes the rows
        ctx.dev_expand_planes(pr, keep["planes"][s], N, fck, fk)
        ctx.sync()
        keep["fk_coeff"][s], keep["fk"][s] = fck, fk


def run_batch(d, W, kappa, S, packed, rounds=1, rho_long=False, cu_split=0, zero_w=False):
    import torch
    pr = params(d)
    N = W * pr.L
    A = rand(kappa * N * d, 7000 + d)
    ctxs = [LA.Context(0) for _ in range(S)]
    try:
        if cu_split:  # bench.py --cu-split: step streams and the contraction on disjoint CUs
            ncu = torch.cuda.get_device_properties(0).multi_processor_count
            for c in ctxs:
                c.use_cu_mask(range(ncu - cu_split))
            ctxs[0].set_contract_stream(ctxs[0].cu_mask_stream(range(ncu - cu_split, ncu)))
        At = torch.from_numpy(A.view(np.int64)).cuda()
        sch = LA.AjtaiCommitmentScheme(ctxs[0], device_tensor=At, kappa=kappa, ncols=N, d=d)
        for rnd in range(rounds):
            steps = [make_step(torch, A, kappa, d, W, 100 * rnd + 10 * i + 1, packed,
                               rho=rand(2 * pr.K * d, 900 + i) if rho_long and i % 2 else None,
                               zero_w=zero_w and i % 2 == 1)
                     for i in range(S)]
            torch.cuda.synchronize()  # torch wrote the inputs on its own stream
            ctxs[0].dev_fold_step_batch(ctxs[1:], sch, pr, W, [st["b"] for st in steps])
            for c in ctxs:
                c.sync()
            h = lambda t: t.cpu().numpy().view(np.uint64)
            for i, st in enumerate(steps):
                if packed:
                    expand(ctxs[0], torch, pr, st["keep"], N, d)
                check_fold_outputs(h, st["keep"], A, kappa, d, pr, W, st["w_ccs"], st["acc_cm"], st["acc_fc"],
                                   st["rho"])
    finally:
        for c in ctxs:
            c.close()


@pytest.mark.parametrize("d,W,kappa,S", [(1024, 37, 2, 2), (1024, 130, 2, 4), (24, 17, 3, 3), (24, 70, 3, 4),
                                         (4096, 17, 2, 2)])
def test_fold_step_batch_matches_oracle(d, W, kappa, S):
    run_batch(d, W, kappa, S, packed=False)


@pytest.mark.parametrize("d,W,S", [(1024, 37, 4), (1024, 37, 8), (24, 70, 4), (4096, 17, 4), (4096, 33, 2)])
def test_fold_step_batch_packed_planes(d, W, S):
    """the bench's configuration: packed digit planes, four or eight steps per batch, two
    batches on the same contexts (each batch's contraction must see its own rows);
    d = 4096 folds f_0 from the quarter-major operand rows (k_fold_frag)"""
    run_batch(d, W, 3 if d == 24 else 2, S, packed=True, rounds=2)


@pytest.mark.parametrize("d,S", [(1024, 4), (24, 2), (4096, 2)])
def test_fold_step_batch_contract_stream(d, S):
    """the group's contraction on a stream of its own (lf_ctx_set_contract_stream,
    a CU-masked stream beside the step streams' CUs): every step waits for its
    decomposition before the contraction and for the contraction after it"""
    run_batch(d, 37 if d == 1024 else 17, 3 if d == 24 else 2, S, packed=True, rounds=2, cu_split=64)


@pytest.mark.parametrize("d", [24, 1024, 4096])
def test_fold_step_batch_zero_witness(d):
    """every other step of the batch folds a zero witness: all of its new side's
    digit planes are zero, so every one of its operand units is dead (unwritten,
    read as the offset form of 0) next to steps whose units are live, and the
    d = 4096 matrix-core stage 1 and the fold from the rows skip them"""
    run_batch(d, 37 if d == 1024 else 17, 3 if d == 24 else 2, 4 if d != 4096 else 2, packed=True, rounds=2,
              zero_w=True)


def test_fold_step_batch_wide_kappa():
    """kappa > 32: two 32-row A tiles x two steps per launch group"""
    run_batch(1024, 37, 40, 2, packed=True)


@pytest.mark.parametrize("d", [24, 1024, 4096])
def test_fold_step_batch_rho_not_short(d):
    """steps of one batch taking different fold paths (short and full-size rho)"""
    run_batch(d, 17, 3 if d == 24 else 2, 2, packed=True, rho_long=True)


def test_fold_step_batch_rejects_bad_arguments():
    import torch
    d, W, kappa = 1024, 2, 2
    pr = params(d)
    N = W * pr.L
    A = rand(kappa * N * d, 7)
    c = LA.Context(0)
    try:
        sch = LA.AjtaiCommitmentScheme(c, device_tensor=torch.from_numpy(A.view(np.int64)).cuda(), kappa=kappa,
                                       ncols=N, d=d)
        st = make_step(torch, A, kappa, d, W, 5, packed=True)
        with pytest.raises(LA.LfError):  # the same context twice
            c.dev_fold_step_batch([c], sch, pr, W, [st["b"], st["b"]])
        others = [LA.Context(0) for _ in range(8)]
        try:
            with pytest.raises(LA.LfError):  # more steps than one launch takes (8)
                c.dev_fold_step_batch(others, sch, pr, W, [st["b"]] * 9)
        finally:
            for o in others:
                o.close()
    finally:
        c.close()
