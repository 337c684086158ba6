"""Multi-GPU plumbing: one process per GPU, torch.distributed for rendezvous and
timing, RCCL over xGMI (through the C ABI's lf_comm) for the field exchange.

Two ways to spread the commit+fold path over the GPUs of a node:

* independent step streams (BASELINE.json configs[3], the trace-batch shard):
  every rank folds its own trace-step witnesses. Steps never exchange data,
  so there is no collective on the data path (weak scaling), and the ranks'
  accumulators stay separate: summing unrelated accumulators has no
  LatticeFold meaning, so bench.py's N > 1 line does not do it.
  ``AccumulatorReducer`` (lf_fold_reduce_allranks, a mod-p sum of field
  vectors over ranks) remains as a plumbing utility for callers that do own
  a sum over ranks; nothing on the measured path calls it.
* one fold sharded by columns: rank r owns the witness
  columns of groups ``shard_groups(W, r, world)`` and the matching columns of
  the Ajtai matrix. The commitments are sums over columns, so each rank's are
  partial sums; one RCCL all-reduce (mod p) of the 1 + 2(K-1) kappa-element
  commitments per step completes them (lf_dev_fold_step_sharded). f_0 and
  Witness::from_f(f_0) are column-local and stay sharded.

RCCL's integer SUM is mod 2^64, not mod p = 2^64 - 2^32 + 1, so field vectors
travel as 32-bit limbs and are folded back into the field by a HIP kernel; the
whole exchange (split, all-reduce, join) is ordered on the context's stream.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def init(world: int):
    if world <= 1:
        return None
    if not dist.is_initialized():
        backend = "nccl" if torch.cuda.is_available() else "gloo"
        if os.environ.get("LATTICEUM_AMD_REHEARSE_ONE_GPU") == "1":
            backend = "gloo"  # bench.py's one-GPU rehearsal of N ranks
        dist.init_process_group(backend=backend, init_method="env://")
    return dist.group.WORLD


def barrier(pg):
    if pg is not None:
        dist.barrier(group=pg)


def max_over_ranks(pg, value: float) -> float:
    if pg is None:
        return value
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(pg) == "nccl" else "cpu"
    t = torch.tensor([value], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=pg)
    return float(t.item())


def finalize(pg):
    if pg is not None and dist.is_initialized():
        dist.destroy_process_group()


def make_comm(ctx, pg, world: int, rank: int):
    """The lf communicator of this rank: rank 0 makes the RCCL unique id and
    torch.distributed carries it to the others (a Rust host would use its own
    channel). None for a single rank."""
    if world <= 1:
        return None
    from . import Communicator
    obj = [Communicator.unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0, group=pg)
    return Communicator(ctx, world, rank, obj[0])


def shard_groups(W: int, rank: int, world: int, align: int = 16):
    """[g0, g1): the groups (of L witness columns) rank owns in a column-sharded
    fold. Shards are contiguous and, except the last, multiples of `align`
    groups (the fused decomposition's and the MFMA contraction's 16-group unit),
    so every rank's operand layout is the unsharded one restricted to its
    columns."""
    units = (W + align - 1) // align
    lo = units * rank // world
    hi = units * (rank + 1) // world
    return min(W, lo * align), min(W, hi * align)


class AccumulatorReducer:
    """In place, t <- sum over ranks of t (mod p) for each field vector t, over
    the C ABI's RCCL communicator on the context stream. A utility only: the
    bench's N > 1 lines never sum accumulators (see the module docstring)."""

    def __init__(self, comm, tensors):
        self.comm = comm
        self.tensors = list(tensors)

    def reduce(self):
        if self.comm is None or self.comm.size <= 1:
            return
        if len(self.tensors) == 2:
            self.comm.fold_reduce_allranks(*self.tensors)
        else:
            for t in self.tensors:
                self.comm.allreduce_modp(t)


def _step_bufs(LA, torch, device, d, W, kappa, K, L, w_ccs, acc_cm, acc_fc, rho):
    """device buffers of one fold step over W groups (lf_fold_step_bufs) and the tensors behind them"""
    z = lambda n: torch.zeros(n, dtype=torch.int64, device=device)
    N = W * L
    keep = {"w_ccs": w_ccs, "acc_cm": acc_cm, "acc_f_coeff": acc_fc, "rho": rho,
            "f_coeff": z(N * d), "f": z(N * d), "cm": z(kappa * d),
            "fk_coeff": [z(K * N * d) for _ in range(2)], "fk": [z(K * N * d) for _ in range(2)],
            "wk": [z(K * W * d) for _ in range(2)], "y": [z(K * kappa * d) for _ in range(2)],
            "f0": z(N * d), "f0_coeff": z(N * d), "w_ccs0": z(W * d), "cm0": z(kappa * d)}
    b = LA.LfFoldStepBufs()
    for k, v in keep.items():
        if isinstance(v, list):
            for s in range(2):
                getattr(b, k)[s] = v[s].data_ptr()
        else:
            setattr(b, k, v.data_ptr())
    return keep, b


def verify_sharded_step(LA, ctx, pg, local: int, rank: int, world: int, d: int = 1024, w_per_rank: int = 64,
                        kappa: int = 32, seed: int = 0x4C460020) -> bool:
    """Self-check of the column-sharded fold over the real communicator: every
    rank builds the same seeded inputs of a world * w_per_rank-group witness,
    runs its shard with lf_dev_fold_step_sharded (the RCCL all-reduce of the
    partial commitments), runs the unsharded lf_dev_fold_step of the whole
    witness on its own GPU, and compares its shard of every output bit for bit
    (f, f_coeff, f_0, Witness::from_f(f_0), the digit witnesses) and the full
    commitments (cm, y, cm_0). Returns the AND over ranks (on every rank)."""
    import numpy as np
    import torch
    pr = LA.goldilocks_dp(d)
    K, L = pr.K, pr.L
    W = w_per_rank * world
    N = W * L
    dev = torch.device("cuda", local)
    i64 = dict(dtype=torch.int64, device=dev)
    A = torch.empty(kappa * N * d, **i64)
    ctx.dev_fill_uniform(A, seed)
    full = LA.AjtaiCommitmentScheme(ctx, device_tensor=A, kappa=kappa, ncols=N, d=d)
    w_ccs, acc_w = torch.empty(W * d, **i64), torch.empty(W * d, **i64)
    ctx.dev_fill_uniform(w_ccs, seed + 1)
    ctx.dev_fill_uniform(acc_w, seed + 2)
    acc_fc, acc_f, acc_cm = torch.empty(N * d, **i64), torch.empty(N * d, **i64), torch.empty(kappa * d, **i64)
    ctx.check(ctx.lib.lf_dev_witness_from_w_ccs(ctx.h, LA._lib.C.byref(pr), acc_w.data_ptr(), W, acc_fc.data_ptr(),
                                                acc_f.data_ptr()))
    ctx.dev_ajtai_commit(full, [acc_f], acc_cm)
    rng = np.random.default_rng(seed + 3)
    rc = [LA.short_challenge(rng.integers(0, 256, 3 * d // 4, dtype=np.uint8).tobytes(), d) for _ in range(2 * K - 1)]
    one = np.zeros(d, np.uint64)
    one[0] = 1
    rho = torch.from_numpy(np.concatenate(rc + [one]).view(np.int64)).to(dev)
    ctx.dev_crt(rho, d)
    keep, b = _step_bufs(LA, torch, dev, d, W, kappa, K, L, w_ccs, acc_cm, acc_fc, rho)
    ctx.dev_fold_step(full, pr, W, b)
    g0, g1 = shard_groups(W, rank, world)
    Wr = g1 - g0
    Ar = A.view(kappa, N, d)[:, g0 * L:g1 * L].contiguous()
    sch = LA.AjtaiCommitmentScheme(ctx, device_tensor=Ar, kappa=kappa, ncols=Wr * L, d=d)
    kr, br = _step_bufs(LA, torch, dev, d, Wr, kappa, K, L, w_ccs[g0 * d:g1 * d].contiguous(), acc_cm,
                        acc_fc[g0 * L * d:g1 * L * d].contiguous(), rho)
    comm = make_comm(ctx, pg, world, rank)
    try:
        ctx.dev_fold_step_sharded(sch, pr, Wr, br, comm)
        ctx.sync()
    finally:
        if comm is not None:
            comm.close()
    ok = all(torch.equal(kr[k], keep[k]) for k in ("cm", "cm0"))
    ok &= all(torch.equal(kr["y"][s], keep["y"][s]) for s in range(2))
    c0, c1 = g0 * L, g1 * L
    for k in ("f_coeff", "f", "f0", "f0_coeff"):
        ok &= torch.equal(kr[k], keep[k][c0 * d:c1 * d])
    ok &= torch.equal(kr["w_ccs0"], keep["w_ccs0"][g0 * d:g1 * d])
    for s in range(2):
        for k, n_per, a, b_ in (("fk_coeff", N, c0, c1), ("fk", N, c0, c1), ("wk", W, g0, g1)):
            ok &= torch.equal(kr[k][s].view(K, b_ - a, d), keep[k][s].view(K, n_per, d)[:, a:b_])
    if pg is not None:
        t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev if dist.get_backend(pg) == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=pg)
        ok = bool(t.item())
    return ok


def shard(n_units: int, rank: int, world: int):
    """unit indices owned by `rank` (round-robin by step index)."""
    return list(range(rank, n_units, world))


__all__ = ["init", "barrier", "max_over_ranks", "finalize", "make_comm", "shard_groups", "AccumulatorReducer",
           "verify_sharded_step", "shard"]
