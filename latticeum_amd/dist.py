"""Multi-GPU plumbing: one process per GPU, torch.distributed over RCCL (xGMI).

The commit+fold steps of different trace-step witnesses are independent, so
ranks run their own step streams (weak scaling) with no collective in the
data path. The one exchange step is the reduce of the ranks' folded
accumulators (cm_0, f_0) -- BASELINE.json configs[3]. RCCL's integer SUM is
mod 2^64, not mod p = 2^64 - 2^32 + 1, so field vectors travel as 32-bit limbs
(all-reduced as int64, exact for <= 2^31 ranks) and are folded back into the
field by a HIP kernel (lf_dev_limb_join).
"""
from __future__ import annotations

import ctypes as C

import torch
import torch.distributed as dist


def init(world: int):
    if world <= 1:
        return None
    if not dist.is_initialized():
        backend = "nccl" if torch.cuda.is_available() else "gloo"
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


class HipLimbOps:
    """limb split / join on the GPU through the C ABI (the product path)."""

    def __init__(self, ctx):
        self.ctx = ctx

    def split(self, x, lo, hi):
        self.ctx.check(self.ctx.lib.lf_dev_limb_split(self.ctx.h, x.data_ptr(), x.numel(),
                                                      lo.data_ptr(), hi.data_ptr()))

    def join(self, lo, hi, out):
        self.ctx.check(self.ctx.lib.lf_dev_limb_join(self.ctx.h, lo.data_ptr(), hi.data_ptr(),
                                                     out.numel(), out.data_ptr()))


class AccumulatorReducer:
    """In-place  t <- sum over ranks of t  (mod p)  for each field vector t."""

    def __init__(self, ops, world: int, tensors, group=None):
        if not isinstance(ops, (HipLimbOps,)) and hasattr(ops, "check"):  # a Context
            ops = HipLimbOps(ops)
        self.ops, self.world, self.group = ops, world, group
        self.tensors = list(tensors)
        self.lo = [torch.empty_like(t) for t in self.tensors]
        self.hi = [torch.empty_like(t) for t in self.tensors]

    def reduce(self):
        if self.world <= 1:
            return
        for t, lo, hi in zip(self.tensors, self.lo, self.hi):
            self.ops.split(t, lo, hi)
            dist.all_reduce(lo, op=dist.ReduceOp.SUM, group=self.group)
            dist.all_reduce(hi, op=dist.ReduceOp.SUM, group=self.group)
            self.ops.join(lo, hi, t)


def shard(n_units: int, rank: int, world: int):
    """unit indices owned by `rank` (round-robin by step index)."""
    return list(range(rank, n_units, world))


__all__ = ["init", "barrier", "max_over_ranks", "finalize", "HipLimbOps", "AccumulatorReducer", "shard", "C"]
