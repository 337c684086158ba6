"""Multi-GPU plumbing: one process per GPU, torch.distributed for rendezvous and
timing, RCCL over xGMI (through the C ABI's lf_comm) for the field exchange.

Two ways to spread the commit+fold path over the GPUs of a node:

* independent step streams (BASELINE.json configs[3], the trace-batch shard):
  every rank folds its own trace-step witnesses. Steps never exchange data,
  so there is no collective on the data path (weak scaling); the ranks'
  folded accumulators can be summed once with ``AccumulatorReducer``
  (lf_fold_reduce_allranks).
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
    the C ABI's RCCL communicator on the context stream (independent step
    streams: the ranks' folded accumulators cm_0 and f_0)."""

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


def shard(n_units: int, rank: int, world: int):
    """unit indices owned by `rank` (round-robin by step index)."""
    return list(range(rank, n_units, world))


__all__ = ["init", "barrier", "max_over_ranks", "finalize", "make_comm", "shard_groups", "AccumulatorReducer",
           "shard"]
