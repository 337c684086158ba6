"""Multi-process (gloo, world_size 2, CPU) coverage of the N>1 path in
latticeum_amd.dist: rank sharding, barrier, max-over-ranks timing, and the
mod-p accumulator reduce over limb transport (the RCCL exchange of
bench.py). On the GPU box the limb split/join run as HIP kernels
(HipLimbOps, covered by tests/test_gpu_parity.py); here a CPU stand-in with
the same contract lets gloo carry the collective."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

import oracle as O

P = O.P


class CpuLimbOps:
    """test stand-in for HipLimbOps (same contract, host tensors)"""

    def split(self, x, lo, hi):
        lo.copy_(x & 0xFFFFFFFF)
        hi.copy_((x >> 32) & 0xFFFFFFFF)

    def join(self, lo, hi, out):
        lo_u = lo.numpy().astype(object)
        hi_u = hi.numpy().astype(object)
        v = np.array([(int(a) + (int(b) << 32)) % P for a, b in zip(lo_u, hi_u)], dtype=np.uint64)
        out.copy_(torch.from_numpy(v.view(np.int64)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from latticeum_amd import dist as LD
    pg = LD.init(world)
    try:
        # each rank folds its own accumulator; the reduce sums them mod p
        cm0 = torch.from_numpy(O.fill_uniform(32 * 24, 100 + rank).view(np.int64).copy())
        f0 = torch.from_numpy(O.fill_uniform(5 * 24, 200 + rank).view(np.int64).copy())
        red = LD.AccumulatorReducer(CpuLimbOps(), world, [cm0, f0], group=pg)
        LD.barrier(pg)
        red.reduce()
        t = LD.max_over_ranks(pg, float(rank + 1))
        q.put((rank, cm0.numpy().view(np.uint64).copy(), f0.numpy().view(np.uint64).copy(), t,
               LD.shard(10, rank, world)))
    finally:
        LD.finalize(pg)


@pytest.mark.parametrize("world", [2])
def test_accumulator_reduce_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want_cm = sum(O.fill_uniform(32 * 24, 100 + r).astype(object) for r in range(world)) % P
    want_f = sum(O.fill_uniform(5 * 24, 200 + r).astype(object) for r in range(world)) % P
    for rank, cm0, f0, t, sh in res:
        assert [int(x) for x in cm0] == [int(x) for x in want_cm]
        assert [int(x) for x in f0] == [int(x) for x in want_f]
        assert t == float(world)  # max over ranks
    assert sorted(sum((r[4] for r in res), [])) == list(range(10))  # shards partition the steps


def test_single_rank_is_noop():
    from latticeum_amd import dist as LD
    assert LD.init(1) is None
    assert LD.max_over_ranks(None, 3.5) == 3.5
    x = torch.arange(4, dtype=torch.int64)
    LD.AccumulatorReducer(CpuLimbOps(), 1, [x]).reduce()
    assert x.tolist() == [0, 1, 2, 3]
