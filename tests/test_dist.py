"""Multi-process (gloo, world_size 2, CPU) coverage of the N>1 host logic in
latticeum_amd.dist: rendezvous, barrier, max-over-ranks timing, the
column-shard plan (shard_groups), and the exchange it relies on -- partial
commitments over each rank's columns, carried as 32-bit limbs through an
integer SUM all-reduce and joined mod p, finish into the unsharded fold
bit-exactly. Without a GPU the per-rank arithmetic is the oracle's (the same
functions the GPU parity tests compare the HIP path with); the HIP path of the
same exchange runs in tests/test_gpu_parity.py (test_sharded_step_*)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

import oracle as O

P = O.P
D, W, KAPPA, SEED = 24, 40, 4, 2100
B, L, BS, K = 1 << 15, 5, 2, 15


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def inputs():
    N = W * L
    A = O.fill_uniform(KAPPA * N * D, SEED).reshape(KAPPA, N, D)
    w_ccs = O.fill_uniform(W * D, SEED + 1)
    acc_fc, acc_f = O.witness_from_w_ccs(O.fill_uniform(W * D, SEED + 2), D, B, L, 1)
    acc_cm = O.ajtai_commit(A, KAPPA, N, D, acc_f, 1, 1)
    rho = O.crt(O.fill_uniform(2 * K * D, SEED + 3), D)
    return A, w_ccs, acc_fc, acc_cm, rho


def partial_step(A, w_ccs, acc_fc):
    """commit(z) + decompose both sides + the 1 + 2(K-1) commitments of these columns"""
    kappa, n, d = A.shape
    fc, f = O.witness_from_w_ccs(w_ccs, d, B, L, 1)
    sides = [O.decompose_witness(x, d, B, L, BS, K, 1) for x in (acc_fc, fc)]
    vecs = np.concatenate([f] + [s[1].reshape(K, n * d)[1:].ravel() for s in sides])
    part = O.ajtai_commit(A, kappa, n, d, vecs, 1 + 2 * (K - 1), 1)
    return fc, f, sides, part


def finish_step(part_sum, acc_cm, rho, sides, n):
    kd = KAPPA * D
    cm = part_sum[:kd]
    ys = []
    for s, c in enumerate((acc_cm, cm)):
        y = np.zeros((K, kd), np.uint64)
        y[1:] = part_sum[kd + s * (K - 1) * kd:kd + (s + 1) * (K - 1) * kd].reshape(K - 1, kd)
        ys.append(O.commit_witnesses_y0(c, y.ravel(), KAPPA, D, BS, K))
    cm0 = O.fold_cm0(rho, np.concatenate(ys), 2 * K, KAPPA, D)
    f0 = O.fold_f0(rho, np.concatenate([s[1] for s in sides]), 2 * K, n, D, 1)
    f0c, w0 = O.witness_from_f(f0, D, B, L, 1)
    return cm, np.concatenate(ys), cm0, f0, f0c, w0


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import torch.distributed as dist

    from latticeum_amd import dist as LD
    pg = LD.init(world)
    try:
        A, w_ccs, acc_fc, acc_cm, rho = inputs()
        g0, g1 = LD.shard_groups(W, rank, world)
        c0, c1 = g0 * L, g1 * L
        fc, f, sides, part = partial_step(np.ascontiguousarray(A[:, c0:c1]), w_ccs[g0 * D:g1 * D],
                                          acc_fc[c0 * D:c1 * D])
        # the RCCL transport's limb split, an integer SUM all-reduce, the join mod p
        limbs = torch.from_numpy(np.concatenate([part & 0xFFFFFFFF, part >> 32]).view(np.int64).copy())
        dist.all_reduce(limbs, group=pg)
        lo, hi = np.split(limbs.numpy().view(np.uint64), 2)
        part_sum = np.array([(int(a) + (int(b) << 32)) % P for a, b in zip(lo, hi)], np.uint64)
        out = finish_step(part_sum, acc_cm, rho, sides, c1 - c0)
        LD.barrier(pg)
        t = LD.max_over_ranks(pg, float(rank + 1))
        q.put((rank, g0, g1, fc, f, [s[1] for s in sides]) + out + (t,))
    finally:
        LD.finalize(pg)


@pytest.mark.parametrize("world", [2])
def test_column_sharded_fold_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(world)], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    A, w_ccs, acc_fc, acc_cm, rho = inputs()
    N = W * L
    fc, f, sides, part = partial_step(A, w_ccs, acc_fc)
    cm, y, cm0, f0, f0c, w0 = finish_step(part, acc_cm, rho, sides, N)
    assert [r[1:3] for r in res] == [(0, 16), (16, W)]  # contiguous 16-group shards
    for rank, g0, g1, rfc, rf, rfk, rcm, ry, rcm0, rf0, rf0c, rw0, t in res:
        c0, c1 = g0 * L, g1 * L
        assert np.array_equal(rcm, cm) and np.array_equal(ry, y) and np.array_equal(rcm0, cm0)
        assert np.array_equal(rfc, fc[c0 * D:c1 * D]) and np.array_equal(rf, f[c0 * D:c1 * D])
        for s in range(2):
            assert np.array_equal(rfk[s].reshape(K, -1, D), sides[s][1].reshape(K, N, D)[:, c0:c1])
        assert np.array_equal(rf0, f0[c0 * D:c1 * D]) and np.array_equal(rf0c, f0c[c0 * D:c1 * D])
        assert np.array_equal(rw0, w0[g0 * D:g1 * D])
        assert t == float(world)  # max over ranks


def test_shard_plan():
    from latticeum_amd import dist as LD
    for Wt in (1, 15, 16, 17, 37, 1 << 14, 19763):
        for world in (1, 2, 3, 8):
            sh = [LD.shard_groups(Wt, r, world) for r in range(world)]
            assert sh[0][0] == 0 and sh[-1][1] == Wt
            assert all(a[1] == b[0] for a, b in zip(sh, sh[1:]))
            assert all(g0 % 16 == 0 for g0, _ in sh)
    assert LD.shard(10, 1, 3) == [1, 4, 7]


def test_single_rank_is_noop():
    from latticeum_amd import dist as LD
    assert LD.init(1) is None
    assert LD.max_over_ranks(None, 3.5) == 3.5
    assert LD.make_comm(None, None, 1, 0) is None
    LD.AccumulatorReducer(None, [torch.arange(4)]).reduce()
