"""RCCL with every GPU of the box: world = torch.cuda.device_count() processes,
one per GPU, each runs its shard of a column-sharded fold through lf_comm (a
real RCCL communicator over xGMI) and compares it bit for bit with the
unsharded fold on its own GPU (latticeum_amd.dist.verify_sharded_step). Skips
on a one-GPU box, where tests/test_gpu_parity.py covers the one-rank RCCL path
and the two-rank exchange over gloo."""
import os
import socket

import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, q):
    import torch
    import torch.distributed as dist
    import latticeum_amd as LA
    from latticeum_amd import dist as LD
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    try:
        torch.cuda.set_device(rank)
        pg = LD.init(world)
        ctx = LA.Context(rank)
        ctx.set_stream(torch.cuda.current_stream().cuda_stream)
        ok = LD.verify_sharded_step(LA, ctx, pg, rank, rank, world, d=1024, w_per_rank=32, kappa=8)
        ok24 = LD.verify_sharded_step(LA, ctx, pg, rank, rank, world, d=24, w_per_rank=48, kappa=8)
        ctx.close()
        q.put((rank, ok and ok24, ""))
        dist.destroy_process_group()
    except Exception as e:  # reported to the parent
        q.put((rank, False, repr(e)))


def test_rccl_sharded_fold_all_gpus():
    import torch
    import torch.multiprocessing as mp
    world = torch.cuda.device_count()
    if world < 2:
        pytest.skip("one GPU: the multi-rank RCCL path needs >= 2")
    world = min(world, 8)
    ctxm = mp.get_context("spawn")
    q = ctxm.Queue()
    port = _free_port()
    procs = [ctxm.Process(target=_rank_main, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    assert all(ok for _, ok, _ in res), res


def test_verify_sharded_step_one_rank():
    """the self-check bench.py runs after its sharded_fold timing, at one rank
    (no communicator: the sharded step is the unsharded one)"""
    import torch
    import latticeum_amd as LA
    from latticeum_amd import dist as LD
    ctx = LA.Context(0)
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    try:
        assert LD.verify_sharded_step(LA, ctx, None, 0, 0, 1, d=1024, w_per_rank=32, kappa=8)
        assert LD.verify_sharded_step(LA, ctx, None, 0, 0, 1, d=24, w_per_rank=48, kappa=8)
    finally:
        ctx.close()
