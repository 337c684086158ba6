"""Width-8 Poseidon2 Merkle trees of VM memory (SURVEY.md 8(f) rank 3,
zkvm/src/commitments.rs:192-262). Parity is unpinned against the reference
(its internal diagonal is Plonky3's MATRIX_DIAG_8_GOLDILOCKS, not vendored,
and the reference's only Merkle KAT needs an author-local ELF): the CPU tests
pin the oracle's tree and sponge structure with a plain restatement, and the
GPU tests compare the device trees, paths and permutations with the oracle."""
import numpy as np
import pytest

import oracle as O

P = O.P


def test_sponge_structure():
    """PaddingFreeSponge<8, 4, 4>: overwrite four words, permute; a partial
    last block is permuted; an empty input is the zero digest"""
    x = O.fill_uniform(10, 3)
    s = np.zeros(8, np.uint64)
    for blk in (x[0:4], x[4:8], x[8:10]):
        s[:blk.size] = blk
        s = O.p2w8_permute(s)
    assert np.array_equal(O.p2w8_hash(x), s[:4])
    assert not O.p2w8_hash([]).any()


def test_merkle_tree_structure():
    nrows, width = 8, 6
    rows = O.fill_uniform(nrows * width, 5)
    nodes = O.merkle_tree(rows, nrows, width).reshape(-1, 4)
    level = [O.p2w8_hash(rows[i * width:(i + 1) * width]) for i in range(nrows)]
    k = 0
    while True:
        for dgst in level:
            assert np.array_equal(nodes[k], dgst)
            k += 1
        if len(level) == 1:
            break
        level = [O.p2w8_compress(level[2 * i], level[2 * i + 1]) for i in range(len(level) // 2)]
    assert k == 2 * nrows - 1


@pytest.mark.gpu
def test_merkle_gpu_matches_oracle():
    import torch

    import latticeum_amd as LA
    ctx = LA.Context(0)
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    st = O.fill_uniform(8 * 3000, 7)
    t = torch.from_numpy(st.view(np.int64).copy()).cuda()
    ctx.dev_poseidon2_w8_permute(t)
    ctx.sync()
    want = np.concatenate([O.p2w8_permute(st[8 * i:8 * i + 8]) for i in range(3000)])
    assert np.array_equal(t.cpu().numpy().view(np.uint64), want)
    for nrows, width in ((1, 5), (16, 1), (64, 7), (256, 1024)):
        rows = O.fill_uniform(nrows * width, 9 + nrows)
        nodes = torch.zeros((2 * nrows - 1) * 4, dtype=torch.int64, device="cuda")
        ctx.dev_merkle_tree(torch.from_numpy(rows.view(np.int64).copy()).cuda(), nrows, width, nodes)
        ctx.sync()
        want = O.merkle_tree(rows, nrows, width)
        assert np.array_equal(nodes.cpu().numpy().view(np.uint64), want)
        if nrows > 1:
            idx = nrows // 3
            path = ctx.merkle_open(nodes, nrows, idx).reshape(-1, 4)
            # the path recomputes the root (verify_batch)
            dg = O.p2w8_hash(rows[idx * width:(idx + 1) * width])
            i = idx
            for sib in path:
                dg = O.p2w8_compress(dg, sib) if i % 2 == 0 else O.p2w8_compress(sib, dg)
                i //= 2
            assert np.array_equal(dg, want[-4:])
    ctx.close()
