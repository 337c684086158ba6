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


def plonky3_tree(rows, nrows, width):
    """Plonky3 MerkleTree::new over one matrix, restated in plain Python: every
    layer below the root padded to an even length with the zero digest"""
    zero = np.zeros(4, np.uint64)
    level = [O.p2w8_hash(rows[i * width:(i + 1) * width]) for i in range(nrows)]
    if nrows > 1 and nrows % 2:
        level.append(zero)
    layers = [level]
    while len(level) > 1:
        nxt = [O.p2w8_compress(level[2 * i], level[2 * i + 1]) for i in range(len(level) // 2)]
        if len(level) != 2 and len(nxt) % 2:
            nxt.append(zero)
        layers.append(nxt)
        level = nxt
    return layers


@pytest.mark.parametrize("nrows", [1, 2, 3, 5, 6, 7, 12, 13, 33])
def test_merkle_tree_padding(nrows):
    """non-power-of-two heights (vm_code_comm, commitments.rs:314-340): the
    oracle's padded layers equal the plain restatement; a power of two has no padding"""
    width = 3
    rows = O.fill_uniform(nrows * width, 50 + nrows)
    layers = plonky3_tree(rows, nrows, width)
    nodes = O.merkle_tree(rows, nrows, width).reshape(-1, 4)
    assert O.merkle_nodes(nrows) == sum(len(x) for x in layers) == len(nodes)
    assert np.array_equal(nodes, np.concatenate([np.stack(x) for x in layers]))
    if nrows & (nrows - 1) == 0:
        assert len(nodes) == 2 * nrows - 1


def test_host_sponge_and_mem_comm():
    """the library's host width-8 sponge (lf_hash_w8) equals the oracle's, and
    vm_mem_comm (one-row pages: one sponge over all memory in page order) is that
    sponge over the concatenated u32 words"""
    import latticeum_amd as LA
    assert LA.merkle_depth(8) == 3 and LA.merkle_depth(5) == 3 and LA.merkle_depth(1) == 0
    for n in (0, 1, 3, 4, 5, 8, 1000):
        x = O.fill_uniform(n, 70 + n) if n else np.zeros(0, np.uint64)
        assert np.array_equal(LA.hash_w8(x), O.p2w8_hash(x)), n
    words = (O.fill_uniform(4 * 64, 71) % (1 << 32)).astype(np.uint32)  # 4 pages of 64 words
    assert np.array_equal(LA.vm_mem_comm(words), O.p2w8_hash(words.astype(np.uint64)))
    for nrows in (1, 2, 3, 5, 8, 9):
        assert LA.merkle_nodes_len(nrows) == O.merkle_nodes(nrows)


@pytest.mark.gpu
def test_merkle_gpu_any_height_and_code_comm():
    """device trees and openings at non-power-of-two heights against the oracle,
    and vm_code_comm of an odd number of code bytes (last half-word zero-padded)"""
    import torch

    import latticeum_amd as LA
    ctx = LA.Context(0)
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    for nrows, width in ((3, 1), (5, 2), (7, 1), (13, 4), (1000, 1), (4097, 1)):
        rows = O.fill_uniform(nrows * width, 90 + nrows)
        nodes = torch.zeros(LA.merkle_nodes_len(nrows) * 4, dtype=torch.int64, device="cuda")
        ctx.dev_merkle_tree(torch.from_numpy(rows.view(np.int64).copy()).cuda(), nrows, width, nodes)
        ctx.sync()
        want = O.merkle_tree(rows, nrows, width)
        assert np.array_equal(nodes.cpu().numpy().view(np.uint64), want), nrows
        for idx in (0, nrows // 2, nrows - 1):
            path = ctx.merkle_open(nodes, nrows, idx).reshape(-1, 4)
            dg, i = O.p2w8_hash(rows[idx * width:(idx + 1) * width]), idx
            for sib in path:
                dg = O.p2w8_compress(dg, sib) if i % 2 == 0 else O.p2w8_compress(sib, dg)
                i //= 2
            assert np.array_equal(dg, want[-4:]), (nrows, idx)
    rows = O.fill_uniform(300 * 9, 97)
    out = torch.zeros(300 * 4, dtype=torch.int64, device="cuda")
    ctx.dev_hash_w8_rows(torch.from_numpy(rows.view(np.int64).copy()).cuda(), 300, 9, out)
    ctx.sync()
    assert np.array_equal(out.cpu().numpy().view(np.uint64),
                          np.concatenate([O.p2w8_hash(rows[9 * i:9 * i + 9]) for i in range(300)]))
    code = bytes(np.random.default_rng(5).integers(0, 256, 2001, dtype=np.uint8))
    hw = np.array([code[2 * i] | ((code[2 * i + 1] << 8) if 2 * i + 1 < len(code) else 0)
                   for i in range((len(code) + 1) // 2)], np.uint64)
    assert np.array_equal(ctx.vm_code_comm(code), O.merkle_tree(hw, hw.size, 1)[-4:])
    ctx.close()


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
        nodes = torch.zeros(LA.merkle_nodes_len(nrows) * 4, dtype=torch.int64, device="cuda")
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
