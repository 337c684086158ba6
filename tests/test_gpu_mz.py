"""GPU parity of the sparse CCS products against the
oracle's mat_vec_mul restatement: the Mz MLEs of compute_mz_mles, the
zeta-challenged combination of the folding prover, and the MLE evaluations
(u_s, eta_s) -- including empty rows, repeated columns in a row and an empty
matrix -- and, at the zkvm's CCS dimensions (m = 2^17 rows, n = 19 768
columns, t = 125 matrices), the evaluation route (M_j^T eq(r)) . z against
evaluating the materialised MLEs."""
import numpy as np
import pytest

import latticeum_amd as LA
import oracle as O

pytestmark = pytest.mark.gpu
P = LA.P


@pytest.fixture(scope="module")
def ctx():
    import torch
    c = LA.Context(0)
    c.set_stream(torch.cuda.current_stream().cuda_stream)
    yield c
    c.close()


def dev(x=None, n=None):
    import torch
    if x is not None:
        return torch.from_numpy(np.ascontiguousarray(x).view(np.int64)).cuda()
    return torch.zeros(n, dtype=torch.int64, device="cuda")


def host(t):
    return t.cpu().numpy().view(np.uint64)


def scalars(v, d):
    """one scalar per entry as ring elements in NTT form (from_scalar: v in word 0 of
    every slot, zero elsewhere)"""
    tb = 3 if d == 24 else 1
    out = np.zeros((len(v), d), np.uint64)
    out[:, ::tb] = np.asarray(v, np.uint64)[:, None]
    return out.ravel()


def random_ccs(t, m, n, d, seed, max_per_row=3, scalar=False):
    rng = np.random.default_rng(seed)
    mats = []
    for j in range(t):
        if j == 1:  # an empty matrix
            mats.append((np.zeros(m + 1, np.uint64), np.zeros(0, np.uint32), np.zeros(0, np.uint64)))
            continue
        cnt = rng.integers(0, max_per_row + 1, m)
        rp = np.concatenate([[0], np.cumsum(cnt)]).astype(np.uint64)
        col = rng.integers(0, n, int(rp[-1])).astype(np.uint32)
        if col.size > 1:
            col[1] = col[0]  # a repeated column
        if scalar:  # the zkvm's values: small constants, -1 and arbitrary field elements
            v = O.fill_uniform(int(rp[-1]), seed + 7 * j)
            v[::3] = 1
            v[1::5] = LA.P - 1
            val = scalars(v, d)
        else:
            val = O.fill_uniform(int(rp[-1]) * d, seed + 7 * j)
        mats.append((rp, col, val))
    return mats


@pytest.mark.parametrize("scalar", [False, True])
@pytest.mark.parametrize("d", [24, 16, 1024])
def test_mz_products_match_oracle(ctx, d, scalar):
    """ring-valued matrices, and scalar-valued ones (the zkvm's; read one word per
    entry, lf_ccs_is_scalar)"""
    t, m, n, nz, nv = 5, 100, 37, 3, 7
    mats = random_ccs(t, m, n, d, 40 + d, scalar=scalar)
    M = LA.CCSMatrices(ctx, d, m, n, mats)
    assert M.scalar == scalar
    zs = [O.fill_uniform(n * d, 50 + d + i) for i in range(nz)]
    zd = dev(np.concatenate(zs))
    out = dev(n=nz * t * (1 << nv) * d)
    M.mz_mles(zd, nz, nv, out)
    ctx.sync()
    want = np.concatenate([O.mz_mles(mats, z, nv, d) for z in zs])
    assert np.array_equal(host(out), want)
    # the selected matrices only, in the given order (padding rows zeroed over stale data)
    sel = [3, 0, 4, 1]
    part = dev(n=len(sel) * (1 << nv) * d)
    ctx.dev_fill_uniform(part, 55 + d)
    M.mz_mles_sel(zd, sel, nv, part)
    ctx.sync()
    L = (1 << nv) * d
    assert np.array_equal(host(part), np.concatenate([want[j * L:(j + 1) * L] for j in sel]))
    zeta = O.fill_uniform(nz * d, 60 + d)
    ch = dev(n=(1 << nv) * d)
    M.mz_challenged(zd, dev(zeta), nz, nv, ch)
    ctx.sync()
    assert np.array_equal(host(ch), O.mz_challenged(mats, zs, [zeta[i * d:(i + 1) * d] for i in range(nz)], nv, d))
    # the pair form: a second (z, zeta) beside the first, one pass over the entries
    zs2 = [O.fill_uniform(n * d, 150 + d + i) for i in range(nz)]
    zeta2 = O.fill_uniform(nz * d, 160 + d)
    c0, c1 = dev(n=(1 << nv) * d), dev(n=(1 << nv) * d)
    ctx.dev_fill_uniform(c0, 5)
    ctx.dev_fill_uniform(c1, 6)  # padding rows zeroed over stale data
    M.mz_challenged_pair(zd, dev(zeta), dev(np.concatenate(zs2)), dev(zeta2), nz, nv, c0, c1)
    ctx.sync()
    assert np.array_equal(host(c0), host(ch))
    assert np.array_equal(host(c1), O.mz_challenged(mats, zs2, [zeta2[i * d:(i + 1) * d] for i in range(nz)], nv, d))
    point = O.fill_uniform(nv * d, 70 + d)
    ev = dev(n=nz * t * d)
    M.mz_evaluate(zd, nz, nv, dev(point), ev)
    ctx.sync()
    w = want.reshape(nz * t, (1 << nv) * d)
    assert np.array_equal(host(ev), np.concatenate([O.mle_evaluate(w[k], nv, d, point) for k in range(nz * t)]))


@pytest.mark.parametrize("t,n,nz", [(12, 50, 22), (1, 1, 1), (7, 33, 64), (6, 16, 21)])
def test_mz_challenged_tiles(ctx, t, n, nz):
    """the matrix-core zeta combination (d = 24, mz.hip k_zcomb_mfma) at tile edges:
    a last row tile of fewer than 5 values of j, a last column tile of fewer than 16
    columns, K = 3 nz over one, two and three 64-wide chunks (with and without a
    zero tail), one column and one matrix; both sides of the pair form"""
    d, m, nv = 24, 40, 6
    mats = random_ccs(t, m, n, d, 900 + t + n + nz, scalar=(nz % 2 == 0))
    M = LA.CCSMatrices(ctx, d, m, n, mats)
    zs = [O.fill_uniform(n * d, 910 + i) for i in range(nz)]
    zs[0][:d] = P - 1  # the largest residues in the first column
    zeta = O.fill_uniform(nz * d, 920)
    zeta[:3] = P - 1
    want = O.mz_challenged(mats, zs, [zeta[i * d:(i + 1) * d] for i in range(nz)], nv, d)
    ch = dev(n=(1 << nv) * d)
    M.mz_challenged(dev(np.concatenate(zs)), dev(zeta), nz, nv, ch)
    ctx.sync()
    assert np.array_equal(host(ch), want)
    zs2 = [O.fill_uniform(n * d, 930 + i) for i in range(nz)]
    zeta2 = O.fill_uniform(nz * d, 940)
    c0, c1 = dev(n=(1 << nv) * d), dev(n=(1 << nv) * d)
    M.mz_challenged_pair(dev(np.concatenate(zs)), dev(zeta), dev(np.concatenate(zs2)), dev(zeta2), nz, nv, c0, c1)
    ctx.sync()
    assert np.array_equal(host(c0), want)
    assert np.array_equal(host(c1), O.mz_challenged(mats, zs2, [zeta2[i * d:(i + 1) * d] for i in range(nz)], nv, d))


def test_mz_zkvm_dimensions(ctx):
    """m = 2^17, n = 19 768, t = 125 (zkvm ccs.rs:43-67) with ~2 entries per row
    per matrix: sampled rows of the materialised products against the oracle,
    and the transposed evaluation route against evaluating the materialised MLEs"""
    import torch
    d, t, m, n, nz, nv = 24, 125, 1 << 17, 19768, 2, 17
    rng = np.random.default_rng(5)
    mats = []
    for j in range(t):
        cnt = rng.integers(0, 5, m)
        rp = np.concatenate([[0], np.cumsum(cnt)]).astype(np.uint64)
        col = rng.integers(0, n, int(rp[-1])).astype(np.uint32)
        mats.append((rp, col, None))
    nnz = sum(int(x[0][-1]) for x in mats)
    vals = O.fill_uniform(nnz * d, 6)
    off = 0
    full = []
    for rp, col, _ in mats:
        k = int(rp[-1])
        full.append((rp, col, vals[off * d:(off + k) * d]))
        off += k
    M = LA.CCSMatrices(ctx, d, m, n, full)
    zs = O.fill_uniform(nz * n * d, 7)
    zd = dev(zs)
    out = dev(n=nz * t * (1 << nv) * d)
    M.mz_mles(zd, nz, nv, out)
    ctx.sync()
    for i, j, r in ((0, 0, 0), (1, 124, m - 1), (0, 63, 77777), (1, 5, 4096)):
        rp, col, val = full[j]
        a, b = int(rp[r]), int(rp[r + 1])
        want = O.spmv(np.array([0, b - a], np.uint64), col[a:b], val[a * d:b * d], d, zs[i * n * d:(i + 1) * n * d])
        got = host(out[((i * t + j) * (1 << nv) + r) * d:((i * t + j) * (1 << nv) + r + 1) * d])
        assert np.array_equal(got, want), (i, j, r)
    point = dev(O.fill_uniform(nv * d, 8))
    ev, ev2 = dev(n=nz * t * d), dev(n=nz * t * d)
    M.mz_evaluate(zd, nz, nv, point, ev)
    ctx.dev_mle_evaluate(d, out, nz * t, nv, point, ev2)
    ctx.sync()
    assert torch.equal(ev, ev2)
    del out
    torch.cuda.empty_cache()


@pytest.mark.parametrize("d", [24, 1024])
def test_scalar_ccs_montgomery_input(ctx, d):
    """scalar-valued matrices handed over as Montgomery limbs (the zero-copy form of the
    Rust structs) are still detected as scalars and give the canonical products"""
    t, m, n, nz, nv = 4, 64, 21, 2, 6
    mats = random_ccs(t, m, n, d, 90 + d, scalar=True)
    mont = [(rp, col, np.array([(int(v) << 64) % LA.P for v in val], np.uint64)) for rp, col, val in mats]
    A = LA.CCSMatrices(ctx, d, m, n, mats)
    B = LA.CCSMatrices(ctx, d, m, n, mont, repr=LA.REPR_MONTGOMERY)
    assert A.scalar and B.scalar
    zd = dev(O.fill_uniform(nz * n * d, 91 + d))
    oa, ob = dev(n=nz * t * (1 << nv) * d), dev(n=nz * t * (1 << nv) * d)
    A.mz_mles(zd, nz, nv, oa)
    B.mz_mles(zd, nz, nv, ob)
    point = dev(O.fill_uniform(nv * d, 92 + d))
    ea, eb = dev(n=nz * t * d), dev(n=nz * t * d)
    A.mz_evaluate(zd, nz, nv, point, ea)
    B.mz_evaluate(zd, nz, nv, point, eb)
    ctx.sync()
    assert np.array_equal(host(oa), host(ob)) and np.array_equal(host(ea), host(eb))
