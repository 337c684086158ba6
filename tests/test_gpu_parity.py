"""GPU parity: every HIP path through the C ABI against the CPU oracle
(oracle/lf_oracle.c), bit-exact, on seeded inputs at oracle-friendly sizes,
plus the reference's own KATs pushed through the GPU path."""
import json
from pathlib import Path

import numpy as np
import pytest

import latticeum_amd as LA
import oracle as O

pytestmark = pytest.mark.gpu
P = LA.P
KATS = json.loads((Path(__file__).parent / "golden/reference_kats.json").read_text())
NEGA = [16, 64, 256, 1024, 4096]
ALL_D = [24] + NEGA


@pytest.fixture(scope="module")
def ctx():
    import torch
    c = LA.Context(0)
    # the tests fill device buffers with torch: run the library on torch's stream
    c.set_stream(torch.cuda.current_stream().cuda_stream)
    yield c
    c.close()


def rand(n, seed):
    return O.fill_uniform(n, seed)


def params(d):
    return LA.goldilocks_dp(d)


def valid_f_coeff(d, W, seed):
    """an f_coeff produced like the reference's (from_w_ccs of a random w_ccs)"""
    pr = params(d)
    fc, f = O.witness_from_w_ccs(rand(W * d, seed), d, pr.B, pr.L)
    return fc, f


# ------------------------------------------------------------------ transforms
@pytest.mark.parametrize("name", ["test_crt", "test_crt2"])
def test_crt_kat_on_gpu(ctx, name):
    k = KATS["crt"][name]
    y = ctx.crt(np.array(k["coeffs"], np.uint64), 24)
    O.lib().lfo_phi72_dehomogenize(y)
    assert [int(v) for v in y] == k["crt_dehomogenized"]


@pytest.mark.parametrize("name", ["test_icrt", "test_icrt_2"])
def test_icrt_kat_on_gpu(ctx, name):
    k = KATS["crt"][name]
    ev = np.array(k["evaluations_dehomogenized"], np.uint64)
    O.lib().lfo_phi72_homogenize(ev)
    assert [int(v) for v in ctx.icrt(ev, 24)] == k["coeffs"]


@pytest.mark.parametrize("d", ALL_D)
@pytest.mark.parametrize("n", [1, 3, 257])
def test_transform_matches_oracle(ctx, d, n):
    x = rand(n * d, 100 + d + n)
    F = ctx.crt(x, d)
    assert np.array_equal(F, O.crt(x, d))
    assert np.array_equal(ctx.icrt(F, d), x)
    assert np.array_equal(ctx.icrt(x, d), O.icrt(x, d))


def test_transform_edge_values(ctx):
    for d in ALL_D:
        for v in [0, 1, P - 1, (P - 1) // 2]:
            x = np.full(d, v, np.uint64)
            assert np.array_equal(ctx.crt(x, d), O.crt(x, d))
        assert ctx.crt(np.zeros(0, np.uint64), d).size == 0


@pytest.mark.parametrize("d", [24, 1024])
def test_montgomery_repr(ctx, d):
    x = rand(4 * d, 7 + d)
    xm = np.array([O.to_mont(int(v)) for v in x], np.uint64)
    ym = ctx.crt(xm, d, LA.REPR_MONTGOMERY)
    assert [O.from_mont(int(v)) for v in ym] == [int(v) for v in O.crt(x, d)]


@pytest.mark.parametrize("d", ALL_D)
def test_ring_mul(ctx, d):
    a, b = rand(5 * d, 1 + d), rand(5 * d, 2 + d)
    want = np.concatenate([O.slot_mul(a[i * d:(i + 1) * d], b[i * d:(i + 1) * d], d) for i in range(5)])
    assert np.array_equal(ctx.ring_mul(a, b, d), want)
    # CRT(a) (.) CRT(b) = CRT(a * b)   (goldilocks/mod.rs:231-247 test_mul_crt)
    pa, pb = a[:d], b[:d]
    prod = ctx.icrt(ctx.ring_mul(ctx.crt(pa, d), ctx.crt(pb, d), d), d)
    assert np.array_equal(prod, O.poly_mul(pa, pb, d))


# ------------------------------------------------------------------ witness
@pytest.mark.parametrize("d", ALL_D)
@pytest.mark.parametrize("W", [1, 7, 33])
def test_witness_from_w_ccs(ctx, d, W):
    pr = params(d)
    w = rand(W * d, 300 + d + W)
    fc, f = ctx.witness_from_w_ccs(w, pr)
    ofc, of = O.witness_from_w_ccs(w, d, pr.B, pr.L)
    assert np.array_equal(fc, ofc)
    assert np.array_equal(f, of)


@pytest.mark.parametrize("d", ALL_D)
def test_witness_from_f(ctx, d):
    pr = params(d)
    f = rand(5 * pr.L * d, 400 + d)
    fc, w = ctx.witness_from_f(f, pr)
    ofc, ow = O.witness_from_f(f, d, pr.B, pr.L)
    assert np.array_equal(fc, ofc) and np.array_equal(w, ow)


@pytest.mark.parametrize("W", [50, 51, 52, 205])
def test_phi72_witness_block_edges(ctx, W):
    """d = 24 from_w_ccs runs one thread per (element, digit) and from_f packs
    51 whole groups of L = 5 elements per 255-thread block: W around and past
    one block, with a ragged last block"""
    d = 24
    pr = params(d)
    w = rand(W * d, 1300 + W)
    fc, f = ctx.witness_from_w_ccs(w, pr)
    ofc, of = O.witness_from_w_ccs(w, d, pr.B, pr.L)
    assert np.array_equal(fc, ofc) and np.array_equal(f, of)
    f_in = rand(W * pr.L * d, 1400 + W)
    fc2, w2 = ctx.witness_from_f(f_in, pr)
    ofc2, ow2 = O.witness_from_f(f_in, d, pr.B, pr.L)
    assert np.array_equal(fc2, ofc2) and np.array_equal(w2, ow2)


@pytest.mark.parametrize("W", [4095, 4096, 4101])
def test_from_w_ccs_and_from_f_both_kernels_sampled(ctx, W):
    """d = 1024 runs a one-half-wave-per-(element, limb) kernel below W = 4096
    and one half-wave per element above: both, checked on sampled elements
    (every element's output depends on that element alone)"""
    d = 1024
    pr = params(d)
    L = pr.L
    w = rand(W * d, 900 + W)
    fc, f = ctx.witness_from_w_ccs(w, pr)
    f_in = rand(W * L * d, 950 + W)
    fc2, w2 = ctx.witness_from_f(f_in, pr)
    for j in (0, 1, W // 2, W - 2, W - 1):
        ofc, of = O.witness_from_w_ccs(w[j * d:(j + 1) * d], d, pr.B, L)
        assert np.array_equal(fc[j * L * d:(j + 1) * L * d], ofc)
        assert np.array_equal(f[j * L * d:(j + 1) * L * d], of)
        ofc2, ow2 = O.witness_from_f(f_in[j * L * d:(j + 1) * L * d], d, pr.B, L)
        assert np.array_equal(fc2[j * L * d:(j + 1) * L * d], ofc2)
        assert np.array_equal(w2[j * d:(j + 1) * d], ow2)


@pytest.mark.parametrize("d", ALL_D)
@pytest.mark.parametrize("W", [1, 9, 40])
def test_decompose_witness(ctx, d, W):
    pr = params(d)
    fc, _ = valid_f_coeff(d, W, 500 + d + W)
    got = ctx.decompose_witness(fc, pr)
    want = O.decompose_witness(fc, d, pr.B, pr.L, pr.b_small, pr.K)
    for g, w_ in zip(got, want):
        assert np.array_equal(g, w_)


@pytest.mark.parametrize("d", [24, 1024])
def test_decompose_witness_b_small_4(ctx, d):
    """DecompositionParams with b_small = 4 (K = 8): the block-wide Phi_72 kernel
    (k_decompose_phi72) and the generic X^d + 1 one (k_decompose_nega)"""
    base = params(d)
    pr = LA.LfParams(d, base.B, base.L, 4, 8)
    fc, _ = valid_f_coeff(d, 37, 700 + d)
    got = ctx.decompose_witness(fc, pr)
    want = O.decompose_witness(fc, d, pr.B, pr.L, pr.b_small, pr.K)
    for g, w_ in zip(got, want):
        assert np.array_equal(g, w_)


@pytest.mark.parametrize("d", [24, 1024, 4096])
def test_decompose_overflow_is_an_error(ctx, d):
    pr = params(d)
    fc = np.zeros(pr.L * d, np.uint64)
    fc[3] = 1 << 20  # needs more than K=15 binary digits (reference panics)
    with pytest.raises(LA.LfError) as e:
        ctx.decompose_witness(fc, pr)
    assert e.value.code == 6
    ctx.decompose_witness(np.zeros(pr.L * d, np.uint64), pr)  # flag was cleared


@pytest.mark.parametrize("d", [24, 1024, 4096])
def test_decompose_digit_boundary(ctx, d):
    """|v| = 2^K - 1 (either sign) takes exactly K binary digits; |v| = 2^K does
    not (balanced_decomposition/mod.rs:85-87 panics). Several elements, so the
    plane-split launches (one digit plane per block at this size) all run."""
    pr = params(d)
    K = pr.K
    P = (1 << 64) - (1 << 32) + 1
    n = 3 * pr.L * d
    for v in ((1 << K) - 1, P - ((1 << K) - 1)):
        fc = np.zeros(n, np.uint64)
        fc[5] = v
        fc[n - 1] = v
        got = ctx.decompose_witness(fc, pr)
        want = O.decompose_witness(fc, d, pr.B, pr.L, pr.b_small, K)
        for g, w_ in zip(got, want):
            assert np.array_equal(g, w_)
    for v in (1 << K, P - (1 << K)):
        fc = np.zeros(n, np.uint64)
        fc[n - 1] = v
        with pytest.raises(LA.LfError) as e:
            ctx.decompose_witness(fc, pr)
        assert e.value.code == 6


# ------------------------------------------------------------------ Ajtai
@pytest.mark.parametrize("d", ALL_D)
@pytest.mark.parametrize("kappa,ncols", [(1, 1), (3, 17), (9, 300)])
def test_ajtai_commit(ctx, d, kappa, ncols):
    A = rand(kappa * ncols * d, 600 + d + ncols).reshape(kappa, ncols, d)
    f = rand(ncols * d, 700 + d + ncols)
    sch = LA.AjtaiCommitmentScheme(ctx, A)
    assert np.array_equal(sch.commit_ntt(f), O.ajtai_commit(A, kappa, ncols, d, f))


def test_ajtai_closed_form_kat_full_size(ctx):
    # LF/commitment/commitment_scheme.rs:141-159 at the reference's own size
    k = KATS["ajtai_closed_form"]
    kappa, n = k["kappa"], k["n"]
    vals = (np.arange(kappa, dtype=np.uint64)[:, None] * n + np.arange(n, dtype=np.uint64)[None, :])
    A = np.zeros((kappa, n, 24), np.uint64)
    A[:, :, 0::3] = vals[:, :, None]
    f = np.zeros((n, 24), np.uint64)
    f[:, 0::3] = 2
    cm = LA.AjtaiCommitmentScheme(ctx, A).commit_ntt(f.ravel()).reshape(kappa, 24)
    for i in range(kappa):
        e = n * (2 * i * n + n - 1) % P
        assert all(int(cm[i, 3 * s]) == e and cm[i, 3 * s + 1] == 0 for s in range(8))


def test_ajtai_wrong_witness_length(ctx):
    sch = LA.AjtaiCommitmentScheme(ctx, rand(2 * 5 * 24, 1).reshape(2, 5, 24))
    with pytest.raises(LA.LfError) as e:
        sch.commit_ntt(rand(4 * 24, 2))
    assert e.value.code == 3


@pytest.mark.parametrize("d", [24, 64, 1024])
def test_ajtai_batched_vectors(ctx, d):
    kappa, ncols, nvec = 5, 40, 28
    A = rand(kappa * ncols * d, 11 + d).reshape(kappa, ncols, d)
    sch = LA.AjtaiCommitmentScheme(ctx, A)
    import torch
    F = rand(nvec * ncols * d, 12 + d)
    Ft = torch.from_numpy(F.view(np.int64)).cuda()
    cm = torch.zeros(nvec * kappa * d, dtype=torch.int64, device="cuda")
    ctx.dev_ajtai_commit(sch, [Ft[v * ncols * d:(v + 1) * ncols * d] for v in range(nvec)], cm)
    ctx.sync()
    want = O.ajtai_commit(A, kappa, ncols, d, F, nvec)
    assert np.array_equal(cm.cpu().numpy().view(np.uint64), want)


# ------------------------------------------------------------------ commit / fold
def oracle_fold_hot(A, kappa, d, pr, acc_cm, acc_fc, cm_i, wi_fc, rho):
    N = acc_fc.size // d
    K, L = pr.K, pr.L
    sides = [O.decompose_witness(x, d, pr.B, L, pr.b_small, K) for x in (acc_fc, wi_fc)]
    vecs = np.concatenate([s[1].reshape(K, N * d)[1:] for s in sides]).ravel()
    ycat = O.ajtai_commit(A, kappa, N, d, vecs, 2 * (K - 1)).reshape(2, K - 1, kappa * d)
    ys = []
    for s, cm in enumerate((acc_cm, cm_i)):
        y = np.zeros((K, kappa * d), np.uint64)
        y[1:] = ycat[s]
        ys.append(O.commit_witnesses_y0(cm, y.ravel(), kappa, d, pr.b_small, K))
    fall = np.concatenate([s[1] for s in sides])
    f0 = O.fold_f0(rho, fall, 2 * K, N, d)
    cm0 = O.fold_cm0(rho, np.concatenate(ys), 2 * K, kappa, d)
    f0c, w0 = O.witness_from_f(f0, d, pr.B, L)
    return {"y": np.concatenate(ys), "f0": f0, "f0_coeff": f0c, "w_ccs0": w0, "cm0": cm0}, sides


def make_rho(d, K, seed):
    rng = np.random.default_rng(seed)
    rc = [O.short_challenge(rng.integers(0, 256, 3 * d // 4, dtype=np.uint8).tobytes(), d)
          for _ in range(2 * K - 1)]
    one = np.zeros(d, np.uint64)
    one[0] = 1
    rc.append(one)  # get_rhos pushes ONE last (folding/utils.rs:123-126)
    return O.crt(np.concatenate(rc), d)


@pytest.mark.parametrize("d,W,kappa", [(24, 6, 4), (24, 13, 3), (64, 3, 2), (1024, 2, 3)])
def test_commit_then_fold_hot(ctx, d, W, kappa):
    pr = params(d)
    N = W * pr.L
    A = rand(kappa * N * d, 800 + d).reshape(kappa, N, d)
    sch = LA.AjtaiCommitmentScheme(ctx, A)
    # commit(z): z = [x_ccs (l=4) | 1 | w_ccs]
    l = 4
    w_ccs = rand(W * d, 900 + d)
    z = np.concatenate([rand(l * d, 901), np.zeros(d, np.uint64), w_ccs])
    fc, f, cm = ctx.commit(sch, z, l, pr)
    ofc, of = O.witness_from_w_ccs(w_ccs, d, pr.B, pr.L)
    ocm = O.ajtai_commit(A, kappa, N, d, of)
    assert np.array_equal(fc, ofc) and np.array_equal(f, of) and np.array_equal(cm, ocm)
    # fold with an accumulator built like initialize_accumulator / a previous step
    acc_fc, acc_f = valid_f_coeff(d, W, 950 + d)
    acc_cm = O.ajtai_commit(A, kappa, N, d, acc_f)
    rho = make_rho(d, pr.K, 960 + d)
    got = ctx.fold_hot(sch, pr, acc_cm, acc_fc, cm, fc, rho)
    want, _ = oracle_fold_hot(A, kappa, d, pr, acc_cm, acc_fc, cm, fc, rho)
    for key in want:
        assert np.array_equal(got[key], want[key]), key
    # decomposition soundness: y recomposes to cm (decomposition.rs verifier :120-124)
    y = got["y"].reshape(2, pr.K, kappa * d)
    for s, c in enumerate((acc_cm, cm)):
        acc = np.zeros(kappa * d, object)
        for k in reversed(range(pr.K)):
            acc = (acc * 2 + y[s, k].astype(object)) % P
        assert [int(v) for v in acc] == [int(v) for v in c]


@pytest.mark.parametrize("d,W,kappa", [(24, 10, 4), (24, 70, 3), (1024, 2, 2), (1024, 37, 2)])
def test_dev_fold_step_matches_oracle(ctx, d, W, kappa):
    check_dev_fold_step(ctx, d, W, kappa)


@pytest.mark.parametrize("W", [2, 37, 130])
def test_dev_fold_step_without_fk(ctx, W):
    """f_k buffers omitted (the fused X^1024+1 path): the planes exist only as
    MFMA operand rows, plane 0 of each side in rows 29 and 30, and f_0 is folded
    from them (k_fold_frag); every other output equals the oracle's"""
    check_dev_fold_step(ctx, 1024, W, 2, keep_fk=False)
    check_dev_fold_step(ctx, 1024, W, 2, steps=2, keep_fk=False)


@pytest.mark.parametrize("mode", ["default", "0", "1"])
@pytest.mark.parametrize("d,W", [(1024, 37), (4096, 17)])
def test_dev_fold_step_store_modes(ctx, monkeypatch, d, W, mode):
    """the fused d = 1024 / 4096 decompositions with cached (LATTICEUM_AMD_DEC_NT=0),
    streaming (=1) and the default stores (frag.hpp dec_streaming) give the oracle's step"""
    if mode != "default":
        monkeypatch.setenv("LATTICEUM_AMD_DEC_NT", mode)
    check_dev_fold_step(ctx, d, W, 2)


def test_dev_fold_step_without_fk_unfused_is_an_error(ctx):
    with pytest.raises(LA.LfError):
        check_dev_fold_step(ctx, 24, 10, 3, keep_fk=False)


@pytest.mark.parametrize("W", [3, 17, 70])
def test_dev_fold_step_phi72_rho_not_short(ctx, W):
    """Phi_72: rho with full-size coefficients turns the coefficient-form fold
    (k_fold_coeff_phi72) off through its device flag and the NTT-form fold and
    Witness::from_f on; a short rho on the same context folds from the masks again"""
    d, K = 24, params(24).K
    check_dev_fold_step(ctx, d, W, 3, rho=rand(2 * K * d, 5151 + W))
    check_dev_fold_step(ctx, d, W, 3)


@pytest.mark.parametrize("W", [2, 7, 130])
def test_dev_fold_step_rho_not_short(ctx, W):
    """rho with full-size coefficients: the coefficient-form fold's device flag
    turns it off and the NTT-form fold + from_f run instead (no host sync)"""
    d, K = 1024, params(1024).K
    rho = rand(2 * K * d, 4242 + W)
    check_dev_fold_step(ctx, d, W, 2, rho=rho)
    # and a short rho again on the same context: the flag is reset per step
    check_dev_fold_step(ctx, d, W, 2)


def test_dev_fold_step_on_cu_masked_stream():
    """a context on a stream restricted to a block of 64 CUs (and the persistent
    grids sized to it, lf_ctx_set_cu_count) computes the same step"""
    c = LA.Context(0)
    try:
        c.use_cu_mask(range(64, 128))
        check_dev_fold_step(c, 1024, 37, 2)
        check_dev_fold_step(c, 24, 17, 3)
    finally:
        c.close()


def test_dev_fold_step_repeated_in_place(ctx):
    # consecutive steps reuse every buffer (as bench.py and the proving loop do):
    # the fused fold must see each step's own f_k rows, never the previous step's
    check_dev_fold_step(ctx, 1024, 37, 2, steps=3)


@pytest.mark.parametrize("d,W", [(24, 3), (24, 17), (24, 70), (1024, 2), (1024, 37), (1024, 130)])
@pytest.mark.parametrize("short", [True, False])
def test_dev_fold_step_packed_planes(ctx, d, W, short):
    """the decomposed witnesses kept as packed digit planes (lf_fold_step_bufs.planes,
    no u64 f_k / f_coeff_k rows): the step's outputs and the planes expanded by
    lf_dev_expand_planes equal the oracle's decompose_witness; a rho that is not
    short folds from the masks in Z_p (d = 24) or from the operand rows (d = 1024)"""
    K = params(d).K
    check_dev_fold_step(ctx, d, W, 3 if d == 24 else 2, packed=True, rho=None if short else rand(2 * K * d, 6161 + W))


@pytest.mark.parametrize("d", [24, 1024])
def test_dev_fold_step_planes_beside_rows(ctx, d):
    """planes given together with the u64 rows: both are written"""
    check_dev_fold_step(ctx, d, 17, 3 if d == 24 else 2, packed="both")


def test_dev_fold_step_packed_planes_repeated(ctx):
    """consecutive packed d = 1024 steps on the same buffers"""
    check_dev_fold_step(ctx, 1024, 37, 2, steps=3, packed=True)


def test_failed_packed_step_then_decompose_commit(ctx):
    """A d = 1024 packed step whose commit(z) half has run (from_w_ccs wrote the
    new witness's sign|magnitude words into planes[1]) but whose fold_commit then
    fails on a buffer argument must leave nothing behind: a following
    lf_dev_decompose_commit on the same context decomposes the f_coeff it is
    given, not the failed step's packed words (the pre-packed flag is
    an argument, not context state)."""
    import torch
    d, W, kappa = 1024, 17, 2
    pr = params(d)
    K, L = pr.K, pr.L
    N = W * L
    A = rand(kappa * N * d, 4100)
    sch = LA.AjtaiCommitmentScheme(ctx, device_tensor=torch.from_numpy(A.view(np.int64)).cuda(), kappa=kappa,
                                   ncols=N, d=d)
    acc_fc, acc_f = valid_f_coeff(d, W, 4101)
    acc_cm = O.ajtai_commit(A, kappa, N, d, acc_f)
    dev = lambda x: torch.from_numpy(np.ascontiguousarray(x).view(np.int64)).cuda()
    z = lambda n: torch.zeros(n, dtype=torch.int64, device="cuda")
    keep = {"w_ccs": dev(rand(W * d, 4102)), "acc_cm": dev(acc_cm), "acc_f_coeff": dev(acc_fc),
            "rho": dev(make_rho(d, K, 4103)), "f_coeff": z(N * d), "f": z(N * d), "cm": z(kappa * d),
            "wk": [z(K * W * d) for _ in range(2)], "y": [z(K * kappa * d) for _ in range(2)],
            "f0": z(N * d), "f0_coeff": z(N * d), "w_ccs0": z(W * d), "cm0": z(kappa * d),
            "planes": [z(N * 256) for _ in range(2)], "bad": z(K * N * d)}
    b = LA.LfFoldStepBufs()
    for k in ("w_ccs", "acc_cm", "acc_f_coeff", "rho", "f_coeff", "f", "cm", "f0", "f0_coeff", "w_ccs0", "cm0"):
        setattr(b, k, keep[k].data_ptr())
    for s in range(2):
        b.wk[s], b.y[s], b.planes[s] = keep["wk"][s].data_ptr(), keep["y"][s].data_ptr(), keep["planes"][s].data_ptr()
    b.fk_coeff[0] = keep["bad"].data_ptr()  # one side only: fold_commit refuses it after from_w_ccs ran
    torch.cuda.synchronize()
    with pytest.raises(LA.LfError):
        ctx.dev_fold_step(sch, pr, W, b)
    ctx.sync()
    b.fk_coeff[0] = None
    # a different linearized instance in the same f_coeff buffer
    wi_fc, wi_f = valid_f_coeff(d, W, 4104)
    keep["f_coeff"].copy_(dev(wi_fc))
    keep["cm"].copy_(dev(O.ajtai_commit(A, kappa, N, d, wi_f)))
    torch.cuda.synchronize()
    ctx.check(ctx.lib.lf_dev_decompose_commit(ctx.h, sch.h, LA._lib.C.byref(pr), W, LA._lib.C.byref(b)))
    ctx.sync()
    h = lambda t: t.cpu().numpy().view(np.uint64)
    for s, fc in ((0, acc_fc), (1, wi_fc)):
        _, ofk, owk = O.decompose_witness(fc, d, pr.B, L, pr.b_small, K)
        assert np.array_equal(h(keep["wk"][s]), owk), f"w_ccs_k side {s}"
        y = h(keep["y"][s]).reshape(K, kappa * d)
        oy = O.ajtai_commit(A, kappa, N, d, ofk.reshape(K, N * d)[1:].ravel(), K - 1).reshape(K - 1, kappa * d)
        assert np.array_equal(y[1:], oy), f"y side {s}"


def check_dev_fold_step(ctx, d, W, kappa, steps=1, keep_fk=True, rho=None, packed=False):
    import torch
    pr = params(d)
    K, L = pr.K, pr.L
    N = W * L
    A = rand(kappa * N * d, 1000 + d)
    At = torch.from_numpy(A.view(np.int64)).cuda()
    sch = LA.AjtaiCommitmentScheme(ctx, device_tensor=At, kappa=kappa, ncols=N, d=d)
    w_ccs = rand(W * d, 1001 + d)
    acc_fc, acc_f = valid_f_coeff(d, W, 1002 + d)
    acc_cm = O.ajtai_commit(A, kappa, N, d, acc_f)
    if rho is None:
        rho = make_rho(d, K, 1003 + d)

    def dev(x=None, n=None):
        if x is not None:
            return torch.from_numpy(np.ascontiguousarray(x).view(np.int64)).cuda()
        return torch.zeros(n, dtype=torch.int64, device="cuda")

    keep = {
        "w_ccs": dev(w_ccs), "acc_cm": dev(acc_cm), "acc_f_coeff": dev(acc_fc), "rho": dev(rho),
        "f_coeff": dev(n=N * d), "f": dev(n=N * d), "cm": dev(n=kappa * d),
        "fk_coeff": [dev(n=K * N * d) for _ in range(2)] if packed is not True else [None, None],
        "fk": [dev(n=K * N * d) for _ in range(2)] if keep_fk and packed is not True else [None, None],
        "wk": [dev(n=K * W * d) for _ in range(2)], "y": [dev(n=K * kappa * d) for _ in range(2)],
        "f0": dev(n=N * d), "f0_coeff": dev(n=N * d), "w_ccs0": dev(n=W * d), "cm0": dev(n=kappa * d),
        "planes": [dev(n=K * N if d == 24 else N * 256) for _ in range(2)] if packed else [None, None],
    }
    b = LA.LfFoldStepBufs()
    for k, v in keep.items():
        if isinstance(v, list):
            for s in range(2):
                getattr(b, k)[s] = v[s].data_ptr() if v[s] is not None else None
        else:
            setattr(b, k, v.data_ptr())
    h = lambda t: t.cpu().numpy().view(np.uint64)
    for step in range(steps):
        if step:
            w_ccs = rand(W * d, 2000 + step)
            keep["w_ccs"].copy_(dev(w_ccs))
        torch.cuda.synchronize()  # the inputs torch wrote on its stream, before the context's stream reads them
        ctx.dev_fold_step(sch, pr, W, b)
        ctx.sync()
        if packed:  # the rows as lf_dev_expand_planes makes them from the packed planes
            for s in range(2):
                fck, fk = dev(n=K * N * d), dev(n=K * N * d)
                ctx.dev_expand_planes(pr, keep["planes"][s], N, fck, fk)
                ctx.sync()
                if packed == "both":
                    assert torch.equal(fck, keep["fk_coeff"][s]) and torch.equal(fk, keep["fk"][s])
                keep["fk_coeff"][s], keep["fk"][s] = fck, fk
        check_fold_outputs(h, keep, A, kappa, d, pr, W, w_ccs, acc_cm, acc_fc, rho)


def check_fold_outputs(h, keep, A, kappa, d, pr, W, w_ccs, acc_cm, acc_fc, rho):
    L, N = pr.L, W * pr.L
    ofc, of = O.witness_from_w_ccs(w_ccs, d, pr.B, L)
    ocm = O.ajtai_commit(A, kappa, N, d, of)
    assert np.array_equal(h(keep["f"]), of) and np.array_equal(h(keep["cm"]), ocm)
    want, sides = oracle_fold_hot(A, kappa, d, pr, acc_cm, acc_fc, ocm, ofc, rho)
    assert np.array_equal(np.concatenate([h(y) for y in keep["y"]]), want["y"])
    for key in ("f0", "f0_coeff", "w_ccs0", "cm0"):
        assert np.array_equal(h(keep[key]), want[key]), key
    for s in range(2):
        assert np.array_equal(h(keep["fk_coeff"][s]), sides[s][0])
        if keep["fk"][s] is not None:
            assert np.array_equal(h(keep["fk"][s]), sides[s][1])
        assert np.array_equal(h(keep["wk"][s]), sides[s][2])


# ------------------------------------------------------------------ Poseidon2 / misc
def test_poseidon2_batch(ctx):
    st = rand(16 * 1000, 77)
    assert np.array_equal(ctx.poseidon2_permute(st), O.p2_permute(st))


def test_poseidon2_round0_kat_on_device(ctx):
    """the device permutation stopped after round 0 reproduces the reference's
    round vector (sages/inverse_mds.sage, external_initial_rounds.sage: initial MDS,
    round-0 constants, s-box, MDS); one round further differs; 30 rounds is the full
    permutation of k_p2_permute"""
    import torch
    k = KATS["poseidon2"]["P3_round0"]
    x = np.array([int(v) for v in k["input"]], np.uint64)
    st = torch.from_numpy(np.tile(x, 3).view(np.int64).copy()).cuda()
    ctx.check(ctx.lib.lf_dev_poseidon2_permute_rounds(ctx.h, st.data_ptr(), 3, 1))
    ctx.sync()
    assert [int(v) for v in st.cpu().numpy().view(np.uint64)[:16]] == k["mds_sbox_mds"]
    st2 = torch.from_numpy(x.view(np.int64).copy()).cuda()
    ctx.check(ctx.lib.lf_dev_poseidon2_permute_rounds(ctx.h, st2.data_ptr(), 1, 2))
    ctx.sync()
    assert [int(v) for v in st2.cpu().numpy().view(np.uint64)] != k["mds_sbox_mds"]
    st3 = torch.from_numpy(x.view(np.int64).copy()).cuda()
    ctx.check(ctx.lib.lf_dev_poseidon2_permute_rounds(ctx.h, st3.data_ptr(), 1, 30))
    ctx.sync()
    assert np.array_equal(st3.cpu().numpy().view(np.uint64), O.p2_permute(x))


def test_poseidon2_configs4_batch_sampled(ctx):
    """configs[4]'s batch: 2^20 independent width-16 states, sampled states against the oracle"""
    import torch
    m = 1 << 20
    st = torch.empty(16 * m, dtype=torch.int64, device="cuda")
    ctx.dev_fill_uniform(st, 0x4C460007)
    x = st.clone()
    ctx.dev_poseidon2_permute(st)
    ctx.sync()
    picks = [0, 1, 4095, 65536, 524287, m - 1]
    xs = x.view(m, 16)[picks].cpu().numpy().view(np.uint64).ravel()
    got = st.view(m, 16)[picks].cpu().numpy().view(np.uint64).ravel()
    assert np.array_equal(got, O.p2_permute(xs))


def test_fill_uniform_and_modp_sum(ctx):
    import torch
    t = torch.zeros(10007, dtype=torch.int64, device="cuda")
    ctx.dev_fill_uniform(t, 0x4C460003)
    ctx.sync()
    assert np.array_equal(t.cpu().numpy().view(np.uint64), O.fill_uniform(10007, 0x4C460003))
    parts = torch.from_numpy(rand(4 * 1000, 5).view(np.int64)).cuda()
    out = torch.zeros(1000, dtype=torch.int64, device="cuda")
    ctx.dev_modp_sum(parts, 4, 1000, out)
    ctx.sync()
    hp = parts.cpu().numpy().view(np.uint64).reshape(4, 1000).astype(object)
    assert [int(v) for v in out.cpu().numpy().view(np.uint64)] == [int(v) % P for v in hp.sum(0)]


def test_limb_transport_roundtrip(ctx):
    # RCCL transport of field vectors: 32-bit limb sums over ranks join mod p
    import torch
    parts = [rand(5000, 40 + r) for r in range(3)]
    lo_sum = torch.zeros(5000, dtype=torch.int64, device="cuda")
    hi_sum = torch.zeros(5000, dtype=torch.int64, device="cuda")
    for x in parts:
        t = torch.from_numpy(x.view(np.int64).copy()).cuda()
        lo, hi = torch.empty_like(t), torch.empty_like(t)
        ctx.dev_limb_split(t, lo, hi)
        lo_sum += lo
        hi_sum += hi
    out = torch.empty_like(lo_sum)
    ctx.dev_limb_join(lo_sum, hi_sum, out)
    ctx.sync()
    want = sum(x.astype(object) for x in parts) % P
    assert [int(v) for v in out.cpu().numpy().view(np.uint64)] == [int(v) for v in want]


@pytest.mark.parametrize("d,kappa,ncols,nvec", [(16, 3, 40, 5), (64, 32, 70, 29), (1024, 7, 33, 1),
                                                (1024, 32, 96, 29), (256, 17, 64, 32), (24, 3, 40, 5),
                                                (24, 32, 700, 29), (24, 9, 33, 1),
                                                # kappa > 32: 32-row tiles of A (ragged last tile)
                                                (16, 64, 40, 29), (1024, 33, 33, 3), (24, 64, 200, 29),
                                                (4096, 40, 17, 2), (64, 128, 40, 5), (24, 100, 35, 7)])
def test_ajtai_mfma_shapes(ctx, d, kappa, ncols, nvec):
    # the i8-MFMA contraction (signed base-256 limbs, A in registers) agrees with the oracle
    check_ajtai(ctx, d, kappa, ncols, nvec, layout=1)


@pytest.mark.parametrize("d,kappa,ncols,nvec", [(24, 129, 35, 3), (16, 160, 40, 5), (1024, 130, 9, 2)])
def test_ajtai_valu_wide_kappa(ctx, d, kappa, ncols, nvec):
    # kappa > 128 (more than LF_MAX_KTILES 32-row tiles of A): the VALU contraction
    check_ajtai(ctx, d, kappa, ncols, nvec, layout=0)


def check_ajtai(ctx, d, kappa, ncols, nvec, layout):
    import torch
    A = rand(kappa * ncols * d, 21 + d + kappa).reshape(kappa, ncols, d)
    # edge values in A: 0, p-1 and the D8 digit boundaries
    A.reshape(-1)[:6] = [0, P - 1, 0x7F7F7F7F7F7F7F7F, 0x7F7F7F7F7F7F7F80, (P - 1) // 2, 1]
    sch = LA.AjtaiCommitmentScheme(ctx, A)
    assert sch.layout == layout
    F = rand(nvec * ncols * d, 31 + d)
    F[:4] = [P - 1, 0x7F7F7F7F7F7F7F7F, 0x7F7F7F7F7F7F7F80, 0]
    Ft = torch.from_numpy(F.view(np.int64)).cuda()
    cm = torch.zeros(nvec * kappa * d, dtype=torch.int64, device="cuda")
    ctx.dev_ajtai_commit(sch, [Ft[v * ncols * d:(v + 1) * ncols * d] for v in range(nvec)], cm)
    ctx.sync()
    want = O.ajtai_commit(A, kappa, ncols, d, F, nvec)
    assert np.array_equal(cm.cpu().numpy().view(np.uint64), want)


@pytest.mark.parametrize("nch", [320, 329])
def test_ajtai_mfma_extreme_digits(ctx, nch):
    # all-(-128) digit products stress the i32 weight accumulators over a full
    # column split (d = 256: 320 chunks per split), and with 329 chunks a ragged
    # second split of 9 chunks
    import torch
    d, kappa, ncols, nvec = 256, 32, nch * 32, 32
    A = np.full(kappa * ncols * d, P - 1, np.uint64).reshape(kappa, ncols, d)
    F = np.full(nvec * ncols * d, P - 1, np.uint64)
    sch = LA.AjtaiCommitmentScheme(ctx, A)
    assert sch.layout == 1
    Ft = torch.from_numpy(F.view(np.int64)).cuda()
    cm = torch.zeros(nvec * kappa * d, dtype=torch.int64, device="cuda")
    ctx.dev_ajtai_commit(sch, [Ft[v * ncols * d:(v + 1) * ncols * d] for v in range(nvec)], cm)
    ctx.sync()
    # (p-1)^2 = 1 per column, so every entry is ncols mod p
    assert set(cm.cpu().numpy().view(np.uint64).tolist()) == {ncols}


def test_ajtai_mfma_phi72_extreme_digits(ctx):
    # Phi_72 through the Toom-3 virtual slots: all-(p-1) operands (every D8 digit
    # -1, every evaluation at its largest) over many column splits, against the oracle
    import torch
    d, kappa, ncols, nvec = 24, 32, 2000, 8
    A = np.full(kappa * ncols * d, P - 1, np.uint64).reshape(kappa, ncols, d)
    F = np.full(nvec * ncols * d, P - 1, np.uint64)
    sch = LA.AjtaiCommitmentScheme(ctx, A)
    assert sch.layout == 1
    Ft = torch.from_numpy(F.view(np.int64)).cuda()
    cm = torch.zeros(nvec * kappa * d, dtype=torch.int64, device="cuda")
    ctx.dev_ajtai_commit(sch, [Ft[v * ncols * d:(v + 1) * ncols * d] for v in range(nvec)], cm)
    ctx.sync()
    assert np.array_equal(cm.cpu().numpy().view(np.uint64), O.ajtai_commit(A, kappa, ncols, d, F, nvec))


# ------------------------------------------------------------------ the drop-in boundary in Montgomery form
def mont(x):
    return np.array([O.to_mont(int(v)) for v in np.asarray(x, np.uint64).ravel()], np.uint64)


def unmont(x):
    return np.array([O.from_mont(int(v)) for v in np.asarray(x, np.uint64).ravel()], np.uint64)


@pytest.mark.parametrize("d,W,kappa", [(24, 4, 3), (1024, 2, 2)])
def test_montgomery_boundary_commit_fold(ctx, d, W, kappa):
    """INTEGRATION.md's call sequence: a Rust host hands ark-ff limbs (a 2^64
    mod p) zero-copy to lf_ajtai_create, lf_commit and lf_fold_hot with
    LF_REPR_MONTGOMERY and reads Montgomery limbs back"""
    pr = params(d)
    N = W * pr.L
    A = rand(kappa * N * d, 1500 + d).reshape(kappa, N, d)
    sch = LA.AjtaiCommitmentScheme(ctx, mont(A).reshape(kappa, N, d), repr=LA.REPR_MONTGOMERY)
    l = 4
    w_ccs = rand(W * d, 1501 + d)
    z = np.concatenate([rand(l * d, 1502), np.zeros(d, np.uint64), w_ccs])
    z[l * d] = 1  # z = [x_ccs | 1 | w_ccs]
    fc, f, cm = ctx.commit(sch, mont(z), l, pr, repr=LA.REPR_MONTGOMERY)
    ofc, of = O.witness_from_w_ccs(w_ccs, d, pr.B, pr.L)
    ocm = O.ajtai_commit(A, kappa, N, d, of)
    assert np.array_equal(unmont(fc), ofc) and np.array_equal(unmont(f), of) and np.array_equal(unmont(cm), ocm)
    assert np.array_equal(sch.commit_ntt(mont(of), repr=LA.REPR_MONTGOMERY), mont(ocm))
    acc_fc, acc_f = valid_f_coeff(d, W, 1503 + d)
    acc_cm = O.ajtai_commit(A, kappa, N, d, acc_f)
    rho = make_rho(d, pr.K, 1504 + d)
    got = ctx.fold_hot(sch, pr, mont(acc_cm), mont(acc_fc), cm, fc, mont(rho), repr=LA.REPR_MONTGOMERY)
    want, _ = oracle_fold_hot(A, kappa, d, pr, acc_cm, acc_fc, ocm, ofc, rho)
    for key in want:
        assert np.array_equal(unmont(got[key]), want[key]), key


# ------------------------------------------------------------------ column-sharded fold
def dev(x=None, n=None):
    import torch
    if x is not None:
        return torch.from_numpy(np.ascontiguousarray(x).view(np.int64)).cuda()
    return torch.zeros(n, dtype=torch.int64, device="cuda")


def step_buffers(d, W, kappa, K, L, w_ccs, acc_cm, acc_fc, rho):
    N = W * L
    keep = {
        "w_ccs": dev(w_ccs), "acc_cm": dev(acc_cm), "acc_f_coeff": dev(acc_fc), "rho": dev(rho),
        "f_coeff": dev(n=N * d), "f": dev(n=N * d), "cm": dev(n=kappa * d),
        "fk_coeff": [dev(n=K * N * d) for _ in range(2)], "fk": [dev(n=K * N * d) for _ in range(2)],
        "wk": [dev(n=K * W * d) for _ in range(2)], "y": [dev(n=K * kappa * d) for _ in range(2)],
        "f0": dev(n=N * d), "f0_coeff": dev(n=N * d), "w_ccs0": dev(n=W * d), "cm0": dev(n=kappa * d),
    }
    b = LA.LfFoldStepBufs()
    for k, v in keep.items():
        if isinstance(v, list):
            for s_ in range(2):
                getattr(b, k)[s_] = v[s_].data_ptr()
        else:
            setattr(b, k, v.data_ptr())
    return keep, b


def sharded_setup(ctx, d, W, kappa, world, seed):
    """the full step's inputs and outputs, and one shard (scheme + buffers) per rank"""
    from latticeum_amd.dist import shard_groups
    pr = params(d)
    K, L = pr.K, pr.L
    N = W * L
    A = rand(kappa * N * d, seed).reshape(kappa, N, d)
    w_ccs = rand(W * d, seed + 1)
    acc_fc, acc_f = valid_f_coeff(d, W, seed + 2)
    acc_cm = O.ajtai_commit(A, kappa, N, d, acc_f)
    rho = make_rho(d, K, seed + 3)
    full = LA.AjtaiCommitmentScheme(ctx, A)
    keep, b = step_buffers(d, W, kappa, K, L, w_ccs, acc_cm, acc_fc, rho)
    ctx.dev_fold_step(full, pr, W, b)
    ctx.sync()
    shards = []
    for r in range(world):
        g0, g1 = shard_groups(W, r, world)
        Wr = g1 - g0
        sch = LA.AjtaiCommitmentScheme(ctx, np.ascontiguousarray(A[:, g0 * L:g1 * L]))
        kr, br = step_buffers(d, Wr, kappa, K, L, w_ccs[g0 * d:g1 * d], acc_cm, acc_fc[g0 * L * d:g1 * L * d], rho)
        shards.append({"g0": g0, "g1": g1, "W": Wr, "sch": sch, "keep": kr, "bufs": br})
    return pr, keep, shards


def assert_shards_match(pr, d, W, kappa, keep, shards):
    K, L = pr.K, pr.L
    N = W * L
    h = lambda t: t.cpu().numpy().view(np.uint64)
    for sh in shards:
        g0, g1, kr = sh["g0"], sh["g1"], sh["keep"]
        c0, c1 = g0 * L, g1 * L
        for key in ("cm", "cm0"):
            assert np.array_equal(h(kr[key]), h(keep[key])), key
        for s_ in range(2):
            assert np.array_equal(h(kr["y"][s_]), h(keep["y"][s_])), "y"
            for key, n_per, a, b_ in (("fk_coeff", N, c0, c1), ("fk", N, c0, c1), ("wk", W, g0, g1)):
                full = h(keep[key][s_]).reshape(K, n_per, d)[:, a:b_]
                assert np.array_equal(h(kr[key][s_]).reshape(K, b_ - a, d), full), key
        for key, a, b_ in (("f_coeff", c0, c1), ("f", c0, c1), ("f0", c0, c1), ("f0_coeff", c0, c1),
                           ("w_ccs0", g0, g1)):
            assert np.array_equal(h(kr[key]), h(keep[key])[a * d:b_ * d]), key


@pytest.mark.parametrize("d,W,kappa,world", [(24, 40, 4, 2), (1024, 37, 2, 3), (1024, 48, 3, 2), (64, 20, 40, 2)])
def test_sharded_step_partial_finish(ctx, d, W, kappa, world):
    """rank r's partial commitments over its columns, summed over ranks mod p,
    finish into the unsharded step's outputs bit-exactly (each rank's shard of
    the column-local outputs, the full commitments)"""
    import torch
    pr, keep, shards = sharded_setup(ctx, d, W, kappa, world, 1700 + d + W)
    n = ctx.fold_step_partial_len(shards[0]["sch"], pr)
    parts = []
    for sh in shards:
        p_ = dev(n=n)
        ctx.dev_fold_step_partial(sh["sch"], pr, sh["W"], sh["bufs"], p_)
        parts.append(p_)
    total = dev(n=n)
    ctx.dev_modp_sum(torch.cat(parts), world, n, total)
    for sh in shards:
        ctx.dev_fold_step_finish(sh["sch"], pr, sh["W"], sh["bufs"], total)
    ctx.sync()
    assert_shards_match(pr, d, W, kappa, keep, shards)


def test_sharded_step_two_gloo_ranks(ctx):
    """world_size 2 over gloo, one thread per rank, each with its own context
    and stream on GPU 0: partial commitments -> HIP limb split -> gloo
    all-reduce of the limbs -> HIP limb join -> finish, against the unsharded step"""
    import datetime
    import threading

    import torch
    import torch.distributed as dist
    d, W, kappa, world = 1024, 37, 2, 2
    pr, keep, shards = sharded_setup(ctx, d, W, kappa, world, 1800)
    n = ctx.fold_step_partial_len(shards[0]["sch"], pr)
    store = dist.HashStore()
    errors = []

    def rank_main(r):
        try:
            c = LA.Context(0)
            st = torch.cuda.Stream()
            c.set_stream(st.cuda_stream)
            sh = shards[r]
            pg = dist.ProcessGroupGloo(dist.PrefixStore("sharded", store), r, world, datetime.timedelta(seconds=60))
            with torch.cuda.stream(st):
                part, lo, hi = dev(n=n), dev(n=n), dev(n=n)
            c.dev_fold_step_partial(sh["sch"], pr, sh["W"], sh["bufs"], part)
            c.dev_limb_split(part, lo, hi)
            c.sync()
            limbs = torch.cat([lo, hi]).cpu()
            pg.allreduce([limbs]).wait()  # int64 sums of 32-bit limbs: exact
            with torch.cuda.stream(st):
                lo.copy_(limbs[:n].cuda())
                hi.copy_(limbs[n:].cuda())
            c.dev_limb_join(lo, hi, part)
            c.dev_fold_step_finish(sh["sch"], pr, sh["W"], sh["bufs"], part)
            c.sync()
            c.close()
        except Exception as e:  # surfaced by the main thread
            errors.append((r, e))

    th = [threading.Thread(target=rank_main, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert not errors, errors
    assert_shards_match(pr, d, W, kappa, keep, shards)


def test_rccl_comm_one_rank(ctx):
    """the C ABI's own RCCL path on one GPU: a one-rank communicator from a
    unique id; the limb all-reduce is then the identity, and the sharded step
    (partial, RCCL all-reduce, finish) is the unsharded step"""
    import torch
    comm = LA.Communicator(ctx, 1, 0, LA.Communicator.unique_id())
    assert comm.size == 1 and comm.rank == 0
    x = torch.from_numpy(rand(5000, 1900).view(np.int64)).cuda()
    want = x.clone()
    comm.allreduce_modp(x)
    ctx.sync()
    assert torch.equal(x, want)
    pr, keep, shards = sharded_setup(ctx, 1024, 21, 2, 1, 1950)
    sh = shards[0]
    ctx.dev_fold_step_sharded(sh["sch"], pr, sh["W"], sh["bufs"], comm)
    ctx.sync()
    assert_shards_match(pr, 1024, 21, 2, keep, shards)
    comm.close()


# ------------------------------------------------------------------ the rest of the folded LCCCS
@pytest.mark.parametrize("d", [24, 16, 1024, 4096])
def test_fold_lcccs_matches_oracle(ctx, d):
    """u_0 (t = 125 CCS matrices), x_0 (l + 1 = 5) and v_0 over the 2K = 30
    decomposed instances (compute_v0_u0_x0_cm_0, folding/utils.rs:456-517)"""
    pr = params(d)
    nwit, t, l1 = 2 * pr.K, 125, 5
    tau = 3 if d == 24 else 1
    rng = np.random.default_rng(2200 + d)
    rc = [O.short_challenge(rng.integers(0, 256, 3 * d // 4, dtype=np.uint8).tobytes(), d) for _ in range(nwit - 1)]
    one = np.zeros(d, np.uint64)
    one[0] = 1
    rho_coeff = np.concatenate(rc + [one])
    rho = O.crt(rho_coeff, d)
    eta, xwh, theta = rand(nwit * t * d, 2201 + d), rand(nwit * l1 * d, 2202 + d), rand(nwit * tau * d, 2203 + d)
    got = ctx.fold_lcccs(d, rho, rho_coeff, eta, xwh, theta)
    assert np.array_equal(got["u0"], O.fold_cm0(rho, eta, nwit, t, d))
    assert np.array_equal(got["x0"], O.fold_cm0(rho, xwh, nwit, l1, d))
    assert np.array_equal(got["v0"], O.rot_lin_combination(rho_coeff, theta, d))


def test_rot_lin_combination_kat_on_gpu(ctx):
    k = KATS["rot_lin_combination"]
    rc = np.array(k["rho_coeff"], np.uint64)
    got = ctx.fold_lcccs(24, O.crt(rc.ravel(), 24), rc, theta=np.array(k["theta_ntt"], np.uint64))
    assert [int(v) for v in got["v0"]] == k["expected_ntt"]


@pytest.mark.parametrize("d", [24, 1024])
def test_compute_x_s_matches_oracle(ctx, d):
    pr = params(d)
    x = rand(5 * d, 2300 + d)
    assert np.array_equal(ctx.compute_x_s(x, pr), O.compute_x_s(x, d, pr.B, pr.L, pr.b_small, pr.K))
    xm = ctx.compute_x_s(mont(x), pr, repr=LA.REPR_MONTGOMERY)
    assert np.array_equal(unmont(xm), O.compute_x_s(x, d, pr.B, pr.L, pr.b_small, pr.K))


def test_fold_lcccs_montgomery(ctx):
    d, nwit = 24, 30
    rho_coeff = rand(nwit * d, 2400)
    rho = O.crt(rho_coeff, d)
    eta, theta = rand(nwit * 7 * d, 2401), rand(nwit * 3 * d, 2402)
    got = ctx.fold_lcccs(d, mont(rho), mont(rho_coeff), mont(eta), None, mont(theta), repr=LA.REPR_MONTGOMERY)
    assert np.array_equal(unmont(got["u0"]), O.fold_cm0(rho, eta, nwit, 7, d))
    assert np.array_equal(unmont(got["v0"]), O.rot_lin_combination(rho_coeff, theta, d))
