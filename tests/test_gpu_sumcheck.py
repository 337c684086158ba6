"""GPU parity of the multilinear sumcheck prover
against the oracle's restatement: eq tables, fix_variables, MLE evaluation,
single round sums of the folding and linearization polynomials, and whole
proofs through the Poseidon2 transcript (bit-identical messages and
challenges). At the reference's real shape (Phi_72, 17 variables, the 95 MLEs
of the folding polynomial) the device proof is checked with the oracle's
verifier (round sums, interpolation) and its final claim against the MLEs
evaluated at the challenge point."""
import numpy as np
import pytest

import latticeum_amd as LA
import oracle as O
from test_sumcheck_oracle import final_claim, folding_case

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


def dev32(x):
    import torch
    return torch.from_numpy(np.ascontiguousarray(x, np.int32)).cuda()


def host(t):
    return t.cpu().numpy().view(np.uint64)


def rand(n, seed):
    return O.fill_uniform(n, seed)


@pytest.mark.parametrize("d,nv", [(24, 6), (16, 5), (1024, 3)])
def test_eq_table_fix_evaluate(ctx, d, nv):
    n = 1 << nv
    r = rand(nv * d, 10 + d)
    eq = dev(n=n * d)
    ctx.dev_eq_table(d, dev(r), nv, eq)
    ctx.sync()
    assert np.array_equal(host(eq), O.eq_table(r, nv, d))
    nm = 3
    mles = rand(nm * n * d, 11 + d)
    out = dev(n=nm * d)
    ctx.dev_mle_evaluate(d, dev(mles), nm, nv, dev(r), out)
    ctx.sync()
    want = np.concatenate([O.mle_evaluate(mles[m * n * d:(m + 1) * n * d], nv, d, r) for m in range(nm)])
    assert np.array_equal(host(out), want)
    tau = 3 if d == 24 else 1
    rb = rand(tau, 12 + d)
    fixed = dev(n=nm * (n // 2) * d)
    ctx.dev_mle_fix_first(d, dev(mles), n * d, nm, nv, rb, fixed, (n // 2) * d)
    ctx.sync()
    for m in range(nm):
        ref = mles[m * n * d:(m + 1) * n * d].copy()
        O.lib().lfo_mle_fix_first(ref, n // 2, d, O.broadcast(rb, d))
        assert np.array_equal(host(fixed)[m * (n // 2) * d:(m + 1) * (n // 2) * d], ref[:(n // 2) * d])


@pytest.mark.parametrize("d,nv,nk,tau", [(24, 6, 30, 3), (16, 5, 4, 1), (1024, 2, 3, 1), (24, 1, 2, 3)])
def test_folding_round_matches_oracle(ctx, d, nv, nk, tau):
    mles, mu, nm = folding_case(d, nv, nk, tau, 500 + d + nv)
    comb = O.SumcheckComb.folding(mu, nk, tau, 2)
    want = O.sumcheck_round(comb, mles, nm, nv, d, 4)
    ev = dev(n=5 * d)
    ctx.dev_sumcheck_round(LA.Comb.folding(dev(mu), nk, tau, 2), dev(mles), (1 << nv) * d, nm, nv, d, 4, ev)
    ctx.sync()
    assert np.array_equal(host(ev), want)


def lin_case(d, nv, seed):
    """a CCS with degree-3 and degree-1 multisets and a zero coefficient: c = [3, 0, -1, 5],
    S = [[0, 1, 2], [1], [3], [0, 3]]; the MLE list as prepare_lin_sumcheck_polynomial builds it"""
    n = 1 << nv
    one = np.zeros(d, np.uint64)
    one[::3 if d == 24 else 1] = 1
    c = np.concatenate([one * np.uint64(3), np.zeros(d, np.uint64), np.where(one == 1, np.uint64(P - 1), np.uint64(0)),
                        rand(d, seed)])
    S = [[0, 1, 2], [1], [3], [0, 3]]
    mz = [rand(n * d, seed + 1 + j) for j in range(4)]
    beta = rand(nv * d, seed + 9)
    lst = [mz[j] for i, s_ in enumerate(S) if i != 1 for j in s_]
    mles = np.concatenate(lst + [O.eq_table(beta, nv, d)])
    return c, S, mles, len(lst) + 1


@pytest.mark.parametrize("d,nv", [(24, 5), (64, 4)])
def test_linearization_round_matches_oracle(ctx, d, nv):
    c, S, mles, nm = lin_case(d, nv, 600 + d)
    want = O.sumcheck_round(O.SumcheckComb.linearization(c, S), mles, nm, nv, d, 4)
    ev = dev(n=5 * d)
    ctx.dev_sumcheck_round(LA.Comb.linearization(dev(c), S), dev(mles), (1 << nv) * d, nm, nv, d, 4, ev)
    ctx.sync()
    assert np.array_equal(host(ev), want)


@pytest.mark.parametrize("d,nv,nk,tau", [(24, 7, 30, 3), (16, 6, 5, 1)])
def test_folding_prove_matches_oracle(ctx, d, nv, nk, tau):
    mles, mu, nm = folding_case(d, nv, nk, tau, 700 + d)
    want_p, want_r = O.sumcheck_prove(O.new_transcript(), O.SumcheckComb.folding(mu, nk, tau, 2), mles, nm, nv, d, 4)
    t = LA.Poseidon2Transcript()
    proof, rnd = ctx.sumcheck_prove(t, LA.Comb.folding(dev(mu), nk, tau, 2), dev(mles), nm, nv, d, 4)
    assert np.array_equal(proof, want_p) and np.array_equal(rnd, want_r)


def test_linearization_prove_matches_oracle(ctx):
    d, nv = 24, 6
    c, S, mles, nm = lin_case(d, nv, 800)
    want_p, want_r = O.sumcheck_prove(O.new_transcript(), O.SumcheckComb.linearization(c, S), mles, nm, nv, d, 4)
    proof, rnd = ctx.sumcheck_prove(LA.Poseidon2Transcript(), LA.Comb.linearization(dev(c), S), dev(mles), nm, nv,
                                    d, 4)
    assert np.array_equal(proof, want_p) and np.array_equal(rnd, want_r)


def test_folding_sumcheck_real_shape(ctx):
    """the zkvm's folding sumcheck: Phi_72, log m = 17, 2K = 30 instances of
    tau = 3 f_hat MLEs (95 MLEs, 2.4 GB): the device proof passes the oracle's
    verifier and its final claim is the combination at the evaluated MLEs"""
    import torch
    d, nv, nk, tau = 24, 17, 30, 3
    n = 1 << nv
    nm = 5 + nk * tau
    m = dev(n=nm * n * d)
    ctx.dev_fill_uniform(m, 900)
    r = dev(rand(3 * nv * d, 901))
    for i, k in enumerate((0, 2, 4)):  # the eq MLEs
        ctx.dev_eq_table(d, r[i * nv * d:(i + 1) * nv * d], nv, m[k * n * d:(k + 1) * n * d])
    mu = rand(nk * d, 902)
    keep = m.clone()
    proof, rnd = ctx.sumcheck_prove(LA.Poseidon2Transcript(), LA.Comb.folding(dev(mu), nk, tau, 2), m, nm, nv, d, 4)
    asserted = np.array([(int(a) + int(b)) % P for a, b in zip(proof[:d], proof[d:2 * d])], np.uint64)
    rc, expected = O.sumcheck_check(proof, rnd, nv, d, 4, asserted)
    assert rc == 0
    point = np.concatenate([O.broadcast(rnd[i * tau:(i + 1) * tau], d) for i in range(nv)])
    vals = dev(n=nm * d)
    ctx.dev_mle_evaluate(d, keep, nm, nv, dev(point), vals)
    ctx.sync()
    comb = O.SumcheckComb.folding(mu, nk, tau, 2)
    assert np.array_equal(expected, O.comb_eval(comb, host(vals), nm, d))
    del keep, m
    torch.cuda.empty_cache()


@pytest.mark.parametrize("d,N,nv", [(24, 13, 4), (24, 16, 4), (1024, 5, 3), (16, 1, 0)])
def test_get_fhat_matches_oracle(ctx, d, N, nv):
    """Witness::get_fhat (arith.rs:273-297): Phi_72 against the oracle's
    restatement, X^d + 1 as the coefficients themselves; zero past N"""
    fc = rand(N * d, 40 + d + N)
    tau = 3 if d == 24 else 1
    n = 1 << nv
    out = dev(n=tau * n * d)
    ctx.dev_get_fhat(d, dev(fc), N, nv, out)
    ctx.sync()
    got = host(out).reshape(tau, n, d)
    want = O.get_fhat_phi72(fc).reshape(tau, N, d) if d == 24 else fc.reshape(1, N, d)
    assert np.array_equal(got[:, :N], want)
    assert not got[:, N:].any()


def lin_eq_case(d, nv, sizes, seed):
    """multisets of the given sizes over nmz Mz MLEs (indices repeat across multisets), a
    coefficient that is zero in some slots, and the MLE list [mz..., eq(beta)]"""
    rng = np.random.default_rng(seed)
    n = 1 << nv
    nmz = max(3, max(sizes))
    S = [[int(j) for j in rng.integers(0, nmz, k)] for k in sizes]
    c = rand(len(sizes) * d, seed + 1)
    c[:d // 2] = 0  # c_0 vanishes in the first slots
    mz = [rand(n * d, seed + 2 + j) for j in range(nmz)]
    beta = rand(nv * d, seed + 99)
    tb = 3 if d == 24 else 1
    beta = np.concatenate([O.broadcast(beta[i * d:i * d + tb], d) for i in range(nv)])  # base-ring challenges
    return c, S, mz, beta


@pytest.mark.parametrize("d,nv,sizes", [(24, 6, [7, 1, 2, 0, 3]), (24, 5, [8, 5, 6, 4, 1]), (64, 4, [7, 2, 5]),
                                        (24, 1, [3, 2]), (1024, 3, [4, 7])])
def test_linearization_prove_lin_matches_oracle(ctx, d, nv, sizes):
    """lf_sumcheck_prove_lin (eq(beta) split off, pointer table, two-group products) gives
    the oracle's proof over [mz..., eq(beta)], multisets of 0 .. 8 factors"""
    c, S, mz, beta = lin_eq_case(d, nv, sizes, 1000 + d + nv)
    degree = max(sizes) + 1
    mles = np.concatenate(mz + [O.eq_table(beta, nv, d)])
    want_p, want_r = O.sumcheck_prove(O.new_transcript(), O.SumcheckComb.linearization(c, S), mles, len(mz) + 1, nv,
                                      d, degree)
    work = dev(n=max(1, len(mz) * (1 << max(nv - 2, 0)) * d))
    evals = dev(n=len(mz) * d)
    proof, rnd = ctx.sumcheck_prove_lin(LA.Poseidon2Transcript(), LA.Comb.linearization(dev(c), S),
                                        [dev(m) for m in mz], nv, d, degree, beta, work, evals)
    assert np.array_equal(proof, want_p) and np.array_equal(rnd, want_r)
    # the MLEs' final values are their evaluations at the challenge point
    tau = 3 if d == 24 else 1
    point = np.concatenate([O.broadcast(rnd[i * tau:(i + 1) * tau], d) for i in range(nv)])
    ctx.sync()
    assert np.array_equal(host(evals), np.concatenate([O.mle_evaluate(m, nv, d, point) for m in mz]))


def sparse_lists(mz, S, c, nv, d, rng, frac=0.3):
    """zero whole lines (rows 2b, 2b + 1) of each MLE with probability frac; the active
    points of each multiset (every factor's line nonzero; none when c_i vanishes)"""
    half = 1 << (nv - 1)
    live = []
    for m in mz:
        on = rng.random(half) >= frac
        m.reshape(half, 2 * d)[~on] = 0
        live.append(on)
    act, off = [], [0]
    for i, Si in enumerate(S):
        on = np.ones(half, bool)
        for j in Si:
            on &= live[j]
        if not c[i * d:(i + 1) * d].any():
            on[:] = False
        act.extend(np.nonzero(on)[0].tolist())
        off.append(len(act))
    return np.array(act or [0], np.int32), np.array(off, np.uint32)


@pytest.mark.parametrize("d,nv,sizes", [(24, 6, [7, 1, 2, 0, 3]), (24, 5, [8, 5, 6, 4, 1]), (64, 4, [7, 2, 5]),
                                        (24, 1, [3, 2]), (1024, 3, [4, 7])])
def test_linearization_prove_lin_sparse_matches_oracle(ctx, d, nv, sizes):
    """lf_sumcheck_prove_lin_sparse (round 0 over each multiset's active points only) on
    MLEs with zero lines gives the oracle's proof and final values; one multiset's c
    vanishes entirely and gets no points"""
    c, S, mz, beta = lin_eq_case(d, nv, sizes, 2000 + d + nv)
    c[(len(sizes) - 1) * d:] = 0
    act, off = sparse_lists(mz, S, c, nv, d, np.random.default_rng(d + nv))
    degree = max(sizes) + 1
    mles = np.concatenate(mz + [O.eq_table(beta, nv, d)])
    want_p, want_r = O.sumcheck_prove(O.new_transcript(), O.SumcheckComb.linearization(c, S), mles, len(mz) + 1, nv,
                                      d, degree)
    work = dev(n=max(1, len(mz) * (1 << max(nv - 2, 0)) * d))
    evals = dev(n=len(mz) * d)
    act_d = dev32(act)
    proof, rnd = ctx.sumcheck_prove_lin_sparse(LA.Poseidon2Transcript(), LA.Comb.linearization(dev(c), S),
                                               [dev(m) for m in mz], nv, d, degree, beta, act_d, off, work, evals)
    assert np.array_equal(proof, want_p) and np.array_equal(rnd, want_r)
    tau = 3 if d == 24 else 1
    point = np.concatenate([O.broadcast(rnd[i * tau:(i + 1) * tau], d) for i in range(nv)])
    ctx.sync()
    assert np.array_equal(host(evals), np.concatenate([O.mle_evaluate(m, nv, d, point) for m in mz]))


def test_linearization_prove_lin_sparse_matches_dense_at_size(ctx):
    """Phi_72, 14 variables, the zkvm's multiset sizes, a third of the lines zero: the
    sparse round 0 against the dense prover"""
    d, nv = 24, 14
    n = 1 << nv
    sizes = [7] * 6 + [1, 2] * 6 + [0]
    rng = np.random.default_rng(81)
    nmz = 40
    S = [[int(j) for j in rng.integers(0, nmz, k)] for k in sizes]
    c = rand(len(sizes) * d, 82)
    mz = [rand(n * d, 83 + j) for j in range(nmz)]
    act, off = sparse_lists(mz, S, c, nv, d, rng)
    beta = np.concatenate([O.broadcast(rand(3, 180 + i), d) for i in range(nv)])
    mzd = [dev(m) for m in mz]
    work = dev(n=nmz * (n // 4) * d)
    ev0, ev1 = dev(n=nmz * d), dev(n=nmz * d)
    want_p, want_r = ctx.sumcheck_prove_lin(LA.Poseidon2Transcript(), LA.Comb.linearization(dev(c), S), mzd, nv, d, 8,
                                            beta, work, ev0)
    proof, rnd = ctx.sumcheck_prove_lin_sparse(LA.Poseidon2Transcript(), LA.Comb.linearization(dev(c), S), mzd, nv, d,
                                               8, beta, dev32(act), off, work, ev1)
    ctx.sync()
    assert np.array_equal(proof, want_p) and np.array_equal(rnd, want_r)
    assert np.array_equal(host(ev0), host(ev1))


def test_linearization_prove_lin_matches_unsplit_at_size(ctx):
    """the zkvm's shape in miniature on the device: Phi_72, 14 variables, 7-factor S-box
    multisets and 1- and 2-factor ones; the split prover against the unsplit one"""
    d, nv = 24, 14
    n = 1 << nv
    sizes = [7] * 6 + [1, 2] * 6
    rng = np.random.default_rng(77)
    nmz = 40
    S = [[int(j) for j in rng.integers(0, nmz, k)] for k in sizes]
    c = rand(len(sizes) * d, 78)
    mz = dev(n=nmz * n * d)
    ctx.dev_fill_uniform(mz, 79)
    beta = np.concatenate([O.broadcast(rand(3, 80 + i), d) for i in range(nv)])
    full = dev(n=(nmz + 1) * n * d)
    full[:nmz * n * d] = mz
    ctx.dev_eq_table(d, dev(beta), nv, full[nmz * n * d:])
    want_p, want_r = ctx.sumcheck_prove(LA.Poseidon2Transcript(), LA.Comb.linearization(dev(c), S), full, nmz + 1, nv,
                                        d, 8)
    work = dev(n=nmz * (n // 4) * d)
    proof, rnd = ctx.sumcheck_prove_lin(LA.Poseidon2Transcript(), LA.Comb.linearization(dev(c), S),
                                        [mz[j * n * d:(j + 1) * n * d] for j in range(nmz)], nv, d, 8, beta, work)
    assert np.array_equal(proof, want_p) and np.array_equal(rnd, want_r)


@pytest.mark.parametrize("d,nv,K,N", [(24, 6, 3, 50), (24, 9, 4, 512), (16, 5, 2, 30), (1024, 3, 2, 7)])
def test_folding_prove_digits_matches_materialised(ctx, d, nv, K, N):
    """lf_sumcheck_prove_fold_digits (round 0 and its fix read from the digit rows, no f_hat
    MLEs) gives the proof of the prover over the materialised get_fhat MLEs; N < 2^nv and
    N = 2^nv (zero padding and none)"""
    import torch
    tau = 3 if d == 24 else 1
    n = 1 << nv
    rng = np.random.default_rng(d * 7 + nv)

    def digits():
        x = rng.integers(-1, 2, N * d)
        return np.where(x < 0, np.uint64(P - 1), x.astype(np.uint64))
    fc0 = dev(np.concatenate([digits() for _ in range(K)]))
    fc1 = dev(np.concatenate([digits() for _ in range(K)]))
    gen = [rand(n * d, 1300 + d + i) for i in range(5)]
    mu = rand(2 * K * d, 1310 + d)
    nm = 5 + 2 * K * tau
    full = dev(n=nm * n * d)
    full[:5 * n * d] = dev(np.concatenate(gen))
    for side, fc in enumerate((fc0, fc1)):
        for k in range(K):
            o = (5 + (side * K + k) * tau) * n * d
            ctx.dev_get_fhat(d, fc[k * N * d:(k + 1) * N * d], N, nv, full[o:o + tau * n * d])
    mles5 = full[:5 * n * d].clone()
    want_p, want_r = ctx.sumcheck_prove(LA.Poseidon2Transcript(), LA.Comb.folding(dev(mu), 2 * K, tau, 2), full, nm, nv,
                                        d, 4)
    work = dev(n=nm * max(n // 4, 1) * d)
    got_p, got_r = ctx.sumcheck_prove_fold_digits(LA.Poseidon2Transcript(), LA.Comb.folding(dev(mu), 2 * K, tau, 2),
                                                  mles5, fc0, fc1, K, N, N * d, nv, d, work)
    assert np.array_equal(got_p, want_p) and np.array_equal(got_r, want_r)
    del full
    torch.cuda.empty_cache()


def test_linearization_prove_lin_sparse_rejects_bad_lists(ctx):
    """act_off must start at 0, not decrease and hold at most 2^(nv-1) points per multiset"""
    d, nv, sizes = 24, 4, [3, 1]
    c, S, mz, beta = lin_eq_case(d, nv, sizes, 3001)
    work = dev(n=len(mz) * (1 << (nv - 2)) * d)
    act = dev32(np.zeros(4, np.int32))
    for off in ([1, 2, 3], [0, 3, 2], [0, 9, 9]):
        with pytest.raises(LA.LfError):
            ctx.sumcheck_prove_lin_sparse(LA.Poseidon2Transcript(), LA.Comb.linearization(dev(c), S),
                                          [dev(m) for m in mz], nv, d, 4, beta, act, np.array(off, np.uint32), work)
