"""The oracle's sumcheck restatement pinned by the
reference's own prove -> verify relation (latticefold/src/utils/sumcheck.rs
tests, folding/tests/mod.rs): the prover's messages pass the verifier's
round checks (verifier.rs:100-129) for the hypercube sum computed by brute
force, and the final claim equals the combination function at the MLEs'
evaluations at the challenge point. The reference holds no sumcheck KAT, so
this relation (plus eq-table and evaluation identities) is the pin; the GPU
prover is compared with this oracle bit for bit in tests/test_gpu_sumcheck.py."""
import numpy as np
import pytest

import oracle as O

P = O.P


def rand(n, seed):
    return O.fill_uniform(n, seed)


def folding_case(d, nv, nk, tau, seed):
    """MLEs shaped like create_sumcheck_polynomial's (folding/utils.rs:196-255):
    [eq(r0), g0, eq(r1), g1, eq(beta), f_hat (nk x tau)]"""
    n = 1 << nv
    r0, r1, beta = (rand(nv * d, seed + i) for i in range(3))
    mles = [O.eq_table(r0, nv, d), rand(n * d, seed + 3), O.eq_table(r1, nv, d), rand(n * d, seed + 4),
            O.eq_table(beta, nv, d)]
    mles += [rand(n * d, seed + 10 + i) for i in range(nk * tau)]
    mu = rand(nk * d, seed + 5)
    return np.concatenate(mles), mu, 5 + nk * tau


def brute_sum(comb, mles, nm, nv, d):
    n = 1 << nv
    m = mles.reshape(nm, n, d)
    s = np.zeros(d, object)
    for x in range(n):
        s = (s + O.comb_eval(comb, m[:, x].ravel(), nm, d).astype(object)) % P
    return s.astype(np.uint64)


def final_claim(comb, mles, nm, nv, d, rnd):
    n = 1 << nv
    tau = 3 if d == 24 else 1
    point = np.concatenate([O.broadcast(rnd[i * tau:(i + 1) * tau], d) for i in range(nv)])
    vals = np.concatenate([O.mle_evaluate(mles.reshape(nm, n * d)[m], nv, d, point) for m in range(nm)])
    return O.comb_eval(comb, vals, nm, d)


@pytest.mark.parametrize("d", [24, 16])
def test_eq_table_and_evaluate(d):
    nv = 4
    r = rand(nv * d, 7 + d)
    eq = O.eq_table(r, nv, d).reshape(1 << nv, d)
    one = np.zeros(d, np.uint64)
    one[::3 if d == 24 else 1] = 1
    for x in range(1 << nv):  # eq[x] = prod_k (x_k ? r_k : 1 - r_k)
        acc = one
        for k in range(nv):
            rk = r[k * d:(k + 1) * d]
            f = rk if (x >> k) & 1 else np.array([(int(a) - int(b)) % P for a, b in zip(one, rk)], np.uint64)
            acc = O.slot_mul(acc, f, d)
        assert np.array_equal(eq[x], acc)
    mle = rand((1 << nv) * d, 8 + d)
    want = np.zeros(d, object)
    for x in range(1 << nv):  # evaluate(point) = sum_x eq(point, x) mle(x)
        want = (want + O.slot_mul(eq[x], mle[x * d:(x + 1) * d], d).astype(object)) % P
    assert np.array_equal(O.mle_evaluate(mle, nv, d, r), want.astype(np.uint64))


@pytest.mark.parametrize("d,nv,nk,tau", [(24, 4, 4, 3), (16, 5, 6, 1)])
def test_folding_sumcheck_prove_verify(d, nv, nk, tau):
    mles, mu, nm = folding_case(d, nv, nk, tau, 100 + d)
    comb = O.SumcheckComb.folding(mu, nk, tau, 2)
    proof, rnd = O.sumcheck_prove(O.new_transcript(), comb, mles, nm, nv, d, 4)
    asserted = brute_sum(comb, mles, nm, nv, d)
    rc, expected = O.sumcheck_check(proof, rnd, nv, d, 4, asserted)
    assert rc == 0
    assert np.array_equal(expected, final_claim(comb, mles, nm, nv, d, rnd))
    bad = proof.copy()
    bad[3 * (4 + 1) * d] ^= 1  # round 3's p(0)
    assert O.sumcheck_check(bad, rnd, nv, d, 4, asserted)[0] == -4


@pytest.mark.parametrize("d", [24, 64])
def test_linearization_sumcheck_prove_verify(d):
    """R1CS-shaped CCS (arith/ccs.rs x^3 + x + 5): c = [1, -1], S = [[0, 1], [2]],
    degree d_ccs + 1 = 3; MLE list [M0 z, M1 z, M2 z, eq(beta)]"""
    nv = 4
    n = 1 << nv
    mz = [rand(n * d, 300 + d + j) for j in range(3)]
    beta = rand(nv * d, 310 + d)
    mles = np.concatenate(mz + [O.eq_table(beta, nv, d)])
    one = np.zeros(d, np.uint64)
    one[::3 if d == 24 else 1] = 1
    c = np.concatenate([one, np.where(one == 1, np.uint64(P - 1), np.uint64(0))])
    comb = O.SumcheckComb.linearization(c, [[0, 1], [2]])
    proof, rnd = O.sumcheck_prove(O.new_transcript(), comb, mles, 4, nv, d, 3)
    asserted = brute_sum(comb, mles, 4, nv, d)
    rc, expected = O.sumcheck_check(proof, rnd, nv, d, 3, asserted)
    assert rc == 0
    assert np.array_equal(expected, final_claim(comb, mles, 4, nv, d, rnd))


def test_mz_oracle_identities():
    """mat_vec_mul row by row, zero-padded MLEs, and the challenged Horner
    (folding.rs:208-234) = sum_j zeta^(j+1) M_j z"""
    d, m, n, nv = 24, 6, 5, 3
    rp = np.array([0, 2, 2, 5, 6, 6, 8], np.uint64)
    col = np.array([0, 4, 1, 1, 3, 2, 0, 4], np.uint32)
    val = O.fill_uniform(8 * d, 3)
    z = O.fill_uniform(n * d, 4)
    y = O.spmv(rp, col, val, d, z).reshape(m, d)
    for r in range(m):
        acc = np.zeros(d, object)
        for k in range(int(rp[r]), int(rp[r + 1])):
            acc = (acc + O.slot_mul(val[k * d:(k + 1) * d], z[col[k] * d:(col[k] + 1) * d], d).astype(object)) % P
        assert np.array_equal(y[r], acc.astype(np.uint64))
    mats = [(rp, col, val), (rp, col[::-1].copy(), val[::-1].copy())]
    ml = O.mz_mles(mats, z, nv, d).reshape(2, 1 << nv, d)
    assert not ml[:, m:].any()
    zeta = O.fill_uniform(d, 5)
    z2 = O.slot_mul(zeta, zeta, d)
    want = O.fold_cm0(np.concatenate([zeta, z2]), ml.ravel(), 2, 1 << nv, d)
    assert np.array_equal(O.mz_challenged(mats, [z], [zeta], nv, d), want)
