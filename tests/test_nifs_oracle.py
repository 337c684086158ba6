"""The oracle's restatement of the zkvm's fold() prover (oracle/nifs.py,
zk_latticefold_prove, ZK/zk_latticefold.rs:37-102) pinned by relations, as the
reference pins its own NIFS (LF/nifs/tests.rs:58-203 prove -> verify): on a
satisfied CCS the restated NIFS verifier accepts the proof and re-derives the
prover's folded LCCCS; the folded LCCCS is the folded witness's (cm_0 = A f_0,
v_0 = f_hat(f_0)(r_0), u_0 = MLE(M_j z_0)(r_0)); a tampered proof or an
unsatisfied CCS is rejected. CPU only (small CCS)."""
import numpy as np
import pytest

import nifs as N
import oracle as O


def instance(d, W=5, l=2, t=4, deg=2, kappa=3, seed=7, satisfied=True):
    pr = N.Params(d)
    ccs = N.satisfied_ccs(d, W, l, t, deg, seed, pr)
    xa, wa = N.satisfying_z(ccs, W, seed + 4)
    xi, wi = N.satisfying_z(ccs, W, seed + 5)
    if not satisfied:
        wi = wi.copy()
        wi[-d:] = O.fill_uniform(d, seed + 9)  # a product column that no longer matches its row
    Nn = W * pr.L
    A = O.fill_uniform(kappa * Nn * d, seed + 6)

    def wit(w):
        fc, f = O.witness_from_w_ccs(w, d, pr.B, pr.L)
        return N.Witness(w_ccs=w, f=f, f_coeff=fc)

    Wa, Wi = wit(wa), wit(wi)
    cma = O.ajtai_commit(A, kappa, Nn, d, Wa.f)
    cmi = O.ajtai_commit(A, kappa, Nn, d, Wi.f)
    acc = N.linearize_fresh(ccs, cma, xa, Wa, pr)
    return pr, ccs, A, kappa, acc, Wa, cmi, xi, Wi


def same_lcccs(a, b):
    for k in ("r", "v", "u", "x_w"):
        x, y = getattr(a, k), getattr(b, k)
        assert len(x) == len(y) and all(np.array_equal(p, q) for p, q in zip(x, y)), k
    assert np.array_equal(a.cm, b.cm) and np.array_equal(a.h, b.h)


@pytest.mark.parametrize("d,deg", [(24, 2), (24, 3), (16, 2)])
def test_fold_prove_verifies(d, deg):
    pr, ccs, A, kappa, acc, Wa, cmi, xi, Wi = instance(d, deg=deg, t=deg + 2)
    for x, w in ((acc.x_w, Wa.w_ccs), (xi, Wi.w_ccs)):
        assert N.check_relation(ccs, np.concatenate(list(x) + [N.one(d), w]))
    out, w0, proof = N.fold_prove(ccs, A, kappa, acc, Wa, cmi, xi, Wi, pr)
    same_lcccs(out, N.fold_verify(ccs, acc, cmi, xi, proof, pr))
    # the folded instance is the folded witness's
    s, Nn = ccs.s, w0.f.size // d
    assert np.array_equal(out.cm, O.ajtai_commit(A, kappa, Nn, d, w0.f))
    r0 = np.concatenate(out.r)
    assert np.array_equal(np.concatenate(out.v), N.evaluate(N.fhat(w0.f_coeff, Nn, s, d), s, d, r0))
    z0 = np.concatenate(list(out.x_w) + [out.h, w0.w_ccs])
    assert np.array_equal(np.concatenate(out.u), N.evaluate(N.mz_mles(ccs, z0), s, d, r0))
    # and it folds again: the folded accumulator with a third instance
    x3, w3 = N.satisfying_z(ccs, Wa.w_ccs.size // d, 99)
    fc3, f3 = O.witness_from_w_ccs(w3, d, pr.B, pr.L)
    W3 = N.Witness(w_ccs=w3, f=f3, f_coeff=fc3)
    cm3 = O.ajtai_commit(A, kappa, Nn, d, f3)
    out2, _, proof2 = N.fold_prove(ccs, A, kappa, out, w0, cm3, x3, W3, pr)
    same_lcccs(out2, N.fold_verify(ccs, out, cm3, x3, proof2, pr))


def test_fold_verify_rejects_tampering():
    pr, ccs, A, kappa, acc, Wa, cmi, xi, Wi = instance(24)
    _, _, proof = N.fold_prove(ccs, A, kappa, acc, Wa, cmi, xi, Wi, pr)
    bad = N.Proof(**{**proof.__dict__, "theta_s": [list(t) for t in proof.theta_s]})
    bad.theta_s[3][1] = N.add(bad.theta_s[3][1], N.one(24))
    with pytest.raises(ValueError, match="folding evaluation claim"):
        N.fold_verify(ccs, acc, cmi, xi, bad, pr)
    bad = N.Proof(**{**proof.__dict__, "dec": [dict(proof.dec[0]), proof.dec[1]]})
    bad.dec[0]["y_s"] = [list(y) for y in proof.dec[0]["y_s"]]
    bad.dec[0]["y_s"][2][0] = N.add(bad.dec[0]["y_s"][2][0], N.one(24))
    with pytest.raises(ValueError, match="recompose y"):
        N.fold_verify(ccs, acc, cmi, xi, bad, pr)
    bad = N.Proof(**{**proof.__dict__, "lin_u": list(proof.lin_u)})
    bad.lin_u[0] = N.add(bad.lin_u[0], N.one(24))
    with pytest.raises(ValueError, match="linearization evaluation claim"):
        N.fold_verify(ccs, acc, cmi, xi, bad, pr)


def test_fold_verify_rejects_unsatisfied_ccs():
    pr, ccs, A, kappa, acc, Wa, cmi, xi, Wi = instance(24, satisfied=False)
    assert not N.check_relation(ccs, np.concatenate(list(xi) + [N.one(24), Wi.w_ccs]))
    _, _, proof = N.fold_prove(ccs, A, kappa, acc, Wa, cmi, xi, Wi, pr)
    with pytest.raises(ValueError, match="linearization"):
        N.fold_verify(ccs, acc, cmi, xi, proof, pr)


def test_vectorised_ccs_builder_is_satisfied():
    """satisfied_ccs_np (the large-shape builder) gives satisfiable CCS instances too"""
    pr = N.Params(24)
    ccs = N.satisfied_ccs_np(24, 13, 4, 6, 3, 5, pr)
    x, w = N.satisfying_z(ccs, 13, 6)
    assert N.check_relation(ccs, np.concatenate(list(x) + [N.one(24), w]))
    # and it folds: prove -> verify
    Nn = 13 * pr.L
    A = O.fill_uniform(2 * Nn * 24, 8)

    def wit(ww):
        fc, f = O.witness_from_w_ccs(ww, 24, pr.B, pr.L)
        return N.Witness(w_ccs=ww, f=f, f_coeff=fc)

    xa, wa = N.satisfying_z(ccs, 13, 9)
    Wa, Wi = wit(wa), wit(w)
    acc = N.linearize_fresh(ccs, O.ajtai_commit(A, 2, Nn, 24, Wa.f), xa, Wa, pr)
    cmi = O.ajtai_commit(A, 2, Nn, 24, Wi.f)
    out, _, proof = N.fold_prove(ccs, A, 2, acc, Wa, cmi, x, Wi, pr)
    same_lcccs(out, N.fold_verify(ccs, acc, cmi, x, proof, pr))


def test_replay_consistent_with_prover_and_verifier():
    """the verifier-variable replay (generate_verification_witness_vars) on an honest
    proof: its challenges are the prover's (r, r_0, the folded LCCCS's rho-weighted
    sums), the sumcheck claims chain (claimed sum i+1 = the interpolation at the
    round's challenge, the sum of its terms), the linearization's final claim is
    eq(r, beta) * inner and the folding's equals should_equal_s"""
    pr, ccs, A, kappa, acc, Wa, cmi, xi, Wi = instance(24, W=5, t=4, deg=2)
    out, w0, proof = N.fold_prove(ccs, A, kappa, acc, Wa, cmi, xi, Wi, pr)
    v = N.fold_replay(ccs, acc, cmi, xi, proof, pr)
    assert all(np.array_equal(a, b) for a, b in zip(v["fold_point"], out.r))
    assert np.array_equal(v["fold_expected"], v["should_equal_s"])
    e, _ = N.zk_eq(v["lin_point"], v["lin_beta"], 24)
    assert np.array_equal(N.mul(e, v["lin_inner"], 24), v["lin_expected"])
    assert np.array_equal(v["claim_g1"], N.add(v["claim_g1"], N.zero(24)))
    # cm_0 = sum of the final cm products
    kd = kappa
    cm0 = [N.zero(24) for _ in range(kd)]
    for i in range(2 * pr.K):
        for j in range(kd):
            cm0[j] = N.add(cm0[j], v["final_cm"][i * kd + j])
    assert np.array_equal(np.concatenate(cm0), out.cm)
    # each round's terms sum to the next claimed sum
    deg = 2 * pr.b_small + 1
    for i in range(ccs.s):
        tot = N.zero(24)
        for t_ in v["fold_subterms"][i * deg:(i + 1) * deg]:
            tot = N.add(tot, t_)
        assert np.array_equal(tot, v["fold_claimed_sums"][i + 1])
