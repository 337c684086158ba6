"""lf_fold_verify: the product's host folding verifier (NIFSVerifier::verify,
latticefold/src/nifs.rs:117-162, as zkvm main.rs:408-426 runs it after every fold())
against the oracle's restated verifier (oracle/nifs.py fold_verify): it accepts
the honest proofs and re-derives the same folded LCCCS (both representations),
and rejects the tampered proofs and the unsatisfied CCS the oracle rejects, at
the same check. Host code only (no device call)."""
import numpy as np
import pytest

import latticeum_amd as LA
import nifs as N
import oracle as O
from test_nifs_oracle import instance
from test_replay import acc_dict, flat, proof_dict


def verify(ccs, kappa, acc, cmi, xi, proof, repr=LA.REPR_CANONICAL, conv=lambda a: a):
    return LA.fold_verify(LA.goldilocks_dp(24), ccs.t, ccs.m, ccs.l, ccs.degree, conv(flat(ccs.c)), ccs.S, kappa,
                          {k: conv(v) for k, v in acc_dict(acc).items()}, conv(np.asarray(cmi, np.uint64)),
                          conv(flat(xi)), {k: ([conv(x) for x in v] if isinstance(v, list) else conv(v))
                                           for k, v in proof_dict(proof).items()}, repr)


def lcccs_dict(L):
    return {"r": flat(L.r), "v": flat(L.v), "cm": np.asarray(L.cm, np.uint64), "u": flat(L.u), "x_w": flat(L.x_w),
            "h": np.asarray(L.h, np.uint64)}


@pytest.mark.parametrize("W,l,t,deg,kappa", [(5, 2, 4, 2, 3), (13, 4, 6, 3, 4), (7, 0, 3, 2, 2)])
def test_verify_accepts_and_folds_like_the_oracle(W, l, t, deg, kappa):
    pr, ccs, A, kappa, acc, Wa, cmi, xi, Wi = instance(24, W=W, l=l, t=t, deg=deg, kappa=kappa, seed=W + t)
    out, _, proof = N.fold_prove(ccs, A, kappa, acc, Wa, cmi, xi, Wi, pr)
    want = lcccs_dict(N.fold_verify(ccs, acc, cmi, xi, proof, pr))
    got = verify(ccs, kappa, acc, cmi, xi, proof)
    for k in want:
        assert np.array_equal(got[k], want[k]), k
    # and it is the prover's folded LCCCS
    for k, v in lcccs_dict(out).items():
        assert np.array_equal(got[k], v), k


def test_verify_montgomery_boundary():
    pr, ccs, A, kappa, acc, Wa, cmi, xi, Wi = instance(24)
    _, _, proof = N.fold_prove(ccs, A, kappa, acc, Wa, cmi, xi, Wi, pr)
    mont = np.vectorize(O.to_mont, otypes=[np.uint64])
    unmont = np.vectorize(O.from_mont, otypes=[np.uint64])
    a = verify(ccs, kappa, acc, cmi, xi, proof)
    b = verify(ccs, kappa, acc, cmi, xi, proof, LA.REPR_MONTGOMERY, mont)
    for k in a:
        assert np.array_equal(unmont(b[k]), a[k]), k


def tampered(proof, field, idx, side=None):
    """a copy of the oracle proof with one ring element of `field` bumped by ONE"""
    p = N.Proof(**{**proof.__dict__})
    if side is None:
        vals = [list(x) if isinstance(x, list) else x for x in getattr(proof, field)]
        i, j = idx
        if isinstance(vals[i], list):
            vals[i][j] = N.add(vals[i][j], N.one(24))
        else:
            vals[i] = N.add(vals[i], N.one(24))
        setattr(p, field, vals)
    else:
        p.dec = [dict(proof.dec[0]), dict(proof.dec[1])]
        rows = [list(x) for x in proof.dec[side][field]]
        i, j = idx
        rows[i][j] = N.add(rows[i][j], N.one(24))
        p.dec[side][field] = rows
    return p


@pytest.mark.parametrize("field,idx,side,check", [
    ("theta_s", (3, 1), None, "folding evaluation claim"),
    ("y_s", (2, 0), 0, "decomposition recompose y"),
    ("u_s", (4, 1), 1, "decomposition recompose u"),
    ("v_s", (0, 2), 1, "decomposition recompose v"),
    ("x_s", (1, 0), 0, "decomposition recompose x"),
    ("lin_u", (0, None), None, "linearization evaluation claim"),
])
def test_verify_rejects_tampering_like_the_oracle(field, idx, side, check):
    pr, ccs, A, kappa, acc, Wa, cmi, xi, Wi = instance(24)
    _, _, proof = N.fold_prove(ccs, A, kappa, acc, Wa, cmi, xi, Wi, pr)
    bad = tampered(proof, field, (idx[0], idx[1]) if idx[1] is not None else (idx[0], 0), side) \
        if idx[1] is not None else tampered_flat(proof, field, idx[0])
    with pytest.raises(ValueError, match=check.split()[-1] if "recompose" in check else check):
        N.fold_verify(ccs, acc, cmi, xi, bad, pr)
    with pytest.raises(LA.VerificationError) as e:
        verify(ccs, kappa, acc, cmi, xi, bad)
    assert LA.VERIFY_CHECKS[e.value.check] == check


def tampered_flat(proof, field, i):
    p = N.Proof(**{**proof.__dict__})
    vals = list(getattr(proof, field))
    vals[i] = N.add(vals[i], N.one(24))
    setattr(p, field, vals)
    return p


def test_verify_rejects_sumcheck_messages():
    """a round message whose p(0) + p(1) no longer meets the claim (both sumchecks)"""
    pr, ccs, A, kappa, acc, Wa, cmi, xi, Wi = instance(24)
    _, _, proof = N.fold_prove(ccs, A, kappa, acc, Wa, cmi, xi, Wi, pr)
    for field, check in (("lin_sumcheck", 1), ("fold_sumcheck", 7)):
        p = N.Proof(**{**proof.__dict__})
        sc = np.array(getattr(proof, field), np.uint64).copy()
        sc[0] = (int(sc[0]) + 1) % LA.P  # round 0, evaluation at 0, slot 0
        setattr(p, field, sc)
        with pytest.raises(ValueError):
            N.fold_verify(ccs, acc, cmi, xi, p, pr)
        with pytest.raises(LA.VerificationError) as e:
            verify(ccs, kappa, acc, cmi, xi, p)
        assert e.value.check == check


def test_verify_rejects_unsatisfied_ccs():
    pr, ccs, A, kappa, acc, Wa, cmi, xi, Wi = instance(24, satisfied=False)
    _, _, proof = N.fold_prove(ccs, A, kappa, acc, Wa, cmi, xi, Wi, pr)
    with pytest.raises(ValueError, match="linearization"):
        N.fold_verify(ccs, acc, cmi, xi, proof, pr)
    with pytest.raises(LA.VerificationError) as e:
        verify(ccs, kappa, acc, cmi, xi, proof)
    assert "linearization" in LA.VERIFY_CHECKS[e.value.check]
