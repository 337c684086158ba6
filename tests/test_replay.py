"""lf_fold_replay (generate_verification_witness_vars, ZK/zk_latticefold.rs:111-148):
the host replay of a fold() proof against the oracle's restatement
(oracle/nifs.py fold_replay), every verifier variable bit-exact, in both
boundary representations; malformed shapes are rejected. Host code only: runs
without a GPU (the C ABI library is loaded, no device call is made)."""
import numpy as np
import pytest

import latticeum_amd as LA
import nifs as N
import oracle as O


def flat(xs):
    return np.concatenate([np.asarray(x, np.uint64).ravel() for x in xs]) if len(xs) else np.zeros(0, np.uint64)


def proof_dict(p):
    """oracle Proof -> the flat buffers lf_fold_prove writes (lf_lfproof_mut)"""
    out = {"lin_sumcheck": np.asarray(p.lin_sumcheck, np.uint64).ravel(), "lin_v": flat(p.lin_v),
           "lin_u": flat(p.lin_u), "fold_sumcheck": np.asarray(p.fold_sumcheck, np.uint64).ravel(),
           "theta_s": flat([flat(x) for x in p.theta_s]), "eta_s": flat([flat(x) for x in p.eta_s])}
    for k in ("u_s", "v_s", "x_s", "y_s"):
        out[k] = [flat([flat(x) for x in p.dec[side][k]]) for side in range(2)]
    return out


def acc_dict(L):
    return {"r": flat(L.r), "v": flat(L.v), "cm": np.asarray(L.cm, np.uint64), "u": flat(L.u), "x_w": flat(L.x_w),
            "h": np.asarray(L.h, np.uint64)}


def case(W=5, l=2, t=4, deg=2, kappa=3, seed=7):
    d = 24
    pr = N.Params(d)
    ccs = N.satisfied_ccs(d, W, l, t, deg, seed, pr)
    xa, wa = N.satisfying_z(ccs, W, seed + 4)
    xi, wi = N.satisfying_z(ccs, W, seed + 5)
    Nn = W * pr.L
    A = O.fill_uniform(kappa * Nn * d, seed + 6)

    def wit(w):
        fc, f = O.witness_from_w_ccs(w, d, pr.B, pr.L)
        return N.Witness(w_ccs=w, f=f, f_coeff=fc)

    Wa, Wi = wit(wa), wit(wi)
    cma, cmi = O.ajtai_commit(A, kappa, Nn, d, Wa.f), O.ajtai_commit(A, kappa, Nn, d, Wi.f)
    acc = N.linearize_fresh(ccs, cma, xa, Wa, pr)
    out, _, proof = N.fold_prove(ccs, A, kappa, acc, Wa, cmi, xi, Wi, pr)
    return pr, ccs, kappa, acc, cmi, xi, proof, out


def replay(ccs, kappa, acc, cmi, xi, proof, repr=LA.REPR_CANONICAL, conv=lambda a: a, samples=None):
    return LA.fold_replay(LA.goldilocks_dp(24), ccs.t, ccs.m, ccs.l, ccs.degree, conv(flat(ccs.c)), ccs.S, kappa,
                          {k: conv(v) for k, v in acc_dict(acc).items()}, conv(np.asarray(cmi, np.uint64)),
                          conv(flat(xi)), {k: ([conv(x) for x in v] if isinstance(v, list) else conv(v))
                                           for k, v in proof_dict(proof).items()}, repr, samples=samples)


@pytest.mark.parametrize("W,l,t,deg,kappa", [(5, 2, 4, 2, 3), (13, 4, 6, 3, 4)])
def test_replay_from_sample_log(W, l, t, deg, kappa):
    """lf_fold_replay_samples: the replay's challenges from a sample log (what
    lf_fold_prove records) instead of a second sponge -- every variable equal to
    the full replay's; a short or long log is rejected"""
    pr, ccs, kappa, acc, cmi, xi, proof, _ = case(W, l, t, deg, kappa, seed=W + t)
    log = []
    N.fold_replay(ccs, acc, cmi, xi, proof, pr, log=log)
    full = replay(ccs, kappa, acc, cmi, xi, proof)
    got = replay(ccs, kappa, acc, cmi, xi, proof, samples=log)
    for k in full:
        assert np.array_equal(got[k], full[k]), k
    mont = np.vectorize(O.to_mont, otypes=[np.uint64])
    unmont = np.vectorize(O.from_mont, otypes=[np.uint64])
    gm = replay(ccs, kappa, acc, cmi, xi, proof, LA.REPR_MONTGOMERY, mont, samples=log)
    for k in full:
        assert np.array_equal(unmont(gm[k]), full[k]), k
    for bad in (log[:-1], log + [5]):
        with pytest.raises(LA.LfError):
            replay(ccs, kappa, acc, cmi, xi, proof, samples=bad)


def test_transcript_record_and_playback():
    """a recording transcript's samples, played back to a transcript that observes
    the same values (dropped) and samples in the same pattern, come out in order"""
    lib = LA.load()
    rng = np.random.default_rng(3)
    t = lib.lf_transcript_new()
    lib.lf_transcript_record(t)
    ops, drawn = [], []
    for _ in range(300):
        if rng.integers(0, 3):
            v = int(rng.integers(0, 1 << 63, dtype=np.uint64))
            lib.lf_transcript_observe(t, v)
            ops.append(("o", v))
        else:
            drawn.append(lib.lf_transcript_sample(t))
            ops.append(("s", None))
    n = lib.lf_transcript_samples(t, None, 0)
    log = np.zeros(n, np.uint64)
    lib.lf_transcript_samples(t, log.ctypes.data, n)
    lib.lf_transcript_free(t)
    assert [int(x) for x in log] == drawn
    pb = lib.lf_transcript_new_playback(log.ctypes.data, n)
    again = [lib.lf_transcript_sample(pb) if op == "s" else lib.lf_transcript_observe(pb, v) for op, v in ops]
    assert [x for (op, _), x in zip(ops, again) if op == "s"] == drawn
    assert lib.lf_transcript_playback_status(pb) == 0
    lib.lf_transcript_sample(pb)  # one past the log
    assert lib.lf_transcript_playback_status(pb) != 0
    lib.lf_transcript_free(pb)


@pytest.mark.parametrize("W,l,t,deg,kappa", [(5, 2, 4, 2, 3), (13, 4, 6, 3, 4), (7, 0, 3, 2, 2)])
def test_replay_matches_oracle(W, l, t, deg, kappa):
    pr, ccs, kappa, acc, cmi, xi, proof, out = case(W, l, t, deg, kappa, seed=W + t)
    got = replay(ccs, kappa, acc, cmi, xi, proof)
    want = N.fold_replay(ccs, acc, cmi, xi, proof, pr)
    for k, v in want.items():
        w = flat(v) if isinstance(v, list) else np.asarray(v, np.uint64)
        assert np.array_equal(got[k], w), k
    # the replayed challenges are the prover's
    assert np.array_equal(got["fold_point"], flat(out.r))
    assert np.array_equal(got["fold_expected"], got["should_equal_s"])


def test_replay_montgomery_boundary():
    pr, ccs, kappa, acc, cmi, xi, proof, _ = case()
    mont = np.vectorize(O.to_mont, otypes=[np.uint64])
    unmont = np.vectorize(O.from_mont, otypes=[np.uint64])
    a = replay(ccs, kappa, acc, cmi, xi, proof)
    b = replay(ccs, kappa, acc, cmi, xi, proof, LA.REPR_MONTGOMERY, mont)
    for k in a:
        assert np.array_equal(unmont(b[k]), a[k]), k


def test_replay_rejects_bad_shapes():
    pr, ccs, kappa, acc, cmi, xi, proof, _ = case()
    p = LA.goldilocks_dp(24)
    S_bad = [list(x) for x in ccs.S]
    S_bad[0][0] = ccs.t  # a multiset index past the matrices
    with pytest.raises(LA.LfError):
        LA.fold_replay(p, ccs.t, ccs.m, ccs.l, ccs.degree, flat(ccs.c), S_bad, kappa, acc_dict(acc), cmi, flat(xi),
                       proof_dict(proof))
    with pytest.raises(LA.LfError):  # m not a power of two
        LA.fold_replay(p, ccs.t, ccs.m + 1, ccs.l, ccs.degree, flat(ccs.c), ccs.S, kappa, acc_dict(acc), cmi,
                       flat(xi), proof_dict(proof))
    with pytest.raises(LA.LfError):  # the X^d + 1 rings: the replay is the Phi_72 verifier's
        LA.fold_replay(LA.goldilocks_dp(1024), ccs.t, ccs.m, ccs.l, ccs.degree, flat(ccs.c), ccs.S, kappa,
                       acc_dict(acc), cmi, flat(xi), proof_dict(proof))
