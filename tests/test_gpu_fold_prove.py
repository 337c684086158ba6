"""lf_fold_prove (the zkvm's fold(), zk_latticefold_prove, ZK/zk_latticefold.rs:37-102)
against the oracle's restatement (oracle/nifs.py): the folded LCCCS, the folded
witness and every LFProof message bit-exact, and the restated NIFS verifier
accepts the device's proof. Small satisfied CCS instances (the oracle is
Python glue over its C primitives)."""
import numpy as np
import pytest

import latticeum_amd as LA
import nifs as N
import oracle as O

LF_ERR_INVALID_ARG = 1  # lf.h

pytestmark = pytest.mark.gpu


def dev(x):
    import torch
    return torch.from_numpy(np.ascontiguousarray(x, np.uint64).view(np.int64).copy()).cuda()


def zeros(n):
    import torch
    return torch.zeros(n, dtype=torch.int64, device="cuda")


def host(t):
    return t.cpu().numpy().view(np.uint64)


def flat(xs):
    return np.concatenate([np.asarray(x, np.uint64).ravel() for x in xs]) if len(xs) else np.zeros(0, np.uint64)


def setup(ctx, d, W, l, t, deg, kappa, seed, empty=0.0, scalar=False):
    pr_o = N.Params(d)
    ccs = N.satisfied_ccs(d, W, l, t, deg, seed, pr_o, empty=empty, scalar=scalar)
    Nn = W * pr_o.L
    A = O.fill_uniform(kappa * Nn * d, seed + 6)
    sch = LA.AjtaiCommitmentScheme(ctx, A.reshape(kappa, Nn, d))
    M = LA.CCSMatrices(ctx, d, ccs.m, ccs.n, ccs.mats)
    prover = LA.Prover(ctx, sch, LA.goldilocks_dp(d), M, l, deg, np.concatenate(ccs.c), ccs.S)
    return pr_o, ccs, A, prover


def witness(ccs, pr_o, seed):
    x, w = N.satisfying_z(ccs, ccs.n - ccs.l - 1, seed)
    fc, f = O.witness_from_w_ccs(w, ccs.d, pr_o.B, pr_o.L)
    return x, N.Witness(w_ccs=w, f=f, f_coeff=fc)


def acc_dict(L):
    return {"r": flat(L.r), "v": flat(L.v), "cm": np.asarray(L.cm, np.uint64), "u": flat(L.u), "x_w": flat(L.x_w),
            "h": np.asarray(L.h, np.uint64)}


def dev_wit(w):
    return {"w_ccs": dev(w.w_ccs), "f": dev(w.f), "f_coeff": dev(w.f_coeff)}


def proof_from_device(pf, d, K, tau, t, l, kappa):
    el = lambda a: N.elems(a, d)
    dec = []
    for side in range(2):
        dec.append({"u_s": [el(x) for x in pf["u_s"][side].reshape(K, t * d)],
                    "v_s": [el(x) for x in pf["v_s"][side].reshape(K, tau * d)],
                    "x_s": [el(x) for x in pf["x_s"][side].reshape(K, (l + 1) * d)],
                    "y_s": [el(x) for x in pf["y_s"][side].reshape(K, kappa * d)]})
    return N.Proof(lin_sumcheck=pf["lin_sumcheck"], lin_v=el(pf["lin_v"]), lin_u=el(pf["lin_u"]), dec=dec,
                   fold_sumcheck=pf["fold_sumcheck"], theta_s=[el(x) for x in pf["theta_s"].reshape(2 * K, tau * d)],
                   eta_s=[el(x) for x in pf["eta_s"].reshape(2 * K, t * d)])


def check_replay(prover, acc, cm_i, x_ccs, pf, out, kappa):
    """lf_fold_replay on the device prover's proof: the verifier's replayed
    transcript meets the prover's (r_0, the claims chain, cm_0 / u_0 / x_0 as the
    rho-weighted sums of the decomposed instances)"""
    d, K, t, l = 24, prover.pr.K, prover.t, prover.l
    v = prover.replay(acc, cm_i, x_ccs, pf)
    assert np.array_equal(v["fold_point"], out["r"]), "r_0"
    assert np.array_equal(v["fold_expected"], v["should_equal_s"]), "folding claim"
    e, _ = N.zk_eq(N.elems(v["lin_point"], d), N.elems(v["lin_beta"], d), d)
    assert np.array_equal(N.mul(e, v["lin_inner"], d), v["lin_expected"]), "linearization claim"

    def rho_sum(a, n):
        rows = a.reshape(2 * K, n, d)
        tot = [N.zero(d) for _ in range(n)]
        for i in range(2 * K):
            for j in range(n):
                tot[j] = N.add(tot[j], rows[i, j])
        return flat(tot)

    assert np.array_equal(rho_sum(v["final_cm"], kappa), out["cm"]), "cm_0"
    assert np.array_equal(rho_sum(v["final_u"], t), out["u"]), "u_0"
    x0 = rho_sum(v["final_x"], l + 1)
    assert np.array_equal(x0[:l * d], out["x_w"]) and np.array_equal(x0[l * d:], out["h"]), "x_0"
    return v


def check_against_oracle(out, pf, w_out, o_out, o_w0, o_proof):
    assert np.array_equal(out["r"], flat(o_out.r)), "r_0"
    assert np.array_equal(out["v"], flat(o_out.v)), "v_0"
    assert np.array_equal(out["cm"], o_out.cm), "cm_0"
    assert np.array_equal(out["u"], flat(o_out.u)), "u_0"
    assert np.array_equal(out["x_w"], flat(o_out.x_w)), "x_w"
    assert np.array_equal(out["h"], o_out.h), "h"
    assert np.array_equal(pf["lin_sumcheck"], o_proof.lin_sumcheck), "linearization sumcheck"
    assert np.array_equal(pf["lin_v"], flat(o_proof.lin_v)) and np.array_equal(pf["lin_u"], flat(o_proof.lin_u))
    for side in range(2):
        for k in ("u_s", "v_s", "x_s", "y_s"):
            want = flat([flat(x) for x in o_proof.dec[side][k]])
            assert np.array_equal(pf[k][side], want), f"{k} side {side}"
    assert np.array_equal(pf["fold_sumcheck"], o_proof.fold_sumcheck), "folding sumcheck"
    assert np.array_equal(pf["theta_s"], flat([flat(x) for x in o_proof.theta_s])), "theta_s"
    assert np.array_equal(pf["eta_s"], flat([flat(x) for x in o_proof.eta_s])), "eta_s"
    for k, want in (("f", o_w0.f), ("f_coeff", o_w0.f_coeff), ("w_ccs", o_w0.w_ccs)):
        assert np.array_equal(host(w_out[k]), want), f"folded witness {k}"


@pytest.mark.parametrize("d,W,l,t,deg,kappa", [(24, 5, 2, 4, 2, 3), (24, 13, 4, 6, 3, 4), (1024, 5, 2, 4, 2, 2),
                                               (16, 7, 1, 5, 3, 3)])
def test_fold_prove_matches_oracle(d, W, l, t, deg, kappa):
    ctx = LA.Context(0)
    try:
        pr_o, ccs, A, prover = setup(ctx, d, W, l, t, deg, kappa, 7 + d + W)
        xa, Wa = witness(ccs, pr_o, 11)
        xi, Wi = witness(ccs, pr_o, 12)
        Nn = W * pr_o.L
        cma = O.ajtai_commit(A, kappa, Nn, d, Wa.f)
        cmi = O.ajtai_commit(A, kappa, Nn, d, Wi.f)
        acc = N.linearize_fresh(ccs, cma, xa, Wa, pr_o)
        o_out, o_w0, o_proof = N.fold_prove(ccs, A, kappa, acc, Wa, cmi, xi, Wi, pr_o)
        w_out = {"w_ccs": zeros(W * d), "f": zeros(Nn * d), "f_coeff": zeros(Nn * d)}
        out, pf = prover.fold_prove(acc_dict(acc), dev_wit(Wa), cmi, flat(xi), dev_wit(Wi), w_out)
        check_against_oracle(out, pf, w_out, o_out, o_w0, o_proof)
        # the restated verifier accepts the device's proof and re-derives its LCCCS
        K, tau = pr_o.K, N.tb(d) if d == 24 else 1
        v = N.fold_verify(ccs, acc, cmi, xi, proof_from_device(pf, d, K, tau, ccs.t, l, kappa), pr_o)
        assert np.array_equal(flat(v.r), out["r"]) and np.array_equal(v.cm, out["cm"])
        if d == 24:
            v = check_replay(prover, acc_dict(acc), cmi, flat(xi), pf, out, kappa)
            # lf_fold_prove_vars: the same fold() with the vars from its own sample log
            w_v = {"w_ccs": zeros(W * d), "f": zeros(Nn * d), "f_coeff": zeros(Nn * d)}
            out_v, pf_v, vv = prover.fold_prove(acc_dict(acc), dev_wit(Wa), cmi, flat(xi), dev_wit(Wi), w_v, vars=True)
            check_against_oracle(out_v, pf_v, w_v, o_out, o_w0, o_proof)
            for k in v:
                assert np.array_equal(vv[k], v[k]), k
        # fold again: the device's folded accumulator with a third instance
        x3, W3 = witness(ccs, pr_o, 13)
        cm3 = O.ajtai_commit(A, kappa, Nn, d, W3.f)
        acc2 = N.LCCCS(r=N.elems(out["r"], d), v=N.elems(out["v"], d), cm=out["cm"], u=N.elems(out["u"], d),
                       x_w=N.elems(out["x_w"], d), h=out["h"])
        wacc2 = N.Witness(w_ccs=host(w_out["w_ccs"]), f=host(w_out["f"]), f_coeff=host(w_out["f_coeff"]))
        o_out2, o_w2, o_proof2 = N.fold_prove(ccs, A, kappa, acc2, wacc2, cm3, x3, W3, pr_o)
        w_out2 = {"w_ccs": zeros(W * d), "f": zeros(Nn * d), "f_coeff": zeros(Nn * d)}
        out2, pf2 = prover.fold_prove(acc_dict(acc2), w_out, cm3, flat(x3), dev_wit(W3), w_out2)
        check_against_oracle(out2, pf2, w_out2, o_out2, o_w2, o_proof2)
    finally:
        ctx.close()


@pytest.mark.parametrize("scalar", [False, True])
@pytest.mark.parametrize("d,W,l,t,deg,kappa", [(24, 13, 4, 6, 3, 4), (1024, 9, 2, 4, 2, 2)])
def test_fold_prove_empty_rows_matches_oracle(d, W, l, t, deg, kappa, scalar):
    """A_j rows without entries (some lines of every multiset's factors vanish, so the
    linearization's round 0 skips points: lf_sumcheck_prove_lin_sparse), and with
    scalar-valued matrices as the zkvm's (lf_ccs_is_scalar): the oracle's fold(), bit
    for bit"""
    ctx = LA.Context(0)
    try:
        pr_o, ccs, A, prover = setup(ctx, d, W, l, t, deg, kappa, 31 + d + W, empty=0.5, scalar=scalar)
        M = LA.CCSMatrices(ctx, d, ccs.m, ccs.n, ccs.mats)
        assert M.scalar == scalar
        active = np.ones(ccs.m // 2, bool)
        for j in range(deg):
            live = M.row_live(j, ccs.m)
            assert np.array_equal(live, np.diff(ccs.mats[j][0].astype(np.int64)) > 0)
            active &= live.reshape(-1, 2).any(1)
        assert not active.all(), "the case must skip some points"
        del M
        xa, Wa = witness(ccs, pr_o, 21)
        xi, Wi = witness(ccs, pr_o, 22)
        Nn = W * pr_o.L
        cma = O.ajtai_commit(A, kappa, Nn, d, Wa.f)
        cmi = O.ajtai_commit(A, kappa, Nn, d, Wi.f)
        acc = N.linearize_fresh(ccs, cma, xa, Wa, pr_o)
        o_out, o_w0, o_proof = N.fold_prove(ccs, A, kappa, acc, Wa, cmi, xi, Wi, pr_o)
        w_out = {"w_ccs": zeros(W * d), "f": zeros(Nn * d), "f_coeff": zeros(Nn * d)}
        out, pf = prover.fold_prove(acc_dict(acc), dev_wit(Wa), cmi, flat(xi), dev_wit(Wi), w_out)
        check_against_oracle(out, pf, w_out, o_out, o_w0, o_proof)
    finally:
        ctx.close()


def test_fold_prove_montgomery_boundary():
    """repr = LF_REPR_MONTGOMERY: ark-ff limbs in, ark-ff limbs out (zero-copy from Rust)"""
    d, W, l, t, deg, kappa = 24, 5, 2, 4, 2, 3
    ctx = LA.Context(0)
    try:
        pr_o, ccs, A, prover = setup(ctx, d, W, l, t, deg, kappa, 31)
        xa, Wa = witness(ccs, pr_o, 11)
        xi, Wi = witness(ccs, pr_o, 12)
        Nn = W * pr_o.L
        cma, cmi = O.ajtai_commit(A, kappa, Nn, d, Wa.f), O.ajtai_commit(A, kappa, Nn, d, Wi.f)
        acc = N.linearize_fresh(ccs, cma, xa, Wa, pr_o)
        mont = np.vectorize(O.to_mont, otypes=[np.uint64])
        unmont = np.vectorize(O.from_mont, otypes=[np.uint64])
        w1 = {"w_ccs": zeros(W * d), "f": zeros(Nn * d), "f_coeff": zeros(Nn * d)}
        out_c, pf_c, vc = prover.fold_prove(acc_dict(acc), dev_wit(Wa), cmi, flat(xi), dev_wit(Wi), w1, vars=True)
        accm = {k: mont(v) for k, v in acc_dict(acc).items()}
        w2 = {"w_ccs": zeros(W * d), "f": zeros(Nn * d), "f_coeff": zeros(Nn * d)}
        out_m, pf_m, vm = prover.fold_prove(accm, dev_wit(Wa), mont(cmi), mont(flat(xi)), dev_wit(Wi), w2,
                                            repr=LA.REPR_MONTGOMERY, vars=True)
        for k in vc:
            assert np.array_equal(unmont(vm[k]), vc[k]), k
        for k in out_c:
            assert np.array_equal(unmont(out_m[k]), out_c[k]) if out_c[k].size else True, k
        assert np.array_equal(unmont(pf_m["fold_sumcheck"]), pf_c["fold_sumcheck"])
        assert np.array_equal(unmont(pf_m["y_s"][1]), pf_c["y_s"][1])
    finally:
        ctx.close()


def test_prover_rejects_multiset_over_eq_beta():
    """S_idx names list positions of the linearization's MLE list; the position
    just past the Mz MLEs is eq(beta) itself (linearization/utils.rs:71-84). The
    split-eq sumcheck cannot put a second eq factor into one term, so
    lf_prover_create rejects such a CCS by name (LF_ERR_UNSUPPORTED_CCS)
    instead of failing inside fold()"""
    d, W, l, t, deg, kappa = 24, 5, 2, 6, 2, 3
    pr_o = N.Params(d)
    ccs = N.satisfied_ccs(d, W, l, t, deg, 77, pr_o)
    Nn = W * pr_o.L
    ctx = LA.Context(0)
    try:
        sch = LA.AjtaiCommitmentScheme(ctx, O.fill_uniform(kappa * Nn * d, 78).reshape(kappa, Nn, d))
        M = LA.CCSMatrices(ctx, d, ccs.m, ccs.n, ccs.mats)
        c = O.fill_uniform(2 * d, 79)
        # lin_list = [0, 3, 1]: position 3 == len(lin_list) is the eq(beta) slot
        with pytest.raises(LA.LfError) as e:
            LA.Prover(ctx, sch, LA.goldilocks_dp(d), M, l, deg, c, [[0, 3], [1]])
        assert e.value.code == 13 and "eq(beta)" in str(e.value)
        # position 5 is past the eq(beta) slot: malformed (the reference panics on the index), not unsupported
        for bad in ([[0, 5], [1]], [[0, 4], [1]]):
            with pytest.raises(LA.LfError) as e:
                LA.Prover(ctx, sch, LA.goldilocks_dp(d), M, l, deg, c, bad)
            assert e.value.code == LF_ERR_INVALID_ARG and "negative or past" in str(e.value)
        with pytest.raises(LA.LfError) as e:  # negative: refused with the CCS structure already
            LA.Prover(ctx, sch, LA.goldilocks_dp(d), M, l, deg, c, [[0, -1], [1]])
        assert e.value.code == LF_ERR_INVALID_ARG
        LA.Prover(ctx, sch, LA.goldilocks_dp(d), M, l, deg, c, [[0, 2], [1]])  # every position a Mz MLE
    finally:
        ctx.close()


def test_linearize_matches_oracle():
    """lf_linearize (initialize_accumulator's LFLinearizationProver::prove) against the oracle"""
    d, W, l, t, deg, kappa = 24, 13, 4, 6, 3, 4
    ctx = LA.Context(0)
    try:
        pr_o, ccs, A, prover = setup(ctx, d, W, l, t, deg, kappa, 41)
        x, Wt = witness(ccs, pr_o, 42)
        cm = O.ajtai_commit(A, kappa, W * pr_o.L, d, Wt.f)
        out, sc = prover.linearize(cm, flat(x), dev_wit(Wt))
        tr = N.Transcript(d)
        o, (oproof, _, _) = N.linearize(tr, ccs, cm, x, Wt, pr_o)
        assert np.array_equal(sc, oproof)
        for k in ("r", "v", "u", "x_w"):
            assert np.array_equal(out[k], flat(getattr(o, k))), k
        assert np.array_equal(out["cm"], cm) and np.array_equal(out["h"], N.one(d))
    finally:
        ctx.close()


def test_fold_prove_zkvm_dimensions():
    """the zkvm's shape (ZK/ccs.rs:26-67): Phi_72, W = 19 763 (n = 19 768, l = 4),
    m = 2^17, t = 125 matrices, a degree-7 multiset (the Poseidon2 S-box's),
    kappa = 32, GoldiLocksDP. The accumulator comes from lf_linearize; the
    restated NIFS verifier accepts the device's proof and re-derives its LCCCS,
    and that LCCCS is the folded witness's (cm_0 = A f_0, v_0, u_0)."""
    import torch
    d, W, l, t, deg, kappa = 24, 19763, 4, 125, 7, 32
    pr_o = N.Params(d)
    ccs = N.satisfied_ccs_np(d, W, l, t, deg, 0x4C46, pr_o, extra_density=1 / 16)
    assert ccs.m == 1 << 17 and ccs.n == 19768
    ctx = LA.Context(0)
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    try:
        pr = LA.goldilocks_dp(d)
        Nn = W * pr.L
        A = torch.empty(kappa * Nn * d, dtype=torch.int64, device="cuda")
        ctx.dev_fill_uniform(A, 0x4C460004)
        sch = LA.AjtaiCommitmentScheme(ctx, device_tensor=A, kappa=kappa, ncols=Nn, d=d)
        M = LA.CCSMatrices(ctx, d, ccs.m, ccs.n, ccs.mats)
        prover = LA.Prover(ctx, sch, pr, M, l, deg, np.concatenate(ccs.c), ccs.S)

        def dwit(seed):
            x, w = N.satisfying_z(ccs, W, seed)
            wd = {"w_ccs": dev(w), "f": zeros(Nn * d), "f_coeff": zeros(Nn * d)}
            ctx.check(ctx.lib.lf_dev_witness_from_w_ccs(ctx.h, LA._lib.C.byref(pr), wd["w_ccs"].data_ptr(), W,
                                                        wd["f_coeff"].data_ptr(), wd["f"].data_ptr()))
            cm = zeros(kappa * d)
            ctx.dev_ajtai_commit(sch, [wd["f"]], cm)
            ctx.sync()
            return flat(x), wd, host(cm)

        xa, wa, cma = dwit(101)
        xi, wi, cmi = dwit(102)
        acc, _ = prover.linearize(cma, xa, wa)
        w_out = {"w_ccs": zeros(W * d), "f": zeros(Nn * d), "f_coeff": zeros(Nn * d)}
        out, pf, vv = prover.fold_prove(acc, wa, cmi, xi, wi, w_out, vars=True)
        el = lambda a: N.elems(a, d)
        acc_o = N.LCCCS(r=el(acc["r"]), v=el(acc["v"]), cm=acc["cm"], u=el(acc["u"]), x_w=el(acc["x_w"]), h=acc["h"])
        v = N.fold_verify(ccs, acc_o, cmi, el(xi), proof_from_device(pf, d, pr.K, 3, t, l, kappa), pr_o)
        for k in ("r", "v", "u", "x_w"):
            assert np.array_equal(flat(getattr(v, k)), out[k]), k
        assert np.array_equal(v.cm, out["cm"]) and np.array_equal(v.h, out["h"])
        v = check_replay(prover, acc, cmi, xi, pf, out, kappa)
        for k in v:  # the vars from the prover's sample log = the full replay's
            assert np.array_equal(vv[k], v[k]), k
        # the IVC step commitments of the folded accumulator (main.rs:195-196): acc_comm
        # over its 182 ring elements (364 permutations), both reprs, and ivc_step_comm
        assert [out[k].size // d for k in ("r", "v", "cm", "u", "x_w", "h")] == [17, 3, 32, 125, 4, 1]
        ac = LA.acc_comm(out)
        assert np.array_equal(ac, O.acc_comm(out))
        mont = np.vectorize(O.to_mont, otypes=[np.uint64])
        assert np.array_equal(LA.acc_comm({k: mont(x) for k, x in out.items()}, repr=LA.REPR_MONTGOMERY), ac)
        z0c = O.fill_uniform(4, 9)
        dg, st = LA.ivc_step_comm(1, z0c, O.fill_uniform(4, 10), ac)
        odg, ost = O.ivc_step_comm(1, z0c, O.fill_uniform(4, 10), ac)
        assert np.array_equal(dg, odg) and np.array_equal(st, ost)
        # the folded instance is the folded witness's
        cm0 = zeros(kappa * d)
        ctx.dev_ajtai_commit(sch, [w_out["f"]], cm0)
        r0 = dev(out["r"])
        v0 = zeros(3 * d)
        ctx.check(ctx.lib.lf_dev_fhat_evaluate(ctx.h, d, w_out["f_coeff"].data_ptr(), Nn, 0, 1, 17, r0.data_ptr(),
                                               v0.data_ptr()))
        z0 = torch.cat([dev(out["x_w"]), dev(out["h"]), w_out["w_ccs"]])
        u0 = zeros(t * d)
        M.mz_evaluate(z0, 1, 17, r0, u0)
        ctx.sync()
        assert np.array_equal(host(cm0), out["cm"]) and np.array_equal(host(v0), out["v"])
        assert np.array_equal(host(u0), out["u"])
        check_wire(pf, out, d, pr.K, t, l, kappa)
    finally:
        ctx.close()


def ark_vec(elems, d):
    """ark-serialize 0.5 of Vec<RingElem>: u64 LE length, then d canonical u64 LE per element"""
    import struct
    e = np.asarray(elems, np.uint64).ravel()
    return struct.pack("<Q", e.size // d) + e.astype("<u8").tobytes()


def ark_vecvec(rows, d):
    import struct
    return struct.pack("<Q", len(rows)) + b"".join(ark_vec(r, d) for r in rows)


def check_wire(pf, out, d, K, t, l, kappa):
    """SURVEY 8(f) rank 4 on the device path: the LFProof lf_fold_prove produced at the
    zkvm's shape through lf_lfproof_serialize (CanonicalSerialize, latticefold/src/nifs.rs:28-34),
    its size by the ark layout formula (the size zkvm/src/main.rs:231-234 reports), the bytes
    against a plain ark restatement, and the folded LCCCS round-tripping in both reprs"""
    from latticeum_amd import wire
    tau, rounds = 3, 17
    lin_evals = pf["lin_sumcheck"].size // (rounds * d)
    fold_evals = pf["fold_sumcheck"].size // (rounds * d)
    assert lin_evals == 9 and fold_evals == 5  # degree 7 + 2 (linearization), the folding's degree 4 + 1
    dec = [{k: list(pf[k][s].reshape(K, -1)) for k in ("u_s", "v_s", "x_s", "y_s")} for s in range(2)]
    th = list(pf["theta_s"].reshape(2 * K, tau * d))
    et = list(pf["eta_s"].reshape(2 * K, t * d))
    b = wire.serialize_lfproof(d, pf["lin_sumcheck"], rounds, lin_evals, pf["lin_v"], pf["lin_u"], dec,
                               pf["fold_sumcheck"], rounds, fold_evals, th, et)
    elems = (rounds * lin_evals + tau + t + 2 * K * (t + tau + (l + 1) + kappa) + rounds * fold_evals
             + 2 * K * tau + 2 * K * t)
    lens = (1 + rounds) + 2 + 2 * (4 + 4 * K) + (1 + rounds) + 2 * (1 + 2 * K)
    assert len(b) == elems * d * 8 + lens * 8, len(b)
    ls = pf["lin_sumcheck"].reshape(rounds, lin_evals * d)
    fs = pf["fold_sumcheck"].reshape(rounds, fold_evals * d)
    want = ark_vecvec(list(ls), d) + ark_vec(pf["lin_v"], d) + ark_vec(pf["lin_u"], d)
    for s in range(2):
        want += b"".join(ark_vecvec(dec[s][k], d) for k in ("u_s", "v_s", "x_s", "y_s"))
    want += ark_vecvec(list(fs), d) + ark_vecvec(th, d) + ark_vecvec(et, d)
    assert b == want
    # the folded accumulator: serialise, deserialise, in canonical and Montgomery form
    lc = wire.serialize_lcccs(d, out["r"], out["v"], out["cm"], out["u"], out["x_w"], out["h"])
    back = wire.deserialize_lcccs(lc, d)
    for k in ("r", "v", "cm", "u", "x_w", "h"):
        assert np.array_equal(back[k], out[k]), k
    mont = np.vectorize(O.to_mont, otypes=[np.uint64])
    om = {k: mont(out[k]) for k in ("r", "v", "cm", "u", "x_w", "h")}
    assert wire.serialize_lcccs(d, om["r"], om["v"], om["cm"], om["u"], om["x_w"], om["h"],
                                repr=wire.REPR_MONTGOMERY) == lc
    backm = wire.deserialize_lcccs(lc, d, repr=wire.REPR_MONTGOMERY)
    for k in om:
        assert np.array_equal(backm[k], om[k]), k
