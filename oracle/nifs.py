"""CPU restatement of the zkvm's fold() prover and of the NIFS verifier -- TEST
INFRASTRUCTURE ONLY (the checker of lf_fold_prove; nothing in the product
imports it).

The prover follows zk_latticefold_prove (ZK/zk_latticefold.rs:37-102) step by
step, with the same Poseidon2 transcript (the C oracle's DuplexChallenger,
oracle/lf_oracle.c) and the C oracle's ring, decomposition, Ajtai, MLE and
sumcheck primitives:

* absorb_public_input (ZK/zk_latticefold.rs:162-184);
* LFLinearizationProver::prove (LF/nifs/linearization.rs:153-197, utils.rs:63-124);
* LFDecompositionProver::prove, accumulator side then linearized side
  (LF/nifs/decomposition.rs:33-88, 162-256);
* LFFoldingProver::prove (LF/nifs/folding.rs:42-130, folding/utils.rs:51-127,
  196-255, 456-541).

The verifier restates NIFSVerifier::verify's three steps
(linearization.rs:200-285, decomposition.rs:90-155, folding.rs:133-392) and is
the relation that pins the prover (the reference has no fold() KAT): an honest
proof of a satisfied CCS is accepted and yields the prover's folded LCCCS.
Paths: LF = latticeum/crates/latticefold/src, ZK = latticeum/crates/zkvm/src.
Pure-Python glue over the C primitives: small CCS instances only.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

import oracle as O

P = O.P


# ---------------------------------------------------------------- ring helpers (NTT form, [n][d] u64)
def tb(d: int) -> int:
    """words of a base-ring element: Fq3 for Phi_72, Fq for X^d + 1"""
    return 3 if d == 24 else 1


def add(a, b):
    return ((np.asarray(a, np.uint64).astype(object) + np.asarray(b, np.uint64).astype(object)) % P).astype(np.uint64)


def sub(a, b):
    return ((np.asarray(a, np.uint64).astype(object) - np.asarray(b, np.uint64).astype(object)) % P).astype(np.uint64)


def mul(a, b, d: int):
    """slot-wise product of two equally long vectors of ring elements"""
    a, b = O._u64(a), O._u64(b)
    return np.concatenate([O.slot_mul(a[i:i + d], b[i:i + d], d) for i in range(0, a.size, d)]) if a.size else a


def smul(s, v, d: int):
    """one ring element s times every element of v"""
    v = O._u64(v)
    return mul(np.tile(O._u64(s), v.size // d), v, d)


def scal(base, d: int):
    """From<BaseRing> = from_scalar: the base-ring element in every NTT slot"""
    b = [int(x) % P for x in base]
    return np.array([b[i % tb(d)] for i in range(d)], np.uint64)


def one(d: int):
    return scal([1, 0, 0][:tb(d)], d)


def from_u(x: int, d: int):
    return scal([x % P, 0, 0][:tb(d)], d)


def zero(d: int):
    return np.zeros(d, np.uint64)


def is_zero(a) -> bool:
    return not np.any(O._u64(a))


def label(b: bytes) -> int:
    """BasePrimeField::from_be_bytes_mod_order"""
    return int.from_bytes(b, "big") % P


def pad_mle(x, nv: int, d: int):
    out = np.zeros((1 << nv) * d, np.uint64)
    x = O._u64(x)
    out[:x.size] = x
    return out


def evaluate(mles, nv: int, d: int, point):
    """evaluate_mles (LF/utils/mle_helpers.rs:65-95)"""
    return np.concatenate([O.mle_evaluate(m, nv, d, point) for m in mles]) if len(mles) else np.zeros(0, np.uint64)


def eq_eval(x, y, d: int):
    """LF/utils/sumcheck/utils.rs:78-92: prod (2 x_i y_i - x_i - y_i + 1)"""
    res = one(d)
    for xi, yi in zip(x, y):
        p = mul(xi, yi, d)
        res = mul(res, add(sub(sub(add(p, p), xi), yi), one(d)), d)
    return res


def powers_dot(base, vals, d: int):
    """sum_j base^(j+1) vals[j] (the successors(Some(a), a * ..) sums of folding/utils.rs)"""
    acc, pw = zero(d), base
    for v in vals:
        acc = add(acc, mul(pw, v, d))
        pw = mul(pw, base, d)
    return acc


# ---------------------------------------------------------------- transcript (ZK/fiat_shamir.rs)
class Transcript:
    def __init__(self, d: int, log: list | None = None):
        self.d = d
        self.t = O.new_transcript()
        self.log = log  # a list: every sampled value is appended (the product's sample log)

    def _sample(self) -> int:
        v = O.lib().lfo_tr_sample(O.C.byref(self.t))
        self.log.append(int(v))
        return v

    def absorb(self, elems):
        e = O._u64(elems)
        if e.size:
            O.lib().lfo_tr_absorb_ring(O.C.byref(self.t), e, e.size // self.d, self.d)

    def absorb_label(self, b: bytes):
        """absorb_field_element(BaseRing::from_base_prime_field(from_be_bytes_mod_order(b)))"""
        self.absorb(from_u(label(b), self.d))

    def get_challenge(self):
        """one base-ring challenge: 3 samples + their re-observation for Fq3
        (fiat_shamir.rs:69-86); one sample + re-observation for Fq (this
        project's convention for the X^d + 1 rings)"""
        if tb(self.d) == 3:
            out = np.zeros(3, np.uint64)
            if self.log is None:
                O.lib().lfo_tr_get_challenge(O.C.byref(self.t), out)
            else:  # lfo_tr_get_challenge's three samples, then their observes
                out[:] = [self._sample() for _ in range(3)]
                for v in out:
                    O.lib().lfo_tr_observe(O.C.byref(self.t), int(v))
            return out
        v = O.lib().lfo_tr_sample(O.C.byref(self.t)) if self.log is None else self._sample()
        O.lib().lfo_tr_observe(O.C.byref(self.t), v)
        return np.array([v], np.uint64)

    def get_challenges(self, n: int):
        """n challenges, each broadcast into an NTT element ([n][d])"""
        return [scal(self.get_challenge(), self.d) for _ in range(n)]

    def squeeze_bytes(self, n: int) -> bytes:
        if self.log is not None:  # lfo_tr_squeeze_bytes: one sample per 8 bytes, little-endian
            return b"".join(int(self._sample()).to_bytes(8, "little") for _ in range(-(-n // 8)))[:n]
        out = np.zeros(n, np.uint8)
        O.lib().lfo_tr_squeeze_bytes(O.C.byref(self.t), out, n)
        return out.tobytes()

    def short_challenge(self):
        """get_short_challenge (fiat_shamir.rs:105-113): coefficient form"""
        return O.short_challenge(self.squeeze_bytes(3 * self.d // 4), self.d)


def sumcheck_verify(tr: Transcript, proof, nv: int, degree: int, claim):
    """MLSumcheck::verify_as_subprotocol (LF/utils/sumcheck.rs:90-111): replays the
    transcript for the challenges, then the round checks; returns (ok, point, expected)"""
    d = tr.d
    tr.absorb(from_u(nv, d))
    tr.absorb(from_u(degree, d))
    proof = O._u64(proof).reshape(nv, (degree + 1) * d)
    rnd = []
    for i in range(nv):
        tr.absorb(proof[i])
        ch = tr.get_challenge()
        rnd.append(ch)
        tr.absorb(scal(ch, d))
    rc, expected = O.sumcheck_check(proof.ravel(), np.concatenate(rnd), nv, d, degree, claim)
    return rc == 0, [scal(c, d) for c in rnd], expected


# ---------------------------------------------------------------- structures
@dataclass
class CCS:
    """LF/arith.rs:51-74; mats: [(row_ptr, col, val)] of m x n NTT elements"""
    d: int
    m: int
    n: int
    l: int
    mats: list
    c: list          # q NTT elements
    S: list          # q multisets of matrix indices
    degree: int      # ccs.d

    @property
    def t(self):
        return len(self.mats)

    @property
    def s(self):
        return self.m.bit_length() - 1


@dataclass
class LCCCS:
    """LF/arith.rs:192-206 (lists of NTT elements)"""
    r: list
    v: list
    cm: np.ndarray   # [kappa][d]
    u: list
    x_w: list
    h: np.ndarray


@dataclass
class Witness:
    """LF/arith.rs:214-223 (f_hat is made on demand)"""
    w_ccs: np.ndarray
    f: np.ndarray
    f_coeff: np.ndarray


@dataclass
class Proof:
    """LFProof (LF/nifs.rs:28-34)"""
    lin_sumcheck: np.ndarray = None
    lin_v: list = None
    lin_u: list = None
    dec: list = field(default_factory=list)   # two dicts: u_s, v_s, x_s, y_s
    fold_sumcheck: np.ndarray = None
    theta_s: list = None
    eta_s: list = None


@dataclass
class Params:
    d: int
    B: int = 1 << 15
    L: int = 5
    b_small: int = 2
    K: int = 15


def fhat(f_coeff, N: int, nv: int, d: int):
    """Witness::get_fhat (LF/arith.rs:273-297), zero-padded to 2^nv: tau MLEs"""
    if d == 24:
        fh = O.get_fhat_phi72(f_coeff).reshape(3, N * 24)
        return [pad_mle(fh[j], nv, d) for j in range(3)]
    return [pad_mle(f_coeff, nv, d)]


def mz_mles(ccs: CCS, z):
    """calculate_Mz_mles (LF/utils/mle_helpers.rs:137-146) as [t][2^s d]"""
    return list(O.mz_mles(ccs.mats, z, ccs.s, ccs.d).reshape(ccs.t, -1))


def elems(x, d: int):
    x = O._u64(x)
    return [x[i:i + d] for i in range(0, x.size, d)]


def flat(part):
    """a list of NTT elements (or an already flat array) as one array"""
    if isinstance(part, np.ndarray):
        return part
    return np.concatenate([O._u64(x) for x in part]) if len(part) else np.zeros(0, np.uint64)


def absorb_public_input(tr: Transcript, acc: LCCCS, cm_i, x_ccs):
    """ZK/zk_latticefold.rs:162-184"""
    tr.absorb_label(b"acc")
    for part in (acc.r, acc.v, acc.cm, acc.u, acc.x_w):
        tr.absorb(flat(part))
    tr.absorb(acc.h)
    tr.absorb_label(b"cm_i")
    tr.absorb(cm_i)
    tr.absorb(flat(x_ccs))


def sanity_check(ccs: CCS, pr: Params):
    """ZK/zk_latticefold.rs:152-158"""
    want = max((ccs.n - ccs.l - 1) * pr.L, ccs.m)
    want = 1 << (want - 1).bit_length()
    if ccs.m != want:
        raise ValueError("CSError::InvalidSizeBounds")


# ---------------------------------------------------------------- prover
def linearize(tr: Transcript, ccs: CCS, cm, x_ccs, w: Witness, pr: Params):
    """LFLinearizationProver::prove (LF/nifs/linearization.rs:153-197)"""
    d, s = ccs.d, ccs.s
    tr.absorb_label(b"beta_s")  # squeeze_beta_challenges (linearization/utils.rs:111-124)
    beta = tr.get_challenges(s)
    z = np.concatenate(list(x_ccs) + [one(d), O._u64(w.w_ccs)])  # get_z_vector: x || 1 || w
    Mz = mz_mles(ccs, z)
    g = [Mz[j] for i, c in enumerate(ccs.c) if not is_zero(c) for j in ccs.S[i]]
    g.append(O.eq_table(np.concatenate(beta), s, d))
    comb = O.SumcheckComb.linearization(np.concatenate(ccs.c), ccs.S)
    proof, rnd = O.sumcheck_prove(tr.t, comb, np.concatenate(g), len(g), s, d, ccs.degree + 1)
    r = [scal(rnd[i * tb(d):(i + 1) * tb(d)], d) for i in range(s)]
    N = O._u64(w.f_coeff).size // d
    v = elems(evaluate(fhat(w.f_coeff, N, s, d), s, d, np.concatenate(r)), d)
    u = elems(evaluate(Mz, s, d, np.concatenate(r)), d)
    tr.absorb(np.concatenate(v))
    tr.absorb(np.concatenate(u))
    lcccs = LCCCS(r=r, v=v, cm=O._u64(cm), u=u, x_w=list(x_ccs), h=one(d))
    return lcccs, (proof, v, u)


def decompose(tr: Transcript, ccs: CCS, A, kappa: int, acc: LCCCS, w: Witness, pr: Params):
    """LFDecompositionProver::prove (LF/nifs/decomposition.rs:33-88)"""
    d, s, K, L = ccs.d, ccs.s, pr.K, pr.L
    N = O._u64(w.f_coeff).size // d
    fck, fk, wk = O.decompose_witness(w.f_coeff, d, pr.B, L, pr.b_small, K)
    fck, fk, wk = fck.reshape(K, -1), fk.reshape(K, -1), wk.reshape(K, -1)
    xs = O.compute_x_s(np.concatenate(list(acc.x_w) + [acc.h]), d, pr.B, L, pr.b_small, K).reshape(K, -1)
    # commit_witnesses (:178-201): y_k = A f_k for k >= 1, y_0 = cm - sum_k b^k y_k
    y = np.zeros((K, kappa * d), np.uint64)
    for k in range(1, K):
        y[k] = O.ajtai_commit(A, kappa, N, d, fk[k])
    y = O.commit_witnesses_y0(O._u64(acc.cm), y.ravel(), kappa, d, pr.b_small, K).reshape(K, -1)
    r = np.concatenate(acc.r)
    v_s = [elems(evaluate(fhat(fck[k], N, s, d), s, d, r), d) for k in range(K)]
    mz = [mz_mles(ccs, np.concatenate([xs[k], wk[k]])) for k in range(K)]
    u_s = [elems(evaluate(mz[k], s, d, r), d) for k in range(K)]
    lcccs = []
    for k in range(K):
        tr.absorb(xs[k])
        tr.absorb(y[k])
        tr.absorb(np.concatenate(u_s[k]))
        tr.absorb(np.concatenate(v_s[k]))
        xk = elems(xs[k], d)
        lcccs.append(LCCCS(r=list(acc.r), v=v_s[k], cm=y[k], u=u_s[k], x_w=xk[:-1], h=xk[-1]))
    wits = [Witness(w_ccs=wk[k], f=fk[k], f_coeff=fck[k]) for k in range(K)]
    proof = {"u_s": u_s, "v_s": v_s, "x_s": [elems(xs[k], d) for k in range(K)], "y_s": [elems(y[k], d) for k in range(K)]}
    return mz, lcccs, wits, proof


def squeeze_alpha_beta_zeta_mu(tr: Transcript, K: int, log_m: int):
    """LF/nifs/folding/utils.rs:51-96"""
    tr.absorb_label(b"alpha_s")
    alpha = tr.get_challenges(2 * K)
    tr.absorb_label(b"zeta_s")
    zeta = tr.get_challenges(2 * K)
    tr.absorb_label(b"mu_s")
    mu = tr.get_challenges(2 * K - 1) + [one(tr.d)]
    tr.absorb_label(b"beta_s")
    beta = tr.get_challenges(log_m)
    return alpha, beta, zeta, mu


def get_rhos(tr: Transcript, K: int):
    """LF/nifs/folding/utils.rs:116-127: 2K - 1 short challenges + ONE, and their CRT"""
    d = tr.d
    tr.absorb_label(b"rho_s")
    rc = [tr.short_challenge() for _ in range(2 * K - 1)]
    c1 = np.zeros(d, np.uint64)
    c1[0] = 1
    rc.append(c1)
    rho = elems(O.crt(np.concatenate(rc), d), d)
    return rc, rho


def combined_g(fhats, alphas, challenged, d: int):
    """prepare_g1_and_3_k_mles_list (LF/nifs/folding/utils.rs:519-541)"""
    comb = np.zeros_like(challenged)
    for fh, a in zip(fhats, alphas):
        mle = np.zeros_like(challenged)
        for f in reversed(fh):
            mle = smul(a, add(mle, f), d)
        comb = add(comb, mle)
    return add(comb, challenged)


def challenged_mz(mzs, zetas, d: int):
    """calculate_challenged_mz_mle (LF/nifs/folding.rs:208-234)"""
    total = np.zeros_like(mzs[0][0])
    for mz, zeta in zip(mzs, zetas):
        mle = np.zeros_like(total)
        for M in reversed(mz):
            mle = smul(zeta, add(mle, M), d)
        total = add(total, mle)
    return total


def fold(tr: Transcript, ccs: CCS, lcccs: list, wits: list, mzs: list, pr: Params):
    """LFFoldingProver::prove (LF/nifs/folding.rs:42-130)"""
    d, s, K = ccs.d, ccs.s, pr.K
    alpha, beta, zeta, mu = squeeze_alpha_beta_zeta_mu(tr, K, s)
    N = O._u64(wits[0].f_coeff).size // d
    fhats = [fhat(w.f_coeff, N, s, d) for w in wits]
    g1 = combined_g(fhats[:K], alpha[:K], challenged_mz(mzs[:K], zeta[:K], d), d)
    g3 = combined_g(fhats[K:], alpha[K:], challenged_mz(mzs[K:], zeta[K:], d), d)
    mles = [O.eq_table(np.concatenate(lcccs[0].r), s, d), g1, O.eq_table(np.concatenate(lcccs[K].r), s, d), g3,
            O.eq_table(np.concatenate(beta), s, d)] + [f for fh in fhats for f in fh]
    tau = len(fhats[0])
    comb = O.SumcheckComb.folding(np.concatenate(mu), 2 * K, tau, pr.b_small)
    proof, rnd = O.sumcheck_prove(tr.t, comb, np.concatenate(mles), len(mles), s, d, 2 * pr.b_small)
    r0 = [scal(rnd[i * tb(d):(i + 1) * tb(d)], d) for i in range(s)]
    pt = np.concatenate(r0)
    theta = [elems(evaluate(fh, s, d, pt), d) for fh in fhats]
    eta = [elems(evaluate(mz, s, d, pt), d) for mz in mzs]
    for th in theta:
        tr.absorb(np.concatenate(th))
    for et in eta:
        tr.absorb(np.concatenate(et))
    rc, rho = get_rhos(tr, K)
    f0 = O.fold_f0(np.concatenate(rho), np.concatenate([w.f for w in wits]), 2 * K, N, d)
    out = fold_public(rc, rho, theta, lcccs, eta, r0, ccs)
    fc0, w0 = O.witness_from_f(f0, d, pr.B, pr.L)
    return out, Witness(w_ccs=w0, f=f0, f_coeff=fc0), (proof, theta, eta), rc, rho


def fold_public(rc, rho, theta, lcccs, eta, r0, ccs: CCS):
    """compute_v0_u0_x0_cm_0 (LF/nifs/folding/utils.rs:456-517) + prepare_public_output (folding.rs:381-392)"""
    d = ccs.d
    v0 = elems(O.rot_lin_combination(np.concatenate(rc), np.concatenate([np.concatenate(t) for t in theta]), d), d)
    kappa = O._u64(lcccs[0].cm).size // d
    cm0 = np.zeros(kappa * d, np.uint64)
    for r_i, L_i in zip(rho, lcccs):
        cm0 = add(cm0, smul(r_i, L_i.cm, d))
    u0 = np.zeros(ccs.t * d, np.uint64)
    for r_i, e_i in zip(rho, eta):
        u0 = add(u0, smul(r_i, np.concatenate(e_i), d))
    x0 = np.zeros((ccs.l + 1) * d, np.uint64)
    for r_i, L_i in zip(rho, lcccs):
        x0 = add(x0, smul(r_i, np.concatenate(list(L_i.x_w) + [L_i.h]), d))
    x0 = elems(x0, d)
    return LCCCS(r=r0, v=v0, cm=cm0, u=elems(u0, d), x_w=x0[:-1], h=x0[-1])


def fold_prove(ccs: CCS, A, kappa: int, acc: LCCCS, w_acc: Witness, cm_i, x_ccs, w_i: Witness, pr: Params):
    """zk_latticefold_prove (ZK/zk_latticefold.rs:37-102) with a fresh transcript
    (fold(), ZK/main.rs:394): -> (folded LCCCS, its witness, LFProof)"""
    sanity_check(ccs, pr)
    tr = Transcript(ccs.d)
    absorb_public_input(tr, acc, cm_i, x_ccs)
    lin, (lproof, lv, lu) = linearize(tr, ccs, cm_i, x_ccs, w_i, pr)
    mz_l, lc_l, wit_l, dp_l = decompose(tr, ccs, A, kappa, acc, w_acc, pr)
    mz_r, lc_r, wit_r, dp_r = decompose(tr, ccs, A, kappa, lin, w_i, pr)
    out, w0, (fproof, theta, eta), _, _ = fold(tr, ccs, lc_l + lc_r, wit_l + wit_r, mz_l + mz_r, pr)
    proof = Proof(lin_sumcheck=lproof, lin_v=lv, lin_u=lu, dec=[dp_l, dp_r], fold_sumcheck=fproof,
                  theta_s=theta, eta_s=eta)
    return out, w0, proof


def linearize_fresh(ccs: CCS, cm, x_ccs, w: Witness, pr: Params):
    """an accumulator the way initialize_accumulator makes one (ZK/main.rs:305-344):
    LFLinearizationProver::prove of a CCCS on a fresh transcript"""
    lc, _ = linearize(Transcript(ccs.d), ccs, cm, x_ccs, w, pr)
    return lc


# ---------------------------------------------------------------- verifier
def recompose(vals, b_s, d: int):
    """LFDecompositionVerifier::recompose (decomposition.rs:236-256)"""
    out = [zero(d) for _ in vals[0]]
    for k, row in enumerate(vals):
        for j, x in enumerate(row):
            out[j] = add(out[j], mul(b_s[k], x, d))
    return out


def fold_verify(ccs: CCS, acc: LCCCS, cm_i, x_ccs, proof: Proof, pr: Params):
    """NIFSVerifier::verify (LF/nifs.rs:117-162) over the zkvm's public-input
    absorption: raises ValueError on a rejected proof, returns the folded LCCCS"""
    d, s, K = ccs.d, ccs.s, pr.K
    tr = Transcript(d)
    absorb_public_input(tr, acc, cm_i, x_ccs)
    # linearization (linearization.rs:265-285)
    tr.absorb_label(b"beta_s")
    beta = tr.get_challenges(s)
    ok, r, expected = sumcheck_verify(tr, proof.lin_sumcheck, s, ccs.degree + 1, zero(d))
    if not ok:
        raise ValueError("linearization sumcheck")
    e = eq_eval(r, beta, d)
    total = zero(d)
    for c_i, S_i in zip(ccs.c, ccs.S):
        term = O._u64(c_i)
        for j in S_i:
            term = mul(term, proof.lin_u[j], d)
        total = add(total, term)
    if not np.array_equal(mul(e, total, d), expected):
        raise ValueError("linearization evaluation claim")
    tr.absorb(np.concatenate(proof.lin_v))
    tr.absorb(np.concatenate(proof.lin_u))
    lin = LCCCS(r=r, v=list(proof.lin_v), cm=O._u64(cm_i), u=list(proof.lin_u), x_w=list(x_ccs), h=one(d))
    # decompositions (decomposition.rs:90-155)
    b_s = [from_u(pr.b_small ** k, d) for k in range(K)]
    lcccs = []
    for src, dp in ((acc, proof.dec[0]), (lin, proof.dec[1])):
        for k in range(K):
            tr.absorb(np.concatenate(dp["x_s"][k]))
            tr.absorb(np.concatenate(dp["y_s"][k]))
            tr.absorb(np.concatenate(dp["u_s"][k]))
            tr.absorb(np.concatenate(dp["v_s"][k]))
            xk = dp["x_s"][k]
            lcccs.append(LCCCS(r=list(src.r), v=dp["v_s"][k], cm=np.concatenate(dp["y_s"][k]), u=dp["u_s"][k],
                               x_w=xk[:-1], h=xk[-1]))
        checks = (("y", dp["y_s"], elems(src.cm, d)), ("v", dp["v_s"], src.v), ("u", dp["u_s"], src.u),
                  ("x", dp["x_s"], list(src.x_w) + [src.h]))
        for name, parts, want in checks:
            got = recompose(parts, b_s, d)
            if not all(np.array_equal(a, b) for a, b in zip(got, want)) or len(got) != len(want):
                raise ValueError(f"decomposition recompose {name}")
    # folding (folding.rs:133-200)
    alpha, beta, zeta, mu = squeeze_alpha_beta_zeta_mu(tr, K, s)
    claim = zero(d)
    for a_i, z_i, L_i in zip(alpha, zeta, lcccs):
        claim = add(claim, add(powers_dot(a_i, L_i.v, d), powers_dot(z_i, L_i.u, d)))
    ok, r0, expected = sumcheck_verify(tr, proof.fold_sumcheck, s, 2 * pr.b_small, claim)
    if not ok:
        raise ValueError("folding sumcheck")
    e_ast = eq_eval(beta, r0, d)
    want = zero(d)
    for i in range(2 * K):  # compute_sumcheck_claim_expected_value (folding/utils.rs:380-421)
        e_i = eq_eval(lcccs[i].r, r0, d)
        th = proof.theta_s[i]
        sm = mul(powers_dot(alpha[i], th, d), e_i, d)
        norm, pw = zero(d), mu[i]
        for t_ in th:
            prod = t_
            for j in range(1, pr.b_small):
                jh = from_u(j, d)
                prod = mul(prod, mul(sub(t_, jh), add(t_, jh), d), d)
            norm = add(norm, mul(pw, prod, d))
            pw = mul(pw, mu[i], d)
        sm = add(sm, mul(e_ast, norm, d))
        sm = add(sm, mul(e_i, powers_dot(zeta[i], proof.eta_s[i], d), d))
        want = add(want, sm)
    if not np.array_equal(want, expected):
        raise ValueError("folding evaluation claim")
    for th in proof.theta_s:
        tr.absorb(np.concatenate(th))
    for et in proof.eta_s:
        tr.absorb(np.concatenate(et))
    rc, rho = get_rhos(tr, K)
    return fold_public(rc, rho, proof.theta_s, lcccs, proof.eta_s, r0, ccs)


# ---------------------------------------------------------------- satisfied test instances
def random_ring(n: int, d: int, seed: int):
    return O.fill_uniform(n * d, seed)


def satisfied_ccs(d: int, W: int, l: int, t: int, deg: int, seed: int, pr: Params, per_row: int = 2,
                  empty: float = 0.0, scalar: bool = False):
    """A CCS of t matrices, q = 2 multisets S = [[0, .., deg-1], [deg]] and
    c = [1, -1] (a degree-`deg` R1CS generalisation) with m = (W L) rounded up to
    a power of two: A_j (j < deg) read only the 'free' columns (x, 1, the first
    half of w); matrix deg reads one 'product' column in each of the first
    rows; later rows repeat earlier ones; matrices past deg are random extras.
    satisfying_z makes z vectors that satisfy it. empty: the share of A_j rows (j < deg)
    left without entries (their product column is then 0). scalar: every entry a
    scalar (from_u), as the zkvm's R1CS-derived matrices hold."""
    rng = np.random.default_rng(seed)
    rng_e = np.random.default_rng(seed + 7)
    n = l + 1 + W
    m = 1 << ((W * pr.L) - 1).bit_length()
    free = l + 1 + W // 2
    nprod = n - free
    vseed = seed + 100
    rows = {j: [] for j in range(t)}
    for r_ in range(m):
        for j in range(t):
            if r_ >= nprod and j <= deg:
                rows[j].append(rows[j][r_ % nprod])
            elif j == deg:
                rows[j].append(([free + r_], [one(d)]))
            elif j < deg and empty and rng_e.random() < empty:
                rows[j].append(([], []))
            else:
                k = int(rng.integers(1, per_row + 1))
                cols = sorted(set(int(c) for c in rng.integers(0, free if j < deg else n, k)))
                if scalar:
                    vals = [from_u(int(O.fill_uniform(1, vseed + i)[0]), d) for i in range(len(cols))]
                else:
                    vals = [random_ring(1, d, vseed + i) for i in range(len(cols))]
                vseed += len(cols)
                rows[j].append((cols, vals))
    mats = []
    for j in range(t):
        rp = np.zeros(m + 1, np.uint64)
        col, val = [], []
        for r_, (cols, vals) in enumerate(rows[j]):
            col += cols
            val += vals
            rp[r_ + 1] = rp[r_] + len(cols)
        mats.append((rp, np.array(col, np.uint32), np.concatenate(val) if val else np.zeros(0, np.uint64)))
    return CCS(d=d, m=m, n=n, l=l, mats=mats, c=[one(d), from_u(P - 1, d)], S=[list(range(deg)), [deg]], degree=deg)


def satisfied_ccs_np(d: int, W: int, l: int, t: int, deg: int, seed: int, pr: Params, per_row: int = 2,
                     extra_density: float = 1.0):
    """satisfied_ccs's construction vectorised with numpy for large shapes (the
    zkvm's t = 125, m = 2^17): the same row rules (A_j, j < deg: 1..per_row
    entries on the free columns, rows past the product columns repeating row
    r mod nprod; matrix deg: the product column of the row's owner; extras:
    random entries anywhere, in a random extra_density share of the rows)"""
    rng = np.random.default_rng(seed)
    n = l + 1 + W
    m = 1 << ((W * pr.L) - 1).bit_length()
    free = l + 1 + W // 2
    nprod = n - free
    src = np.arange(m) % nprod  # the row every row repeats (itself for r < nprod)
    mats = []
    for j in range(t):
        if j == deg:
            col = (free + src).astype(np.uint32)
            rp = np.arange(m + 1, dtype=np.uint64)
            val = np.tile(one(d), m)
        else:
            base = nprod if j < deg else m
            cnt = rng.integers(1, per_row + 1, base)
            if j > deg and extra_density < 1.0:
                cnt[rng.random(base) >= extra_density] = 0
            off = np.concatenate([[0], np.cumsum(cnt)])
            cols = rng.integers(0, free if j < deg else n, int(off[-1])).astype(np.uint32)
            vals = O.fill_uniform(int(off[-1]) * d, seed + 1000 + j).reshape(-1, d)
            rows = src if j < deg else np.arange(m)
            c_r = cnt[rows]
            rp = np.concatenate([[0], np.cumsum(c_r)]).astype(np.uint64)
            gather = np.repeat(off[rows], c_r) + (np.arange(int(rp[-1])) - np.repeat(rp[:-1].astype(np.int64), c_r))
            col = cols[gather]
            val = vals[gather].ravel()
        mats.append((rp, col, val))
    return CCS(d=d, m=m, n=n, l=l, mats=mats, c=[one(d), from_u(P - 1, d)], S=[list(range(deg)), [deg]], degree=deg)


def satisfying_z(ccs: CCS, W: int, seed: int):
    """(x_ccs [l][d], w_ccs [W d]) with z = x || 1 || w satisfying satisfied_ccs's CCS:
    random free columns, then each product column = prod_j (A_j z) of its row"""
    d, l, n = ccs.d, ccs.l, ccs.n
    deg = ccs.S[1][0]
    free = l + 1 + W // 2
    z = np.concatenate([random_ring(l, d, seed + 1), one(d), random_ring(W, d, seed + 2)]).reshape(n, d)
    z[free:] = 0
    acc = np.tile(one(d), n - free)
    for j in range(deg):
        rp, col, val = ccs.mats[j]
        acc = mul(acc, O.spmv(rp, col, val, d, z.ravel())[:(n - free) * d], d)
    z[free:] = acc.reshape(n - free, d)
    return [z[i].copy() for i in range(l)], z[l + 1:].ravel().copy()


def check_relation(ccs: CCS, z):
    """CCS::check_relation (LF/arith.rs:77-103)"""
    d = ccs.d
    total = np.zeros(ccs.m * d, np.uint64)
    for c_i, S_i in zip(ccs.c, ccs.S):
        had = np.tile(one(d), ccs.m)
        for j in S_i:
            rp, col, val = ccs.mats[j]
            had = mul(had, O.spmv(rp, col, val, d, z), d)
        total = add(total, smul(c_i, had, d))
    return not np.any(total)


# ---------------------------------------------------------------- verifier-variable replay
def fq3_inv(a):
    """inverse in Fq3 = Fq[u]/(u^3 - 2^40) (via the norm)"""
    w = 1 << 40
    a0, a1, a2 = (int(x) for x in a)
    t0 = (a0 * a0 - w * a1 * a2) % P
    t1 = (w * a2 * a2 - a0 * a1) % P
    t2 = (a1 * a1 - a0 * a2) % P
    n = (a0 * t0 + w * (a2 * t1 + a1 * t2)) % P
    ni = pow(n, P - 2, P)
    return [t0 * ni % P, t1 * ni % P, t2 * ni % P]


def fq3_mul(a, b):
    w = 1 << 40
    a0, a1, a2 = (int(x) for x in a)
    b0, b1, b2 = (int(x) for x in b)
    return [(a0 * b0 + w * (a1 * b2 + a2 * b1)) % P, (a0 * b1 + a1 * b0 + w * a2 * b2) % P,
            (a0 * b2 + a1 * b1 + a2 * b0) % P]


def zk_interpolate(p, r3, d: int):
    """zk_interpolate_uni_poly (LF/utils/sumcheck/verifier.rs:267-340): the value at
    r of the polynomial through (i, p_i) and its terms p_i L_i(r), i from len - 1 down"""
    n = len(p)
    terms = []
    for i in reversed(range(n)):
        num = [1, 0, 0]
        den = 1
        for j in range(n):
            if j != i:
                num = fq3_mul(num, [(int(r3[0]) - j) % P, int(r3[1]), int(r3[2])])
                den = den * (i - j) % P
        x = fq3_mul(num, [pow(den, P - 2, P), 0, 0])
        terms.append(mul(p[i], scal(x, d), d))
    res = zero(d)
    for t_ in terms:
        res = add(res, t_)
    return res, terms


def zk_eq(x, y, d: int):
    """zk_eq_eval (LF/utils/sumcheck/utils.rs:100-131): eq(x, y) and its helper values"""
    res, xy, fac, sub_res = one(d), [], [], [one(d)]
    for xi, yi in zip(x, y):
        p = mul(xi, yi, d)
        xy.append(p)
        f = add(sub(sub(add(p, p), xi), yi), one(d))
        fac.append(f)
        res = mul(res, f, d)
        sub_res.append(res)
    return res, {"xi_yis": xy, "factors": fac, "sub_res": sub_res}


def replay_sumcheck(tr: Transcript, proof, nv: int, degree: int, claim):
    """collect_*_sumcheck_vars (ZK/zk_latticefold.rs:283-345, 596-659)"""
    d = tr.d
    tr.absorb(from_u(nv, d))
    tr.absorb(from_u(degree, d))
    msgs = O._u64(proof).reshape(nv, degree + 1, d)
    claimed, subterms, point = [claim], [], []
    for i in range(nv):
        tr.absorb(msgs[i].ravel())
        ch = tr.get_challenge()
        point.append(ch)
        cs, terms = zk_interpolate(list(msgs[i]), ch, d)
        claimed.append(cs)
        subterms += terms
        tr.absorb(scal(ch, d))
    return {"claimed_sums": claimed, "subterms": subterms, "point": [scal(c, d) for c in point],
            "expected": claimed[-1]}


def fold_replay(ccs: CCS, acc: LCCCS, cm_i, x_ccs, proof: Proof, pr: Params, log: list | None = None):
    """generate_verification_witness_vars (ZK/zk_latticefold.rs:111-148): the
    transcript replay of a fold() proof and the values the in-CCS verifier needs.
    log: a list that receives every sampled value (the product's sample log)"""
    d, s, K, t = ccs.d, ccs.s, pr.K, ccs.t
    assert d == 24, "the zkvm's replay is written for the Phi_72 ring (TAU = 3)"
    tr = Transcript(d, log)
    absorb_public_input(tr, acc, cm_i, x_ccs)
    # collect_linearization_vars (:204-277)
    tr.absorb_label(b"beta_s")
    beta = tr.get_challenges(s)
    lin = replay_sumcheck(tr, proof.lin_sumcheck, s, ccs.degree + 1, zero(d))
    _, eqv = zk_eq(lin["point"], beta, d)
    inner, products = zero(d), []
    for c_i, S_i in zip(ccs.c, ccs.S):
        prod = one(d)
        for j in S_i:
            prod = mul(prod, proof.lin_u[j], d)
        products.append(prod)
        inner = add(inner, mul(c_i, prod, d))
    tr.absorb(np.concatenate(proof.lin_v))
    tr.absorb(np.concatenate(proof.lin_u))
    lin_lcccs = LCCCS(r=lin["point"], v=list(proof.lin_v), cm=O._u64(cm_i), u=list(proof.lin_u), x_w=list(x_ccs),
                      h=one(d))
    # collect_decomposition_vars (:393-432)
    lcccs = []
    for src, dp in ((acc, proof.dec[0]), (lin_lcccs, proof.dec[1])):
        for k in range(K):
            for part in (dp["x_s"][k], dp["y_s"][k], dp["u_s"][k], dp["v_s"][k]):
                tr.absorb(np.concatenate(part))
            xk = dp["x_s"][k]
            lcccs.append(LCCCS(r=list(src.r), v=dp["v_s"][k], cm=np.concatenate(dp["y_s"][k]), u=dp["u_s"][k],
                               x_w=xk[:-1], h=xk[-1]))
    # collect_folding_vars (:465-581)
    alpha, fbeta, zeta, mu = squeeze_alpha_beta_zeta_mu(tr, K, s)
    h1s, h2s, g1t, g3h, g3t = [], [], [], [], []
    g1, g3 = zero(d), zero(d)
    for i in range(2 * K):
        v_i, u_i = lcccs[i].v, lcccs[i].u
        h1 = add(mul(alpha[i], v_i[2], d), v_i[1])
        h2 = add(mul(alpha[i], h1, d), v_i[0])
        ci = mul(alpha[i], h2, d)
        h1s.append(h1)
        h2s.append(h2)
        g1t.append(ci)
        g1 = add(g1, ci)
        h = add(mul(zeta[i], u_i[t - 1], d), u_i[t - 2])
        g3h.append(h)
        for j in reversed(range(t - 2)):
            h = add(mul(zeta[i], h, d), u_i[j])
            g3h.append(h)
        c3 = mul(zeta[i], h, d)
        g3t.append(c3)
        g3 = add(g3, c3)
    fs = replay_sumcheck(tr, proof.fold_sumcheck, s, 2 * pr.b_small, add(g1, g3))
    r0 = fs["point"]
    e_ast, _ = zk_eq(fbeta, r0, d)
    should = zero(d)
    for i in range(2 * K):
        e_i, _ = zk_eq(lcccs[i].r, r0, d)
        th = proof.theta_s[i]
        sm = mul(powers_dot(alpha[i], th, d), e_i, d)
        norm, pw = zero(d), mu[i]
        for t_ in th:
            prod = t_
            for j in range(1, pr.b_small):
                jh = from_u(j, d)
                prod = mul(prod, mul(sub(t_, jh), add(t_, jh), d), d)
            norm = add(norm, mul(pw, prod, d))
            pw = mul(pw, mu[i], d)
        sm = add(sm, mul(e_ast, norm, d))
        sm = add(sm, mul(e_i, powers_dot(zeta[i], proof.eta_s[i], d), d))
        should = add(should, sm)
    for th in proof.theta_s:
        tr.absorb(np.concatenate(th))
    for et in proof.eta_s:
        tr.absorb(np.concatenate(et))
    _, rho = get_rhos(tr, K)
    final_cm = [mul(cm_j, rho[i], d) for i in range(2 * K) for cm_j in elems(lcccs[i].cm, d)]
    final_u = [mul(e, rho[i], d) for i in range(2 * K) for e in proof.eta_s[i]]
    final_x = [mul(x, rho[i], d) for i in range(2 * K) for x in list(lcccs[i].x_w) + [lcccs[i].h]]
    return {"lin_beta": beta, "lin_claimed_sums": lin["claimed_sums"], "lin_subterms": lin["subterms"],
            "lin_point": lin["point"], "lin_expected": lin["expected"], "lin_inner": inner,
            "lin_products": products, "lin_eq_xy": eqv["xi_yis"], "lin_eq_factors": eqv["factors"],
            "lin_eq_sub": eqv["sub_res"], "alpha": alpha, "beta": fbeta, "zeta": zeta, "mu": mu,
            "claim_g1_h1": h1s, "claim_g1_h2": h2s, "claim_g1_terms": g1t, "claim_g1": g1, "claim_g3_h": g3h,
            "claim_g3_terms": g3t, "claim_g3": g3, "fold_claimed_sums": fs["claimed_sums"],
            "fold_subterms": fs["subterms"], "fold_point": r0, "fold_expected": fs["expected"],
            "should_equal_s": should, "rho": rho, "final_cm": final_cm, "final_u": final_u, "final_x": final_x}
