// replay.cpp -- the zkvm's verifier-variable replay on the host:
// generate_verification_witness_vars (zkvm/src/zk_latticefold.rs:111-148) replays
// a fold() proof's Poseidon2 transcript (a second pass of the same sponge per
// step) and collects the values the in-CCS folding verifier consumes:
//   collect_linearization_vars (:204-277) with its sumcheck (:283-345),
//   collect_decomposition_vars (:393-432),
//   collect_folding_vars (:465-581) with its sumcheck (:596-659).
// Sequential scalar work (the transcript and a few thousand Fq3 products), so
// it is host code; Phi_72 only (the replay is written for TAU = 3).
#include <array>
#include <cstring>

#include <vector>

#include "../../include/lf.h"
#include "ring.hpp"

namespace {

constexpr int D = 24, S8 = 8;
using Elem = std::array<uint64_t, 24>;  // one NTT element: 8 Fq3 slots (no heap traffic per operation)

// Fq3 product: each output is a sum of products taken in 128 bits and reduced
// once (gl::reduce128 takes any 128-bit value); the nonresidue 2^40 a shift
inline uint64_t dot2(uint64_t a, uint64_t b, uint64_t c, uint64_t e) {  // a b + c e mod p
  const unsigned __int128 x = (unsigned __int128)a * b, y = (unsigned __int128)c * e;
  const unsigned __int128 s = x + y;
  const uint64_t r = gl::canon(gl::reduce128((uint64_t)s, (uint64_t)(s >> 64)));
  return s < x ? gl::add(r, 0xFFFFFFFE00000001ull) : r;  // a carry out: + 2^128 == -2^32 == p - 2^32
}
void f3mul(const uint64_t *a, const uint64_t *b, uint64_t *o) {
  const uint64_t c0 = gl::add(gl::mul(a[0], b[0]), gl::shl96(dot2(a[1], b[2], a[2], b[1]), 40));
  const uint64_t c1 = gl::add(dot2(a[0], b[1], a[1], b[0]), gl::shl96(gl::mul(a[2], b[2]), 40));
  const uint64_t c2 = gl::add(dot2(a[0], b[2], a[1], b[1]), gl::mul(a[2], b[0]));
  o[0] = c0;
  o[1] = c1;
  o[2] = c2;
}
// Fq3 inverse through the norm: a^-1 = (t0 + t1 u + t2 u^2) / N(a)
void f3inv(const uint64_t *a, uint64_t *o) {
  const uint64_t w = 1ull << 40;
  const uint64_t t0 = gl::sub(gl::mul(a[0], a[0]), gl::mul(w, gl::mul(a[1], a[2])));
  const uint64_t t1 = gl::sub(gl::mul(w, gl::mul(a[2], a[2])), gl::mul(a[0], a[1]));
  const uint64_t t2 = gl::sub(gl::mul(a[1], a[1]), gl::mul(a[0], a[2]));
  const uint64_t n =
      gl::add(gl::mul(a[0], t0), gl::mul(w, gl::add(gl::mul(a[2], t1), gl::mul(a[1], t2))));
  const uint64_t ni = gl::inv(n);
  o[0] = gl::mul(t0, ni);
  o[1] = gl::mul(t1, ni);
  o[2] = gl::mul(t2, ni);
}
// the per-instance loops (2K instances, each writing only its own outputs; the
// sums over instances are taken afterwards)
template <class F>
void each(int n, F fn) {
  for (int i = 0; i < n; i++) fn(i);
}

Elem zero() { return Elem{}; }
Elem scal(const uint64_t *b) {  // from_scalar of an Fq3
  Elem e;
  for (int i = 0; i < D; i++) e[i] = b[i % 3];
  return e;
}
Elem one() {
  const uint64_t b[3] = {1, 0, 0};
  return scal(b);
}
Elem fromu(uint64_t x) {
  const uint64_t b[3] = {x, 0, 0};
  return scal(b);
}
Elem mul(const Elem &a, const Elem &b) {
  Elem r;
  for (int s = 0; s < S8; s++) f3mul(&a[3 * s], &b[3 * s], &r[3 * s]);
  return r;
}
Elem add(const Elem &a, const Elem &b) {
  Elem r;
  for (int i = 0; i < D; i++) r[i] = gl::add(a[i], b[i]);
  return r;
}
Elem sub(const Elem &a, const Elem &b) {
  Elem r;
  for (int i = 0; i < D; i++) r[i] = gl::sub(a[i], b[i]);
  return r;
}
Elem at(const uint64_t *p, size_t i) {
  Elem e;
  memcpy(e.data(), p + i * D, D * 8);
  return e;
}
void put(uint64_t *p, size_t i, const Elem &e) { memcpy(p + i * D, e.data(), D * 8); }

struct Tr {
  lf_transcript *t;
  explicit Tr(lf_transcript *tt) : t(tt) {}
  ~Tr() { lf_transcript_free(t); }
  void absorb(const uint64_t *e, size_t n) { lf_transcript_absorb_ring(t, e, n, D, LF_REPR_CANONICAL); }
  void absorb(const Elem &e) { absorb(e.data(), 1); }
  void label(const char *s) {
    uint64_t v = 0;
    for (const char *p = s; *p; p++) v = gl::add(gl::mul(v, 256), (uint8_t)*p);
    absorb(fromu(v));
  }
  Elem challenge(uint64_t *base3 = nullptr) {
    uint64_t b[3];
    lf_transcript_get_challenge(t, b);
    if (base3) memcpy(base3, b, 24);
    return scal(b);
  }
};

// zk_interpolate_uni_poly (latticefold/src/utils/sumcheck/verifier.rs:267-340):
// sum_i p_i L_i(r) and its terms, i from len - 1 down; L_i(r) = prod_{j != i}
// (r - j) / (i - j), exact in Fq3
Elem interpolate(const uint64_t *p, int len, const uint64_t *r3, uint64_t *terms) {
  Elem res = zero();
  for (int k = 0; k < len; k++) {
    const int i = len - 1 - k;
    uint64_t num[3] = {1, 0, 0};
    uint64_t den = 1;
    for (int j = 0; j < len; j++) {
      if (j == i) continue;
      const uint64_t rj[3] = {gl::sub(r3[0], (uint64_t)j), r3[1], r3[2]};
      uint64_t nx[3];
      f3mul(num, rj, nx);
      memcpy(num, nx, 24);
      den = gl::mul(den, i > j ? (uint64_t)(i - j) : gl::P - (uint64_t)(j - i));
    }
    const uint64_t di = gl::inv(den);
    const uint64_t x3[3] = {gl::mul(num[0], di), gl::mul(num[1], di), gl::mul(num[2], di)};
    const Elem term = mul(at(p, i), scal(x3));
    put(terms, k, term);
    res = add(res, term);
  }
  return res;
}

// collect_*_sumcheck_vars: the round messages absorbed, challenges sampled and
// absorbed, the claims interpolated; point (s), claimed sums (s + 1), terms
void sumcheck(Tr &T, const uint64_t *proof, int nv, int degree, const Elem &claim, uint64_t *point,
              uint64_t *claimed, uint64_t *subterms) {
  T.absorb(fromu((uint64_t)nv));
  T.absorb(fromu((uint64_t)degree));
  put(claimed, 0, claim);
  for (int i = 0; i < nv; i++) {
    const uint64_t *msg = proof + (size_t)i * (degree + 1) * D;
    T.absorb(msg, degree + 1);
    uint64_t r3[3];
    const Elem r = T.challenge(r3);
    put(point, i, r);
    put(claimed, i + 1, interpolate(msg, degree + 1, r3, subterms + (size_t)i * (degree + 1) * D));
    T.absorb(r);
  }
}

// zk_eq_eval (latticefold/src/utils/sumcheck/utils.rs:100-131)
Elem eq(const uint64_t *x, const uint64_t *y, int n, uint64_t *xy, uint64_t *fac, uint64_t *sub_res) {
  Elem res = one();
  if (sub_res) put(sub_res, 0, res);
  for (int i = 0; i < n; i++) {
    const Elem xi = at(x, i), yi = at(y, i);
    const Elem p = mul(xi, yi);
    const Elem f = add(sub(sub(add(p, p), xi), yi), one());
    res = mul(res, f);
    if (xy) put(xy, i, p);
    if (fac) put(fac, i, f);
    if (sub_res) put(sub_res, i + 1, res);
  }
  return res;
}

// the replay on transcript `tr` (owned: freed here) -- a fresh one, or a playback
// of the prover's own sample log
int replay(const lf_ccs_desc *ccs, const lf_params *pr, const lf_lcccs *acc, const uint64_t *cm_i,
           const uint64_t *x_ccs, const lf_lfproof_mut *proof, lf_replay_vars *out, int repr, lf_transcript *tr) {
  Tr T(tr);
  if (!tr) return LF_ERR_INVALID_ARG;
  if (!ccs || !pr || !acc || !cm_i || !proof || !out) return LF_ERR_INVALID_ARG;
  if (pr->d != D || acc->d != D) return LF_ERR_UNSUPPORTED_RING;  // TAU = 3 (zk_latticefold.rs:487)
  const int t = ccs->t, q = ccs->q, degree = ccs->degree;
  const size_t m = ccs->m, l = ccs->l;
  if (t < 2 || q < 1 || degree < 1 || !m || (m & (m - 1)) || (!x_ccs && l) || !ccs->c || !ccs->S_off ||
      !ccs->S_idx)
    return LF_ERR_INVALID_ARG;
  int s = 0;
  while (((size_t)1 << s) < m) s++;
  const int K = pr->K, bs = (int)pr->b_small, tau = 3;
  const size_t kappa = acc->cm.n;
  if (acc->r.n != (size_t)s || acc->v.n != (size_t)tau || acc->u.n != (size_t)t || acc->x_w.n != l)
    return LF_ERR_INCORRECT_LENGTH;
  const std::vector<int> S_off(ccs->S_off, ccs->S_off + q + 1);
  for (int i = 0; i < q; i++)
    if (S_off[i] < 0 || S_off[i + 1] < S_off[i]) return LF_ERR_INVALID_ARG;
  const std::vector<int> S_idx(ccs->S_idx, ccs->S_idx + S_off[q]);
  for (int j : S_idx)
    if (j < 0 || j >= t) return LF_ERR_INVALID_ARG;
  // canonical copies of every input the replay reads
  auto cp = [&](const uint64_t *p, size_t elems) {
    std::vector<uint64_t> v(p, p + elems);
    if (repr == LF_REPR_MONTGOMERY)
      for (auto &x : v) x = gl::from_mont(x);
    return v;
  };
  const auto c = cp(ccs->c, (size_t)q * D);
  const auto ar = cp(acc->r.elems, (size_t)s * D), av = cp(acc->v.elems, tau * D), acm = cp(acc->cm.elems, kappa * D),
             au = cp(acc->u.elems, (size_t)t * D), axw = cp(acc->x_w.elems, l * D), ah = cp(acc->h, D),
             cmi = cp(cm_i, kappa * D), xc = cp(x_ccs ? x_ccs : cm_i, x_ccs ? l * D : 0),
             lsc = cp(proof->lin_sumcheck, (size_t)s * (degree + 2) * D), lv = cp(proof->lin_v, tau * D),
             lu = cp(proof->lin_u, (size_t)t * D), fsc = cp(proof->fold_sumcheck, (size_t)s * (2 * bs + 1) * D),
             th = cp(proof->theta_s, 2 * (size_t)K * tau * D), et = cp(proof->eta_s, 2 * (size_t)K * t * D);
  std::vector<uint64_t> us[2], vs[2], xs[2], ys[2];
  for (int side = 0; side < 2; side++) {
    us[side] = cp(proof->u_s[side], (size_t)K * t * D);
    vs[side] = cp(proof->v_s[side], (size_t)K * tau * D);
    xs[side] = cp(proof->x_s[side], (size_t)K * (l + 1) * D);
    ys[side] = cp(proof->y_s[side], (size_t)K * kappa * D);
  }
  // absorb_public_input (:162-184)
  T.label("acc");
  T.absorb(ar.data(), s);
  T.absorb(av.data(), tau);
  T.absorb(acm.data(), kappa);
  T.absorb(au.data(), t);
  T.absorb(axw.data(), l);
  T.absorb(ah.data(), 1);
  T.label("cm_i");
  T.absorb(cmi.data(), kappa);
  T.absorb(xc.data(), l);
  // collect_linearization_vars
  T.label("beta_s");
  for (int i = 0; i < s; i++) put(out->lin_beta, i, T.challenge());
  sumcheck(T, lsc.data(), s, degree + 1, zero(), out->lin_point, out->lin_claimed_sums, out->lin_subterms);
  memcpy(out->lin_expected, out->lin_claimed_sums + (size_t)s * D, D * 8);
  eq(out->lin_point, out->lin_beta, s, out->lin_eq_xy, out->lin_eq_factors, out->lin_eq_sub);
  Elem inner = zero();
  for (int i = 0; i < q; i++) {
    Elem prod = one();
    for (int k = S_off[i]; k < S_off[i + 1]; k++) prod = mul(prod, at(lu.data(), S_idx[k]));
    put(out->lin_products, i, prod);
    inner = add(inner, mul(at(c.data(), i), prod));
  }
  put(out->lin_inner, 0, inner);
  T.absorb(lv.data(), tau);
  T.absorb(lu.data(), t);
  // collect_decomposition_vars: the decomposed instances' messages
  for (int side = 0; side < 2; side++)
    for (int k = 0; k < K; k++) {
      T.absorb(xs[side].data() + (size_t)k * (l + 1) * D, l + 1);
      T.absorb(ys[side].data() + (size_t)k * kappa * D, kappa);
      T.absorb(us[side].data() + (size_t)k * t * D, t);
      T.absorb(vs[side].data() + (size_t)k * tau * D, tau);
    }
  // collect_folding_vars: squeeze_alpha_beta_zeta_mu (folding/utils.rs:51-96)
  T.label("alpha_s");
  for (int i = 0; i < 2 * K; i++) put(out->alpha, i, T.challenge());
  T.label("zeta_s");
  for (int i = 0; i < 2 * K; i++) put(out->zeta, i, T.challenge());
  T.label("mu_s");
  for (int i = 0; i < 2 * K - 1; i++) put(out->mu, i, T.challenge());
  put(out->mu, 2 * K - 1, one());
  T.label("beta_s");
  for (int i = 0; i < s; i++) put(out->beta, i, T.challenge());
  Elem g1 = zero(), g3 = zero();
  each(2 * K, [&](int i) {
    const int side = i / K, k = i % K;
    const uint64_t *v = vs[side].data() + (size_t)k * tau * D, *u = us[side].data() + (size_t)k * t * D;
    const Elem a = at(out->alpha, i), z = at(out->zeta, i);
    const Elem h1 = add(mul(a, at(v, 2)), at(v, 1));
    const Elem h2 = add(mul(a, h1), at(v, 0));
    const Elem ci = mul(a, h2);
    put(out->claim_g1_h1, i, h1);
    put(out->claim_g1_h2, i, h2);
    put(out->claim_g1_terms, i, ci);
    Elem h = add(mul(z, at(u, t - 1)), at(u, t - 2));
    size_t hk = (size_t)i * (t - 1);
    put(out->claim_g3_h, hk++, h);
    for (int j = t - 3; j >= 0; j--) {
      h = add(mul(z, h), at(u, j));
      put(out->claim_g3_h, hk++, h);
    }
    put(out->claim_g3_terms, i, mul(z, h));
  });
  for (int i = 0; i < 2 * K; i++) {
    g1 = add(g1, at(out->claim_g1_terms, i));
    g3 = add(g3, at(out->claim_g3_terms, i));
  }
  put(out->claim_g1, 0, g1);
  put(out->claim_g3, 0, g3);
  sumcheck(T, fsc.data(), s, 2 * bs, add(g1, g3), out->fold_point, out->fold_claimed_sums, out->fold_subterms);
  memcpy(out->fold_expected, out->fold_claimed_sums + (size_t)s * D, D * 8);
  // compute_sumcheck_claim_expected_value (folding/utils.rs:380-421)
  const Elem e_ast = eq(out->beta, out->fold_point, s, nullptr, nullptr, nullptr);
  Elem should = zero();
  std::vector<Elem> should_i(2 * K);
  each(2 * K, [&](int i) {
    const uint64_t *ri = i < K ? ar.data() : out->lin_point;
    const Elem e_i = eq(ri, out->fold_point, s, nullptr, nullptr, nullptr);
    const Elem a = at(out->alpha, i), z = at(out->zeta, i), mu = at(out->mu, i);
    Elem sa = zero(), norm = zero(), pa = a, pm = mu;
    for (int j = 0; j < tau; j++) {
      const Elem tj = at(th.data(), (size_t)i * tau + j);
      sa = add(sa, mul(pa, tj));
      pa = mul(pa, a);
      Elem prod = tj;
      for (int b = 1; b < bs; b++) prod = mul(prod, mul(sub(tj, fromu(b)), add(tj, fromu(b))));
      norm = add(norm, mul(pm, prod));
      pm = mul(pm, mu);
    }
    // zeta_i is a base-ring challenge in every slot, so its powers are one Fq3 chain
    Elem se = zero();
    uint64_t pz[3], z3[3] = {z[0], z[1], z[2]};
    memcpy(pz, z3, 24);
    for (int j = 0; j < t; j++) {
      se = add(se, mul(scal(pz), at(et.data(), (size_t)i * t + j)));
      uint64_t nx[3];
      f3mul(pz, z3, nx);
      memcpy(pz, nx, 24);
    }
    should_i[i] = add(add(mul(sa, e_i), mul(e_ast, norm)), mul(e_i, se));
  });
  for (int i = 0; i < 2 * K; i++) should = add(should, should_i[i]);
  put(out->should_equal_s, 0, should);
  for (int i = 0; i < 2 * K; i++) T.absorb(th.data() + (size_t)i * tau * D, tau);
  for (int i = 0; i < 2 * K; i++) T.absorb(et.data() + (size_t)i * t * D, t);
  // get_rhos (folding/utils.rs:116-127)
  T.label("rho_s");
  std::vector<uint64_t> rc(2 * (size_t)K * D, 0);
  if (lf_transcript_get_short_challenges(T.t, D, 2 * K - 1, rc.data()) != LF_OK) return LF_ERR_CHALLENGE_BYTES;
  rc[(size_t)(2 * K - 1) * D] = 1;
  memcpy(out->rho, rc.data(), rc.size() * 8);
  for (int i = 0; i < 2 * K; i++) ring::phi72_crt(out->rho + (size_t)i * D);
  // the rho-weighted products of the folded instance (:549-569)
  each(2 * K, [&](int i) {
    const int side = i / K, k = i % K;
    const Elem r = at(out->rho, i);
    for (size_t j = 0; j < kappa; j++)
      put(out->final_cm, (size_t)i * kappa + j, mul(at(ys[side].data() + (size_t)k * kappa * D, j), r));
    for (int j = 0; j < t; j++) put(out->final_u, (size_t)i * t + j, mul(at(et.data(), (size_t)i * t + j), r));
    for (size_t j = 0; j <= l; j++)
      put(out->final_x, (size_t)i * (l + 1) + j, mul(at(xs[side].data() + (size_t)k * (l + 1) * D, j), r));
  });
  const int pb = lf_transcript_playback_status(T.t);
  if (pb != LF_ERR_INVALID_ARG && pb != LF_OK) return pb;  // a playback must draw exactly the logged samples
  if (repr == LF_REPR_MONTGOMERY) {
    uint64_t *bufs[] = {out->lin_beta, out->lin_claimed_sums, out->lin_subterms, out->lin_point, out->lin_expected,
                        out->lin_inner, out->lin_products, out->lin_eq_xy, out->lin_eq_factors, out->lin_eq_sub,
                        out->alpha, out->beta, out->zeta, out->mu, out->claim_g1_h1, out->claim_g1_h2,
                        out->claim_g1_terms, out->claim_g1, out->claim_g3_h, out->claim_g3_terms, out->claim_g3,
                        out->fold_claimed_sums, out->fold_subterms, out->fold_point, out->fold_expected,
                        out->should_equal_s, out->rho, out->final_cm, out->final_u, out->final_x};
    const size_t lens[] = {(size_t)s, (size_t)s + 1, (size_t)s * (degree + 2), (size_t)s, 1, 1, (size_t)q,
                           (size_t)s, (size_t)s, (size_t)s + 1, 2 * (size_t)K, (size_t)s, 2 * (size_t)K,
                           2 * (size_t)K, 2 * (size_t)K, 2 * (size_t)K, 2 * (size_t)K, 1,
                           2 * (size_t)K * (t - 1), 2 * (size_t)K, 1, (size_t)s + 1, (size_t)s * (2 * bs + 1),
                           (size_t)s, 1, 1, 2 * (size_t)K, 2 * (size_t)K * kappa, 2 * (size_t)K * t,
                           2 * (size_t)K * (l + 1)};
    for (size_t b = 0; b < sizeof(lens) / sizeof(lens[0]); b++)
      for (size_t i = 0; i < lens[b] * D; i++) bufs[b][i] = gl::to_mont(bufs[b][i]);
  }
  return LF_OK;
}

// RotSum of the short challenges (coefficient form) with the flattened theta_i:
// v0[j][c] = sum_i sum_r theta_i[r][c] coeff_j(X^r rho_i) (rotation.rs:84-101), Phi_72
// (X^24 = X^12 - 1, X^36 = -1); the host twin of kernels.hip k_rot_lin
uint64_t rot_coeff(const uint64_t *a, int j, int r) {
  uint64_t v = j >= r ? a[j - r] : 0;
  if (j >= 12 && r > j - 12) v = gl::add(v, a[j + 12 - r]);
  if (j < 12 && r > j) v = gl::sub(v, a[j + 24 - r]);
  if (j < 12 && r > j + 12) v = gl::sub(v, a[j + 36 - r]);
  return v;
}

bool same(const uint64_t *a, const Elem &b) { return memcmp(a, b.data(), D * 8) == 0; }

}  // namespace

extern "C" {

int lf_fold_verify(const lf_ccs_desc *ccs, const lf_params *pr, const lf_lcccs *acc, const uint64_t *cm_i,
                   const uint64_t *x_ccs, const lf_lfproof_mut *proof, lf_lcccs_mut *out, int *failed, int repr) {
  if (failed) *failed = LF_VERIFY_OK;
  if (!ccs || !pr || !acc || !cm_i || !proof || !out) return LF_ERR_INVALID_ARG;
  if (pr->d != D || acc->d != D) return LF_ERR_UNSUPPORTED_RING;
  if (repr != LF_REPR_CANONICAL && repr != LF_REPR_MONTGOMERY) return LF_ERR_INVALID_ARG;
  const int t = ccs->t, q = ccs->q, degree = ccs->degree, K = pr->K, bs = (int)pr->b_small, tau = 3;
  const size_t m = ccs->m, l = ccs->l, kappa = acc->cm.n;
  int s = 0;
  while (m && ((size_t)1 << s) < m) s++;
  // the replay draws the challenges and forms every claim (generate_verification_witness_vars
  // computes exactly what NIFSVerifier::verify checks, nifs.rs:117-162)
  const size_t L1 = l + 1;
  std::vector<uint64_t> vb[30];
  const size_t lens[30] = {(size_t)s, (size_t)s + 1, (size_t)s * (degree + 2), (size_t)s, 1, 1, (size_t)q, (size_t)s,
                           (size_t)s, (size_t)s + 1, 2 * (size_t)K, (size_t)s, 2 * (size_t)K, 2 * (size_t)K,
                           2 * (size_t)K, 2 * (size_t)K, 2 * (size_t)K, 1, 2 * (size_t)K * (t > 1 ? t - 1 : 1),
                           2 * (size_t)K, 1, (size_t)s + 1, (size_t)s * (2 * bs + 1), (size_t)s, 1, 1, 2 * (size_t)K,
                           2 * (size_t)K * kappa, 2 * (size_t)K * t, 2 * (size_t)K * L1};
  for (int i = 0; i < 30; i++) vb[i].assign(lens[i] * D, 0);
  lf_replay_vars V;
  uint64_t **f = reinterpret_cast<uint64_t **>(&V);
  for (int i = 0; i < 30; i++) f[i] = vb[i].data();
  const int rc = replay(ccs, pr, acc, cm_i, x_ccs, proof, &V, repr, lf_transcript_new());
  if (rc != LF_OK) return rc;
  if (repr == LF_REPR_MONTGOMERY)
    for (auto &v : vb)
      for (auto &x : v) x = gl::from_mont(x);
  auto cp = [&](const uint64_t *p, size_t elems) {
    std::vector<uint64_t> v(p, p + elems);
    if (repr == LF_REPR_MONTGOMERY)
      for (auto &x : v) x = gl::from_mont(x);
    return v;
  };
  auto reject = [&](int what) {
    if (failed) *failed = what;
    return LF_ERR_VERIFICATION;
  };
  // sumcheck rounds (verifier.rs): p_i(0) + p_i(1) = the running claim
  auto rounds = [&](const std::vector<uint64_t> &msgs, int deg1, const uint64_t *claimed) {
    for (int i = 0; i < s; i++) {
      const uint64_t *p0 = msgs.data() + (size_t)i * deg1 * D;
      if (!same(claimed + (size_t)i * D, add(at(p0, 0), at(p0, 1)))) return false;
    }
    return true;
  };
  const auto lsc = cp(proof->lin_sumcheck, (size_t)s * (degree + 2) * D);
  if (!rounds(lsc, degree + 2, vb[1].data())) return reject(LF_VERIFY_LIN_SUMCHECK);
  // linearization.rs:265-285: e(r, beta) sum_i c_i prod_{j in S_i} u_j = the final claim
  if (!same(vb[4].data(), mul(at(vb[9].data(), s), at(vb[5].data(), 0)))) return reject(LF_VERIFY_LIN_CLAIM);
  // decomposition.rs:90-155: every decomposed vector recomposes (b^k weights) to its source
  const auto lv = cp(proof->lin_v, tau * D), lu = cp(proof->lin_u, (size_t)t * D);
  const auto acm = cp(acc->cm.elems, kappa * D), av = cp(acc->v.elems, tau * D), au = cp(acc->u.elems, (size_t)t * D),
             axw = cp(acc->x_w.elems, l * D), ah = cp(acc->h, D), cmi = cp(cm_i, kappa * D),
             xc = cp(x_ccs ? x_ccs : cm_i, x_ccs ? l * D : 0);
  std::vector<uint64_t> xh[2] = {axw, xc};
  xh[0].insert(xh[0].end(), ah.begin(), ah.end());
  const Elem onev = one();
  xh[1].insert(xh[1].end(), onev.begin(), onev.end());
  const std::vector<uint64_t> *src_cm[2] = {&acm, &cmi}, *src_v[2] = {&av, &lv}, *src_u[2] = {&au, &lu};
  for (int side = 0; side < 2; side++) {
    const auto ys = cp(proof->y_s[side], (size_t)K * kappa * D), vs = cp(proof->v_s[side], (size_t)K * tau * D),
               us = cp(proof->u_s[side], (size_t)K * t * D), xs = cp(proof->x_s[side], (size_t)K * L1 * D);
    struct Chk {
      const std::vector<uint64_t> &parts, &want;
      size_t n;
      int code;
    } chks[4] = {{ys, *src_cm[side], kappa, LF_VERIFY_DEC_Y}, {vs, *src_v[side], (size_t)tau, LF_VERIFY_DEC_V},
                 {us, *src_u[side], (size_t)t, LF_VERIFY_DEC_U}, {xs, xh[side], L1, LF_VERIFY_DEC_X}};
    for (const Chk &c : chks)
      for (size_t j = 0; j < c.n; j++) {
        Elem acc_e = zero();
        uint64_t bk = 1;
        for (int k = 0; k < K; k++) {
          acc_e = add(acc_e, mul(at(c.parts.data(), (size_t)k * c.n + j), fromu(bk)));
          bk = gl::mul(bk, pr->b_small % gl::P);
        }
        if (!same(c.want.data() + j * D, acc_e)) return reject(c.code);
      }
  }
  // folding.rs:133-200: the rounds from sum_i (alpha_i powers . v_i + zeta_i powers . u_i)
  // (the replay's claim_g1 + claim_g3), then the expected evaluation
  const auto fsc = cp(proof->fold_sumcheck, (size_t)s * (2 * bs + 1) * D);
  if (!rounds(fsc, 2 * bs + 1, vb[21].data())) return reject(LF_VERIFY_FOLD_SUMCHECK);
  if (!same(vb[24].data(), at(vb[25].data(), 0))) return reject(LF_VERIFY_FOLD_CLAIM);
  // the folded instance (compute_v0_u0_x0_cm_0, folding/utils.rs:456-517; prepare_public_output)
  std::vector<uint64_t> cm0(kappa * D, 0), u0((size_t)t * D, 0), x0(L1 * D, 0), v0(tau * D, 0);
  for (int i = 0; i < 2 * K; i++) {
    for (size_t j = 0; j < kappa; j++) put(cm0.data(), j, add(at(cm0.data(), j), at(vb[27].data(), (size_t)i * kappa + j)));
    for (int j = 0; j < t; j++) put(u0.data(), j, add(at(u0.data(), j), at(vb[28].data(), (size_t)i * t + j)));
    for (size_t j = 0; j < L1; j++) put(x0.data(), j, add(at(x0.data(), j), at(vb[29].data(), (size_t)i * L1 + j)));
  }
  const auto th = cp(proof->theta_s, 2 * (size_t)K * tau * D);
  for (int i = 0; i < 2 * K; i++) {
    uint64_t rc_i[D];
    memcpy(rc_i, vb[26].data() + (size_t)i * D, D * 8);
    ring::phi72_icrt(rc_i);  // rho_i in coefficient form
    const uint64_t *ti = th.data() + (size_t)i * tau * D;  // theta_i flattened: 24 Fq3 values
    for (int j = 0; j < D; j++)
      for (int c = 0; c < 3; c++) {
        uint64_t acc_v = v0[(size_t)j * 3 + c];
        for (int r = 0; r < D; r++) acc_v = gl::add(acc_v, gl::mul(ti[(size_t)r * 3 + c], rot_coeff(rc_i, j, r)));
        v0[(size_t)j * 3 + c] = acc_v;
      }
  }
  auto emit = [&](uint64_t *dst, const uint64_t *src, size_t elems) {
    for (size_t i = 0; i < elems; i++) dst[i] = repr == LF_REPR_MONTGOMERY ? gl::to_mont(src[i]) : src[i];
  };
  emit(out->r, vb[23].data(), (size_t)s * D);
  emit(out->v, v0.data(), tau * D);
  emit(out->cm, cm0.data(), kappa * D);
  emit(out->u, u0.data(), (size_t)t * D);
  if (l) emit(out->x_w, x0.data(), l * D);
  emit(out->h, x0.data() + l * D, D);
  return LF_OK;
}

int lf_fold_replay(const lf_ccs_desc *ccs, const lf_params *pr, const lf_lcccs *acc, const uint64_t *cm_i,
                   const uint64_t *x_ccs, const lf_lfproof_mut *proof, lf_replay_vars *out, int repr) {
  return replay(ccs, pr, acc, cm_i, x_ccs, proof, out, repr, lf_transcript_new());
}

int lf_fold_replay_samples(const lf_ccs_desc *ccs, const lf_params *pr, const lf_lcccs *acc, const uint64_t *cm_i,
                           const uint64_t *x_ccs, const lf_lfproof_mut *proof, const uint64_t *samples, size_t nsamples,
                           lf_replay_vars *out, int repr) {
  if (!samples && nsamples) return LF_ERR_INVALID_ARG;
  return replay(ccs, pr, acc, cm_i, x_ccs, proof, out, repr, lf_transcript_new_playback(samples, nsamples));
}

}  // extern "C"
