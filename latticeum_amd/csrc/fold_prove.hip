// fold_prove.hip -- the zkvm's fold() as one call: zk_latticefold_prove
// (zkvm/src/zk_latticefold.rs:37-102) with a fresh Poseidon2 transcript
// (zkvm/src/main.rs:394), in the reference's exact transcript order:
//   sanity_check; absorb_public_input (:152-184);
//   LFLinearizationProver::prove (latticefold/src/nifs/linearization.rs:153-197);
//   LFDecompositionProver::prove of (acc, w_acc), then of the linearized
//     (cm_i, w_i) (nifs/decomposition.rs:33-88);
//   LFFoldingProver::prove (nifs/folding.rs:42-130).
// This is host code above the C ABI, the way a Rust fold() would drive it: every
// heavy step is an lf_dev_* call on the context's stream (the decomposition and
// commitments, the Mz products, both sumchecks, the MLE evaluations, the fold),
// the transcript stays on the host, and only the protocol's messages -- a few
// hundred ring elements -- cross PCIe. The witnesses stay in HBM.
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/lf.h"
#include "gl.hpp"
#include "kernels.hpp"

struct lf_prover {
  lf_ctx *ctx = nullptr;
  const lf_ajtai *aj = nullptr;
  const lf_ccs *ccs = nullptr;
  lf_params pr{};
  int device = 0;
  // shape
  int d = 0, tb = 1, tau = 1, s = 0, K = 0, t = 0, q = 0, degree = 0, nm_lin = 0, nm_fold = 0;
  size_t W = 0, N = 0, n = 0, nn = 0, l = 0, kappa = 0;
  std::vector<uint64_t> c;  // q NTT elements
  std::vector<int> S_off, S_idx;
  std::vector<int> lin_list;  // the matrix of every linearization MLE (c_i != 0, j in S_i)
  // the Mz MLEs are materialised live matrices first (mz_order: the matrices read by the
  // linearization's combination, then the others); S_live: each multiset entry's
  // position among the nlive live ones; bad_S: a multiset index past the MLE list
  std::vector<int> mz_order, S_live;
  int nlive = 0;
  bool bad_S = false;
  // the linearization's round-0 points per multiset: b is active for S_i when every
  // factor's matrix has an entry in row 2b or 2b + 1 (lf_sumcheck_prove_lin_sparse);
  // act_off [q + 1] into the device list act
  std::vector<uint32_t> act_off, act_host;
  uint32_t *act = nullptr;
  // device memory: one allocation, carved
  uint64_t *mem = nullptr;
  uint64_t *z = nullptr, *mz = nullptr, *lin = nullptr, *pt = nullptr, *beta = nullptr, *val = nullptr;
  uint64_t *fkc[2] = {}, *fk[2] = {}, *wk[2] = {}, *y[2] = {}, *cmd[2] = {}, *xw[2] = {}, *xs = nullptr;
  uint64_t *zdec[2] = {}, *vs = nullptr, *us = nullptr, *fold = nullptr, *coef[2] = {}, *zeta = nullptr, *mu = nullptr;
  uint64_t *theta = nullptr, *eta = nullptr, *rho = nullptr, *rhoc = nullptr, *cm0 = nullptr, *u0 = nullptr, *x0 = nullptr,
           *v0 = nullptr, *r0 = nullptr;
  // eq(r_0) and one point's Mz weights M_j^T eq (shared by the sides evaluated there)
  uint64_t *eq0 = nullptr, *mzw = nullptr;
  uint64_t *lev = nullptr;  // the live Mz MLEs at r_lin (the linearization sumcheck's final values)
  std::string err;
  // every value the last lf_fold_prove sampled from its transcript, in order
  // (lf_fold_prove_vars replays the proof on them instead of a second sponge)
  std::vector<uint64_t> samples;
  // tracing spans (the reference's #[instrument] spans, zkvm/src/main.rs:56-63):
  // wall ms of each fold() phase, measured with a stream sync at its end
  bool timing = false;
  double span_ms[LF_SPAN_COUNT] = {};
  // pinned host staging: the messages the host absorbs come back through it with
  // asynchronous copies (so the device keeps working while the host hashes), and
  // the points the device needs go out through it
  uint64_t *pin = nullptr;
  uint64_t *hx[2] = {}, *hy[2] = {}, *hu[2] = {}, *hv[2] = {}, *hr[2] = {}, *htheta = nullptr, *heta = nullptr;
  // ev[0], ev[1]: per-side / theta readiness; ev[2 + g]: instance group g's messages
  hipEvent_t ev[2 + 2 * 16] = {};
  ~lf_prover() {
    int prev = -1;
    if (hipGetDevice(&prev) == hipSuccess && prev != device) (void)hipSetDevice(device);
    if (mem) (void)hipFree(mem);
    if (pin) (void)hipHostFree(pin);
    for (auto &e : ev)
      if (e) (void)hipEventDestroy(e);
    if (prev >= 0 && prev != device) (void)hipSetDevice(prev);
  }
};

namespace {

// instances per u_s / eta_s launch (and per host wait): two fill the chip with
// t blocks each, and the host starts absorbing after the first group
constexpr int MZ_GROUP = 2;

// the Fq3 = Fq[u]/(u^3 - 2^40) product of two base-ring elements (tb = 3), or the Fq one
void base_mul(const uint64_t *a, const uint64_t *b, uint64_t *o, int tb) {
  if (tb == 1) {
    o[0] = gl::mul(a[0], b[0]);
    return;
  }
  const uint64_t nr = 1ull << 40;
  const uint64_t c0 = gl::add(gl::mul(a[0], b[0]), gl::mul(nr, gl::add(gl::mul(a[1], b[2]), gl::mul(a[2], b[1]))));
  const uint64_t c1 = gl::add(gl::add(gl::mul(a[0], b[1]), gl::mul(a[1], b[0])), gl::mul(nr, gl::mul(a[2], b[2])));
  const uint64_t c2 = gl::add(gl::add(gl::mul(a[0], b[2]), gl::mul(a[1], b[1])), gl::mul(a[2], b[0]));
  o[0] = c0;
  o[1] = c1;
  o[2] = c2;
}

// From<BaseRing> = from_scalar: the base-ring element in every NTT slot
void broadcast(const uint64_t *base, int tb, int d, uint64_t *out) {
  for (int i = 0; i < d; i++) out[i] = base[i % tb];
}

struct Run {
  lf_prover *P;
  lf_transcript *T;
  hipStream_t st;
  int rc = LF_OK;
  std::string *err = nullptr;  // where this Run records its first error (default P->err)
  std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
  std::string &errs() { return err ? *err : P->err; }

  // close the span that ran since the last mark (only with timing on); sync = false
  // where the device work of the span overlaps the next span's host work (the
  // span then ends when its work is enqueued, and the wait lands in the next one)
  void mark(int span, bool sync = true) {
    if (!P->timing) return;
    if (sync) (void)hipStreamSynchronize(st);
    const auto now = std::chrono::steady_clock::now();
    P->span_ms[span] += std::chrono::duration<double, std::milli>(now - t0).count();
    t0 = now;
  }

  int check(int r, const char *what) {
    if (r != LF_OK && rc == LF_OK) {
      rc = r;
      errs() = std::string(what) + ": " + lf_ctx_last_error(P->ctx);
    }
    return r;
  }
  int hip(hipError_t e, const char *what) {
    if (e != hipSuccess && rc == LF_OK) {
      rc = e == hipErrorOutOfMemory ? LF_ERR_OUT_OF_MEMORY : LF_ERR_DEVICE;
      errs() = std::string(what) + ": " + hipGetErrorString(e);
    }
    return rc;
  }
  int h2d(uint64_t *dst, const uint64_t *src, size_t elems) {
    return elems ? hip(hipMemcpyAsync(dst, src, elems * 8, hipMemcpyHostToDevice, st), "upload") : rc;
  }
  int d2h(uint64_t *dst, const uint64_t *src, size_t elems) {
    if (!elems) return rc;
    hip(hipMemcpyAsync(dst, src, elems * 8, hipMemcpyDeviceToHost, st), "download");
    return hip(hipStreamSynchronize(st), "sync");
  }
  int d2d(uint64_t *dst, const uint64_t *src, size_t elems) {
    return elems ? hip(hipMemcpyAsync(dst, src, elems * 8, hipMemcpyDeviceToDevice, st), "copy") : rc;
  }
  // device -> pinned host, asynchronous (completion: an event recorded after it)
  int d2p(uint64_t *dst, const uint64_t *src, size_t elems) {
    return elems ? hip(hipMemcpyAsync(dst, src, elems * 8, hipMemcpyDeviceToHost, st), "download") : rc;
  }
  // host -> device through a pinned copy of the source (no stream synchronisation)
  int h2p2d(uint64_t *dst, uint64_t *pinned, const uint64_t *src, size_t elems) {
    if (!elems) return rc;
    memcpy(pinned, src, elems * 8);
    return hip(hipMemcpyAsync(dst, pinned, elems * 8, hipMemcpyHostToDevice, st), "upload");
  }
  int wait(hipEvent_t e) { return hip(hipEventSynchronize(e), "event wait"); }
  void absorb(const uint64_t *e, size_t n) { lf_transcript_absorb_ring(T, e, n, P->d, LF_REPR_CANONICAL); }
  // absorb_field_element(BaseRing::from_base_prime_field(from_be_bytes_mod_order(label)))
  void absorb_label(const char *label) {
    uint64_t v = 0;
    for (const char *p = label; *p; p++) v = gl::add(gl::mul(v, 256), (uint8_t)*p);
    std::vector<uint64_t> e(P->d, 0);
    for (int i = 0; i < P->d; i += P->tb) e[i] = v;
    absorb(e.data(), 1);
  }
  // get_challenge (fiat_shamir.rs:69-86): three samples re-observed for Fq3;
  // one sample re-observed for Fq (this project's convention for X^d + 1)
  void challenge(uint64_t *out) {
    if (P->tb == 3) {
      lf_transcript_get_challenge(T, out);
    } else {
      out[0] = lf_transcript_sample(T);
      lf_transcript_observe(T, out[0]);
    }
  }
  // get_challenges(n) mapped into NTT elements: [n][d]
  std::vector<uint64_t> challenges(size_t n) {
    std::vector<uint64_t> out(n * P->d);
    uint64_t b[3];
    for (size_t i = 0; i < n; i++) {
      challenge(b);
      broadcast(b, P->tb, P->d, out.data() + i * P->d);
    }
    return out;
  }
};

// z = x_ccs || 1 || w_ccs (Instance::get_z_vector) and its Mz MLEs: independent of the
// transcript, so enqueued before the public input is absorbed (the device computes
// them while the host hashes). Live matrices first (lf_prover::mz_order).
int linearize_prepare(lf_prover *P, Run &R, const std::vector<uint64_t> &xc, const lf_witness *w_i) {
  lf_ctx *C = P->ctx;
  const int d = P->d, tb = P->tb;
  const size_t W = P->W, l = P->l;
  if (P->bad_S) {
    P->err = "multiset index past the MLE list";
    return R.rc = LF_ERR_INVALID_ARG;
  }
  std::vector<uint64_t> one(d, 0);
  for (int i = 0; i < d; i += tb) one[i] = 1;
  R.h2d(P->z, xc.data(), l * d);
  R.h2d(P->z + l * d, one.data(), d);
  R.d2d(P->z + (l + 1) * d, w_i->w_ccs, W * d);
  return R.check(lf_dev_mz_mles_sel(C, P->ccs, P->z, P->mz_order.data(), P->t, P->s, P->mz), "Mz MLEs");
}

// LFLinearizationProver::prove (linearization.rs:153-197) of the CCCS (cm, x_ccs)
// with witness w (its Mz MLEs from linearize_prepare), on the transcript R.T: the
// sumcheck messages into lin_sumcheck (host), and r, v, u of the linearized instance
// {r, v, cm, u, x_ccs, ONE}
int linearize(lf_prover *P, Run &R, const lf_witness *w_i, uint64_t *lin_sumcheck, std::vector<uint64_t> &r_lin,
              std::vector<uint64_t> &lv, std::vector<uint64_t> &lu) {
  lf_ctx *C = P->ctx;
  const int d = P->d, tb = P->tb, tau = P->tau, s = P->s, t = P->t, nlive = P->nlive;
  const size_t N = P->N, nn = P->nn, len = nn * d;
  R.absorb_label("beta_s");  // squeeze_beta_challenges (linearization/utils.rs:111-124)
  const std::vector<uint64_t> beta = R.challenges(s);
  // The MLE list is [MLE(M_j z) for each (i, j in S_i) with c_i != 0] + [eq(beta)]
  // (linearization/utils.rs:71-84), and the combination reads list position j for
  // matrix index j (as the reference does) and the last entry -- so only the live
  // matrices' MLEs are read, each where the Mz products left it (a pointer table;
  // no copies), and eq(beta) is split off each round (lf_sumcheck_prove_lin: beta
  // itself, no eq MLE); P->lin (nlive x m/4 elements) serves the later rounds.
  std::vector<const uint64_t *> ptr(nlive);
  for (int i = 0; i < nlive; i++) ptr[i] = P->mz + (size_t)i * len;
  std::vector<uint64_t> rnd((size_t)s * tb);
  {
    lf_comb cb{};
    cb.kind = LF_COMB_LINEARIZATION;
    cb.q = P->q;
    cb.c = lf_ccs_c_device(P->ccs);
    cb.S_off = P->S_off.data();
    cb.S_idx = P->S_live.data();
    if (R.rc == LF_OK)
      R.check(lf_sumcheck_prove_lin_sparse(C, R.T, &cb, ptr.data(), nlive, s, d, P->degree + 1, beta.data(), P->act,
                                           P->act_off.data(), P->lin, lin_sumcheck, rnd.data(), P->lev),
              "linearization sumcheck");
  }
  if (R.rc) return R.rc;
  r_lin.assign((size_t)s * d, 0);
  for (int i = 0; i < s; i++) broadcast(rnd.data() + (size_t)i * tb, tb, d, r_lin.data() + (size_t)i * d);
  R.h2d(P->pt, r_lin.data(), (size_t)s * d);
  // v = f_hat(w_i) at r, u = MLE(M_j z)(r) (compute_evaluation_vectors, :130-147): the
  // live matrices' u are the sumcheck's final values, the others are evaluated against
  // one eq(r) table -- built where the folding prover's eq(r_1) MLE lives, which it is
  uint64_t *eq_lin = P->fold + 2 * nn * d;
  R.check(lf_dev_eq_table(C, d, P->pt, s, eq_lin), "eq(r)");
  R.check(lf_dev_fhat_evaluate_eq(C, d, w_i->f_coeff, N, 0, 1, s, eq_lin, P->val), "v");
  if (t > nlive)
    R.check(lf_dev_mle_evaluate_eq(C, d, P->mz + (size_t)nlive * len, t - nlive, s, eq_lin, P->val + (size_t)tau * d),
            "u");
  lv.assign((size_t)tau * d, 0);
  std::vector<uint64_t> ub((size_t)t * d);
  R.d2h(lv.data(), P->val, (size_t)tau * d);
  R.d2h(ub.data(), P->val + (size_t)tau * d, (size_t)(t - nlive) * d);
  R.d2h(ub.data() + (size_t)(t - nlive) * d, P->lev, (size_t)nlive * d);
  if (R.rc) return R.rc;
  lu.assign((size_t)t * d, 0);
  for (int i = 0; i < t; i++) {  // position i of mz_order is matrix mz_order[i]
    const uint64_t *src = i < nlive ? ub.data() + (size_t)(t - nlive + i) * d : ub.data() + (size_t)(i - nlive) * d;
    memcpy(lu.data() + (size_t)P->mz_order[i] * d, src, d * 8);
  }
  R.absorb(lv.data(), tau);
  R.absorb(lu.data(), t);
  return LF_OK;
}

int bad(lf_prover *P, int code, const char *msg) {
  P->err = msg;
  return code;
}

}  // namespace

extern "C" {

int lf_prover_create(lf_ctx *ctx, const lf_ajtai *aj, const lf_params *pr, const lf_ccs *ccs, lf_prover **out) {
  if (!ctx || !aj || !pr || !ccs || !out) return LF_ERR_INVALID_ARG;
  *out = nullptr;
  auto P = new lf_prover;
  P->ctx = ctx;
  P->aj = aj;
  P->ccs = ccs;
  P->pr = *pr;
  P->device = lf_ctx_device(ctx);
  const int d = pr->d;
  size_t m = 0, n = 0, l = 0;
  int t = 0, q = 0, degree = 0;
  if (lf_ccs_shape(ccs, &t, &m, &n, &l, &q, &degree) != LF_OK || q < 1) {
    delete P;
    return LF_ERR_INVALID_ARG;  // lf_ccs_set_structure first
  }
  if (lf_ajtai_d(aj) != d || (m & (m - 1)) || m < 2 || pr->b_small < 2 || pr->K < 1 || pr->K > 16 || pr->L < 1 ||
      n < l + 2) {
    delete P;
    return LF_ERR_INVALID_ARG;
  }
  P->d = d;
  P->tb = d == 24 ? 3 : 1;
  P->tau = d == 24 ? 3 : 1;
  P->K = pr->K;
  P->t = t;
  P->q = q;
  P->degree = degree;
  P->n = n;
  P->l = l;
  P->W = n - l - 1;
  P->N = P->W * (size_t)pr->L;
  P->nn = m;
  while (((size_t)1 << P->s) < m) P->s++;
  P->kappa = lf_ajtai_kappa(aj);
  // sanity_check (zk_latticefold.rs:152-158): m = max((n - l - 1) L, m).next_power_of_two();
  // Witness::get_fhat gives MLEs of log2(N.next_power_of_two()) variables, which the
  // sumchecks over s = log2 m variables need to be s as well
  size_t want = std::max(P->N, m), pw = 1;
  while (pw < want) pw <<= 1;
  size_t npw = 1;
  while (npw < P->N) npw <<= 1;
  if (pw != m || npw != m || lf_ajtai_width(aj) != P->N) {
    delete P;
    return LF_ERR_INVALID_ARG;  // CSError::InvalidSizeBounds / a witness of another width
  }
  P->c.resize((size_t)q * d);
  P->S_off.resize(q + 1);
  lf_ccs_get_structure(ccs, P->c.data(), P->S_off.data(), nullptr);
  P->S_idx.resize(P->S_off[q]);
  lf_ccs_get_structure(ccs, nullptr, nullptr, P->S_idx.data());
  for (int i = 0; i < q; i++) {
    bool zero = true;
    for (int k = 0; k < d; k++) zero &= P->c[(size_t)i * d + k] == 0;
    if (zero) continue;  // prepare_lin_sumcheck_polynomial skips c_i = 0 (linearization/utils.rs:71-84)
    for (int k = P->S_off[i]; k < P->S_off[i + 1]; k++) P->lin_list.push_back(P->S_idx[k]);
  }
  P->nm_lin = (int)P->lin_list.size() + 1;
  {
    std::vector<int> pos_of(t, -1);
    P->S_live.resize(P->S_idx.size());
    for (size_t k = 0; k < P->S_idx.size(); k++) {
      const int p = P->S_idx[k];
      if (p < 0 || (size_t)p > P->lin_list.size()) {
        // past the eq(beta) slot or negative: malformed, the reference would panic on the index
        delete P;
        lf_ctx_set_error(ctx, "lf_prover_create: a multiset index is negative or past the Mz MLE list and its "
                              "eq(beta) slot");
        return LF_ERR_INVALID_ARG;
      }
      if ((size_t)p == P->lin_list.size()) {
        P->bad_S = true;
        P->S_live[k] = 0;
        continue;
      }
      const int j = P->lin_list[p];
      if (pos_of[j] < 0) {
        pos_of[j] = (int)P->mz_order.size();
        P->mz_order.push_back(j);
      }
      P->S_live[k] = pos_of[j];
    }
    P->nlive = (int)P->mz_order.size();
    for (int j = 0; j < t; j++)
      if (pos_of[j] < 0) P->mz_order.push_back(j);
  }
  if (P->bad_S) {
    // The reference's list position lin_list.size() is the eq(beta) MLE itself
    // (linearization/utils.rs:71-84): a multiset naming it would put a second eq
    // factor into its term, which the split-eq sumcheck (eq(beta) taken out of every
    // term) does not express. Rejected here, by name, rather than mid-fold.
    delete P;
    lf_ctx_set_error(ctx, "lf_prover_create: a multiset index is the position of eq(beta) in the MLE list; "
                          "multisets over eq(beta) are not supported");
    return LF_ERR_UNSUPPORTED_CCS;
  }
  if (!P->bad_S) {
    const size_t half = m / 2;
    std::vector<uint8_t> row(m);
    std::vector<std::vector<uint8_t>> pair(P->nlive, std::vector<uint8_t>(half));
    for (int i = 0; i < P->nlive; i++) {
      lf_ccs_row_live(ccs, P->mz_order[i], row.data());
      for (size_t b = 0; b < half; b++) pair[i][b] = row[2 * b] | row[2 * b + 1];
    }
    P->act_off.assign(q + 1, 0);
    for (int i = 0; i < q; i++) {
      bool zero = true;  // c_i = 0: no active point
      for (int k = 0; k < d; k++) zero &= P->c[(size_t)i * d + k] == 0;
      if (!zero)
        for (size_t b = 0; b < half; b++) {
          bool on = true;
          for (int k = P->S_off[i]; k < P->S_off[i + 1] && on; k++) on = pair[P->S_live[k]][b];
          if (on) P->act_host.push_back((uint32_t)b);
        }
      P->act_off[i + 1] = (uint32_t)P->act_host.size();
    }
  }
  P->nm_fold = 5 + 2 * P->K * P->tau;
  // device memory, carved from one allocation
  const size_t K = P->K, N = P->N, W = P->W, nn = P->nn, kd = P->kappa * d, tau = P->tau;
  struct Part {
    uint64_t **p;
    size_t elems;
  };
  std::vector<Part> parts = {
      {&P->z, n * d}, {&P->mz, (size_t)t * nn * d}, {&P->lin, (size_t)std::max(P->nlive, 1) * std::max<size_t>(nn / 4, 1) * d},
      {&P->pt, (size_t)P->s * d}, {&P->beta, (size_t)P->s * d}, {&P->val, (size_t)(t + 3) * d},
      {&P->fkc[0], K * N * d}, {&P->fkc[1], K * N * d}, {&P->fk[0], K * N * d}, {&P->fk[1], K * N * d},
      {&P->wk[0], K * W * d}, {&P->wk[1], K * W * d}, {&P->y[0], K * kd}, {&P->y[1], K * kd},
      {&P->cmd[0], kd}, {&P->cmd[1], kd}, {&P->xw[0], (l + 1) * d}, {&P->xw[1], (l + 1) * d},
      {&P->xs, 2 * K * (l + 1) * d}, {&P->zdec[0], K * n * d}, {&P->zdec[1], K * n * d},
      {&P->vs, 2 * K * tau * d}, {&P->us, 2 * K * t * d}, {&P->fold, (size_t)P->nm_fold * nn * d},
      {&P->coef[0], K * tau * d}, {&P->coef[1], K * tau * d}, {&P->zeta, 2 * K * d}, {&P->mu, 2 * K * d},
      {&P->theta, 2 * K * tau * d}, {&P->eta, 2 * K * t * d}, {&P->rho, 2 * K * d}, {&P->rhoc, 2 * K * d},
      {&P->cm0, kd}, {&P->u0, (size_t)t * d}, {&P->x0, (l + 1) * d}, {&P->v0, tau * d}, {&P->r0, (size_t)P->s * d},
      {&P->eq0, nn * d}, {&P->mzw, lf_ccs_weights_len(ccs)}, {&P->lev, (size_t)t * d},
      {reinterpret_cast<uint64_t **>(&P->act), (P->act_host.size() + 1) / 2}};
  size_t total = 0;
  for (auto &x : parts) total += (x.elems + 31) / 32 * 32;  // 256-B aligned parts
  int prev = -1;
  if (hipGetDevice(&prev) == hipSuccess && prev != P->device) (void)hipSetDevice(P->device);
  hipError_t e = hipMalloc(&P->mem, total * 8);
  if (prev >= 0 && prev != P->device) (void)hipSetDevice(prev);
  if (e != hipSuccess) {
    P->mem = nullptr;
    delete P;
    return e == hipErrorOutOfMemory ? LF_ERR_OUT_OF_MEMORY : LF_ERR_DEVICE;
  }
  size_t off = 0;
  for (auto &x : parts) {
    *x.p = P->mem + off;
    off += (x.elems + 31) / 32 * 32;
  }
  if (!P->act_host.empty()) {
    if (hipGetDevice(&prev) == hipSuccess && prev != P->device) (void)hipSetDevice(P->device);
    e = hipMemcpy(P->act, P->act_host.data(), P->act_host.size() * 4, hipMemcpyHostToDevice);
    if (prev >= 0 && prev != P->device) (void)hipSetDevice(prev);
    if (e != hipSuccess) {
      delete P;
      return LF_ERR_DEVICE;
    }
    P->act_host = std::vector<uint32_t>();
  }
  std::vector<Part> pins = {
      {&P->hx[0], K * (l + 1) * d}, {&P->hx[1], K * (l + 1) * d}, {&P->hy[0], K * kd}, {&P->hy[1], K * kd},
      {&P->hu[0], K * t * d}, {&P->hu[1], K * t * d}, {&P->hv[0], K * tau * d}, {&P->hv[1], K * tau * d},
      {&P->hr[0], (size_t)P->s * d}, {&P->hr[1], (size_t)P->s * d}, {&P->htheta, 2 * K * tau * d},
      {&P->heta, 2 * K * t * d}};
  size_t ptotal = 0;
  for (auto &x : pins) ptotal += (x.elems + 7) / 8 * 8;
  if (hipGetDevice(&prev) == hipSuccess && prev != P->device) (void)hipSetDevice(P->device);
  e = hipHostMalloc(reinterpret_cast<void **>(&P->pin), ptotal * 8, hipHostMallocDefault);
  for (auto &ev : P->ev)
    if (e == hipSuccess) e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  if (prev >= 0 && prev != P->device) (void)hipSetDevice(prev);
  if (e != hipSuccess) {
    delete P;
    return e == hipErrorOutOfMemory ? LF_ERR_OUT_OF_MEMORY : LF_ERR_DEVICE;
  }
  off = 0;
  for (auto &x : pins) {
    *x.p = P->pin + off;
    off += (x.elems + 7) / 8 * 8;
  }
  *out = P;
  return LF_OK;
}

void lf_prover_destroy(lf_prover *P) { delete P; }

int lf_linearize(lf_prover *P, const uint64_t *cm, const uint64_t *x_ccs, const lf_witness *w, lf_lcccs_mut *out,
                 uint64_t *lin_sumcheck, int repr) {
  if (!P || !cm || (!x_ccs && P->l) || !w || !w->w_ccs || !w->f_coeff || !out || !lin_sumcheck || !out->r || !out->v ||
      !out->cm || !out->u || (P->l && !out->x_w) || !out->h)
    return LF_ERR_INVALID_ARG;
  if (repr != LF_REPR_CANONICAL && repr != LF_REPR_MONTGOMERY) return bad(P, LF_ERR_INVALID_ARG, "repr");
  const int d = P->d, s = P->s, tau = P->tau, t = P->t;
  const size_t l = P->l, kd = P->kappa * d;
  std::vector<uint64_t> cmv(cm, cm + kd), xc(x_ccs ? x_ccs : cm, x_ccs ? x_ccs + l * d : cm);
  if (repr == LF_REPR_MONTGOMERY) {
    for (auto &x : cmv) x = gl::from_mont(x);
    for (auto &x : xc) x = gl::from_mont(x);
  }
  Run R{P, lf_transcript_new(), (hipStream_t)lf_ctx_get_stream(P->ctx)};
  struct TGuard {
    lf_transcript *t;
    ~TGuard() { lf_transcript_free(t); }
  } tg{R.T};
  std::vector<uint64_t> r_lin, lv, lu;
  if (linearize_prepare(P, R, xc, w) || linearize(P, R, w, lin_sumcheck, r_lin, lv, lu)) return R.rc;
  // the LCCCS {r, v, cm, u, x_w = x_ccs, h = ONE} (linearization.rs:185-193)
  memcpy(out->r, r_lin.data(), r_lin.size() * 8);
  memcpy(out->v, lv.data(), lv.size() * 8);
  memcpy(out->cm, cmv.data(), kd * 8);
  memcpy(out->u, lu.data(), lu.size() * 8);
  if (l) memcpy(out->x_w, xc.data(), l * d * 8);
  for (int i = 0; i < d; i++) out->h[i] = i % P->tb == 0 ? 1 : 0;
  if (repr == LF_REPR_MONTGOMERY) {
    auto mont = [](uint64_t *p, size_t elems) {
      for (size_t i = 0; i < elems; i++) p[i] = gl::to_mont(p[i]);
    };
    mont(out->r, (size_t)s * d);
    mont(out->v, (size_t)tau * d);
    mont(out->cm, kd);
    mont(out->u, (size_t)t * d);
    mont(out->x_w, l * d);
    mont(out->h, d);
    mont(lin_sumcheck, (size_t)s * (P->degree + 2) * d);
  }
  return LF_OK;
}

const char *lf_prover_last_error(const lf_prover *P) { return P ? P->err.c_str() : ""; }

int lf_prover_timing(lf_prover *P, int enable, double *span_ms) {
  if (!P) return LF_ERR_INVALID_ARG;
  if (span_ms) memcpy(span_ms, P->span_ms, sizeof(P->span_ms));
  P->timing = enable != 0;
  memset(P->span_ms, 0, sizeof(P->span_ms));
  return LF_OK;
}

int lf_fold_prove(lf_prover *P, const lf_lcccs *acc, const lf_witness *w_acc, const uint64_t *cm_i,
                  const uint64_t *x_ccs, const lf_witness *w_i, lf_lcccs_mut *out, const lf_witness *w_out,
                  lf_lfproof_mut *proof, int repr) {
  if (!P || !acc || !w_acc || !cm_i || (!x_ccs && P->l) || !w_i || !out || !w_out || !proof) return LF_ERR_INVALID_ARG;
  if (repr != LF_REPR_CANONICAL && repr != LF_REPR_MONTGOMERY) return bad(P, LF_ERR_INVALID_ARG, "repr");
  const int d = P->d, tb = P->tb, tau = P->tau, s = P->s, K = P->K, t = P->t;
  const size_t N = P->N, W = P->W, n = P->n, nn = P->nn, l = P->l, kappa = P->kappa, kd = kappa * d;
  const size_t ND = N * d;
  if (acc->d != d || acc->r.n != (size_t)s || acc->v.n != (size_t)tau || acc->cm.n != kappa || acc->u.n != (size_t)t ||
      acc->x_w.n != l || !acc->h)
    return bad(P, LF_ERR_INCORRECT_LENGTH, "accumulator LCCCS sizes (r: s, v: tau, cm: kappa, u: t, x_w: l)");
  if (!w_acc->f_coeff || !w_i->f_coeff || !w_i->w_ccs || !w_out->f || !w_out->f_coeff || !w_out->w_ccs)
    return bad(P, LF_ERR_INVALID_ARG, "missing witness buffer");
  if (!proof->lin_sumcheck || !proof->lin_v || !proof->lin_u || !proof->fold_sumcheck || !proof->theta_s ||
      !proof->eta_s || !out->r || !out->v || !out->cm || !out->u || (l && !out->x_w) || !out->h)
    return bad(P, LF_ERR_INVALID_ARG, "missing output buffer");
  for (int side = 0; side < 2; side++)
    if (!proof->u_s[side] || !proof->v_s[side] || !proof->x_s[side] || !proof->y_s[side])
      return bad(P, LF_ERR_INVALID_ARG, "missing decomposition proof buffer");
  // host copies of the public inputs in canonical form
  auto canon = [&](const uint64_t *src, size_t elems) {
    std::vector<uint64_t> v(src, src + elems);
    if (repr == LF_REPR_MONTGOMERY)
      for (auto &x : v) x = gl::from_mont(x);
    return v;
  };
  const std::vector<uint64_t> ar = canon(acc->r.elems, (size_t)s * d), av = canon(acc->v.elems, (size_t)tau * d),
                              acm = canon(acc->cm.elems, kd), au = canon(acc->u.elems, (size_t)t * d),
                              axw = canon(acc->x_w.elems, l * d), ah = canon(acc->h, d), cmi = canon(cm_i, kd),
                              xc = canon(x_ccs, l * d);
  lf_ctx *C = P->ctx;
  Run R{P, lf_transcript_new(), (hipStream_t)lf_ctx_get_stream(C)};
  struct TGuard {
    lf_transcript *t;
    ~TGuard() { lf_transcript_free(t); }
  } tg{R.T};
  lf_transcript_record(R.T);
  P->samples.clear();
  int prev = -1;
  if (hipGetDevice(&prev) == hipSuccess && prev != P->device) (void)hipSetDevice(P->device);
  struct DGuard {
    int prev, dev;
    ~DGuard() {
      if (prev >= 0 && prev != dev) (void)hipSetDevice(prev);
    }
  } dg{prev, P->device};
  std::vector<uint64_t> one(d, 0);
  for (int i = 0; i < d; i += tb) one[i] = 1;

  // the linearization's Mz MLEs need no challenge: on the device while the host absorbs
  if (linearize_prepare(P, R, xc, w_i)) return R.rc;
  // ---- absorb_public_input (zk_latticefold.rs:162-184)
  R.absorb_label("acc");
  R.absorb(ar.data(), s);
  R.absorb(av.data(), tau);
  R.absorb(acm.data(), kappa);
  R.absorb(au.data(), t);
  R.absorb(axw.data(), l);
  R.absorb(ah.data(), 1);
  R.absorb_label("cm_i");
  R.absorb(cmi.data(), kappa);
  R.absorb(xc.data(), l);

  R.mark(LF_SPAN_PUBLIC_INPUT, false);
  // ---- linearization (linearization.rs:153-197)
  std::vector<uint64_t> r_lin, lv, lu;
  if (linearize(P, R, w_i, proof->lin_sumcheck, r_lin, lv, lu)) return R.rc;
  R.mark(LF_SPAN_LINEARIZATION);
  // the linearized instance: {r, v, cm_i, u, x_ccs, h = ONE}

  // ---- the two decompositions (decomposition.rs:33-88), device work of both first
  R.h2d(P->cmd[0], acm.data(), kd);
  R.h2d(P->cmd[1], cmi.data(), kd);
  R.h2d(P->xw[0], axw.data(), l * d);  // x_w || h of each side
  R.h2d(P->xw[0] + l * d, ah.data(), d);
  R.h2d(P->xw[1], xc.data(), l * d);
  R.h2d(P->xw[1] + l * d, one.data(), d);
  for (int side = 0; side < 2; side++)
    R.check(lf_dev_compute_x_s(C, &P->pr, P->xw[side], l + 1, P->xs + (size_t)side * K * (l + 1) * d), "compute_x_s");
  lf_fold_step_bufs b{};
  b.acc_f_coeff = w_acc->f_coeff;
  b.f_coeff = const_cast<uint64_t *>(w_i->f_coeff);
  b.acc_cm = P->cmd[0];
  b.cm = P->cmd[1];
  for (int side = 0; side < 2; side++) {
    b.fk_coeff[side] = P->fkc[side];
    b.fk[side] = P->fk[side];
    b.wk[side] = P->wk[side];
    b.y[side] = P->y[side];
  }
  if (R.rc == LF_OK) R.check(lf_dev_decompose_commit(C, P->aj, &P->pr, W, &b), "decompose + commit_witnesses");
  // z_k = x_s[k] || w_ccs_k (compute_mz_mles, :229-256) for the u_s (and later eta_s), one
  // launch per side (the stream's queue holds a bounded number of commands: every one
  // saved is host time the transcript gets back)
  for (int side = 0; side < 2; side++)
    R.hip(lfk::assemble_z(P->xs + (size_t)side * K * (l + 1) * d, P->wk[side], K, l + 1, W, d, P->zdec[side], R.st),
          "z_k");
  // per side: v_s, u_s at the side's point, then its messages back to pinned memory
  // behind events, so the host absorbs while the device evaluates: x_s, y_s and v_s
  // of a side first, then u_s in groups of MZ_GROUP instances (one event each: the
  // host starts on instance 0 as soon as its u_s is back), and the challenge-
  // independent folding MLEs (the f_hat MLEs of the 2K decomposed witnesses, eq(r_i);
  // create_sumcheck_polynomial, folding/utils.rs:196-255) behind them
  uint64_t *M = P->fold;
  const size_t mstride = nn * d;
  // eq(r_i) of each side is the folding prover's eq(r_i) MLE (M slots 0 and 2; the
  // linearization left eq(r_lin) in slot 2): v_s and u_s read it from there
  R.h2p2d(P->pt, P->hr[0], ar.data(), (size_t)s * d);
  R.check(lf_dev_eq_table(C, d, P->pt, s, M), "eq(r_0)");
  const int G = MZ_GROUP, ng = (K + G - 1) / G;
  // The u_s groups go to the device from a second host thread (its own Run, so the
  // error state is not shared): with the stream's queue deep, every enqueue blocks the
  // calling thread for tens of microseconds, which the transcript thread would
  // otherwise spend before and between its absorbs. `posted` counts the groups whose
  // event is recorded; the absorb loop waits on a group's event only after that.
  const bool digits = P->pr.b_small == 2;  // f_hat values in {-1, 0, 1}: read from the coefficient rows
  std::atomic<int> posted{0};
  Run RE = R;
  std::string err_enq;  // the enqueue thread's own error text, merged into P->err after the join
  RE.err = &err_enq;
  auto enqueue_side = [&](Run &Q, int side) {
    const uint64_t *eq_s = M + (size_t)(2 * side) * mstride;
    Q.check(lf_dev_fhat_evaluate_eq(C, d, P->fkc[side], N, ND, K, s, eq_s, P->vs + (size_t)side * K * tau * d), "v_s");
    Q.d2p(P->hx[side], P->xs + (size_t)side * K * (l + 1) * d, (size_t)K * (l + 1) * d);
    Q.d2p(P->hy[side], P->y[side], (size_t)K * kd);
    Q.d2p(P->hv[side], P->vs + (size_t)side * K * tau * d, (size_t)K * tau * d);
    Q.check(lf_dev_mz_weights(C, P->ccs, s, eq_s, P->mzw), "u_s weights");
    for (int g = 0; g < ng; g++) {
      const int k0 = g * G, nk = std::min(G, K - k0);
      uint64_t *us = P->us + ((size_t)side * K + k0) * t * d;
      Q.check(lf_dev_mz_dots(C, P->ccs, P->mzw, P->zdec[side] + (size_t)k0 * n * d, nk, us), "u_s");
      Q.d2p(P->hu[side] + (size_t)k0 * t * d, us, (size_t)nk * t * d);
      Q.hip(hipEventRecord(P->ev[2 + side * ng + g], Q.st), "event");
      posted.store(side * ng + g + 1, std::memory_order_release);
    }
  };
  auto enqueue_all = [&] {
    (void)hipSetDevice(P->device);
    if (RE.rc == LF_OK) {
      enqueue_side(RE, 0);
      enqueue_side(RE, 1);
      if (!digits)
        for (int sd = 0; sd < 2; sd++)
          RE.hip(lfk::get_fhat(P->fkc[sd], N, d, s, M + (5 + (size_t)sd * K * tau) * mstride, RE.st, K, ND), "f_hat");
    }
    posted.store(1 << 30, std::memory_order_release);  // done (also on an error)
  };
  std::thread enq;
  try {
    enq = std::thread(enqueue_all);
  } catch (const std::exception &) {  // no thread to be had: enqueue everything here first
    enqueue_all();
  }
  auto join = [&] {
    if (enq.joinable()) enq.join();
    if (RE.rc != LF_OK && R.rc == LF_OK) {
      R.rc = RE.rc;
      P->err = err_enq;
    }
    return R.rc;
  };
  R.mark(LF_SPAN_DECOMPOSITION, false);
  for (int side = 0; side < 2; side++)
    for (int k = 0; k < K; k++) {  // the decomposed instances' messages (:58-64)
      if (k % G == 0) {
        const int g = side * ng + k / G;
        while (posted.load(std::memory_order_acquire) <= g) std::this_thread::yield();
        if (posted.load(std::memory_order_acquire) >= (1 << 30) && RE.rc != LF_OK) return join();
        if (R.wait(P->ev[2 + g])) return join();
      }
      const size_t ox = (size_t)k * (l + 1) * d, oy = (size_t)k * kd, ou = (size_t)k * t * d, ov = (size_t)k * tau * d;
      memcpy(proof->x_s[side] + ox, P->hx[side] + ox, (l + 1) * d * 8);
      memcpy(proof->y_s[side] + oy, P->hy[side] + oy, kd * 8);
      memcpy(proof->u_s[side] + ou, P->hu[side] + ou, (size_t)t * d * 8);
      memcpy(proof->v_s[side] + ov, P->hv[side] + ov, (size_t)tau * d * 8);
      R.absorb(proof->x_s[side] + ox, l + 1);
      R.absorb(proof->y_s[side] + oy, kappa);
      R.absorb(proof->u_s[side] + ou, t);
      R.absorb(proof->v_s[side] + ov, tau);
    }
  if (join()) return R.rc;
  R.mark(LF_SPAN_DECOMPOSITION_TRANSCRIPT, false);
  // ---- folding (folding.rs:42-130)
  R.absorb_label("alpha_s");  // squeeze_alpha_beta_zeta_mu (folding/utils.rs:51-96)
  const std::vector<uint64_t> alpha = R.challenges(2 * K);
  R.absorb_label("zeta_s");
  const std::vector<uint64_t> zeta = R.challenges(2 * K);
  R.absorb_label("mu_s");
  std::vector<uint64_t> mu = R.challenges(2 * K - 1);
  mu.insert(mu.end(), one.begin(), one.end());
  R.absorb_label("beta_s");
  const std::vector<uint64_t> fbeta = R.challenges(s);
  R.h2d(P->zeta, zeta.data(), 2 * (size_t)K * d);
  R.h2d(P->mu, mu.data(), 2 * (size_t)K * d);
  R.h2d(P->beta, fbeta.data(), (size_t)s * d);
  // Horner weights alpha_k^(j+1) of each side's f_hat MLEs (prepare_g1_and_3_k_mles_list, :519-541)
  for (int side = 0; side < 2; side++) {
    std::vector<uint64_t> cf((size_t)K * tau * d);
    for (int k = 0; k < K; k++) {
      const uint64_t *a = alpha.data() + (size_t)(side * K + k) * d;  // broadcast: slot 0 holds the base value
      uint64_t pw[3] = {a[0], tb == 3 ? a[1] : 0, tb == 3 ? a[2] : 0};
      for (int j = 0; j < tau; j++) {
        broadcast(pw, tb, d, cf.data() + ((size_t)k * tau + j) * d);
        uint64_t nx[3];
        base_mul(pw, a, nx, tb);
        memcpy(pw, nx, sizeof(pw));
      }
    }
    R.h2d(P->coef[side], cf.data(), cf.size());
  }
  // the MLEs [eq(r_0), g1, eq(r_1), g3, eq(beta), f_hat (2K x tau)] (create_sumcheck_polynomial,
  // :196-255): eq(r_i) were enqueued before the decomposition transcript; the f_hat MLEs
  // (Witness::get_fhat of the decomposed witnesses) are not materialised for B_SMALL = 2 --
  // their values are the digits of the coefficient rows P->fkc, which g1 / g3 and the
  // sumcheck's first round read directly (lf_sumcheck_prove_fold_digits)
  // both sides' challenged Mz MLEs in one pass over the matrices (g1, g3 slots)
  R.check(lf_dev_mz_challenged_pair(C, P->ccs, P->zdec[0], P->zeta, P->zdec[1], P->zeta + (size_t)K * d, K, s,
                                    M + mstride, M + 3 * mstride),
          "challenged Mz");
  for (int side = 0; side < 2; side++) {
    uint64_t *g = M + (size_t)(2 * side + 1) * mstride;
    if (digits)
      R.hip(lfk::fhat_lincomb_digits(P->fkc[side], K, N, ND, P->coef[side], s, d, g, R.st), "g");
    else
      R.check(lf_dev_mle_lincomb(C, d, M + (5 + (size_t)side * K * tau) * mstride, mstride, K * tau, s, P->coef[side], g),
              "g");
  }
  R.check(lf_dev_eq_table(C, d, P->beta, s, M + 4 * mstride), "eq(beta)");
  std::vector<uint64_t> rnd((size_t)s * tb);
  R.mark(LF_SPAN_FOLDING_MLES);
  {
    lf_comb cb{};
    cb.kind = LF_COMB_FOLDING;
    cb.nk = 2 * K;
    cb.tau = tau;
    cb.bsmall = (int)P->pr.b_small;
    cb.mu = P->mu;
    if (R.rc == LF_OK)
      R.check(digits
                  ? lf_sumcheck_prove_fold_digits(C, R.T, &cb, M, P->fkc[0], P->fkc[1], K, N, ND, s, d, M + 5 * mstride,
                                                  proof->fold_sumcheck, rnd.data())
                  : lf_sumcheck_prove(C, R.T, &cb, M, P->nm_fold, s, d, 2 * cb.bsmall, proof->fold_sumcheck, rnd.data()),
              "folding sumcheck");
  }
  if (R.rc) return R.rc;
  R.mark(LF_SPAN_FOLDING_SUMCHECK);
  std::vector<uint64_t> r0((size_t)s * d);
  for (int i = 0; i < s; i++) broadcast(rnd.data() + (size_t)i * tb, tb, d, r0.data() + (size_t)i * d);
  R.h2d(P->r0, r0.data(), (size_t)s * d);
  // theta_s = f_hat(w_i)(r_0), eta_s = MLE(M_j z_i)(r_0) (get_thetas / get_etas, :236-256):
  // theta_s and side 0's eta_s come back first, so the host absorbs them while the
  // device evaluates side 1's eta_s
  // one eq(r_0) table and one set of Mz weights at r_0 for both sides
  R.check(lf_dev_eq_table(C, d, P->r0, s, P->eq0), "eq(r_0)");
  for (int side = 0; side < 2; side++)
    R.check(lf_dev_fhat_evaluate_eq(C, d, P->fkc[side], N, ND, K, s, P->eq0, P->theta + (size_t)side * K * tau * d),
            "theta");
  R.d2p(P->htheta, P->theta, 2 * (size_t)K * tau * d);
  R.hip(hipEventRecord(P->ev[0], R.st), "event");
  R.check(lf_dev_mz_weights(C, P->ccs, s, P->eq0, P->mzw), "eta weights");
  if (R.rc) return R.rc;
  // the eta_s groups of both sides from a second host thread, as the u_s groups above
  std::atomic<int> eposted{0};
  Run RQ = R;
  std::thread eenq([&] {
    (void)hipSetDevice(P->device);
    for (int side = 0; side < 2 && RQ.rc == LF_OK; side++)
      for (int gg = 0; gg < ng; gg++) {  // instance groups in absorb order
        const int g = side * ng + gg, k0 = gg * G, nk = std::min(G, K - k0);
        const size_t o = ((size_t)side * K + k0) * t * d;
        RQ.check(lf_dev_mz_dots(C, P->ccs, P->mzw, P->zdec[side] + (size_t)k0 * n * d, nk, P->eta + o), "eta");
        RQ.d2p(P->heta + o, P->eta + o, (size_t)nk * t * d);
        RQ.hip(hipEventRecord(P->ev[2 + g], RQ.st), "event");
        eposted.store(g + 1, std::memory_order_release);
      }
    eposted.store(1 << 30, std::memory_order_release);
  });
  auto ejoin = [&] {
    if (eenq.joinable()) eenq.join();
    if (RQ.rc != LF_OK && R.rc == LF_OK) R.rc = RQ.rc;
    return R.rc;
  };
  R.mark(LF_SPAN_EVALUATIONS, false);
  if (R.wait(P->ev[0])) return ejoin();
  memcpy(proof->theta_s, P->htheta, 2 * (size_t)K * tau * d * 8);
  for (int i = 0; i < 2 * K; i++) R.absorb(proof->theta_s + (size_t)i * tau * d, tau);
  for (int side = 0; side < 2; side++)
    for (int k = 0; k < K; k++) {
      if (k % G == 0) {
        const int g = side * ng + k / G;
        while (eposted.load(std::memory_order_acquire) <= g) std::this_thread::yield();
        if (eposted.load(std::memory_order_acquire) >= (1 << 30) && RQ.rc != LF_OK) return ejoin();
        if (R.wait(P->ev[2 + g])) return ejoin();
      }
      const size_t o = ((size_t)side * K + k) * t * d;
      memcpy(proof->eta_s + o, P->heta + o, (size_t)t * d * 8);
      R.absorb(proof->eta_s + o, t);
    }
  if (ejoin()) return R.rc;
  // get_rhos (folding/utils.rs:116-127): 2K - 1 short challenges and ONE, then CRT
  R.absorb_label("rho_s");
  std::vector<uint64_t> rc(2 * (size_t)K * d, 0);
  if (lf_transcript_get_short_challenges(R.T, d, 2 * K - 1, rc.data()) != LF_OK)
    return bad(P, LF_ERR_CHALLENGE_BYTES, "short challenges");
  rc[(size_t)(2 * K - 1) * d] = 1;
  R.mark(LF_SPAN_FOLDING_TRANSCRIPT);
  R.h2d(P->rhoc, rc.data(), rc.size());
  R.d2d(P->rho, P->rhoc, rc.size());
  R.check(lf_dev_crt(C, P->rho, 2 * K, d), "CRT(rho)");
  // f_0, cm_0, Witness::from_f(f_0) (:112-122), then v_0, u_0, x_0 (compute_v0_u0_x0_cm_0, :456-517)
  b.rho = P->rho;
  b.f0 = w_out->f;
  b.f0_coeff = w_out->f_coeff;
  b.w_ccs0 = w_out->w_ccs;
  b.cm0 = P->cm0;
  if (R.rc == LF_OK) R.check(lf_dev_fold_combine(C, P->aj, &P->pr, W, &b), "fold");
  R.check(lf_dev_fold_lcccs(C, d, 2 * K, P->rho, P->rhoc, P->eta, t, P->xs, l + 1, P->theta, P->u0, P->x0, P->v0),
          "v_0, u_0, x_0");
  if (R.rc) return R.rc;
  // prepare_public_output (folding.rs:381-392): x_w = x_0[..l], h = x_0[l]
  std::vector<uint64_t> x0((l + 1) * d);
  R.d2h(out->cm, P->cm0, kd);
  R.d2h(out->u, P->u0, (size_t)t * d);
  R.d2h(out->v, P->v0, (size_t)tau * d);
  R.d2h(x0.data(), P->x0, (l + 1) * d);
  R.check(lf_ctx_sync(C), "sync");
  if (R.rc) return R.rc;
  R.mark(LF_SPAN_FOLD);
  P->samples.resize(lf_transcript_samples(R.T, nullptr, 0));
  lf_transcript_samples(R.T, P->samples.data(), P->samples.size());
  memcpy(out->r, r0.data(), r0.size() * 8);
  if (l) memcpy(out->x_w, x0.data(), l * d * 8);
  memcpy(out->h, x0.data() + l * d, d * 8);
  memcpy(proof->lin_v, lv.data(), lv.size() * 8);
  memcpy(proof->lin_u, lu.data(), lu.size() * 8);
  if (repr == LF_REPR_MONTGOMERY) {
    auto mont = [](uint64_t *p, size_t elems) {
      for (size_t i = 0; i < elems; i++) p[i] = gl::to_mont(p[i]);
    };
    mont(out->r, (size_t)s * d);
    mont(out->v, (size_t)tau * d);
    mont(out->cm, kd);
    mont(out->u, (size_t)t * d);
    mont(out->x_w, l * d);
    mont(out->h, d);
    mont(proof->lin_sumcheck, (size_t)s * (P->degree + 2) * d);
    mont(proof->lin_v, (size_t)tau * d);
    mont(proof->lin_u, (size_t)t * d);
    for (int side = 0; side < 2; side++) {
      mont(proof->u_s[side], (size_t)K * t * d);
      mont(proof->v_s[side], (size_t)K * tau * d);
      mont(proof->x_s[side], (size_t)K * (l + 1) * d);
      mont(proof->y_s[side], (size_t)K * kd);
    }
    mont(proof->fold_sumcheck, (size_t)s * (2 * P->pr.b_small + 1) * d);
    mont(proof->theta_s, 2 * (size_t)K * tau * d);
    mont(proof->eta_s, 2 * (size_t)K * t * d);
  }
  return LF_OK;
}

// fold() followed by generate_verification_witness_vars (zk_latticefold.rs:111-148),
// as main.rs:175-185 runs them: the vars come from a replay of the proof on this
// call's own sample log (lf_fold_replay_samples) -- bit for bit what lf_fold_replay's
// second Poseidon2 pass over the same messages gives, without the permutations
int lf_fold_prove_vars(lf_prover *P, const lf_lcccs *acc, const lf_witness *w_acc, const uint64_t *cm_i,
                       const uint64_t *x_ccs, const lf_witness *w_i, lf_lcccs_mut *out, const lf_witness *w_out,
                       lf_lfproof_mut *proof, lf_replay_vars *vars, int repr) {
  if (!vars) return LF_ERR_INVALID_ARG;
  const int rc = lf_fold_prove(P, acc, w_acc, cm_i, x_ccs, w_i, out, w_out, proof, repr);
  if (rc != LF_OK) return rc;
  if (P->d != 24) return bad(P, LF_ERR_UNSUPPORTED_RING, "verification vars: Phi_72 only (TAU = 3)");
  const auto t0 = std::chrono::steady_clock::now();
  std::vector<uint64_t> c = P->c;
  if (repr == LF_REPR_MONTGOMERY)
    for (auto &x : c) x = gl::to_mont(x);
  lf_ccs_desc desc{};
  desc.t = P->t;
  desc.m = P->nn;
  desc.l = P->l;
  desc.degree = P->degree;
  desc.q = P->q;
  desc.c = c.data();
  desc.S_off = P->S_off.data();
  desc.S_idx = P->S_idx.data();
  const int r = lf_fold_replay_samples(&desc, &P->pr, acc, cm_i, x_ccs, proof, P->samples.data(), P->samples.size(),
                                       vars, repr);
  if (P->timing)
    P->span_ms[LF_SPAN_VARS] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return r == LF_OK ? LF_OK : bad(P, r, "verification vars replay");
}

size_t lf_prover_samples(const lf_prover *P, uint64_t *out, size_t cap) {
  if (!P) return 0;
  if (out) memcpy(out, P->samples.data(), (cap < P->samples.size() ? cap : P->samples.size()) * 8);
  return P->samples.size();
}

}  // extern "C"
