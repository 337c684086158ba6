// serialize.cpp -- the wire format of the folding proof and the accumulator
// (SURVEY.md 8(f) rank 4): ark-serialize 0.5 CanonicalSerialize, as derived on
// the reference's types. For these types compressed and uncompressed are the
// same bytes:
//   Fq        8 bytes little-endian of the canonical value (ark-ff into_bigint)
//   Fq3       c0, c1, c2
//   RqNTT     its slot values in order, no length ([C::BaseCRTField; D],
//             stark-rings cyclotomic_ring/ntt_form.rs:24-27)
//   Vec<T>    u64 little-endian length, then the items
//   Commitment { val: Vec<R> }            (commitment/homomorphic_commitment.rs:7-9)
//   sumcheck::Proof(Vec<ProverMsg>), ProverMsg { evaluations: Vec<R> }
//   LFProof { linearization_proof, decomposition_proof_l, decomposition_proof_r,
//             folding_proof }             (latticefold/src/nifs.rs:28-34)
//   LCCCS has no CanonicalSerialize in the reference; its fields are written in
//   declaration order the same way (arith.rs:192-206), which is what the
//   rank-to-rank and host-to-device accumulator interchange uses.
// Host code only: these are byte layouts, no device work.
#include <cstring>
#include <vector>

#include "../../include/lf.h"
#include "gl.hpp"

namespace {

struct Writer {
  uint8_t *out;
  size_t cap, pos = 0;
  int repr;
  bool overflow = false;
  void bytes(const void *p, size_t n) {
    if (out && pos + n <= cap) memcpy(out + pos, p, n);
    if (out && pos + n > cap) overflow = true;
    pos += n;
  }
  void u64(uint64_t v) {
    uint8_t b[8];
    for (int i = 0; i < 8; i++) b[i] = (uint8_t)(v >> (8 * i));
    bytes(b, 8);
  }
  void fq(uint64_t v) { u64(repr == LF_REPR_MONTGOMERY ? gl::from_mont(v) : gl::canon(v)); }
  void ring_vec(const lf_ring_slice &s, int d) {
    u64(s.n);
    if (s.n && s.elems)
      for (size_t i = 0; i < s.n * (size_t)d; i++) fq(s.elems[i]);
  }
  void ring_vecvec(const lf_ring_slice *v, size_t n, int d) {
    u64(n);
    for (size_t i = 0; i < n; i++) ring_vec(v[i], d);
  }
  void commitments(const lf_ring_slice *v, size_t n, int d) { ring_vecvec(v, n, d); }
  void sumcheck(const uint64_t *msgs, size_t rounds, size_t evals, int d) {
    u64(rounds);
    for (size_t r = 0; r < rounds; r++) ring_vec({msgs + r * evals * d, evals}, d);
  }
};

struct Reader {
  const uint8_t *in;
  size_t len, pos = 0;
  int repr;
  bool bad = false;
  uint64_t u64() {
    if (pos + 8 > len) {
      bad = true;
      return 0;
    }
    uint64_t v = 0;
    for (int i = 0; i < 8; i++) v |= (uint64_t)in[pos + i] << (8 * i);
    pos += 8;
    return v;
  }
  uint64_t fq() {
    const uint64_t v = u64();
    if (v >= gl::P) bad = true;  // ark's deserialize_with_flags rejects non-canonical values
    return repr == LF_REPR_MONTGOMERY ? gl::to_mont(v) : v;
  }
};

}  // namespace

extern "C" {

int lf_lcccs_serialize(const lf_lcccs *a, int repr, uint8_t *out, size_t cap, size_t *len) {
  if (!a || !len || a->d < 1 || !a->h || (repr != LF_REPR_CANONICAL && repr != LF_REPR_MONTGOMERY))
    return LF_ERR_INVALID_ARG;
  Writer w{out, cap, 0, repr};
  w.ring_vec(a->r, a->d);
  w.ring_vec(a->v, a->d);
  w.ring_vec(a->cm, a->d);  // Commitment { val }
  w.ring_vec(a->u, a->d);
  w.ring_vec(a->x_w, a->d);
  for (int i = 0; i < a->d; i++) w.fq(a->h[i]);
  *len = w.pos;
  return w.overflow ? LF_ERR_INCORRECT_LENGTH : LF_OK;
}

int lf_lcccs_deserialize(const uint8_t *in, size_t len, int d, int repr, uint64_t *buf, size_t buf_elems,
                         lf_lcccs *out) {
  if (!in || !out || d < 1 || (repr != LF_REPR_CANONICAL && repr != LF_REPR_MONTGOMERY)) return LF_ERR_INVALID_ARG;
  Reader r{in, len, 0, repr};
  size_t used = 0;
  lf_ring_slice *fields[5] = {&out->r, &out->v, &out->cm, &out->u, &out->x_w};
  out->d = d;
  for (lf_ring_slice *f : fields) {
    const uint64_t n = r.u64();
    if (r.bad || n > (len - r.pos) / (8 * (size_t)d) || used + n * d > buf_elems) return LF_ERR_INCORRECT_LENGTH;
    f->elems = buf + used;
    f->n = n;
    for (size_t i = 0; i < n * (size_t)d; i++) buf[used + i] = r.fq();
    used += n * d;
  }
  if (used + d > buf_elems) return LF_ERR_INCORRECT_LENGTH;
  for (int i = 0; i < d; i++) buf[used + i] = r.fq();
  out->h = buf + used;
  if (r.bad || r.pos != len) return LF_ERR_INCORRECT_LENGTH;
  return LF_OK;
}

int lf_lfproof_serialize(const lf_lfproof *p, int repr, uint8_t *out, size_t cap, size_t *len) {
  if (!p || !len || p->d < 1 || (repr != LF_REPR_CANONICAL && repr != LF_REPR_MONTGOMERY)) return LF_ERR_INVALID_ARG;
  const int d = p->d;
  Writer w{out, cap, 0, repr};
  // LinearizationProof { linearization_sumcheck, v, u } (linearization/structs.rs:15-38)
  w.sumcheck(p->lin_sumcheck, p->lin_rounds, p->lin_evals, d);
  w.ring_vec(p->lin_v, d);
  w.ring_vec(p->lin_u, d);
  // DecompositionProof { u_s, v_s, x_s, y_s } x 2 (decomposition/structs.rs:19-48)
  for (int s = 0; s < 2; s++) {
    w.ring_vecvec(p->dec[s].u_s, p->dec[s].n_u, d);
    w.ring_vecvec(p->dec[s].v_s, p->dec[s].n_v, d);
    w.ring_vecvec(p->dec[s].x_s, p->dec[s].n_x, d);
    w.commitments(p->dec[s].y_s, p->dec[s].n_y, d);
  }
  // FoldingProof { pointshift_sumcheck_proof, theta_s, eta_s } (folding/structs.rs:17-40)
  w.sumcheck(p->fold_sumcheck, p->fold_rounds, p->fold_evals, d);
  w.ring_vecvec(p->theta_s, p->n_theta, d);
  w.ring_vecvec(p->eta_s, p->n_eta, d);
  *len = w.pos;
  return w.overflow ? LF_ERR_INCORRECT_LENGTH : LF_OK;
}

}  // extern "C"
