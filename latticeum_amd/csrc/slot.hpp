// slot.hpp -- one NTT slot of a ring element as a value type: an Fq3 =
// Fq[u]/(u^3 - 2^40) for Phi_72 (TB = 3 words), an Fq for X^d + 1 (TB = 1).
// Ring products in NTT form are slot-wise (ntt_form.rs:159-189), so kernels
// that treat slots independently (sumcheck.hip, mz.hip) work on these.
#pragma once
#include "gl.hpp"

namespace lfk {

template <int TB>
struct Sv {
  uint64_t c[TB];
};
template <int TB>
__device__ __forceinline__ Sv<TB> s_load(const uint64_t *p) {
  Sv<TB> r;
#pragma unroll
  for (int i = 0; i < TB; i++) r.c[i] = p[i];
  return r;
}
template <int TB>
__device__ __forceinline__ void s_store(uint64_t *p, const Sv<TB> &v) {
#pragma unroll
  for (int i = 0; i < TB; i++) p[i] = v.c[i];
}
template <int TB>
__device__ __forceinline__ Sv<TB> s_add(const Sv<TB> &a, const Sv<TB> &b) {
  Sv<TB> r;
#pragma unroll
  for (int i = 0; i < TB; i++) r.c[i] = gl::add(a.c[i], b.c[i]);
  return r;
}
template <int TB>
__device__ __forceinline__ Sv<TB> s_sub(const Sv<TB> &a, const Sv<TB> &b) {
  Sv<TB> r;
#pragma unroll
  for (int i = 0; i < TB; i++) r.c[i] = gl::sub(a.c[i], b.c[i]);
  return r;
}
template <int TB>
__device__ __forceinline__ Sv<TB> s_zero() {
  Sv<TB> r;
#pragma unroll
  for (int i = 0; i < TB; i++) r.c[i] = 0;
  return r;
}
template <int TB>
__device__ __forceinline__ Sv<TB> s_one() {
  Sv<TB> r = s_zero<TB>();
  r.c[0] = 1;
  return r;
}
// small scalar k as a slot value (k, 0, 0)
template <int TB>
__device__ __forceinline__ Sv<TB> s_scalar(uint64_t k) {
  Sv<TB> r = s_zero<TB>();
  r.c[0] = k;
  return r;
}
// slot product: Fq, or Fq3 = Fq[u]/(u^3 - 2^40) (goldilocks/mod.rs:34-54) with
// the carry-chain accumulators and one reduction per output word
__device__ __forceinline__ Sv<1> s_mul(const Sv<1> &a, const Sv<1> &b) {
  Sv<1> r;
  r.c[0] = gl::mul(a.c[0], b.c[0]);
  return r;
}
// c0 = a0 b0 + a1 (2^40 b2) + a2 (2^40 b1), c1 = a0 b1 + a1 b0 + a2 (2^40 b2),
// c2 = a0 b2 + a1 b1 + a2 b0: the nonresidue folded into the operands (two
// shifts) so each output word is one carry-chain accumulator and one reduction
__device__ __forceinline__ Sv<3> s_mul(const Sv<3> &a, const Sv<3> &b) {
  const uint64_t b1n = gl::shl96(b.c[1], 40), b2n = gl::shl96(b.c[2], 40);
  // word by word (each accumulator reduced before the next starts: 9 live
  // accumulator registers instead of 27)
  Sv<3> r;
  gl::CAcc x;
  gl::cacc_zero(x);
  gl::cacc_mad(x, a.c[0], b.c[0]);
  gl::cacc_mad(x, a.c[1], b2n);
  gl::cacc_mad(x, a.c[2], b1n);
  r.c[0] = gl::cacc_reduce(x);
  gl::cacc_zero(x);
  gl::cacc_mad(x, a.c[0], b.c[1]);
  gl::cacc_mad(x, a.c[1], b.c[0]);
  gl::cacc_mad(x, a.c[2], b2n);
  r.c[1] = gl::cacc_reduce(x);
  gl::cacc_zero(x);
  gl::cacc_mad(x, a.c[0], b.c[2]);
  gl::cacc_mad(x, a.c[1], b.c[1]);
  gl::cacc_mad(x, a.c[2], b.c[0]);
  r.c[2] = gl::cacc_reduce(x);
  return r;
}
// a b with a any u64 words (weakly reduced) and b canonical, the result weakly reduced:
// for chains of products (each output feeds the next product's left operand), with
// one canonicalisation at the chain's end (s_canon)
__device__ __forceinline__ Sv<1> s_mul_w(const Sv<1> &a, const Sv<1> &b) {
  uint64_t lo, hi;
  gl::mul_wide(a.c[0], b.c[0], lo, hi);
  Sv<1> r;
  r.c[0] = gl::reduce128(lo, hi);
  return r;
}
__device__ __forceinline__ Sv<3> s_mul_w(const Sv<3> &a, const Sv<3> &b) {
  const uint64_t b1n = gl::shl96(b.c[1], 40), b2n = gl::shl96(b.c[2], 40);
  Sv<3> r;
  gl::CAcc x;
  gl::cacc_zero(x);
  gl::cacc_mad(x, a.c[0], b.c[0]);
  gl::cacc_mad(x, a.c[1], b2n);
  gl::cacc_mad(x, a.c[2], b1n);
  r.c[0] = gl::cacc_reduce_weak(x);
  gl::cacc_zero(x);
  gl::cacc_mad(x, a.c[0], b.c[1]);
  gl::cacc_mad(x, a.c[1], b.c[0]);
  gl::cacc_mad(x, a.c[2], b2n);
  r.c[1] = gl::cacc_reduce_weak(x);
  gl::cacc_zero(x);
  gl::cacc_mad(x, a.c[0], b.c[2]);
  gl::cacc_mad(x, a.c[1], b.c[1]);
  gl::cacc_mad(x, a.c[2], b.c[0]);
  r.c[2] = gl::cacc_reduce_weak(x);
  return r;
}
template <int TB>
__device__ __forceinline__ Sv<TB> s_canon(const Sv<TB> &a) {
  Sv<TB> r;
#pragma unroll
  for (int i = 0; i < TB; i++) r.c[i] = gl::canon(a.c[i]);
  return r;
}
// a b + u v, word by word with one reduction per word
__device__ __forceinline__ Sv<1> s_mad2(const Sv<1> &a, const Sv<1> &b, const Sv<1> &u, const Sv<1> &v) {
  gl::CAcc x;
  gl::cacc_zero(x);
  gl::cacc_mad(x, a.c[0], b.c[0]);
  gl::cacc_mad(x, u.c[0], v.c[0]);
  Sv<1> r;
  r.c[0] = gl::cacc_reduce(x);
  return r;
}
__device__ __forceinline__ Sv<3> s_mad2(const Sv<3> &a, const Sv<3> &b, const Sv<3> &u, const Sv<3> &v) {
  const uint64_t b1n = gl::shl96(b.c[1], 40), b2n = gl::shl96(b.c[2], 40);
  const uint64_t v1n = gl::shl96(v.c[1], 40), v2n = gl::shl96(v.c[2], 40);
  Sv<3> r;
  gl::CAcc x;
  gl::cacc_zero(x);
  gl::cacc_mad(x, a.c[0], b.c[0]);
  gl::cacc_mad(x, a.c[1], b2n);
  gl::cacc_mad(x, a.c[2], b1n);
  gl::cacc_mad(x, u.c[0], v.c[0]);
  gl::cacc_mad(x, u.c[1], v2n);
  gl::cacc_mad(x, u.c[2], v1n);
  r.c[0] = gl::cacc_reduce(x);
  gl::cacc_zero(x);
  gl::cacc_mad(x, a.c[0], b.c[1]);
  gl::cacc_mad(x, a.c[1], b.c[0]);
  gl::cacc_mad(x, a.c[2], b2n);
  gl::cacc_mad(x, u.c[0], v.c[1]);
  gl::cacc_mad(x, u.c[1], v.c[0]);
  gl::cacc_mad(x, u.c[2], v2n);
  r.c[1] = gl::cacc_reduce(x);
  gl::cacc_zero(x);
  gl::cacc_mad(x, a.c[0], b.c[2]);
  gl::cacc_mad(x, a.c[1], b.c[1]);
  gl::cacc_mad(x, a.c[2], b.c[0]);
  gl::cacc_mad(x, u.c[0], v.c[2]);
  gl::cacc_mad(x, u.c[1], v.c[1]);
  gl::cacc_mad(x, u.c[2], v.c[0]);
  r.c[2] = gl::cacc_reduce(x);
  return r;
}
template <int TB>
__device__ __forceinline__ bool s_is_zero(const Sv<TB> &a) {
  uint64_t o = 0;
#pragma unroll
  for (int i = 0; i < TB; i++) o |= a.c[i];
  return o == 0;
}


// lazy multiply-accumulate of slot products: sum_i a_i b_i with one reduction
// per output word at the end (carry-chain accumulators, gl::CAcc: 8 VALU per
// 64 x 64 product instead of a full product and reduction each)
template <int TB>
struct SAcc;
template <>
struct SAcc<1> {
  gl::CAcc x;
};
template <>
struct SAcc<3> {
  gl::CAcc x0, x1, x2;  // the three output words (nonresidue folded into the operands)
};
__device__ __forceinline__ void sacc_zero(SAcc<1> &a) { gl::cacc_zero(a.x); }
__device__ __forceinline__ void sacc_zero(SAcc<3> &a) {
  gl::cacc_zero(a.x0);
  gl::cacc_zero(a.x1);
  gl::cacc_zero(a.x2);
}
__device__ __forceinline__ void sacc_mad(SAcc<1> &a, const Sv<1> &x, const Sv<1> &y) { gl::cacc_mad(a.x, x.c[0], y.c[0]); }
__device__ __forceinline__ void sacc_mad(SAcc<3> &a, const Sv<3> &x, const Sv<3> &y) {
  const uint64_t y1n = gl::shl96(y.c[1], 40), y2n = gl::shl96(y.c[2], 40);
  gl::cacc_mad(a.x0, x.c[0], y.c[0]);
  gl::cacc_mad(a.x0, x.c[1], y2n);
  gl::cacc_mad(a.x0, x.c[2], y1n);
  gl::cacc_mad(a.x1, x.c[0], y.c[1]);
  gl::cacc_mad(a.x1, x.c[1], y.c[0]);
  gl::cacc_mad(a.x1, x.c[2], y2n);
  gl::cacc_mad(a.x2, x.c[0], y.c[2]);
  gl::cacc_mad(a.x2, x.c[1], y.c[1]);
  gl::cacc_mad(a.x2, x.c[2], y.c[0]);
}
// a scalar (s, 0, 0) times y: one product per word, no nonresidue
__device__ __forceinline__ void sacc_smad(SAcc<1> &a, uint64_t s, const Sv<1> &y) { gl::cacc_mad(a.x, s, y.c[0]); }
__device__ __forceinline__ void sacc_smad(SAcc<3> &a, uint64_t s, const Sv<3> &y) {
  gl::cacc_mad(a.x0, s, y.c[0]);
  gl::cacc_mad(a.x1, s, y.c[1]);
  gl::cacc_mad(a.x2, s, y.c[2]);
}
__device__ __forceinline__ Sv<1> sacc_final(const SAcc<1> &a) {
  Sv<1> r;
  r.c[0] = gl::cacc_reduce(a.x);
  return r;
}
__device__ __forceinline__ Sv<3> sacc_final(const SAcc<3> &a) {
  Sv<3> r;
  r.c[0] = gl::cacc_reduce(a.x0);
  r.c[1] = gl::cacc_reduce(a.x1);
  r.c[2] = gl::cacc_reduce(a.x2);
  return r;
}
// k v for a small integer k (the finite-difference and cubic-evaluation weights)
template <int TB>
__device__ __forceinline__ Sv<TB> s_smul(const Sv<TB> &v, uint64_t k) {
  Sv<TB> r;
#pragma unroll
  for (int i = 0; i < TB; i++) r.c[i] = gl::mul(v.c[i], k);
  return r;
}

}  // namespace lfk
