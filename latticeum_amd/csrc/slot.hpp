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
__device__ __forceinline__ Sv<3> s_mul(const Sv<3> &a, const Sv<3> &b) {
  gl::CAcc x0, x0n, x1, x1n, x2;
  gl::cacc_zero(x0);
  gl::cacc_zero(x0n);
  gl::cacc_zero(x1);
  gl::cacc_zero(x1n);
  gl::cacc_zero(x2);
  gl::cacc_mad(x0, a.c[0], b.c[0]);
  gl::cacc_mad(x0n, a.c[1], b.c[2]);
  gl::cacc_mad(x0n, a.c[2], b.c[1]);
  gl::cacc_mad(x1, a.c[0], b.c[1]);
  gl::cacc_mad(x1, a.c[1], b.c[0]);
  gl::cacc_mad(x1n, a.c[2], b.c[2]);
  gl::cacc_mad(x2, a.c[0], b.c[2]);
  gl::cacc_mad(x2, a.c[1], b.c[1]);
  gl::cacc_mad(x2, a.c[2], b.c[0]);
  Sv<3> r;
  r.c[0] = gl::add(gl::cacc_reduce(x0), gl::shl96(gl::cacc_reduce(x0n), 40));
  r.c[1] = gl::add(gl::cacc_reduce(x1), gl::shl96(gl::cacc_reduce(x1n), 40));
  r.c[2] = gl::cacc_reduce(x2);
  return r;
}
template <int TB>
__device__ __forceinline__ bool s_is_zero(const Sv<TB> &a) {
  uint64_t o = 0;
#pragma unroll
  for (int i = 0; i < TB; i++) o |= a.c[i];
  return o == 0;
}


}  // namespace lfk
