// digits.hpp -- signed representatives, balanced digits and the device error
// flag shared by the transform/decomposition kernels.
#pragma once
#include "gl.hpp"

namespace lfk {

// error flag bit 0: a balanced decomposition needed more digits than provided
// (the reference indexes out of bounds and panics:
//  stark-rings balanced_decomposition/mod.rs:85-87)
__device__ __forceinline__ void raise(int *err, int bit) {
  if (err) atomicOr(err, bit);
}

__device__ __forceinline__ int64_t signed_rep(uint64_t v) {
  // fq_convertible.rs:22-34: (q-1)/2 < v  ->  v - q  (fits in int64)
  return v > (gl::P - 1) / 2 ? (int64_t)(v - gl::P) : (int64_t)v;
}
__device__ __forceinline__ uint64_t from_signed(int64_t x) {
  return x < 0 ? gl::P - (uint64_t)(-x) : (uint64_t)x;
}
// one balanced digit step (balanced_decomposition/mod.rs:76-91) for b = 2^lb
__device__ __forceinline__ int64_t bal_digit(int64_t &curr, int lb) {
  const int64_t b = (int64_t)1 << lb, bh = b >> 1;
  // truncating division / remainder by 2^lb (Rust `/` and `%` semantics)
  int64_t q = (curr + ((curr >> 63) & (b - 1))) >> lb;
  int64_t rem = curr - (q << lb);
  int64_t ar = rem < 0 ? -rem : rem;
  if (ar <= bh) {
    curr = q;
    return rem;
  }
  // rounded_div(rem, b) = sign(rem) since b/2 < |rem| < b  (linear_algebra ops.rs:64-80)
  int64_t sg = rem < 0 ? -1 : 1;
  curr = q + sg;
  return rem - sg * b;
}

}  // namespace lfk
