// ntt1024.hpp -- one-wavefront 1024-point Goldilocks DFT for X^1024 + 1.
//
// One wave (64 lanes x 16 values) computes X[k] = sum_j x[j] w^(jk), w = psi^2
// a primitive 1024th root, in natural order, with no workgroup barriers:
//   1024 = 16 (registers) x 64 (lanes);  64 = 16 (registers) x 4 (lanes).
// pass 1: per lane t, 16-point DFT over x[t + 64 i]; twiddle w^(t k2)  (general)
// pass 2: per (k2, t1), 16-point DFT over z[t1 + 4 t2]; twiddle w64^(t1 m2) (shift)
// pass 3: per (k2, q), four 4-point DFTs over t1 (shift)
// Every root of order <= 64 is a power of two for this psi (w16 = 2^156,
// w64 = 2^39, w4 = 2^48; checked at context creation), so only the 1024
// pass-1 twiddles need a general 64x64 product. The two transposes go
// through a per-wave LDS tile (no s_barrier; a wave's LDS ops are in order).
//
// Lane contract (lane = threadIdx.x & 63):
//   input  v[i]          = x[lane + 64 i]                          i < 16
//   output v[4 r + m1]   = X[256 m1 + 16 (4 q + r) + k2]           k2 = lane >> 2, q = lane & 3
#pragma once
#include "gl.hpp"

namespace n1k {

constexpr int LDS_U64 = 16 * 68;  // per-wave scratch (rows padded 64 -> 68: conflict-free)

__host__ __device__ constexpr int out_index(int lane, int reg) {
  // position of output register `reg` of lane `lane`
  return 256 * (reg & 3) + 16 * (4 * (lane & 3) + (reg >> 2)) + (lane >> 2);
}

__device__ __forceinline__ void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

template <int E4>
__device__ __forceinline__ void dft4(uint64_t &a0, uint64_t &a1, uint64_t &a2, uint64_t &a3) {
  uint64_t t0 = gl::add(a0, a2), t1 = gl::sub(a0, a2), t2 = gl::add(a1, a3);
  uint64_t t3 = gl::mul_pow2(gl::sub(a1, a3), E4);
  a0 = gl::add(t0, t2);
  a1 = gl::add(t1, t3);
  a2 = gl::sub(t0, t2);
  a3 = gl::sub(t1, t3);
}

// 16-point DFT, natural order in and out, root 2^E16 (E4 = 4 E16 mod 192)
template <int E16>
__device__ __forceinline__ void dft16(uint64_t *v) {
  constexpr int E4 = (4 * E16) % 192;
  // i = i1 + 4 i2: 4-point DFTs over i2 -> y[i1][k2] kept at v[i1 + 4 k2]
#pragma unroll
  for (int i1 = 0; i1 < 4; i1++) dft4<E4>(v[i1], v[i1 + 4], v[i1 + 8], v[i1 + 12]);
  // twiddle w16^(i1 k2)
#pragma unroll
  for (int i1 = 1; i1 < 4; i1++)
#pragma unroll
    for (int k2 = 1; k2 < 4; k2++) v[i1 + 4 * k2] = gl::mul_pow2(v[i1 + 4 * k2], (E16 * i1 * k2) % 192);
  // 4-point DFTs over i1 -> X[4 k1 + k2] at v[4 k2 + k1]
#pragma unroll
  for (int k2 = 0; k2 < 4; k2++) dft4<E4>(v[4 * k2], v[4 * k2 + 1], v[4 * k2 + 2], v[4 * k2 + 3]);
  // transpose register indices so that v[n] = X[n]
  uint64_t t[16];
#pragma unroll
  for (int k1 = 0; k1 < 4; k1++)
#pragma unroll
    for (int k2 = 0; k2 < 4; k2++) t[4 * k1 + k2] = v[4 * k2 + k1];
#pragma unroll
  for (int n = 0; n < 16; n++) v[n] = t[n];
}

// tw1[k2] = w^(lane k2) (forward) or w^-(lane k2) (inverse); lds = this wave's LDS_U64 scratch
template <bool INV>
__device__ __forceinline__ void dft1024(uint64_t *v, const uint64_t *tw1, uint64_t *lds, int lane) {
  constexpr int E16 = INV ? 36 : 156, E64 = INV ? 153 : 39;
  dft16<E16>(v);
#pragma unroll
  for (int k2 = 1; k2 < 16; k2++) v[k2] = gl::mul(v[k2], tw1[k2]);
#pragma unroll
  for (int k2 = 0; k2 < 16; k2++) lds[k2 * 68 + lane] = v[k2];
  wave_lds_sync();
  const int k2 = lane >> 2, t1 = lane & 3;
#pragma unroll
  for (int t2 = 0; t2 < 16; t2++) v[t2] = lds[k2 * 68 + t1 + 4 * t2];
  wave_lds_sync();
  dft16<E16>(v);
#pragma unroll
  for (int m2 = 1; m2 < 16; m2++) v[m2] = gl::mul_pow2(v[m2], (E64 * t1 * m2) % 192);
#pragma unroll
  for (int m2 = 0; m2 < 16; m2++) lds[k2 * 68 + 4 * m2 + t1] = v[m2];
  wave_lds_sync();
  const int q = lane & 3;
  const uint64_t *src = lds + k2 * 68 + 16 * q;
#pragma unroll
  for (int n = 0; n < 16; n++) v[n] = src[n];  // v[4 r + t1'] = c[m2 = 4q + r][t1']
  wave_lds_sync();
  constexpr int E4 = (16 * E64) % 192;
#pragma unroll
  for (int r = 0; r < 4; r++) dft4<E4>(v[4 * r], v[4 * r + 1], v[4 * r + 2], v[4 * r + 3]);
  // v[4 r + m1] = X[16 (16 m1 + 4 q + r) + k2] = X[out_index(lane, 4 r + m1)]
}

}  // namespace n1k
