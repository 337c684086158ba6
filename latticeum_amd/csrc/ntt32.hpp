// ntt32.hpp -- 1024-point negacyclic Goldilocks NTT as a 32 x 32 four-step
// transform held in registers: half a wave (32 lanes) owns one ring element,
// each lane 32 values, so a wave transforms two elements with one LDS
// transpose and no workgroup barrier.
//
// Slot m of f is f(psi^(2m+1)), psi = 7^((p-1)/2048). With j = j1 + 32 j2 and
// m = m1 + 32 m2:
//   X[m1 + 32 m2] = sum_j1 w32^(m2 j1) * psi^((2m1+1) j1) * Y[j1][m1]
//   Y[j1][m1]     = sum_j2 x[j1 + 32 j2] * zeta^((2m1+1) j2)
// zeta = psi^32 = 2^39 (order 64) and w32 = psi^64 = 2^78 (order 32) are
// powers of two (checked when the tables are built), so both 32-point stages
// are shift-only; the only general products are the 1024 middle factors
// psi^((2m1+1) j1) (table `mid`). Stage 1 is the merged Cooley-Tukey network
// for X^32 + 1 (bit-reversed output), stage 2 a radix-2 DIF DFT (bit-reversed
// output); the inverse runs the DIF DFT with w32^-1, the middle factors
// d^-1 psi^-((2m1+1) j1), and the transposed (Gentleman-Sande) network with
// zeta^-1. Index model: tools/ntt32_model.py.
//
// Register/lane contract (r = lane & 31):
//   coefficient layout  v[j2] = x[r + 32 j2]                 (forward in / inverse out)
//   slot layout         v[i]  = X[r + 32 brv5(i)]            (forward out)
//   slot input          v[m2] = X[r + 32 m2]                 (inverse in)
#pragma once
#include "gl.hpp"

namespace n32 {

constexpr int RS = 33;                  // LDS row stride in u64 (conflict-free column reads)
constexpr int HALF_U64 = 32 * RS;       // LDS scratch per half-wave
constexpr int WAVE_U64 = 2 * HALF_U64;  // per wave

__host__ __device__ constexpr int brv5(int i) {
  return ((i & 1) << 4) | ((i & 2) << 2) | (i & 4) | ((i & 8) >> 2) | ((i & 16) >> 4);
}
// zeta^brv5(k) = 2^(39 brv5(k)); zeta^-1 = 2^153; w32 = 2^78, w32^-1 = 2^114
__host__ __device__ constexpr int zexp(int k, bool inv) { return ((inv ? 153 : 39) * brv5(k)) % 192; }
__host__ __device__ constexpr int wexp(int e, bool inv) { return ((inv ? 114 : 78) * e) % 192; }

// issue 32 row loads before the first use: the asm consumes the values in
// groups of 8, so the scheduler cannot interleave load -> wait -> use per value
__device__ __forceinline__ void load_row32(const uint64_t *p, uint64_t *v) {
#pragma unroll
  for (int k = 0; k < 32; k++) v[k] = p[32 * k];
#pragma unroll
  for (int k = 0; k < 32; k += 8)
    asm volatile("" : "+v"(v[k]), "+v"(v[k + 1]), "+v"(v[k + 2]), "+v"(v[k + 3]), "+v"(v[k + 4]), "+v"(v[k + 5]),
                 "+v"(v[k + 6]), "+v"(v[k + 7]));
}
__device__ __forceinline__ void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// forward merged CT network for X^32 + 1, levels [LV0, 5): natural in, bit-reversed out
template <int LV0 = 0>
__device__ __forceinline__ void neg_ct32(uint64_t *a) {
#pragma unroll
  for (int lv = LV0; lv < 5; lv++) {
    const int ln = 16 >> lv;
#pragma unroll
    for (int blk = 0; blk < (1 << lv); blk++) {
      const int k = (1 << lv) + blk, st = 2 * ln * blk;
#pragma unroll
      for (int j = st; j < st + ln; j++) {
        const int e = zexp(k, false);  // 2^e = -2^(e-96) for e >= 96: swap the add and the sub
        const uint64_t t = gl::shl96(a[j + ln], e % 96);
        const uint64_t lo = gl::sub(a[j], t), hi = gl::add(a[j], t);
        a[j + ln] = e < 96 ? lo : hi;
        a[j] = e < 96 ? hi : lo;
      }
    }
  }
}

// the transposed network with zeta^-1: bit-reversed in, natural out
__device__ __forceinline__ void neg_gs32_inv(uint64_t *a) {
#pragma unroll
  for (int lv = 4; lv >= 0; lv--) {
    const int ln = 16 >> lv;
#pragma unroll
    for (int blk = (1 << lv) - 1; blk >= 0; blk--) {
      const int k = (1 << lv) + blk, st = 2 * ln * blk;
#pragma unroll
      for (int j = st; j < st + ln; j++) {
        const uint64_t u = a[j], v = a[j + ln];
        const int e = zexp(k, true);
        a[j] = gl::add(u, v);
        a[j + ln] = gl::shl96(e < 96 ? gl::sub(u, v) : gl::sub(v, u), e % 96);
      }
    }
  }
}

// radix-2 DIF DFT of length 32 with w32^(+-1): natural in, bit-reversed out
template <bool INV>
__device__ __forceinline__ void cyc_dif32(uint64_t *a) {
#pragma unroll
  for (int lv = 0; lv < 5; lv++) {
    const int ln = 16 >> lv;
#pragma unroll
    for (int st = 0; st < 32; st += 2 * ln)
#pragma unroll
      for (int j = 0; j < ln; j++) {
        const uint64_t u = a[st + j], v = a[st + j + ln];
        a[st + j] = gl::add(u, v);
        const int e = wexp(j * (16 / ln), INV);
        a[st + j + ln] = gl::shl96(e < 96 ? gl::sub(u, v) : gl::sub(v, u), e % 96);
      }
  }
}

// first two CT levels for small signed inputs (|d| <= 1: balanced base-2
// digits), exact in int64 using 2^96 == -1 and 2^72 == 2^40 - 2^8; levels 3..5
// then run in the field. zeta^brv5(1) = 2^48, zeta^brv5(2) = 2^120 == -2^24,
// zeta^brv5(3) = 2^168 == -2^72, 2^216 == 2^24.
__device__ __forceinline__ uint64_t from_i64(int64_t x) { return x < 0 ? (uint64_t)x + gl::P : (uint64_t)x; }
__device__ __forceinline__ void neg_ct32_digits(const int32_t *dg, uint64_t *a) {
  constexpr int64_t S8_40 = (1ll << 8) - (1ll << 40);  // 2^72 mod p as a small signed value's negative
#pragma unroll
  for (int j = 0; j < 8; j++) {
    const int64_t d0 = dg[j], d1 = dg[j + 8], d2 = dg[j + 16], d3 = dg[j + 24];
    // level 1 (len 16, 2^48): v_j = d0 + 2^48 d2, v_{j+16} = d0 - 2^48 d2, v_{j+8} = d1 + 2^48 d3, ...
    // level 2, block 0 (2^120): t = 2^120 v_{j+8} = -2^24 d1 + (2^8 - 2^40) d3
    const int64_t t0 = -(d1 << 24) + S8_40 * d3;
    const int64_t v0 = d0 + (d2 << 48);
    // block 1 (2^168): t' = 2^168 v_{j+24} = (2^8 - 2^40) d1 - 2^24 d3
    const int64_t t1 = S8_40 * d1 - (d3 << 24);
    const int64_t v2 = d0 - (d2 << 48);
    a[j] = from_i64(v0 + t0);
    a[j + 8] = from_i64(v0 - t0);
    a[j + 16] = from_i64(v2 + t1);
    a[j + 24] = from_i64(v2 - t1);
  }
  neg_ct32<2>(a);
}

// transposes through this half-wave's LDS scratch (lds = base of the half's 32 x RS tile)
// forward: lane j1 holds m1 = brv5(i) in v[i]  ->  lane m1 holds j1 in v[j1]
__device__ __forceinline__ void transpose_fwd(uint64_t *v, uint64_t *lds, int r) {
#pragma unroll
  for (int i = 0; i < 32; i++) lds[brv5(i) * RS + r] = v[i];
  wave_lds_sync();
#pragma unroll
  for (int j = 0; j < 32; j++) v[j] = lds[r * RS + j];
  wave_lds_sync();
}
// inverse: lane m1 holds j1 = brv5(i) in v[i]  ->  lane j1 holds m1 = brv5(i) in v[i]
__device__ __forceinline__ void transpose_inv(uint64_t *v, uint64_t *lds, int r) {
#pragma unroll
  for (int i = 0; i < 32; i++) lds[brv5(i) * RS + r] = v[i];
  wave_lds_sync();
#pragma unroll
  for (int i = 0; i < 32; i++) v[i] = lds[r * RS + brv5(i)];
  wave_lds_sync();
}

// The same two transposes through a 32-bit tile (the low words, then the high
// words): half the LDS per half-wave, for kernels whose occupancy the LDS bounds
constexpr int HALF_U32 = 32 * RS;  // u32 scratch per half-wave
// (the transposed low words go into the low halves of v, which the first pass
// has already written out, so no extra registers)
__device__ __forceinline__ void transpose_fwd_w(uint64_t *v, uint32_t *lds, int r) {
#pragma unroll
  for (int i = 0; i < 32; i++) lds[brv5(i) * RS + r] = (uint32_t)v[i];
  wave_lds_sync();
#pragma unroll
  for (int j = 0; j < 32; j++) v[j] = (v[j] & 0xFFFFFFFF00000000ull) | lds[r * RS + j];  // new low, old high
  wave_lds_sync();
#pragma unroll
  for (int i = 0; i < 32; i++) lds[brv5(i) * RS + r] = (uint32_t)(v[i] >> 32);
  wave_lds_sync();
#pragma unroll
  for (int j = 0; j < 32; j++) v[j] = ((uint64_t)lds[r * RS + j] << 32) | (uint32_t)v[j];
  wave_lds_sync();
}
__device__ __forceinline__ void transpose_inv_w(uint64_t *v, uint32_t *lds, int r) {
#pragma unroll
  for (int i = 0; i < 32; i++) lds[brv5(i) * RS + r] = (uint32_t)v[i];
  wave_lds_sync();
#pragma unroll
  for (int i = 0; i < 32; i++) v[i] = (v[i] & 0xFFFFFFFF00000000ull) | lds[r * RS + brv5(i)];
  wave_lds_sync();
#pragma unroll
  for (int i = 0; i < 32; i++) lds[brv5(i) * RS + r] = (uint32_t)(v[i] >> 32);
  wave_lds_sync();
#pragma unroll
  for (int i = 0; i < 32; i++) v[i] = ((uint64_t)lds[r * RS + brv5(i)] << 32) | (uint32_t)v[i];
  wave_lds_sync();
}

// The two halves' rows to one element per lane: y0 / y1 hold elements 0 / 1 at
// rows j1 = (i & 3) + 8 (i >> 2) + 4 h; a half exchange (lanes 32-63 of the first
// operand with lanes 0-31 of the second) leaves lane (r, h) element h's rows
// j1 = .. in the first and j1 = .. + 4 in the second.
__device__ __forceinline__ void halves_to_elements(const uint64_t *y0, const uint64_t *y1, uint64_t *v) {
#pragma unroll
  for (int i = 0; i < 16; i++) {
    const auto lo = __builtin_amdgcn_permlane32_swap((uint32_t)y0[i], (uint32_t)y1[i], false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap((uint32_t)(y0[i] >> 32), (uint32_t)(y1[i] >> 32), false, false);
    const int j = (i & 3) + 8 * (i >> 2);
    v[j] = ((uint64_t)hi[0] << 32) | lo[0];
    v[j + 4] = ((uint64_t)hi[1] << 32) | lo[1];
  }
}

// middle factors: v[i] *= mid[r][i]. The 32 x 32 table is staged once per
// block into LDS as midT[i][r] (conflict-free column reads; LDS waits do not
// drain the wave's outstanding global stores the way a vmcnt wait would).
constexpr int MID_U64 = 1024;
__device__ __forceinline__ void stage_mid(uint64_t *midT, const uint64_t *mid) {
  for (int q = threadIdx.x; q < MID_U64; q += blockDim.x) {
    const int r = q >> 5, i = q & 31;
    midT[i * 32 + r] = mid[q];
  }
}
__device__ __forceinline__ void mul_mid(uint64_t *v, const uint64_t *midT, int r) {
  // reads issued 16 at a time before their products (two LDS waits, not 16)
#pragma unroll
  for (int i0 = 0; i0 < 32; i0 += 16) {
    uint64_t t[16];
#pragma unroll
    for (int i = 0; i < 16; i++) t[i] = midT[(i0 + i) * 32 + r];
#pragma unroll
    for (int i = 0; i < 16; i += 8)
      asm volatile("" : "+v"(t[i]), "+v"(t[i + 1]), "+v"(t[i + 2]), "+v"(t[i + 3]), "+v"(t[i + 4]), "+v"(t[i + 5]),
                   "+v"(t[i + 6]), "+v"(t[i + 7]));
#pragma unroll
    for (int i = 0; i < 16; i++) v[i0 + i] = gl::mul(v[i0 + i], t[i]);
  }
}

// forward from coefficient layout to slot layout (stage 1 done by the caller
// for digit inputs: pass STAGE1 = false)
template <bool STAGE1 = true>
__device__ __forceinline__ void forward(uint64_t *v, const uint64_t *mid, uint64_t *lds, int r) {
  if (STAGE1) neg_ct32(v);
  mul_mid(v, mid, r);
  transpose_fwd(v, lds, r);
  cyc_dif32<false>(v);
}
// forward / inverse with the 32-bit-tile transposes
__device__ __forceinline__ void forward_w(uint64_t *v, const uint64_t *mid, uint32_t *lds, int r) {
  neg_ct32(v);
  mul_mid(v, mid, r);
  transpose_fwd_w(v, lds, r);
  cyc_dif32<false>(v);
}
__device__ __forceinline__ void inverse_w(uint64_t *v, const uint64_t *mid_inv, uint32_t *lds, int r) {
  cyc_dif32<true>(v);
  mul_mid(v, mid_inv, r);
  transpose_inv_w(v, lds, r);
  neg_gs32_inv(v);
}
// inverse from slot input layout v[m2] = X[r + 32 m2] to coefficient layout
__device__ __forceinline__ void inverse(uint64_t *v, const uint64_t *mid_inv, uint64_t *lds, int r) {
  cyc_dif32<true>(v);
  mul_mid(v, mid_inv, r);
  transpose_inv(v, lds, r);
  neg_gs32_inv(v);
}

}  // namespace n32
