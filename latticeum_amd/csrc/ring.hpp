// ring.hpp -- device-side ring transforms for the two ring families.
//
//  * Phi_72 = X^24 - X^12 + 1 (the reference's Goldilocks ring, d = 24): CRT to
//    8 slots of Fq3, restating stark-rings goldilocks/ntt.rs:135-346. Every
//    root of unity in that file is a power of two (omega_24 = 2^40, 2^192 == 1),
//    so all twiddle products are shifts (gl::shl192);
//    only the ICRT's KAPPA (ntt.rs:43) is a general product.
//  * X^d + 1, d = 4^k (this project's negacyclic ring, no reference analogue):
//    slot k = f(psi^(2k+1)), psi = 7^((p-1)/2d), natural order. Radix-4
//    Stockham (self-sorting) DFT in LDS after a psi^j twist.
#pragma once
#include "gl.hpp"

namespace ring {

// omega_24^k = (2^40)^k = 2^(40k mod 192)
__host__ __device__ constexpr int W(int k) { return (40 * k) % 192; }
constexpr uint64_t KAPPA = 12297829382473034411ull;  // ntt.rs:43 literal (= 1/(2 w^4 - 1))

LF_HD uint64_t mw(uint64_t x, int k) { return gl::shl192(x, W(k)); }

// goldilocks/ntt.rs:326-334
LF_HD void phi72_homogenize(uint64_t *c) {
  uint64_t t;
  c[4] = gl::neg(c[4]);
  c[7] = mw(c[7], 2);
  c[8] = mw(c[8], 4);
  c[10] = mw(c[10], 6);
  c[11] = mw(c[11], 12);
  t = c[13];
  c[13] = mw(c[14], 3);
  c[14] = mw(t, 1);
  t = c[16];
  c[16] = mw(c[17], 11);
  c[17] = mw(t, 5);
  t = c[19];
  c[19] = mw(c[20], 7);
  c[20] = mw(t, 3);
  t = c[22];
  c[22] = mw(c[23], 15);
  c[23] = mw(t, 7);
}

// goldilocks/ntt.rs:338-346
LF_HD void phi72_dehomogenize(uint64_t *c) {
  uint64_t t;
  c[4] = gl::neg(c[4]);
  c[7] = mw(c[7], 22);
  c[8] = mw(c[8], 20);
  c[10] = mw(c[10], 18);
  c[11] = mw(c[11], 12);
  t = c[13];
  c[13] = mw(c[14], 23);
  c[14] = mw(t, 21);
  t = c[16];
  c[16] = mw(c[17], 19);
  c[17] = mw(t, 13);
  t = c[19];
  c[19] = mw(c[20], 21);
  c[20] = mw(t, 17);
  t = c[22];
  c[22] = mw(c[23], 17);
  c[23] = mw(t, 9);
}

// goldilocks/ntt.rs:135-228
LF_HD void phi72_crt(uint64_t *c) {
#pragma unroll
  for (int i = 0; i < 12; i++) {
    uint64_t a = c[i], b = c[12 + i];
    uint64_t zb = mw(b, 4);
    c[i] = gl::add(a, zb);
    c[12 + i] = gl::sub(gl::add(a, b), zb);
  }
#pragma unroll
  for (int i = 0; i < 6; i++) {
    uint64_t a = c[i], b = mw(c[6 + i], 2);
    c[i] = gl::add(a, b);
    c[6 + i] = gl::sub(a, b);
    a = c[12 + i];
    b = mw(c[18 + i], 10);
    c[12 + i] = gl::add(a, b);
    c[18 + i] = gl::sub(a, b);
  }
  constexpr int tw[4] = {1, 7, 5, 11};
#pragma unroll
  for (int q = 0; q < 4; q++)
#pragma unroll
    for (int i = 0; i < 3; i++) {
      uint64_t a = c[6 * q + i], b = mw(c[6 * q + 3 + i], tw[q]);
      c[6 * q + i] = gl::add(a, b);
      c[6 * q + 3 + i] = gl::sub(a, b);
    }
  phi72_homogenize(c);
}

// phi72_crt of a balanced ternary digit plane (digit i = sign bit i of ng,
// magnitude bit i of nz): the first level is exact in int64, since
// mw(b, 4) = 2^160 b == (1 - 2^32) b for b in {-1, 0, 1} (2^96 == -1,
// 2^64 == 2^32 - 1), so its 12 butterflies are integer adds instead of a
// shift and three canonical field operations each; the rest as phi72_crt
LF_HD void phi72_crt_ternary(uint32_t nz, uint32_t ng, uint64_t *c) {
#pragma unroll
  for (int i = 0; i < 12; i++) {
    const int64_t a = (nz >> i & 1) ? ((ng >> i & 1) ? -1 : 1) : 0;
    const int64_t b = (nz >> (12 + i) & 1) ? ((ng >> (12 + i) & 1) ? -1 : 1) : 0;
    const int64_t zb = b - b * ((int64_t)1 << 32);
    const int64_t lo = a + zb, hi = a + b - zb;  // |.| <= 2^32 + 2
    c[i] = lo < 0 ? (uint64_t)lo + gl::P : (uint64_t)lo;
    c[12 + i] = hi < 0 ? (uint64_t)hi + gl::P : (uint64_t)hi;
  }
#pragma unroll
  for (int i = 0; i < 6; i++) {
    uint64_t a = c[i], b = mw(c[6 + i], 2);
    c[i] = gl::add(a, b);
    c[6 + i] = gl::sub(a, b);
    a = c[12 + i];
    b = mw(c[18 + i], 10);
    c[12 + i] = gl::add(a, b);
    c[18 + i] = gl::sub(a, b);
  }
  constexpr int tw[4] = {1, 7, 5, 11};
#pragma unroll
  for (int q = 0; q < 4; q++)
#pragma unroll
    for (int i = 0; i < 3; i++) {
      uint64_t a = c[6 * q + i], b = mw(c[6 * q + 3 + i], tw[q]);
      c[6 * q + i] = gl::add(a, b);
      c[6 * q + 3 + i] = gl::sub(a, b);
    }
  phi72_homogenize(c);
}

// goldilocks/ntt.rs:240-319
LF_HD void phi72_icrt(uint64_t *c) {
  phi72_dehomogenize(c);
  constexpr int tw[4] = {23, 17, 19, 13};
#pragma unroll
  for (int q = 0; q < 4; q++)
#pragma unroll
    for (int i = 0; i < 3; i++) {
      uint64_t a = c[6 * q + i], b = c[6 * q + 3 + i];
      c[6 * q + i] = gl::add(a, b);
      c[6 * q + 3 + i] = mw(gl::sub(a, b), tw[q]);
    }
#pragma unroll
  for (int i = 0; i < 6; i++) {
    uint64_t a = c[i], b = c[6 + i];
    c[i] = gl::add(a, b);
    c[6 + i] = mw(gl::sub(a, b), 22);
    a = c[12 + i];
    b = c[18 + i];
    c[12 + i] = gl::add(a, b);
    c[18 + i] = mw(gl::sub(a, b), 14);
  }
#pragma unroll
  for (int i = 0; i < 12; i++) {
    uint64_t a = c[i], b = c[12 + i];
    uint64_t kd = gl::mul(KAPPA, gl::sub(a, b));
    c[i] = gl::shl192(gl::sub(gl::add(a, b), kd), 189);  // * 1/8 = 2^-3 = 2^189
    c[12 + i] = gl::shl192(kd, 190);                         // * 1/4 = 2^190
  }
}

// Toom-3 evaluation for the i8-MFMA Ajtai (ajtai_mfma.hip): virtual slot
// vs = 5 slot + t of a Phi_72 NTT element e (24 canonical u64, [s.c0, s.c1, s.c2]
// per slot) is the slot's polynomial c0 + c1 u + c2 u^2 at u = 0, 1, -1, 2, inf
__device__ __forceinline__ uint64_t phi72_eval(const uint64_t *e, int vs) {
  const int slot = vs / 5, t = vs - 5 * slot;
  const uint64_t a0 = e[3 * slot], a1 = e[3 * slot + 1], a2 = e[3 * slot + 2];
  switch (t) {
    case 0: return a0;
    case 1: return gl::add(gl::add(a0, a1), a2);
    case 2: return gl::add(gl::sub(a0, a1), a2);
    case 3: return gl::add(gl::add(a0, gl::add(a1, a1)), gl::shl96(a2, 2));
    default: return a2;
  }
}

// Fq3 slot multiply-accumulate into lazy accumulators:
//   c0 = sum a0b0 + 2^40 * sum(a1b2 + a2b1)
//   c1 = sum(a0b1 + a1b0) + 2^40 * sum a2b2
//   c2 = sum(a0b2 + a1b1 + a2b0)
struct Fq3Acc {
  gl::Acc s00, s0n, s1, s1n, s2;
};
__device__ __forceinline__ void fq3acc_zero(Fq3Acc &a) {
  gl::acc_zero(a.s00);
  gl::acc_zero(a.s0n);
  gl::acc_zero(a.s1);
  gl::acc_zero(a.s1n);
  gl::acc_zero(a.s2);
}
__device__ __forceinline__ void fq3acc_mad(Fq3Acc &s, uint64_t a0, uint64_t a1, uint64_t a2,
                                           uint64_t b0, uint64_t b1, uint64_t b2) {
  gl::acc_mad(s.s00, a0, b0);
  gl::acc_mad(s.s0n, a1, b2);
  gl::acc_mad(s.s0n, a2, b1);
  gl::acc_mad(s.s1, a0, b1);
  gl::acc_mad(s.s1, a1, b0);
  gl::acc_mad(s.s1n, a2, b2);
  gl::acc_mad(s.s2, a0, b2);
  gl::acc_mad(s.s2, a1, b1);
  gl::acc_mad(s.s2, a2, b0);
}
__device__ __forceinline__ void fq3acc_final(const Fq3Acc &s, uint64_t *c) {
  c[0] = gl::add(gl::acc_reduce(s.s00), gl::shl96(gl::acc_reduce(s.s0n), 40));
  c[1] = gl::add(gl::acc_reduce(s.s1), gl::shl96(gl::acc_reduce(s.s1n), 40));
  c[2] = gl::acc_reduce(s.s2);
}

// ---------------------------------------------------------------- negacyclic
struct NegaTables {
  const uint64_t *twist;      // fwd: psi^j ; inv: d^-1 psi^-j
  const uint64_t *roots;      // fwd: omega^e ; inv: omega^-e   (omega = psi^2), e < d
  const uint64_t *mid;        // d = 1024 only: 32 x 32 middle factors of the four-step NTT (ntt32.hpp)
                              // (d = 4096: those of its 1024-point sub-transforms, kernels_n4k.hip)
  const uint64_t *tw4 = nullptr;   // d = 4096: radix-4 twists [m0][a] (fwd psi^((2m0-3)a), inv 4^-1 psi^-((2m0-3)a))
  const uint64_t *ztab = nullptr;  // d = 4096 fwd: butterflies of four balanced bits [m0][nibble | signs << 4]
  const uint64_t *az = nullptr;    // d = 1024 fwd: D8 byte planes of zeta^((2 m1 + 1) j2), int8 [8][32][32]
  // d = 4096 fwd, stage 1 of each quarter m0 on the matrix cores (kernels_n4k.hip k_decompose_n4k_mx):
  const uint64_t *zq = nullptr;    // D8 byte planes of Z''_m0[m1][32 b + j2], int8 [4][8][32][128]
  const uint64_t *midq = nullptr;  // middle factors with the j1 twist, [4][j1 32][brv5(m1) 32]
};

// Radix-4 Stockham DFT of size D over LDS buffers x -> y (ping-pong), T threads.
// Returns the buffer holding the result. Caller has already applied the twist
// (forward) and applies the inverse twist afterwards (inverse). The 4th root
// omega^(D/4) = 7^((p-1)/4) = 2^48 for every D (checked when the tables are
// built), so that factor is a shift; the inverse uses 2^-48 = 2^144.
template <int D, int T, bool INV>
__device__ __forceinline__ uint64_t *stockham4(uint64_t *x, uint64_t *y, const uint64_t *roots,
                                               int tid) {
  constexpr int E4 = INV ? 144 : 48;
#pragma unroll 1
  for (int p = 1; p < D; p <<= 2) {
    const int s = D / (4 * p);
#pragma unroll
    for (int i = tid; i < D / 4; i += T) {
      const int k = i & (p - 1);
      uint64_t a0 = x[i], a1 = x[i + D / 4], a2 = x[i + D / 2], a3 = x[i + 3 * D / 4];
      if (p > 1) {
        a1 = gl::mul(a1, roots[s * k]);
        a2 = gl::mul(a2, roots[2 * s * k]);
        a3 = gl::mul(a3, roots[3 * s * k]);
      }
      uint64_t t0 = gl::add(a0, a2), t1 = gl::sub(a0, a2);
      uint64_t t2 = gl::add(a1, a3), t3 = gl::mul_pow2(gl::sub(a1, a3), E4);
      const int j = ((i - k) << 2) + k;
      y[j] = gl::add(t0, t2);
      y[j + p] = gl::add(t1, t3);
      y[j + 2 * p] = gl::sub(t0, t2);
      y[j + 3 * p] = gl::sub(t1, t3);
    }
    __syncthreads();
    uint64_t *t = x;
    x = y;
    y = t;
  }
  return x;
}

}  // namespace ring
