// gl.hpp -- Goldilocks field arithmetic for gfx950 (and the host side of the
// library). p = 2^64 - 2^32 + 1 (reference: stark-rings goldilocks/mod.rs:16-27).
//
// Device representation is canonical u64 in [0, p). Internally a value may be
// carried "weakly reduced" (any u64, congruent mod p); gl_canon() fixes it.
// Reduction uses 2^64 == 2^32 - 1 and 2^96 == -1 (mod p), so a 128-bit product
// folds into 64 bits with two 32-bit pieces and two carry fix-ups.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define LF_HD __host__ __device__ __forceinline__

namespace gl {

constexpr uint64_t P = 0xFFFFFFFF00000001ull;
constexpr uint64_t EPS = 0xFFFFFFFFull;  // 2^64 mod p

LF_HD uint64_t canon(uint64_t x) {  // x >= p  <=>  x + EPS carries; then x - p == x + EPS
  uint64_t u;
  return __builtin_uaddll_overflow(x, EPS, reinterpret_cast<unsigned long long *>(&u)) ? u : x;
}

// a + b with the carry out (lowers to one 64-bit add + carry compare on gfx950)
LF_HD bool addc64(uint64_t a, uint64_t b, uint64_t &r) {
  return __builtin_uaddll_overflow(a, b, reinterpret_cast<unsigned long long *>(&r));
}
LF_HD bool subb64(uint64_t a, uint64_t b, uint64_t &r) {
  return __builtin_usubll_overflow(a, b, reinterpret_cast<unsigned long long *>(&r));
}

LF_HD uint64_t add(uint64_t a, uint64_t b) {  // canonical in -> canonical out
  // t = a + b; the result is t - p exactly when a + b >= p, i.e. when the sum
  // carried out of 64 bits (t - p = t + EPS) or t + EPS carries (t >= p)
  uint64_t t, u;
  const bool c1 = addc64(a, b, t);
  const bool c2 = addc64(t, EPS, u);
  return (c1 | c2) ? u : t;
}

LF_HD uint64_t sub(uint64_t a, uint64_t b) {  // canonical in -> canonical out
#if defined(__HIP_DEVICE_COMPILE__)
  // on a 32-bit borrow chain, so the borrow out is the chain's own (no compare)
  unsigned int b1, b2;
  const uint32_t dl = __builtin_subc((uint32_t)a, (uint32_t)b, 0u, &b1);
  const uint32_t dh = __builtin_subc((uint32_t)(a >> 32), (uint32_t)(b >> 32), b1, &b2);
  const uint64_t d = ((uint64_t)dh << 32) | dl;
  return b2 ? d - EPS : d;
#else
  uint64_t d;
  const bool br = subb64(a, b, d);
  return br ? d - EPS : d;  // borrow: d wrapped by +2^64 == +EPS, remove it
#endif
}

LF_HD uint64_t neg(uint64_t a) { return a ? P - a : 0; }

// X + Y 2^32 (mod p), canonical, for signed |X|, |Y| < 2^62 (the i8-MFMA epilogues' quarter
// sums): Y 2^32 = yh 2^64 + yl 2^32 == yh (2^32 - 1) + yl 2^32 (yh = Y >> 32), and
// U = yl + yh = c 2^32 + ul (c in {-1, 0, 1}) folds the same way, leaving V + ul 2^32 with
// V = X - yh + c (2^32 - 1); that 65-bit sum is t + k 2^64 with k = carry - [V < 0],
// == t + k (2^32 - 1) without wrapping (t < 2^63 when k = 1, t > 2^63 when k = -1)
LF_HD uint64_t from_x_y32(int64_t X, int64_t Y) {
  const int64_t yh = Y >> 32;
  const int64_t U = (int64_t)(uint32_t)Y + yh;
  const int64_t c = U >> 32;
  const int64_t V = X - yh + c * (int64_t)EPS;
  uint64_t t;
  const int k = (int)addc64((uint64_t)V, (uint64_t)(uint32_t)U << 32, t) - (V < 0);
  return canon(t + (uint64_t)((int64_t)k * (int64_t)EPS));
}

// 64x64 -> 128 from four 32x32 -> 64 multiply-adds (v_mad_u64_u32 each; no
// intermediate sum overflows: (2^32-1)^2 + 2 (2^32-1) = 2^64 - 1)
LF_HD void mul_wide(uint64_t a, uint64_t b, uint64_t &lo, uint64_t &hi) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t a0 = (uint32_t)a, a1 = (uint32_t)(a >> 32), b0 = (uint32_t)b, b1 = (uint32_t)(b >> 32);
  const uint64_t p0 = (uint64_t)a0 * b0;
  const uint64_t t = (uint64_t)a0 * b1 + (p0 >> 32);
  const uint64_t u = (uint64_t)a1 * b0 + (uint32_t)t;
  hi = (uint64_t)a1 * b1 + (t >> 32) + (u >> 32);
  lo = (u << 32) | (uint32_t)p0;
#else
  unsigned __int128 t = (unsigned __int128)a * b;
  lo = (uint64_t)t;
  hi = (uint64_t)(t >> 64);
#endif
}

// x = lo + 2^64 hi  ->  weakly reduced u64 congruent to x:
//   hi = h0 + 2^32 h1:  x == lo + h0 (2^32 - 1) - h1   (2^64 == EPS, 2^96 == -1)
LF_HD uint64_t reduce128(uint64_t lo, uint64_t hi) {
  const uint64_t h0 = hi & EPS, h1 = hi >> 32;
  uint64_t r, s;
  if (addc64(lo, h0 * EPS, r)) r += EPS;  // r + EPS < 2^64 after a carry
  if (subb64(r, h1, s)) s -= EPS;         // s >= p after a borrow
  return s;
}

LF_HD uint64_t mul(uint64_t a, uint64_t b) {
  uint64_t lo, hi;
  mul_wide(a, b, lo, hi);
  return canon(reduce128(lo, hi));
}

// multiply by 2^s, 0 <= s < 192, any u64 input; canonical output.
// 2^96 == -1, so 2^s for s in [96,192) is -(2^(s-96)); 2^128 == -2^32.
LF_HD uint64_t mul_pow2(uint64_t a, int s) {
  bool negate = s >= 96;
  if (negate) s -= 96;
  uint64_t r;
  if (s < 64) {
    uint64_t lo = s ? (a << s) : a, hi = s ? (a >> (64 - s)) : 0;
    r = canon(reduce128(lo, hi));
  } else {  // a*2^s = (a<<t)*2^64 with t = s-64 < 32: limbs [0, lo, hi<2^32]
    int t = s - 64;
    uint64_t lo = t ? (a << t) : a, hi = t ? (a >> (64 - t)) : 0;
    r = sub(canon(reduce128(0, lo)), canon(hi << 32));
  }
  return negate ? neg(r) : r;
}

// x 2^s for canonical x and 0 <= s < 96, canonical result, written for shift
// amounts that fold to constants (NTT twiddles). For 32 <= s < 96, with the
// 32-bit limbs of the 96-bit product, 2^64 == 2^32 - 1 and 2^96 == -1 turn the
// reduction into one subtraction from a value <= p - 1 and one borrow fix,
// written on 32-bit carry chains (12-14 VALU instead of 21 for mul_pow2).
// Callers fold s >= 96 (a negation) into their add/sub.
LF_HD uint64_t shl96(uint64_t x, int s) {
  const uint32_t x0 = (uint32_t)x, x1 = (uint32_t)(x >> 32);
  uint64_t r;
  bool br;
  if (s == 0) return x;  // x is canonical (a twiddle of 2^0 or 2^96 costs only the add/sub swap)
  if (s < 32) {
    // x 2^s = lo + 2^64 hi == lo + hi EPS with hi < 2^s, and lo + hi EPS < 2p.
    // t = lo + EPS (hi + 1) = (lo + hi EPS) + 2^64 - p: with a carry out, t mod
    // 2^64 is the reduced value; without one, lo + hi EPS = t - EPS < p.
    const uint64_t lo = x << s;
    const uint64_t nq = (x >> (64 - s)) * EPS + EPS;  // one v_mad_u64_u32
    unsigned int c1, c2;
    const uint32_t tl = __builtin_addc((uint32_t)lo, (uint32_t)nq, 0u, &c1);
    const uint32_t th = __builtin_addc((uint32_t)(lo >> 32), (uint32_t)(nq >> 32), c1, &c2);
    const uint64_t t = ((uint64_t)th << 32) | tl;
    return c2 ? t : t + P;  // t + P == t - EPS mod 2^64
  }
  if (s < 64) {
    // y = x 2^(s-32); x 2^s = y 2^32 == (y0 + y1) 2^32 - (y1 + y2)
    const int u = s - 32;
    const uint32_t y0 = u ? x0 << u : x0, y1 = u ? (uint32_t)(x >> (32 - u)) : x1, y2 = u ? x1 >> (32 - u) : 0;
    // on 32-bit carry chains: H = y0 + y1 + c (no wrap: y0 has u low zero bits,
    // and x < p), L = y1 + y2 + c = Lh 2^32 + Ll; r = H 2^32 - L
    unsigned int c, lh, b1, b2;
    const uint32_t al = __builtin_addc(y0, y1, 0u, &c);
    const uint32_t ll = __builtin_addc(y1, y2, c, &lh);
    const uint32_t rl = __builtin_subc(0u, ll, 0u, &b1);
    const uint32_t rh = __builtin_subc(al + c, lh, b1, &b2);
    r = ((uint64_t)rh << 32) | rl;
    br = b2;
  } else {
    // a division: 2^s = 2^96 2^-k == -2^-k with k = 96 - s in (0, 32]. Splitting
    // x = (x >> k) 2^k + xl, and 2^-k == -2^(96-k) == 2^(32-k) - 2^(64-k):
    //   x 2^-k == (x >> k) + xl 2^(32-k) - xl 2^(64-k) = D - B,
    // D = (x >> k) + C, C = xl 2^(32-k) = (u32)x << (32-k) < 2^32, B = C 2^32.
    // So x 2^s == B - D = C (2^32 - 1) - (x >> k): one 32 x 32 multiply and a
    // 64-bit subtraction. Without a borrow the result is <= C (2^32 - 1) < p;
    // with one, x >> k < 2^63 < p and adding p lands in (0, p). Canonical for
    // any u64 x.
    const int k = 96 - s;
    const uint32_t C = x0 << (32 - k);
    const uint64_t m = (uint64_t)C * EPS, a = x >> k;
    unsigned int b1, b2;
    const uint32_t rl = __builtin_subc((uint32_t)m, (uint32_t)a, 0u, &b1);
    const uint32_t rh = __builtin_subc((uint32_t)(m >> 32), (uint32_t)(a >> 32), b1, &b2);
    r = ((uint64_t)rh << 32) | rl;
    br = b2;
  }
  return br ? r + P : r;
}

// Weakly reduced Horner pieces: any u64 in, a u64 congruent mod p out (the
// caller canonicalises once at the end).
// x 2^s for 0 < s < 32: x 2^s = lo + 2^64 hi, hi < 2^s, and 2^64 == EPS. A
// carry out of lo + hi EPS leaves t < hi EPS < 2^63, so t + EPS cannot wrap.
LF_HD uint64_t shl_small_weak(uint64_t x, int s) {
  const uint64_t lo = x << s;
  const uint64_t hi = x >> (64 - s);
  uint64_t t;
  const bool c = addc64(lo, hi * EPS, t);
  return c ? t + EPS : t;
}
// a (any u64) + b (canonical): after a carry t = a + b - 2^64 < b < p, so t + EPS cannot wrap
LF_HD uint64_t add_weak(uint64_t a, uint64_t b) {
  uint64_t t;
  const bool c = addc64(a, b, t);
  return c ? t + EPS : t;
}

// x 2^e for canonical x and a constant 0 <= e < 192 (2^96 == -1): the
// shl96 forms plus a negation, against mul_pow2's generic 128-bit fold
LF_HD uint64_t shl192(uint64_t x, int e) { return e < 96 ? shl96(x, e) : neg(shl96(x, e - 96)); }

LF_HD uint64_t pow(uint64_t a, uint64_t e) {
  uint64_t r = 1;
  while (e) {
    if (e & 1) r = mul(r, a);
    a = mul(a, a);
    e >>= 1;
  }
  return r;
}
LF_HD uint64_t inv(uint64_t a) { return pow(a, P - 2); }

// ark-ff Montgomery limb <-> canonical (R = 2^64 mod p = EPS)
LF_HD uint64_t to_mont(uint64_t a) { return mul(a, EPS); }
constexpr uint64_t R_INV = 0xFFFFFFFE00000001ull;  // (2^32 - 1)^-1 mod p
LF_HD uint64_t from_mont(uint64_t m) { return mul(canon(m), R_INV); }

// ---- Fq3 = Fq[u]/(u^3 - 2^40)  (reference goldilocks/mod.rs:34-54) ----
LF_HD void fq3_mul(const uint64_t *a, const uint64_t *b, uint64_t *c) {
  uint64_t a0 = a[0], a1 = a[1], a2 = a[2], b0 = b[0], b1 = b[1], b2 = b[2];
  uint64_t t0 = add(mul(a1, b2), mul(a2, b1));
  uint64_t c0 = add(mul(a0, b0), mul_pow2(t0, 40));
  uint64_t c1 = add(add(mul(a0, b1), mul(a1, b0)), mul_pow2(mul(a2, b2), 40));
  uint64_t c2 = add(add(mul(a0, b2), mul(a1, b1)), mul(a2, b0));
  c[0] = c0;
  c[1] = c1;
  c[2] = c2;
}

// ---- lazy 128-bit multiply-accumulate: acc = sum of a_i*b_i as
// (lo:64, hi:64, top:32) -- reduce once at the end ----
struct Acc {
  uint64_t lo, hi;
  uint32_t top;
};
LF_HD void acc_zero(Acc &s) {
  s.lo = 0;
  s.hi = 0;
  s.top = 0;
}
LF_HD void acc_mad(Acc &s, uint64_t a, uint64_t b) {
  uint64_t lo, hi;
  mul_wide(a, b, lo, hi);
  uint64_t nlo = s.lo + lo;
  hi += (nlo < lo) ? 1 : 0;  // hi <= 2^64-2 so no wrap
  s.lo = nlo;
  uint64_t nhi = s.hi + hi;
  s.top += (nhi < hi) ? 1 : 0;
  s.hi = nhi;
}
LF_HD void acc_add(Acc &s, uint64_t v) {
  uint64_t nlo = s.lo + v;
  uint64_t c = (nlo < v) ? 1 : 0;
  s.lo = nlo;
  uint64_t nhi = s.hi + c;
  s.top += (nhi < c) ? 1 : 0;
  s.hi = nhi;
}
// value = lo + 2^64 hi + 2^128 top;  2^128 == (2^64)^2 == EPS^2 == 2^64 - 2^33 + 1 == -2^32 (mod p)
LF_HD uint64_t acc_reduce(const Acc &s) {
  uint64_t r = canon(reduce128(s.lo, s.hi));
  uint64_t t = canon(((uint64_t)s.top) << 32);
  return sub(r, t);
}

// ---- column accumulator: sum of 64x64-bit products kept as
//   S0 + 2^64 c0  (sum a0*b0)  +  2^32 (S1 + 2^64 c1)  (sum a0*b1 + a1*b0)
//   + 2^64 (S2 + 2^64 c2)  (sum a1*b1)
// On the device each 32x32 partial product is one v_mad_u64_u32 whose carry-out
// feeds a v_addc_co_u32 counter: 8 VALU instructions per multiply-accumulate
// (the compiler's own lowering of a*b / __umul64hi needs ~22).
struct CAcc {
  uint64_t s0, s1, s2;
  uint32_t c0, c1, c2;
};
LF_HD void cacc_zero(CAcc &a) {
  a.s0 = a.s1 = a.s2 = 0;
  a.c0 = a.c1 = a.c2 = 0;
}
LF_HD void cacc_mad(CAcc &a, uint64_t x, uint64_t y) {
  uint32_t x0 = (uint32_t)x, x1 = (uint32_t)(x >> 32), y0 = (uint32_t)y, y1 = (uint32_t)(y >> 32);
#if defined(__HIP_DEVICE_COMPILE__)
  uint64_t cc;
  asm(
      "v_mad_u64_u32 %0, %6, %7, %9, %0\n\t"
      "v_addc_co_u32_e64 %3, %6, 0, %3, %6\n\t"
      "v_mad_u64_u32 %1, %6, %7, %10, %1\n\t"
      "v_addc_co_u32_e64 %4, %6, 0, %4, %6\n\t"
      "v_mad_u64_u32 %1, %6, %8, %9, %1\n\t"
      "v_addc_co_u32_e64 %4, %6, 0, %4, %6\n\t"
      "v_mad_u64_u32 %2, %6, %8, %10, %2\n\t"
      "v_addc_co_u32_e64 %5, %6, 0, %5, %6"
      : "+v"(a.s0), "+v"(a.s1), "+v"(a.s2), "+v"(a.c0), "+v"(a.c1), "+v"(a.c2), "=&s"(cc)
      : "v"(x0), "v"(x1), "v"(y0), "v"(y1));
#else
  auto addc = [](uint64_t &s, uint32_t &c, uint64_t p) {
    s += p;
    c += s < p;
  };
  addc(a.s0, a.c0, (uint64_t)x0 * y0);
  addc(a.s1, a.c1, (uint64_t)x0 * y1);
  addc(a.s1, a.c1, (uint64_t)x1 * y0);
  addc(a.s2, a.c2, (uint64_t)x1 * y1);
#endif
}
// mod p: 2^64 == EPS, 2^96 == -1, 2^128 == -2^32
// V = s0 + s1 2^32 + (s2 + c0) 2^64 + c1 2^96 + c2 2^128, first normalised into
// 32-bit limbs x0 .. x4 (one carry chain), then with 2^64 == 2^32 - 1, 2^96 == -1,
// 2^128 == -2^32:  V == (x1:x0) + x2 2^32 - x4 2^32 - (x2 + x3), three 64-bit
// steps with one carry/borrow fix each and a final canonicalisation (about 30 VALU
// against 70 for the term-by-term fold, cacc_reduce_terms)
// (written on 32-bit carry chains: the compiler's 64-bit lowering of the same sums
// zero-extends every limb with moves)
LF_HD uint64_t cacc_reduce_weak(const CAcc &a);
LF_HD uint64_t cacc_reduce(const CAcc &a) { return canon(cacc_reduce_weak(a)); }
// the same fold without the final canonicalisation: any u64 congruent to V (for
// products that feed further products, which accept any u64 on this side)
LF_HD uint64_t cacc_reduce_weak(const CAcc &a) {
  const uint32_t s0l = (uint32_t)a.s0, s0h = (uint32_t)(a.s0 >> 32), s1l = (uint32_t)a.s1,
                 s1h = (uint32_t)(a.s1 >> 32), s2l = (uint32_t)a.s2, s2h = (uint32_t)(a.s2 >> 32);
  unsigned int k1, ka, kb, kc, kd;
  const uint32_t x1 = __builtin_addc(s0h, s1l, 0u, &k1);
  const uint32_t y = __builtin_addc(s1h, s2l, k1, &ka);
  const uint32_t x2 = __builtin_addc(y, a.c0, 0u, &kb);
  const uint32_t z = __builtin_addc(s2h, a.c1, ka, &kc);
  const uint32_t x3 = __builtin_addc(z, 0u, kb, &kd);
  const uint32_t x4 = a.c2 + kc + kd;  // a small count
  // u = (x1 : s0l) + x2 2^32; a carry is 2^64 == EPS (u < 2^64 - 2^32 then, no second carry)
  unsigned int c, c2, b, b2, b3, b4;
  uint32_t uh = __builtin_addc(x1, x2, 0u, &c);
  uint32_t ul = __builtin_addc(s0l, 0u - c, 0u, &c2);
  uh = __builtin_addc(uh, 0u, c2, &c2);
  // v = u - x4 2^32; a borrow is -EPS (v >= 2^64 - 2^32 x4 > EPS then)
  uint32_t vh = __builtin_subc(uh, x4, 0u, &b);
  uint32_t vl = __builtin_subc(ul, 0u - b, 0u, &b2);
  vh = __builtin_subc(vh, 0u, b2, &b2);
  // w = v - (x2 + x3); a borrow is -EPS (w >= 2^64 - 2^33 then)
  unsigned int sc;
  const uint32_t sl = __builtin_addc(x2, x3, 0u, &sc);
  uint32_t wl = __builtin_subc(vl, sl, 0u, &b3);
  uint32_t wh = __builtin_subc(vh, sc, b3, &b3);
  wl = __builtin_subc(wl, 0u - b3, 0u, &b4);
  wh = __builtin_subc(wh, 0u, b4, &b4);
  return ((uint64_t)wh << 32) | wl;
}
LF_HD uint64_t cacc_reduce_terms(const CAcc &a) {
  uint64_t r = canon(a.s0);
  r = add(r, canon((uint64_t)a.c0 * EPS));                      // c0 2^64
  uint64_t s1l = a.s1 & EPS, s1h = a.s1 >> 32;                 // S1 2^32 = s1l 2^32 + s1h 2^64
  r = add(r, canon(s1l << 32));
  r = add(r, canon(s1h * EPS));
  r = sub(r, canon((uint64_t)a.c1));                           // c1 2^96 = -c1
  r = add(r, canon(reduce128(0, a.s2)));                       // S2 2^64
  r = sub(r, canon((uint64_t)a.c2 << 32));                     // c2 2^128 = -c2 2^32
  return r;
}

}  // namespace gl
