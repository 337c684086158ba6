#include <cstdint>
#include <cstdio>
#include <cstring>
#include <chrono>
#include "gl.hpp"
namespace {
#include "p2_consts.inc"
const uint64_t EXT_INIT[64] = LF_P2_EXT_INIT;
const uint64_t EXT_TERM[64] = LF_P2_EXT_TERM;
const uint64_t INTERNAL[22] = LF_P2_INTERNAL;
const uint64_t DIAG_M1[16] = LF_P2_DIAG_M1;
inline uint64_t wadd(uint64_t a, uint64_t b) {  // any u64 in and out
#if defined(__x86_64__)
  uint64_t m;
  // a + b; a carry wrapped by 2^64 == EPS: + EPS, which can carry once more (then the sum is < EPS)
  asm("addq %[b], %[a]\n\tsbbq %[m], %[m]\n\tmovl %k[m], %k[m]\n\taddq %[m], %[a]\n\t"
      "sbbq %[m], %[m]\n\tmovl %k[m], %k[m]\n\taddq %[m], %[a]"
      : [a] "+r"(a), [m] "=&r"(m)
      : [b] "r"(b)
      : "cc");
  return a;
#else
  uint64_t s, t;
  const uint64_t c = __builtin_add_overflow(a, b, &s);
  const uint64_t c2 = __builtin_add_overflow(s, c * gl::EPS, &t);
  return t + c2 * gl::EPS;
#endif
}
inline uint64_t wmul(uint64_t a, uint64_t b) {  // any u64 in and out
  const unsigned __int128 t = (unsigned __int128)a * b;
  uint64_t r = (uint64_t)t;
  const uint64_t hi = (uint64_t)(t >> 64), h1 = hi >> 32, h0 = hi & gl::EPS, u = (h0 << 32) - h0;
  // r - h1 (2^96 == -1): a borrow wrapped r by 2^64 == EPS and left r >= EPS, so - EPS;
  // + h0 (2^32 - 1) (2^64 == EPS): after a carry r < 2^64 - EPS, so + EPS
#if defined(__x86_64__)
  uint64_t m;
  asm("subq %[h1], %[r]\n\tsbbq %[m], %[m]\n\tmovl %k[m], %k[m]\n\tsubq %[m], %[r]\n\t"
      "addq %[u], %[r]\n\tsbbq %[m], %[m]\n\tmovl %k[m], %k[m]\n\taddq %[m], %[r]"
      : [r] "+r"(r), [m] "=&r"(m)
      : [h1] "r"(h1), [u] "r"(u)
      : "cc");
  return r;
#else
  const uint64_t br = __builtin_sub_overflow(r, h1, &r);
  r -= br * gl::EPS;
  const uint64_t c = __builtin_add_overflow(r, u, &r);
  return r + c * gl::EPS;
#endif
}
inline uint64_t sbox7(uint64_t x) {  // x^7 = x^3 x^4: three products deep, not four
  const uint64_t x2 = wmul(x, x), x4 = wmul(x2, x2);
  return wmul(wmul(x4, x2), x);
}
// sums of up to 16 u64 in 128 bits, folded once: x = lo + 2^64 hi, hi < 2^32
inline uint64_t wsum(const uint64_t *v, int n) {
  unsigned __int128 acc = 0;
#pragma unroll
  for (int i = 0; i < n; i++) acc += v[i];
  const uint64_t lo = (uint64_t)acc, hi = (uint64_t)(acc >> 64);
  return wadd(lo, (hi << 32) - hi);
}
inline void mds4(uint64_t *x) {  // one 4 x 4 block of the external linear layer (as before: t + x_i + 2 x_(i+1))
  const uint64_t x0 = x[0], x1 = x[1], x2 = x[2], x3 = x[3];
  const uint64_t t = wadd(wadd(x0, x1), wadd(x2, x3));
  x[0] = wadd(t, wadd(x0, wadd(x1, x1)));
  x[1] = wadd(t, wadd(x1, wadd(x2, x2)));
  x[2] = wadd(t, wadd(x2, wadd(x3, x3)));
  x[3] = wadd(t, wadd(x3, wadd(x0, x0)));
}
void mds16(uint64_t *s) {
  #pragma unroll
  for (int c = 0; c < 16; c += 4) mds4(s + c);
  #pragma unroll
  for (int k = 0; k < 4; k++) {
    const uint64_t col[4] = {s[k], s[4 + k], s[8 + k], s[12 + k]};
    const uint64_t sum = wsum(col, 4);
    #pragma unroll
    for (int j = k; j < 16; j += 4) s[j] = wadd(s[j], sum);
  }
}
void permute(uint64_t *s) {
  mds16(s);
  #pragma unroll
  for (int r = 0; r < 4; r++) {
    #pragma unroll
    for (int i = 0; i < 16; i++) s[i] = sbox7(wadd(s[i], EXT_INIT[16 * r + i]));
    mds16(s);
  }
  #pragma unroll
  for (int r = 0; r < 22; r++) {
    // the sum of s_1 .. s_15 does not wait for the S-box of s_0 (its chain of
    // products is the round's critical path)
    const uint64_t rest = wsum(s + 1, 15);
    s[0] = sbox7(wadd(s[0], INTERNAL[r]));
    const uint64_t sum = wadd(rest, s[0]);
    #pragma unroll
    for (int i = 0; i < 16; i++) s[i] = wadd(wmul(s[i], DIAG_M1[i]), sum);
  }
  #pragma unroll
  for (int r = 0; r < 4; r++) {
    #pragma unroll
    for (int i = 0; i < 16; i++) s[i] = sbox7(wadd(s[i], EXT_TERM[16 * r + i]));
    mds16(s);
  }
  #pragma unroll
  for (int i = 0; i < 16; i++) s[i] = gl::canon(s[i]);
}

// variant: partial rounds with the sum of s_1..s_15 carried as P + 15 sum
inline uint64_t wmul15(uint64_t a) {  // 15 a, any u64 in and out
  const unsigned __int128 t = (unsigned __int128)a * 15;
  const uint64_t lo = (uint64_t)t, hi = (uint64_t)(t >> 64);  // hi < 15
  return wadd(lo, hi * gl::EPS);
}
inline uint64_t wsum2(const uint64_t *v, int n) {
  unsigned __int128 a0 = 0, a1 = 0;
#pragma unroll
  for (int i = 0; i < n; i += 2) { a0 += v[i]; if (i + 1 < n) a1 += v[i + 1]; }
  a0 += a1;
  const uint64_t lo = (uint64_t)a0, hi = (uint64_t)(a0 >> 64);
  return wadd(lo, (hi << 32) - hi);
}
void permute_b(uint64_t *s) {
  mds16(s);
#pragma unroll
  for (int r = 0; r < 4; r++) {
#pragma unroll
    for (int i = 0; i < 16; i++) s[i] = sbox7(wadd(s[i], EXT_INIT[16 * r + i]));
    mds16(s);
  }
  uint64_t rest = wsum2(s + 1, 15);
#pragma unroll
  for (int r = 0; r < 22; r++) {
    uint64_t p[16];
#pragma unroll
    for (int i = 1; i < 16; i++) p[i] = wmul(s[i], DIAG_M1[i]);
    const uint64_t P = wsum2(p + 1, 15);
    const uint64_t x = sbox7(wadd(s[0], INTERNAL[r]));
    const uint64_t sum = wadd(rest, x);
    s[0] = wadd(wmul(x, DIAG_M1[0]), sum);
#pragma unroll
    for (int i = 1; i < 16; i++) s[i] = wadd(p[i], sum);
    rest = wadd(P, wmul15(sum));
  }
#pragma unroll
  for (int r = 0; r < 4; r++) {
#pragma unroll
    for (int i = 0; i < 16; i++) s[i] = sbox7(wadd(s[i], EXT_TERM[16 * r + i]));
    mds16(s);
  }
#pragma unroll
  for (int i = 0; i < 16; i++) s[i] = gl::canon(s[i]);
}

// variant c: b + the external linear layer on 128-bit sums, reduced once per output
typedef unsigned __int128 u128;
inline uint64_t red128(u128 v) {  // v < 2^96: lo + hi (2^32 - 1), one carry fix
  const uint64_t lo = (uint64_t)v, hi = (uint64_t)(v >> 64);
  return wadd(lo, (hi << 32) - hi);
}
inline void mds16_lazy(uint64_t *s) {
  u128 y[16];
#pragma unroll
  for (int c = 0; c < 16; c += 4) {
    const u128 x0 = s[c], x1 = s[c + 1], x2 = s[c + 2], x3 = s[c + 3];
    const u128 t = x0 + x1 + x2 + x3;
    y[c] = t + x0 + 2 * x1;
    y[c + 1] = t + x1 + 2 * x2;
    y[c + 2] = t + x2 + 2 * x3;
    y[c + 3] = t + x3 + 2 * x0;
  }
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const u128 col = y[k] + y[4 + k] + y[8 + k] + y[12 + k];
#pragma unroll
    for (int j = k; j < 16; j += 4) s[j] = red128(y[j] + col);
  }
}
void permute_c(uint64_t *s) {
  mds16_lazy(s);
#pragma unroll
  for (int r = 0; r < 4; r++) {
#pragma unroll
    for (int i = 0; i < 16; i++) s[i] = sbox7(wadd(s[i], EXT_INIT[16 * r + i]));
    mds16_lazy(s);
  }
  uint64_t rest = wsum2(s + 1, 15);
#pragma unroll
  for (int r = 0; r < 22; r++) {
    uint64_t p[16];
#pragma unroll
    for (int i = 1; i < 16; i++) p[i] = wmul(s[i], DIAG_M1[i]);
    const uint64_t P = wsum2(p + 1, 15);
    const uint64_t x = sbox7(wadd(s[0], INTERNAL[r]));
    const uint64_t sum = wadd(rest, x);
    s[0] = wadd(wmul(x, DIAG_M1[0]), sum);
#pragma unroll
    for (int i = 1; i < 16; i++) s[i] = wadd(p[i], sum);
    rest = wadd(P, wmul15(sum));
  }
#pragma unroll
  for (int r = 0; r < 4; r++) {
#pragma unroll
    for (int i = 0; i < 16; i++) s[i] = sbox7(wadd(s[i], EXT_TERM[16 * r + i]));
    mds16_lazy(s);
  }
#pragma unroll
  for (int i = 0; i < 16; i++) s[i] = gl::canon(s[i]);
}
// variant d: the original partial rounds + the lazy external layer
void permute_d(uint64_t *s) {
  mds16_lazy(s);
#pragma unroll
  for (int r = 0; r < 4; r++) {
#pragma unroll
    for (int i = 0; i < 16; i++) s[i] = sbox7(wadd(s[i], EXT_INIT[16 * r + i]));
    mds16_lazy(s);
  }
#pragma unroll
  for (int r = 0; r < 22; r++) {
    const uint64_t rest = wsum(s + 1, 15);
    s[0] = sbox7(wadd(s[0], INTERNAL[r]));
    const uint64_t sum = wadd(rest, s[0]);
#pragma unroll
    for (int i = 0; i < 16; i++) s[i] = wadd(wmul(s[i], DIAG_M1[i]), sum);
  }
#pragma unroll
  for (int r = 0; r < 4; r++) {
#pragma unroll
    for (int i = 0; i < 16; i++) s[i] = sbox7(wadd(s[i], EXT_TERM[16 * r + i]));
    mds16_lazy(s);
  }
#pragma unroll
  for (int i = 0; i < 16; i++) s[i] = gl::canon(s[i]);
}
// variant e: d + the partial rounds' diagonal products and the sum fused into one 128-bit reduction
inline uint64_t wmuladd(uint64_t a, uint64_t b, uint64_t c) {  // a b + c, any u64 in and out
  const unsigned __int128 t = (unsigned __int128)a * b + c;  // < 2^128: no wrap
  uint64_t r = (uint64_t)t;
  const uint64_t hi = (uint64_t)(t >> 64), h1 = hi >> 32, h0 = hi & gl::EPS, u = (h0 << 32) - h0;
#if defined(__x86_64__)
  uint64_t m;
  asm("subq %[h1], %[r]\n\tsbbq %[m], %[m]\n\tmovl %k[m], %k[m]\n\tsubq %[m], %[r]\n\t"
      "addq %[u], %[r]\n\tsbbq %[m], %[m]\n\tmovl %k[m], %k[m]\n\taddq %[m], %[r]"
      : [r] "+r"(r), [m] "=&r"(m)
      : [h1] "r"(h1), [u] "r"(u)
      : "cc");
  return r;
#else
  const uint64_t br = __builtin_sub_overflow(r, h1, &r);
  r -= br * gl::EPS;
  const uint64_t c2 = __builtin_add_overflow(r, u, &r);
  return r + c2 * gl::EPS;
#endif
}
void permute_e(uint64_t *s) {
  mds16_lazy(s);
#pragma unroll
  for (int r = 0; r < 4; r++) {
#pragma unroll
    for (int i = 0; i < 16; i++) s[i] = sbox7(wadd(s[i], EXT_INIT[16 * r + i]));
    mds16_lazy(s);
  }
#pragma unroll
  for (int r = 0; r < 22; r++) {
    const uint64_t rest = wsum(s + 1, 15);
    s[0] = sbox7(wadd(s[0], INTERNAL[r]));
    const uint64_t sum = wadd(rest, s[0]);
#pragma unroll
    for (int i = 0; i < 16; i++) s[i] = wmuladd(s[i], DIAG_M1[i], sum);
  }
#pragma unroll
  for (int r = 0; r < 4; r++) {
#pragma unroll
    for (int i = 0; i < 16; i++) s[i] = sbox7(wadd(s[i], EXT_TERM[16 * r + i]));
    mds16_lazy(s);
  }
#pragma unroll
  for (int i = 0; i < 16; i++) s[i] = gl::canon(s[i]);
}
// variant f: e + the next round's constants folded into the external layer's 128-bit sums
inline void mds16_lazy_rc(uint64_t *s, const uint64_t *rc) {
  u128 y[16];
#pragma unroll
  for (int c = 0; c < 16; c += 4) {
    const u128 x0 = s[c], x1 = s[c + 1], x2 = s[c + 2], x3 = s[c + 3];
    const u128 t = x0 + x1 + x2 + x3;
    y[c] = t + x0 + 2 * x1;
    y[c + 1] = t + x1 + 2 * x2;
    y[c + 2] = t + x2 + 2 * x3;
    y[c + 3] = t + x3 + 2 * x0;
  }
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const u128 col = y[k] + y[4 + k] + y[8 + k] + y[12 + k];
#pragma unroll
    for (int j = k; j < 16; j += 4) s[j] = red128(y[j] + col + (rc ? rc[j] : 0));
  }
}
void permute_f(uint64_t *s) {
  mds16_lazy_rc(s, EXT_INIT);
#pragma unroll
  for (int r = 0; r < 4; r++) {
#pragma unroll
    for (int i = 0; i < 16; i++) s[i] = sbox7(s[i]);
    mds16_lazy_rc(s, r < 3 ? EXT_INIT + 16 * (r + 1) : nullptr);
  }
#pragma unroll
  for (int r = 0; r < 22; r++) {
    const uint64_t rest = wsum(s + 1, 15);
    s[0] = sbox7(wadd(s[0], INTERNAL[r]));
    const uint64_t sum = wadd(rest, s[0]);
#pragma unroll
    for (int i = 0; i < 16; i++) s[i] = wmuladd(s[i], DIAG_M1[i], sum + 0 * r);
    if (r == 21) {
#pragma unroll
      for (int i = 0; i < 16; i++) s[i] = wadd(s[i], EXT_TERM[i]);
    }
  }
#pragma unroll
  for (int r = 0; r < 4; r++) {
#pragma unroll
    for (int i = 0; i < 16; i++) s[i] = sbox7(s[i]);
    mds16_lazy_rc(s, r < 3 ? EXT_TERM + 16 * (r + 1) : nullptr);
  }
#pragma unroll
  for (int i = 0; i < 16; i++) s[i] = gl::canon(s[i]);
}
}  // namespace
template <class F> double timeit(F f) {
  uint64_t s[16]; for (int i = 0; i < 16; i++) s[i] = i * 0x9E3779B97F4A7C15ull;
  auto a = std::chrono::steady_clock::now();
  for (int k = 0; k < 200000; k++) f(s);
  auto b = std::chrono::steady_clock::now();
  printf("  %llx\n", (unsigned long long)s[0]);
  return std::chrono::duration<double, std::micro>(b - a).count() / 200000;
}
int main() {
  // equality on random and extreme states first
  uint64_t bad = 0;
  for (int it = 0; it < 20000; it++) {
    uint64_t a[16], b[16], c[16], d[16], e[16], f[16];
    for (int i = 0; i < 16; i++) {
      uint64_t v = (uint64_t)it * 0x9E3779B97F4A7C15ull ^ ((uint64_t)i << 40) ^ ((uint64_t)it * it);
      if (it % 3 == 0) v = gl::P - 1 - (uint64_t)(i % 3);
      a[i] = b[i] = c[i] = d[i] = e[i] = f[i] = gl::canon(v);
    }
    permute(a); permute_b(b); permute_c(c); permute_d(d); permute_e(e); permute_f(f);
    for (int i = 0; i < 16; i++) bad += (a[i] != b[i]) + (a[i] != c[i]) + (a[i] != d[i]) + (a[i] != e[i]) + (a[i] != f[i]);
  }
  printf("mismatches %llu\n", (unsigned long long)bad);
  for (int rep = 0; rep < 3; rep++)
    printf("a %.3f b %.3f c %.3f d %.3f e %.3f f %.3f\n", timeit(permute), timeit(permute_b), timeit(permute_c), timeit(permute_d), timeit(permute_e), timeit(permute_f));
}
