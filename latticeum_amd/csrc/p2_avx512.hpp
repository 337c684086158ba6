// p2_avx512.hpp -- the host Poseidon2 width-16 permutation's arithmetic on AVX-512
// (8 lanes per register, the state in two registers), on the same weakly reduced
// values as transcript.cpp's scalar forms: wmul8 / wmuladd8 / wadd8 are wmul /
// wmuladd / wadd lane-wise (the 128-bit product from four 32 x 32 products),
// mds16_rc8 the external layer with its sums on 32-bit halves (no lane overflows)
// and one fold per output. Host only; transcript.cpp selects it at run time when
// the CPU has AVX-512F (the box's EPYC 9575F does).
#pragma once
#include <immintrin.h>
#include <cstdint>

#define LF_AVX512 __attribute__((target("avx512f")))

namespace p2avx {

LF_AVX512 inline __m512i eps8() { return _mm512_set1_epi64(0xFFFFFFFFll); }

// a b for any u64 a, b: the 128-bit product from four 32 x 32 products, folded with
// 2^64 == 2^32 - 1 and 2^96 == -1 (as wmul: r - h1 with a borrow fix, + h0 EPS with a carry fix)
LF_AVX512 inline __m512i wmul8(__m512i a, __m512i b) {
  const __m512i M = eps8();
  const __m512i ah = _mm512_srli_epi64(a, 32), bh = _mm512_srli_epi64(b, 32);
  const __m512i ll = _mm512_mul_epu32(a, b), lh = _mm512_mul_epu32(a, bh), hl = _mm512_mul_epu32(ah, b),
                hh = _mm512_mul_epu32(ah, bh);
  const __m512i t = _mm512_add_epi64(_mm512_add_epi64(_mm512_srli_epi64(ll, 32), _mm512_and_si512(lh, M)),
                                     _mm512_and_si512(hl, M));  // < 3 2^32
  const __m512i lo = _mm512_mask_blend_epi32(0x5555, _mm512_slli_epi64(t, 32), ll);
  const __m512i hi = _mm512_add_epi64(_mm512_add_epi64(hh, _mm512_srli_epi64(lh, 32)),
                                      _mm512_add_epi64(_mm512_srli_epi64(hl, 32), _mm512_srli_epi64(t, 32)));
  // r = lo - h1; a borrow: - EPS
  const __m512i h1 = _mm512_srli_epi64(hi, 32);
  __m512i r = _mm512_sub_epi64(lo, h1);
  r = _mm512_mask_sub_epi64(r, _mm512_cmplt_epu64_mask(lo, h1), r, M);
  // + h0 (2^32 - 1) = (h0 << 32) - h0; a carry: + EPS
  const __m512i u = _mm512_sub_epi64(_mm512_slli_epi64(hi, 32), _mm512_and_si512(hi, M));
  const __m512i r2 = _mm512_add_epi64(r, u);
  return _mm512_mask_add_epi64(r2, _mm512_cmplt_epu64_mask(r2, u), r2, M);
}
// a b + c for any u64 (as wmuladd: the sum < 2^128, one fold)
LF_AVX512 inline __m512i wmuladd8(__m512i a, __m512i b, __m512i c) {
  const __m512i M = eps8();
  const __m512i ah = _mm512_srli_epi64(a, 32), bh = _mm512_srli_epi64(b, 32);
  const __m512i ll = _mm512_mul_epu32(a, b), lh = _mm512_mul_epu32(a, bh), hl = _mm512_mul_epu32(ah, b),
                hh = _mm512_mul_epu32(ah, bh);
  const __m512i t = _mm512_add_epi64(_mm512_add_epi64(_mm512_srli_epi64(ll, 32), _mm512_and_si512(lh, M)),
                                     _mm512_and_si512(hl, M));
  const __m512i lo0 = _mm512_mask_blend_epi32(0x5555, _mm512_slli_epi64(t, 32), ll);
  __m512i hi = _mm512_add_epi64(_mm512_add_epi64(hh, _mm512_srli_epi64(lh, 32)),
                                _mm512_add_epi64(_mm512_srli_epi64(hl, 32), _mm512_srli_epi64(t, 32)));
  const __m512i lo = _mm512_add_epi64(lo0, c);
  hi = _mm512_mask_add_epi64(hi, _mm512_cmplt_epu64_mask(lo, c), hi, _mm512_set1_epi64(1));
  const __m512i h1 = _mm512_srli_epi64(hi, 32);
  __m512i r = _mm512_sub_epi64(lo, h1);
  r = _mm512_mask_sub_epi64(r, _mm512_cmplt_epu64_mask(lo, h1), r, M);
  const __m512i u = _mm512_sub_epi64(_mm512_slli_epi64(hi, 32), _mm512_and_si512(hi, M));
  const __m512i r2 = _mm512_add_epi64(r, u);
  return _mm512_mask_add_epi64(r2, _mm512_cmplt_epu64_mask(r2, u), r2, M);
}
// the sum of lanes 1 .. 15 as (lo-half sum, hi-half sum), each < 2^36
LF_AVX512 inline void hsum_rest8(__m512i x0, __m512i x1, uint64_t &sl, uint64_t &sh) {
  const __m512i M = eps8();
  const __m512i z0 = _mm512_maskz_mov_epi64(0xFE, x0);
  sl = (uint64_t)_mm512_reduce_add_epi64(_mm512_add_epi64(_mm512_and_si512(z0, M), _mm512_and_si512(x1, M)));
  sh = (uint64_t)_mm512_reduce_add_epi64(_mm512_add_epi64(_mm512_srli_epi64(z0, 32), _mm512_srli_epi64(x1, 32)));
}
// a^2: three 32 x 32 products (the cross product doubled), the same fold as wmul8
LF_AVX512 inline __m512i wsqr8(__m512i a) {
  const __m512i M = eps8();
  const __m512i ah = _mm512_srli_epi64(a, 32);
  const __m512i ll = _mm512_mul_epu32(a, a), lh = _mm512_mul_epu32(a, ah), hh = _mm512_mul_epu32(ah, ah);
  // a^2 = ll + 2 lh 2^32 + hh 2^64; t = (ll >> 32) + 2 (lh mod 2^32) < 3 2^32
  const __m512i t = _mm512_add_epi64(_mm512_srli_epi64(ll, 32), _mm512_slli_epi64(_mm512_and_si512(lh, M), 1));
  const __m512i lo = _mm512_mask_blend_epi32(0x5555, _mm512_slli_epi64(t, 32), ll);
  const __m512i hi = _mm512_add_epi64(_mm512_add_epi64(hh, _mm512_slli_epi64(_mm512_srli_epi64(lh, 32), 1)),
                                      _mm512_srli_epi64(t, 32));
  const __m512i h1 = _mm512_srli_epi64(hi, 32);
  __m512i r = _mm512_sub_epi64(lo, h1);
  r = _mm512_mask_sub_epi64(r, _mm512_cmplt_epu64_mask(lo, h1), r, M);
  const __m512i u = _mm512_sub_epi64(_mm512_slli_epi64(hi, 32), _mm512_and_si512(hi, M));
  const __m512i r2 = _mm512_add_epi64(r, u);
  return _mm512_mask_add_epi64(r2, _mm512_cmplt_epu64_mask(r2, u), r2, M);
}
LF_AVX512 inline __m512i sbox8(__m512i x) {  // x^3 x^4: three products deep
  const __m512i x2 = wsqr8(x), x3 = wmul8(x2, x), x4 = wsqr8(x2);
  return wmul8(x4, x3);
}
// a + b, any u64 (as wadd): a carry + EPS, which can carry once more
LF_AVX512 inline __m512i wadd8(__m512i a, __m512i b) {
  const __m512i M = eps8();
  __m512i s = _mm512_add_epi64(a, b);
  const __mmask8 c1 = _mm512_cmplt_epu64_mask(s, b);
  s = _mm512_mask_add_epi64(s, c1, s, M);
  return _mm512_mask_add_epi64(s, _mm512_mask_cmplt_epu64_mask(c1, s, M), s, M);
}
// L + 2^32 H for L, H < 2^40 -> a u64 congruent mod p
LF_AVX512 inline __m512i fold8(__m512i L, __m512i H) {
  const __m512i M = eps8();
  const __m512i A = _mm512_slli_epi64(H, 32), B = _mm512_srli_epi64(H, 32);  // H 2^32 = A + B 2^64
  const __m512i Lp = _mm512_add_epi64(L, _mm512_sub_epi64(_mm512_slli_epi64(B, 32), B));  // + B EPS, < 2^41
  const __m512i s = _mm512_add_epi64(A, Lp);
  return _mm512_mask_add_epi64(s, _mm512_cmplt_epu64_mask(s, Lp), s, M);  // a carry leaves s < 2^41
}
// MDSMat4 on each 4-lane chunk (y_i = t + x_i + 2 x_(i+1), t the chunk sum), then the
// column sums over the four chunks, + rc: on one 32-bit half of the words
LF_AVX512 inline void mds_half(__m512i x0, __m512i x1, __m512i &o0, __m512i &o1) {
  const __m512i r10 = _mm512_permutex_epi64(x0, 0x39), r11 = _mm512_permutex_epi64(x1, 0x39);  // x_(i+1)
  const __m512i p0 = _mm512_add_epi64(x0, _mm512_permutex_epi64(x0, 0x4E)),
                p1 = _mm512_add_epi64(x1, _mm512_permutex_epi64(x1, 0x4E));  // x_i + x_(i+2)
  const __m512i t0 = _mm512_add_epi64(p0, _mm512_permutex_epi64(p0, 0x39)),
                t1 = _mm512_add_epi64(p1, _mm512_permutex_epi64(p1, 0x39));  // chunk sums
  const __m512i y0 = _mm512_add_epi64(_mm512_add_epi64(t0, x0), _mm512_add_epi64(r10, r10));
  const __m512i y1 = _mm512_add_epi64(_mm512_add_epi64(t1, x1), _mm512_add_epi64(r11, r11));
  const __m512i c = _mm512_add_epi64(y0, y1);
  const __m512i col = _mm512_add_epi64(c, _mm512_shuffle_i64x2(c, c, 0x4E));
  o0 = _mm512_add_epi64(y0, col);
  o1 = _mm512_add_epi64(y1, col);
}
LF_AVX512 inline void mds16_rc8(__m512i &x0, __m512i &x1, const uint64_t *rc) {
  const __m512i M = eps8();
  __m512i l0, l1, h0, h1;
  mds_half(_mm512_and_si512(x0, M), _mm512_and_si512(x1, M), l0, l1);
  mds_half(_mm512_srli_epi64(x0, 32), _mm512_srli_epi64(x1, 32), h0, h1);
  if (rc) {
    const __m512i c0 = _mm512_loadu_si512(rc), c1 = _mm512_loadu_si512(rc + 8);
    l0 = _mm512_add_epi64(l0, _mm512_and_si512(c0, M));
    l1 = _mm512_add_epi64(l1, _mm512_and_si512(c1, M));
    h0 = _mm512_add_epi64(h0, _mm512_srli_epi64(c0, 32));
    h1 = _mm512_add_epi64(h1, _mm512_srli_epi64(c1, 32));
  }
  x0 = fold8(l0, h0);
  x1 = fold8(l1, h1);
}

}  // namespace p2avx
