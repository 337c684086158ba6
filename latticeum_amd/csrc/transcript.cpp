// transcript.cpp -- host side of the boundary: the zkvm's Poseidon2 Fiat-Shamir
// transcript. It is a strictly sequential sponge (each permutation depends on
// the previous one), exactly as in the reference, so it runs on the host:
//   zkvm/src/fiat_shamir.rs:20-114  Poseidon2Transcript over Plonky3
//       DuplexChallenger<Goldilocks, WideZkVMPoseidon2Perm, 16, 12>
//   zkvm/src/poseidon2.rs:100-173   the width-16 permutation
//   zkvm/src/poseidon2.rs:206-235   hash_iter (overwrite sponge)
// Batched independent permutations run on the GPU (lf_dev_poseidon2_permute).
#include <cstring>
#include <vector>

#include "../../include/lf.h"
#include "gl.hpp"
#include "ring.hpp"
#if defined(__x86_64__) && !defined(__HIP_DEVICE_COMPILE__)
#define LF_P2_AVX512 1
#include <cstdlib>
#include "p2_avx512.hpp"
#endif

namespace {
#include "p2_consts.inc"
const uint64_t EXT_INIT[64] = LF_P2_EXT_INIT;
const uint64_t EXT_TERM[64] = LF_P2_EXT_TERM;
const uint64_t INTERNAL[22] = LF_P2_INTERNAL;
const uint64_t DIAG_M1[16] = LF_P2_DIAG_M1;
const uint64_t W8_EXT_INIT[32] = LF_P2W8_EXT_INIT;
const uint64_t W8_EXT_TERM[32] = LF_P2W8_EXT_TERM;
const uint64_t W8_DIAG_M1[8] = LF_P2W8_DIAG_M1;

// The permutation keeps its state weakly reduced (any u64 congruent mod p) and
// canonicalises once at the end, as Plonky3's Goldilocks arithmetic does: a
// product is one 64 x 64 -> 128 multiply and a branch-free fold, a sum one add
// and carry fix-ups, with no per-operation comparison against p.
// (x86-64: the carry fix-ups as sbb masks; compilers otherwise branch on the
// carries, which are data-dependent and mispredict about half the time)
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
  const uint64_t x2 = wmul(x, x), x3 = wmul(x2, x), x4 = wmul(x2, x2);
  return wmul(x4, x3);
}
// sums of up to 16 u64 in 128 bits, folded once: x = lo + 2^64 hi, hi < 2^32
inline uint64_t wsum(const uint64_t *v, int n) {
  unsigned __int128 acc = 0;
#pragma unroll
  for (int i = 0; i < n; i++) acc += v[i];
  const uint64_t lo = (uint64_t)acc, hi = (uint64_t)(acc >> 64);
  return wadd(lo, (hi << 32) - hi);
}
// a b + c with one 128-bit fold (any u64 in and out; a b + c < 2^128)
inline uint64_t wmuladd(uint64_t a, uint64_t b, uint64_t c) {
  const unsigned __int128 t = (unsigned __int128)a * b + c;
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
  const uint64_t cr = __builtin_add_overflow(r, u, &r);
  return r + cr * gl::EPS;
#endif
}
typedef unsigned __int128 u128;
inline uint64_t red96(u128 v) {  // v < 2^96: lo + hi (2^32 - 1)
  const uint64_t lo = (uint64_t)v, hi = (uint64_t)(v >> 64);
  return wadd(lo, (hi << 32) - hi);
}
// The external linear layer (MDSMat4 on each 4-chunk, then the column sums) on
// 128-bit sums of the u64 inputs with one fold per output, and the next round's
// constants (rc, or none) added inside the same sum: 16 folds instead of the 76
// modular additions of the word-by-word form (mds16)
inline void mds16_rc(uint64_t *s, const uint64_t *rc) {
  u128 y[16];
#pragma unroll
  for (int c = 0; c < 16; c += 4) {
    const u128 x0 = s[c], x1 = s[c + 1], x2 = s[c + 2], x3 = s[c + 3];
    const u128 t = x0 + x1 + x2 + x3;
    y[c] = t + x0 + 2 * x1;  // as mds4: t + x_i + 2 x_(i+1)
    y[c + 1] = t + x1 + 2 * x2;
    y[c + 2] = t + x2 + 2 * x3;
    y[c + 3] = t + x3 + 2 * x0;
  }
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const u128 col = y[k] + y[4 + k] + y[8 + k] + y[12 + k];
#pragma unroll
    for (int j = k; j < 16; j += 4) s[j] = red96(y[j] + col + (rc ? rc[j] : 0));
  }
}
void mds16(uint64_t *s) { mds16_rc(s, nullptr); }
#if LF_P2_AVX512
// permute() on AVX-512: the external rounds' S-boxes and layers on the two state
// registers; in the internal rounds s_0's S-box chain runs in scalar registers (it
// is the round's critical path) while the diagonal layer runs on the vectors, the
// next round's s_0 from the scalar copy and the sum of the rest from the lanes.
// The same field elements as the scalar form (tools/exp/p2_avx_test.cpp).
LF_AVX512 void permute_avx512(uint64_t *s) {
  using namespace p2avx;
  __m512i x0 = _mm512_loadu_si512(s), x1 = _mm512_loadu_si512(s + 8);
  mds16_rc8(x0, x1, EXT_INIT);
  for (int r = 0; r < 4; r++) {
    x0 = sbox8(x0);
    x1 = sbox8(x1);
    mds16_rc8(x0, x1, r < 3 ? EXT_INIT + 16 * (r + 1) : nullptr);
  }
  {
    const __m512i D0 = _mm512_loadu_si512(DIAG_M1), D1 = _mm512_loadu_si512(DIAG_M1 + 8);
    uint64_t sl, sh;
    hsum_rest8(x0, x1, sl, sh);
    // rest = s_1 + .. + s_15 before the round. t0 = s_0 + the round's constant; the
    // next one is y (d_0 + 1) + (rest + rc'), so the chain between S-boxes is one
    // multiply-add. The next rest is sum_(i>=1) d_i s_i + 15 (rest + y): the lanes'
    // products D x and their horizontal sum u are formed from the state before the
    // round's S-box, so the recurrence's only work after y is one multiply-add and
    // the vector update and its sum stay off the S-box chain (EPYC 9575F: 0.72 ->
    // 0.65 us per permutation; same field elements, tools/exp/p2_avx_test.cpp)
    uint64_t rest = red96((u128)sl + ((u128)sh << 32));
    uint64_t t0 = wadd((uint64_t)_mm_cvtsi128_si64(_mm512_castsi512_si128(x0)), INTERNAL[0]);
    for (int r = 0; r < 22; r++) {
      const __m512i dx0 = wmul8(x0, D0), dx1 = wmul8(x1, D1);  // lane 0 of dx0 is replaced below
      hsum_rest8(dx0, dx1, sl, sh);
      const uint64_t u = red96((u128)sl + ((u128)sh << 32));
      const uint64_t y = sbox7(t0);
      const uint64_t sum = wadd(rest, y);
      const __m512i S = _mm512_set1_epi64((long long)sum);
      x0 = wadd8(_mm512_mask_mov_epi64(dx0, 1, _mm512_set1_epi64((long long)wmul(y, DIAG_M1[0]))), S);
      x1 = wadd8(dx1, S);
      if (r + 1 < 22) {
        t0 = wmuladd(y, DIAG_M1[0] + 1, wadd(rest, INTERNAL[r + 1]));  // y d_0 + y + rest + rc
        rest = wmuladd(sum, 15, u);
      }
    }
  }
  x0 = wadd8(x0, _mm512_loadu_si512(EXT_TERM));
  x1 = wadd8(x1, _mm512_loadu_si512(EXT_TERM + 8));
  for (int r = 0; r < 4; r++) {
    x0 = sbox8(x0);
    x1 = sbox8(x1);
    mds16_rc8(x0, x1, r < 3 ? EXT_TERM + 16 * (r + 1) : nullptr);
  }
  _mm512_storeu_si512(s, x0);
  _mm512_storeu_si512(s + 8, x1);
  for (int i = 0; i < 16; i++) s[i] = gl::canon(s[i]);
}
// AVX-512F present, unless LATTICEUM_AMD_P2_SCALAR=1 (the scalar form, for A/B runs)
bool use_avx512() {
  static const bool on = __builtin_cpu_supports("avx512f") && !(getenv("LATTICEUM_AMD_P2_SCALAR") &&
                                                                 getenv("LATTICEUM_AMD_P2_SCALAR")[0] == '1');
  return on;
}
#endif
// The sponge's permutation. Round constants ride in the preceding layer's sums
// (the initial MDS carries round 0's, the last internal round adds the terminal
// rounds' first); the internal rounds' diagonal product and the sum share one fold.
void permute_scalar(uint64_t *s) {
  mds16_rc(s, EXT_INIT);
  #pragma unroll
  for (int r = 0; r < 4; r++) {
    #pragma unroll
    for (int i = 0; i < 16; i++) s[i] = sbox7(s[i]);
    mds16_rc(s, r < 3 ? EXT_INIT + 16 * (r + 1) : nullptr);
  }
  #pragma unroll
  for (int r = 0; r < 22; r++) {
    // the sum of s_1 .. s_15 does not wait for the S-box of s_0 (its chain of
    // products is the round's critical path)
    const uint64_t rest = wsum(s + 1, 15);
    s[0] = sbox7(wadd(s[0], INTERNAL[r]));
    const uint64_t sum = wadd(rest, s[0]);
    #pragma unroll
    for (int i = 0; i < 16; i++) s[i] = wmuladd(s[i], DIAG_M1[i], sum);
  }
  #pragma unroll
  for (int i = 0; i < 16; i++) s[i] = wadd(s[i], EXT_TERM[i]);
  #pragma unroll
  for (int r = 0; r < 4; r++) {
    #pragma unroll
    for (int i = 0; i < 16; i++) s[i] = sbox7(s[i]);
    mds16_rc(s, r < 3 ? EXT_TERM + 16 * (r + 1) : nullptr);
  }
  #pragma unroll
  for (int i = 0; i < 16; i++) s[i] = gl::canon(s[i]);
}
void permute(uint64_t *s) {
#if LF_P2_AVX512
  if (use_avx512()) return permute_avx512(s);
#endif
  permute_scalar(s);
}
// permute() with WideZkVMPoseidon2Perm::permute_mut's PermutationIntermediateStates
// (poseidon2.rs:91-96, 104-171): the state after the initial MDS, after each of
// the 4 initial external, 22 internal and 4 terminal rounds -- 31 x 16 words,
// canonical (the in-CCS verifier reads them with as_canonical_u64, ccs.rs:517-580)
void permute_states(uint64_t *s, uint64_t *st) {
  auto keep = [&](int k) {
    for (int i = 0; i < 16; i++) st[16 * k + i] = gl::canon(s[i]);
  };
  mds16(s);
  keep(0);
  for (int r = 0; r < 4; r++) {
    for (int i = 0; i < 16; i++) s[i] = sbox7(wadd(s[i], EXT_INIT[16 * r + i]));
    mds16(s);
    keep(1 + r);
  }
  for (int r = 0; r < 22; r++) {
    const uint64_t rest = wsum(s + 1, 15);
    s[0] = sbox7(wadd(s[0], INTERNAL[r]));
    const uint64_t sum = wadd(rest, s[0]);
    for (int i = 0; i < 16; i++) s[i] = wmuladd(s[i], DIAG_M1[i], sum);
    keep(5 + r);
  }
  for (int r = 0; r < 4; r++) {
    for (int i = 0; i < 16; i++) s[i] = sbox7(wadd(s[i], EXT_TERM[16 * r + i]));
    mds16(s);
    keep(27 + r);
  }
  for (int i = 0; i < 16; i++) s[i] = gl::canon(s[i]);
}
// Poseidon2Goldilocks<8> (poseidon2.rs:31-49): the same round structure at
// width 8 (MDSMat4 on both 4-chunks, then the column sums), the reference's
// width-8 external constants (crypto_consts.rs:9-96) and Plonky3's
// MATRIX_DIAG_8_GOLDILOCKS (not vendored: restated, parity unpinned)
// width 8: MDSMat4 on both 4-chunks, then the column sums, on 128-bit sums with the
// next round's constants inside (as mds16_rc)
inline void mds8_rc(uint64_t *s, const uint64_t *rc) {
  u128 y[8];
#pragma unroll
  for (int c = 0; c < 8; c += 4) {
    const u128 x0 = s[c], x1 = s[c + 1], x2 = s[c + 2], x3 = s[c + 3];
    const u128 t = x0 + x1 + x2 + x3;
    y[c] = t + x0 + 2 * x1;
    y[c + 1] = t + x1 + 2 * x2;
    y[c + 2] = t + x2 + 2 * x3;
    y[c + 3] = t + x3 + 2 * x0;
  }
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const u128 col = y[k] + y[4 + k];
    s[k] = red96(y[k] + col + (rc ? rc[k] : 0));
    s[4 + k] = red96(y[4 + k] + col + (rc ? rc[4 + k] : 0));
  }
}
void permute8(uint64_t *s) {
  mds8_rc(s, W8_EXT_INIT);
  #pragma unroll
  for (int r = 0; r < 4; r++) {
    #pragma unroll
    for (int i = 0; i < 8; i++) s[i] = sbox7(s[i]);
    mds8_rc(s, r < 3 ? W8_EXT_INIT + 8 * (r + 1) : nullptr);
  }
  #pragma unroll
  for (int r = 0; r < 22; r++) {
    const uint64_t rest = wsum(s + 1, 7);
    s[0] = sbox7(wadd(s[0], INTERNAL[r]));
    const uint64_t sum = wadd(rest, s[0]);
    #pragma unroll
    for (int i = 0; i < 8; i++) s[i] = wmuladd(s[i], W8_DIAG_M1[i], sum);
  }
  #pragma unroll
  for (int i = 0; i < 8; i++) s[i] = wadd(s[i], W8_EXT_TERM[i]);
  #pragma unroll
  for (int r = 0; r < 4; r++) {
    #pragma unroll
    for (int i = 0; i < 8; i++) s[i] = sbox7(s[i]);
    mds8_rc(s, r < 3 ? W8_EXT_TERM + 8 * (r + 1) : nullptr);
  }
  #pragma unroll
  for (int i = 0; i < 8; i++) s[i] = gl::canon(s[i]);
}
// PaddingFreeSponge<_, 8, 4, 4>::hash_iter: overwrite state[0..4), permute; a
// partial last block is permuted; an empty input is the zero digest
template <class Next>
void sponge8(Next next, size_t n, uint64_t out4[4]) {
  uint64_t s[8] = {0};
  size_t pos = 0;
  for (;;) {
    for (int i = 0; i < 4; i++) {
      if (pos < n) {
        s[i] = next(pos++);
      } else {
        if (i != 0) permute8(s);
        memcpy(out4, s, 4 * sizeof(uint64_t));
        return;
      }
    }
    permute8(s);
  }
}
}  // namespace

struct lf_transcript {
  uint64_t state[16] = {0};
  // Plonky3 DuplexChallenger's input and output buffers (at most RATE = 12 each)
  uint64_t in[12], out[12];
  int nin = 0, nout = 0;
  // record: every sampled value is appended to `log`. playback: samples come
  // from `log` in order and observes are dropped -- a transcript that absorbs
  // the same messages in the same order samples the same values, so a replay of
  // a recorded proof needs no permutation at all
  bool recording = false, playback = false;
  std::vector<uint64_t> log;
  size_t pos = 0;
  bool underrun = false;
  void duplexing() {  // Plonky3 DuplexChallenger::duplexing (overwrite mode)
    for (int i = 0; i < nin; i++) state[i] = in[i];
    nin = 0;
    permute(state);
    memcpy(out, state, sizeof(out));
    nout = 12;
  }
  void observe(uint64_t v) {  // v canonical
    nout = 0;
    in[nin++] = v;
    if (nin == 12) duplexing();
  }
};

extern "C" {

lf_transcript *lf_transcript_new(void) { return new lf_transcript; }
void lf_transcript_free(lf_transcript *t) { delete t; }

void lf_transcript_observe(lf_transcript *t, uint64_t v) {
  if (t->playback) return;
  t->observe(gl::canon(v));
}

uint64_t lf_transcript_sample(lf_transcript *t) {
  if (t->playback) {
    if (t->pos < t->log.size()) return t->log[t->pos++];
    t->underrun = true;
    return 0;
  }
  if (t->nin || !t->nout) t->duplexing();
  const uint64_t v = t->out[--t->nout];
  if (t->recording) t->log.push_back(v);
  return v;
}

void lf_transcript_record(lf_transcript *t) {
  t->recording = true;
  t->log.clear();
}
size_t lf_transcript_samples(const lf_transcript *t, uint64_t *out, size_t cap) {
  if (out) memcpy(out, t->log.data(), (cap < t->log.size() ? cap : t->log.size()) * sizeof(uint64_t));
  return t->log.size();
}
lf_transcript *lf_transcript_new_playback(const uint64_t *samples, size_t n) {
  if (!samples && n) return nullptr;
  lf_transcript *t = new lf_transcript;
  t->playback = true;
  t->log.assign(samples, samples + n);
  return t;
}
int lf_transcript_playback_status(const lf_transcript *t) {
  if (!t->playback) return LF_ERR_INVALID_ARG;
  return t->underrun || t->pos != t->log.size() ? LF_ERR_INCORRECT_LENGTH : LF_OK;
}

void lf_transcript_absorb_ring(lf_transcript *t, const uint64_t *e, size_t n, int d, int repr) {
  // fiat_shamir.rs:51-60: observe elem.0.0[0], the ark Montgomery limb
  if (t->playback) return;
  const size_t m = n * (size_t)d;
  auto limb = [repr](uint64_t x) { return gl::canon(repr == LF_REPR_MONTGOMERY ? x : wmul(x, gl::EPS)); };
  size_t i = 0;
  // whole rate blocks straight into the state (what observe() does 12 times: overwrite
  // state[0..12), permute, the outputs become the sample buffer)
  if (t->nin == 0)
    for (; i + 12 <= m; i += 12) {
      for (int k = 0; k < 12; k++) t->state[k] = limb(e[i + k]);
      permute(t->state);
      memcpy(t->out, t->state, sizeof(t->out));
      t->nout = 12;
    }
  for (; i < m; i++) t->observe(limb(e[i]));
}

void lf_transcript_get_challenge(lf_transcript *t, uint64_t out3[3]) {
  for (int i = 0; i < 3; i++) out3[i] = lf_transcript_sample(t);  // fiat_shamir.rs:69-86
  for (int i = 0; i < 3; i++) lf_transcript_observe(t, out3[i]);
}

void lf_transcript_squeeze_bytes(lf_transcript *t, uint8_t *out, size_t n) {
  while (n) {  // fiat_shamir.rs:88-102
    uint64_t v = lf_transcript_sample(t);
    size_t take = n < 8 ? n : 8;
    for (size_t i = 0; i < take; i++) *out++ = (uint8_t)(v >> (8 * i));
    n -= take;
  }
}

int lf_transcript_get_short_challenges(lf_transcript *t, int d, size_t count, uint64_t *coeffs) {
  if (!t || !coeffs || d % 4) return LF_ERR_INVALID_ARG;
  std::vector<uint8_t> bytes(3 * d / 4);
  for (size_t i = 0; i < count; i++) {  // fiat_shamir.rs:105-113
    lf_transcript_squeeze_bytes(t, bytes.data(), bytes.size());
    int r = lf_short_challenge(bytes.data(), bytes.size(), d, coeffs + i * d);
    if (r != LF_OK) return r;
  }
  return LF_OK;
}

void lf_hash_iter(const uint64_t *in, size_t n, uint64_t out4[4]) {
  uint64_t s[16] = {0};
  size_t pos = 0;
  for (;;) {  // poseidon2.rs:215-227
    for (int i = 0; i < 12; i++) {
      if (pos < n) {
        s[i] = gl::canon(in[pos++]);
      } else {
        if (i != 0) permute(s);
        memcpy(out4, s, 4 * sizeof(uint64_t));
        return;
      }
    }
    permute(s);
  }
}

size_t lf_hash_iter_nperm(size_t n) { return (n + 11) / 12; }

int lf_hash_iter_states(const uint64_t *in, size_t n, uint64_t out4[4], uint64_t *states, size_t cap) {
  if ((!in && n) || !out4 || (states && cap < lf_hash_iter_nperm(n))) return LF_ERR_INVALID_ARG;
  uint64_t s[16] = {0};
  size_t pos = 0, np = 0;
  auto perm = [&]() {  // poseidon2.rs:221,226: one IntermediateStates record per permutation
    if (states) permute_states(s, states + (size_t)LF_P2_STATES * 16 * np);
    else permute(s);
    np++;
  };
  for (;;) {  // poseidon2.rs:215-227
    for (int i = 0; i < 12; i++) {
      if (pos < n) {
        s[i] = gl::canon(in[pos++]);
      } else {
        if (i != 0) perm();
        memcpy(out4, s, 4 * sizeof(uint64_t));
        return LF_OK;
      }
    }
    perm();
  }
}

int lf_acc_comm(const lf_lcccs *acc, int repr, uint64_t out4[4]) {
  // commitments.rs:143-176 + flatten (:349-361): r, v, cm, u, x_w, h in that
  // order, every NTT element ICRT'd and each coefficient's ark limb (its
  // Montgomery form) hashed as a Goldilocks value. The ICRT is linear, so on
  // Montgomery-limb input it yields the coefficients' Montgomery limbs directly.
  if (!acc || !out4 || (repr != LF_REPR_CANONICAL && repr != LF_REPR_MONTGOMERY)) return LF_ERR_INVALID_ARG;
  if (acc->d != 24) return LF_ERR_UNSUPPORTED_RING;  // the zkvm's GoldilocksRingNTT
  const lf_ring_slice parts[6] = {acc->r, acc->v, acc->cm, acc->u, acc->x_w, {acc->h, 1}};
  std::vector<uint64_t> flat;
  for (const lf_ring_slice &p : parts) {
    if (p.n && !p.elems) return LF_ERR_INVALID_ARG;
    for (size_t e = 0; e < p.n; e++) {
      uint64_t c[24];
      for (int i = 0; i < 24; i++) c[i] = gl::canon(p.elems[e * 24 + i]);
      ring::phi72_icrt(c);
      for (int i = 0; i < 24; i++) flat.push_back(repr == LF_REPR_MONTGOMERY ? c[i] : gl::to_mont(c[i]));
    }
  }
  return lf_hash_iter_states(flat.data(), flat.size(), out4, nullptr, 0);
}

int lf_ivc_step_comm(uint64_t i, const uint64_t state_0_comm[4], const uint64_t state_i_comm[4],
                     const uint64_t acc_comm[4], uint64_t out4[4], uint64_t *states) {
  if (!state_0_comm || !state_i_comm || !acc_comm) return LF_ERR_INVALID_ARG;
  uint64_t in[13];  // commitments.rs:83-105
  in[0] = i;
  for (int k = 0; k < 4; k++) {
    in[1 + k] = state_0_comm[k];
    in[5 + k] = state_i_comm[k];
    in[9 + k] = acc_comm[k];
  }
  return lf_hash_iter_states(in, 13, out4, states, 2);
}

int lf_state_i_comm(const uint64_t code_comm[4], uint64_t pc, const uint64_t memory_comm[4],
                    const uint64_t regs_comm[4], const uint64_t mem_ops_vec_comm[4], uint64_t out4[4]) {
  if (!code_comm || !memory_comm || !regs_comm || !mem_ops_vec_comm) return LF_ERR_INVALID_ARG;
  uint64_t in[17];  // commitments.rs:107-141
  for (int k = 0; k < 4; k++) {
    in[k] = code_comm[k];
    in[5 + k] = memory_comm[k];
    in[9 + k] = regs_comm[k];
    in[13 + k] = mem_ops_vec_comm[k];
  }
  in[4] = pc;
  return lf_hash_iter_states(in, 17, out4, nullptr, 0);
}

int lf_vm_regs_comm(const uint32_t *regs, size_t n, uint64_t out4[4]) {
  if (!regs && n) return LF_ERR_INVALID_ARG;  // commitments.rs:178-189 (N_REGS = 32)
  std::vector<uint64_t> in(regs, regs + n);
  return lf_hash_iter_states(in.data(), n, out4, nullptr, 0);
}

int lf_vm_mem_ops_vec_comm(const uint64_t prev[4], uint64_t cycle, uint32_t address, uint32_t value,
                           uint64_t out4[4]) {
  // commitments.rs:290-307: TruncatedPermutation<Poseidon2<8>, 2, 4, 8>::compress of
  // [previous_comm, (cycle, address, value, 0)]: permute the concatenation, keep 4
  if (!prev || !out4) return LF_ERR_INVALID_ARG;
  uint64_t s[8] = {gl::canon(prev[0]), gl::canon(prev[1]), gl::canon(prev[2]), gl::canon(prev[3]),
                   gl::canon(cycle), address, value, 0};
  permute8(s);
  memcpy(out4, s, 4 * sizeof(uint64_t));
  return LF_OK;
}

void lf_hash_w8(const uint64_t *in, size_t n, uint64_t out4[4]) {
  sponge8([&](size_t i) { return gl::canon(in[i]); }, n, out4);
}

int lf_vm_mem_comm(const uint32_t *words, size_t nwords, uint64_t out4[4]) {
  // vm_mem_comm (commitments.rs:192-217) hands MerkleTree::new PAGE_COUNT
  // one-row matrices: all of height 1, so the first digest layer is the
  // root, one sponge over every page's row in page order
  if (!out4 || (nwords && !words)) return LF_ERR_INVALID_ARG;
  sponge8([&](size_t i) { return (uint64_t)words[i]; }, nwords, out4);
  return LF_OK;
}

}  // extern "C"
