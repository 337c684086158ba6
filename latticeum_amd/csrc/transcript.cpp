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

namespace {
#include "p2_consts.inc"
const uint64_t EXT_INIT[64] = LF_P2_EXT_INIT;
const uint64_t EXT_TERM[64] = LF_P2_EXT_TERM;
const uint64_t INTERNAL[22] = LF_P2_INTERNAL;
const uint64_t DIAG_M1[16] = LF_P2_DIAG_M1;
const uint64_t W8_EXT_INIT[32] = LF_P2W8_EXT_INIT;
const uint64_t W8_EXT_TERM[32] = LF_P2W8_EXT_TERM;
const uint64_t W8_DIAG_M1[8] = LF_P2W8_DIAG_M1;

uint64_t sbox7(uint64_t x) {
  uint64_t x2 = gl::mul(x, x), x4 = gl::mul(x2, x2);
  return gl::mul(gl::mul(x4, x2), x);
}
void mds16(uint64_t *s) {
  for (int c = 0; c < 16; c += 4) {
    uint64_t x0 = s[c], x1 = s[c + 1], x2 = s[c + 2], x3 = s[c + 3];
    uint64_t t = gl::add(gl::add(x0, x1), gl::add(x2, x3));
    s[c] = gl::add(t, gl::add(x0, gl::add(x1, x1)));
    s[c + 1] = gl::add(t, gl::add(x1, gl::add(x2, x2)));
    s[c + 2] = gl::add(t, gl::add(x2, gl::add(x3, x3)));
    s[c + 3] = gl::add(t, gl::add(x3, gl::add(x0, x0)));
  }
  for (int k = 0; k < 4; k++) {
    uint64_t sum = gl::add(gl::add(s[k], s[4 + k]), gl::add(s[8 + k], s[12 + k]));
    for (int j = k; j < 16; j += 4) s[j] = gl::add(s[j], sum);
  }
}
void permute(uint64_t *s) {
  mds16(s);
  for (int r = 0; r < 4; r++) {
    for (int i = 0; i < 16; i++) s[i] = sbox7(gl::add(s[i], EXT_INIT[16 * r + i]));
    mds16(s);
  }
  for (int r = 0; r < 22; r++) {
    s[0] = sbox7(gl::add(s[0], INTERNAL[r]));
    uint64_t sum = 0;
    for (int i = 0; i < 16; i++) sum = gl::add(sum, s[i]);
    for (int i = 0; i < 16; i++) s[i] = gl::add(gl::mul(s[i], DIAG_M1[i]), sum);
  }
  for (int r = 0; r < 4; r++) {
    for (int i = 0; i < 16; i++) s[i] = sbox7(gl::add(s[i], EXT_TERM[16 * r + i]));
    mds16(s);
  }
}
// Poseidon2Goldilocks<8> (poseidon2.rs:31-49): the same round structure at
// width 8 (MDSMat4 on both 4-chunks, then the column sums), the reference's
// width-8 external constants (crypto_consts.rs:9-96) and Plonky3's
// MATRIX_DIAG_8_GOLDILOCKS (not vendored: restated, parity unpinned)
void mds8(uint64_t *s) {
  for (int c = 0; c < 8; c += 4) {
    uint64_t x0 = s[c], x1 = s[c + 1], x2 = s[c + 2], x3 = s[c + 3];
    uint64_t t = gl::add(gl::add(x0, x1), gl::add(x2, x3));
    s[c] = gl::add(t, gl::add(x0, gl::add(x1, x1)));
    s[c + 1] = gl::add(t, gl::add(x1, gl::add(x2, x2)));
    s[c + 2] = gl::add(t, gl::add(x2, gl::add(x3, x3)));
    s[c + 3] = gl::add(t, gl::add(x3, gl::add(x0, x0)));
  }
  for (int k = 0; k < 4; k++) {
    uint64_t sum = gl::add(s[k], s[4 + k]);
    s[k] = gl::add(s[k], sum);
    s[4 + k] = gl::add(s[4 + k], sum);
  }
}
void permute8(uint64_t *s) {
  mds8(s);
  for (int r = 0; r < 4; r++) {
    for (int i = 0; i < 8; i++) s[i] = sbox7(gl::add(s[i], W8_EXT_INIT[8 * r + i]));
    mds8(s);
  }
  for (int r = 0; r < 22; r++) {
    s[0] = sbox7(gl::add(s[0], INTERNAL[r]));
    uint64_t sum = 0;
    for (int i = 0; i < 8; i++) sum = gl::add(sum, s[i]);
    for (int i = 0; i < 8; i++) s[i] = gl::add(gl::mul(s[i], W8_DIAG_M1[i]), sum);
  }
  for (int r = 0; r < 4; r++) {
    for (int i = 0; i < 8; i++) s[i] = sbox7(gl::add(s[i], W8_EXT_TERM[8 * r + i]));
    mds8(s);
  }
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
  std::vector<uint64_t> in, out;
  void duplexing() {  // Plonky3 DuplexChallenger::duplexing (overwrite mode)
    for (size_t i = 0; i < in.size(); i++) state[i] = in[i];
    in.clear();
    permute(state);
    out.assign(state, state + 12);
  }
};

extern "C" {

lf_transcript *lf_transcript_new(void) { return new lf_transcript; }
void lf_transcript_free(lf_transcript *t) { delete t; }

void lf_transcript_observe(lf_transcript *t, uint64_t v) {
  t->out.clear();
  t->in.push_back(gl::canon(v));
  if (t->in.size() == 12) t->duplexing();
}

uint64_t lf_transcript_sample(lf_transcript *t) {
  if (!t->in.empty() || t->out.empty()) t->duplexing();
  uint64_t v = t->out.back();
  t->out.pop_back();
  return v;
}

void lf_transcript_absorb_ring(lf_transcript *t, const uint64_t *e, size_t n, int d, int repr) {
  // fiat_shamir.rs:51-60: observe elem.0.0[0], the ark Montgomery limb
  for (size_t i = 0; i < n * (size_t)d; i++)
    lf_transcript_observe(t, repr == LF_REPR_MONTGOMERY ? e[i] : gl::to_mont(e[i]));
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
