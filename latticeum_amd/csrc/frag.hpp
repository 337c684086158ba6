// frag.hpp -- the signed base-256 digit form (D8) of a residue and the byte
// transposition into i8-MFMA operand pieces (ajtai_mfma.hip, kernels_n32.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "gl.hpp"
#include "kernels.hpp"

namespace lfk {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

// x == sum_k d_k 256^k (mod p) with digits d_k in [-128, 127], stored as bytes:
//   t = x <= 0x7F..7F ? x : x + 2^32 - 1;  digits = bytes of (t + 0x80..80) ^ 0x80..80
__device__ __forceinline__ uint64_t d8(uint64_t x) {
  const uint64_t t = x <= 0x7F7F7F7F7F7F7F7Full ? x : x + 0xFFFFFFFFull;
  return (t + 0x8080808080808080ull) ^ 0x8080808080808080ull;
}
// The vector operand (F) rows use the offset form instead: the bytes of the
// canonical x with their top bits flipped. Read as signed bytes they are
// b_k - 128, so they stand for the integer x - FOFF, FOFF = 0x80..80 =
// 128 sum_k 256^k, and a contraction sum_j a_j F_j comes out short by FOFF
// sum_j a_j: the scheme keeps FOFF * (row sums of A) per (row, slot) and the
// contraction's epilogue adds them back (ajtai_mfma.hip, `kr`). Two VALU per
// value against about nine for d8; A keeps the D8 form (it is built once).
constexpr uint64_t FOFF = 0x8080808080808080ull;
__device__ __forceinline__ uint64_t fenc(uint64_t x) { return x ^ FOFF; }

// 16 D8 words (16 columns of one slot) -> 8 operand pieces: u[b] holds digit b
// of the 16 columns, column jj in byte jj
__device__ __forceinline__ void d8_transpose16(const uint64_t *x, uint4 *u) {
  uint32_t lo[16], hi[16];
#pragma unroll
  for (int jj = 0; jj < 16; jj++) {
    lo[jj] = (uint32_t)x[jj];
    hi[jj] = (uint32_t)(x[jj] >> 32);
  }
#pragma unroll
  for (int half = 0; half < 2; half++) {
    const uint32_t *w = half ? hi : lo;
#pragma unroll
    for (int bb = 0; bb < 4; bb += 2) {  // digits 4*half + bb and + bb + 1
      uint32_t dw0[4], dw1[4];
#pragma unroll
      for (int q = 0; q < 4; q++) {
        // [x0_b, x1_b, x0_b+1, x1_b+1] and [x2_b, x3_b, x2_b+1, x3_b+1]
        const uint32_t sel = (uint32_t)bb | ((uint32_t)(4 + bb) << 8) | ((uint32_t)(bb + 1) << 16) |
                             ((uint32_t)(5 + bb) << 24);
        const uint32_t t01 = __builtin_amdgcn_perm(w[4 * q + 1], w[4 * q], sel);
        const uint32_t t23 = __builtin_amdgcn_perm(w[4 * q + 3], w[4 * q + 2], sel);
        dw0[q] = __builtin_amdgcn_perm(t23, t01, 0x05040100u);
        dw1[q] = __builtin_amdgcn_perm(t23, t01, 0x07060302u);
      }
      u[4 * half + bb] = make_uint4(dw0[0], dw0[1], dw0[2], dw0[3]);
      u[4 * half + bb + 1] = make_uint4(dw1[0], dw1[1], dw1[2], dw1[3]);
    }
  }
}

// 4 x 4 byte transpose: o[k] byte i = w[i] byte k
__device__ __forceinline__ void byte_tr4(const uint32_t *w, uint32_t *o) {
#pragma unroll
  for (int bb = 0; bb < 4; bb += 2) {
    const uint32_t sel =
        (uint32_t)bb | ((uint32_t)(4 + bb) << 8) | ((uint32_t)(bb + 1) << 16) | ((uint32_t)(5 + bb) << 24);
    const uint32_t t01 = __builtin_amdgcn_perm(w[1], w[0], sel);
    const uint32_t t23 = __builtin_amdgcn_perm(w[3], w[2], sel);
    o[bb] = __builtin_amdgcn_perm(t23, t01, 0x05040100u);
    o[bb + 1] = __builtin_amdgcn_perm(t23, t01, 0x07060302u);
  }
}
// the inverse of d8_transpose16 on offset-form (fenc) operand rows: 8 operand
// pieces (byte b of 16 columns) -> the 16 residues (canonical)
__device__ __forceinline__ void fenc_untranspose16(const uint4 *u, uint64_t *x) {
#pragma unroll
  for (int q = 0; q < 4; q++) {
    uint32_t w[8], lo[4], hi[4];
#pragma unroll
    for (int k = 0; k < 8; k++) w[k] = q == 0 ? u[k].x : q == 1 ? u[k].y : q == 2 ? u[k].z : u[k].w;
    byte_tr4(w, lo);
    byte_tr4(w + 4, hi);
#pragma unroll
    for (int cc = 0; cc < 4; cc++) x[4 * q + cc] = ((uint64_t)lo[cc] | ((uint64_t)hi[cc] << 32)) ^ FOFF;
  }
}

// Streaming (nontemporal) stores for outputs written once and not re-read by
// the writing launch. At W = 2^14 (61 GB of decomposition outputs per step)
// they keep the outputs from cycling through the caches (15.5 -> 14.2 ms); at
// small sizes the next launches re-read the outputs from the caches, and
// plain stores are better (d = 24, W = 19 763: 706 -> 376 steps/s with nt).
__device__ __forceinline__ void nt_store(uint64_t *p, uint64_t v) { __builtin_nontemporal_store(v, p); }
__device__ __forceinline__ void nt_store(uint4 *p, uint4 v) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  const u32x4 t = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(t, reinterpret_cast<u32x4 *>(p));
}
template <bool NT, class T>
__device__ __forceinline__ void out_store(T *p, T v) {
  if (NT)
    nt_store(p, v);
  else
    *p = v;
}
// outputs above this many bytes per launch are written with streaming stores
constexpr size_t STREAM_OUT_BYTES = (size_t)4 << 30;
// Streaming (nontemporal) stores for the fused decompositions' outputs. When
// nothing later in the step re-reads f_coeff_k or f_k (d = 1024: the fold runs
// in coefficient form from the packed digits), they stream at every size: the
// contraction's single pass over the operand rows is faster from HBM than after
// the rows went through the caches (W = 464, 4 streams: contraction 0.27 ->
// 0.235 ms, 1,288-1,318 -> 1,345-1,347 steps/s). When the step folds f_0 from
// f_k in NTT form (`refold`: d = 4096), cached stores are kept below 4 GiB of
// outputs so the fold finds f_k in the caches. LATTICEUM_AMD_DEC_NT=0 never
// streams, =1 always streams.
inline bool dec_streaming(size_t out_bytes, bool refold) {
  const char *e = getenv("LATTICEUM_AMD_DEC_NT");
  if (e && e[0] == '0') return false;
  if (e && e[0] == '1') return true;
  return !refold || out_bytes > STREAM_OUT_BYTES;
}

// vector-major operand layout (uint4 index of digit 0; digit k adds 4k, chunk c adds c FV_CHUNK)
constexpr size_t FV_CHUNK = 32 * 2 * 8 * 4;
__device__ __forceinline__ size_t fv_index(size_t s, int nch, int c, int r, int h) {
  return ((((s >> 2) * nch + c) * 32 + r) * 2 + h) * 32 + (s & 3);
}

// column of operand column t (< 32) of chunk c in the contraction order (Lp, Wp: FragGeom)
__device__ __forceinline__ size_t frag_column(int c, int t, int Lp, size_t Wp, bool &ok) {
  const size_t u = 2 * (size_t)c + (t >> 4);
  const size_t G = u / Lp, l = u % Lp, g = 16 * G + (t & 15);
  ok = g < Wp;
  return g * Lp + l;
}

// folding.rs:258-268 compute_f_0 from the D8 operand rows (the packed / f_k-free
// steps' fallback for a rho that is not short, and d = 4096's fold): virtual block
// vb < (d / 16) nch takes 16 slots (four slot quads, one 128-B line of every
// element) of one 32-column chunk; thread (quad, slot, half, column part, vector
// group) undoes the byte transposition of its CW columns (CW = 16: all of its
// half's, 256 threads; CW = 8: one of two parts, 512 threads and about half the
// registers, so twice the waves keep loads in flight) for vectors v = vg, vg + 8,
// .. and multiply-accumulates rho_v (.) f_v lazily; the 8 vector groups meet in LDS
// (red: 512 x 9 u64) and each output column's 16 slots go out as one 128-B run.
// Each thread reads its rows' dead flags and rho values before any operand row.
// Block-uniform (it synchronises the block). qd > 0: the operand slots are
// quarter-major (FragGeom::qperm, d = 4096): operand slot o holds slot
// (o % qd) 4 + o / qd, so one block's 16 operand slots are every 4th slot.
__device__ __forceinline__ int frag_slot(int o, int qd) { return qd ? (o % qd) * 4 + o / qd : o; }
template <int CW = 16>
__device__ __forceinline__ void fold_frag_block(size_t vb, const uint4 *frag, int nch, int Lp, size_t Wp,
                                                const FoldRows &fr, const uint64_t *rho, int d, size_t N,
                                                uint64_t *out, uint64_t *red, int qd = 0) {
  static_assert(CW == 16 || CW == 8, "16 or 8 columns per thread");
  constexpr int NT = CW == 16 ? 256 : 512;  // threads of the block
  // CW = 16: tid = (qq, sl, h, vg); CW = 8: tid = (qq, vg, h, sl, cp), so the 8 lanes
  // of one (vector, half) read one 64-B run (4 slots x 2 column parts x 8 B)
  const int tid = threadIdx.x;
  const int vg = CW == 8 ? (tid >> 4) & 7 : tid & 7;
  const int cp = CW == 8 ? tid & 1 : 0;  // which 8 of the half's 16 columns
  const int h = CW == 8 ? (tid >> 3) & 1 : (tid >> 3) & 1;
  const int sl = CW == 8 ? (tid >> 1) & 3 : (tid >> 4) & 3;
  const int qq = CW == 8 ? tid >> 7 : tid >> 6;
  const int ng = d >> 4, G = (int)(vb % ng), c = (int)(vb / ng);
  const int s = 16 * G + 4 * qq + sl, sr = frag_slot(s, qd);
  constexpr int MAXR = (LF_MAX_VECS + 7) / 8;  // rows per vector group
  // Three rounds of independent loads (no load waits on another of its round):
  // the rows' metadata, then their dead flags and rho values, then every live
  // row's operand bytes -- so a block pays three memory latencies, not one per row
  bool use[MAXR];
  int row[MAXR], rix[MAXR];
#pragma unroll
  for (int i = 0; i < MAXR; i++) {
    const int v = vg + 8 * i;
    use[i] = v < fr.n;
    row[i] = fr.row[use[i] ? v : 0];
    rix[i] = fr.rho[use[i] ? v : 0];
  }
  uint64_t rv[MAXR];
  const uint4 *pr[MAXR];
  if (fr.dead.flags) {  // uniform
    // a unit the decomposition left unwritten holds zero: nothing to add
    uint8_t fl[MAXR];
#pragma unroll
    for (int i = 0; i < MAXR; i++) fl[i] = fr.dead.flags[(2 * (size_t)c + h) * 32 + row[i]];
#pragma unroll
    for (int i = 0; i < MAXR; i++)
      if (((fr.dead.rows >> row[i]) & 1) && fl[i]) use[i] = false;
  }
#pragma unroll
  for (int i = 0; i < MAXR; i++) {
    rv[i] = rho[(size_t)rix[i] * d + sr];
    pr[i] = frag + fv_index(s, nch, c, row[i], h);
  }
  gl::CAcc acc[CW];
#pragma unroll
  for (int j = 0; j < CW; j++) gl::cacc_zero(acc[j]);
  if (CW == 16) {
#pragma unroll
    for (int i = 0; i < MAXR; i++) {
      if (!use[i]) continue;
      uint64_t x[CW];
      uint4 u[8];
#pragma unroll
      for (int k = 0; k < 8; k++) u[k] = pr[i][4 * k];
      fenc_untranspose16(u, x);
#pragma unroll
      for (int j = 0; j < CW; j++) gl::cacc_mad(acc[j], rv[i], x[j]);
    }
  } else {
#pragma unroll
    for (int i = 0; i < MAXR; i++) {
      if (!use[i]) continue;
      // columns 8 cp .. 8 cp + 7 are bytes 8 cp .. 8 cp + 7 of each digit's piece
      uint2 u2[8];
#pragma unroll
      for (int k = 0; k < 8; k++) u2[k] = reinterpret_cast<const uint2 *>(pr[i] + 4 * k)[cp];
      uint64_t x[CW];
#pragma unroll
      for (int q = 0; q < 2; q++) {
        uint32_t w[8], lo[4], hi[4];
#pragma unroll
        for (int k = 0; k < 8; k++) w[k] = q == 0 ? u2[k].x : u2[k].y;
        byte_tr4(w, lo);
        byte_tr4(w + 4, hi);
#pragma unroll
        for (int cc = 0; cc < 4; cc++) x[4 * q + cc] = ((uint64_t)lo[cc] | ((uint64_t)hi[cc] << 32)) ^ FOFF;
      }
#pragma unroll
      for (int j = 0; j < CW; j++) gl::cacc_mad(acc[j], rv[i], x[j]);
    }
  }
  // output o = column (32) x slot (16): o = (16 h + jj) 16 + 4 qq + sl
#pragma unroll
  for (int j = 0; j < CW; j++) {
    const int jj = CW * cp + j;
    red[((16 * h + jj) * 16 + 4 * qq + sl) * 9 + vg] = gl::cacc_reduce(acc[j]);
  }
  __syncthreads();
#pragma unroll
  for (int rep = 0; rep < 512 / NT; rep++) {
    const int o = tid + NT * rep, j = o >> 4, s16 = o & 15;
    uint64_t t = red[o * 9];
#pragma unroll
    for (int g = 1; g < 8; g++) t = gl::add(t, red[o * 9 + g]);
    bool ok;
    const size_t col = frag_column(c, j, Lp, Wp, ok);
    if (ok && col < N) out[col * d + frag_slot(16 * G + s16, qd)] = t;
  }
  __syncthreads();  // red is free for the next virtual block
}

}  // namespace lfk
