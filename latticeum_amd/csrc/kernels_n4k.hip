// kernels_n4k.hip -- the X^4096 + 1 ring (BASELINE configs[4]) on the
// register-resident 1024-point transform of ntt32.hpp. With j = a + 1024 b and
// m = m0 + 4 m1 (a, m1 < 1024; b, m0 < 4), tools/ntt4096_model.py:
//   X[m0 + 4 m1] = NTT1024_{psi^4}(y_m0)[m1]
//   y_m0[a]      = psi^((2 m0 - 3) a) * sum_b x[a + 1024 b] w8^(b (2 m0 + 1)),  w8 = psi^1024 = 2^120
// psi^4 is the X^1024 + 1 root, so the sub-transform is n32::forward with the
// d = 1024 middle factors. Each quarter m0 is independent: a wave owns one m0
// (wave-uniform) and its two halves two different work items, so no wave waits
// for another and there is no s_barrier in the loop. The four waves of one
// work item share a block (one CU, one L2), so their interleaved slot stores
// (stride 4) merge into whole lines before they reach HBM.
#include <stdlib.h>
#include <string.h>

#include "digits.hpp"
#include "frag.hpp"
#include "kernels.hpp"
#include "ntt32.hpp"

namespace lfk {

namespace {
constexpr int D4 = 4096, Q4 = 1024;
constexpr int WPB4 = 8;  // two work-item pairs x four quarters; one block per CU (LDS)

// bit t of a 16-bit value -> bit 4 t (Morton spread for four interleaved values)
__device__ __forceinline__ uint64_t spread4(uint32_t v) {
  uint64_t x = v & 0xFFFFu;
  x = (x | (x << 24)) & 0x000000FF000000FFull;
  x = (x | (x << 12)) & 0x000F000F000F000Full;
  x = (x | (x << 6)) & 0x0303030303030303ull;
  x = (x | (x << 3)) & 0x1111111111111111ull;
  return x;
}
__device__ __forceinline__ uint32_t sign_mag16(uint64_t x, int K, bool &bad) {
  const int64_t a = signed_rep(x);
  const uint64_t m = a < 0 ? (uint64_t)(-a) : (uint64_t)a;
  bad |= (m >> K) != 0;
  return (uint32_t)(m & 0x7FFF) | (a < 0 ? 0x8000u : 0u);
}
}  // namespace

// ---------------------------------------------------------------- decompose_witness, d = 4096
// The coefficients of element e at a, a + 1024, a + 2048, a + 3072 as one word:
// magnitude bit t of quarter b at bit 4 t + b, the sign of quarter b at bit 60 + b
// (K <= 15), so digit plane k of all four is the nibble at 4 k and one shift.
__global__ void k_pack_sm4(FusedSides sd, size_t N, int K, uint64_t *sm4, int *err) {
  const size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;  // (side, element, a)
  if (t >= sd.nside * N * Q4) return;
  const int side = t >= N * Q4;
  const size_t ea = t - side * N * Q4;
  const uint64_t *x = sd.f_coeff[side] + (ea >> 10) * D4 + (ea & (Q4 - 1));
  bool bad = false;
  uint64_t w = 0;
#pragma unroll
  for (int b = 0; b < 4; b++) w |= spread4(sign_mag16(x[b * Q4], K, bad)) << b;
  if (bad) raise(err, 1);
  sm4[t] = w;
}

// One quarter m0 of digit plane kb of one element, from the element's packed
// words (lane r: words of a = r + 32 k): this quarter's digits (b = m0) to oc[32 k],
// y_m0 (the radix-4 butterfly of the four digits is a table lookup: 81 values
// per m0, zt[nibble | signs << 4]; then the twist), and its 1024-point transform:
// v[i] = slot m0 + 4 (r + 32 brv5(i)).
template <bool NT>
__device__ __forceinline__ void quarter_ntt(const uint64_t *words, int kb, int m0, const uint64_t *zt,
                                            const uint64_t *tw, uint64_t *oc, const uint64_t *mid, uint64_t *T, int r,
                                            uint64_t *v) {
  n32::load_row32(words, v);
#pragma unroll
  for (int k = 0; k < 32; k++) {
    const uint64_t w = v[k];
    const uint32_t nib = (uint32_t)(w >> (4 * kb)) & 15u, sg = (uint32_t)(w >> 60);
    const uint32_t bit = (nib >> m0) & 1u, neg = (sg >> m0) & 1u;
    // this quarter's digit: 0, 1 or p - 1 = 0xFFFFFFFF00000000
    const uint64_t own = ((uint64_t)(bit & neg) * 0xFFFFFFFF00000000ull) | (uint64_t)(bit & (neg ^ 1u));
    out_store<NT>(&oc[32 * k], own);
    v[k] = zt[nib | (sg << 4)];
  }
#pragma unroll
  for (int k0 = 0; k0 < 32; k0 += 8) {
    uint64_t t8[8];
#pragma unroll
    for (int k = 0; k < 8; k++) t8[k] = tw[32 * (k0 + k)];
#pragma unroll
    for (int k = 0; k < 8; k++) v[k0 + k] = gl::mul(v[k0 + k], t8[k]);
  }
  n32::forward(v, mid, T, r);
}
// w_ccs_k's Horner step (B = 2^lb) over the limbs, from the top one
__device__ __forceinline__ void horner_step(uint64_t *acc, const uint64_t *v, bool first, int lb, uint64_t b_pow) {
  if (first) {
#pragma unroll
    for (int i = 0; i < 32; i++) acc[i] = v[i];
  } else if (lb == 15) {  // GoldiLocksDP B = 2^15: a shift instead of a product
#pragma unroll
    for (int i = 0; i < 32; i++) acc[i] = gl::add_weak(gl::shl_small_weak(acc[i], 15), v[i]);
  } else {
#pragma unroll
    for (int i = 0; i < 32; i++) acc[i] = gl::add(gl::mul(acc[i], b_pow), v[i]);
  }
}

// LF/nifs/decomposition.rs:162-167, decomposition/utils.rs:45-49, arith.rs:324-338
// for b_small = 2 (digit = sign(v) bit_k(|v|)). A work item is (side, group g,
// plane k); per limb l the wave's quarter m0 writes f_coeff_k's quarter b = m0
// and slots m0 + 4 m1 of f_k; w_ccs_k = sum_l B^l f_k[gL + l] accumulates in
// the same registers.
__global__ void __launch_bounds__(512, 1) k_decompose_n4k(const uint64_t *sm4_all, size_t N, int L, int lb, int K,
                                                         FusedSides sd, const uint64_t *mid_fg, const uint64_t *tw_g,
                                                         const uint64_t *ztab_g, uint64_t *sink) {
  __shared__ uint64_t lds_all[WPB4 * n32::WAVE_U64];
  __shared__ uint64_t mid_f[n32::MID_U64];
  __shared__ uint64_t ztab[4 * 256];
  n32::stage_mid(mid_f, mid_fg);
  for (int q = threadIdx.x; q < 4 * 256; q += blockDim.x) ztab[q] = ztab_g[q];
  __syncthreads();
  const int lane = threadIdx.x & 63, wib = threadIdx.x >> 6;
  const int r = lane & 31, h = lane >> 5, m0 = wib & 3;
  uint64_t *T = lds_all + wib * n32::WAVE_U64 + h * n32::HALF_U64;
  const uint64_t *zt = ztab + m0 * 256;
  const uint64_t *tw = tw_g + m0 * Q4 + r;
  const size_t W = N / L, ntask = sd.nside * W * K, npair = (ntask + 1) / 2;
  const uint64_t b_pow = gl::mul_pow2(1, lb);  // B = 2^lb
  for (size_t tp = (size_t)blockIdx.x * 2 + (wib >> 2); tp < npair; tp += (size_t)gridDim.x * 2) {
    // the two halves: consecutive planes of (mostly) one group, so both read the same words
    const size_t t = 2 * tp + h;
    const bool ok = t < ntask;
    const size_t tt = ok ? t : 0;
    const int kb = (int)(tt % K);
    const size_t gt = tt / K;
    const int side = gt >= W;
    const size_t g = gt - side * W;
    const uint64_t *sm4 = sm4_all + side * N * Q4;
    uint64_t acc[32];
    for (int l = L - 1; l >= 0; l--) {
      const size_t e = (size_t)kb * N + g * L + l;
      uint64_t v[32];
      quarter_ntt<false>(sm4 + (g * L + l) * Q4 + r, kb, m0, zt, tw,
                         (ok ? sd.f_coeff_k[side] + e * D4 + m0 * Q4 : sink) + r, mid_f, T, r, v);
      uint64_t *of = (ok ? sd.f_k[side] + e * D4 : sink) + m0 + 4 * r;
#pragma unroll
      for (int i = 0; i < 32; i++) of[128 * n32::brv5(i)] = v[i];
      horner_step(acc, v, l == L - 1, lb, b_pow);
    }
    uint64_t *ow = (ok ? sd.w_ccs_k[side] + ((size_t)kb * W + g) * D4 : sink) + m0 + 4 * r;
#pragma unroll
    for (int i = 0; i < 32; i++) ow[128 * n32::brv5(i)] = gl::canon(acc[i]);
  }
}

// ---------------------------------------------------------------- fused with the Ajtai operands
// As decompose_fused (kernels_n32.hip) for d = 1024: a block of 8 waves owns 16
// consecutive groups (one per half-wave) at one digit plane and one quarter m0,
// so for each limb l it holds one 16-column unit of the contraction order
// (Lp = L) and writes the plane (k >= 1) straight into the vector-major operand
// buffer. The operand slots are quarter-major (FragGeom::qperm): one quarter's
// 1024 slots are 256 whole slot quads, so the pieces of a quad (4 neighbouring
// threads) form whole 64-B segments. The blocks of the four quarters of a unit
// are b, b + 8, b + 16, b + 24: the same XCD (blocks are dealt round-robin over
// the 8), so the interleaved f_k slot stores of the four meet in one L2.
//
// The digits come as one byte per coefficient quad and plane (k_pack_sm8:
// nibble | signs << 4, the index of the butterfly table), 32 bytes per lane per
// limb, prefetched one limb ahead (issued before the limb's stores, so waiting
// for them does not drain those stores). The quarter's twists, the table and
// the middle factors stay in LDS.
constexpr int FQ_WAVES = 8;
constexpr int FQ_SROW = 17;  // staging row stride in u64 (16 groups + pad: conflict-free)
constexpr int FQ_T_U64 = FQ_WAVES * n32::WAVE_U64;
constexpr int FQ_S_U64 = Q4 * FQ_SROW;
constexpr int FQ_LDS_U64 = FQ_T_U64 > FQ_S_U64 ? FQ_T_U64 : FQ_S_U64;

// byte (element e, plane kb, lane r, k) at ((e K + kb) 32 + r) 32 + k; one
// thread per (side, e, r, j) packs k = 4 j .. 4 j + 3 (one word per plane)
__global__ void k_pack_sm8(FusedSides sd, size_t N, int K, int *err) {
  const size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;  // (side, element, r, j)
  if (t >= sd.nside * N * 256) return;
  const int side = t >= N * 256;
  const size_t erj = t - side * N * 256, e = erj >> 8;
  const int r = (int)((erj >> 3) & 31), j = (int)(erj & 7);
  const uint64_t *x = sd.f_coeff[side] + e * D4 + r + 128 * j;
  uint64_t w[4];
  bool bad = false;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    w[k] = 0;
#pragma unroll
    for (int b = 0; b < 4; b++) w[k] |= spread4(sign_mag16(x[32 * k + b * Q4], K, bad)) << b;
  }
  if (bad) raise(err, 1);
  uint32_t *o = sd.smg[side] + (e * K * 32 + r) * 8 + j;
  for (int kb = 0; kb < K; kb++) {
    uint32_t q = 0;
#pragma unroll
    for (int k = 0; k < 4; k++)
      q |= (((uint32_t)(w[k] >> (4 * kb)) & 15u) | ((uint32_t)(w[k] >> 60) << 4)) << (8 * k);
    o[kb * 256] = q;
  }
}

template <bool NT>
__global__ void __launch_bounds__(512, 1) k_decompose_n4k_fused(size_t N, int L, int lb, int K,
                                                               FusedSides sd, const uint64_t *mid_fg,
                                                               const uint64_t *tw_g, const uint64_t *ztab_g,
                                                               uint4 *frag, int nch, uint64_t *sink) {
  __shared__ uint64_t lds_all[FQ_LDS_U64];
  __shared__ uint64_t mid_f[n32::MID_U64];
  __shared__ uint64_t twl[Q4];
  __shared__ uint64_t zt[256];
  __shared__ uint32_t vote[2][FQ_WAVES];  // per wave: its plane is nonzero in the current unit (as decompose_fused)
  const int m0 = (blockIdx.x >> 3) & 3;
  n32::stage_mid(mid_f, mid_fg);
  for (int q = threadIdx.x; q < Q4; q += blockDim.x) twl[q] = tw_g[m0 * Q4 + q];
  for (int q = threadIdx.x; q < 256; q += blockDim.x) zt[q] = ztab_g[m0 * 256 + q];
  __syncthreads();
  const int lane = threadIdx.x & 63, wib = threadIdx.x >> 6;
  const int r = lane & 31, h = lane >> 5, hw = 2 * wib + h;  // hw: this half's group within the block
  uint64_t *T = lds_all + wib * n32::WAVE_U64 + h * n32::HALF_U64;
  uint64_t *S = lds_all;
  const size_t W = N / L, nblk = (W + 15) / 16, nunit = sd.nside * nblk * K;
  const uint64_t b_pow = gl::mul_pow2(1, lb);  // B = 2^lb
  const size_t ustride = 8 * (size_t)(gridDim.x >> 5);
  int nvote = 0;  // units voted on so far (block-uniform)
  for (size_t unit = (blockIdx.x & 7) + 8 * (size_t)(blockIdx.x >> 5); unit < nunit; unit += ustride) {
    const int side = unit >= nblk * K;
    const size_t B = unit / K - side * nblk;
    const int kb = (int)(unit % K);
    const size_t g = 16 * B + hw;
    const bool ok = g < W;
    const size_t gg = ok ? g : 0;
    // this lane's 32 bytes of limb l: 8 words
    const uint32_t *sm8 = sd.smg[side];
    auto bytes_of = [&](int l) { return sm8 + (((gg * L + l) * K + kb) * 32 + r) * 8; };
    // f_coeff_k / f_k rows only when the caller keeps them (side-uniform); packed
    // steps keep the bytes above as the decomposed witnesses' only form
    uint64_t *fck = sd.f_coeff_k[side], *fk = sd.f_k[side];
    const int row = kb > 0 ? sd.row0[side] + kb - 1 : sd.row_p0[side];
    uint32_t wn[8];
    {
      const uint4 *p = reinterpret_cast<const uint4 *>(bytes_of(L - 1));
      const uint4 a = p[0], c = p[1];
      wn[0] = a.x, wn[1] = a.y, wn[2] = a.z, wn[3] = a.w, wn[4] = c.x, wn[5] = c.y, wn[6] = c.z, wn[7] = c.w;
    }
    asm volatile("" : "+v"(wn[0]), "+v"(wn[1]), "+v"(wn[2]), "+v"(wn[3]), "+v"(wn[4]), "+v"(wn[5]), "+v"(wn[6]),
                 "+v"(wn[7]));
    uint64_t acc[32];
    for (int l = L - 1; l >= 0; l--) {
      const size_t e = (size_t)kb * N + gg * L + l;
      uint64_t v[32], own[32];
      // plane kb of this limb zero on both of the wave's elements (the top limb's
      // planes 4..K-1; kernels_n32.hip decompose_fused): the transform is zero.
      // Every quarter's block reads the same bytes, so the four agree.
      uint32_t nz = 0;
#pragma unroll
      for (int q = 0; q < 8; q++) nz |= wn[q];
      const bool live = __ballot((nz & 0x0F0F0F0Fu) != 0) != 0;
#pragma unroll
      for (int k = 0; k < 32; k++) {
        const uint32_t byte = (wn[k >> 2] >> (8 * (k & 3))) & 0xFFu;
        const uint32_t bit = (byte >> m0) & 1u, neg = (byte >> (4 + m0)) & 1u;
        // this quarter's digit: 0, 1 or p - 1 = 0xFFFFFFFF00000000
        own[k] = ((uint64_t)(bit & neg) * 0xFFFFFFFF00000000ull) | (uint64_t)(bit & (neg ^ 1u));
        v[k] = zt[byte];
      }
      {  // the next limb's bytes (at l = 0 a harmless reload of limb L - 1)
        const uint4 *p = reinterpret_cast<const uint4 *>(bytes_of(l > 0 ? l - 1 : L - 1));
        const uint4 a = p[0], c = p[1];
        wn[0] = a.x, wn[1] = a.y, wn[2] = a.z, wn[3] = a.w, wn[4] = c.x, wn[5] = c.y, wn[6] = c.z, wn[7] = c.w;
      }
      if (fck) {
        uint64_t *oc = (ok ? fck + e * D4 + m0 * Q4 : sink) + r;
#pragma unroll
        for (int k = 0; k < 32; k++) out_store<NT>(&oc[32 * k], own[k]);
      }
      if (live) {
#pragma unroll
        for (int k = 0; k < 32; k++) v[k] = gl::mul(v[k], twl[r + 32 * k]);
        n32::forward(v, mid_f, T, r);
      } else {
#pragma unroll
        for (int k = 0; k < 32; k++) v[k] = 0;
      }
      if (fk) {
        uint64_t *of = (ok ? fk + e * D4 : sink) + m0 + 4 * r;
#pragma unroll
        for (int i = 0; i < 32; i++) of[128 * n32::brv5(i)] = v[i];
      }
      horner_step(acc, v, l == L - 1, lb, b_pow);
      if (row >= 0) {  // planes k >= 1, and plane 0 when it has a row (the f_k-free steps fold from the rows)
        const size_t u = B * L + l;  // contraction unit of these 16 columns
        // dead units as in decompose_fused: the four quarter blocks of a unit vote
        // on the same bytes, so they write the same flag
        const int vs = nvote++ & 1;
        if (sd.dead && lane == 0) vote[vs][wib] = live ? 1u : 0u;
        __syncthreads();  // every wave is past its transpose: S may overwrite T
        bool any = true;
        if (sd.dead) {
          uint32_t a = 0;
#pragma unroll
          for (int q = 0; q < FQ_WAVES; q++) a |= vote[vs][q];
          any = a != 0;
          if (threadIdx.x == 0) sd.dead[u * 32 + row] = any ? 0 : 1;
        }
        if (!any) continue;  // block-uniform: no further barrier for this unit
#pragma unroll
        for (int i = 0; i < 32; i++) S[(r + 32 * n32::brv5(i)) * FQ_SROW + hw] = fenc(v[i]);
        __syncthreads();
        const int c = (int)(u >> 1), uh = (int)(u & 1);
#pragma unroll
        for (int rep = 0; rep < 2; rep++) {
          const int m1 = threadIdx.x + 512 * rep;
          const uint64_t *src = S + m1 * FQ_SROW;
          uint64_t x[16];
#pragma unroll
          for (int j = 0; j < 16; j++) x[j] = src[j];
          uint4 pu[8];
          d8_transpose16(x, pu);
          uint4 *out = frag + fv_index((size_t)m0 * Q4 + m1, nch, c, row, uh);
#pragma unroll
          for (int b = 0; b < 8; b++) out_store<NT>(&out[4 * b], pu[b]);
        }
        __syncthreads();  // S consumed before the next transpose
      }
    }
    uint64_t *ow = (ok ? sd.w_ccs_k[side] + ((size_t)kb * W + g) * D4 : sink) + m0 + 4 * r;
#pragma unroll
    for (int i = 0; i < 32; i++) ow[128 * n32::brv5(i)] = gl::canon(acc[i]);
  }
}

// ---------------------------------------------------------------- stage 1 on the matrix cores
// The same step as k_decompose_n4k_fused with each quarter's stage 1 as one ternary
// i8 product (tools/ntt4096_mx_model.py): with a = j1 + 32 j2 the quarter's input
// is y[a] = s^a sum_b c_b x_b[a] (s = psi^(2 m0 - 3), c_b = 2^(120 b (2 m0 + 1))), so
//   Y[j1][m1] s^-j1 = sum_{b, j2} Z2[m1][32 b + j2] x_b[j1 + 32 j2],
//   Z2[m1][32 b + j2] = zeta^((2 m1 + 1) j2) s^(32 j2) c_b,
// a K = 128 product of Z2's 8 D8 byte planes with the digits, and s^j1 joins the
// middle factors (midq). The product runs transposed (A = the digits, rows j1; B =
// Z2, columns m1), so lane (m1 = r, h) gets rows j1 = (i & 3) + 8 (i >> 2) + 4 h
// of column m1, and one exchange between the wave's halves (v_permlane32_swap) gives
// lane (r, h) all 32 j1 of element h: no transpose tile. Without it the staging tile
// of the operand rows fits in halves (512 slots, two rounds per unit) beside the
// 32 KiB of Z2 planes and the middle factors. The lookup of the radix-4 butterfly,
// the twist (32 products) and the 80 stage-1 butterflies per lane are gone.
// Packed steps only (no f_coeff_k rows): the digits are read as the MFMA's A operand.
constexpr int FM_SROW = 17;                   // staging row stride in u64 (16 groups + pad)
constexpr int FM_S_U64 = (Q4 / 2) * FM_SROW;  // half the quarter's slots per round
// digit bytes (nibble = |digit| bits of the four quarters b, signs << 4) -> the
// signed ternary bytes of quarter b
__device__ __forceinline__ int tern4(uint32_t w, int b) {
  const uint32_t y = (w >> b) & 0x01010101u, sg = (w >> (4 + b)) & 0x01010101u;
  return (int)(y | ((y & sg) * 0xFEu));
}
// one element's stage 1 into 16 values: out[i] = Y'[j1 = (i & 3) + 8 (i >> 2) + 4 h][m1 = r]
// (before its middle factor, midq_apply); w4: this lane's 16 digit bytes (j2 = 16 h .. 16 h + 15)
__device__ __forceinline__ void mx_stage1_q(const int8_t *zl, const uint32_t *w4, int r, int h, uint64_t *out) {
  v4i a[4];
#pragma unroll
  for (int b = 0; b < 4; b++) a[b] = (v4i){tern4(w4[0], b), tern4(w4[1], b), tern4(w4[2], b), tern4(w4[3], b)};
  auto zpiece = [&](int t, int b) { return *reinterpret_cast<const v4i *>(zl + (t * 32 + r) * 128 + 32 * b + 16 * h); };
  auto plane = [&](int t) {
    v16i acc = (v16i){0};
#pragma unroll
    for (int b = 0; b < 4; b++) acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[b], zpiece(t, b), acc, 0, 0, 0);
    return acc;
  };
  // Q = sum_t 2^(8t) D_t over 4 planes (|D_t| <= 128 x 128: pairs fit int32)
  auto quarter = [&](int t0, int64_t *q) {
    v16i a0 = plane(t0), a1 = plane(t0 + 1);
    int32_t p[16];
#pragma unroll
    for (int i = 0; i < 16; i++) p[i] = a0[i] + a1[i] * 256;
    a0 = plane(t0 + 2);
    a1 = plane(t0 + 3);
#pragma unroll
    for (int i = 0; i < 16; i++) q[i] = (int64_t)p[i] + (int64_t)a0[i] * 65536 + (int64_t)a1[i] * (1ll << 24);
  };
  int64_t q0[16], q1[16];
  quarter(0, q0);
  quarter(4, q1);
#pragma unroll
  for (int i = 0; i < 16; i++) {
    // Y = Q0 + Q1 2^32 (|Q| < 2^39) folded as in kernels_n32.hip mx_stage1
    const int64_t q1h = q1[i] >> 32;
    const int64_t A = q0[i] - q1h;
    const int64_t T = (A >> 32) + (int64_t)(uint32_t)q1[i] + q1h;
    const uint64_t U = ((uint64_t)T << 32) | (uint32_t)A;
    const uint64_t y = U + (uint64_t)((T >> 32) * (int64_t)gl::EPS);
    out[i] = y;  // the middle factors follow for both elements at once (midq_apply)
  }
}
// y0, y1 *= midq[j1][brv5(r)], one table read per row for both elements
__device__ __forceinline__ void midq_apply(const uint64_t *midl, uint64_t *y0, uint64_t *y1, int r, int h) {
#pragma unroll
  for (int i = 0; i < 16; i++) {
    const int j1 = (i & 3) + 8 * (i >> 2) + 4 * h;
    const uint64_t m = midl[j1 * 32 + n32::brv5(r)];
    y0[i] = gl::mul(y0[i], m);
    y1[i] = gl::mul(y1[i], m);
  }
}

template <bool NT>
__global__ void __launch_bounds__(512, 1) k_decompose_n4k_mx(size_t N, int L, int lb, int K, FusedSides sd,
                                                            const uint64_t *midq_g, const uint64_t *zq_g,
                                                            uint4 *frag, int nch, uint64_t *sink) {
  __shared__ uint64_t S[FM_S_U64];
  __shared__ uint64_t midl[n32::MID_U64];
  __shared__ uint4 zl4[2048];  // this quarter's 32 KiB of Z2 planes [t][m1][K]
  __shared__ uint32_t vote[2][FQ_WAVES];
  const int m0 = (blockIdx.x >> 3) & 3;
  for (int q = threadIdx.x; q < n32::MID_U64; q += blockDim.x) midl[q] = midq_g[m0 * 1024 + q];
  {
    const uint4 *src = reinterpret_cast<const uint4 *>(zq_g) + (size_t)m0 * 2048;
    for (int q = threadIdx.x; q < 2048; q += blockDim.x) zl4[q] = src[q];
  }
  __syncthreads();
  const int8_t *zl = reinterpret_cast<const int8_t *>(zl4);
  const int lane = threadIdx.x & 63, wib = threadIdx.x >> 6;
  const int r = lane & 31, h = lane >> 5, hw = 2 * wib + h;  // hw: this half's group within the block
  const size_t W = N / L, nblk = (W + 15) / 16, nunit = sd.nside * nblk * K;
  const uint64_t b_pow = gl::mul_pow2(1, lb);  // B = 2^lb
  const size_t ustride = 8 * (size_t)(gridDim.x >> 5);
  int nvote = 0;  // units voted on so far (block-uniform)
  for (size_t unit = (blockIdx.x & 7) + 8 * (size_t)(blockIdx.x >> 5); unit < nunit; unit += ustride) {
    const int side = unit >= nblk * K;
    const size_t B = unit / K - side * nblk;
    const int kb = (int)(unit % K);
    const size_t g = 16 * B + hw;
    const bool ok = g < W;
    // the wave's two groups (past W: group 0); lane (r, h) reads bytes 16 h .. 16 h + 15 of both
    const size_t ge0 = 16 * B + 2 * wib < W ? 16 * B + 2 * wib : 0;
    const size_t ge1 = 16 * B + 2 * wib + 1 < W ? 16 * B + 2 * wib + 1 : 0;
    const uint32_t *sm8 = sd.smg[side];
    auto bytes_of = [&](size_t ge, int l) {
      return reinterpret_cast<const uint4 *>(sm8 + (((ge * L + l) * K + kb) * 32 + r) * 8) + h;
    };
    uint64_t *fk = sd.f_k[side];
    const int row = kb > 0 ? sd.row0[side] + kb - 1 : sd.row_p0[side];
    uint32_t wn[8];
    {
      const uint4 a = *bytes_of(ge0, L - 1), c = *bytes_of(ge1, L - 1);
      wn[0] = a.x, wn[1] = a.y, wn[2] = a.z, wn[3] = a.w, wn[4] = c.x, wn[5] = c.y, wn[6] = c.z, wn[7] = c.w;
    }
    asm volatile("" : "+v"(wn[0]), "+v"(wn[1]), "+v"(wn[2]), "+v"(wn[3]), "+v"(wn[4]), "+v"(wn[5]), "+v"(wn[6]),
                 "+v"(wn[7]));
    uint64_t acc[32];
    for (int l = L - 1; l >= 0; l--) {
      const size_t e = (size_t)kb * N + (ok ? g : 0) * L + l;
      uint64_t v[32];
      uint32_t nz = 0;
#pragma unroll
      for (int q = 0; q < 8; q++) nz |= wn[q];
      const bool live = __ballot((nz & 0x0F0F0F0Fu) != 0) != 0;  // both elements, every quarter's bit
      if (live) {
        uint64_t y0[16], y1[16];
        mx_stage1_q(zl, wn, r, h, y0);
        __builtin_amdgcn_sched_barrier(0);
        mx_stage1_q(zl, wn + 4, r, h, y1);
        midq_apply(midl, y0, y1, r, h);
        n32::halves_to_elements(y0, y1, v);  // lane (r, h): element h, all 32 rows j1
        n32::cyc_dif32<false>(v);  // v[i] = X[r + 32 brv5(i)]
      } else {
#pragma unroll
        for (int k = 0; k < 32; k++) v[k] = 0;
      }
      {  // the next limb's bytes (at l = 0 a harmless reload of limb L - 1)
        const int ln = l > 0 ? l - 1 : L - 1;
        const uint4 a = *bytes_of(ge0, ln), c = *bytes_of(ge1, ln);
        wn[0] = a.x, wn[1] = a.y, wn[2] = a.z, wn[3] = a.w, wn[4] = c.x, wn[5] = c.y, wn[6] = c.z, wn[7] = c.w;
      }
      if (fk) {
        uint64_t *of = (ok ? fk + e * D4 : sink) + m0 + 4 * r;
#pragma unroll
        for (int i = 0; i < 32; i++) of[128 * n32::brv5(i)] = v[i];
      }
      horner_step(acc, v, l == L - 1, lb, b_pow);
      if (row >= 0) {
        const size_t u = B * L + l;  // contraction unit of these 16 columns
        const int vs = nvote++ & 1;
        if (sd.dead && lane == 0) vote[vs][wib] = live ? 1u : 0u;
        __syncthreads();  // votes visible; every wave done reading the previous unit's staging
        bool any = true;
        if (sd.dead) {
          uint32_t a = 0;
#pragma unroll
          for (int q = 0; q < FQ_WAVES; q++) a |= vote[vs][q];
          any = a != 0;
          if (threadIdx.x == 0) sd.dead[u * 32 + row] = any ? 0 : 1;
        }
        if (!any) continue;  // block-uniform
        const int c = (int)(u >> 1), uh = (int)(u & 1);
#pragma unroll
        for (int hs = 0; hs < 2; hs++) {  // slots r + 32 brv5(i): i even -> < 512, i odd -> >= 512
          if (hs) __syncthreads();  // every wave done reading the first half
#pragma unroll
          for (int i = hs; i < 32; i += 2) S[(r + 32 * n32::brv5(i) - 512 * hs) * FM_SROW + hw] = fenc(v[i]);
          __syncthreads();
          const int m1 = threadIdx.x + 512 * hs;
          const uint64_t *src = S + threadIdx.x * FM_SROW;
          uint64_t x[16];
#pragma unroll
          for (int j = 0; j < 16; j++) x[j] = src[j];
          uint4 pu[8];
          d8_transpose16(x, pu);
          uint4 *out = frag + fv_index((size_t)m0 * Q4 + m1, nch, c, row, uh);
#pragma unroll
          for (int b = 0; b < 8; b++) out_store<NT>(&out[4 * b], pu[b]);
        }
      }
    }
    uint64_t *ow = (ok ? sd.w_ccs_k[side] + ((size_t)kb * W + g) * D4 : sink) + m0 + 4 * r;
#pragma unroll
    for (int i = 0; i < 32; i++) ow[128 * n32::brv5(i)] = gl::canon(acc[i]);
  }
}

// the packed bytes (k_pack_sm8's layout) -> the K digit planes in coefficient form:
// f_coeff_k[k][e][a + 1024 b] = digit k of that coefficient, one thread per output
__global__ void k_expand_sm8(const uint32_t *sm8, size_t N, int K, uint64_t *fck) {
  const uint8_t *by = reinterpret_cast<const uint8_t *>(sm8);
  for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < (size_t)K * N * D4;
       t += (size_t)gridDim.x * blockDim.x) {
    const int j = (int)(t % D4), kb = (int)(t / ((size_t)N * D4));
    const size_t e = (t / D4) % N;
    const int a = j & (Q4 - 1), b = j >> 10, r = a & 31, k = a >> 5;
    const uint32_t byte = by[((e * K + kb) * 32 + r) * 32 + k];
    const uint32_t bit = (byte >> b) & 1u, neg = (byte >> (4 + b)) & 1u;
    fck[t] = bit ? (neg ? gl::P - 1 : 1) : 0;
  }
}
hipError_t expand_sm8(const uint32_t *sm8, size_t N, int K, uint64_t *fck, hipStream_t st) {
  if (!N) return hipSuccess;
  if (K < 1 || K > 15) return hipErrorInvalidValue;
  const size_t n = (size_t)K * N * D4, nb = (n + 255) / 256;
  hipLaunchKernelGGL(k_expand_sm8, dim3((unsigned)(nb < 65536 ? nb : 65536)), dim3(256), 0, st, sm8, N, K, fck);
  return hipGetLastError();
}

// ---------------------------------------------------------------- Witness::from_f / from_w_ccs, d = 4096
// The inverse: x[a + 1024 b] = 1/4 sum_m0 w8^(-b (2 m0 + 1)) psi^(-(2 m0 - 3) a) INTT1024(X[m0 + 4 .])[a]
// (tools/ntt4096_model.py). A block of 8 waves holds four elements at a time,
// each on the four half-waves of two waves (one per quarter m0); after its
// quarter's INTT and twist (4^-1 folded into the table) a half-wave leaves
// z_m0 in LDS over its two waves' transpose tiles (E, 4 x 1024 words), and
// half-wave q then combines a in [256 q, 256 q + 256) for all four b:
// sum_m0 w8^(-b (2 m0 + 1)) z_m0 = w8^-b DFT4_{w4^-1}(z)_b, w4 = w8^2 = 2^48, all shifts.
// The forward direction of from_w_ccs runs the same exchange backwards.
namespace {
constexpr int FW_WAVES = 8;
// a quarter's slots in the transform's input order: v[m2] = p[128 m2] (all loads issued first)
__device__ __forceinline__ void load_quarter(const uint64_t *p, uint64_t *v) {
#pragma unroll
  for (int k = 0; k < 32; k++) v[k] = p[128 * k];
#pragma unroll
  for (int k = 0; k < 32; k += 8)
    asm volatile("" : "+v"(v[k]), "+v"(v[k + 1]), "+v"(v[k + 2]), "+v"(v[k + 3]), "+v"(v[k + 4]), "+v"(v[k + 5]),
                 "+v"(v[k + 6]), "+v"(v[k + 7]));
}
__device__ __forceinline__ void dft4_inv(uint64_t z0, uint64_t z1, uint64_t z2, uint64_t z3, uint64_t *x) {
  // X_b = sum_m z_m w^(bm), w = w4^-1 = 2^144 = -2^48; then x_b = w8^-b X_b (w8^-1 = 2^72)
  const uint64_t t0 = gl::add(z0, z2), t1 = gl::sub(z0, z2), t2 = gl::add(z1, z3);
  const uint64_t t3 = gl::shl96(gl::sub(z3, z1), 48);  // (z1 - z3) 2^144
  x[0] = gl::add(t0, t2);
  x[1] = gl::shl96(gl::add(t1, t3), 72);
  x[2] = gl::shl96(gl::sub(t2, t0), 48);  // (t0 - t2) 2^144
  x[3] = gl::shl96(gl::sub(t1, t3), 24);  // w8^-3 = 2^-360 = 2^24
}
__device__ __forceinline__ void dft4_fwd(uint64_t d0, uint64_t d1, uint64_t d2, uint64_t d3, uint64_t *z) {
  // z_m = sum_b d_b w8^(b (2m + 1)) = sum_b (w8^b d_b) w4^(bm), w8 = 2^120 = -2^24, w4 = 2^48
  const uint64_t e1 = gl::neg(gl::shl96(d1, 24)), e2 = gl::shl96(d2, 48), e3 = gl::shl96(d3, 72);  // 2^240 = 2^48, 2^360 = 2^168 = -2^72
  const uint64_t f3 = gl::neg(e3);
  const uint64_t t0 = gl::add(d0, e2), t1 = gl::sub(d0, e2), t2 = gl::add(e1, f3);
  const uint64_t t3 = gl::shl96(gl::sub(e1, f3), 48);  // (e1 - f3) w4
  z[0] = gl::add(t0, t2);
  z[1] = gl::add(t1, t3);
  z[2] = gl::sub(t0, t2);
  z[3] = gl::sub(t1, t3);
}
}  // namespace

// LF/arith.rs:299-313: f_coeff = ICRT(f), w_ccs = recompose(f) in slot form (Horner over the limbs)
__global__ void __launch_bounds__(512, 1) k_from_f_n4k(const uint64_t *f, size_t W, int lb, int L, uint64_t *f_coeff,
                                                      uint64_t *w_ccs, const uint64_t *mid_ig, const uint64_t *twi) {
  __shared__ uint64_t lds_all[FW_WAVES * n32::WAVE_U64];
  __shared__ uint64_t mid_i[n32::MID_U64];
  n32::stage_mid(mid_i, mid_ig);
  __syncthreads();
  const int lane = threadIdx.x & 63, wib = threadIdx.x >> 6;
  const int r = lane & 31, h = lane >> 5, G = wib >> 1, q = 2 * (wib & 1) + h;
  uint64_t *T = lds_all + wib * n32::WAVE_U64 + h * n32::HALF_U64;
  uint64_t *E = lds_all + 2 * G * n32::WAVE_U64;
  const uint64_t b_pow = gl::mul_pow2(1, lb);
  const uint64_t *tw = twi + q * Q4 + r;
  for (size_t g0 = (size_t)blockIdx.x * 4; g0 < W; g0 += (size_t)gridDim.x * 4) {
    const size_t g = g0 + G;
    const bool ok = g < W;
    const size_t gg = ok ? g : 0;
    uint64_t acc[32];
    for (int l = L - 1; l >= 0; l--) {
      const size_t e = gg * L + l;
      uint64_t v[32];
      load_quarter(f + e * D4 + q + 4 * r, v);  // v[m2] = X[q + 4 (r + 32 m2)]
      horner_step(acc, v, l == L - 1, lb, b_pow);
      n32::inverse(v, mid_i, T, r);
#pragma unroll
      for (int k0 = 0; k0 < 32; k0 += 8) {
        uint64_t t8[8];
#pragma unroll
        for (int k = 0; k < 8; k++) t8[k] = tw[32 * (k0 + k)];
#pragma unroll
        for (int k = 0; k < 8; k++) v[k0 + k] = gl::mul(v[k0 + k], t8[k]);
      }
      __syncthreads();  // the group's transposes are done: E may overwrite its tiles
#pragma unroll
      for (int k = 0; k < 32; k++) E[q * Q4 + r + 32 * k] = v[k];
      __syncthreads();
      uint64_t *oc = f_coeff + e * D4 + 256 * q + r;
#pragma unroll
      for (int i = 0; i < 8; i++) {
        const int a = 256 * q + r + 32 * i;
        uint64_t x[4];
        dft4_inv(E[a], E[Q4 + a], E[2 * Q4 + a], E[3 * Q4 + a], x);
        if (ok)
#pragma unroll
          for (int b = 0; b < 4; b++) oc[32 * i + b * Q4] = x[b];
      }
      __syncthreads();  // E read before the next transposes
    }
    if (ok) {
      uint64_t *ow = w_ccs + g * D4 + q + 4 * r;
#pragma unroll
      for (int k = 0; k < 32; k++) ow[128 * k] = gl::canon(acc[k]);
    }
  }
}

// LF/arith.rs:230-248: ICRT -> gadget_decompose(B = 2^lb, L) -> CRT, one element per four half-waves
__global__ void __launch_bounds__(512, 1) k_from_w_ccs_n4k(const uint64_t *w_ccs, size_t W, int lb, int L,
                                                          uint64_t *f_coeff, uint64_t *f, const uint64_t *mid_fg,
                                                          const uint64_t *mid_ig, const uint64_t *twf,
                                                          const uint64_t *twi, int *err) {
  __shared__ uint64_t lds_all[FW_WAVES * n32::WAVE_U64];
  __shared__ uint64_t mid_f[n32::MID_U64];
  n32::stage_mid(mid_f, mid_fg);
  __syncthreads();
  const int lane = threadIdx.x & 63, wib = threadIdx.x >> 6;
  const int r = lane & 31, h = lane >> 5, G = wib >> 1, q = 2 * (wib & 1) + h;
  uint64_t *T = lds_all + wib * n32::WAVE_U64 + h * n32::HALF_U64;
  uint64_t *E = lds_all + 2 * G * n32::WAVE_U64;
  for (size_t j0 = (size_t)blockIdx.x * 4; j0 < W; j0 += (size_t)gridDim.x * 4) {
    const size_t j = j0 + G;
    const bool ok = j < W;
    const size_t jj = ok ? j : 0;
    int64_t cur[32];  // coefficient a + 1024 b, a = 256 q + r + 32 i, at cur[4 i + b]
    {
      uint64_t v[32];
      load_quarter(w_ccs + jj * D4 + q + 4 * r, v);
      // the inverse middle factors from global (an L1-resident 8 KiB table), as k_from_w_ccs_n32 does
      n32::cyc_dif32<true>(v);
#pragma unroll
      for (int i0 = 0; i0 < 32; i0 += 8) {
        uint64_t t8[8];
#pragma unroll
        for (int i = 0; i < 8; i++) t8[i] = mid_ig[r * 32 + i0 + i];
#pragma unroll
        for (int i = 0; i < 8; i++) v[i0 + i] = gl::mul(v[i0 + i], t8[i]);
      }
      n32::transpose_inv(v, T, r);
      n32::neg_gs32_inv(v);
#pragma unroll
      for (int k0 = 0; k0 < 32; k0 += 8) {
        uint64_t t8[8];
#pragma unroll
        for (int k = 0; k < 8; k++) t8[k] = twi[q * Q4 + r + 32 * (k0 + k)];
#pragma unroll
        for (int k = 0; k < 8; k++) v[k0 + k] = gl::mul(v[k0 + k], t8[k]);
      }
      __syncthreads();
#pragma unroll
      for (int k = 0; k < 32; k++) E[q * Q4 + r + 32 * k] = v[k];
      __syncthreads();
#pragma unroll
      for (int i = 0; i < 8; i++) {
        const int a = 256 * q + r + 32 * i;
        uint64_t x[4];
        dft4_inv(E[a], E[Q4 + a], E[2 * Q4 + a], E[3 * Q4 + a], x);
#pragma unroll
        for (int b = 0; b < 4; b++) cur[4 * i + b] = signed_rep(x[b]);
      }
      __syncthreads();
    }
    for (int l = 0; l < L; l++) {
      const size_t e = jj * L + l;
      uint64_t *oc = f_coeff + e * D4 + 256 * q + r;
#pragma unroll
      for (int i = 0; i < 8; i++) {
        uint64_t dg[4], z[4];
#pragma unroll
        for (int b = 0; b < 4; b++) {
          dg[b] = from_signed(bal_digit(cur[4 * i + b], lb));
          if (ok) oc[32 * i + b * Q4] = dg[b];
        }
        dft4_fwd(dg[0], dg[1], dg[2], dg[3], z);
        const int a = 256 * q + r + 32 * i;
#pragma unroll
        for (int m = 0; m < 4; m++) E[m * Q4 + a] = z[m];
      }
      __syncthreads();
      uint64_t v[32];
#pragma unroll
      for (int k0 = 0; k0 < 32; k0 += 8) {
        uint64_t t8[8];
#pragma unroll
        for (int k = 0; k < 8; k++) t8[k] = twf[q * Q4 + r + 32 * (k0 + k)];
#pragma unroll
        for (int k = 0; k < 8; k++) v[k0 + k] = gl::mul(E[q * Q4 + r + 32 * (k0 + k)], t8[k]);
      }
      __syncthreads();  // E read before the transposes overwrite it
      n32::forward(v, mid_f, T, r);
      if (ok) {
        uint64_t *of = f + e * D4 + q + 4 * r;
#pragma unroll
        for (int i = 0; i < 32; i++) of[128 * n32::brv5(i)] = v[i];
      }
      __syncthreads();  // transposes done before the next limb's E writes
    }
    bool bad = false;
#pragma unroll
    for (int k = 0; k < 32; k++) bad |= cur[k] != 0;
    if (ok && bad) raise(err, 1);
  }
}

// grids: one block per 4 elements, capped (the kernels loop)
constexpr size_t FW_GRID_CAP = 4096;
hipError_t from_f_n4k(const uint64_t *f, size_t W, int lb, int L, uint64_t *f_coeff, uint64_t *w_ccs,
                      const ring::NegaTables &inv, hipStream_t st) {
  if (!inv.mid || !inv.tw4) return hipErrorInvalidValue;
  if (!W) return hipSuccess;
  const size_t nb = (W + 3) / 4;
  hipLaunchKernelGGL(k_from_f_n4k, dim3((unsigned)(nb < FW_GRID_CAP ? nb : FW_GRID_CAP)), dim3(512), 0, st,
                     f, W, lb, L, f_coeff, w_ccs, inv.mid, inv.tw4);
  return hipGetLastError();
}
hipError_t from_w_ccs_n4k(const uint64_t *w_ccs, size_t W, int lb, int L, uint64_t *f_coeff, uint64_t *f,
                          const ring::NegaTables &fwd, const ring::NegaTables &inv, int *err, hipStream_t st) {
  if (!fwd.mid || !fwd.tw4 || !inv.mid || !inv.tw4) return hipErrorInvalidValue;
  if (!W) return hipSuccess;
  const size_t nb = (W + 3) / 4;
  hipLaunchKernelGGL(k_from_w_ccs_n4k, dim3((unsigned)(nb < FW_GRID_CAP ? nb : FW_GRID_CAP)), dim3(512), 0,
                     st, w_ccs, W, lb, L, f_coeff, f, fwd.mid, inv.mid, fwd.tw4, inv.tw4, err);
  return hipGetLastError();
}

hipError_t decompose_n4k(const FusedSides &sd, size_t N, int lb, int L, int K, uint64_t *sm4,
                         const ring::NegaTables &fwd, int *err, uint64_t *sink, int ncu, hipStream_t st, uint4 *frag,
                         int nch) {
  if (K > 15 || !fwd.mid || !fwd.tw4 || !fwd.ztab || !sink || ncu < 1 || sd.nside < 1 || sd.nside > 2 || N % L)
    return hipErrorInvalidValue;
  if (N == 0) return hipSuccess;
  if (frag) {
    FusedSides s8 = sd;
    bool refold = false;
    for (int s = 0; s < sd.nside; s++) {
      if (sd.row0[s] < 0 || sd.row0[s] + K - 1 > 32 || sd.row_p0[s] > 32) return hipErrorInvalidValue;
      // the packed bytes (N K 256 words per side): the caller's planes, else the scratch
      if (!s8.smg[s]) s8.smg[s] = reinterpret_cast<uint32_t *>(sm4) + (size_t)s * N * K * 256;
      refold |= sd.f_k[s] != nullptr;
    }
    if (ncu < 32) return hipErrorInvalidValue;
    const size_t threads = sd.nside * N * 256;
    hipLaunchKernelGGL(k_pack_sm8, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, st, s8, N, K, err);
    // 32 blocks per group of 8 units (8 XCDs x 4 quarters), one block per CU
    const unsigned grid = (unsigned)(ncu / 32 * 32);
    // outputs: f_coeff_k, f_k, the operand rows (each K N d words per side) and w_ccs_k
    const bool nt = dec_streaming(sd.nside * (size_t)K * N * D4 * 8 * 3, refold);
    // stage 1 on the matrix cores when no f_coeff_k rows are wanted (the packed steps);
    // LATTICEUM_AMD_N4K=valu keeps the VALU form (A/B runs)
    static const bool valu = [] {
      const char *e = getenv("LATTICEUM_AMD_N4K");
      return e && !strcmp(e, "valu");
    }();
    bool mx = fwd.zq && fwd.midq && !valu;
    for (int s = 0; s < sd.nside; s++) mx = mx && !sd.f_coeff_k[s];
    if (mx) {
      if (nt)
        hipLaunchKernelGGL(k_decompose_n4k_mx<true>, dim3(grid), dim3(512), 0, st, N, L, lb, K, s8, fwd.midq,
                           fwd.zq, frag, nch, sink);
      else
        hipLaunchKernelGGL(k_decompose_n4k_mx<false>, dim3(grid), dim3(512), 0, st, N, L, lb, K, s8, fwd.midq,
                           fwd.zq, frag, nch, sink);
    } else if (nt) {
      hipLaunchKernelGGL(k_decompose_n4k_fused<true>, dim3(grid), dim3(512), 0, st, N, L, lb, K, s8, fwd.mid,
                         fwd.tw4, fwd.ztab, frag, nch, sink);
    } else {
      hipLaunchKernelGGL(k_decompose_n4k_fused<false>, dim3(grid), dim3(512), 0, st, N, L, lb, K, s8, fwd.mid,
                         fwd.tw4, fwd.ztab, frag, nch, sink);
    }
    return hipGetLastError();
  }
  const size_t words = sd.nside * N * Q4;
  hipLaunchKernelGGL(k_pack_sm4, dim3((unsigned)((words + 255) / 256)), dim3(256), 0, st, sd, N, K, sm4, err);
  const size_t npair = (sd.nside * (N / L) * K + 1) / 2;
  // one block per CU, each taking the same number of work-item pairs
  const size_t per = (npair + 2 * ncu - 1) / (2 * ncu);
  const unsigned grid = (unsigned)((npair + 2 * per - 1) / (2 * per));
  hipLaunchKernelGGL(k_decompose_n4k, dim3(grid), dim3(64 * WPB4), 0, st, sm4, N, L, lb, K, sd, fwd.mid, fwd.tw4,
                     fwd.ztab, sink);
  return hipGetLastError();
}

}  // namespace lfk
