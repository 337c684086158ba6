// kernels_n32.hip -- the X^1024 + 1 ring on the register-resident 32 x 32 NTT
// (ntt32.hpp). Half a wave owns one ring element (transforms, from_w_ccs) or
// one group of L elements (decompose, from_f); waves never synchronise with
// each other and there is no s_barrier on this path. Every global access is a
// 256-B row per half-wave (lane r touches x[r + 32 k]).
#include "digits.hpp"
#include "frag.hpp"
#include "kernels.hpp"
#include "ntt32.hpp"

namespace lfk {

namespace {
constexpr int WPB = 4;  // waves per block
constexpr int D = 1024;

struct Half {
  int r, h;        // lane & 31, half of the wave
  size_t unit;     // this half's work unit (ring element or group)
  size_t stride;   // units per grid-stride step
  uint64_t *lds;   // this half's transpose tile
};
template <int NW = WPB>
__device__ __forceinline__ Half half_ctx(uint64_t *lds_all) {
  Half x;
  const int lane = threadIdx.x & 63, wib = threadIdx.x >> 6;
  x.r = lane & 31;
  x.h = lane >> 5;
  x.unit = ((size_t)blockIdx.x * NW + wib) * 2 + x.h;
  x.stride = (size_t)gridDim.x * NW * 2;
  x.lds = lds_all + wib * n32::WAVE_U64 + x.h * n32::HALF_U64;
  return x;
}
using n32::load_row32;
// the loop bound every lane of a wave agrees on (both halves iterate together)
__device__ __forceinline__ size_t pair_bound(size_t n) { return (n + 1) & ~(size_t)1; }
}  // namespace

// ---------------------------------------------------------------- transforms
// dst = transform(src) (src == dst: in place)
template <bool FWD>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) k_xform_n32(const uint64_t *src, uint64_t *data, size_t n,
                                                  const uint64_t *mid_g) {
  // 32-bit transpose tiles (42 KB of LDS per block instead of 76) and no prefetch of
  // the next element's rows (152-165 VGPRs instead of 216-229): three waves per SIMD
  // instead of two
  __shared__ uint32_t lds_w[WPB * 2 * n32::HALF_U32];
  __shared__ uint64_t mid[n32::MID_U64];
  n32::stage_mid(mid, mid_g);
  __syncthreads();
  Half x = half_ctx(nullptr);
  uint32_t *tile = lds_w + ((threadIdx.x >> 6) * 2 + x.h) * n32::HALF_U32;
  for (size_t e = x.unit; e < pair_bound(n); e += x.stride) {
    const bool ok = e < n;
    uint64_t *g = data + (ok ? e : 0) * D + x.r;
    uint64_t v[32];
    load_row32(src + (ok ? e : 0) * D + x.r, v);
    if (FWD)
      n32::forward_w(v, mid, tile, x.r);
    else
      n32::inverse_w(v, mid, tile, x.r);
    if (ok) {
      if (FWD) {
#pragma unroll
        for (int i = 0; i < 32; i++) g[32 * n32::brv5(i)] = v[i];
      } else {
#pragma unroll
        for (int k = 0; k < 32; k++) g[32 * k] = v[k];
      }
    }
  }
}

// the inverse transform with the inverse middle factors read from global (an
// L1-resident 8 KiB table) instead of LDS: slot input -> coefficient layout
__device__ __forceinline__ void inverse_gmid(uint64_t *v, const uint64_t *mid_ig, uint64_t *lds, int r) {
  n32::cyc_dif32<true>(v);
#pragma unroll
  for (int i = 0; i < 32; i++) v[i] = gl::mul(v[i], mid_ig[r * 32 + i]);
  n32::transpose_inv(v, lds, r);
  n32::neg_gs32_inv(v);
}

// ---------------------------------------------------------------- Witness::from_w_ccs
// LF/arith.rs:230-248: ICRT -> gadget_decompose(B = 2^lb, L) -> CRT; one half-wave per element.
// The inverse middle factors read from global (L1-resident 8 KiB table),
// no next-element prefetch, so two blocks (8 waves) fit a CU: 0.71 -> 0.52 ms at
// W = 16 384 against the LDS-table, prefetching form (one block per CU)
// the fused decomposition's packed words of one limb row (k_pack_sm's layout:
// word (q, r) = sm(x[r + 64 q]) | sm(x[r + 64 q + 32]) << 16, sm = 15-bit magnitude |
// sign << 15) straight from the digits this lane holds (x[r + 32 k] = d[k])
__device__ __forceinline__ uint32_t sm16(int64_t d) {
  return (uint32_t)(d < 0 ? -d : d) | (d < 0 ? 0x8000u : 0u);
}
// (from the field elements, so no digit array stays live beside the transform's registers)
__device__ __forceinline__ void store_sm_row(const uint64_t *v, uint32_t *row, int r) {
#pragma unroll
  for (int q = 0; q < 16; q++)
    row[q * 32 + r] = sm16(signed_rep(v[2 * q])) | (sm16(signed_rep(v[2 * q + 1])) << 16);
}
// smg (may be null): the digits' packed words too (from_w_ccs's comment in kernels.hpp)
__global__ void __launch_bounds__(256, 2) k_from_w_ccs_n32(const uint64_t *w_ccs, size_t W, int lb, int L,
                                                          uint64_t *f_coeff, uint64_t *f, const uint64_t *mid_fg,
                                                          const uint64_t *mid_ig, int *err, uint32_t *smg) {
  __shared__ uint64_t lds_all[WPB * n32::WAVE_U64];
  __shared__ uint64_t mid_f[n32::MID_U64];
  n32::stage_mid(mid_f, mid_fg);
  __syncthreads();
  Half x = half_ctx(lds_all);
  for (size_t j = x.unit; j < pair_bound(W); j += x.stride) {
    const bool ok = j < W;
    uint64_t v[32];
    {
      const uint64_t *g = w_ccs + (ok ? j : 0) * D + x.r;
#pragma unroll
      for (int k = 0; k < 32; k++) v[k] = g[32 * k];
    }
    inverse_gmid(v, mid_ig, x.lds, x.r);
    int64_t cur[32];
#pragma unroll
    for (int k = 0; k < 32; k++) cur[k] = signed_rep(v[k]);
    for (int l = 0; l < L; l++) {
      uint64_t *oc = f_coeff + ((ok ? j : 0) * L + l) * D + x.r;
#pragma unroll
      for (int k = 0; k < 32; k++) {
        v[k] = from_signed(bal_digit(cur[k], lb));
        if (ok) oc[32 * k] = v[k];
      }
      if (smg && ok) store_sm_row(v, smg + (j * L + l) * 512, x.r);
      n32::forward(v, mid_f, x.lds, x.r);
      if (ok) {
        uint64_t *of = f + (j * L + l) * D + x.r;
#pragma unroll
        for (int i = 0; i < 32; i++) of[32 * n32::brv5(i)] = v[i];
      }
    }
    bool bad = false;
#pragma unroll
    for (int k = 0; k < 32; k++) bad |= cur[k] != 0;
    if (ok && bad) raise(err, 1);
  }
}

// ---------------------------------------------------------------- Witness::from_f
// LF/arith.rs:299-313: f_coeff = ICRT(f), w_ccs = recompose(f) in slot form; one half-wave per group
__global__ void __launch_bounds__(256) k_from_f_n32(const uint64_t *f, size_t W, int lb, int L,
                                                   uint64_t *f_coeff, uint64_t *w_ccs, const uint64_t *mid_ig,
                                                   const int *run_if) {
  if (run_if && !*run_if) return;  // uniform: the coefficient-form fold produced f_coeff
  __shared__ uint64_t lds_all[WPB * n32::WAVE_U64];
  __shared__ uint64_t mid_i[n32::MID_U64];
  n32::stage_mid(mid_i, mid_ig);
  __syncthreads();
  Half x = half_ctx(lds_all);
  const uint64_t b_pow = gl::mul_pow2(1, lb);  // B = 2^lb
  for (size_t g = x.unit; g < pair_bound(W); g += x.stride) {
    const bool ok = g < W;
    const size_t gg = ok ? g : 0;
    uint64_t acc[32], nx[32];
    {
      const uint64_t *src = f + (gg * L + L - 1) * D + x.r;
#pragma unroll
      for (int k = 0; k < 32; k++) nx[k] = src[32 * k];
    }
    for (int l = L - 1; l >= 0; l--) {
      uint64_t v[32];
#pragma unroll
      for (int k = 0; k < 32; k++) {
        v[k] = nx[k];
        acc[k] = (l == L - 1) ? v[k] : gl::add(gl::mul(acc[k], b_pow), v[k]);
      }
      n32::inverse(v, mid_i, x.lds, x.r);
      if (l > 0) {  // next limb's loads ahead of this limb's stores
        const uint64_t *src = f + (gg * L + l - 1) * D + x.r;
#pragma unroll
        for (int k = 0; k < 32; k++) nx[k] = src[32 * k];
      }
      if (ok) {
        uint64_t *oc = f_coeff + (g * L + l) * D + x.r;
#pragma unroll
        for (int k = 0; k < 32; k++) oc[32 * k] = v[k];
      }
    }
    if (ok) {
      uint64_t *ow = w_ccs + g * D + x.r;
#pragma unroll
      for (int k = 0; k < 32; k++) ow[32 * k] = acc[k];
    }
  }
}

// Witness::from_f when f_0 was folded in coefficient form (fold_coeff.hip): the
// coefficients are the input, f = NTT(f_coeff) and w_ccs = recompose(f) in slot
// form; one half-wave per group. gate: nothing to do when *gate != 0 (rho was
// not short, the NTT-form fold and from_f ran instead)
// gate set and mid_ig given: Witness::from_f of f instead (f_coeff = ICRT(f),
// w_ccs = recompose(f) in slot form), the NTT-form fold's fallback
__device__ __forceinline__ void from_f_group(const uint64_t *f, size_t g, bool ok, int lb, int L, uint64_t *f_coeff,
                                             uint64_t *w_ccs, const uint64_t *mid_ig, uint64_t *lds, int r) {
  const uint64_t b_pow = gl::mul_pow2(1, lb);
  const size_t gg = ok ? g : 0;
  uint64_t acc[32];
  for (int l = L - 1; l >= 0; l--) {
    uint64_t v[32];
    load_row32(f + (gg * L + l) * D + r, v);
#pragma unroll
    for (int k = 0; k < 32; k++) acc[k] = (l == L - 1) ? v[k] : gl::add(gl::mul(acc[k], b_pow), v[k]);
    inverse_gmid(v, mid_ig, lds, r);
    if (ok) {
      uint64_t *oc = f_coeff + (g * L + l) * D + r;
#pragma unroll
      for (int k = 0; k < 32; k++) oc[32 * k] = v[k];
    }
  }
  if (ok) {
    uint64_t *ow = w_ccs + g * D + r;
#pragma unroll
    for (int k = 0; k < 32; k++) ow[32 * k] = acc[k];
  }
}
__global__ void __launch_bounds__(256, 2) k_from_fcoeff_n32(uint64_t *f_coeff, size_t W, int lb, int L,
                                                        uint64_t *f, uint64_t *w_ccs, const uint64_t *mid_fg,
                                                        const int *gate, const uint64_t *mid_ig) {
  if (gate && *gate && !mid_ig) return;
  __shared__ uint64_t lds_all[WPB * n32::WAVE_U64];
  __shared__ uint64_t mid_f[n32::MID_U64];
  if (gate && *gate) {  // uniform over the grid
    Half x = half_ctx(lds_all);
    for (size_t g = x.unit; g < pair_bound(W); g += x.stride)
      from_f_group(f, g, g < W, lb, L, f_coeff, w_ccs, mid_ig, x.lds, x.r);
    return;
  }
  n32::stage_mid(mid_f, mid_fg);
  __syncthreads();
  Half x = half_ctx(lds_all);
  const uint64_t b_pow = gl::mul_pow2(1, lb);  // B = 2^lb
  for (size_t g = x.unit; g < pair_bound(W); g += x.stride) {
    const bool ok = g < W;
    const size_t gg = ok ? g : 0;
    uint64_t acc[32];
    for (int l = L - 1; l >= 0; l--) {
      uint64_t v[32];
      load_row32(f_coeff + (gg * L + l) * D + x.r, v);
      n32::forward(v, mid_f, x.lds, x.r);  // v[i] = X[r + 32 brv5(i)]
      if (l == L - 1) {
#pragma unroll
        for (int i = 0; i < 32; i++) acc[i] = v[i];
      } else if (lb == 15) {  // GoldiLocksDP B = 2^15: a shift instead of a product
#pragma unroll
        for (int i = 0; i < 32; i++) acc[i] = gl::add_weak(gl::shl_small_weak(acc[i], 15), v[i]);
      } else {
#pragma unroll
        for (int i = 0; i < 32; i++) acc[i] = gl::add(gl::mul(acc[i], b_pow), v[i]);
      }
      if (ok) {
        uint64_t *of = f + (g * L + l) * D + x.r;
#pragma unroll
        for (int i = 0; i < 32; i++) of[32 * n32::brv5(i)] = v[i];
      }
    }
    if (ok) {
      uint64_t *ow = w_ccs + g * D + x.r;
#pragma unroll
      for (int i = 0; i < 32; i++) ow[32 * n32::brv5(i)] = gl::canon(acc[i]);
    }
  }
}

// ---------------------------------------------------------------- small-W variants
// When W half-waves cannot fill the chip, from_w_ccs and from_f run one
// half-wave per (element, limb): W L units. Both halves of a wave take the same
// limb of two adjacent elements (unit pair p: limb p % L, elements 2 (p / L) + h).
constexpr int SPLIT_WPB = 8;  // 8 waves: the LDS of one block per CU (T tiles + tables) either way
__device__ __forceinline__ void split_unit(size_t u, int L, size_t &j, int &l) {
  const size_t p = u >> 1;
  l = (int)(p % L);
  j = 2 * (p / L) + (u & 1);
}
// from_w_ccs at small W in two launches: this one inverts each element once (one
// half-wave per element, the inverse middle factors from global) and writes its
// L digit rows (f_coeff, coefficient layout); then a forward transform per
// (element, limb) row, f = NTT(f_coeff) (k_xform_n32, out of place). Against one
// launch of (element, limb) units that each redid their element's inverse
// transform: W + W L transforms instead of 2 W L, in two short latency chains
__global__ void __launch_bounds__(256) k_from_w_ccs_digits(const uint64_t *w_ccs, size_t W, int lb, int L,
                                                          uint64_t *f_coeff, const uint64_t *mid_ig, int *err,
                                                          uint32_t *smg) {
  __shared__ uint64_t lds_all[WPB * n32::WAVE_U64];
  Half x = half_ctx(lds_all);
  for (size_t j = x.unit; j < pair_bound(W); j += x.stride) {
    const bool ok = j < W;
    uint64_t v[32];
    load_row32(w_ccs + (ok ? j : 0) * D + x.r, v);
    inverse_gmid(v, mid_ig, x.lds, x.r);
    int64_t cur[32];
#pragma unroll
    for (int k = 0; k < 32; k++) cur[k] = signed_rep(v[k]);
    for (int l = 0; l < L; l++) {
      uint64_t *oc = f_coeff + ((ok ? j : 0) * L + l) * D + x.r;
      uint64_t dv[32];
#pragma unroll
      for (int k = 0; k < 32; k++) {
        dv[k] = from_signed(bal_digit(cur[k], lb));
        if (ok) oc[32 * k] = dv[k];
      }
      if (smg && ok) store_sm_row(dv, smg + (j * L + l) * 512, x.r);
    }
    bool bad = false;
#pragma unroll
    for (int k = 0; k < 32; k++) bad |= cur[k] != 0;
    if (ok && bad) raise(err, 1);
  }
}
// from_f: each unit inverts its own element; the limb-0 units also recompose
// w_ccs = sum_l B^l f[jL + l] in slot form (Horner from the top limb)
__global__ void __launch_bounds__(512) k_from_f_split(const uint64_t *f, size_t W, int lb, int L,
                                                     uint64_t *f_coeff, uint64_t *w_ccs, const uint64_t *mid_ig,
                                                     const int *run_if) {
  if (run_if && !*run_if) return;  // uniform: the coefficient-form fold produced f_coeff
  __shared__ uint64_t lds_all[SPLIT_WPB * n32::WAVE_U64];
  __shared__ uint64_t mid_i[n32::MID_U64];
  n32::stage_mid(mid_i, mid_ig);
  __syncthreads();
  Half x = half_ctx<SPLIT_WPB>(lds_all);
  const uint64_t b_pow = gl::mul_pow2(1, lb);  // B = 2^lb
  const size_t units = ((W + 1) & ~(size_t)1) * L;
  for (size_t u = x.unit; u < units; u += x.stride) {
    size_t j;
    int l;
    split_unit(u, L, j, l);
    const bool ok = j < W;
    if (!ok) j = 0;
    const size_t e = j * L + l;
    uint64_t v[32];
    load_row32(f + e * D + x.r, v);
    if (l == 0) {  // wave-uniform: both halves hold limb 0
      uint64_t acc[32];
      load_row32(f + (j * L + L - 1) * D + x.r, acc);
      for (int l2 = L - 2; l2 >= 0; l2--) {
        uint64_t t[32];
        if (l2 > 0)
          load_row32(f + (j * L + l2) * D + x.r, t);
        else
#pragma unroll
          for (int k = 0; k < 32; k++) t[k] = v[k];
#pragma unroll
        for (int k = 0; k < 32; k++) acc[k] = gl::add(gl::mul(acc[k], b_pow), t[k]);
      }
      if (ok) {
        uint64_t *ow = w_ccs + j * D + x.r;
#pragma unroll
        for (int k = 0; k < 32; k++) ow[32 * k] = acc[k];
      }
    }
    n32::inverse(v, mid_i, x.lds, x.r);
    if (ok) {
      uint64_t *oc = f_coeff + e * D + x.r;
#pragma unroll
      for (int k = 0; k < 32; k++) oc[32 * k] = v[k];
    }
  }
}

// from f's coefficients (the coefficient-form fold's output) at small W: one
// half-wave per (group, part), part p < L the forward transform of limb p, part
// L the group's w_ccs = NTT(sum_l B^l f_coeff[jL + l]) -- the recomposition in
// coefficient form, which by linearity equals k_from_fcoeff_n32's slot-form
// Horner over the L transforms -- so a group is L + 1 independent transforms
// instead of L in series on one half-wave
__global__ void __launch_bounds__(512) k_from_fcoeff_split(uint64_t *f_coeff, size_t W, int lb, int L,
                                                          uint64_t *f, uint64_t *w_ccs, const uint64_t *mid_fg,
                                                          const int *gate, const uint64_t *mid_ig) {
  if (gate && *gate && !mid_ig) return;
  __shared__ uint64_t lds_all[SPLIT_WPB * n32::WAVE_U64];
  __shared__ uint64_t mid_f[n32::MID_U64];
  const bool fb = gate && *gate;  // uniform: Witness::from_f of f (the NTT-form fold's fallback)
  if (!fb) n32::stage_mid(mid_f, mid_fg);
  __syncthreads();
  Half x = half_ctx<SPLIT_WPB>(lds_all);
  const uint64_t b_pow = gl::mul_pow2(1, lb);  // B = 2^lb
  const size_t units = ((W + 1) & ~(size_t)1) * (L + 1);
  for (size_t u = x.unit; u < units; u += x.stride) {
    // both halves of a wave take the same part of two adjacent groups
    const size_t q = u >> 1;
    const int p = (int)(q % (L + 1));
    size_t j = 2 * (q / (L + 1)) + (u & 1);
    const bool ok = j < W;
    if (!ok) j = 0;
    uint64_t v[32];
    if (fb) {  // part p < L: f_coeff = ICRT(f) of limb p; part L: w_ccs = recompose(f) in slot form
      if (p < L) {
        load_row32(f + (j * L + p) * D + x.r, v);
        inverse_gmid(v, mid_ig, x.lds, x.r);
        if (ok) {
          uint64_t *oc = f_coeff + (j * L + p) * D + x.r;
#pragma unroll
          for (int k = 0; k < 32; k++) oc[32 * k] = v[k];
        }
      } else {
        load_row32(f + (j * L + L - 1) * D + x.r, v);
        for (int l = L - 2; l >= 0; l--) {
          uint64_t t[32];
          load_row32(f + (j * L + l) * D + x.r, t);
#pragma unroll
          for (int k = 0; k < 32; k++) v[k] = gl::add(gl::mul(v[k], b_pow), t[k]);
        }
        if (ok) {
          uint64_t *ow = w_ccs + j * D + x.r;
#pragma unroll
          for (int k = 0; k < 32; k++) ow[32 * k] = v[k];
        }
      }
      continue;
    }
    if (p < L) {
      load_row32(f_coeff + (j * L + p) * D + x.r, v);
    } else {
      load_row32(f_coeff + (j * L + L - 1) * D + x.r, v);
      for (int l = L - 2; l >= 0; l--) {
        uint64_t t[32];
        load_row32(f_coeff + (j * L + l) * D + x.r, t);
        if (lb == 15) {  // GoldiLocksDP B = 2^15: a shift instead of a product
#pragma unroll
          for (int k = 0; k < 32; k++) v[k] = gl::add_weak(gl::shl_small_weak(v[k], 15), t[k]);
        } else {
#pragma unroll
          for (int k = 0; k < 32; k++) v[k] = gl::add(gl::mul(v[k], b_pow), t[k]);
        }
      }
#pragma unroll
      for (int k = 0; k < 32; k++) v[k] = gl::canon(v[k]);
    }
    n32::forward(v, mid_f, x.lds, x.r);
    if (ok) {
      uint64_t *of = (p < L ? f + (j * L + p) * D : w_ccs + j * D) + x.r;
#pragma unroll
      for (int i = 0; i < 32; i++) of[32 * n32::brv5(i)] = v[i];
    }
  }
}

// ---------------------------------------------------------------- decompose_witness
// LF/nifs/decomposition.rs:162-167, decomposition/utils.rs:45-49, arith.rs:324-338,
// specialised to b_small = 2 (GoldiLocksDP): the balanced base-2 digits of v are
// sign(v) * bit_k(|v|) (|rem| <= b/2 always, so no carries), so each digit plane
// is read straight off |v| kept as 16-bit sign|magnitude (K <= 15; |v| < 2^K is
// checked -- the reference panics otherwise). One half-wave per group of L
// elements; the first two NTT levels of a digit plane run exactly in int64
// (n32::neg_ct32_digits), and w_ccs_k = sum_l B^l f_k[gL + l] is accumulated in
// slot form as the planes are produced.
template <int L>
__global__ void __launch_bounds__(256, 1) k_decompose_n32(const uint64_t *f_coeff, size_t N, int lb, int K,
                                                         uint64_t *f_coeff_k, uint64_t *f_k, uint64_t *w_ccs_k,
                                                         const uint64_t *mid_fg, int *err) {
  __shared__ uint64_t lds_all[WPB * n32::WAVE_U64];
  __shared__ uint64_t mid_f[n32::MID_U64];
  // the group's coefficients as 16-bit sign|magnitude, two per word:
  // sm[wave][l][q][lane] = x[r + 32 (2q)] | x[r + 32 (2q + 1)] << 16 of limb l
  // (kept in LDS: in registers they crowd out the NTT's temporaries)
  __shared__ uint32_t sm_all[WPB][L][16][64];
  n32::stage_mid(mid_f, mid_fg);
  __syncthreads();
  Half x = half_ctx(lds_all);
  const int lane = threadIdx.x & 63;
  uint32_t (*sm)[16][64] = sm_all[threadIdx.x >> 6];
  const size_t W = N / L;
  const uint64_t b_pow = gl::mul_pow2(1, lb);  // B = 2^lb
  for (size_t g = x.unit; g < pair_bound(W); g += x.stride) {
    const bool ok = g < W;
    const size_t gg = ok ? g : 0;
    bool bad = false;
    for (int l = 0; l < L; l++) {
      uint64_t raw[32];
      load_row32(f_coeff + (gg * L + l) * D + x.r, raw);
#pragma unroll
      for (int k = 0; k < 32; k += 2) {
        const int64_t a = signed_rep(raw[k]), c = signed_rep(raw[k + 1]);
        const uint64_t ma = a < 0 ? (uint64_t)(-a) : (uint64_t)a, mc = c < 0 ? (uint64_t)(-c) : (uint64_t)c;
        bad |= (ma >> K) != 0 || (mc >> K) != 0;
        const uint32_t ea = (uint32_t)(ma & 0x7FFF) | (a < 0 ? 0x8000u : 0u);
        const uint32_t ec = (uint32_t)(mc & 0x7FFF) | (c < 0 ? 0x8000u : 0u);
        sm[l][k >> 1][lane] = ea | (ec << 16);
      }
    }
    if (ok && bad) raise(err, 1);
    for (int kb = 0; kb < K; kb++) {
      uint64_t acc[32];
#pragma unroll
      for (int i = 0; i < 32; i++) acc[i] = 0;  // Horner from 0: no per-limb branch
#pragma unroll 1
      for (int l = L - 1; l >= 0; l--) {
        const size_t e = (size_t)kb * N + gg * L + l;
        int32_t dg[32];
#pragma unroll
        for (int q = 0; q < 16; q++) {
          const uint32_t w = sm[l][q][lane];
#pragma unroll
          for (int t = 0; t < 2; t++) {
            const uint32_t hw = w >> (16 * t);
            const int32_t bit = (hw >> kb) & 1;
            dg[2 * q + t] = (hw & 0x8000) ? -bit : bit;
          }
        }
        if (ok) {
          uint64_t *oc = f_coeff_k + e * D + x.r;
#pragma unroll
          for (int k = 0; k < 32; k++) oc[32 * k] = from_signed(dg[k]);
        }
        uint64_t v[32];
        n32::neg_ct32_digits(dg, v);
        n32::forward<false>(v, mid_f, x.lds, x.r);
        if (ok) {
          uint64_t *of = f_k + e * D + x.r;
#pragma unroll
          for (int i = 0; i < 32; i++) of[32 * n32::brv5(i)] = v[i];
        }
        if (lb == 15) {  // GoldiLocksDP B = 2^15: a shift instead of a product
#pragma unroll
          for (int i = 0; i < 32; i++) acc[i] = gl::add_weak(gl::shl_small_weak(acc[i], 15), v[i]);
        } else {
#pragma unroll
          for (int i = 0; i < 32; i++) acc[i] = gl::add(gl::mul(acc[i], b_pow), v[i]);
        }
      }
      if (ok) {
        uint64_t *ow = w_ccs_k + ((size_t)kb * W + g) * D + x.r;
#pragma unroll
        for (int i = 0; i < 32; i++) ow[32 * n32::brv5(i)] = gl::canon(acc[i]);
      }
    }
  }
}

// ---------------------------------------------------------------- fused decomposition + Ajtai operands
// The same decomposition, organised for the i8-MFMA commitment: a block of 8
// waves owns 16 consecutive groups (one per half-wave), so for each digit
// plane k >= 1 and limb l the block holds one 16-column unit of the Ajtai
// contraction order (ajtai_mfma.hip, Lp = L) and writes it straight into the
// vector-major operand buffer -- the planes never make a second trip through
// HBM to be re-laid out. Per (k, l): NTT (stage 1 on the matrix cores, its
// transpose a half exchange in registers), then the D8 words of the 16 outputs
// go through a slot-major staging tile S (two barriers per unit: the first also
// orders the previous unit's reads before the new writes), and each thread
// emits two slots' 128-byte operand pieces.
//
// The group's coefficients come pre-packed as 16-bit sign|magnitude
// (k_pack_sm: smg[(col 16 + q) 32 + r] = x[r + 32(2q)] | x[r + 32(2q+1)] << 16),
// read back per (k, l), one plane ahead.
constexpr int FD_WAVES = 8;
constexpr int FD_SROW = 17;  // staging row stride in u64 (16 columns + pad: conflict-free)
constexpr int FD_S_U64 = D * FD_SROW;

// four packed words per thread (t0 = 4 * thread): 2 x 32 contiguous bytes in,
// one 16-B store out
__device__ __forceinline__ uint32_t pack_sm1(uint64_t x, int K, bool &bad) {
  const int64_t a = signed_rep(x);
  const uint64_t m = a < 0 ? (uint64_t)(-a) : (uint64_t)a;
  bad |= (m >> K) != 0;
  return (uint32_t)(m & 0x7FFF) | (a < 0 ? 0x8000u : 0u);
}
__global__ void k_pack_sm(FusedSides sd, size_t N, int K, int *err) {
  const size_t t0 = 4 * (blockIdx.x * (size_t)blockDim.x + threadIdx.x);  // (side, col, q, r..r+3)
  if (t0 >= sd.nside * N * 512) return;
  const int side = t0 >= N * 512;
  const uint64_t *f_coeff = sd.f_coeff[side];
  const size_t col = (t0 >> 9) - side * N;
  const int q = (t0 >> 5) & 15, r = t0 & 31;
  const ulonglong2 *x = reinterpret_cast<const ulonglong2 *>(f_coeff + col * D + r + 64 * q);
  const ulonglong2 a0 = x[0], a1 = x[1], c0 = x[16], c1 = x[17];
  bool bad = false;
  uint4 o;
  o.x = pack_sm1(a0.x, K, bad) | (pack_sm1(c0.x, K, bad) << 16);
  o.y = pack_sm1(a0.y, K, bad) | (pack_sm1(c0.y, K, bad) << 16);
  o.z = pack_sm1(a1.x, K, bad) | (pack_sm1(c1.x, K, bad) << 16);
  o.w = pack_sm1(a1.y, K, bad) | (pack_sm1(c1.y, K, bad) << 16);
  if (bad) raise(err, 1);
  *reinterpret_cast<uint4 *>(sd.smg[side] + (t0 - side * N * 512)) = o;
}

// Stage 1 of the digit planes' NTT on the matrix cores: for one element,
// Y[j1][m1] = sum_j2 zeta^((2 m1 + 1) j2) x[j1 + 32 j2] is a 32 x 32 x 32 product
// of the constant matrix Z[m1][j2] = zeta^((2 m1 + 1) j2) (its 8 signed D8 byte
// planes, az) with the ternary digits B[j2][j1] = x[j1 + 32 j2], so one
// v_mfma_i32_32x32x32_i8 per byte plane (|sum| <= 32 * 128) replaces the two
// integer and three field levels of neg_ct32 per lane. Lane (r, h) holds
// Z_t[r][16 h + j] and B[16 h + j][r] (j < 16) and gets D[m1][j1 = r] for
// m1 = (i & 3) + 8 (i >> 2) + 4 h in register i; Y = Q0 + Q1 2^32 with Q0 =
// sum_{t < 4} 2^(8t) D_t, Q1 = sum_{t >= 4} 2^(8(t-4)) D_t (|Q| < 2^37). A wave
// does both of its halves' elements (16 products), so the transpose into the
// second stage's layout stays inside the wave's own LDS tiles.
__device__ __forceinline__ v4i mx_digits(const uint32_t *w8, int kb) {
  // words q = 8 h + i of one element: x[r + 32 (2q)] | x[r + 32 (2q + 1)] << 16 (15-bit
  // magnitude | sign << 15); byte j of the result = digit kb of x[r + 32 (16 h + j)] in {0, 1, -1}
  v4i b;
#pragma unroll
  for (int p = 0; p < 4; p++) {
    const uint32_t w0 = w8[2 * p], w1 = w8[2 * p + 1];
    const uint32_t m0 = (w0 >> kb) & 0x10001u, m1 = (w1 >> kb) & 0x10001u;
    const uint32_t y0 = m0 | (((w0 >> 15) & m0) * 0xFEu), y1 = m1 | (((w1 >> 15) & m1) * 0xFEu);
    b[p] = (int)__builtin_amdgcn_perm(y1, y0, 0x06040200u);  // bytes 0, 2 of y0, then of y1
  }
  return b;
}
// one element's stage 1 and middle factors into its transpose tile Te[m1][j1];
// azl: the byte planes in LDS ([t][m1][j2] int8), read per product (registers
// are the constraint here: the Horner sums and the prefetched words stay live)
__device__ __forceinline__ v4i az_piece(const int8_t *azl, int t, int r, int h) {
  return *reinterpret_cast<const v4i *>(azl + (t * 32 + r) * 32 + 16 * h);
}
// Transposed: digits as the A operand (rows j1, K = j2), Z as B (K = j2, columns
// m1), so lane (r, h) gets Y[j1][m1 = r] for j1 = (i & 3) + 8 (i >> 2) + 4 h in
// register i -- the rows of column m1 = r that stage 2 wants in lane r, split
// between the two halves. The middle factors come after both elements
// (mid2_apply: mid2[j1][m1] = psi^((2 m1 + 1) j1), staged by mid2_stage).
__device__ __forceinline__ void mx_stage1_t(const int8_t *azl, const uint32_t *w8, int kb, uint64_t *y, int r, int h) {
  const v4i b = mx_digits(w8, kb);
  // Q = sum_t 2^(8t) D_t over 4 planes, two planes at a time (|partial| < 2^21 in int32)
  auto quarter = [&](int t0, int64_t *q) {
    v16i a0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(b, az_piece(azl, t0, r, h), (v16i){0}, 0, 0, 0);
    v16i a1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(b, az_piece(azl, t0 + 1, r, h), (v16i){0}, 0, 0, 0);
    int32_t p[16];
#pragma unroll
    for (int i = 0; i < 16; i++) p[i] = a0[i] + a1[i] * 256;
    a0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(b, az_piece(azl, t0 + 2, r, h), (v16i){0}, 0, 0, 0);
    a1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(b, az_piece(azl, t0 + 3, r, h), (v16i){0}, 0, 0, 0);
#pragma unroll
    for (int i = 0; i < 16; i++) q[i] = (int64_t)(p[i] + a0[i] * 65536) + (int64_t)a1[i] * (1ll << 24);
  };
  int64_t q0[16], q1[16];
  quarter(0, q0);
  quarter(4, q1);
#pragma unroll
  for (int i = 0; i < 16; i++) {
    // Y = Q0 + Q1 2^32 == A + (Q1l + Q1h) 2^32 with Q1 = Q1h 2^32 + Q1l, A = Q0 - Q1h
    // (2^64 == 2^32 - 1); = A.lo + T 2^32 with T = A.hi + Q1l + Q1h in (-2^7, 2^32 + 2^7),
    // = U + th 2^64 == U + th EPS, U = T.lo:A.lo, th = T >> 32 in {-1, 0, 1} (no wrap:
    // th = 1 leaves U < 2^39, th = -1 U > EPS). Any u64 is a valid gl::mul input.
    const int64_t q1h = q1[i] >> 32;
    const int64_t A = q0[i] - q1h;
    const int64_t T = (A >> 32) + (int64_t)(uint32_t)q1[i] + q1h;
    const uint64_t U = ((uint64_t)T << 32) | (uint32_t)A;
    const uint64_t yv = U + (uint64_t)((T >> 32) * (int64_t)gl::EPS);
    y[i] = yv;  // the middle factors follow for both elements at once (mid2_apply)
  }
}
// y0, y1 *= mid2[j1][m1 = r] with one table read per row for both elements
__device__ __forceinline__ void mid2_apply(const uint64_t *mid2, uint64_t *y0, uint64_t *y1, int r, int h) {
#pragma unroll
  for (int i = 0; i < 16; i++) {
    const int j1 = (i & 3) + 8 * (i >> 2) + 4 * h;
    const uint64_t m = mid2[j1 * 32 + r];
    y0[i] = gl::mul(y0[i], m);
    y1[i] = gl::mul(y1[i], m);
  }
}
// mid2[j1][m1] = psi^((2 m1 + 1) j1) from the launcher's table mid[j1][i'] =
// psi^((2 brv5(i') + 1) j1) (n32::stage_mid's source layout)
__device__ __forceinline__ void mid2_stage(uint64_t *mid2, const uint64_t *mid) {
  for (int q = threadIdx.x; q < n32::MID_U64; q += blockDim.x) mid2[q] = mid[(q & ~31) | n32::brv5(q & 31)];
}
template <bool NT>
__global__ void __launch_bounds__(512, 1) k_decompose_fused(size_t N, int L, int lb,
                                                           int K, FusedSides sd, const uint64_t *mid_fg,
                                                           const uint64_t *az_g, uint4 *frag, int nch,
                                                           uint64_t *sink) {
  __shared__ uint64_t lds_all[FD_S_U64];
  __shared__ uint64_t mid2[n32::MID_U64];
  __shared__ uint64_t az_l[1024];  // the 8 KiB of D8 byte planes of zeta^((2 m1 + 1) j2)
  __shared__ uint32_t vote[2][FD_WAVES];  // per wave: its plane is nonzero in the current unit
  mid2_stage(mid2, mid_fg);
  for (int q = threadIdx.x; q < 1024; q += blockDim.x) az_l[q] = az_g[q];
  __syncthreads();
  const int lane = threadIdx.x & 63, wib = threadIdx.x >> 6;
  const int r = lane & 31, h = lane >> 5, hw = 2 * wib + h;  // hw: this half's group within the block
  uint64_t *S = lds_all;
  const size_t W = N / L, nblk = (W + 15) / 16;
  const uint64_t b_pow = gl::mul_pow2(1, lb);  // B = 2^lb
  const int8_t *azl = reinterpret_cast<const int8_t *>(az_l);
  int nvote = 0;  // units voted on so far (block-uniform)
  // a task is one digit plane of one block of 16 groups of one side (planes
  // are independent: small W still fills the chip); consecutive blocks take
  // the planes of the same groups, so the packed words are shared through L2
  for (size_t task = blockIdx.x; task < sd.nside * nblk * K; task += gridDim.x) {
    const int side = task >= nblk * K;
    const size_t B = task / K - side * nblk;
    const int kb = (int)(task % K);
    const uint32_t *smg = sd.smg[side];
    uint64_t *f_k = sd.f_k[side], *w_ccs_k = sd.w_ccs_k[side];
    const int row0 = sd.row0[side], row_p0 = sd.row_p0[side];
    const size_t g = 16 * B + hw;
    const bool ok = g < W;
    const size_t gg = ok ? g : 0;
    // words q = 8 h .. 8 h + 7 of both of the wave's elements (groups 16 B + 2 wib + e; past W: group 0)
    const size_t ge0 = 16 * B + 2 * wib < W ? 16 * B + 2 * wib : 0, ge1 = 16 * B + 2 * wib + 1 < W ? 16 * B + 2 * wib + 1 : 0;
    auto word = [&](int q, int l) { return smg[(((q < 8 ? ge0 : ge1) * L + l) * 16 + 8 * h + (q & 7)) * 32 + r]; };
    uint32_t wn[16];  // next limb's packed words
#pragma unroll
    for (int q = 0; q < 16; q++) wn[q] = word(q, L - 1);
    // consume the first limb's words here, so that at the limb loop's head the
    // only outstanding loads are the prefetch issued before the previous limb's
    // 64-80 stores (the compiler then needs no vmcnt wait there, instead of
    // draining every store of the previous limb)
#pragma unroll
    for (int q = 0; q < 16; q += 8)
      asm volatile("" : "+v"(wn[q]), "+v"(wn[q + 1]), "+v"(wn[q + 2]), "+v"(wn[q + 3]), "+v"(wn[q + 4]),
                   "+v"(wn[q + 5]), "+v"(wn[q + 6]), "+v"(wn[q + 7]));
    {
      uint64_t acc[32];
#pragma unroll
      for (int i = 0; i < 32; i++) acc[i] = 0;
      for (int l = L - 1; l >= 0; l--) {
        const size_t e = (size_t)kb * N + gg * L + l;
        uint64_t v[32];
        // Is digit plane kb of this limb zero on both of the wave's elements? The top
        // limb of a balanced base-B decomposition of a field element has |digit| <= 8
        // (signed representative < 2^63, B^(L-1) = 2^60), so its planes 4..K-1 vanish,
        // and plane K-1 of the other limbs is zero unless a digit is exactly +-B/2. A
        // zero plane's transform is zero: only the Horner shift and the operand rows
        // (the offset form of 0) remain. Checked on the data (wave-uniform), so any
        // input stays exact.
        uint32_t nz = 0;
#pragma unroll
        for (int q = 0; q < 16; q++) nz |= wn[q] >> kb;
        const bool live = __ballot((nz & 0x10001u) != 0) != 0;
        if (live) {
          uint64_t y0[16], y1[16];
          mx_stage1_t(azl, wn, kb, y0, r, h);
          __builtin_amdgcn_sched_barrier(0);  // one element's products and epilogue at a time (registers)
          mx_stage1_t(azl, wn + 8, kb, y1, r, h);
          mid2_apply(mid2, y0, y1, r, h);
          n32::halves_to_elements(y0, y1, v);  // lane m1 = r of element h: its 32 j1
        }
        {  // words for the next limb, in flight through the second stage (at l = 0 a
           // harmless reload of limb L - 1)
          const int ln = l > 0 ? l - 1 : L - 1;
#pragma unroll
          for (int q = 0; q < 16; q++) wn[q] = word(q, ln);
        }
        if (live) {
          n32::cyc_dif32<false>(v);
        } else {
#pragma unroll
          for (int j = 0; j < 32; j++) v[j] = 0;
        }
        if (f_k) {  // uniform: without f_k the planes live only in the operand rows
          uint64_t *of = (ok ? f_k + e * D : sink) + r;
#pragma unroll
          for (int i = 0; i < 32; i++) out_store<NT>(&of[32 * n32::brv5(i)], v[i]);
        }
        if (l == L - 1) {  // Horner's first term
#pragma unroll
          for (int i = 0; i < 32; i++) acc[i] = v[i];
        } else if (lb == 15) {  // GoldiLocksDP B = 2^15: a shift instead of a product
#pragma unroll
          for (int i = 0; i < 32; i++) acc[i] = gl::add_weak(gl::shl_small_weak(acc[i], 15), v[i]);
        } else {
#pragma unroll
          for (int i = 0; i < 32; i++) acc[i] = gl::add(gl::mul(acc[i], b_pow), v[i]);
        }
        if (frag && (kb > 0 || row_p0 >= 0)) {
          const size_t u = B * L + l;  // contraction unit of these 16 columns
          const int row = kb > 0 ? row0 + kb - 1 : row_p0;
          // a unit whose plane is zero on all 16 columns is not written: its flag
          // says so, and the readers take the offset form of 0 there (DeadUnits).
          // The vote slots alternate from unit to unit: a wave cannot rewrite a slot
          // before every wave has passed the next unit's barrier.
          const int vs = nvote++ & 1;
          if (sd.dead && lane == 0) vote[vs][wib] = live ? 1u : 0u;
          __syncthreads();  // votes visible; every wave is done reading the previous unit's S
          bool any = true;
          if (sd.dead) {
            uint32_t a = 0;
#pragma unroll
            for (int q = 0; q < FD_WAVES; q++) a |= vote[vs][q];
            any = a != 0;
            if (threadIdx.x == 0) sd.dead[u * 32 + row] = any ? 0 : 1;
          }
          if (!any) continue;  // block-uniform: no further barrier for this unit
#pragma unroll
          for (int i = 0; i < 32; i++) S[(r + 32 * n32::brv5(i)) * FD_SROW + hw] = fenc(v[i]);
          __syncthreads();
          const int c = (int)(u >> 1), uh = (int)(u & 1);
#pragma unroll
          for (int rep = 0; rep < 2; rep++) {
            const int s = threadIdx.x + 512 * rep;
            const uint64_t *src = S + s * FD_SROW;
            uint64_t x[16];
#pragma unroll
            for (int j = 0; j < 16; j++) x[j] = src[j];
            uint4 pu[8];
            d8_transpose16(x, pu);
            uint4 *out = frag + fv_index(s, nch, c, row, uh);
#pragma unroll
            for (int b = 0; b < 8; b++) out_store<NT>(&out[4 * b], pu[b]);
          }
        }
      }
      if (ok) {
        uint64_t *ow = w_ccs_k + ((size_t)kb * W + g) * D + r;
#pragma unroll
        for (int i = 0; i < 32; i++) out_store<NT>(&ow[32 * n32::brv5(i)], gl::canon(acc[i]));
      }
    }
  }
}

// the packed sign|magnitude words (k_pack_sm's layout) -> the K digit planes in
// coefficient form: f_coeff_k[k][col][j] = sign(x_j) bit_k(|x_j|), one thread per output
__global__ void k_expand_sm(const uint32_t *smg, size_t N, int K, uint64_t *fck) {
  for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < (size_t)K * N * D;
       t += (size_t)gridDim.x * blockDim.x) {
    const int j = (int)(t % D), k = (int)(t / ((size_t)N * D));
    const size_t col = (t / D) % N;
    const int r = j & 31, jt = j >> 5, q = jt >> 1, h = jt & 1;
    const uint32_t hw = (smg[(col * 16 + q) * 32 + r] >> (16 * h)) & 0xFFFFu;
    const int64_t bit = (hw >> k) & 1;
    fck[t] = from_signed((hw & 0x8000u) ? -bit : bit);
  }
}

hipError_t expand_sm(const uint32_t *smg, size_t N, int K, uint64_t *fck, hipStream_t st) {
  if (!N) return hipSuccess;
  if (K < 1 || K > 15) return hipErrorInvalidValue;
  const size_t n = (size_t)K * N * D;
  const size_t nb = (n + 255) / 256;
  hipLaunchKernelGGL(k_expand_sm, dim3((unsigned)(nb < 65536 ? nb : 65536)), dim3(256), 0, st, smg, N, K, fck);
  return hipGetLastError();
}

// ---------------------------------------------------------------- launchers
hipError_t decompose_fused(const FusedSides &sd, size_t N, int lb, int L, int K, const ring::NegaTables &fwd, uint4 *frag, int nch, int *err, uint64_t *sink, int ncu,
                           hipStream_t st) {
  if (K > 15 || !fwd.mid || !sink || ncu < 1 || sd.nside < 1 || sd.nside > 2) return hipErrorInvalidValue;
  for (int s = 0; s < sd.nside; s++)
    if (!sd.smg[s]) return hipErrorInvalidValue;
  // sides whose words from_w_ccs already wrote (only side 1, the step's new witness) are not re-packed
  if ((sd.prepacked & ~2) || ((sd.prepacked & 2) && sd.nside != 2)) return hipErrorInvalidValue;
  FusedSides sp = sd;
  if (sd.prepacked & 2) sp.nside = 1;  // side 0 only
  {
    const size_t words = sp.nside * N * 512;
    hipLaunchKernelGGL(k_pack_sm, dim3((unsigned)((words / 4 + 255) / 256)), dim3(256), 0, st, sp, N, K, err);
  }
  // one 8-wave block per CU (LDS-bound); ntask = nblk K tasks spread evenly
  const size_t ntask = (N / L + 15) / 16 * (size_t)K * sd.nside;
  // every block takes the same number of tasks (no tail round on part of the
  // chip); the CUs left over run other streams' kernels
  const size_t per = (ntask + ncu - 1) / ncu;
  const unsigned grid = (unsigned)((ntask + per - 1) / per);
  // outputs: f_coeff_k, f_k, frag (each K N D words per side) and w_ccs_k
  const size_t out_bytes = sd.nside * (size_t)K * N * D * 8 * 3;
  if (!fwd.az) return hipErrorInvalidValue;
  if (dec_streaming(out_bytes, false))
    hipLaunchKernelGGL(k_decompose_fused<true>, dim3(grid), dim3(512), 0, st, N, L, lb, K, sd, fwd.mid, fwd.az, frag,
                       nch, sink);
  else
    hipLaunchKernelGGL(k_decompose_fused<false>, dim3(grid), dim3(512), 0, st, N, L, lb, K, sd, fwd.mid, fwd.az, frag,
                       nch, sink);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  // the f_coeff_k rows, when wanted, from the packed words
  for (int s = 0; s < sd.nside; s++)
    if (sd.f_coeff_k[s]) {
      e = expand_sm(sd.smg[s], N, K, sd.f_coeff_k[s], st);
      if (e != hipSuccess) return e;
    }
  return hipSuccess;
}
static unsigned half_blocks(size_t units, unsigned cap) {
  size_t b = (units + 2 * WPB - 1) / (2 * WPB);
  if (b < 1) b = 1;
  return (unsigned)(b < cap ? b : cap);
}

hipError_t transform_n32(uint64_t *data, size_t n, bool fwd, const ring::NegaTables &tb, hipStream_t st,
                         const uint64_t *src) {
  if (!src) src = data;
  if (fwd)
    hipLaunchKernelGGL(k_xform_n32<true>, dim3(half_blocks(n, 4096)), dim3(256), 0, st, src, data, n, tb.mid);
  else
    hipLaunchKernelGGL(k_xform_n32<false>, dim3(half_blocks(n, 4096)), dim3(256), 0, st, src, data, n, tb.mid);
  return hipGetLastError();
}
// below this W the one-half-wave-per-element kernels leave CUs idle
#ifndef LF_SPLIT_W
#define LF_SPLIT_W 4096
#endif
constexpr size_t SPLIT_W = LF_SPLIT_W;
size_t witness_split_w() { return SPLIT_W; }
hipError_t from_w_ccs_n32(const uint64_t *w_ccs, size_t W, int lb, int L, uint64_t *f_coeff, uint64_t *f,
                          const ring::NegaTables &fwd, const ring::NegaTables &inv, int *err, hipStream_t st,
                          uint32_t *smg) {
  if (W < SPLIT_W) {
    hipLaunchKernelGGL(k_from_w_ccs_digits, dim3(half_blocks(W, 4096)), dim3(256), 0, st, w_ccs, W, lb, L, f_coeff,
                       inv.mid, err, smg);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return transform_n32(f, W * (size_t)L, true, fwd, st, f_coeff);
  }
  hipLaunchKernelGGL(k_from_w_ccs_n32, dim3(half_blocks(W, 4096)), dim3(256), 0, st, w_ccs, W, lb, L, f_coeff,
                     f, fwd.mid, inv.mid, err, smg);
  return hipGetLastError();
}
hipError_t from_f_n32(const uint64_t *f, size_t W, int lb, int L, uint64_t *f_coeff, uint64_t *w_ccs,
                      const ring::NegaTables &inv, hipStream_t st, const int *run_if) {
  if (W < SPLIT_W) {
    const size_t units = ((W + 1) & ~(size_t)1) * L;
    hipLaunchKernelGGL(k_from_f_split, dim3((unsigned)((units + 2 * SPLIT_WPB - 1) / (2 * SPLIT_WPB))),
                       dim3(64 * SPLIT_WPB), 0, st, f, W, lb, L, f_coeff,
                       w_ccs, inv.mid, run_if);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(k_from_f_n32, dim3(half_blocks(W, 4096)), dim3(256), 0, st, f, W, lb, L, f_coeff, w_ccs,
                     inv.mid, run_if);
  return hipGetLastError();
}
hipError_t from_fcoeff_n32(uint64_t *f_coeff, size_t W, int lb, int L, uint64_t *f, uint64_t *w_ccs,
                           const ring::NegaTables &fwd, const int *gate, hipStream_t st,
                           const ring::NegaTables *inv) {
  if (!W) return hipSuccess;
  if (!fwd.mid || (inv && !inv->mid)) return hipErrorInvalidValue;
  const uint64_t *mid_ig = inv ? inv->mid : nullptr;
  if (W < SPLIT_W) {
    const size_t units = ((W + 1) & ~(size_t)1) * (L + 1);
    hipLaunchKernelGGL(k_from_fcoeff_split, dim3((unsigned)((units + 2 * SPLIT_WPB - 1) / (2 * SPLIT_WPB))),
                       dim3(64 * SPLIT_WPB), 0, st, f_coeff, W, lb, L, f, w_ccs, fwd.mid, gate, mid_ig);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(k_from_fcoeff_n32, dim3(half_blocks(W, 4096)), dim3(256), 0, st, f_coeff, W, lb, L, f, w_ccs,
                     fwd.mid, gate, mid_ig);
  return hipGetLastError();
}
hipError_t decompose_n32(const uint64_t *f_coeff, size_t N, int lb, int L, int K, uint64_t *f_coeff_k,
                         uint64_t *f_k, uint64_t *w_ccs_k, const ring::NegaTables &fwd, int *err,
                         hipStream_t st) {
  if (K > 15 || L > 5) return hipErrorInvalidValue;  // LDS: 4 waves x L x 4 KiB of packed limbs
  const unsigned nb = half_blocks(N / L, 4096);
#define LF_DN(LL)                                                                                        \
  case LL:                                                                                               \
    hipLaunchKernelGGL(k_decompose_n32<LL>, dim3(nb), dim3(256), 0, st, f_coeff, N, lb, K, f_coeff_k, f_k, \
                       w_ccs_k, fwd.mid, err);                                                           \
    break;
  switch (L) {
    LF_DN(1) LF_DN(2) LF_DN(3) LF_DN(4) LF_DN(5) default : return hipErrorInvalidValue;
  }
#undef LF_DN
  return hipGetLastError();
}

}  // namespace lfk
