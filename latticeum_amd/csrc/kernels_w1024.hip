// kernels_w1024.hip -- d = 1024 negacyclic kernels built on the one-wave DFT
// (ntt1024.hpp). One wavefront owns one ring element (transforms, from_w_ccs)
// or one group of L elements (decompose, from_f); waves never synchronise
// with each other, so there is no s_barrier anywhere on this path.
#include "kernels.hpp"
#include "ntt1024.hpp"

namespace lfk {

namespace {
constexpr int WPB = 4;  // waves per block

__device__ __forceinline__ int64_t sgn_rep(uint64_t v) {
  return v > (gl::P - 1) / 2 ? (int64_t)(v - gl::P) : (int64_t)v;
}
__device__ __forceinline__ uint64_t from_sgn(int64_t x) { return x < 0 ? gl::P - (uint64_t)(-x) : (uint64_t)x; }

struct WaveCtx {
  int lane, wave_global, nwaves;
  uint64_t *lds;
};
__device__ __forceinline__ WaveCtx wave_ctx(uint64_t *lds_all) {
  WaveCtx w;
  w.lane = threadIdx.x & 63;
  const int wib = threadIdx.x >> 6;
  w.wave_global = blockIdx.x * WPB + wib;
  w.nwaves = gridDim.x * WPB;
  w.lds = lds_all + wib * n1k::LDS_U64;
  return w;
}
__device__ __forceinline__ void load_tw1(uint64_t *tw, const uint64_t *tab, int lane) {
  const ulonglong2 *p = reinterpret_cast<const ulonglong2 *>(tab + lane * 16);
#pragma unroll
  for (int i = 0; i < 8; i++) {
    ulonglong2 x = p[i];
    tw[2 * i] = x.x;
    tw[2 * i + 1] = x.y;
  }
}
}  // namespace

// ---------------------------------------------------------------- transforms
template <bool FWD>
__global__ void __launch_bounds__(256) k_xform_w1024(uint64_t *data, size_t n, ring::NegaTables tb) {
  __shared__ uint64_t lds_all[WPB * n1k::LDS_U64];
  WaveCtx w = wave_ctx(lds_all);
  uint64_t tw1[16];
  load_tw1(tw1, tb.tw1, w.lane);
  for (size_t e = w.wave_global; e < n; e += w.nwaves) {
    uint64_t *g = data + e * 1024;
    uint64_t v[16];
#pragma unroll
    for (int i = 0; i < 16; i++) {
      const int j = w.lane + 64 * i;
      v[i] = FWD ? gl::mul(g[j], tb.twist[j]) : g[j];
    }
    n1k::dft1024<!FWD>(v, tw1, w.lds, w.lane);
#pragma unroll
    for (int r = 0; r < 16; r++) {
      const int j = n1k::out_index(w.lane, r);
      g[j] = FWD ? v[r] : gl::mul(v[r], tb.twist[j]);
    }
  }
}

// ---------------------------------------------------------------- Witness::from_w_ccs
// LF/arith.rs:230-248: ICRT -> gadget_decompose(B = 2^lb, L) -> CRT, one wave per element
__global__ void __launch_bounds__(256) k_from_w_ccs_w1024(const uint64_t *w_ccs, size_t W, int lb, int L,
                                                         uint64_t *f_coeff, uint64_t *f,
                                                         ring::NegaTables fwd, ring::NegaTables inv,
                                                         int *err) {
  __shared__ uint64_t lds_all[WPB * n1k::LDS_U64];
  WaveCtx w = wave_ctx(lds_all);
  uint64_t twf[16], twi[16];
  load_tw1(twf, fwd.tw1, w.lane);
  load_tw1(twi, inv.tw1, w.lane);
  const int64_t b = (int64_t)1 << lb, bh = b >> 1;
  for (size_t j = w.wave_global; j < W; j += w.nwaves) {
    const uint64_t *g = w_ccs + j * 1024;
    uint64_t v[16];
#pragma unroll
    for (int i = 0; i < 16; i++) v[i] = g[w.lane + 64 * i];
    n1k::dft1024<true>(v, twi, w.lds, w.lane);
    int64_t cur[16];
#pragma unroll
    for (int r = 0; r < 16; r++) cur[r] = sgn_rep(gl::mul(v[r], inv.twist[n1k::out_index(w.lane, r)]));
    for (int l = 0; l < L; l++) {
      uint64_t *oc = f_coeff + (j * L + l) * 1024;
#pragma unroll
      for (int r = 0; r < 16; r++) {
        // balanced digit (balanced_decomposition/mod.rs:76-91)
        int64_t q = (cur[r] + ((cur[r] >> 63) & (b - 1))) >> lb;  // truncating cur / 2^lb
        int64_t rem = cur[r] - (q << lb), ar = rem < 0 ? -rem : rem;
        int64_t dg = rem;
        if (ar > bh) {
          int64_t sg = rem < 0 ? -1 : 1;
          dg = rem - sg * b;
          q += sg;
        }
        cur[r] = q;
        const uint64_t fd = from_sgn(dg);
        const int p = n1k::out_index(w.lane, r);
        oc[p] = fd;
        w.lds[p] = fd;  // re-layout to the DFT input order
      }
      n1k::wave_lds_sync();
#pragma unroll
      for (int i = 0; i < 16; i++) {
        const int p = w.lane + 64 * i;
        v[i] = gl::mul(w.lds[p], fwd.twist[p]);
      }
      n1k::wave_lds_sync();
      n1k::dft1024<false>(v, twf, w.lds, w.lane);
      uint64_t *of = f + (j * L + l) * 1024;
#pragma unroll
      for (int r = 0; r < 16; r++) of[n1k::out_index(w.lane, r)] = v[r];
    }
    bool bad = false;
#pragma unroll
    for (int r = 0; r < 16; r++) bad |= cur[r] != 0;
    if (bad) atomicOr(err, 1);
  }
}

// ---------------------------------------------------------------- Witness::from_f
// LF/arith.rs:299-313: f_coeff = ICRT(f), w_ccs = recompose(f) -- one wave per group
__global__ void __launch_bounds__(256) k_from_f_w1024(const uint64_t *f, size_t W, int lb, int L,
                                                     uint64_t *f_coeff, uint64_t *w_ccs,
                                                     ring::NegaTables inv) {
  __shared__ uint64_t lds_all[WPB * n1k::LDS_U64];
  WaveCtx w = wave_ctx(lds_all);
  uint64_t twi[16];
  load_tw1(twi, inv.tw1, w.lane);
  for (size_t g = w.wave_global; g < W; g += w.nwaves) {
    uint64_t acc[16];
    for (int l = L - 1; l >= 0; l--) {
      const uint64_t *src = f + (g * L + l) * 1024;
      uint64_t v[16];
#pragma unroll
      for (int i = 0; i < 16; i++) {
        v[i] = src[w.lane + 64 * i];
        acc[i] = (l == L - 1) ? v[i] : gl::add(gl::mul_pow2(acc[i], lb), v[i]);
      }
      n1k::dft1024<true>(v, twi, w.lds, w.lane);
      uint64_t *oc = f_coeff + (g * L + l) * 1024;
#pragma unroll
      for (int r = 0; r < 16; r++) {
        const int p = n1k::out_index(w.lane, r);
        oc[p] = gl::mul(v[r], inv.twist[p]);
      }
    }
    uint64_t *ow = w_ccs + g * 1024;
#pragma unroll
    for (int i = 0; i < 16; i++) ow[w.lane + 64 * i] = acc[i];
  }
}

// ---------------------------------------------------------------- decompose_witness
// LF/nifs/decomposition.rs:162-167, decomposition/utils.rs:45-49, arith.rs:324-338,
// specialised to b_small = 2 (GoldiLocksDP): the balanced base-2 digits of v are
// sign(v) * bit_k(|v|) with no carries (|rem| <= b/2 always), so each digit is
// computed directly. One wave per group of L elements; |v| < 2^K is checked
// (the reference panics otherwise) and kept as 16-bit sign|magnitude (K <= 15).
constexpr int DW_LMAX = 8;
template <int L>
__global__ void __launch_bounds__(256) k_decompose_w1024(const uint64_t *f_coeff, size_t N, int lb,
                                                        int K, uint64_t *f_coeff_k, uint64_t *f_k,
                                                        uint64_t *w_ccs_k, ring::NegaTables fwd, int *err) {
  __shared__ uint64_t lds_all[WPB * n1k::LDS_U64];
  WaveCtx w = wave_ctx(lds_all);
  uint64_t twf[16], psi[16];
  load_tw1(twf, fwd.tw1, w.lane);
#pragma unroll
  for (int i = 0; i < 16; i++) psi[i] = fwd.twist[w.lane + 64 * i];
  const size_t W = N / L;
  for (size_t g = w.wave_global; g < W; g += w.nwaves) {
    uint32_t sm[L][8];  // 16-bit sign|magnitude pairs: [l][i/2]
    bool bad = false;
#pragma unroll
    for (int l = 0; l < L; l++) {
      const uint64_t *src = f_coeff + (g * L + l) * 1024;
#pragma unroll
      for (int i = 0; i < 16; i += 2) {
        int64_t a = sgn_rep(src[w.lane + 64 * i]), c = sgn_rep(src[w.lane + 64 * (i + 1)]);
        uint64_t ma = a < 0 ? (uint64_t)(-a) : (uint64_t)a, mc = c < 0 ? (uint64_t)(-c) : (uint64_t)c;
        bad |= (ma >> K) != 0 || (mc >> K) != 0;
        uint32_t ea = (uint32_t)(ma & 0x7FFF) | (a < 0 ? 0x8000u : 0u);
        uint32_t ec = (uint32_t)(mc & 0x7FFF) | (c < 0 ? 0x8000u : 0u);
        sm[l][i >> 1] = ea | (ec << 16);
      }
    }
    if (bad) atomicOr(err, 1);
    for (int k = 0; k < K; k++) {
      uint64_t acc[16];
#pragma unroll
      for (int l = L - 1; l >= 0; l--) {
        const size_t e = (size_t)k * N + g * L + l;
        uint64_t *oc = f_coeff_k + e * 1024;
        uint64_t v[16];
#pragma unroll
        for (int i = 0; i < 16; i++) {
          uint32_t h = (sm[l][i >> 1] >> ((i & 1) * 16)) & 0xFFFF;
          const bool bit = (h >> k) & 1, neg = h >> 15;
          oc[w.lane + 64 * i] = bit ? (neg ? gl::P - 1 : 1) : 0;
          v[i] = bit ? (neg ? gl::neg(psi[i]) : psi[i]) : 0;  // digit * psi^j without a product
        }
        n1k::dft1024<false>(v, twf, w.lds, w.lane);
        uint64_t *of = f_k + e * 1024;
#pragma unroll
        for (int r = 0; r < 16; r++) {
          of[n1k::out_index(w.lane, r)] = v[r];
          acc[r] = (l == L - 1) ? v[r] : gl::add(gl::mul_pow2(acc[r], lb), v[r]);
        }
      }
      uint64_t *ow = w_ccs_k + ((size_t)k * W + g) * 1024;
#pragma unroll
      for (int r = 0; r < 16; r++) ow[n1k::out_index(w.lane, r)] = acc[r];
    }
  }
}

// ---------------------------------------------------------------- launchers
static unsigned wave_blocks(size_t waves) {
  size_t b = (waves + WPB - 1) / WPB;
  return (unsigned)(b < 8192 ? (b ? b : 1) : 8192);
}

hipError_t transform_w1024(uint64_t *data, size_t n, bool fwd, const ring::NegaTables &tb, hipStream_t st) {
  if (fwd)
    hipLaunchKernelGGL(k_xform_w1024<true>, dim3(wave_blocks(n)), dim3(256), 0, st, data, n, tb);
  else
    hipLaunchKernelGGL(k_xform_w1024<false>, dim3(wave_blocks(n)), dim3(256), 0, st, data, n, tb);
  return hipGetLastError();
}
hipError_t from_w_ccs_w1024(const uint64_t *w_ccs, size_t W, int lb, int L, uint64_t *f_coeff, uint64_t *f,
                            const ring::NegaTables &fwd, const ring::NegaTables &inv, int *err,
                            hipStream_t st) {
  hipLaunchKernelGGL(k_from_w_ccs_w1024, dim3(wave_blocks(W)), dim3(256), 0, st, w_ccs, W, lb, L, f_coeff, f,
                     fwd, inv, err);
  return hipGetLastError();
}
hipError_t from_f_w1024(const uint64_t *f, size_t W, int lb, int L, uint64_t *f_coeff, uint64_t *w_ccs,
                        const ring::NegaTables &inv, hipStream_t st) {
  hipLaunchKernelGGL(k_from_f_w1024, dim3(wave_blocks(W)), dim3(256), 0, st, f, W, lb, L, f_coeff, w_ccs, inv);
  return hipGetLastError();
}
hipError_t decompose_w1024(const uint64_t *f_coeff, size_t N, int lb, int L, int K, uint64_t *f_coeff_k,
                           uint64_t *f_k, uint64_t *w_ccs_k, const ring::NegaTables &fwd, int *err,
                           hipStream_t st) {
  if (L > DW_LMAX || K > 15) return hipErrorInvalidValue;
#define LF_DW(LL)                                                                                       \
  case LL:                                                                                              \
    hipLaunchKernelGGL(k_decompose_w1024<LL>, dim3(wave_blocks(N / L)), dim3(256), 0, st, f_coeff, N, lb, K, \
                       f_coeff_k, f_k, w_ccs_k, fwd, err);                                              \
    break;
  switch (L) {
    LF_DW(1) LF_DW(2) LF_DW(3) LF_DW(4) LF_DW(5) LF_DW(6) LF_DW(7) LF_DW(8) default : return hipErrorInvalidValue;
  }
#undef LF_DW
  return hipGetLastError();
}

}  // namespace lfk
