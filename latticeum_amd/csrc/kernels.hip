// kernels.hip -- hand-written gfx950 kernels for the LatticeFold commit+fold
// hot path. Data layout in HBM: AoS ring elements, d u64 each (d = 24 for
// Phi_72 in the reference's in-place CRT layout [s0.c0, s0.c1, s0.c2, s1.c0, ..]
// (stark-rings crt.rs:53-77), d = 4^k for the negacyclic rings), canonical
// values. Every launcher returns hipError_t and takes the stream explicitly.
#include <cstdlib>
#include <cstring>

#include "digits.hpp"
#include "frag.hpp"
#include "kernels.hpp"
#include "ring.hpp"

namespace lfk {

using gl::Acc;

// ============================================================ Phi_72 transforms
// one thread per ring element; 16-B vector loads of the 192-B element
template <bool FWD>
__global__ void __launch_bounds__(256) k_phi72_transform(uint64_t *data, size_t n) {
  size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (e >= n) return;
  uint64_t c[24];
  const ulonglong2 *src = reinterpret_cast<const ulonglong2 *>(data + e * 24);
#pragma unroll
  for (int i = 0; i < 12; i++) {
    ulonglong2 v = src[i];
    c[2 * i] = v.x;
    c[2 * i + 1] = v.y;
  }
  if (FWD)
    ring::phi72_crt(c);
  else
    ring::phi72_icrt(c);
  ulonglong2 *dst = reinterpret_cast<ulonglong2 *>(data + e * 24);
#pragma unroll
  for (int i = 0; i < 12; i++) dst[i] = make_ulonglong2(c[2 * i], c[2 * i + 1]);
}

// ============================================================ negacyclic transforms
template <int D>
struct NT {
  static constexpr int T = D / 4 < 256 ? D / 4 : 256;  // threads per element
};

template <int D, bool FWD>
__global__ void __launch_bounds__(NT<D>::T) k_nega_transform(uint64_t *data, size_t n,
                                                            ring::NegaTables tb) {
  constexpr int T = NT<D>::T;
  __shared__ uint64_t buf[2][D];
  const int tid = threadIdx.x;
  for (size_t e = blockIdx.x; e < n; e += gridDim.x) {
    uint64_t *g = data + e * D;
#pragma unroll
    for (int i = tid; i < D; i += T) {
      uint64_t v = g[i];
      buf[0][i] = FWD ? gl::mul(v, tb.twist[i]) : v;
    }
    __syncthreads();
    uint64_t *r = ring::stockham4<D, T, !FWD>(buf[0], buf[1], tb.roots, tid);
#pragma unroll
    for (int i = tid; i < D; i += T) g[i] = FWD ? r[i] : gl::mul(r[i], tb.twist[i]);
    __syncthreads();
  }
}

// ============================================================ slot-wise ring product
__global__ void k_slot_mul_phi72(const uint64_t *a, const uint64_t *b, uint64_t *out, size_t nslots) {
  size_t s = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (s >= nslots) return;
  uint64_t x[3] = {a[3 * s], a[3 * s + 1], a[3 * s + 2]};
  uint64_t y[3] = {b[3 * s], b[3 * s + 1], b[3 * s + 2]};
  uint64_t z[3];
  gl::fq3_mul(x, y, z);
  out[3 * s] = z[0];
  out[3 * s + 1] = z[1];
  out[3 * s + 2] = z[2];
}
__global__ void k_slot_mul_nega(const uint64_t *a, const uint64_t *b, uint64_t *out, size_t n) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i < n) out[i] = gl::mul(a[i], b[i]);
}

// ============================================================ Montgomery edge
__global__ void k_mont(uint64_t *x, size_t n, int to) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i < n) x[i] = to ? gl::to_mont(gl::canon(x[i])) : gl::from_mont(x[i]);
}

// ============================================================ Witness::from_w_ccs
// LF/arith.rs:230-248: ICRT -> gadget_decompose(B, L) -> CRT.
// Phi_72: one thread per (w_ccs element j, digit l), so a launch has W * L
// threads (about 1,500 waves at the real zkvm shape instead of 310). Each
// thread redoes the ICRT of its element and the digit steps up to l; the last
// digit's thread checks that the carry ran out. Neighbouring threads write
// neighbouring 192-B outputs.
__global__ void __launch_bounds__(128) k_from_w_ccs_phi72(const uint64_t *w_ccs, size_t W, int lb,
                                                         int L, uint64_t *f_coeff, uint64_t *f,
                                                         int *err) {
  const size_t u = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (u >= W * (size_t)L) return;
  const size_t j = u / L;
  const int l = (int)(u - j * L);
  uint64_t c[24];
  const ulonglong2 *src = reinterpret_cast<const ulonglong2 *>(w_ccs + j * 24);
#pragma unroll
  for (int i = 0; i < 12; i++) {
    ulonglong2 v = src[i];
    c[2 * i] = v.x;
    c[2 * i + 1] = v.y;
  }
  ring::phi72_icrt(c);
  int64_t cur[24], dg[24];
#pragma unroll
  for (int i = 0; i < 24; i++) cur[i] = signed_rep(c[i]);
  for (int s = 0; s <= l; s++) {
#pragma unroll
    for (int i = 0; i < 24; i++) dg[i] = bal_digit(cur[i], lb);
  }
#pragma unroll
  for (int i = 0; i < 24; i++) c[i] = from_signed(dg[i]);
  ulonglong2 *dc = reinterpret_cast<ulonglong2 *>(f_coeff + u * 24);
#pragma unroll
  for (int i = 0; i < 12; i++) dc[i] = make_ulonglong2(c[2 * i], c[2 * i + 1]);
  ring::phi72_crt(c);
  ulonglong2 *df = reinterpret_cast<ulonglong2 *>(f + u * 24);
#pragma unroll
  for (int i = 0; i < 12; i++) df[i] = make_ulonglong2(c[2 * i], c[2 * i + 1]);
  if (l == L - 1) {
    bool bad = false;
#pragma unroll
    for (int i = 0; i < 24; i++) bad |= cur[i] != 0;
    if (bad) raise(err, 1);
  }
}

// negacyclic: one workgroup per w_ccs element.
template <int D>
__global__ void __launch_bounds__(NT<D>::T) k_from_w_ccs_nega(const uint64_t *w_ccs, size_t W,
                                                             int lb, int L, uint64_t *f_coeff,
                                                             uint64_t *f, ring::NegaTables fwd,
                                                             ring::NegaTables inv, int *err) {
  constexpr int T = NT<D>::T, PER = D / T;
  __shared__ uint64_t buf[2][D];
  const int tid = threadIdx.x;
  for (size_t j = blockIdx.x; j < W; j += gridDim.x) {
    const uint64_t *g = w_ccs + j * D;
#pragma unroll
    for (int i = tid; i < D; i += T) buf[0][i] = g[i];
    __syncthreads();
    uint64_t *r = ring::stockham4<D, T, true>(buf[0], buf[1], inv.roots, tid);
    int64_t cur[PER];
#pragma unroll
    for (int q = 0; q < PER; q++) cur[q] = signed_rep(gl::mul(r[tid + q * T], inv.twist[tid + q * T]));
    __syncthreads();
    for (int l = 0; l < L; l++) {
      uint64_t *oc = f_coeff + (j * L + l) * D;
#pragma unroll
      for (int q = 0; q < PER; q++) {
        const int i = tid + q * T;
        uint64_t dgt = from_signed(bal_digit(cur[q], lb));
        oc[i] = dgt;
        buf[0][i] = gl::mul(dgt, fwd.twist[i]);
      }
      __syncthreads();
      uint64_t *rr = ring::stockham4<D, T, false>(buf[0], buf[1], fwd.roots, tid);
      uint64_t *of = f + (j * L + l) * D;
#pragma unroll
      for (int q = 0; q < PER; q++) of[tid + q * T] = rr[tid + q * T];
      __syncthreads();
    }
    bool bad = false;
#pragma unroll
    for (int q = 0; q < PER; q++) bad |= cur[q] != 0;
    if (bad) raise(err, 1);
  }
}

// ============================================================ Witness::from_f
// LF/arith.rs:299-313: f_coeff = ICRT(f); w_ccs = gadget_recompose(f, B, L).
// Phi_72: one thread per f element (j, l); a block holds G = blockDim / L whole
// groups. The raw elements go through LDS, where the block's threads run the
// Horner recompose (balanced_decomposition/mod.rs:105-117) over the G * 24
// w_ccs coefficients and store them contiguously.
__global__ void __launch_bounds__(256) k_from_f_phi72(const uint64_t *f, size_t W, int lb, int L,
                                                     uint64_t *f_coeff, uint64_t *w_ccs, const int *run_if) {
  if (run_if && !*run_if) return;    // uniform: the coefficient-form fold produced f_coeff and w_ccs
  extern __shared__ uint64_t lds[];  // [G * L][24]
  const int G = blockDim.x / L, t = threadIdx.x;
  const size_t j0 = (size_t)blockIdx.x * G;
  const size_t u = j0 * L + t;
  if (t < G * L && u < W * (size_t)L) {
    uint64_t c[24];
    const ulonglong2 *src = reinterpret_cast<const ulonglong2 *>(f + u * 24);
#pragma unroll
    for (int i = 0; i < 12; i++) {
      ulonglong2 v = src[i];
      c[2 * i] = v.x;
      c[2 * i + 1] = v.y;
    }
#pragma unroll
    for (int i = 0; i < 24; i++) lds[t * 24 + i] = c[i];
    ring::phi72_icrt(c);
    ulonglong2 *dc = reinterpret_cast<ulonglong2 *>(f_coeff + u * 24);
#pragma unroll
    for (int i = 0; i < 12; i++) dc[i] = make_ulonglong2(c[2 * i], c[2 * i + 1]);
  }
  __syncthreads();
  const size_t ng = W - j0 < (size_t)G ? W - j0 : (size_t)G;
  for (int o = t; o < (int)ng * 24; o += blockDim.x) {
    const int g = o / 24, i = o - g * 24;
    const uint64_t *row = lds + g * L * 24 + i;
    uint64_t acc = row[(L - 1) * 24];
    for (int l = L - 2; l >= 0; l--) acc = gl::add(gl::mul_pow2(acc, lb), row[l * 24]);
    w_ccs[j0 * 24 + o] = acc;
  }
}

template <int D>
__global__ void __launch_bounds__(NT<D>::T) k_from_f_nega(const uint64_t *f, size_t W, int lb, int L,
                                                         uint64_t *f_coeff, uint64_t *w_ccs,
                                                         ring::NegaTables inv) {
  constexpr int T = NT<D>::T, PER = D / T;
  __shared__ uint64_t buf[2][D];
  const int tid = threadIdx.x;
  for (size_t j = blockIdx.x; j < W; j += gridDim.x) {
    uint64_t acc[PER];
    for (int l = L - 1; l >= 0; l--) {
      const uint64_t *g = f + (j * L + l) * D;
#pragma unroll
      for (int q = 0; q < PER; q++) {
        const int i = tid + q * T;
        uint64_t v = g[i];
        buf[0][i] = v;
        acc[q] = (l == L - 1) ? v : gl::add(gl::mul_pow2(acc[q], lb), v);
      }
      __syncthreads();
      uint64_t *r = ring::stockham4<D, T, true>(buf[0], buf[1], inv.roots, tid);
      uint64_t *oc = f_coeff + (j * L + l) * D;
#pragma unroll
      for (int q = 0; q < PER; q++) oc[tid + q * T] = gl::mul(r[tid + q * T], inv.twist[tid + q * T]);
      __syncthreads();
    }
    uint64_t *ow = w_ccs + j * D;
#pragma unroll
    for (int q = 0; q < PER; q++) ow[tid + q * T] = acc[q];
  }
}

// ============================================================ decompose_witness
// LF/nifs/decomposition.rs:162-167 + decomposition/utils.rs:45-49 + arith.rs:324-338:
// K balanced base-b_small digit vectors of f_coeff; per digit vector:
// f_k = CRT(f_coeff_k), w_ccs_k = recompose(f_k, B, L).
// Phi_72: one thread per element, 64 groups of L elements per block; the
// recompose across the L elements of a group goes through LDS.
constexpr int DEC_GROUPS = 48;  // 3 units of 16 groups: 240 of the 256 threads own an element
constexpr int DEC_SROW = 41;  // operand staging row (40 virtual slots + pad) of the fused d = 24 decomposition
// With frag != nullptr, planes k >= 1 are also written as i8-MFMA operand rows
// row0 + k - 1 (ajtai_mfma.hip, vector-major, Lp = L column order): the block's
// 48 groups are the 16-group units (G, l), G = 3 blockIdx.x + {0, 1, 2}, and each
// (unit, virtual slot) piece is assembled from the plane's NTT values in LDS.
// Every HBM access of the block is a run of whole 16-B pieces over contiguous
// rows: f_coeff comes in and f_coeff_k / f_k go out through LDS (the element
// rows [e][SROW] and a byte copy of the digits), not as one 192-B row per thread.
// blockIdx.z selects the side (both sides of a fold step in one launch)
__global__ void __launch_bounds__(256) k_decompose_phi72(FusedSides sd, size_t N, int lb, int L, int lbs, int K,
                                                        int *err, uint4 *frag, int nch, int srow) {
  extern __shared__ uint64_t lds[];  // [DEC_GROUPS * L][srow] u64; a row's words 25..27 hold the digit bytes
  const int side = blockIdx.z;
  const uint64_t *f_coeff = sd.f_coeff[side];
  uint64_t *f_coeff_k = sd.f_coeff_k[side], *f_k = sd.f_k[side], *w_ccs_k = sd.w_ccs_k[side];
  const int row0 = sd.row0[side];
  const int t = threadIdx.x, ne = DEC_GROUPS * L;
  int8_t *dgl = reinterpret_cast<int8_t *>(lds + 25);  // element e's digits at dgl[e * 8 srow + i]
  const size_t W = N / L;
  const size_t j0 = (size_t)blockIdx.x * ne, j = j0 + t;  // element index
  const int nv = (int)(N - j0 < (size_t)ne ? N - j0 : (size_t)ne);  // valid elements of the block
  const bool act = t < nv;
  // the block's f_coeff rows, 16 B per thread per step
  for (int q = t; q < nv * 12; q += blockDim.x) {
    const int e = q / 12, pr = q - 12 * e;
    const ulonglong2 v = reinterpret_cast<const ulonglong2 *>(f_coeff + j0 * 24)[q];
    lds[e * srow + 2 * pr] = v.x;
    lds[e * srow + 2 * pr + 1] = v.y;
  }
  __syncthreads();
  int64_t cur[24];
  if (act) {
#pragma unroll
    for (int i = 0; i < 24; i++) cur[i] = signed_rep(lds[t * srow + i]);
  }
  // b = 2 (lbs = 1): the balanced digits are sign(v) bit_k(|v|) (bal_digit's
  // remainder is never rounded), so the planes are independent and
  // blockIdx.y takes a range of them; otherwise gridDim.y = 1 and the planes
  // run in order on the residual
  const int KP = (K + (int)gridDim.y - 1) / (int)gridDim.y;
  const int k0 = (int)blockIdx.y * KP, k1 = k0 + KP < K ? k0 + KP : K;
  for (int k = k0; k < k1; k++) {
    uint64_t c[24];
    if (act) {
#pragma unroll
      for (int i = 0; i < 24; i++) {
        int64_t dg;
        if (lbs == 1) {
          const int64_t m = cur[i] < 0 ? -cur[i] : cur[i], bit = (m >> k) & 1;
          dg = cur[i] < 0 ? -bit : bit;
        } else {
          dg = bal_digit(cur[i], lbs);
        }
        c[i] = from_signed(dg);
        // |digit| <= b/2 fits a byte for b_small <= 2^8; larger b_small keeps the u64 path below
        if (lbs <= 8) dgl[t * 8 * srow + i] = (int8_t)dg;
      }
      if (lbs > 8) {
        ulonglong2 *dc = reinterpret_cast<ulonglong2 *>(f_coeff_k + ((size_t)k * N + j) * 24);
#pragma unroll
        for (int i = 0; i < 12; i++) dc[i] = make_ulonglong2(c[2 * i], c[2 * i + 1]);
      }
      ring::phi72_crt(c);
    }
    __syncthreads();  // the f_coeff rows (first plane) or the previous plane's rows are consumed
    if (act) {
#pragma unroll
      for (int i = 0; i < 24; i++) lds[t * srow + i] = c[i];
    }
    __syncthreads();
    // f_coeff_k and f_k rows of the block, and the recompose: one thread per (group, coefficient)
    {
      uint64_t *fck = f_coeff_k + ((size_t)k * N + j0) * 24, *fk = f_k + ((size_t)k * N + j0) * 24;
      for (int q = t; q < nv * 12; q += blockDim.x) {
        const int e = q / 12, pr = q - 12 * e;
        if (lbs <= 8)
          reinterpret_cast<ulonglong2 *>(fck)[q] =
              make_ulonglong2(from_signed(dgl[e * 8 * srow + 2 * pr]), from_signed(dgl[e * 8 * srow + 2 * pr + 1]));
        reinterpret_cast<ulonglong2 *>(fk)[q] = make_ulonglong2(lds[e * srow + 2 * pr], lds[e * srow + 2 * pr + 1]);
      }
    }
    for (int u = t; u < DEC_GROUPS * 24; u += blockDim.x) {
      const int g = u / 24, i = u % 24;
      const size_t wj = (size_t)blockIdx.x * DEC_GROUPS + g;
      if (wj < W) {
        uint64_t a = lds[(g * L + L - 1) * srow + i];
        for (int l = L - 2; l >= 0; l--) a = gl::add(gl::mul_pow2(a, lb), lds[(g * L + l) * srow + i]);
        w_ccs_k[((size_t)k * W + wj) * 24 + i] = a;
      }
    }
    if (frag && k > 0) {
      // each element's 40 virtual slots (Toom-3 evaluations, ring::phi72_eval) as
      // D8 words into LDS rows of srow, then one thread per (unit, virtual
      // slot) gathers the unit's 16 columns into the 8 operand pieces
      __syncthreads();  // the copy-out and recompose reads of lds are done
      if (act) {
#pragma unroll
        for (int vs = 0; vs < 40; vs++) lds[t * srow + vs] = fenc(ring::phi72_eval(c, vs));
      }
      __syncthreads();
      for (int tk = t; tk < DEC_GROUPS / 16 * L * 40; tk += blockDim.x) {
        const int vs = tk % 40, ul = tk / 40, gh = ul / L, l = ul - gh * L;
        const size_t u = ((size_t)blockIdx.x * (DEC_GROUPS / 16) + gh) * L + l;  // contraction unit
        if (u >= 2 * (size_t)nch) continue;
        uint64_t x[16];
#pragma unroll
        for (int jj = 0; jj < 16; jj++) {
          const int g = gh * 16 + jj;
          x[jj] = (size_t)blockIdx.x * DEC_GROUPS + g < W ? lds[(g * L + l) * srow + vs] : 0;
        }
        uint4 pu[8];
        d8_transpose16(x, pu);
        uint4 *out = frag + fv_index(vs, nch, (int)(u >> 1), row0 + k - 1, (int)(u & 1));
#pragma unroll
        for (int b = 0; b < 8; b++) out[4 * b] = pu[b];
      }
    }
    if (k + 1 < k1) __syncthreads();  // this plane's reads of the digit bytes and rows are done
  }
  if (act && blockIdx.y == 0) {
    bool bad = false;
#pragma unroll
    for (int i = 0; i < 24; i++) bad |= lbs == 1 ? ((cur[i] < 0 ? -cur[i] : cur[i]) >> K) != 0 : cur[i] != 0;
    if (bad) raise(err, 1);
  }
}

// Phi_72 with b_small = 2, wave-local (the default d = 24 decomposition): a wave
// owns 16 groups -- one 16-column contraction unit per limb -- at 4 digit
// planes; lane 16 kq + gi owns group 16 G + gi at plane 4 pass + kq and walks
// the group's L limbs. The plane's digits of a limb are kept as two bit masks,
// so w_ccs_k = sum_l B^l f_k[gL + l] = CRT(sum_l B^l D_l) (linearity; an exact
// integer for (L - 1) lb < 62) is one more CRT per group, not a 24-value
// accumulator in registers. Every store instruction writes whole 192-B rows:
// lane t stores piece t % 12 of row t / 12 (64 lanes = 5.3 rows), the rows
// coming from the owning lane's masks (f_coeff_k, by ds_bpermute) or from a
// wave-private LDS tile (f_k, w_ccs_k) -- one request per line instead of one
// per 16-B piece, which is what bounds a store stream scattered over 192-B
// rows. The operand pieces of a (unit, plane) are a byte transpose over the 16
// lanes of a quarter, 8 virtual slots at a time through the same tile; each
// lane then emits the 4 pieces of one (plane, virtual slot, digit half). The
// waves of a block never synchronise with each other.
constexpr int PW_VS = 8;     // virtual slots per staging round (4 kq x 8 vs x 2 halves = one task per lane)
constexpr int PW_ROW = 17;   // u64 per operand staging row: 16 columns + pad
constexpr int PW_RROW = 25;  // u64 per element row in the tile: 24 + pad
constexpr int PW_WAVE_U64 = 64 * PW_RROW;  // 12.8 KB per wave (>= 4 PW_VS PW_ROW)
template <int NT>
__device__ __forceinline__ void st16(ulonglong2 *p, ulonglong2 v) {
  if (NT)
    nt_store(reinterpret_cast<uint4 *>(p), make_uint4((uint32_t)v.x, (uint32_t)(v.x >> 32), (uint32_t)v.y, (uint32_t)(v.y >> 32)));
  else
    *p = v;
}
__device__ __forceinline__ uint64_t pw_digit(uint32_t nz, uint32_t ng, int i) {
  return (nz >> i & 1) ? ((ng >> i & 1) ? gl::P - 1 : 1) : 0;
}
// the coefficients of every (element, limb) of both sides as 16-bit
// sign|magnitude (bit 15 the sign, bits 0..14 |x|) once, so the K planes'
// waves read 48 B and take a bit instead of 24 u64 and a signed magnitude each
// (the range check |x| < 2^K is here too); thread = (side, element, pair)
__global__ void k_pack_sm24(FusedSides sd, size_t N, int K, int *err) {
  const size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (t >= (size_t)sd.nside * N * 12) return;
  const int side = t >= N * 12;
  const size_t q = t - side * N * 12;  // (element, pair)
  const ulonglong2 v2 = reinterpret_cast<const ulonglong2 *>(sd.f_coeff[side])[q];
  bool bad = false;
  uint32_t o = 0;
#pragma unroll
  for (int h = 0; h < 2; h++) {
    const int64_t v = signed_rep(h ? v2.y : v2.x);
    const uint64_t m = v < 0 ? (uint64_t)(-v) : (uint64_t)v;
    bad |= (m >> K) != 0;
    o |= ((uint32_t)(m & 0x7FFF) | (v < 0 ? 0x8000u : 0u)) << (16 * h);
  }
  if (bad) raise(err, 1);
  sd.smg[side][q] = o;
}

// NTM: streaming stores, bit 0 f_coeff_k, bit 1 f_k, bit 2 operand pieces; bit 3:
// packed planes only -- no u64 f_coeff_k / f_k rows, the decomposed witnesses
// stay as the digit masks (lf_fold_step_bufs.planes, lf_dev_expand_planes)
template <int NTM>
__global__ void __launch_bounds__(256) k_decompose_phi72_w(FusedSides sd, size_t N, int lb, int L, int K, int *err,
                                                          uint4 *frag, int nch, size_t nblk) {
  constexpr bool ROWS = !(NTM & 8);
  __shared__ uint64_t lds_all[4 * PW_WAVE_U64];
  const int lane = threadIdx.x & 63, wib = threadIdx.x >> 6;
  uint64_t *S = lds_all + wib * PW_WAVE_U64;
  const int npass = (K + 3) / 4;
  const size_t task = (size_t)blockIdx.x * 4 + wib;  // (side, G, pass), pass fastest
  if (task >= (size_t)sd.nside * nblk * npass) return;  // wave-uniform; the kernel has no block barrier
  const int pass = (int)(task % npass);
  const size_t rest = task / npass;
  const int side = rest >= nblk ? 1 : 0;
  const size_t G = rest - side * nblk;
  const int kq = lane >> 4, gi = lane & 15, k = 4 * pass + kq;
  const bool kok = k < K;
  const size_t W = N / L, g = 16 * G + gi;
  const bool ok = g < W;
  uint64_t *f_coeff_k = sd.f_coeff_k[side], *f_k = sd.f_k[side], *w_ccs_k = sd.w_ccs_k[side];
  const int row0 = sd.row0[side];
  // this lane's operand task: plane kq_t, virtual slot PW_VS r + vl_t, digit half hf_t
  const int kq_t = lane >> 4, vl_t = (lane & 3) | ((lane >> 3 & 1) << 2), hf_t = lane >> 2 & 1;
  const int k_t = 4 * pass + kq_t;
  const bool emit = frag && k_t >= 1 && k_t < K;
  // this lane's row pieces: piece (64 it + lane) % 12 of the row of source lane
  // (64 it + lane) / 12, it < 12. The lane index goes through an empty asm at
  // each use, so these per-piece offsets are recomputed (a few integer
  // operations) instead of being hoisted out of the limb loop into 100+ VGPRs
  auto opaque_lane = [&]() {
    int x = lane;
    asm volatile("" : "+v"(x));
    return x;
  };
  auto row_live = [&](int j) { return 16 * G + (j & 15) < W && 4 * pass + (j >> 4) < K; };
  uint32_t nzm[8], ngm[8];
  for (int l = L - 1; l >= 0; l--) {
    uint32_t nz = 0, ng = 0;
    if (ok && kok) {  // plane k of the 24 packed sign|magnitude coefficients (k_pack_sm24)
      const uint4 *src = reinterpret_cast<const uint4 *>(sd.smg[side] + (g * L + l) * 12);
#pragma unroll
      for (int q = 0; q < 3; q++) {
        const uint4 w4 = src[q];
        const uint32_t w[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
        for (int i = 0; i < 8; i++) {
          const uint32_t hw = w[i >> 1] >> (16 * (i & 1));
          const uint32_t bit = (hw >> k) & 1u;
          nz |= bit << (8 * q + i);
          ng |= (bit & (hw >> 15)) << (8 * q + i);
        }
      }
    }
#pragma unroll
    for (int q = 0; q < 8; q++)
      if (q == l) {
        nzm[q] = nz;
        ngm[q] = ng;
      }
    if (sd.masks[side] && ok && kok) sd.masks[side][(size_t)k * N + g * L + l] = make_uint2(nz, ng);
    // f_coeff_k rows from the owners' masks
    if constexpr (ROWS) {
    const int ln0 = opaque_lane();
#pragma unroll
    for (int it = 0; it < 12; it++) {
      const int j = (64 * it + ln0) / 12, pq = (64 * it + ln0) % 12;
      const uint32_t nzj = (uint32_t)__builtin_amdgcn_ds_bpermute(4 * j, (int)nz);
      const uint32_t ngj = (uint32_t)__builtin_amdgcn_ds_bpermute(4 * j, (int)ng);
      if (row_live(j)) {
        const size_t ej = (16 * G + (j & 15)) * L + l;
        st16<NTM & 1>(reinterpret_cast<ulonglong2 *>(f_coeff_k + ((size_t)(4 * pass + (j >> 4)) * N + ej) * 24) + pq,
                      make_ulonglong2(pw_digit(nzj, ngj, 2 * pq), pw_digit(nzj, ngj, 2 * pq + 1)));
      }
    }
    }
    // Planes that are zero on all 16 groups of this unit (the top limb's planes 4..K-1
    // of a balanced decomposition of a field element; fused d = 1024 / 4096 do the
    // same): bit 16 kq + gi of bal = lane's digits nonzero. A wave whose 4 planes are
    // all zero skips the transform and the operand rounds; a zero plane's operand
    // rows are left unwritten and flagged (lfk::DeadUnits)
    const uint64_t bal = __ballot(nz != 0);
    uint64_t c[24];
    if (bal) {
      ring::phi72_crt_ternary(nz, ng, c);
    } else {
#pragma unroll
      for (int i = 0; i < 24; i++) c[i] = 0;
    }
    // f_k rows through the tile
    if constexpr (ROWS) {
#pragma unroll
    for (int i = 0; i < 12; i++)
      *reinterpret_cast<ulonglong2 *>(S + lane * PW_RROW + 2 * i) = make_ulonglong2(c[2 * i], c[2 * i + 1]);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const int ln1 = opaque_lane();
#pragma unroll
    for (int it = 0; it < 12; it++) {
      const int j = (64 * it + ln1) / 12, pq = (64 * it + ln1) % 12;
      const ulonglong2 v = *reinterpret_cast<const ulonglong2 *>(S + j * PW_RROW + 2 * pq);
      if (row_live(j)) {
        const size_t ej = (16 * G + (j & 15)) * L + l;
        st16<NTM & 2>(reinterpret_cast<ulonglong2 *>(f_k + ((size_t)(4 * pass + (j >> 4)) * N + ej) * 24) + pq, v);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the tile is read before the operand rounds reuse it
    }
    if (frag && sd.dead && gi == 0 && k >= 1 && k < K)  // one lane per plane writes its flag
      sd.dead[(G * L + l) * 32 + row0 + k - 1] = ((bal >> (16 * kq)) & 0xFFFFull) ? 0 : 1;
    if (frag && (bal || !sd.dead)) {
      const size_t u = G * L + l;  // contraction unit of these 16 columns
      const int ch = (int)(u >> 1), uh = (int)(u & 1);
      const bool live_t = !sd.dead || ((bal >> (16 * kq_t)) & 0xFFFFull) != 0;  // this lane's task's plane
#pragma unroll
      for (int r = 0; r < 40 / PW_VS; r++) {
        // keep the rounds in order (the compiler would otherwise evaluate all
        // 40 virtual slots up front)
#pragma unroll
        for (int i = 0; i < 24; i += 4) asm volatile("" : "+v"(c[i]), "+v"(c[i + 1]), "+v"(c[i + 2]), "+v"(c[i + 3]));
#pragma unroll
        for (int v = 0; v < PW_VS; v++) S[(kq * PW_VS + v) * PW_ROW + gi] = fenc(ring::phi72_eval(c, PW_VS * r + v));
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's tile writes landed
        const uint32_t *row = reinterpret_cast<const uint32_t *>(S + (kq_t * PW_VS + vl_t) * PW_ROW) + hf_t;
        uint32_t w[16];
#pragma unroll
        for (int jj = 0; jj < 16; jj++) w[jj] = row[2 * jj];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // read before the next round overwrites the tile
        if (emit && live_t) {
          // 4 pieces: digit 4 hf_t + b of the 16 columns (byte jj = column jj)
          uint32_t o[4][4];
#pragma unroll
          for (int q = 0; q < 4; q++) byte_tr4(w + 4 * q, o[q]);
          const int vs = PW_VS * r + vl_t;
          uint4 *out = frag + fv_index(vs, nch, ch, row0 + k_t - 1, uh) + 16 * hf_t;
#pragma unroll
          for (int b = 0; b < 4; b++) out_store<(NTM & 4) != 0>(&out[4 * b], make_uint4(o[0][b], o[1][b], o[2][b], o[3][b]));
        }
      }
    }
  }
  {  // w_ccs_k = CRT(sum_l B^l D_l), rows w_ccs_k[k][16 G ..] through the tile
    uint64_t c[24];
#pragma unroll
    for (int i = 0; i < 24; i++) {
      int64_t a = 0;
      for (int l = L - 1; l >= 0; l--) {
        uint32_t nz = 0, ng = 0;
#pragma unroll
        for (int q = 0; q < 8; q++)
          if (q == l) {
            nz = nzm[q];
            ng = ngm[q];
          }
        a = a * ((int64_t)1 << lb) + ((nz >> i & 1) ? ((ng >> i & 1) ? -1 : 1) : 0);
      }
      c[i] = from_signed(a);
    }
    ring::phi72_crt(c);
#pragma unroll
    for (int i = 0; i < 12; i++)
      *reinterpret_cast<ulonglong2 *>(S + lane * PW_RROW + 2 * i) = make_ulonglong2(c[2 * i], c[2 * i + 1]);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int it = 0; it < 12; it++) {
      const int j = (64 * it + lane) / 12, pq = (64 * it + lane) % 12;
      const ulonglong2 v = *reinterpret_cast<const ulonglong2 *>(S + j * PW_RROW + 2 * pq);
      if (row_live(j))
        reinterpret_cast<ulonglong2 *>(w_ccs_k + ((size_t)(4 * pass + (j >> 4)) * W + 16 * G + (j & 15)) * 24)[pq] = v;
    }
  }
}

// negacyclic: one workgroup per group of L elements; coefficients of the
// group kept in registers as int64 "cur" (|v| < 2^K for a valid witness).
template <int D>
__global__ void __launch_bounds__(NT<D>::T) k_decompose_nega(const uint64_t *f_coeff, size_t N, int lb,
                                                            int L, int lbs, int K, uint64_t *f_coeff_k,
                                                            uint64_t *f_k, uint64_t *w_ccs_k,
                                                            ring::NegaTables fwd, int *err) {
  constexpr int T = NT<D>::T, PER = D / T, LMAX = 8;
  __shared__ uint64_t buf[2][D];
  const int tid = threadIdx.x;
  const size_t W = N / L;
  for (size_t g = blockIdx.x; g < W; g += gridDim.x) {
    int64_t cur[LMAX][PER];
#pragma unroll
    for (int l = 0; l < LMAX; l++)
      if (l < L)
#pragma unroll
        for (int q = 0; q < PER; q++) cur[l][q] = signed_rep(f_coeff[(g * L + l) * D + tid + q * T]);
    for (int k = 0; k < K; k++) {
      uint64_t acc[PER];
#pragma unroll
      for (int l = LMAX - 1; l >= 0; l--) {
        if (l >= L) continue;
        const size_t e = (size_t)k * N + g * L + l;
#pragma unroll
        for (int q = 0; q < PER; q++) {
          const int i = tid + q * T;
          int64_t dg = bal_digit(cur[l][q], lbs);
          f_coeff_k[e * D + i] = from_signed(dg);
          uint64_t tw = fwd.twist[i];
          buf[0][i] = dg == 0 ? 0 : (dg == 1 ? tw : (dg == -1 ? gl::neg(tw) : gl::mul(from_signed(dg), tw)));
        }
        __syncthreads();
        uint64_t *r = ring::stockham4<D, T, false>(buf[0], buf[1], fwd.roots, tid);
#pragma unroll
        for (int q = 0; q < PER; q++) {
          uint64_t v = r[tid + q * T];
          f_k[e * D + tid + q * T] = v;
          acc[q] = (l == L - 1) ? v : gl::add(gl::mul_pow2(acc[q], lb), v);
        }
        __syncthreads();
      }
#pragma unroll
      for (int q = 0; q < PER; q++) w_ccs_k[((size_t)k * W + g) * D + tid + q * T] = acc[q];
    }
    bool bad = false;
#pragma unroll
    for (int l = 0; l < LMAX; l++)
      if (l < L)
#pragma unroll
        for (int q = 0; q < PER; q++) bad |= cur[l][q] != 0;
    if (bad) raise(err, 1);
  }
}

// ============================================================ Ajtai commitment
// LF/commitment/commitment_scheme.rs:37-54 -> LA/matrix.rs:168-178:
//   cm[v][i] = sum_j A[i][j] (.) f_v[j]    (slot-wise products)
// Work units: (slot chunk, row tile, column split) x vector tile. Each thread
// owns one slot position and an R x V tile of column accumulators (gl::CAcc,
// 8 VALU ops per 64x64 MAC). Units that read the same A tile (same slot
// chunk / row tile / column split, different vector tiles) get block ids
// that are congruent mod 8, i.e. land on one XCD under round-robin dispatch,
// so A is re-read from that XCD's L2 rather than HBM (speed only). Loads of
// column j+1 are issued before the MACs of column j.
struct AjtaiGrid {
  int nsc, nrt, nsplit, nvt;  // slot chunks, row tiles, column splits, vector tiles
  __host__ __device__ int others() const { return nsc * nrt * nsplit; }
  __host__ __device__ unsigned blocks() const { return (unsigned)(((others() + 7) / 8) * nvt * 8); }
};
__device__ __forceinline__ bool ajtai_unit(const AjtaiGrid &g, int &sc, int &rt, int &js, int &vt) {
  const int L = blockIdx.x;
  const int lo = L % 8, hi = L / 8;
  vt = hi % g.nvt;
  const int other = (hi / g.nvt) * 8 + lo;
  if (other >= g.others()) return false;
  sc = other % g.nsc;
  rt = (other / g.nsc) % g.nrt;
  js = other / (g.nsc * g.nrt);
  return true;
}

template <int R, int V>
__global__ void __launch_bounds__(256) k_ajtai_nega(const uint64_t *A, size_t kappa, size_t ncols,
                                                   int d, VecPtrs fv, int nvec, size_t jchunk,
                                                   AjtaiGrid g, uint64_t *partial) {
  int sc, rt, js, vt;
  if (!ajtai_unit(g, sc, rt, js, vt)) return;
  const int s = sc * 256 + threadIdx.x;  // slot
  if (s >= d) return;
  const int i0 = rt * R, v0 = vt * V;
  const size_t j0 = (size_t)js * jchunk, j1 = min(ncols, j0 + jchunk);
  const uint64_t *pa[R];
  const uint64_t *pb[V];
#pragma unroll
  for (int r = 0; r < R; r++) pa[r] = A + ((size_t)min(i0 + r, (int)kappa - 1) * ncols) * d + s;
#pragma unroll
  for (int v = 0; v < V; v++) pb[v] = fv.p[min(v0 + v, nvec - 1)] + s;
  gl::CAcc acc[R][V];
#pragma unroll
  for (int r = 0; r < R; r++)
#pragma unroll
    for (int v = 0; v < V; v++) gl::cacc_zero(acc[r][v]);
  uint64_t a[R], b[V];
  if (j0 < j1) {
#pragma unroll
    for (int r = 0; r < R; r++) a[r] = pa[r][j0 * d];
#pragma unroll
    for (int v = 0; v < V; v++) b[v] = pb[v][j0 * d];
  }
  for (size_t j = j0; j < j1; j++) {
    uint64_t an[R], bn[V];
    const size_t jn = (j + 1 < j1 ? j + 1 : j) * d;
#pragma unroll
    for (int r = 0; r < R; r++) an[r] = pa[r][jn];
#pragma unroll
    for (int v = 0; v < V; v++) bn[v] = pb[v][jn];
#pragma unroll
    for (int r = 0; r < R; r++)
#pragma unroll
      for (int v = 0; v < V; v++) gl::cacc_mad(acc[r][v], a[r], b[v]);
#pragma unroll
    for (int r = 0; r < R; r++) a[r] = an[r];
#pragma unroll
    for (int v = 0; v < V; v++) b[v] = bn[v];
  }
#pragma unroll
  for (int r = 0; r < R; r++)
#pragma unroll
    for (int v = 0; v < V; v++)
      if (i0 + r < (int)kappa && v0 + v < nvec)
        partial[(((size_t)js * nvec + v0 + v) * kappa + i0 + r) * d + s] = gl::cacc_reduce(acc[r][v]);
}

// Phi_72: lanes = 8 Fq3 slots x 8 column phases; R x V tile of Fq3 accumulators
// (9 column-accumulated products per Fq3 MAC into 5 sums, ring::fq3acc layout).
struct Fq3CAcc {
  gl::CAcc s00, s0n, s1, s1n, s2;
};
template <int R, int V>
__global__ void __launch_bounds__(256) k_ajtai_phi72(const uint64_t *A, size_t kappa, size_t ncols,
                                                    VecPtrs fv, int nvec, size_t jchunk,
                                                    uint64_t *partial) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int slot = lane & 7, ph = lane >> 3;  // column phase 0..7
  const int i0 = blockIdx.y * R;
  const int nvt = (nvec + V - 1) / V;
  const int v0 = (blockIdx.z % nvt) * V;
  const int js = blockIdx.x * 4 + wave;  // column split index
  const size_t j0 = (size_t)js * jchunk, j1 = min(ncols, j0 + jchunk);
  Fq3CAcc acc[R][V];
#pragma unroll
  for (int r = 0; r < R; r++)
#pragma unroll
    for (int v = 0; v < V; v++) {
      gl::cacc_zero(acc[r][v].s00);
      gl::cacc_zero(acc[r][v].s0n);
      gl::cacc_zero(acc[r][v].s1);
      gl::cacc_zero(acc[r][v].s1n);
      gl::cacc_zero(acc[r][v].s2);
    }
  for (size_t j = j0 + ph; j < j1; j += 8) {
    uint64_t a[R][3], b[V][3];
#pragma unroll
    for (int r = 0; r < R; r++) {
      const uint64_t *p = A + ((size_t)min(i0 + r, (int)kappa - 1) * ncols + j) * 24 + 3 * slot;
      a[r][0] = p[0];
      a[r][1] = p[1];
      a[r][2] = p[2];
    }
#pragma unroll
    for (int v = 0; v < V; v++) {
      const uint64_t *p = fv.p[min(v0 + v, nvec - 1)] + j * 24 + 3 * slot;
      b[v][0] = p[0];
      b[v][1] = p[1];
      b[v][2] = p[2];
    }
#pragma unroll
    for (int r = 0; r < R; r++)
#pragma unroll
      for (int v = 0; v < V; v++) {
        Fq3CAcc &q = acc[r][v];
        gl::cacc_mad(q.s00, a[r][0], b[v][0]);
        gl::cacc_mad(q.s0n, a[r][1], b[v][2]);
        gl::cacc_mad(q.s0n, a[r][2], b[v][1]);
        gl::cacc_mad(q.s1, a[r][0], b[v][1]);
        gl::cacc_mad(q.s1, a[r][1], b[v][0]);
        gl::cacc_mad(q.s1n, a[r][2], b[v][2]);
        gl::cacc_mad(q.s2, a[r][0], b[v][2]);
        gl::cacc_mad(q.s2, a[r][1], b[v][1]);
        gl::cacc_mad(q.s2, a[r][2], b[v][0]);
      }
  }
  // c0 = s00 + 2^40 s0n, c1 = s1 + 2^40 s1n, c2 = s2; then sum the 8 column phases
#pragma unroll
  for (int r = 0; r < R; r++)
#pragma unroll
    for (int v = 0; v < V; v++) {
      const Fq3CAcc &q = acc[r][v];
      uint64_t c[3];
      c[0] = gl::add(gl::cacc_reduce(q.s00), gl::mul_pow2(gl::cacc_reduce(q.s0n), 40));
      c[1] = gl::add(gl::cacc_reduce(q.s1), gl::mul_pow2(gl::cacc_reduce(q.s1n), 40));
      c[2] = gl::cacc_reduce(q.s2);
#pragma unroll
      for (int off = 8; off < 64; off <<= 1)
#pragma unroll
        for (int k = 0; k < 3; k++) c[k] = gl::add(c[k], __shfl_xor(c[k], off));
      if (ph == 0 && i0 + r < (int)kappa && v0 + v < nvec) {  // empty splits write zeros
        uint64_t *o = partial + (((size_t)js * nvec + v0 + v) * kappa + i0 + r) * 24 + 3 * slot;
        o[0] = c[0];
        o[1] = c[1];
        o[2] = c[2];
      }
    }
}

// sum nsplit partial planes of len u64 each (mod p)
__global__ void k_sum_planes(const uint64_t *partial, int nsplit, size_t len, uint64_t *out,
                             size_t out_stride_vec, size_t per_vec) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i >= len) return;
  Acc a;
  gl::acc_zero(a);
  for (int s = 0; s < nsplit; s++) gl::acc_add(a, partial[(size_t)s * len + i]);
  size_t v = i / per_vec, r = i % per_vec;
  out[v * out_stride_vec + r] = gl::acc_reduce(a);
}

// 64 outputs x 4 split groups per block: wave g sums splits g, g + 4, ... of
// its 64 outputs (coalesced), and the 4 partial sums meet in LDS
__global__ void __launch_bounds__(256) k_sum_planes_to(const uint64_t *partial, int nsplit, size_t len, int nvec,
                                                      OutPtrs out) {
  __shared__ uint64_t part[3][64];
  const int o = threadIdx.x & 63, g = threadIdx.x >> 6;
  const size_t i = blockIdx.x * (size_t)64 + o;
  const bool ok = i < len * nvec;
  Acc a;
  gl::acc_zero(a);
  if (ok)
    for (int s = g; s < nsplit; s += 4) gl::acc_add(a, partial[(size_t)s * len * nvec + i]);
  const uint64_t v = gl::acc_reduce(a);
  if (g > 0) part[g - 1][o] = v;
  __syncthreads();
  if (g == 0 && ok) out.p[i / len][i % len] = gl::add(gl::add(v, part[0][o]), gl::add(part[1][o], part[2][o]));
}

// ============================================================ commit_witnesses y_0
// LF/nifs/decomposition.rs:183-200: y_0 = cm - sum_{k>=1} b^k y_k (scalar b)
__global__ void k_commit_y0(const uint64_t *cm, uint64_t *y, size_t n, int lbs, int K) {
  size_t c = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (c >= n) return;
  uint64_t acc = 0;
  for (int k = K - 1; k >= 1; k--) acc = gl::mul_pow2(gl::add(acc, y[(size_t)k * n + c]), lbs);
  y[c] = gl::sub(cm[c], acc);
}

// both sides' y_0 and the folded commitment in one pass (see kernels.hpp y0_cm0)
// one thread per commitment slot; K <= Y0_KMAX: every plane's y and rho of a side
// are loaded before the Horner chain, so the 2 (K - 1) loads of a thread are in
// flight together instead of one latency per plane (W = 464: 18.6 us per launch
// with the loads inside the chain)
constexpr int Y0_KMAX = 16;
__global__ void k_y0_cm0(const uint64_t *cm0s, const uint64_t *cm1s, uint64_t *y0, uint64_t *y1,
                         const uint64_t *rho, size_t n, int d, int lbs, int K, uint64_t *cm0) {
  const size_t c = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (c >= n) return;
  const int s = c % d;
  gl::CAcc a;
  gl::cacc_zero(a);
#pragma unroll
  for (int side = 0; side < 2; side++) {
    uint64_t *y = side ? y1 : y0;
    const uint64_t *rs = rho + (size_t)side * K * d + s;
    uint64_t yv[Y0_KMAX], rv[Y0_KMAX];
#pragma unroll
    for (int k = 1; k < Y0_KMAX; k++)
      if (k < K) {
        yv[k] = y[(size_t)k * n + c];
        rv[k] = rs[(size_t)k * d];
      }
    uint64_t acc = 0;
#pragma unroll
    for (int k = Y0_KMAX - 1; k >= 1; k--)
      if (k < K) {
        gl::cacc_mad(a, rv[k], yv[k]);
        acc = gl::mul_pow2(gl::add(acc, yv[k]), lbs);
      }
    const uint64_t v0 = gl::sub((side ? cm1s : cm0s)[c], acc);
    y[c] = v0;
    gl::cacc_mad(a, rs[0], v0);
  }
  cm0[c] = gl::cacc_reduce(a);
}

// Phi_72: 16 slots x 16 k-lanes per block. Lane q of slot u takes the planes
// k = q, q + 16, ... (k >= 1) of both sides: y_k 2^(k lbs) (the Horner sum of
// y_0, unrolled) and rho_k (.) y_k (the Fq3 slot product of the fold); the
// lanes' sums meet in LDS, and lane 0 forms y_0 = cm - sum and adds rho_0 (.) y_0
__global__ void __launch_bounds__(256) k_y0_cm0_phi72(const uint64_t *cm0s, const uint64_t *cm1s, uint64_t *y0,
                                                     uint64_t *y1, const uint64_t *rho, size_t nslots, int lbs,
                                                     int K, uint64_t *cm0) {
  __shared__ uint64_t part[16][16][9];
  const int q = threadIdx.x & 15, ul = threadIdx.x >> 4;
  const size_t u = blockIdx.x * (size_t)16 + ul;
  const bool ok = u < nslots;
  const size_t n = nslots * 3;
  const int s = u % 8;
  ring::Fq3Acc a;
  ring::fq3acc_zero(a);
  uint64_t hs[2][3] = {{0, 0, 0}, {0, 0, 0}};
  if (ok)
    for (int side = 0; side < 2; side++) {
      const uint64_t *y = side ? y1 : y0;
      for (int k = q > 0 ? q : 16; k < K; k += 16) {
        const uint64_t *v = y + (size_t)k * n + 3 * u, *r = rho + ((size_t)side * K + k) * 24 + 3 * s;
        ring::fq3acc_mad(a, r[0], r[1], r[2], v[0], v[1], v[2]);
        const int e = (int)(((long long)k * lbs) % 192);
#pragma unroll
        for (int c = 0; c < 3; c++) hs[side][c] = gl::add(hs[side][c], gl::mul_pow2(v[c], e));
      }
    }
  uint64_t cc[3];
  ring::fq3acc_final(a, cc);
#pragma unroll
  for (int c = 0; c < 3; c++) {
    part[ul][q][c] = cc[c];
    part[ul][q][3 + c] = hs[0][c];
    part[ul][q][6 + c] = hs[1][c];
  }
  __syncthreads();
  if (q != 0 || !ok) return;
  uint64_t t[9];
#pragma unroll
  for (int c = 0; c < 9; c++) t[c] = part[ul][0][c];
  for (int l = 1; l < 16; l++)
#pragma unroll
    for (int c = 0; c < 9; c++) t[c] = gl::add(t[c], part[ul][l][c]);
  ring::Fq3Acc a0;
  ring::fq3acc_zero(a0);
  for (int side = 0; side < 2; side++) {
    uint64_t *y = side ? y1 : y0;
    const uint64_t *cm = (side ? cm1s : cm0s) + 3 * u, *r = rho + (size_t)side * K * 24 + 3 * s;
    uint64_t v0[3];
#pragma unroll
    for (int c = 0; c < 3; c++) {
      v0[c] = gl::sub(cm[c], t[3 + 3 * side + c]);
      y[3 * u + c] = v0[c];
    }
    ring::fq3acc_mad(a0, r[0], r[1], r[2], v0[0], v0[1], v0[2]);
  }
  ring::fq3acc_final(a0, cc);
#pragma unroll
  for (int c = 0; c < 3; c++) cm0[3 * u + c] = gl::add(cc[c], t[c]);
}

// ============================================================ linear fold
// LF/nifs/folding.rs:258-268 (f_0) and folding/utils.rs:470-476 (cm_0):
//   out[j] = sum_i rho_i (.) x_i[j]
// two adjacent slots per thread (16-B streaming loads; d is even)
// run_if: when given, nothing to do unless *run_if != 0 (the fallback of the
// coefficient-form fold, fold_coeff.hip; its launch is then grid-capped and strides)
__global__ void __launch_bounds__(256) k_fold_nega(const uint64_t *rho, VecPtrs x, int nwit, size_t n,
                                                  int d, uint64_t *out, const int *run_if) {
  if (run_if && !*run_if) return;
  for (size_t c = 2 * (blockIdx.x * (size_t)blockDim.x + threadIdx.x); c < n * (size_t)d;
       c += 2 * (size_t)gridDim.x * blockDim.x) {
  const int s = c % d;
  gl::CAcc a0, a1;
  gl::cacc_zero(a0);
  gl::cacc_zero(a1);
  typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
  // witnesses in batches of FB: the batch's loads are all in flight before its MACs
  constexpr int FB = 6;
  int i = 0;
  for (; i + FB <= nwit; i += FB) {
    u64x2 v[FB];
#pragma unroll
    for (int q = 0; q < FB; q++) v[q] = __builtin_nontemporal_load(reinterpret_cast<const u64x2 *>(x.p[i + q] + c));
#pragma unroll
    for (int q = 0; q < FB; q++) {
      const ulonglong2 r = *reinterpret_cast<const ulonglong2 *>(rho + (i + q) * d + s);
      gl::cacc_mad(a0, r.x, v[q].x);
      gl::cacc_mad(a1, r.y, v[q].y);
    }
  }
  for (; i < nwit; i++) {
    const u64x2 v = __builtin_nontemporal_load(reinterpret_cast<const u64x2 *>(x.p[i] + c));
    const ulonglong2 r = *reinterpret_cast<const ulonglong2 *>(rho + i * d + s);
    gl::cacc_mad(a0, r.x, v.x);
    gl::cacc_mad(a1, r.y, v.y);
  }
  *reinterpret_cast<ulonglong2 *>(out + c) = make_ulonglong2(gl::cacc_reduce(a0), gl::cacc_reduce(a1));
  }
}
__global__ void __launch_bounds__(256) k_fold_phi72(const uint64_t *rho, VecPtrs x, int nwit, size_t n,
                                                   uint64_t *out, const int *run_if) {
  if (run_if && !*run_if) return;  // uniform: the coefficient-form fold produced f_0
  for (size_t u = blockIdx.x * (size_t)blockDim.x + threadIdx.x; u < n * 8; u += (size_t)gridDim.x * blockDim.x) {
  const int s = u % 8;  // Fq3 slot index u
  ring::Fq3Acc a;
  ring::fq3acc_zero(a);
  for (int i = 0; i < nwit; i++) {
    const uint64_t *r = rho + i * 24 + 3 * s, *p = x.p[i] + 3 * u;
    ring::fq3acc_mad(a, r[0], r[1], r[2], p[0], p[1], p[2]);
  }
  uint64_t c[3];
  ring::fq3acc_final(a, c);
  out[3 * u] = c[0];
  out[3 * u + 1] = c[1];
  out[3 * u + 2] = c[2];
  }
}

static inline unsigned blocks(size_t n, int t) { return (unsigned)((n + t - 1) / t); }
static inline unsigned grid_cap(size_t n) { return (unsigned)(n < 65536 ? n : 65536); }

// ============================================================ Phi_72 fold in coefficient form
// The 2K folded witnesses are digit planes, f_i = CRT(D_i) with D_i in {-1, 0, 1}^24,
// and get_rhos' challenges are short (coefficients in [-32, 31],
// rings/goldilocks.rs:41-67). CRT is a ring isomorphism, so f_0 = CRT(f0_coeff)
// with f0_coeff = sum_i rho_i * D_i, the product in Z[X]/(X^24 - X^12 + 1) of
// small integers. Before the reduction every coefficient of the degree-46 sum is
// at most 2K 24 32 = 23 040 in magnitude, so it runs on packed 16-bit lanes
// (v_pk_mad_i16: two coefficients per instruction). It replaces reading the 2K
// NTT-form planes (30 x 192 B per element) with 30 x 8 B of digit masks, and
// Witness::from_f's ICRT with a CRT.
constexpr int RHO24_BOUND = 32;
constexpr int RHO24_WORDS = 25;  // per witness: 12 pairs (rho_2b, rho_2b+1), 13 pairs (rho_2b-1, rho_2b)
typedef short s16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pack16(int lo, int hi) { return (uint32_t)(uint16_t)lo | ((uint32_t)(uint16_t)hi << 16); }
__global__ void k_rho_phi72(const uint64_t *rho, int nw, uint32_t *rc, int *bad) {
  const int i = threadIdx.x;  // one block of >= nw threads: it also clears / sets the flag
  bool out = false;
  if (i < nw) {
  uint64_t c[24];
#pragma unroll
  for (int t = 0; t < 24; t++) c[t] = rho[(size_t)i * 24 + t];
  ring::phi72_icrt(c);
  int v[26];
  v[0] = v[25] = 0;  // rho_-1, rho_24
#pragma unroll
  for (int t = 0; t < 24; t++) {
    const int64_t x = signed_rep(c[t]);
    out |= x > RHO24_BOUND || x < -RHO24_BOUND;
    v[t + 1] = (int)(x > RHO24_BOUND ? 0 : x < -RHO24_BOUND ? 0 : x);
  }
#pragma unroll
  for (int b = 0; b < 12; b++) rc[i * RHO24_WORDS + b] = pack16(v[2 * b + 1], v[2 * b + 2]);
#pragma unroll
  for (int b = 0; b < 13; b++) rc[i * RHO24_WORDS + 12 + b] = pack16(v[2 * b], v[2 * b + 1]);
  }
  out = __syncthreads_or(out);
  if (i == 0) *bad = out ? 1 : 0;
}

// one thread per element (blocks of whole groups, G = blockDim / L); the f0
// elements meet in LDS for w_ccs0 = sum_l B^l f0[gL + l], as in k_from_f_phi72.
// acc2[q] holds coefficients (2q, 2q + 1) of the degree-46 sum: digit j = 2a
// adds dg (rho_2b, rho_2b+1) to acc2[a + b], digit j = 2a + 1 adds
// dg (rho_2b-1, rho_2b) to acc2[a + b]
__global__ void __launch_bounds__(256) k_fold_coeff_phi72(const uint2 *masks0, const uint2 *masks1,
                                                          const uint32_t *rc, const int *bad, size_t N, int K, int L,
                                                          int lb, uint64_t *f0_coeff, uint64_t *f0,
                                                          uint64_t *w_ccs0) {
  if (*bad) return;  // uniform: a challenge is not short, the NTT-form fold runs instead
  extern __shared__ uint64_t lds[];  // [G L][24] f0 elements, then the 2K x 25 packed rho words
  // PW_SPLIT lanes per element (consecutive, one quad): lane h takes witnesses
  // h, h + PW_SPLIT, ..; their partial sums meet by two xor-shuffles
  constexpr int PW_SPLIT = 4;
  const int G = blockDim.x / (PW_SPLIT * L), t = threadIdx.x, nw = 2 * K, h = t & (PW_SPLIT - 1);
  uint32_t *rl = reinterpret_cast<uint32_t *>(lds + (size_t)G * L * 24);
  for (int q = t; q < nw * RHO24_WORDS; q += blockDim.x) rl[q] = rc[q];
  __syncthreads();
  const size_t W = N / L, j0 = (size_t)blockIdx.x * G;
  const int el = t / PW_SPLIT;  // element within the block
  const size_t e = j0 * L + el;
  const bool live = el < G * L && e < N;
  {
    s16x2 acc2[24];
#pragma unroll
    for (int q = 0; q < 24; q++) acc2[q] = (s16x2){0, 0};
    // the next witness's masks load while this one's products run
    auto mask_of = [&](int i) {
      return live ? (i < K ? masks0 : masks1)[(size_t)(i < K ? i : i - K) * N + e] : make_uint2(0u, 0u);
    };
    uint2 mn = mask_of(h);
    for (int i = h; i < nw; i += PW_SPLIT) {
      const uint2 m = mn;
      if (i + PW_SPLIT < nw) mn = mask_of(i + PW_SPLIT);
      s16x2 r[RHO24_WORDS];
#pragma unroll
      for (int u = 0; u < RHO24_WORDS; u++) r[u] = __builtin_bit_cast(s16x2, rl[i * RHO24_WORDS + u]);
#pragma unroll
      for (int jj = 0; jj < 24; jj++) {
        const short dv = (m.x >> jj & 1) ? ((m.y >> jj & 1) ? (short)-1 : (short)1) : (short)0;
        const s16x2 dg = {dv, dv};
        const int a = jj >> 1;
        if ((jj & 1) == 0) {
#pragma unroll
          for (int b2 = 0; b2 < 12; b2++) acc2[a + b2] += dg * r[b2];
        } else {
#pragma unroll
          for (int b2 = 0; b2 < 13; b2++)
            if (a + b2 < 24) acc2[a + b2] += dg * r[12 + b2];
        }
      }
    }
    // sum over the quad (exact in 16 bits: the total is the one bounded above)
#pragma unroll
    for (int q = 0; q < 24; q++) {
      uint32_t v = __builtin_bit_cast(uint32_t, acc2[q]);
      v = __builtin_bit_cast(uint32_t, acc2[q] + __builtin_bit_cast(s16x2, (uint32_t)__shfl_xor((int)v, 1)));
      acc2[q] = __builtin_bit_cast(s16x2, v) + __builtin_bit_cast(s16x2, (uint32_t)__shfl_xor((int)v, 2));
    }
    if (live && h == 0) {
    int32_t acc[48];
#pragma unroll
    for (int q = 0; q < 24; q++) {
      acc[2 * q] = acc2[q].x;
      acc[2 * q + 1] = acc2[q].y;
    }
    // X^24 = X^12 - 1:  X^s = X^(s-12) - X^(s-24) for 24 <= s < 36, X^s = -X^(s-36) for s >= 36
#pragma unroll
    for (int s2 = 46; s2 >= 36; s2--) acc[s2 - 36] -= acc[s2];
#pragma unroll
    for (int s2 = 35; s2 >= 24; s2--) {
      acc[s2 - 12] += acc[s2];
      acc[s2 - 24] -= acc[s2];
    }
    uint64_t c[24];
#pragma unroll
    for (int u = 0; u < 24; u++) c[u] = from_signed(acc[u]);
    ulonglong2 *dc = reinterpret_cast<ulonglong2 *>(f0_coeff + e * 24);
#pragma unroll
    for (int u = 0; u < 12; u++) dc[u] = make_ulonglong2(c[2 * u], c[2 * u + 1]);
    ring::phi72_crt(c);
    ulonglong2 *df = reinterpret_cast<ulonglong2 *>(f0 + e * 24);
#pragma unroll
    for (int u = 0; u < 12; u++) df[u] = make_ulonglong2(c[2 * u], c[2 * u + 1]);
#pragma unroll
    for (int u = 0; u < 24; u++) lds[el * 24 + u] = c[u];
    }
  }
  __syncthreads();
  const size_t ng = W - j0 < (size_t)G ? W - j0 : (size_t)G;
  for (int o = t; o < (int)ng * 24; o += blockDim.x) {
    const int g = o / 24, i = o - g * 24;
    const uint64_t *row = lds + g * L * 24 + i;
    uint64_t acc = row[(L - 1) * 24];
    for (int l = L - 2; l >= 0; l--) acc = gl::add(gl::mul_pow2(acc, lb), row[l * 24]);
    w_ccs0[j0 * 24 + o] = acc;
  }
}

hipError_t fold_phi72_rho(const uint64_t *rho, int nw, uint32_t *rc, int *bad, hipStream_t st) {
  if (nw < 1 || nw > 64) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_rho_phi72, dim3(1), dim3(64), 0, st, rho, nw, rc, bad);
  return hipGetLastError();
}

hipError_t fold_phi72_coeff(const uint2 *masks0, const uint2 *masks1, const uint32_t *rc, const int *bad, size_t N,
                            int K, int L, int lb, uint64_t *f0_coeff, uint64_t *f0, uint64_t *w_ccs0, hipStream_t st) {
  const size_t W = N / L;
  if (W == 0) return hipSuccess;
  if (L < 1 || L > 64 || K < 1 || 2 * K > 64) return hipErrorInvalidValue;
  const int G = 256 / (4 * L);  // 4 lanes per element (k_fold_coeff_phi72's PW_SPLIT)
  if (G < 1) return hipErrorInvalidValue;
  const size_t lds = (size_t)G * L * 24 * 8 + (size_t)2 * K * RHO24_WORDS * 4;
  hipLaunchKernelGGL(k_fold_coeff_phi72, dim3((unsigned)((W + G - 1) / G)), dim3(4 * G * L), lds, st, masks0, masks1,
                     rc, bad, N, K, L, lb, f0_coeff, f0, w_ccs0);
  return hipGetLastError();
}

// f_0 from the digit masks for any rho (the fallback of k_fold_coeff_phi72 when
// the planes are kept packed, lf_fold_step_bufs.fk == NULL): the same ring
// product in coefficient form, f0_coeff = sum_i ICRT(rho_i) * D_i mod p, one
// thread per element, then f_0 = CRT(f0_coeff). Every block takes the 2K
// inverse transforms of rho (and their negatives) into LDS itself.
__global__ void __launch_bounds__(256) k_fold_phi72_masks(const uint2 *masks0, const uint2 *masks1, const uint64_t *rho,
                                                          int K, size_t N, uint64_t *f0, const int *run_if) {
  if (run_if && !*run_if) return;  // uniform: the short-challenge fold produced f_0
  __shared__ uint64_t rc[2][64 * 24];  // [sign][witness][coefficient]
  const int nw = 2 * K;
  for (int i = threadIdx.x; i < nw; i += blockDim.x) {
    uint64_t c[24];
#pragma unroll
    for (int t = 0; t < 24; t++) c[t] = rho[(size_t)i * 24 + t];
    ring::phi72_icrt(c);
#pragma unroll
    for (int t = 0; t < 24; t++) {
      rc[0][i * 24 + t] = c[t];
      rc[1][i * 24 + t] = gl::sub(0, c[t]);
    }
  }
  __syncthreads();
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < N; e += (size_t)gridDim.x * blockDim.x) {
    uint64_t acc[47];
#pragma unroll
    for (int t = 0; t < 47; t++) acc[t] = 0;
    for (int i = 0; i < nw; i++) {
      const uint2 m = (i < K ? masks0 : masks1)[(size_t)(i < K ? i : i - K) * N + e];
#pragma unroll
      for (int j = 0; j < 24; j++) {
        if (!(m.x >> j & 1)) continue;
        const uint64_t *r = rc[m.y >> j & 1] + i * 24;
#pragma unroll
        for (int t = 0; t < 24; t++) acc[j + t] = gl::add(acc[j + t], r[t]);
      }
    }
    // X^24 = X^12 - 1 (as in k_fold_coeff_phi72)
#pragma unroll
    for (int s2 = 46; s2 >= 36; s2--) acc[s2 - 36] = gl::sub(acc[s2 - 36], acc[s2]);
#pragma unroll
    for (int s2 = 35; s2 >= 24; s2--) {
      acc[s2 - 12] = gl::add(acc[s2 - 12], acc[s2]);
      acc[s2 - 24] = gl::sub(acc[s2 - 24], acc[s2]);
    }
    ring::phi72_crt(acc);
    ulonglong2 *df = reinterpret_cast<ulonglong2 *>(f0 + e * 24);
#pragma unroll
    for (int u = 0; u < 12; u++) df[u] = make_ulonglong2(acc[2 * u], acc[2 * u + 1]);
  }
}

hipError_t fold_phi72_masks(const uint2 *masks0, const uint2 *masks1, const uint64_t *rho, int K, size_t N,
                            uint64_t *f0, const int *run_if, hipStream_t st) {
  if (N == 0) return hipSuccess;
  if (K < 1 || 2 * K > 64) return hipErrorInvalidValue;
  unsigned nb = blocks(N, 256);
  if (run_if && nb > 1024) nb = 1024;  // usually returns at once
  hipLaunchKernelGGL(k_fold_phi72_masks, dim3(nb), dim3(256), 0, st, masks0, masks1, rho, K, N, f0, run_if);
  return hipGetLastError();
}

// packed Phi_72 digit planes (one u64 per element: bit i of the low word =
// coefficient i is nonzero, of the high word = it is negative) -> the u64
// witness forms f_coeff (the digits mod p) and f = CRT(f_coeff); either may be null
__global__ void __launch_bounds__(256) k_expand_phi72(const uint2 *planes, size_t n, uint64_t *fc, uint64_t *f) {
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n; e += (size_t)gridDim.x * blockDim.x) {
    const uint2 m = planes[e];
    uint64_t c[24];
#pragma unroll
    for (int i = 0; i < 24; i++) c[i] = pw_digit(m.x, m.y, i);
    if (fc) {
      ulonglong2 *o = reinterpret_cast<ulonglong2 *>(fc + e * 24);
#pragma unroll
      for (int u = 0; u < 12; u++) o[u] = make_ulonglong2(c[2 * u], c[2 * u + 1]);
    }
    if (f) {
      ring::phi72_crt(c);
      ulonglong2 *o = reinterpret_cast<ulonglong2 *>(f + e * 24);
#pragma unroll
      for (int u = 0; u < 12; u++) o[u] = make_ulonglong2(c[2 * u], c[2 * u + 1]);
    }
  }
}

hipError_t expand_phi72(const uint2 *planes, size_t n, uint64_t *fc, uint64_t *f, hipStream_t st) {
  if (n == 0 || (!fc && !f)) return hipSuccess;
  hipLaunchKernelGGL(k_expand_phi72, dim3(grid_cap(blocks(n, 256))), dim3(256), 0, st, planes, n, fc, f);
  return hipGetLastError();
}

// ============================================================ Poseidon2-16
// zkvm/src/poseidon2.rs:100-173 (+ Plonky3 add_rc_and_sbox_generic, matmul_internal)
#include "p2_consts.inc"
__constant__ uint64_t P2_EXT_INIT[64] = LF_P2_EXT_INIT;
__constant__ uint64_t P2_EXT_TERM[64] = LF_P2_EXT_TERM;
__constant__ uint64_t P2_INTERNAL[22] = LF_P2_INTERNAL;
__constant__ uint64_t P2_DIAG_M1[16] = LF_P2_DIAG_M1;

__device__ __forceinline__ uint64_t sbox7(uint64_t x) {
  uint64_t x2 = gl::mul(x, x), x4 = gl::mul(x2, x2);
  return gl::mul(gl::mul(x4, x2), x);
}
__device__ __forceinline__ void mds16(uint64_t *s) {  // poseidon2.rs:243-268
#pragma unroll
  for (int c = 0; c < 16; c += 4) {
    uint64_t x0 = s[c], x1 = s[c + 1], x2 = s[c + 2], x3 = s[c + 3];
    uint64_t t = gl::add(gl::add(x0, x1), gl::add(x2, x3));
    s[c] = gl::add(t, gl::add(x0, gl::add(x1, x1)));
    s[c + 1] = gl::add(t, gl::add(x1, gl::add(x2, x2)));
    s[c + 2] = gl::add(t, gl::add(x2, gl::add(x3, x3)));
    s[c + 3] = gl::add(t, gl::add(x3, gl::add(x0, x0)));
  }
#pragma unroll
  for (int k = 0; k < 4; k++) {
    uint64_t sum = gl::add(gl::add(s[k], s[4 + k]), gl::add(s[8 + k], s[12 + k]));
#pragma unroll
    for (int j = k; j < 16; j += 4) s[j] = gl::add(s[j], sum);
  }
}
// rounds < 30 stops after the initial MDS and that many rounds (a debug entry
// that lets the reference's round-0 vector, sages/inverse_mds.sage, pin the device)
__global__ void __launch_bounds__(256) k_p2_permute(uint64_t *states, size_t n, int rounds) {
  size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (e >= n) return;
  uint64_t s[16];
  const ulonglong2 *src = reinterpret_cast<const ulonglong2 *>(states + e * 16);
#pragma unroll
  for (int i = 0; i < 8; i++) {
    ulonglong2 v = src[i];
    s[2 * i] = gl::canon(v.x);
    s[2 * i + 1] = gl::canon(v.y);
  }
  mds16(s);
  const int ri = rounds < 4 ? rounds : 4, rp = rounds - 4 < 0 ? 0 : rounds - 4 > 22 ? 22 : rounds - 4;
  const int rt = rounds - 26 < 0 ? 0 : rounds - 26 > 4 ? 4 : rounds - 26;
#pragma unroll 1
  for (int r = 0; r < ri; r++) {
#pragma unroll
    for (int i = 0; i < 16; i++) s[i] = sbox7(gl::add(s[i], P2_EXT_INIT[16 * r + i]));
    mds16(s);
  }
#pragma unroll 1
  for (int r = 0; r < rp; r++) {
    s[0] = sbox7(gl::add(s[0], P2_INTERNAL[r]));
    uint64_t sum = 0;
#pragma unroll
    for (int i = 0; i < 16; i++) sum = gl::add(sum, s[i]);
#pragma unroll
    for (int i = 0; i < 16; i++) s[i] = gl::add(gl::mul(s[i], P2_DIAG_M1[i]), sum);
  }
#pragma unroll 1
  for (int r = 0; r < rt; r++) {
#pragma unroll
    for (int i = 0; i < 16; i++) s[i] = sbox7(gl::add(s[i], P2_EXT_TERM[16 * r + i]));
    mds16(s);
  }
  ulonglong2 *dst = reinterpret_cast<ulonglong2 *>(states + e * 16);
#pragma unroll
  for (int i = 0; i < 8; i++) dst[i] = make_ulonglong2(s[2 * i], s[2 * i + 1]);
}

// ============================================================ synthetic inputs / reductions
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
// element i = SplitMix64(counter i) re-mixed until < p (oracle lfo_fill_uniform)
__global__ void k_fill_uniform(uint64_t *out, size_t n, uint64_t seed) {
  const uint64_t G = 0x9e3779b97f4a7c15ull;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint64_t x = mix64(seed + (uint64_t)(i + 1) * G);
    while (x >= gl::P) x = mix64(x + G);
    out[i] = x;
  }
}
// out[c] = sum_r in[r*len + c] mod p  (cross-rank accumulator reduce)
__global__ void k_modp_sum(const uint64_t *in, int nparts, size_t len, uint64_t *out) {
  size_t c = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (c >= len) return;
  Acc a;
  gl::acc_zero(a);
  for (int r = 0; r < nparts; r++) gl::acc_add(a, gl::canon(in[(size_t)r * len + c]));
  out[c] = gl::acc_reduce(a);
}

// ============================================================ rot_lin_combination
// v_0 of the folded LCCCS (CR/rotation.rs:84-101, rot_sum :45-63):
//   v0[j][c] = sum_i sum_r theta_i[r][c] coeff_j(X^r rho_i)
// theta_i flattened to d base-ring values of comp components (Fq3 for Phi_72).
// coeff_j(X^r a) in closed form: X^d + 1: a_(j-r), or -a_(d+j-r) when r > j;
// Phi_72: the terms a_k X^m, m = k + r < 48, folded back with X^24 = X^12 - 1
// (m in [24, 36): +X^(m-12) - X^(m-24)) and X^36 = -1 (m >= 36: -X^(m-36)).
__device__ __forceinline__ uint64_t rot_coeff(const uint64_t *a, int d, int j, int r) {
  if (d != 24) return j >= r ? a[j - r] : gl::sub(0, a[d + j - r]);
  uint64_t v = j >= r ? a[j - r] : 0;
  if (j >= 12 && r > j - 12) v = gl::add(v, a[j + 12 - r]);
  if (j < 12 && r > j) v = gl::sub(v, a[j + 24 - r]);
  if (j < 12 && r > j + 12) v = gl::sub(v, a[j + 36 - r]);
  return v;
}
// one block per output value (j, c); threads stride over (i, r)
__global__ void __launch_bounds__(256) k_rot_lin(const uint64_t *rho_coeff, const uint64_t *theta, int n, int d,
                                                int comp, uint64_t *v0) {
  __shared__ uint64_t red[256];
  const int j = blockIdx.x / comp, c = blockIdx.x % comp;
  gl::CAcc a;
  gl::cacc_zero(a);
  for (int t = threadIdx.x; t < n * d; t += blockDim.x) {
    const int i = t / d, r = t - i * d;
    gl::cacc_mad(a, gl::canon(theta[((size_t)i * d + r) * comp + c]), rot_coeff(rho_coeff + (size_t)i * d, d, j, r));
  }
  red[threadIdx.x] = gl::cacc_reduce(a);
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) red[threadIdx.x] = gl::add(red[threadIdx.x], red[threadIdx.x + s]);
    __syncthreads();
  }
  if (threadIdx.x == 0) v0[(size_t)j * comp + c] = red[0];
}

// ============================================================ RCCL limb transport
// RCCL sums u64 mod 2^64, not mod p: ship 32-bit limbs (sums of <= 2^8 ranks
// stay < 2^40) and fold the limb sums back into the field afterwards.
__global__ void k_limb_split(const uint64_t *x, size_t n, uint64_t *lo, uint64_t *hi) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t v = x[i];
  lo[i] = v & 0xFFFFFFFFull;
  hi[i] = v >> 32;
}
__global__ void k_limb_join(const uint64_t *lo, const uint64_t *hi, size_t n, uint64_t *out) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t h = hi[i], wl = h << 32, wh = h >> 32;  // h * 2^32 as 128 bits
  uint64_t s = wl + lo[i];
  wh += s < wl ? 1 : 0;
  out[i] = gl::canon(gl::reduce128(s, wh));
}

// ============================================================ launchers

hipError_t transform(uint64_t *data, size_t n, int d, bool fwd, const ring::NegaTables &tb,
                     hipStream_t st) {
  if (n == 0) return hipSuccess;
  if (d == 1024 && tb.mid) return transform_n32(data, n, fwd, tb, st);
  if (d == 24) {
    if (fwd)
      hipLaunchKernelGGL(k_phi72_transform<true>, dim3(blocks(n, 256)), dim3(256), 0, st, data, n);
    else
      hipLaunchKernelGGL(k_phi72_transform<false>, dim3(blocks(n, 256)), dim3(256), 0, st, data, n);
    return hipGetLastError();
  }
#define LF_NEGA_T(DD)                                                                             \
  case DD:                                                                                        \
    if (fwd)                                                                                      \
      hipLaunchKernelGGL((k_nega_transform<DD, true>), dim3(grid_cap(n)), dim3(NT<DD>::T), 0, st, \
                         data, n, tb);                                                            \
    else                                                                                          \
      hipLaunchKernelGGL((k_nega_transform<DD, false>), dim3(grid_cap(n)), dim3(NT<DD>::T), 0,    \
                         st, data, n, tb);                                                        \
    break;
  switch (d) {
    LF_NEGA_T(16)
    LF_NEGA_T(64)
    LF_NEGA_T(256)
    LF_NEGA_T(1024)
    LF_NEGA_T(4096)
    default:
      return hipErrorInvalidValue;
  }
#undef LF_NEGA_T
  return hipGetLastError();
}

hipError_t slot_mul(const uint64_t *a, const uint64_t *b, uint64_t *out, size_t n, int d,
                    hipStream_t st) {
  if (n == 0) return hipSuccess;
  if (d == 24)
    hipLaunchKernelGGL(k_slot_mul_phi72, dim3(blocks(n * 8, 256)), dim3(256), 0, st, a, b, out, n * 8);
  else
    hipLaunchKernelGGL(k_slot_mul_nega, dim3(blocks(n * d, 256)), dim3(256), 0, st, a, b, out, n * d);
  return hipGetLastError();
}

hipError_t mont(uint64_t *x, size_t n, bool to, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_mont, dim3(blocks(n, 256)), dim3(256), 0, st, x, n, to ? 1 : 0);
  return hipGetLastError();
}

hipError_t from_w_ccs(const uint64_t *w_ccs, size_t W, int d, int lb, int L, uint64_t *f_coeff,
                      uint64_t *f, const ring::NegaTables &fwd, const ring::NegaTables &inv, int *err,
                      hipStream_t st, uint32_t *smg) {
  if (W == 0) return hipSuccess;
  if (smg && (d != 1024 || lb > 15 || !fwd.mid || !inv.mid)) return hipErrorInvalidValue;
  if (d == 1024 && fwd.mid && inv.mid) return from_w_ccs_n32(w_ccs, W, lb, L, f_coeff, f, fwd, inv, err, st, smg);
  if (d == 4096 && fwd.tw4 && inv.tw4) return from_w_ccs_n4k(w_ccs, W, lb, L, f_coeff, f, fwd, inv, err, st);
  if (d == 24) {
    hipLaunchKernelGGL(k_from_w_ccs_phi72, dim3(blocks(W * L, 128)), dim3(128), 0, st, w_ccs, W, lb,
                       L, f_coeff, f, err);
    return hipGetLastError();
  }
#define LF_CASE(DD)                                                                                \
  case DD:                                                                                         \
    hipLaunchKernelGGL((k_from_w_ccs_nega<DD>), dim3(grid_cap(W)), dim3(NT<DD>::T), 0, st, w_ccs, W, \
                       lb, L, f_coeff, f, fwd, inv, err);                                          \
    break;
  switch (d) {
    LF_CASE(16) LF_CASE(64) LF_CASE(256) LF_CASE(1024) LF_CASE(4096) default : return hipErrorInvalidValue;
  }
#undef LF_CASE
  return hipGetLastError();
}

hipError_t from_f(const uint64_t *f, size_t N, int d, int lb, int L, uint64_t *f_coeff,
                  uint64_t *w_ccs, const ring::NegaTables &inv, hipStream_t st, const int *run_if) {
  const size_t W = N / L;
  if (W == 0) return hipSuccess;
  if (d == 1024 && inv.mid) return from_f_n32(f, W, lb, L, f_coeff, w_ccs, inv, st, run_if);
  if (d == 24) {
    if (L < 1 || L > 256) return hipErrorInvalidValue;
    const int G = 256 / L;
    hipLaunchKernelGGL(k_from_f_phi72, dim3(blocks(W, G)), dim3(G * L), (size_t)G * L * 24 * 8, st, f,
                       W, lb, L, f_coeff, w_ccs, run_if);
    return hipGetLastError();
  }
  if (run_if) return hipErrorInvalidValue;
  if (d == 4096 && inv.tw4) return from_f_n4k(f, W, lb, L, f_coeff, w_ccs, inv, st);
#define LF_CASE(DD)                                                                              \
  case DD:                                                                                       \
    hipLaunchKernelGGL((k_from_f_nega<DD>), dim3(grid_cap(W)), dim3(NT<DD>::T), 0, st, f, W, lb, L, \
                       f_coeff, w_ccs, inv);                                                     \
    break;
  switch (d) {
    LF_CASE(16) LF_CASE(64) LF_CASE(256) LF_CASE(1024) LF_CASE(4096) default : return hipErrorInvalidValue;
  }
#undef LF_CASE
  return hipGetLastError();
}

hipError_t decompose_phi72_sides(const FusedSides &sd, size_t N, int lb, int L, int lbs, int K, int *err,
                                 uint4 *frag, int nch, hipStream_t st, bool *masks_written, bool *dead_written) {
  const size_t W = N / L;
  if (masks_written) *masks_written = false;
  if (dead_written) *dead_written = false;
  if (W == 0) return hipSuccess;
  if (DEC_GROUPS * L > 256 || sd.nside < 1 || sd.nside > 2) return hipErrorInvalidValue;
  if (frag) {
    if (L > 5) return hipErrorInvalidValue;
    for (int s = 0; s < sd.nside; s++)
      if (sd.row0[s] < 0 || sd.row0[s] + K - 1 > 32) return hipErrorInvalidValue;
  }
  bool packed_sm = K <= 15;  // the wave kernel reads k_pack_sm24's 16-bit words
  for (int s = 0; s < sd.nside; s++) packed_sm &= sd.smg[s] != nullptr;
  if (lbs == 1 && L <= 8 && (L - 1) * lb < 62 && packed_sm) {
    const size_t nblk = (W + 15) / 16, waves = (size_t)sd.nside * nblk * ((K + 3) / 4);
    {
      const size_t np = (size_t)sd.nside * N * 12;
      hipLaunchKernelGGL(k_pack_sm24, dim3((unsigned)((np + 255) / 256)), dim3(256), 0, st, sd, N, K, err);
    }
    // streaming stores for the f_coeff_k, f_k and operand rows (mask 7):
    // nothing in the step re-reads f_coeff_k or f_k (the fold reads the digit
    // masks), and the contraction's one pass over the operand rows does not gain
    // from them sitting in the caches either (W = 19 763, 4 streams: cached 0.65
    // ms per launch, 900 steps/s; mask 3 0.50-0.53 ms; mask 7 0.47-0.49 ms with
    // the contraction 0.385 -> 0.36 ms, 1,133-1,138 -> 1,141-1,150 steps/s)
    int ntm = 7;
    // no f_coeff_k / f_k buffers: the planes stay packed (the masks must be kept)
    bool all = true, none = true;  // every side has its u64 rows / no side has
    for (int s = 0; s < sd.nside; s++) {
      all &= sd.f_k[s] != nullptr && sd.f_coeff_k[s] != nullptr;
      none &= sd.f_k[s] == nullptr && sd.f_coeff_k[s] == nullptr;
    }
    if (!all && !none) return hipErrorInvalidValue;
    if (none) {
      for (int s = 0; s < sd.nside; s++)
        if (!sd.masks[s]) return hipErrorInvalidValue;
      ntm = 12;  // packed only (bit 3), the operand rows still streamed
    }
    const dim3 grid((unsigned)((waves + 3) / 4));
#define LF_PW(M)                                                                                          \
  case M:                                                                                                \
    hipLaunchKernelGGL(k_decompose_phi72_w<M>, grid, dim3(256), 0, st, sd, N, lb, L, K, err, frag, nch, nblk); \
    break;
    switch (ntm) { LF_PW(7) LF_PW(12) default: return hipErrorInvalidValue; }
#undef LF_PW
    if (masks_written) *masks_written = sd.masks[0] != nullptr && (sd.nside < 2 || sd.masks[1] != nullptr);
    if (dead_written) *dead_written = frag && sd.dead;  // the wave-local kernel flags its zero units
    return hipGetLastError();
  }
  const int srow = frag ? DEC_SROW : 28;
  const size_t lds = (size_t)DEC_GROUPS * L * srow * sizeof(uint64_t);
  // with independent planes (b = 2), split them over blockIdx.y until about
  // 1024 blocks run per side: the real zkvm shape (W = 19 763) has only 412
  // element blocks (one plane per block is no faster there: 0.30 against 0.29 ms)
  const unsigned nb = blocks(W, DEC_GROUPS);
  unsigned ys = lbs == 1 ? (1024 + nb - 1) / nb : 1;
  if (ys > (unsigned)K) ys = K;
  if (ys < 1) ys = 1;
  hipLaunchKernelGGL(k_decompose_phi72, dim3(nb, ys, (unsigned)sd.nside), dim3(256), lds, st, sd, N, lb, L, lbs, K,
                     err, frag, nch, srow);
  return hipGetLastError();
}

hipError_t decompose_witness(const uint64_t *f_coeff, size_t N, int d, int lb, int L, int lbs, int K,
                             uint64_t *f_coeff_k, uint64_t *f_k, uint64_t *w_ccs_k,
                             const ring::NegaTables &fwd, int *err, hipStream_t st, uint4 *frag, int nch,
                             int row0) {
  const size_t W = N / L;
  if (W == 0) return hipSuccess;
  if (d == 1024 && fwd.mid && lbs == 1 && K <= 15 && L <= 5)
    return decompose_n32(f_coeff, N, lb, L, K, f_coeff_k, f_k, w_ccs_k, fwd, err, st);
  if (d == 24) {
    FusedSides sd{};
    sd.nside = 1;
    sd.f_coeff[0] = f_coeff;
    sd.f_coeff_k[0] = f_coeff_k;
    sd.f_k[0] = f_k;
    sd.w_ccs_k[0] = w_ccs_k;
    sd.row0[0] = row0;
    return decompose_phi72_sides(sd, N, lb, L, lbs, K, err, frag, nch, st);
  }
  if (L > 8) return hipErrorInvalidValue;
#define LF_CASE(DD)                                                                                  \
  case DD:                                                                                           \
    hipLaunchKernelGGL((k_decompose_nega<DD>), dim3(grid_cap(W)), dim3(NT<DD>::T), 0, st, f_coeff, N, \
                       lb, L, lbs, K, f_coeff_k, f_k, w_ccs_k, fwd, err);                            \
    break;
  switch (d) {
    LF_CASE(16) LF_CASE(64) LF_CASE(256) LF_CASE(1024) LF_CASE(4096) default : return hipErrorInvalidValue;
  }
#undef LF_CASE
  return hipGetLastError();
}

int ajtai_nsplit(size_t ncols, int d, int nvec) {
  if (d == 24) {
    // one wave per column split; ~64 columns per lane phase minimum
    size_t want = (ncols + 511) / 512;
    if (want > 1024) want = 1024;
    return (int)((want + 3) / 4 * 4);
  }
  // enough units to fill 256 CUs: (d/256) slot chunks x (kappa/R) row tiles x nsplit x nvt
  size_t want = (ncols + 127) / 128;
  if (want > 40) want = 40;
  if (want < 1) want = 1;
  return (int)want;
}
size_t ajtai_partial_elems(size_t kappa, size_t ncols, int d, int nvec) {
  size_t nsplit = ajtai_nsplit(ncols, d, nvec);
  return nsplit * (size_t)nvec * kappa * (size_t)d;
}

hipError_t ajtai_commit(const uint64_t *A, size_t kappa, size_t ncols, int d, const VecPtrs &fv,
                        int nvec, uint64_t *partial, uint64_t *cm, hipStream_t st, hipEvent_t ev0,
                        hipEvent_t ev1) {
  if (nvec <= 0 || nvec > LF_MAX_VECS) return hipErrorInvalidValue;
  const int nsplit = ajtai_nsplit(ncols, d, nvec);
  const size_t jchunk = (ncols + nsplit - 1) / nsplit;
  if (ev0) (void)hipEventRecord(ev0, st);
  if (d == 24) {
    constexpr int R = 2, V = 2;
    const int nvt = (nvec + V - 1) / V;
    dim3 grid(nsplit / 4, (unsigned)((kappa + R - 1) / R), nvt);
    hipLaunchKernelGGL((k_ajtai_phi72<R, V>), grid, dim3(256), 0, st, A, kappa, ncols, fv, nvec, jchunk,
                       partial);
  } else if (nvec == 1) {
    constexpr int R = 8, V = 1;
    AjtaiGrid g{(d + 255) / 256, (int)((kappa + R - 1) / R), nsplit, 1};
    hipLaunchKernelGGL((k_ajtai_nega<R, V>), dim3(g.blocks()), dim3(256), 0, st, A, kappa, ncols, d, fv,
                       nvec, jchunk, g, partial);
  } else {
    constexpr int R = 4, V = 4;
    AjtaiGrid g{(d + 255) / 256, (int)((kappa + R - 1) / R), nsplit, (nvec + V - 1) / V};
    hipLaunchKernelGGL((k_ajtai_nega<R, V>), dim3(g.blocks()), dim3(256), 0, st, A, kappa, ncols, d, fv,
                       nvec, jchunk, g, partial);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  if (ev1) (void)hipEventRecord(ev1, st);
  const size_t len = (size_t)nvec * kappa * d;
  hipLaunchKernelGGL(k_sum_planes, dim3(blocks(len, 256)), dim3(256), 0, st, partial, nsplit, len, cm,
                     kappa * (size_t)d, kappa * (size_t)d);
  return hipGetLastError();
}

hipError_t sum_planes(const uint64_t *partial, int nsplit, size_t len, uint64_t *out, hipStream_t st) {
  if (len == 0) return hipSuccess;
  hipLaunchKernelGGL(k_sum_planes, dim3(blocks(len, 256)), dim3(256), 0, st, partial, nsplit, len, out, len, len);
  return hipGetLastError();
}

hipError_t sum_planes_to(const uint64_t *partial, int nsplit, size_t len, int nvec, const OutPtrs &out,
                         hipStream_t st) {
  if (len == 0 || nvec < 1) return hipSuccess;
  hipLaunchKernelGGL(k_sum_planes_to, dim3(blocks(len * nvec, 64)), dim3(256), 0, st, partial, nsplit, len, nvec,
                     out);
  return hipGetLastError();
}

hipError_t y0_cm0(const uint64_t *cm0s, const uint64_t *cm1s, uint64_t *y0, uint64_t *y1, const uint64_t *rho,
                  size_t kappa, int d, int lbs, int K, uint64_t *cm0, hipStream_t st) {
  const size_t n = kappa * (size_t)d;
  if (n == 0) return hipSuccess;
  if (K < 1 || K > Y0_KMAX) return hipErrorInvalidValue;
  if (d == 24) {
    hipLaunchKernelGGL(k_y0_cm0_phi72, dim3(blocks(kappa * 8, 16)), dim3(256), 0, st, cm0s, cm1s, y0, y1, rho,
                       kappa * 8, lbs, K, cm0);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(k_y0_cm0, dim3(blocks(n, 256)), dim3(256), 0, st, cm0s, cm1s, y0, y1, rho, n, d, lbs, K, cm0);
  return hipGetLastError();
}

hipError_t commit_y0(const uint64_t *cm, uint64_t *y, size_t kappa, int d, int lbs, int K,
                     hipStream_t st) {
  size_t n = kappa * (size_t)d;
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_commit_y0, dim3(blocks(n, 256)), dim3(256), 0, st, cm, y, n, lbs, K);
  return hipGetLastError();
}

hipError_t fold(const uint64_t *rho, const VecPtrs &x, int nwit, size_t n, int d, uint64_t *out,
                hipStream_t st, const int *run_if) {
  if (n == 0) return hipSuccess;
  if (nwit <= 0 || nwit > LF_MAX_VECS) return hipErrorInvalidValue;
  if (d == 24) {
    unsigned nb = blocks(n * 8, 256);
    if (run_if && nb > 1024) nb = 1024;  // usually returns at once: do not launch a block per 256 slots
    hipLaunchKernelGGL(k_fold_phi72, dim3(nb), dim3(256), 0, st, rho, x, nwit, n, out, run_if);
  } else {
    unsigned nb = blocks(n * d / 2, 256);
    if (run_if && nb > 8192) nb = 8192;  // usually returns at once: do not launch a block per 512 slots
    hipLaunchKernelGGL(k_fold_nega, dim3(nb), dim3(256), 0, st, rho, x, nwit, n, d, out, run_if);
  }
  return hipGetLastError();
}

hipError_t p2_permute(uint64_t *states, size_t n, hipStream_t st, int rounds) {
  if (n == 0) return hipSuccess;
  if (rounds < 0 || rounds > 30) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_p2_permute, dim3(blocks(n, 256)), dim3(256), 0, st, states, n, rounds);
  return hipGetLastError();
}

hipError_t fill_uniform(uint64_t *out, size_t n, uint64_t seed, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_fill_uniform, dim3(grid_cap(blocks(n, 256))), dim3(256), 0, st, out, n, seed);
  return hipGetLastError();
}

hipError_t modp_sum(const uint64_t *in, int nparts, size_t len, uint64_t *out, hipStream_t st) {
  if (len == 0) return hipSuccess;
  hipLaunchKernelGGL(k_modp_sum, dim3(blocks(len, 256)), dim3(256), 0, st, in, nparts, len, out);
  return hipGetLastError();
}

hipError_t rot_lin(const uint64_t *rho_coeff, const uint64_t *theta, int n, int d, uint64_t *v0, hipStream_t st) {
  if (n < 1 || (d != 24 && (d < 2 || (d & (d - 1))))) return hipErrorInvalidValue;
  const int comp = d == 24 ? 3 : 1;
  hipLaunchKernelGGL(k_rot_lin, dim3((unsigned)(d * comp)), dim3(256), 0, st, rho_coeff, theta, n, d, comp, v0);
  return hipGetLastError();
}

hipError_t limb_split(const uint64_t *x, size_t n, uint64_t *lo, uint64_t *hi, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_limb_split, dim3(blocks(n, 256)), dim3(256), 0, st, x, n, lo, hi);
  return hipGetLastError();
}
hipError_t limb_join(const uint64_t *lo, const uint64_t *hi, size_t n, uint64_t *out, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_limb_join, dim3(blocks(n, 256)), dim3(256), 0, st, lo, hi, n, out);
  return hipGetLastError();
}

}  // namespace lfk
