// mz.hip -- the sparse CCS products of the decomposition and folding provers
// (SURVEY.md 8(f) rank 2): M_j z MLEs (calculate_Mz_mles, mle_helpers.rs:137-146;
// compute_mz_mles, nifs/decomposition.rs:229-256), their zeta-challenged
// combination (calculate_challenged_mz_mle, nifs/folding.rs:208-234) and their
// evaluations at a point (compute_u_s, decomposition.rs:214-227; get_etas,
// folding.rs:247-256; compute_u, linearization/utils.rs:24-29).
//
// The matrices are CSR of ring elements (SparseMatrix rows of (value, col),
// linear_algebra/src/sparse_matrix.rs:18-22). mat_vec_mul (arith/utils.rs:52-65)
// is one thread per (row, NTT slot) summing value (.) z[col] over the row.
// The challenged combination sum_i sum_j zeta_i^(j+1) M_j z_i is linear, so it
// runs as y_j = sum_i zeta_i^(j+1) z_i and one product with the row-merged
// matrix [M_0 | .. | M_(t-1)] (SparseMatrix::hconcat, sparse_matrix.rs:42-70);
// the evaluations MLE(M_j z_i)(r) = sum_x eq(r, x) (M_j z_i)[x] run as
// w_j = M_j^T eq(r) and dot products w_j . z_i -- the same field elements
// without materialising the t x nz MLEs of 2^s ring elements each.
#include "frag.hpp"
#include "kernels.hpp"
#include "slot.hpp"

namespace lfk {

namespace {

constexpr int MT = 256;

// out[task][r] = sum_k val[vidx ? vidx[k] : k] (.) z[col[k]], k in [rp[r], rp[r+1]);
// task = (a, b) = (task % na, task / na) selects rp + A rp_stride (A = sel ? sel[a] : a)
// and z + b z_stride. SC: val holds one scalar per entry (CcsDev::sval), the zkvm's
// matrices (R::one(), from_goldilocks constants: zkvm/src/constraints.rs:127-364).
// NT: streaming stores (outputs larger than the caches; CSR_NT_BYTES)
template <int TB, bool SC, bool NT>
__global__ void __launch_bounds__(MT) k_csr(const uint64_t *rp, size_t rp_stride, int na, const int *sel,
                                           const uint32_t *col, const uint32_t *vidx, const uint64_t *val,
                                           size_t nrows, int d, const uint64_t *z, size_t z_stride, uint64_t *out,
                                           size_t out_stride, int spb) {
  const int slot_l = threadIdx.x % spb, lane_r = threadIdx.x / spb, rpb = MT / spb;
  const int slot = blockIdx.z * spb + slot_l;
  const size_t r = (size_t)blockIdx.x * rpb + lane_r;
  if (r >= nrows) return;
  const int task = blockIdx.y, a = task % na, b = task / na;
  const uint64_t *rpa = rp + (size_t)(sel ? sel[a] : a) * rp_stride;
  const uint64_t *zb = z + b * z_stride + slot * TB;
  SAcc<TB> acc;
  sacc_zero(acc);
  auto term = [&](uint64_t vi, uint32_t c) {
    if (SC)
      sacc_smad(acc, val[vi], s_load<TB>(zb + (size_t)c * d));
    else
      sacc_mad(acc, s_load<TB>(val + vi * d + slot * TB), s_load<TB>(zb + (size_t)c * d));
  };
  uint64_t k = rpa[r];
  const uint64_t e = rpa[r + 1];
  // four entries at a time: their index loads, then their value and z loads, are issued
  // together (long rows -- the row-merged matrix, the transposes -- are load-latency bound)
  for (; k + 4 <= e; k += 4) {
    uint64_t vi[4];
    uint32_t c[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      vi[u] = vidx ? vidx[k + u] : k + u;
      c[u] = col[k + u];
    }
#pragma unroll
    for (int u = 0; u < 4; u++) term(vi[u], c[u]);
  }
  for (; k < e; k++) term(vidx ? vidx[k] : k, col[k]);
  const Sv<TB> v = sacc_final(acc);
  uint64_t *o = out + task * out_stride + r * d + slot * TB;
#pragma unroll
  for (int w = 0; w < TB; w++) out_store<NT>(o + w, v.c[w]);
}

// Two challenged products over the same rows (the folding prover's g1 and g3, one per
// decomposed side): each entry's index and value are read once for both
template <int TB, bool SC>
__global__ void __launch_bounds__(MT) k_csr_pair(const uint64_t *rp, const uint32_t *col, const uint32_t *vidx,
                                                const uint64_t *val, size_t nrows, int d, const uint64_t *z0,
                                                const uint64_t *z1, uint64_t *out0, uint64_t *out1, int spb) {
  const int slot_l = threadIdx.x % spb, lane_r = threadIdx.x / spb, rpb = MT / spb;
  const int slot = blockIdx.z * spb + slot_l;
  const size_t r = (size_t)blockIdx.x * rpb + lane_r;
  if (r >= nrows) return;
  const uint64_t *zb0 = z0 + slot * TB, *zb1 = z1 + slot * TB;
  SAcc<TB> a0, a1;
  sacc_zero(a0);
  sacc_zero(a1);
  auto term = [&](uint64_t vi, uint32_t c) {
    const Sv<TB> y0 = s_load<TB>(zb0 + (size_t)c * d), y1 = s_load<TB>(zb1 + (size_t)c * d);
    if (SC) {
      const uint64_t v = val[vi];
      sacc_smad(a0, v, y0);
      sacc_smad(a1, v, y1);
    } else {
      const Sv<TB> v = s_load<TB>(val + vi * d + slot * TB);
      sacc_mad(a0, v, y0);
      sacc_mad(a1, v, y1);
    }
  };
  uint64_t k = rp[r];
  const uint64_t e = rp[r + 1];
  for (; k + 4 <= e; k += 4) {
    uint64_t vi[4];
    uint32_t c[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      vi[u] = vidx ? vidx[k + u] : k + u;
      c[u] = col[k + u];
    }
#pragma unroll
    for (int u = 0; u < 4; u++) term(vi[u], c[u]);
  }
  for (; k < e; k++) term(vidx ? vidx[k] : k, col[k]);
  s_store(out0 + r * d + slot * TB, sacc_final(a0));
  s_store(out1 + r * d + slot * TB, sacc_final(a1));
}

// pw[j][i] = zeta_i^(j+1), one thread per (j, instance, slot) by square-and-multiply
// (a chain of t dependent products per (instance, slot) was 60 us of latency)
template <int TB>
__global__ void k_zeta_pows(const uint64_t *zeta, int nz, int t, int d, uint64_t *pw) {
  const int ns = d / TB;
  const size_t u = blockIdx.x * (size_t)blockDim.x + threadIdx.x;  // (j nz + instance) ns + slot
  if (u >= (size_t)t * nz * ns) return;
  const int s = (int)(u % ns);
  const size_t ji = u / ns;
  const int zi = (int)(ji % nz);
  unsigned e = (unsigned)(ji / nz) + 1;
  Sv<TB> b = s_load<TB>(zeta + (size_t)zi * d + s * TB), p = s_one<TB>();
  for (; e; e >>= 1) {
    if (e & 1) p = s_mul(p, b);
    if (e > 1) b = s_mul(b, b);
  }
  s_store(pw + ji * d + s * TB, p);
}

// The zeta combination on the matrix cores (d = 24, Fq3 slots): per slot s,
// y_s[j][c] = sum_i P_s[j][i] z_i[c][s] with P = zeta_i^(j+1) in Fq3 = F[u]/(u^3 - 2^40)
// (calculate_challenged_mz_mle, folding.rs:208-234, through its linearity) is the
// product of the M-form matrix A_s[(j, a)][(i, b)] = m_ab(P_s[j][i]) -- m_ab = p_(a-b),
// or 2^40 p_(a-b+3) when a < b, so that c_a = sum_b m_ab z_b is the Fq3 product
// (goldilocks/mod.rs:34-54) -- with B_s[(i, b)][c] = z_i[c][s][b]: (3t x 3nz) by
// (3nz x n) per slot. Both operands go to the D8 signed-byte form (8 digits each,
// frag.hpp) and the 64 digit products run as v_mfma_i32_16x16x64_i8 into the 15
// weights the ajtai contraction's epilogue folds (ajtai_mfma.hip mfma_epilogue):
// |acc_t| <= kcn 64 * 8 * 128^2 = kcn 2^23. Tiles: 16 rows = ZC_J = 5 values of j
// times 3 components (row 15 zero) by 16 columns, K = 3 nz in chunks of 64.
// Operand pieces (one 16-byte piece per lane and digit, 1 KiB per digit):
// lane l holds A[row l & 15][k = 16 (l >> 4) + jj] and B[k = 16 (l >> 4) + jj][col l & 15]
// in byte jj; D register i of lane l is row 4 (l >> 4) + i, column l & 15.
constexpr int ZC_J = 5, ZC_WAVES = 4, ZC_D = 24;

// af[((s nrt + rt) kcn + kc) 8 + digit][lane]: the M-form tiles from pw[j][i][slot] (k_zeta_pows<3>)
__global__ void k_zc_afrag(const uint64_t *pw, int nz, int t, int nrt, int kcn, v4i *af) {
  constexpr int ns = ZC_D / 3;
  const size_t u = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (u >= (size_t)ns * nrt * kcn * 64) return;
  const int l = (int)(u & 63);
  const size_t q = u >> 6;
  const int kc = (int)(q % kcn), rt = (int)(q / kcn % nrt), s = (int)(q / kcn / nrt);
  const int r = l & 15, g = l >> 4, jl = r / 3, a = r - 3 * jl, j = ZC_J * rt + jl;
  uint64_t x[16];
#pragma unroll
  for (int jj = 0; jj < 16; jj++) {
    const int k = 64 * kc + 16 * g + jj, i = k / 3, b = k - 3 * i;
    uint64_t v = 0;
    if (r < 3 * ZC_J && j < t && i < nz) {
      const uint64_t *p = pw + ((size_t)j * nz + i) * ZC_D + s * 3;
      v = a >= b ? p[a - b] : gl::shl96(p[a - b + 3], 40);
    }
    x[jj] = d8(v);
  }
  uint4 pc[8];
  d8_transpose16(x, pc);
#pragma unroll
  for (int dg = 0; dg < 8; dg++) af[(q * 8 + dg) * 64 + l] = *reinterpret_cast<const v4i *>(&pc[dg]);
}

// bf[((ct ns + s) kcn + kc) 8 + digit][lane]: the z operand of column tile ct (16 columns)
__global__ void k_zc_bfrag(const uint64_t *z, int nz, size_t n, int kcn, size_t nct, v4i *bf) {
  constexpr int ns = ZC_D / 3;
  const size_t u = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (u >= nct * ns * kcn * 64) return;
  const int l = (int)(u & 63);
  const size_t q = u >> 6;  // (ct, kc, s): one block of 8 waves reads a column tile's whole rows
  const int s = (int)(q % ns), kc = (int)(q / ns % kcn);
  const size_t ct = q / ns / kcn, c = 16 * ct + (l & 15);
  const int g = l >> 4;
  uint64_t x[16];
#pragma unroll
  for (int jj = 0; jj < 16; jj++) {
    const int k = 64 * kc + 16 * g + jj, i = k / 3, b = k - 3 * i;
    x[jj] = d8(c < n && i < nz ? z[((size_t)i * n + c) * ZC_D + s * 3 + b] : 0);
  }
  uint4 pc[8];
  d8_transpose16(x, pc);
  const size_t o = ((ct * ns + s) * kcn + kc) * 8;
#pragma unroll
  for (int dg = 0; dg < 8; dg++) bf[(o + dg) * 64 + l] = *reinterpret_cast<const v4i *>(&pc[dg]);
}

// the 64 digit products of one K chunk into the 15 weights; FIRST: the chunk that starts
// the sums (each weight's first product, (0, t) or (t - 7, 7), takes a zero accumulator)
template <bool FIRST>
__device__ __forceinline__ void zc_products(const v4i *A, const v4i *B, v4i *acc) {
#pragma unroll
  for (int ka = 0; ka < 8; ka++)
#pragma unroll
    for (int kb = 0; kb < 8; kb++)
      acc[ka + kb] = __builtin_amdgcn_mfma_i32_16x16x64_i8(
          A[ka], B[kb], FIRST && (ka == 0 || kb == 7) ? (v4i){0, 0, 0, 0} : acc[ka + kb], 0, 0, 0);
}

// one wave per (column tile ct, row tile rt), the block's waves on consecutive rt of
// one ct (their z pieces come from the same L1 lines), and the blocks of one ct on one
// XCD (blocks are dealt round-robin over the 8 XCDs: block b runs on XCD b & 7), so a
// column tile's pieces come into one L2 once. Per slot 64 MFMAs per K chunk, the next
// chunk's pieces loaded behind them, and the epilogue into the wave's LDS rows
// [jl][c][24]; then one pass of whole 192-byte (j, c) elements out (16 consecutive
// columns: 3 KiB contiguous per j).
// SK (3 nz < 64, one K chunk with a zero tail: |acc_t| <= 3 nz 8 128^2 < 2^31 / 257): the
// weights pair up in 32 bits first, W_m = acc_2m + 2^8 acc_2m+1, halving the 64-bit work
template <bool SK>
__global__ void __launch_bounds__(64 * ZC_WAVES) k_zcomb_mfma(const v4i *af, const v4i *bf, int t, size_t n, int nrt,
                                                           int kcn, size_t nct, uint64_t *y) {
  constexpr int ns = ZC_D / 3;
  __shared__ uint64_t stg[ZC_WAVES][ZC_J * 16 * ZC_D];
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int nbr = (nrt + ZC_WAVES - 1) / ZC_WAVES;  // blocks per column tile
  const size_t k = blockIdx.x >> 3, ct = (k / nbr) * 8 + (blockIdx.x & 7);
  const int rt = (int)(k % nbr) * ZC_WAVES + w;
  if (ct >= nct || rt >= nrt) return;  // no block-wide synchronisation below
  uint64_t *sg = stg[w];
  v4i A[8], B[8], acc[15];
  auto load = [&](int u) {
    const int s = u / kcn, kc = u - s * kcn;
    const v4i *ap = af + (((size_t)s * nrt + rt) * kcn + kc) * 512 + l;
    const v4i *bp = bf + ((ct * ns + s) * kcn + kc) * 512 + l;
#pragma unroll
    for (int q = 0; q < 8; q++) {
      A[q] = ap[64 * q];
      B[q] = bp[64 * q];
    }
  };
  load(0);
  for (int u = 0; u < ns * kcn; u++) {
    const int s = u / kcn, kc = u - s * kcn;
    if (kc == 0)
      zc_products<true>(A, B, acc);
    else
      zc_products<false>(A, B, acc);
    if (u + 1 < ns * kcn) load(u + 1);
    if (kc < kcn - 1) continue;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      int64_t S[4] = {0, 0, 0, 0};
      if (SK) {
        int32_t W[8];
#pragma unroll
        for (int m = 0; m < 7; m++) W[m] = acc[2 * m][i] + acc[2 * m + 1][i] * 256;
        W[7] = acc[14][i];
#pragma unroll
        for (int q = 0; q < 4; q++) S[q] = (int64_t)W[2 * q] + (int64_t)W[2 * q + 1] * 65536;
      } else {
#pragma unroll
        for (int q = 0; q < 15; q++) S[q >> 2] += (int64_t)acc[q][i] << (8 * (q & 3));
      }
      const uint64_t v = gl::from_x_y32(S[0] - S[2] - S[3], S[1] + S[2]);  // sum_t 2^(8t) acc_t
      const int row = 4 * (l >> 4) + i, jl = row / 3, a = row - 3 * jl;
      if (row < 3 * ZC_J) sg[(jl * 16 + (l & 15)) * ZC_D + s * 3 + a] = v;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const uint4 *sq = reinterpret_cast<const uint4 *>(sg);
  constexpr int PJ = 16 * ZC_D / 2, NQ = ZC_J * PJ / 64;  // 16-byte pieces per j, per lane
  if (ZC_J * (rt + 1) <= t && 16 * (ct + 1) <= n) {  // a whole tile: all reads, then all stores
    uint4 v[NQ];
#pragma unroll
    for (int q = 0; q < NQ; q++) v[q] = sq[64 * q + l];
#pragma unroll
    for (int q = 0; q < NQ; q++) {
      const int x = 64 * q + l, jl = x / PJ;
      reinterpret_cast<uint4 *>(y + ((size_t)(ZC_J * rt + jl) * n + 16 * ct) * ZC_D)[x - jl * PJ] = v[q];
    }
    return;
  }
  const int words = (int)((n - 16 * ct < 16 ? n - 16 * ct : 16) * ZC_D);
  for (int jl = 0; jl < ZC_J; jl++) {
    const int j = ZC_J * rt + jl;
    if (j >= t) break;
    uint64_t *dst = y + ((size_t)j * n + 16 * ct) * ZC_D;
    const uint64_t *src = sg + jl * 16 * ZC_D;
    for (int o = 2 * l; o < words; o += 128)
      *reinterpret_cast<uint4 *>(dst + o) = *reinterpret_cast<const uint4 *>(src + o);
  }
}

// y[j][c] = sum_i pw[j][i] (.) z_i[c]
template <int TB>
__global__ void k_zcomb(const uint64_t *pw, const uint64_t *z, int nz, int t, size_t n, int d, uint64_t *y) {
  const int ns = d / TB;
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;  // (j, c, slot)
  if (i >= (size_t)t * n * ns) return;
  const size_t jc = i / ns;
  const int s = (int)(i - jc * ns);
  const size_t j = jc / n, c = jc - j * n;
  SAcc<TB> acc;
  sacc_zero(acc);
  for (int zi = 0; zi < nz; zi++)
    sacc_mad(acc, s_load<TB>(pw + (j * nz + zi) * d + s * TB), s_load<TB>(z + (zi * n + c) * d + s * TB));
  s_store(y + jc * d + s * TB, sacc_final(acc));
}

// out[i][j] = sum_c w[j][c] (.) z_i[c]: one block per (j, group of DOTS_NB instances,
// slot chunk, column split), so each weight word is read once for the group's
// instances (one block per instance read the 474 MB of weights of the zkvm's CCS
// once per instance: 4.3 ms of k_dots per fold() for u_s and eta_s in pairs);
// with nsplit > 1 the block sums columns [split n / nsplit, (split + 1) n / nsplit)
// into out[split][i][j] (the partial sums k_dots_sum adds up)
constexpr int DOTS_NB = 4;
template <int TB>
__global__ void __launch_bounds__(MT) k_dots(const uint64_t *w, const uint64_t *z, int t, int nz, size_t n, int d,
                                            int spb, int nsplit, uint64_t *out) {
  __shared__ uint64_t red[DOTS_NB * MT * TB];
  const int slot_l = threadIdx.x % spb, lane_c = threadIdx.x / spb, cpb = MT / spb;
  const int split = blockIdx.z % nsplit, slot = (blockIdx.z / nsplit) * spb + slot_l;
  const int i0 = blockIdx.y * DOTS_NB, j = blockIdx.x;
  const int nb = nz - i0 < DOTS_NB ? nz - i0 : DOTS_NB;  // uniform
  const uint64_t *wj = w + (size_t)j * n * d + slot * TB, *zb = z + (size_t)i0 * n * d + slot * TB;
  const size_t c0 = n * split / nsplit, c1 = n * (split + 1) / nsplit;
  SAcc<TB> la[DOTS_NB];
#pragma unroll
  for (int b = 0; b < DOTS_NB; b++) sacc_zero(la[b]);
  for (size_t c = c0 + lane_c; c < c1; c += cpb) {
    const Sv<TB> wv = s_load<TB>(wj + c * d);
#pragma unroll
    for (int b = 0; b < DOTS_NB; b++)
      if (b < nb) sacc_mad(la[b], wv, s_load<TB>(zb + ((size_t)b * n + c) * d));
  }
#pragma unroll
  for (int b = 0; b < DOTS_NB; b++) s_store(red + ((size_t)b * MT + threadIdx.x) * TB, sacc_final(la[b]));
  __syncthreads();
  for (int h = cpb / 2; h > 0; h >>= 1) {
    if (lane_c < h)
#pragma unroll
      for (int b = 0; b < DOTS_NB; b++) {
        uint64_t *r0 = red + ((size_t)b * MT + threadIdx.x) * TB;
        s_store(r0, s_add(s_load<TB>(r0), s_load<TB>(r0 + (size_t)h * spb * TB)));
      }
    __syncthreads();
  }
  if (lane_c == 0)
    for (int b = 0; b < nb; b++)
      s_store(out + (((size_t)split * nz + i0 + b) * t + j) * d + slot * TB,
              s_load<TB>(red + ((size_t)b * MT + threadIdx.x) * TB));
}
// out[x] = sum_s part[s][x], one thread per word
__global__ void k_dots_sum(const uint64_t *part, int nsplit, size_t len, uint64_t *out) {
  const size_t x = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (x >= len) return;
  uint64_t a = part[x];
  for (int s = 1; s < nsplit; s++) a = gl::add(a, part[(size_t)s * len + x]);
  out[x] = a;
}
// column splits: enough blocks for the chip (about 2048) when t nz is small
int dots_nsplit(const CcsDev &M, int nz) {
  const int tb = slot_words(M.d), ns = M.d / tb, spb = ns < MT ? ns : MT;
  const size_t blocks = (size_t)M.t * ((nz + DOTS_NB - 1) / DOTS_NB) * (ns / spb);
  int k = (int)((2048 + blocks - 1) / blocks);
  if (k > 16) k = 16;
  if ((size_t)k * 64 > M.n) k = (int)(M.n / 64) > 1 ? (int)(M.n / 64) : 1;
  return k < 1 ? 1 : k;
}

unsigned nblk(size_t n, int t) { return (unsigned)((n + t - 1) / t); }

// Mz MLE outputs above this many bytes are written with streaming stores: the zkvm's
// 3.1 GB otherwise cycle through L2 and evict the z rows the gathers re-read (k_csr
// 1.43 -> 1.32 ms; the transposes' 474 MB of weights gain nothing and keep plain stores)
constexpr size_t CSR_NT_BYTES = (size_t)256 << 20;

// out[i][from + x] = 0 for x < tail, i < total / tail (MLE i of len u64)
__global__ void k_zero_tails(uint64_t *out, size_t len, size_t from, size_t tail, size_t total) {
  const size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (t >= total) return;
  const size_t i = t / tail;
  out[i * len + from + (t - i * tail)] = 0;
}

// sv: the scalar values in this CSR's entry order (CcsDev::sval / svh / svc), read
// without vidx; otherwise the ring values through vidx
hipError_t csr(const CcsDev &M, const uint64_t *rp, size_t rp_stride, int na, const uint32_t *col,
               const uint32_t *vidx, const uint64_t *sv, size_t nrows, const uint64_t *z, size_t z_stride,
               uint64_t *out, size_t out_stride, int ntask, hipStream_t st, const int *sel = nullptr,
               bool nt = false, const uint64_t *rv = nullptr) {
  if (!nrows || !ntask) return hipSuccess;
  const int d = M.d, tb = slot_words(d), ns = d / tb, spb = ns < MT ? ns : MT;
  const dim3 grid(nblk(nrows, MT / spb), (unsigned)ntask, (unsigned)(ns / spb));
  // the entries' values in this product's own order when there is a copy (sv: scalar,
  // rv: ring-valued), else gathered through vidx
  const uint64_t *val = M.sval ? sv : (rv ? rv : M.val);
  if (M.sval || rv) vidx = nullptr;
#define LF_CSR(TB, SC)                                                                                          \
  if (nt)                                                                                                       \
    hipLaunchKernelGGL((k_csr<TB, SC, true>), grid, dim3(MT), 0, st, rp, rp_stride, na, sel, col, vidx, val, nrows, \
                       d, z, z_stride, out, out_stride, spb);                                                   \
  else                                                                                                          \
    hipLaunchKernelGGL((k_csr<TB, SC, false>), grid, dim3(MT), 0, st, rp, rp_stride, na, sel, col, vidx, val,     \
                       nrows, d, z, z_stride, out, out_stride, spb)
  if (tb == 3) {
    if (M.sval) {
      LF_CSR(3, true);
    } else {
      LF_CSR(3, false);
    }
  } else {
    if (M.sval) {
      LF_CSR(1, true);
    } else {
      LF_CSR(1, false);
    }
  }
#undef LF_CSR
  return hipGetLastError();
}

// words of one side's scratch before y: the powers pw and, for d = 24, the operand pieces
size_t zc_front(const CcsDev &M, int nz) {
  if (slot_words(M.d) != 3) return 2 * (size_t)M.t * nz * M.d;
  const size_t kcn = (3 * (size_t)nz + 63) / 64, nrt = ((size_t)M.t + ZC_J - 1) / ZC_J, nct = (M.n + 15) / 16;
  return (size_t)M.t * nz * M.d + (nrt + nct) * (ZC_D / 3) * kcn * 512 * 2;
}

// y[j][c] = sum_i zeta_i^(j+1) (.) z_i[c] in one side's scratch (pw | pieces | y)
hipError_t zcomb(const CcsDev &M, const uint64_t *z, const uint64_t *zeta, int nz, uint64_t *scr, uint64_t *&y,
                 hipStream_t st) {
  const int tb = slot_words(M.d), ns = M.d / tb;
  uint64_t *pw = scr;
  y = scr + zc_front(M, nz);
  if (!M.t || !M.n || nz < 1) return hipSuccess;
  if (tb == 3) {
    if (M.d != ZC_D) return hipErrorInvalidValue;
    const int kcn = (3 * nz + 63) / 64, nrt = (M.t + ZC_J - 1) / ZC_J;
    const size_t nct = (M.n + 15) / 16;
    v4i *af = reinterpret_cast<v4i *>(scr + (size_t)M.t * nz * M.d), *bf = af + (size_t)ns * nrt * kcn * 512;
    hipLaunchKernelGGL(k_zeta_pows<3>, dim3(nblk((size_t)M.t * nz * ns, 256)), dim3(256), 0, st, zeta, nz, M.t, M.d, pw);
    hipLaunchKernelGGL(k_zc_afrag, dim3(nblk((size_t)ns * nrt * kcn * 64, 256)), dim3(256), 0, st, pw, nz, M.t, nrt,
                       kcn, af);
    hipLaunchKernelGGL(k_zc_bfrag, dim3(nblk(nct * ns * kcn * 64, 512)), dim3(512), 0, st, z, nz, M.n, kcn, nct, bf);
    const dim3 grid((unsigned)(8 * ((nct + 7) / 8) * ((nrt + ZC_WAVES - 1) / ZC_WAVES)));
    if (3 * nz < 64)
      hipLaunchKernelGGL(k_zcomb_mfma<true>, grid, dim3(64 * ZC_WAVES), 0, st, af, bf, M.t, M.n, nrt, kcn, nct, y);
    else
      hipLaunchKernelGGL(k_zcomb_mfma<false>, grid, dim3(64 * ZC_WAVES), 0, st, af, bf, M.t, M.n, nrt, kcn, nct, y);
  } else {
    hipLaunchKernelGGL(k_zeta_pows<1>, dim3(nblk((size_t)M.t * nz * ns, 256)), dim3(256), 0, st, zeta, nz, M.t, M.d, pw);
    hipLaunchKernelGGL(k_zcomb<1>, dim3(nblk((size_t)M.t * M.n * ns, 256)), dim3(256), 0, st, pw, z, nz, M.t, M.n,
                       M.d, y);
  }
  return hipGetLastError();
}

__global__ void k_gather_entries(const uint64_t *val, const uint32_t *idx, size_t nnz, int d, uint64_t *out) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;  // (entry, word)
  if (i >= nnz * d) return;
  const size_t k = i / d;
  out[i] = val[(size_t)idx[k] * d + (i - k * d)];
}

}  // namespace

hipError_t gather_entries(const uint64_t *val, const uint32_t *idx, size_t nnz, int d, uint64_t *out, hipStream_t st) {
  if (!nnz) return hipSuccess;
  hipLaunchKernelGGL(k_gather_entries, dim3(nblk(nnz * d, 256)), dim3(256), 0, st, val, idx, nnz, d, out);
  return hipGetLastError();
}

size_t mz_chall_elems(const CcsDev &M, int nz) { return zc_front(M, nz) + (size_t)M.t * M.n * M.d; }

size_t mz_scratch_elems(const CcsDev &M, int nz, int nv) {
  const size_t e = ((size_t)1 << nv) * M.d, tn = (size_t)M.t * M.n * M.d;
  const size_t chall = mz_chall_elems(M, nz), eval = e + tn + mz_dots_partial_elems(M, nz);
  return chall > eval ? chall : eval;
}

hipError_t mz_mles(const CcsDev &M, const uint64_t *z, int nz, int nv, uint64_t *out, hipStream_t st, const int *sel,
                   int nsel) {
  const size_t len = ((size_t)1 << nv) * M.d;
  if (M.m > ((size_t)1 << nv)) return hipErrorInvalidValue;
  const int na = sel ? nsel : M.t;
  if (na < 1) return hipSuccess;
  if (M.m < ((size_t)1 << nv)) {  // the MLEs' zero padding: rows m .. 2^nv - 1 of each
    const size_t tail = len - M.m * M.d, total = (size_t)nz * na * tail;
    hipLaunchKernelGGL(k_zero_tails, dim3(nblk(total, 256)), dim3(256), 0, st, out, len, M.m * M.d, tail, total);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return csr(M, M.rp, M.m + 1, na, M.col, nullptr, M.sval, M.m, z, M.n * M.d, out, len, nz * na, st, sel,
             (size_t)nz * na * len * 8 >= CSR_NT_BYTES);
}

hipError_t mz_challenged(const CcsDev &M, const uint64_t *z, const uint64_t *zeta, int nz, int nv, uint64_t *out,
                         uint64_t *scratch, hipStream_t st) {
  const size_t len = ((size_t)1 << nv) * M.d;
  if (M.m > ((size_t)1 << nv)) return hipErrorInvalidValue;
  uint64_t *y;
  hipError_t e = zcomb(M, z, zeta, nz, scratch, y, st);
  if (e != hipSuccess) return e;
  if (len > M.m * M.d) {
    e = hipMemsetAsync(out + M.m * M.d, 0, (len - M.m * M.d) * 8, st);
    if (e != hipSuccess) return e;
  }
  return csr(M, M.hrp, 0, 1, M.hcol, M.hidx, M.svh, M.m, y, 0, out, 0, 1, st, nullptr, false, M.vh);
}

hipError_t mz_challenged_pair(const CcsDev &M, const uint64_t *z0, const uint64_t *zeta0, const uint64_t *z1,
                              const uint64_t *zeta1, int nz, int nv, uint64_t *out0, uint64_t *out1,
                              uint64_t *scratch, hipStream_t st) {
  const size_t len = ((size_t)1 << nv) * M.d;
  if (M.m > ((size_t)1 << nv)) return hipErrorInvalidValue;
  const int tb = slot_words(M.d), ns = M.d / tb;
  const size_t per = mz_chall_elems(M, nz);  // pw | pieces | y of one side
  const uint64_t *zs[2] = {z0, z1}, *zetas[2] = {zeta0, zeta1};
  uint64_t *ys[2], *outs[2] = {out0, out1};
  for (int q = 0; q < 2; q++) {
    hipError_t e = zcomb(M, zs[q], zetas[q], nz, scratch + q * per, ys[q], st);
    if (e != hipSuccess) return e;
    if (len > M.m * M.d) {
      e = hipMemsetAsync(outs[q] + M.m * M.d, 0, (len - M.m * M.d) * 8, st);
      if (e != hipSuccess) return e;
    }
  }
  if (!M.m) return hipSuccess;
  const int spb = ns < MT ? ns : MT;
  const dim3 grid(nblk(M.m, MT / spb), 1, (unsigned)(ns / spb));
  const uint64_t *val = M.sval ? M.svh : (M.vh ? M.vh : M.val);
  const uint32_t *vidx = M.sval || M.vh ? nullptr : M.hidx;
#define LF_CSRP(TB, SC)                                                                                       \
  hipLaunchKernelGGL((k_csr_pair<TB, SC>), grid, dim3(MT), 0, st, M.hrp, M.hcol, vidx, val, M.m, M.d, ys[0], ys[1], \
                     out0, out1, spb)
  if (tb == 3) {
    if (M.sval)
      LF_CSRP(3, true);
    else
      LF_CSRP(3, false);
  } else {
    if (M.sval)
      LF_CSRP(1, true);
    else
      LF_CSRP(1, false);
  }
#undef LF_CSRP
  return hipGetLastError();
}

hipError_t mz_weights(const CcsDev &M, const uint64_t *eq, uint64_t *w, hipStream_t st) {
  // w_j[c] = sum over column c of M_j of value (.) eq[row]
  return csr(M, M.crp, M.n + 1, M.t, M.crow, M.cidx, M.svc, M.n, eq, 0, w, M.n * M.d, M.t, st, nullptr, false, M.vc);
}

hipError_t mz_evaluate(const CcsDev &M, const uint64_t *z, int nz, int nv, const uint64_t *point, uint64_t *out,
                       uint64_t *scratch, hipStream_t st) {
  if (M.m > ((size_t)1 << nv)) return hipErrorInvalidValue;
  uint64_t *eq = scratch, *w = scratch + ((size_t)1 << nv) * M.d;
  hipError_t e = eq_table(point, nv, M.d, eq, st);
  if (e != hipSuccess) return e;
  e = mz_weights(M, eq, w, st);
  if (e != hipSuccess) return e;
  return mz_dots(M, w, z, nz, out, st, w + (size_t)M.t * M.n * M.d);
}

size_t mz_dots_partial_elems(const CcsDev &M, int nz) {
  const int k = dots_nsplit(M, nz);
  return k > 1 ? (size_t)k * nz * M.t * M.d : 0;
}

hipError_t mz_dots(const CcsDev &M, const uint64_t *w, const uint64_t *z, int nz, uint64_t *out, hipStream_t st,
                   uint64_t *partial) {
  if (!nz) return hipSuccess;
  const int tb = slot_words(M.d), ns = M.d / tb, spb = ns < MT ? ns : MT;
  const int nsplit = partial ? dots_nsplit(M, nz) : 1;
  uint64_t *dst = nsplit > 1 ? partial : out;
  const dim3 grid((unsigned)M.t, (unsigned)((nz + DOTS_NB - 1) / DOTS_NB), (unsigned)(ns / spb * nsplit));
  if (tb == 3)
    hipLaunchKernelGGL(k_dots<3>, grid, dim3(MT), 0, st, w, z, M.t, nz, M.n, M.d, spb, nsplit, dst);
  else
    hipLaunchKernelGGL(k_dots<1>, grid, dim3(MT), 0, st, w, z, M.t, nz, M.n, M.d, spb, nsplit, dst);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || nsplit == 1) return e;
  const size_t len = (size_t)nz * M.t * M.d;
  hipLaunchKernelGGL(k_dots_sum, dim3(nblk(len, 256)), dim3(256), 0, st, partial, nsplit, len, out);
  return hipGetLastError();
}

}  // namespace lfk
