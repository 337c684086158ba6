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
#include "kernels.hpp"
#include "slot.hpp"

namespace lfk {

namespace {

constexpr int MT = 256;

// out[task][r] = sum_k val[vidx ? vidx[k] : k] (.) z[col[k]], k in [rp[r], rp[r+1]);
// task = (a, b) = (task % na, task / na) selects rp + A rp_stride (A = sel ? sel[a] : a)
// and z + b z_stride. SC: val holds one scalar per entry (CcsDev::sval), the zkvm's
// matrices (R::one(), from_goldilocks constants: zkvm/src/constraints.rs:127-364)
template <int TB, bool SC>
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
  s_store(out + task * out_stride + r * d + slot * TB, sacc_final(acc));
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

// pw[j][i] = zeta_i^(j+1)
template <int TB>
__global__ void k_zeta_pows(const uint64_t *zeta, int nz, int t, int d, uint64_t *pw) {
  const int ns = d / TB;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;  // (instance, slot)
  if (i >= nz * ns) return;
  const int zi = i / ns, s = i - zi * ns;
  const Sv<TB> zt = s_load<TB>(zeta + (size_t)zi * d + s * TB);
  Sv<TB> p = zt;
  for (int j = 0; j < t; j++) {
    s_store(pw + ((size_t)j * nz + zi) * d + s * TB, p);
    p = s_mul(p, zt);
  }
}

// Fq3 (d = 24): the powers with their pairwise sums, pk[j][i][slot] = (p0, p1, p2,
// p0 + p1, p0 + p2, p1 + p2), for the Karatsuba form of k_zcomb3
__global__ void k_zeta_pows3k(const uint64_t *zeta, int nz, int t, int d, uint64_t *pk) {
  const int ns = d / 3;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;  // (instance, slot)
  if (i >= nz * ns) return;
  const int zi = i / ns, s = i - zi * ns;
  const Sv<3> zt = s_load<3>(zeta + (size_t)zi * d + s * 3);
  Sv<3> p = zt;
  for (int j = 0; j < t; j++) {
    uint64_t *o = pk + ((size_t)j * nz + zi) * 2 * d + s * 6;
    o[0] = p.c[0];
    o[1] = p.c[1];
    o[2] = p.c[2];
    o[3] = gl::add(p.c[0], p.c[1]);
    o[4] = gl::add(p.c[0], p.c[2]);
    o[5] = gl::add(p.c[1], p.c[2]);
    p = s_mul(p, zt);
  }
}
// y[j][c] = sum_i pw[j][i] (.) z_i[c] in Fq3 with Karatsuba's six products per term, each
// summed lazily over i (P_k = sum p_k z_k, Q_kl = sum (p_k + p_l)(z_k + z_l)) and combined
// once: a1 b2 + a2 b1 = Q12 - P1 - P2 and so on; c0 = P0 + 2^40 (a1 b2 + a2 b1),
// c1 = (a0 b1 + a1 b0) + 2^40 P2, c2 = (a0 b2 + a2 b0) + P1. Six multiply-accumulates
// and three additions per term instead of nine and two shifts (goldilocks/mod.rs:34-54).
__global__ void k_zcomb3k(const uint64_t *pk, const uint64_t *z, int nz, int t, size_t n, int d, uint64_t *y) {
  const int ns = d / 3;
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;  // (j, c, slot)
  if (i >= (size_t)t * n * ns) return;
  const size_t jc = i / ns;
  const int s = (int)(i - jc * ns);
  const size_t j = jc / n, c = jc - j * n;
  gl::CAcc a[6];
#pragma unroll
  for (int k = 0; k < 6; k++) gl::cacc_zero(a[k]);
  for (int zi = 0; zi < nz; zi++) {
    const uint64_t *pp = pk + (j * nz + zi) * 2 * d + s * 6;
    const Sv<3> zv = s_load<3>(z + (zi * n + c) * d + s * 3);
    gl::cacc_mad(a[0], pp[0], zv.c[0]);
    gl::cacc_mad(a[1], pp[1], zv.c[1]);
    gl::cacc_mad(a[2], pp[2], zv.c[2]);
    gl::cacc_mad(a[3], pp[3], gl::add(zv.c[0], zv.c[1]));
    gl::cacc_mad(a[4], pp[4], gl::add(zv.c[0], zv.c[2]));
    gl::cacc_mad(a[5], pp[5], gl::add(zv.c[1], zv.c[2]));
  }
  uint64_t v[6];
#pragma unroll
  for (int k = 0; k < 6; k++) v[k] = gl::cacc_reduce(a[k]);
  const uint64_t m12 = gl::sub(gl::sub(v[5], v[1]), v[2]);  // sum a1 b2 + a2 b1
  const uint64_t m01 = gl::sub(gl::sub(v[3], v[0]), v[1]);
  const uint64_t m02 = gl::sub(gl::sub(v[4], v[0]), v[2]);
  uint64_t *o = y + jc * d + s * 3;
  o[0] = gl::add(v[0], gl::shl96(m12, 40));
  o[1] = gl::add(m01, gl::shl96(v[2], 40));
  o[2] = gl::add(m02, v[1]);
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
               uint64_t *out, size_t out_stride, int ntask, hipStream_t st, const int *sel = nullptr) {
  if (!nrows || !ntask) return hipSuccess;
  const int d = M.d, tb = slot_words(d), ns = d / tb, spb = ns < MT ? ns : MT;
  const dim3 grid(nblk(nrows, MT / spb), (unsigned)ntask, (unsigned)(ns / spb));
  const uint64_t *val = M.sval ? sv : M.val;
  if (M.sval) vidx = nullptr;
#define LF_CSR(TB, SC)                                                                                            \
  hipLaunchKernelGGL((k_csr<TB, SC>), grid, dim3(MT), 0, st, rp, rp_stride, na, sel, col, vidx, val, nrows, d, z, \
                     z_stride, out, out_stride, spb)
  if (tb == 3) {
    if (M.sval)
      LF_CSR(3, true);
    else
      LF_CSR(3, false);
  } else {
    if (M.sval)
      LF_CSR(1, true);
    else
      LF_CSR(1, false);
  }
#undef LF_CSR
  return hipGetLastError();
}

}  // namespace

size_t mz_scratch_elems(const CcsDev &M, int nz, int nv) {
  const size_t e = ((size_t)1 << nv) * M.d, tn = (size_t)M.t * M.n * M.d;
  const size_t chall = 2 * (size_t)M.t * nz * M.d + tn, eval = e + tn + mz_dots_partial_elems(M, nz);
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
  return csr(M, M.rp, M.m + 1, na, M.col, nullptr, M.sval, M.m, z, M.n * M.d, out, len, nz * na, st, sel);
}

hipError_t mz_challenged(const CcsDev &M, const uint64_t *z, const uint64_t *zeta, int nz, int nv, uint64_t *out,
                         uint64_t *scratch, hipStream_t st) {
  const size_t len = ((size_t)1 << nv) * M.d;
  if (M.m > ((size_t)1 << nv)) return hipErrorInvalidValue;
  const int tb = slot_words(M.d), ns = M.d / tb;
  uint64_t *pw = scratch, *y = scratch + 2 * (size_t)M.t * nz * M.d;
  if (tb == 3)
    hipLaunchKernelGGL(k_zeta_pows3k, dim3(nblk((size_t)nz * ns, 256)), dim3(256), 0, st, zeta, nz, M.t, M.d, pw);
  else
    hipLaunchKernelGGL(k_zeta_pows<1>, dim3(nblk((size_t)nz * ns, 256)), dim3(256), 0, st, zeta, nz, M.t, M.d, pw);
  const size_t ny = (size_t)M.t * M.n * ns;
  if (tb == 3)
    hipLaunchKernelGGL(k_zcomb3k, dim3(nblk(ny, 256)), dim3(256), 0, st, pw, z, nz, M.t, M.n, M.d, y);
  else
    hipLaunchKernelGGL(k_zcomb<1>, dim3(nblk(ny, 256)), dim3(256), 0, st, pw, z, nz, M.t, M.n, M.d, y);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  if (len > M.m * M.d) {
    e = hipMemsetAsync(out + M.m * M.d, 0, (len - M.m * M.d) * 8, st);
    if (e != hipSuccess) return e;
  }
  return csr(M, M.hrp, 0, 1, M.hcol, M.hidx, M.svh, M.m, y, 0, out, 0, 1, st);
}

hipError_t mz_challenged_pair(const CcsDev &M, const uint64_t *z0, const uint64_t *zeta0, const uint64_t *z1,
                              const uint64_t *zeta1, int nz, int nv, uint64_t *out0, uint64_t *out1,
                              uint64_t *scratch, hipStream_t st) {
  const size_t len = ((size_t)1 << nv) * M.d;
  if (M.m > ((size_t)1 << nv)) return hipErrorInvalidValue;
  const int tb = slot_words(M.d), ns = M.d / tb;
  const size_t per = 2 * (size_t)M.t * nz * M.d + (size_t)M.t * M.n * M.d;  // pw | y of one side
  const uint64_t *zs[2] = {z0, z1}, *zetas[2] = {zeta0, zeta1};
  uint64_t *ys[2], *outs[2] = {out0, out1};
  for (int q = 0; q < 2; q++) {
    uint64_t *pw = scratch + q * per, *y = pw + 2 * (size_t)M.t * nz * M.d;
    ys[q] = y;
    if (tb == 3)
      hipLaunchKernelGGL(k_zeta_pows3k, dim3(nblk((size_t)nz * ns, 256)), dim3(256), 0, st, zetas[q], nz, M.t, M.d, pw);
    else
      hipLaunchKernelGGL(k_zeta_pows<1>, dim3(nblk((size_t)nz * ns, 256)), dim3(256), 0, st, zetas[q], nz, M.t, M.d,
                         pw);
    const size_t ny = (size_t)M.t * M.n * ns;
    if (tb == 3)
      hipLaunchKernelGGL(k_zcomb3k, dim3(nblk(ny, 256)), dim3(256), 0, st, pw, zs[q], nz, M.t, M.n, M.d, y);
    else
      hipLaunchKernelGGL(k_zcomb<1>, dim3(nblk(ny, 256)), dim3(256), 0, st, pw, zs[q], nz, M.t, M.n, M.d, y);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (len > M.m * M.d) {
      e = hipMemsetAsync(outs[q] + M.m * M.d, 0, (len - M.m * M.d) * 8, st);
      if (e != hipSuccess) return e;
    }
  }
  if (!M.m) return hipSuccess;
  const int spb = ns < MT ? ns : MT;
  const dim3 grid(nblk(M.m, MT / spb), 1, (unsigned)(ns / spb));
  const uint64_t *val = M.sval ? M.svh : M.val;
  const uint32_t *vidx = M.sval ? nullptr : M.hidx;
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
  return csr(M, M.crp, M.n + 1, M.t, M.crow, M.cidx, M.svc, M.n, eq, 0, w, M.n * M.d, M.t, st);
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
