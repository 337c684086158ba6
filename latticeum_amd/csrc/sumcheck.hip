// sumcheck.hip -- the multilinear sumcheck prover's device work (SURVEY.md
// 8(f) rank 1): eq tables, fix_variables, the per-round sums of the folding and
// linearization polynomials, and MLE evaluation.
//
// Reference: latticefold/src/utils/sumcheck/prover.rs:62-168 (prove_round),
// utils/sumcheck/utils.rs:140-210 (build_eq_x_r), poly/src/mle/dense.rs:107-199
// (evaluate, fix_variables), nifs/folding/utils.rs:196-331 (the folding
// polynomial and its combination function), nifs/linearization/utils.rs:63-104.
//
// An MLE over nv variables is 2^nv ring elements in NTT form (d u64 each; the
// reference's zero-truncated vectors read as zero-padded, dense.rs:397-418),
// and a batch of nm MLEs is one contiguous [nm][2^nv][d] buffer. The
// challenges are base-ring elements broadcast into every NTT slot, so every
// slot runs its own sumcheck: a thread owns one (point, slot) pair, where a
// slot is an Fq3 (Phi_72, TB = 3 words) or an Fq (X^d + 1, TB = 1).
#include "gl.hpp"
#include "kernels.hpp"
#include "ring.hpp"
#include "slot.hpp"

namespace lfk {

namespace {

// ---------------------------------------------------------------- eq table
// build_eq_x_r (sumcheck/utils.rs:140-210): eq[x] = prod_k (x_k ? r_k : 1 - r_k),
// x_0 = the least significant bit. The reference builds it by doubling with
// b - r b and r b; the product of the same factors is the same field element.
template <int TB>
__global__ void k_eq_table(const uint64_t *r, int nv, int d, uint64_t *out) {
  const int ns = d / TB;
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i >= ((size_t)ns << nv)) return;
  const size_t x = i / ns;
  const int s = (int)(i - x * ns);
  Sv<TB> acc = s_one<TB>();
  for (int k = 0; k < nv; k++) {
    const Sv<TB> rk = s_load<TB>(r + (size_t)k * d + s * TB);
    acc = s_mul(acc, (x >> k) & 1 ? rk : s_sub(s_one<TB>(), rk));
  }
  s_store(out + x * d + s * TB, acc);
}

// ---------------------------------------------------------------- fix_variables
// dense.rs:171-199 for one point: out[m][b] = in[m][2b] + r (in[m][2b+1] - in[m][2b]),
// r a base-ring value in every slot; out-of-place (ping-pong buffers)
// ptrs (optional, device): MLE m starts at ptrs[m] instead of in + m in_stride (the
// linearization's first round reads its MLEs where the Mz products left them)
template <int TB>
__global__ void k_fix_first(const uint64_t *in, size_t in_stride, const uint64_t *const *ptrs, int nm, size_t half,
                            int d, Sv<TB> r, uint64_t *out, size_t out_stride) {
  const int ns = d / TB;
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;  // (m, b, slot)
  if (i >= (size_t)nm * half * ns) return;
  const size_t mb = i / ns;
  const int s = (int)(i - mb * ns);
  const size_t m = mb / half, b = mb - m * half;
  const uint64_t *p = (ptrs ? ptrs[m] : in + m * in_stride) + 2 * b * d + s * TB;
  const Sv<TB> left = s_load<TB>(p), right = s_load<TB>(p + d);
  // r on the right: the nonresidue shifts of its words are uniform (scalar unit), not per lane
  s_store(out + m * out_stride + b * d + s * TB, s_add(left, s_mul(s_sub(right, left), r)));
}

// ---------------------------------------------------------------- round sums
// A block holds PPB points x SPB slots; a thread loops over points with a grid
// stride, keeps its per-evaluation-point sums in registers, and the block
// writes partial[blockIdx.x][e][slot] after an LDS reduction over its points.
constexpr int RT = 256;
constexpr int MAX_EVALS = 10;  // degree + 1 <= 10

// dst: this block's sums, evaluation point e at dst + e d (slot words at slot TB)
template <int TB, int NE>
__device__ __forceinline__ void block_partial(const Sv<TB> (&acc)[NE], int spb, int ppb, int slot, int lane_p,
                                              int d, uint64_t *dst) {
  __shared__ uint64_t red[RT * TB];
#pragma unroll
  for (int e = 0; e < NE; e++) {
    s_store(red + threadIdx.x * TB, acc[e]);
    __syncthreads();
    for (int w = ppb / 2; w > 0; w >>= 1) {
      if (lane_p < w) {
        const int o = threadIdx.x + w * spb;
        s_store(red + threadIdx.x * TB, s_add(s_load<TB>(red + threadIdx.x * TB), s_load<TB>(red + o * TB)));
      }
      __syncthreads();
    }
    if (lane_p == 0) s_store(dst + (size_t)e * d + slot * TB, s_load<TB>(red + threadIdx.x * TB));
    __syncthreads();
  }
}

// The folding polynomial (folding/utils.rs:196-331), MLEs [eq_r0, g0, eq_r1, g1,
// eq_beta, f_hat (nk x tau)]:
//   comb = v0 v1 + v2 v3 + sum_k Horner_dd( v4 f (prod_{b<B_SMALL} (f^2 - b^2)) ) in mu_k
// The Horner over dd = tau-1 .. 0 is sum_dd mu_k^(dd+1) e_dd, so with
// w_(k,dd) = mu_k^(dd+1) (k_fold_weights) the per-point value is
//   v0 v1 + v2 v3 + v4 S,  S = sum_(k,dd) w_(k,dd) g(f_(k,dd)),  g(f) = f prod (f^2 - b^2)
// (the reference's zero short-cuts do not change values). S is linear in the
// f_hat MLEs, so a launch may split them over blockIdx.z chunks: every chunk
// adds v4 S_chunk and chunk 0 also v0 v1 + v2 v3; the block sums meet in
// k_sum_partials. On the point line f(e) = a + e s:
//  * B_SMALL = 2 (GoldiLocksDP): g = f^3 - f, and w g(f(e)) is the cubic
//    C0 + C1 e + C2 e^2 + C3 e^3 with C3 = (w s^2) s, C2 = 3 (w s^2) a,
//    C1 = (w s)(3 a^2 - 1), C0 = (w a)(a^2 - 1): four products and four lazy
//    multiply-accumulates per MLE value, and S(e) from the summed coefficients;
//  * otherwise S is evaluated at e < degree and extrapolated to e = degree by
//    finite differences (S has degree 2 B_SMALL - 1).
template <int TB, int BS>
__global__ void __launch_bounds__(RT) k_round_folding(const uint64_t *mles, size_t stride, int nf, const uint64_t *w,
                                                      size_t half, int d, int spb, uint64_t *partial) {
  const int slot_l = threadIdx.x % spb, lane_p = threadIdx.x / spb, ppb = RT / spb;
  const int slot = blockIdx.y * spb + slot_l;
  const int chunk = blockIdx.z, nchunk = gridDim.z;
  const int f0 = (int)((long)nf * chunk / nchunk), f1 = (int)((long)nf * (chunk + 1) / nchunk);
  constexpr int degree = 2 * BS;
  Sv<TB> acc[degree + 1];
#pragma unroll
  for (int e = 0; e <= degree; e++) acc[e] = s_zero<TB>();
  for (size_t b = (size_t)blockIdx.x * ppb + lane_p; b < half; b += (size_t)gridDim.x * ppb) {
    const uint64_t *pb = mles + 2 * b * d + slot * TB;
    Sv<TB> S[degree + 1];
    if (BS == 2) {
      SAcc<TB> c0, c1, c2, c3;
      sacc_zero(c0);
      sacc_zero(c1);
      sacc_zero(c2);
      sacc_zero(c3);
      for (int f = f0; f < f1; f++) {
        const uint64_t *p = pb + (size_t)(5 + f) * stride;
        const Sv<TB> a = s_load<TB>(p), st = s_sub(s_load<TB>(p + d), a);
        const Sv<TB> wf = s_load<TB>(w + (size_t)f * d + slot * TB);
        // ws, ws2 and wa only enter products on their left (any u64 there): weakly reduced
        const Sv<TB> ws = s_mul_w(wf, st), ws2 = s_mul_w(ws, st), a2 = s_mul(a, a), wa = s_mul_w(wf, a);
        sacc_mad(c3, ws2, st);
        sacc_mad(c2, ws2, a);
        sacc_mad(c1, ws, s_sub(s_smul(a2, 3), s_one<TB>()));
        sacc_mad(c0, wa, s_sub(a2, s_one<TB>()));
      }
      const Sv<TB> C0 = sacc_final(c0), C1 = sacc_final(c1), C2 = s_smul(sacc_final(c2), 3), C3 = sacc_final(c3);
#pragma unroll
      for (int e = 0; e <= degree; e++)
        S[e] = s_add(s_add(C0, s_smul(C1, e)), s_add(s_smul(C2, e * e), s_smul(C3, e * e * e)));
    } else {
#pragma unroll
      for (int e = 0; e < degree; e++) S[e] = s_zero<TB>();
      for (int f = f0; f < f1; f++) {
        const uint64_t *p = pb + (size_t)(5 + f) * stride;
        const Sv<TB> a = s_load<TB>(p), st = s_sub(s_load<TB>(p + d), a);
        const Sv<TB> wf = s_load<TB>(w + (size_t)f * d + slot * TB);
        Sv<TB> x = a;
#pragma unroll
        for (int e = 0; e < degree; e++) {
          const Sv<TB> x2 = s_mul(x, x);
          Sv<TB> g = x;
#pragma unroll
          for (int bb = 1; bb < BS; bb++) g = s_mul(g, s_sub(x2, s_scalar<TB>((uint64_t)bb * bb)));
          S[e] = s_add(S[e], s_mul(wf, g));
          x = s_add(x, st);
        }
      }
      // S(degree) from S(0 .. degree-1): sum_j (-1)^(degree-1-j) C(degree, j) S(j)
      Sv<TB> ext = s_zero<TB>();
      uint64_t binom = 1;  // C(degree, j)
#pragma unroll
      for (int j = 0; j < degree; j++) {
        const Sv<TB> scaled = s_smul(S[j], binom);
        ext = ((degree - 1 - j) & 1) ? s_sub(ext, scaled) : s_add(ext, scaled);
        binom = binom * (uint64_t)(degree - j) / (uint64_t)(j + 1);
      }
      S[degree] = ext;
    }
    Sv<TB> v[5], sv[5];
#pragma unroll
    for (int m = 0; m < 5; m++) {
      const uint64_t *p = pb + (size_t)m * stride;
      v[m] = s_load<TB>(p);
      sv[m] = s_sub(s_load<TB>(p + d), v[m]);
    }
#pragma unroll
    for (int e = 0; e <= degree; e++) {
      Sv<TB> t = s_mul(v[4], S[e]);
      if (chunk == 0) t = s_add(t, s_add(s_mul(v[0], v[1]), s_mul(v[2], v[3])));
      acc[e] = s_add(acc[e], t);
#pragma unroll
      for (int m = 0; m < 5; m++) v[m] = s_add(v[m], sv[m]);
    }
  }
  block_partial<TB, degree + 1>(acc, spb, ppb, slot, lane_p, d,
                                partial + ((size_t)chunk * gridDim.x + blockIdx.x) * (degree + 1) * d);
}

// ---------------------------------------------------------------- folding round 0 on digits
// In lf_fold_prove the folding polynomial's f_hat MLEs are Witness::get_fhat of the
// decomposed witnesses, whose coefficients are balanced base-2 digits (b_small = 2):
// every f_hat value of round 0 is 0, 1 or -1. On the line f(e) = a + e dd with a, a + dd
// in {-1, 0, 1}, g(f) = f^3 - f is the cubic C1 e + C2 e^2 + C3 e^3 (C0 = a^3 - a = 0)
// with C1 = (3 a^2 - 1) dd, C2 = 3 a dd^2, C3 = dd^3, small integers, so
// S(e) = sum_f w_f g(f(e)) = A1 e + A2 e^2 + A3 e^3 with A_k = sum_f C_k(f) w_f: three
// small-integer multiply-accumulates of the weight per value instead of four Fq3
// products and four lazy Fq3 products, read straight from the coefficient rows (no
// f_hat MLEs). The same field elements as k_round_folding<TB, 2> on the materialised
// MLEs. C + 12 is non-negative, so A_k = sum_f (C_k + 12) w_f - 12 W, W = sum_f w_f.
struct SmallAcc {  // sum of u64 x small (< 2^32): lo + 2^64 c + 2^32 mid
  uint64_t lo, mid;
  uint32_t c;
};
__device__ __forceinline__ void small_mad(SmallAcc &a, uint64_t x, uint32_t k) {
  uint64_t t;
  a.c += gl::addc64(a.lo, (uint64_t)(uint32_t)x * k, t);
  a.lo = t;
  a.mid += (x >> 32) * k;
}
__device__ __forceinline__ uint64_t small_final(const SmallAcc &a) {
  gl::CAcc x;
  gl::cacc_zero(x);
  x.s0 = a.lo;
  x.c0 = a.c;
  x.s1 = a.mid;
  return gl::cacc_reduce(x);
}
__device__ __forceinline__ int digit_of(uint64_t v) { return v == 0 ? 0 : (v == 1 ? 1 : -1); }

// f_hat value (w, j) at point x, slot: f_coeff_w[x][j ns + slot] (zero past N)
template <int TB>
__global__ void __launch_bounds__(RT) k_round_folding0_digits(const uint64_t *mles, size_t stride,
                                                              const uint64_t *fc0, const uint64_t *fc1, int K,
                                                              size_t N, size_t wstride, int nf, const uint64_t *w,
                                                              size_t half, int d, int spb, uint64_t *partial) {
  constexpr int tau = TB == 3 ? 3 : 1;
  const int slot_l = threadIdx.x % spb, lane_p = threadIdx.x / spb, ppb = RT / spb;
  const int slot = blockIdx.y * spb + slot_l, ns = d / TB;
  const int chunk = blockIdx.z, nchunk = gridDim.z;
  const int f0 = (int)((long)nf * chunk / nchunk), f1 = (int)((long)nf * (chunk + 1) / nchunk);
  constexpr int degree = 4;
  Sv<TB> acc[degree + 1];
#pragma unroll
  for (int e = 0; e <= degree; e++) acc[e] = s_zero<TB>();
  // 12 W over this chunk's weights (the offset's correction, the same at every point)
  Sv<TB> w12 = s_zero<TB>();
  for (int f = f0; f < f1; f++) w12 = s_add(w12, s_load<TB>(w + (size_t)f * d + slot * TB));
  w12 = s_smul(w12, 12);
  for (size_t b = (size_t)blockIdx.x * ppb + lane_p; b < half; b += (size_t)gridDim.x * ppb) {
    const size_t x0 = 2 * b;
    SmallAcc A[3][TB];
#pragma unroll
    for (int k = 0; k < 3; k++)
#pragma unroll
      for (int q = 0; q < TB; q++) A[k][q] = SmallAcc{0, 0, 0};
    for (int f = f0; f < f1; f++) {
      const int kg = f / tau, j = f - kg * tau;
      const uint64_t *fc = (kg < K ? fc0 + (size_t)kg * wstride : fc1 + (size_t)(kg - K) * wstride) + (size_t)j * ns + slot;
      const int a = x0 < N ? digit_of(fc[x0 * d]) : 0;
      const int bv = x0 + 1 < N ? digit_of(fc[(x0 + 1) * d]) : 0;
      const int dd = bv - a;
      const uint32_t c1 = (uint32_t)((3 * a * a - 1) * dd + 12), c2 = (uint32_t)(3 * a * dd * dd + 12),
                     c3 = (uint32_t)(dd * dd * dd + 12);
      const Sv<TB> wf = s_load<TB>(w + (size_t)f * d + slot * TB);
#pragma unroll
      for (int q = 0; q < TB; q++) {
        small_mad(A[0][q], wf.c[q], c1);
        small_mad(A[1][q], wf.c[q], c2);
        small_mad(A[2][q], wf.c[q], c3);
      }
    }
    Sv<TB> Ak[3];
#pragma unroll
    for (int k = 0; k < 3; k++) {
#pragma unroll
      for (int q = 0; q < TB; q++) Ak[k].c[q] = small_final(A[k][q]);
      Ak[k] = s_sub(Ak[k], w12);
    }
    const uint64_t *pb = mles + 2 * b * d + slot * TB;
    Sv<TB> v[5], sv[5];
#pragma unroll
    for (int m = 0; m < 5; m++) {
      const uint64_t *p = pb + (size_t)m * stride;
      v[m] = s_load<TB>(p);
      sv[m] = s_sub(s_load<TB>(p + d), v[m]);
    }
#pragma unroll
    for (int e = 0; e <= degree; e++) {
      // S(e) = ((A3 e + A2) e + A1) e
      const Sv<TB> S = s_smul(s_add(s_smul(s_add(s_smul(Ak[2], e), Ak[1]), e), Ak[0]), e);
      Sv<TB> t = s_mul(v[4], S);
      if (chunk == 0) t = s_add(t, s_add(s_mul(v[0], v[1]), s_mul(v[2], v[3])));
      acc[e] = s_add(acc[e], t);
#pragma unroll
      for (int m = 0; m < 5; m++) v[m] = s_add(v[m], sv[m]);
    }
  }
  block_partial<TB, degree + 1>(acc, spb, ppb, slot, lane_p, d,
                                partial + ((size_t)chunk * gridDim.x + blockIdx.x) * (degree + 1) * d);
}

// the f_hat MLEs fixed by the first challenge r, from the digits: out[f][b] =
// a + r (b - a) (a base-ring digit plus r times a small integer), f = (k, j) as above
template <int TB>
__global__ void k_fix_fhat_digits(const uint64_t *fc0, const uint64_t *fc1, int K, size_t N, size_t wstride, int nf,
                                  size_t half, int d, Sv<TB> r, uint64_t *out, size_t out_stride) {
  constexpr int tau = TB == 3 ? 3 : 1;
  const int ns = d / TB;
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;  // (f, b, slot)
  if (i >= (size_t)nf * half * ns) return;
  const size_t fb = i / ns;
  const int s = (int)(i - fb * ns);
  const int f = (int)(fb / half);
  const size_t b = fb - (size_t)f * half, x0 = 2 * b;
  const int kg = f / tau, j = f - kg * tau;
  const uint64_t *fc = (kg < K ? fc0 + (size_t)kg * wstride : fc1 + (size_t)(kg - K) * wstride) + (size_t)j * ns + s;
  const int a = x0 < N ? digit_of(fc[x0 * d]) : 0;
  const int bv = x0 + 1 < N ? digit_of(fc[(x0 + 1) * d]) : 0;
  const int dd = bv - a;
  Sv<TB> o;
#pragma unroll
  for (int q = 0; q < TB; q++) {
    const uint64_t m = gl::mul(r.c[q], (uint64_t)(dd < 0 ? -dd : dd));
    o.c[q] = dd < 0 ? gl::neg(m) : m;
  }
  o.c[0] = gl::add(o.c[0], a < 0 ? gl::P - 1 : (uint64_t)a);
  s_store(out + (size_t)f * out_stride + b * d + s * TB, o);
}

// io[x] += sum_(k, j) coef[k tau + j] fhat_(k, j)[x] from the digits (x < npts)
template <int TB>
__global__ void k_fhat_lincomb_digits(const uint64_t *fc, int nw, size_t N, size_t wstride, const uint64_t *coef,
                                      size_t npts, int d, uint64_t *io) {
  constexpr int tau = TB == 3 ? 3 : 1;
  const int ns = d / TB;
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i >= npts * ns) return;
  const size_t x = i / ns;
  const int s = (int)(i - x * ns);
  Sv<TB> pos = s_zero<TB>(), neg = s_zero<TB>();
  if (x < N)
    for (int k = 0; k < nw; k++)
      for (int j = 0; j < tau; j++) {
        const int a = digit_of(fc[(size_t)k * wstride + x * d + (size_t)j * ns + s]);
        if (a) {
          const Sv<TB> cf = s_load<TB>(coef + (size_t)(k * tau + j) * d + s * TB);
          if (a > 0)
            pos = s_add(pos, cf);
          else
            neg = s_add(neg, cf);
        }
      }
  uint64_t *o = io + x * d + s * TB;
  s_store(o, s_add(s_load<TB>(o), s_sub(pos, neg)));
}

// w_(k,dd) = mu_k^(dd+1), the Horner weights of the folding combination
template <int TB>
__global__ void k_fold_weights(const uint64_t *mu, int nk, int tau, int d, uint64_t *w) {
  const int ns = d / TB;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;  // (k, slot)
  if (i >= nk * ns) return;
  const int k = i / ns, s = i - k * ns;
  const Sv<TB> m = s_load<TB>(mu + (size_t)k * d + s * TB);
  Sv<TB> p = m;
  for (int dd = 0; dd < tau; dd++) {
    s_store(w + ((size_t)k * tau + dd) * d + s * TB, p);
    p = s_mul(p, m);
  }
}

// The linearization polynomial (linearization/utils.rs:63-104):
//   comb = v_last * sum_i c_i prod_(j in S_i) v_j
// v_j indexes the MLE list by the matrix index j, as the reference does.
template <int TB, int DEG>
__global__ void __launch_bounds__(RT) k_round_lin(const uint64_t *mles, size_t stride, const uint64_t *const *ptrs,
                                                  int nm, const uint64_t *c, CombS cs, size_t half, int d, int spb,
                                                  uint64_t *partial) {
  const int slot_l = threadIdx.x % spb, lane_p = threadIdx.x / spb, ppb = RT / spb;
  const int slot = blockIdx.y * spb + slot_l;
  // the sum over the multisets is split over blockIdx.z chunks when the points are few
  const int chunk = blockIdx.z, nchunk = gridDim.z;
  const int i0 = (int)((long)cs.q * chunk / nchunk), i1 = (int)((long)cs.q * (chunk + 1) / nchunk);
  constexpr int degree = DEG;
  Sv<TB> acc[degree + 1];
#pragma unroll
  for (int e = 0; e <= degree; e++) acc[e] = s_zero<TB>();
  for (size_t b = (size_t)blockIdx.x * ppb + lane_p; b < half; b += (size_t)gridDim.x * ppb) {
    const size_t pofs = 2 * b * d + slot * TB;
    auto mle = [&](int m) { return (ptrs ? ptrs[m] : mles + (size_t)m * stride) + pofs; };
    const uint64_t *pe = mle(nm - 1);
    // every MLE value of a multiset is loaded once and walked along the line
    // x(e) = a + e (b - a) by additions, multiplied into all degree + 1 terms
    Sv<TB> sum[degree + 1];
#pragma unroll
    for (int e = 0; e <= degree; e++) sum[e] = s_zero<TB>();
    for (int i = i0; i < i1; i++) {
      const Sv<TB> ci = s_load<TB>(c + (size_t)i * d + slot * TB);
      if (s_is_zero(ci)) continue;  // the term vanishes in this slot
      const int s0 = cs.off[i], s1 = cs.off[i + 1];
      Sv<TB> term[degree + 1];
      if (s1 == s0) {
#pragma unroll
        for (int e = 0; e <= degree; e++) term[e] = ci;
      } else {
        // c_i times the first one or two factors in coefficient form (2 or 6
        // products instead of 9 or 18), then the values at e = 0 .. degree by
        // forward differences (additions only)
        const uint64_t *p = mle(cs.idx[s0]);
        const Sv<TB> a = s_load<TB>(p);
        const Sv<TB> u0 = s_mul(ci, a), u1 = s_mul(ci, s_sub(s_load<TB>(p + d), a));  // c_i x1(e) = u0 + u1 e
        if (s1 - s0 == 1) {
          Sv<TB> x = u0;
#pragma unroll
          for (int e = 0; e <= degree; e++) {
            term[e] = x;
            if (e < degree) x = s_add(x, u1);
          }
        } else {
          const uint64_t *q = mle(cs.idx[s0 + 1]);
          const Sv<TB> g0 = s_load<TB>(q), g1 = s_sub(s_load<TB>(q + d), g0);  // x2(e) = g0 + g1 e
          // (u0 + u1 e)(g0 + g1 e) = k0 + k1 e + k2 e^2: f(0) = k0, delta_0 = k1 + k2, second difference 2 k2
          const Sv<TB> k0 = s_mul(u0, g0), k2 = s_mul(u1, g1);
          const Sv<TB> k1 = s_add(s_mul(u0, g1), s_mul(u1, g0));
          Sv<TB> x = k0, dx = s_add(k1, k2);
          const Sv<TB> d2 = s_add(k2, k2);
#pragma unroll
          for (int e = 0; e <= degree; e++) {
            term[e] = x;
            if (e < degree) {
              x = s_add(x, dx);
              dx = s_add(dx, d2);
            }
          }
        }
      }
      for (int sx = s0 + 2 < s1 ? s0 + 2 : s1; sx < s1; sx++) {
        const uint64_t *p = mle(cs.idx[sx]);
        Sv<TB> x = s_load<TB>(p);
        const Sv<TB> st = s_sub(s_load<TB>(p + d), x);
#pragma unroll
        for (int e = 0; e <= degree; e++) {
          term[e] = s_mul(term[e], x);
          if (e < degree) x = s_add(x, st);
        }
      }
#pragma unroll
      for (int e = 0; e <= degree; e++) sum[e] = s_add(sum[e], term[e]);
    }
    Sv<TB> ev = s_load<TB>(pe);
    const Sv<TB> es = s_sub(s_load<TB>(pe + d), ev);
#pragma unroll
    for (int e = 0; e <= degree; e++) {
      acc[e] = s_add(acc[e], s_mul(sum[e], ev));
      if (e < degree) ev = s_add(ev, es);
    }
  }
  block_partial<TB, degree + 1>(acc, spb, ppb, slot, lane_p, d,
                                partial + ((size_t)blockIdx.z * gridDim.x + blockIdx.x) * (degree + 1) * d);
}

// ---------------------------------------------------------------- linearization with eq split off
// The same round polynomial with eq(beta, x) factored as eq(beta_0, X) E[b]
// (E = eq over the variables not yet bound, a constant along each line):
//   p(X) = P eq(beta_0, X) q(X),  q(X) = sum_b E[b] sum_i c_i prod_(j in S_i) m_j(X, b)
// q has one degree less than p, so NQ = degree values q(0 .. NQ-1) suffice; the
// host extrapolates q(NQ) and multiplies in the eq factors (sumcheck_run_lin,
// lf_api.hip). p(e) is the same field element either way, so the messages are
// the reference's (prover.rs:62-168 over linearization/utils.rs:63-104).
//
// A multiset's product c_i prod_f (a_f + d_f e) is formed in two groups in
// coefficient form (c_i and the first KA factors; the other KB), each walked
// along e = 0 .. NQ-1 by forward differences, and the groups multiplied
// pointwise: for |S_i| = 7 that is 20 + 10 + 8 products instead of 6 + 5 x 9.

// c <- c (a + d e) for a degree-M polynomial in coefficient form (in place, from the top;
// each new coefficient one lazy multiply-accumulate pair)
template <int TB, int M>
__device__ __forceinline__ void poly_mul_lin(Sv<TB> (&c)[5], const Sv<TB> &a, const Sv<TB> &dd) {
  c[M + 1] = s_mul(c[M], dd);
#pragma unroll
  for (int j = M; j >= 1; j--) c[j] = s_mad2(c[j], a, c[j - 1], dd);
  c[0] = s_mul(c[0], a);
}

// coefficients -> the forward-difference table at e = 0: D_j = sum_k c_k j! S(k, j)
//   D1 = c1 + c2 + c3 + c4, D2 = 2 c2 + 6 c3 + 14 c4, D3 = 6 c3 + 36 c4, D4 = 24 c4
template <int TB, int M>
__device__ __forceinline__ void poly_to_diff(Sv<TB> (&c)[5]) {
  if constexpr (M == 1) return;
  if constexpr (M == 2) {
    c[1] = s_add(c[1], c[2]);
    c[2] = s_add(c[2], c[2]);
  }
  if constexpr (M == 3) {
    const Sv<TB> c3x6 = s_smul(c[3], 6);
    c[1] = s_add(s_add(c[1], c[2]), c[3]);
    c[2] = s_add(s_add(c[2], c[2]), c3x6);
    c[3] = c3x6;
  }
  if constexpr (M == 4) {
    const Sv<TB> c3x6 = s_smul(c[3], 6);
    c[1] = s_add(s_add(c[1], c[2]), s_add(c[3], c[4]));
    c[2] = s_add(s_add(s_add(c[2], c[2]), c3x6), s_smul(c[4], 14));
    c[3] = s_add(c3x6, s_smul(c[4], 36));
    c[4] = s_smul(c[4], 24);
  }
}

template <int TB, int M>
__device__ __forceinline__ void diff_step(Sv<TB> (&c)[5]) {
#pragma unroll
  for (int j = 0; j < M; j++) c[j] = s_add(c[j], c[j + 1]);
}

// sum[e] += c_i prod_(f < KA + KB) (a_f + d_f e), e < NQ; fac(f, a, d) loads factor f
template <int TB, int NQ, int KA, int KB, class Fac>
__device__ __forceinline__ void multiset_add(const Sv<TB> &ci, Fac fac, Sv<TB> (&sum)[NQ]) {
  Sv<TB> A[5], B[5], a, dd;
  fac(0, a, dd);
  A[0] = s_mul(ci, a);
  A[1] = s_mul(ci, dd);
#pragma unroll
  for (int f = 1; f < KA; f++) {
    __builtin_amdgcn_sched_barrier(0);  // one factor's loads and products at a time (registers)
    fac(f, a, dd);
    if (f == 1) poly_mul_lin<TB, 1>(A, a, dd);
    if (f == 2) poly_mul_lin<TB, 2>(A, a, dd);
    if (f == 3) poly_mul_lin<TB, 3>(A, a, dd);
  }
  poly_to_diff<TB, KA>(A);
  if constexpr (KB == 0) {
#pragma unroll
    for (int e = 0; e < NQ; e++) {
      sum[e] = s_add(sum[e], A[0]);
      if (e + 1 < NQ) diff_step<TB, KA>(A);
    }
  } else {
    __builtin_amdgcn_sched_barrier(0);
    fac(KA, B[0], B[1]);
#pragma unroll
    for (int f = 1; f < KB; f++) {
      __builtin_amdgcn_sched_barrier(0);
      fac(KA + f, a, dd);
      if (f == 1) poly_mul_lin<TB, 1>(B, a, dd);
      if (f == 2) poly_mul_lin<TB, 2>(B, a, dd);
      if (f == 3) poly_mul_lin<TB, 3>(B, a, dd);
    }
    poly_to_diff<TB, KB>(B);
#pragma unroll
    for (int e = 0; e < NQ; e++) {
      __builtin_amdgcn_sched_barrier(0);
      sum[e] = s_add(sum[e], s_mul(A[0], B[0]));
      if (e + 1 < NQ) {
        diff_step<TB, KA>(A);
        diff_step<TB, KB>(B);
      }
    }
  }
}

template <int TB, int NQ>
__global__ void __launch_bounds__(RT) k_round_lin_eq(const uint64_t *mles, size_t stride, const uint64_t *const *ptrs,
                                                     const uint64_t *E, const uint64_t *c, CombS cs, size_t half, int d,
                                                     int spb, uint64_t *partial) {
  const int slot_l = threadIdx.x % spb, lane_p = threadIdx.x / spb, ppb = RT / spb;
  const int slot = blockIdx.y * spb + slot_l;
  const int chunk = blockIdx.z, nchunk = gridDim.z;
  const int i0 = (int)((long)cs.q * chunk / nchunk), i1 = (int)((long)cs.q * (chunk + 1) / nchunk);
  // the per-thread sums over points live in LDS (word w of value e at [e TB + w][thread]),
  // which leaves the registers to the multiset products
  __shared__ uint64_t lacc[NQ * TB * RT];
#pragma unroll
  for (int k = 0; k < NQ * TB; k++) lacc[k * RT + threadIdx.x] = 0;
  for (size_t b = (size_t)blockIdx.x * ppb + lane_p; b < half; b += (size_t)gridDim.x * ppb) {
    const size_t pofs = 2 * b * d + slot * TB;
    Sv<TB> sum[NQ];
#pragma unroll
    for (int e = 0; e < NQ; e++) sum[e] = s_zero<TB>();
    for (int i = i0; i < i1; i++) {
      // no per-slot zero test: a branch on c_i would make the multiset loop divergent
      // and move the (uniform) multiset indices and MLE pointers into vector registers
      const Sv<TB> ci = s_load<TB>(c + (size_t)i * d + slot * TB);
      const int s0 = cs.off[i], k = cs.off[i + 1] - s0;
      auto fac = [&](int f, Sv<TB> &a, Sv<TB> &dd) {
        const int m = cs.idx[s0 + f];
        const uint64_t *p = (ptrs ? ptrs[m] : mles + (size_t)m * stride) + pofs;
        a = s_load<TB>(p);
        dd = s_sub(s_load<TB>(p + d), a);
      };
      if (k == 0) {
#pragma unroll
        for (int e = 0; e < NQ; e++) sum[e] = s_add(sum[e], ci);
      } else if (k == 1) {
        multiset_add<TB, NQ, 1, 0>(ci, fac, sum);
      } else if (k == 2) {
        multiset_add<TB, NQ, 2, 0>(ci, fac, sum);
      } else {
        // c_i and the first two factors in coefficient form, walked along e by
        // differences; every further factor multiplied in at the NQ points
        Sv<TB> term[NQ], A[5], a, dd;
        fac(0, a, dd);
        A[0] = s_mul(ci, a);
        A[1] = s_mul(ci, dd);
        fac(1, a, dd);
        poly_mul_lin<TB, 1>(A, a, dd);
        poly_to_diff<TB, 2>(A);
#pragma unroll
        for (int e = 0; e < NQ; e++) {
          term[e] = A[0];
          if (e + 1 < NQ) diff_step<TB, 2>(A);
        }
        for (int f = 2; f < k; f++) {
          fac(f, a, dd);
#pragma unroll
          for (int e = 0; e < NQ; e++) {
            term[e] = s_mul_w(term[e], a);  // weakly reduced along the chain
            if (e + 1 < NQ) a = s_add(a, dd);
          }
        }
#pragma unroll
        for (int e = 0; e < NQ; e++) sum[e] = s_add(sum[e], s_canon(term[e]));
      }
    }
    const Sv<TB> w = s_load<TB>(E + b * d + slot * TB);
#pragma unroll
    for (int e = 0; e < NQ; e++) {
      const Sv<TB> v = s_mul(sum[e], w);
#pragma unroll
      for (int k = 0; k < TB; k++) {
        uint64_t &a = lacc[(e * TB + k) * RT + threadIdx.x];
        a = gl::add(a, v.c[k]);
      }
    }
  }
  Sv<TB> acc[NQ];
#pragma unroll
  for (int e = 0; e < NQ; e++)
#pragma unroll
    for (int k = 0; k < TB; k++) acc[e].c[k] = lacc[(e * TB + k) * RT + threadIdx.x];
  block_partial<TB, NQ>(acc, spb, ppb, slot, lane_p, d,
                        partial + ((size_t)blockIdx.z * gridDim.x + blockIdx.x) * NQ * d);
}

// Round 0 of the split-eq linearization over each multiset's active points only: a
// point b whose line (rows 2b, 2b + 1) is identically zero in some factor of S_i has a
// zero term at every e (the reference's zero short-cut, linearization/utils.rs:86-104
// skips such products), and which lines are identically zero is fixed by the CCS rows
// alone. Block g works on multiset bms[g] and its active points act[boff[g] ..
// boff[g] + PPB ST) (ST points per thread, strided); E[b] is folded into c_i (one
// product per term instead of NQ at the end). partial[g][e][slot].
template <int TB, int NQ>
__global__ void __launch_bounds__(RT) k_round_lin_eq_sparse(const uint64_t *const *ptrs, const uint64_t *E,
                                                            const uint64_t *c, CombS cs, const uint32_t *act,
                                                            const int *bms, const uint32_t *boff, const uint32_t *bend,
                                                            int d, int spb, uint64_t *partial) {
  const int slot_l = threadIdx.x % spb, lane_p = threadIdx.x / spb, ppb = RT / spb;
  const int slot = blockIdx.y * spb + slot_l;
  const int i = bms[blockIdx.x];
  const uint32_t p0 = boff[blockIdx.x], p1 = bend[blockIdx.x];
  const int s0 = cs.off[i], k = cs.off[i + 1] - s0;
  Sv<TB> acc[NQ];
#pragma unroll
  for (int e = 0; e < NQ; e++) acc[e] = s_zero<TB>();
  const Sv<TB> ci0 = s_load<TB>(c + (size_t)i * d + slot * TB);
  for (uint32_t p = p0 + lane_p; p < p1; p += ppb) {
    const size_t b = act[p], pofs = 2 * b * d + slot * TB;
    const Sv<TB> ci = s_mul(ci0, s_load<TB>(E + b * d + slot * TB));
    auto fac = [&](int f, Sv<TB> &a, Sv<TB> &dd) {
      const uint64_t *q = ptrs[cs.idx[s0 + f]] + pofs;
      a = s_load<TB>(q);
      dd = s_sub(s_load<TB>(q + d), a);
    };
    if (k == 0) {
#pragma unroll
      for (int e = 0; e < NQ; e++) acc[e] = s_add(acc[e], ci);
    } else if (k == 1) {
      multiset_add<TB, NQ, 1, 0>(ci, fac, acc);
    } else if (k == 2) {
      multiset_add<TB, NQ, 2, 0>(ci, fac, acc);
    } else {
      Sv<TB> term[NQ], A[5], a, dd;
      fac(0, a, dd);
      A[0] = s_mul(ci, a);
      A[1] = s_mul(ci, dd);
      fac(1, a, dd);
      poly_mul_lin<TB, 1>(A, a, dd);
      poly_to_diff<TB, 2>(A);
#pragma unroll
      for (int e = 0; e < NQ; e++) {
        term[e] = A[0];
        if (e + 1 < NQ) diff_step<TB, 2>(A);
      }
      for (int f = 2; f < k; f++) {
        fac(f, a, dd);
#pragma unroll
        for (int e = 0; e < NQ; e++) {
          term[e] = s_mul_w(term[e], a);  // weakly reduced along the chain
          if (e + 1 < NQ) a = s_add(a, dd);
        }
      }
#pragma unroll
      for (int e = 0; e < NQ; e++) acc[e] = s_add(acc[e], s_canon(term[e]));
    }
  }
  block_partial<TB, NQ>(acc, spb, ppb, slot, lane_p, d, partial + (size_t)blockIdx.x * NQ * d);
}

// The same sums for rounds with few points (late rounds): one thread per (point, slot,
// multiset chunk, evaluation point e), so a thread multiplies |S_i| + 1 values instead
// of walking all NQ points of a multiset (the chain of dependent products, not the
// work, bounds those rounds). partial[(chunk gx + x) NQ + e][slot]
template <int TB>
__global__ void __launch_bounds__(RT) k_round_lin_eq_pt(const uint64_t *mles, size_t stride,
                                                        const uint64_t *const *ptrs, const uint64_t *E,
                                                        const uint64_t *c, CombS cs, size_t half, int d, int spb,
                                                        int nq, uint64_t *partial) {
  const int slot_l = threadIdx.x % spb, lane_p = threadIdx.x / spb, ppb = RT / spb;
  const int slot = blockIdx.y * spb + slot_l;
  const int e = blockIdx.z % nq, chunk = blockIdx.z / nq, nchunk = gridDim.z / nq;
  const int i0 = (int)((long)cs.q * chunk / nchunk), i1 = (int)((long)cs.q * (chunk + 1) / nchunk);
  Sv<TB> acc[1];
  acc[0] = s_zero<TB>();
  for (size_t b = (size_t)blockIdx.x * ppb + lane_p; b < half; b += (size_t)gridDim.x * ppb) {
    const size_t pofs = 2 * b * d + slot * TB;
    Sv<TB> sum = s_zero<TB>();
    for (int i = i0; i < i1; i++) {
      Sv<TB> term = s_load<TB>(c + (size_t)i * d + slot * TB);
      for (int f = cs.off[i]; f < cs.off[i + 1]; f++) {
        const int m = cs.idx[f];
        const uint64_t *p = (ptrs ? ptrs[m] : mles + (size_t)m * stride) + pofs;
        const Sv<TB> a = s_load<TB>(p);
        const Sv<TB> x = s_add(a, s_smul(s_sub(s_load<TB>(p + d), a), (uint64_t)e));  // a + e (b - a)
        term = s_mul(term, x);
      }
      sum = s_add(sum, term);
    }
    acc[0] = s_add(acc[0], s_mul(sum, s_load<TB>(E + b * d + slot * TB)));
  }
  block_partial<TB, 1>(acc, spb, ppb, slot, lane_p, d,
                       partial + (((size_t)chunk * gridDim.x + blockIdx.x) * nq + e) * d);
}

// E_next[b] = E[2b] + E[2b + 1]: eq over one variable fewer (eq(beta, 0) + eq(beta, 1) = 1)
__global__ void k_pair_sum(const uint64_t *in, size_t half, int d, uint64_t *out) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i >= half * d) return;
  const size_t b = i / d, w = i - b * d;
  out[i] = gl::add(in[2 * b * d + w], in[(2 * b + 1) * d + w]);
}

// out[i] = sum over blocks of partial[blk][i]: one block per output word,
// its threads striding over the blocks, then an LDS tree
__global__ void __launch_bounds__(256) k_sum_partials(const uint64_t *partial, int nblk, size_t len, uint64_t *out) {
  __shared__ uint64_t red[256];
  const size_t i = blockIdx.x;
  uint64_t s = 0;
  for (int b = threadIdx.x; b < nblk; b += 256) s = gl::add(s, partial[(size_t)b * len + i]);
  red[threadIdx.x] = s;
  __syncthreads();
  for (int h = 128; h > 0; h >>= 1) {
    if ((int)threadIdx.x < h) red[threadIdx.x] = gl::add(red[threadIdx.x], red[threadIdx.x + h]);
    __syncthreads();
  }
  if (threadIdx.x == 0) out[i] = red[0];
}

// ---------------------------------------------------------------- MLE evaluation
// evaluate (dense.rs:107-113) = sum_x eq(point, x) mle(x): partial sums over x
// ranges, out[m] from k_sum_partials over the ranges
template <int TB>
__global__ void __launch_bounds__(RT) k_mle_dot(const uint64_t *mles, size_t stride, const uint64_t *eq, size_t n,
                                                int d, int spb, int nsplit, uint64_t *partial, int nm) {
  const int slot_l = threadIdx.x % spb, lane_p = threadIdx.x / spb, ppb = RT / spb;
  const int slot = blockIdx.y * spb + slot_l;
  const int m = blockIdx.z;
  SAcc<TB> la;
  sacc_zero(la);
  for (size_t x = (size_t)blockIdx.x * ppb + lane_p; x < n; x += (size_t)nsplit * ppb)
    sacc_mad(la, s_load<TB>(eq + x * d + slot * TB), s_load<TB>(mles + m * stride + x * d + slot * TB));
  const Sv<TB> acc[1] = {sacc_final(la)};
  block_partial<TB, 1>(acc, spb, ppb, slot, lane_p, d, partial + ((size_t)blockIdx.x * nm + m) * d);
}

// evaluate_mles of Witness::get_fhat's MLEs straight from the coefficient rows
// (no materialised f_hat): the value of MLE j at point x < N, slot s, is the
// base-ring scalar f_coeff[x][j NS + s] (zero past N), so
// out[w][j] = sum_x eq[x] (.) fhat_wj[x]; blockIdx.z = w tau + j
template <int TB>
__global__ void __launch_bounds__(RT) k_fhat_dot(const uint64_t *fc, size_t N, size_t wstride, const uint64_t *eq,
                                                 size_t n, int d, int spb, int nsplit, uint64_t *partial, int nm) {
  const int slot_l = threadIdx.x % spb, lane_p = threadIdx.x / spb, ppb = RT / spb;
  const int slot = blockIdx.y * spb + slot_l, ns = d / TB, tau = TB == 3 ? 3 : 1;
  const int m = blockIdx.z, w = m / tau, j = m - w * tau;
  const uint64_t *f = fc + (size_t)w * wstride + (size_t)j * ns + slot;
  SAcc<TB> la;
  sacc_zero(la);
  for (size_t x = (size_t)blockIdx.x * ppb + lane_p; x < n && x < N; x += (size_t)nsplit * ppb)
    sacc_mad(la, s_load<TB>(eq + x * d + slot * TB), s_scalar<TB>(f[x * d]));
  const Sv<TB> acc[1] = {sacc_final(la)};
  block_partial<TB, 1>(acc, spb, ppb, slot, lane_p, d, partial + ((size_t)blockIdx.x * nm + m) * d);
}

// io[x] += sum_m coef[m] (.) mles[m][x] for the n points (one thread per point and slot)
template <int TB>
__global__ void __launch_bounds__(256) k_mle_lincomb(const uint64_t *mles, size_t stride, int nm, const uint64_t *coef,
                                                     size_t n, int d, uint64_t *io) {
  const int ns = d / TB;
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i >= n * ns) return;
  const size_t x = i / ns;
  const int s = (int)(i - x * ns);
  SAcc<TB> la;
  sacc_zero(la);
  for (int m = 0; m < nm; m++)
    sacc_mad(la, s_load<TB>(coef + (size_t)m * d + s * TB), s_load<TB>(mles + m * stride + x * d + s * TB));
  uint64_t *o = io + x * d + s * TB;
  s_store(o, s_add(s_load<TB>(o), sacc_final(la)));
}

unsigned blocks_of(size_t n, int t) { return (unsigned)((n + t - 1) / t); }

template <int TB>
hipError_t dispatch_eq(const uint64_t *r, int nv, int d, uint64_t *out, hipStream_t st) {
  const size_t n = ((size_t)(d / TB)) << nv;
  hipLaunchKernelGGL(k_eq_table<TB>, dim3(blocks_of(n, 256)), dim3(256), 0, st, r, nv, d, out);
  return hipGetLastError();
}

}  // namespace

int slot_words(int d) { return d == 24 ? 3 : 1; }

hipError_t eq_table(const uint64_t *r, int nv, int d, uint64_t *out, hipStream_t st) {
  if (nv < 1 || nv > 40) return hipErrorInvalidValue;
  return d == 24 ? dispatch_eq<3>(r, nv, d, out, st) : dispatch_eq<1>(r, nv, d, out, st);
}

hipError_t mle_fix_first(const uint64_t *in, size_t in_stride, int nm, size_t half, int d, const uint64_t *r_base,
                         uint64_t *out, size_t out_stride, hipStream_t st, const uint64_t *const *ptrs) {
  const int tb = slot_words(d);
  const size_t n = (size_t)nm * half * (d / tb);
  if (!n) return hipSuccess;
  if (tb == 3) {
    Sv<3> r;
    for (int i = 0; i < 3; i++) r.c[i] = r_base[i];
    hipLaunchKernelGGL(k_fix_first<3>, dim3(blocks_of(n, 256)), dim3(256), 0, st, in, in_stride, ptrs, nm, half, d, r,
                       out, out_stride);
  } else {
    Sv<1> r;
    r.c[0] = r_base[0];
    hipLaunchKernelGGL(k_fix_first<1>, dim3(blocks_of(n, 256)), dim3(256), 0, st, in, in_stride, ptrs, nm, half, d, r,
                       out, out_stride);
  }
  return hipGetLastError();
}

// the round-sum launch geometry: spb slots per block (all of a Phi_72
// element's 8, or up to 256 of X^d + 1), enough blocks for the points, and --
// when the points are too few to fill the chip (late rounds) -- the f_hat
// MLEs split over up to `nf` chunks (grid.z)
constexpr size_t FILL_THREADS = (size_t)1 << 18;
// at or below this many (point, slot) threads the linearization round runs per evaluation point
constexpr size_t PT_THREADS = (size_t)1 << 13;
static void round_geom(int d, size_t half, int nf, int &spb, dim3 &grid) {
  const int ns = d / slot_words(d);
  spb = ns < RT ? ns : RT;
  const int ppb = RT / spb;
  size_t bx = (half + ppb - 1) / ppb;
  const size_t cap = 1024;  // partial sums: at most this many blocks along the points
  if (bx > cap) bx = cap;
  if (bx < 1) bx = 1;
  size_t nchunk = 1;
  const size_t threads = half * (size_t)ns;
  if (nf > 1 && threads < FILL_THREADS) {
    nchunk = (FILL_THREADS + threads - 1) / threads;
    if (nchunk > (size_t)nf) nchunk = nf;
  }
  grid = dim3((unsigned)bx, (unsigned)(ns / spb), (unsigned)nchunk);
}
size_t round_partial_elems(int d, size_t half, int nevals, int nf) {
  int spb;
  dim3 g;
  round_geom(d, half, nf, spb, g);
  return (size_t)g.x * g.z * nevals * d;
}

hipError_t fold_weights(const uint64_t *mu, int nk, int tau, int d, uint64_t *w, hipStream_t st) {
  const int tb = slot_words(d), n = nk * (d / tb);
  if (tb == 3)
    hipLaunchKernelGGL(k_fold_weights<3>, dim3(blocks_of(n, 256)), dim3(256), 0, st, mu, nk, tau, d, w);
  else
    hipLaunchKernelGGL(k_fold_weights<1>, dim3(blocks_of(n, 256)), dim3(256), 0, st, mu, nk, tau, d, w);
  return hipGetLastError();
}

hipError_t round_folding(const uint64_t *mles, size_t stride, int nf, const uint64_t *w, int bsmall, size_t half, int d,
                         uint64_t *partial, uint64_t *evals, hipStream_t st) {
  if (bsmall < 1 || bsmall > 4 || !half) return hipErrorInvalidValue;
  int spb;
  dim3 grid;
  round_geom(d, half, nf, spb, grid);
#define LF_RF(TB, BS)                                                                                           \
  hipLaunchKernelGGL((k_round_folding<TB, BS>), grid, dim3(RT), 0, st, mles, stride, nf, w, half, d, spb, partial)
#define LF_RF_BS(TB)          \
  switch (bsmall) {           \
    case 1: LF_RF(TB, 1); break; \
    case 2: LF_RF(TB, 2); break; \
    case 3: LF_RF(TB, 3); break; \
    default: LF_RF(TB, 4); break; \
  }
  if (slot_words(d) == 3) {
    LF_RF_BS(3)
  } else {
    LF_RF_BS(1)
  }
#undef LF_RF_BS
#undef LF_RF
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const size_t len = (size_t)(2 * bsmall + 1) * d;
  hipLaunchKernelGGL(k_sum_partials, dim3((unsigned)len), dim3(256), 0, st, partial, (int)(grid.x * grid.z), len,
                     evals);
  return hipGetLastError();
}

hipError_t round_folding0_digits(const uint64_t *mles, size_t stride, const uint64_t *fc0, const uint64_t *fc1, int K,
                                size_t N, size_t wstride, int nf, const uint64_t *w, size_t half, int d,
                                uint64_t *partial, uint64_t *evals, hipStream_t st) {
  if (!half) return hipErrorInvalidValue;
  int spb;
  dim3 grid;
  round_geom(d, half, nf, spb, grid);
  if (slot_words(d) == 3)
    hipLaunchKernelGGL(k_round_folding0_digits<3>, grid, dim3(RT), 0, st, mles, stride, fc0, fc1, K, N, wstride, nf, w,
                       half, d, spb, partial);
  else
    hipLaunchKernelGGL(k_round_folding0_digits<1>, grid, dim3(RT), 0, st, mles, stride, fc0, fc1, K, N, wstride, nf, w,
                       half, d, spb, partial);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const size_t len = (size_t)5 * d;
  hipLaunchKernelGGL(k_sum_partials, dim3((unsigned)len), dim3(256), 0, st, partial, (int)(grid.x * grid.z), len,
                     evals);
  return hipGetLastError();
}

hipError_t fix_fhat_digits(const uint64_t *fc0, const uint64_t *fc1, int K, size_t N, size_t wstride, int nf,
                           size_t half, int d, const uint64_t *r_base, uint64_t *out, size_t out_stride,
                           hipStream_t st) {
  const int tb = slot_words(d);
  const size_t n = (size_t)nf * half * (d / tb);
  if (!n) return hipSuccess;
  if (tb == 3) {
    Sv<3> r;
    for (int i = 0; i < 3; i++) r.c[i] = r_base[i];
    hipLaunchKernelGGL(k_fix_fhat_digits<3>, dim3(blocks_of(n, 256)), dim3(256), 0, st, fc0, fc1, K, N, wstride, nf,
                       half, d, r, out, out_stride);
  } else {
    Sv<1> r;
    r.c[0] = r_base[0];
    hipLaunchKernelGGL(k_fix_fhat_digits<1>, dim3(blocks_of(n, 256)), dim3(256), 0, st, fc0, fc1, K, N, wstride, nf,
                       half, d, r, out, out_stride);
  }
  return hipGetLastError();
}

hipError_t fhat_lincomb_digits(const uint64_t *fc, int nw, size_t N, size_t wstride, const uint64_t *coef, int nv,
                               int d, uint64_t *io, hipStream_t st) {
  const size_t npts = (size_t)1 << nv, n = npts * (size_t)(d / slot_words(d));
  if (slot_words(d) == 3)
    hipLaunchKernelGGL(k_fhat_lincomb_digits<3>, dim3(blocks_of(n, 256)), dim3(256), 0, st, fc, nw, N, wstride, coef,
                       npts, d, io);
  else
    hipLaunchKernelGGL(k_fhat_lincomb_digits<1>, dim3(blocks_of(n, 256)), dim3(256), 0, st, fc, nw, N, wstride, coef,
                       npts, d, io);
  return hipGetLastError();
}

hipError_t round_lin(const uint64_t *mles, size_t stride, int nm, const uint64_t *c, const CombS &cs, int degree,
                     size_t half, int d, uint64_t *partial, uint64_t *evals, hipStream_t st,
                     const uint64_t *const *ptrs) {
  if (degree + 1 > MAX_EVALS || degree < 1 || !half) return hipErrorInvalidValue;
  int spb;
  dim3 grid;
  round_geom(d, half, cs.q, spb, grid);
#define LF_RL(TB, DG) \
  hipLaunchKernelGGL((k_round_lin<TB, DG>), grid, dim3(RT), 0, st, mles, stride, ptrs, nm, c, cs, half, d, spb, partial)
#define LF_RL_DEG(TB)                          \
  switch (degree) {                            \
    case 1: LF_RL(TB, 1); break;               \
    case 2: LF_RL(TB, 2); break;               \
    case 3: LF_RL(TB, 3); break;               \
    case 4: LF_RL(TB, 4); break;               \
    case 5: LF_RL(TB, 5); break;               \
    case 6: LF_RL(TB, 6); break;               \
    case 7: LF_RL(TB, 7); break;               \
    case 8: LF_RL(TB, 8); break;               \
    default: LF_RL(TB, 9); break;              \
  }
  if (slot_words(d) == 3) {
    LF_RL_DEG(3)
  } else {
    LF_RL_DEG(1)
  }
#undef LF_RL_DEG
#undef LF_RL
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const size_t len = (size_t)(degree + 1) * d;
  hipLaunchKernelGGL(k_sum_partials, dim3((unsigned)len), dim3(256), 0, st, partial, (int)(grid.x * grid.z), len,
                     evals);
  return hipGetLastError();
}

hipError_t round_lin_eq(const uint64_t *mles, size_t stride, const uint64_t *E, const uint64_t *c, const CombS &cs,
                        int degree, size_t half, int d, uint64_t *partial, uint64_t *evals, hipStream_t st,
                        const uint64_t *const *ptrs) {
  if (degree + 1 > MAX_EVALS || degree < 1 || !half) return hipErrorInvalidValue;
  int spb;
  dim3 grid;
  round_geom(d, half, cs.q, spb, grid);
  if (half * (size_t)(d / slot_words(d)) <= PT_THREADS) {  // few points: a thread per (point, slot, chunk, e)
    const dim3 g2(grid.x, grid.y, grid.z * degree);
    if (slot_words(d) == 3)
      hipLaunchKernelGGL(k_round_lin_eq_pt<3>, g2, dim3(RT), 0, st, mles, stride, ptrs, E, c, cs, half, d, spb, degree,
                         partial);
    else
      hipLaunchKernelGGL(k_round_lin_eq_pt<1>, g2, dim3(RT), 0, st, mles, stride, ptrs, E, c, cs, half, d, spb, degree,
                         partial);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const size_t len = (size_t)degree * d;
    hipLaunchKernelGGL(k_sum_partials, dim3((unsigned)len), dim3(256), 0, st, partial, (int)(grid.x * grid.z), len,
                       evals);
    return hipGetLastError();
  }
#define LF_RLE(TB, NQ)                                                                                      \
  hipLaunchKernelGGL((k_round_lin_eq<TB, NQ>), grid, dim3(RT), 0, st, mles, stride, ptrs, E, c, cs, half, d, spb, \
                     partial)
#define LF_RLE_DEG(TB)                \
  switch (degree) {                   \
    case 1: LF_RLE(TB, 1); break;     \
    case 2: LF_RLE(TB, 2); break;     \
    case 3: LF_RLE(TB, 3); break;     \
    case 4: LF_RLE(TB, 4); break;     \
    case 5: LF_RLE(TB, 5); break;     \
    case 6: LF_RLE(TB, 6); break;     \
    case 7: LF_RLE(TB, 7); break;     \
    case 8: LF_RLE(TB, 8); break;     \
    default: LF_RLE(TB, 9); break;    \
  }
  if (slot_words(d) == 3) {
    LF_RLE_DEG(3)
  } else {
    LF_RLE_DEG(1)
  }
#undef LF_RLE_DEG
#undef LF_RLE
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const size_t len = (size_t)degree * d;
  hipLaunchKernelGGL(k_sum_partials, dim3((unsigned)len), dim3(256), 0, st, partial, (int)(grid.x * grid.z), len,
                     evals);
  return hipGetLastError();
}

hipError_t round_lin_eq_sparse(const uint64_t *const *ptrs, const uint64_t *E, const uint64_t *c, const CombS &cs,
                               int degree, const uint32_t *act, const int *bms, const uint32_t *boff,
                               const uint32_t *bend, int nblk, int d, uint64_t *partial, uint64_t *evals,
                               hipStream_t st) {
  if (degree + 1 > MAX_EVALS || degree < 1 || nblk < 1) return hipErrorInvalidValue;
  const int ns = d / slot_words(d), spb = ns < RT ? ns : RT;
  const dim3 grid((unsigned)nblk, (unsigned)(ns / spb), 1);
#define LF_RLS(TB, NQ)                                                                                          \
  hipLaunchKernelGGL((k_round_lin_eq_sparse<TB, NQ>), grid, dim3(RT), 0, st, ptrs, E, c, cs, act, bms, boff, bend, \
                     d, spb, partial)
#define LF_RLS_DEG(TB)                \
  switch (degree) {                   \
    case 1: LF_RLS(TB, 1); break;     \
    case 2: LF_RLS(TB, 2); break;     \
    case 3: LF_RLS(TB, 3); break;     \
    case 4: LF_RLS(TB, 4); break;     \
    case 5: LF_RLS(TB, 5); break;     \
    case 6: LF_RLS(TB, 6); break;     \
    case 7: LF_RLS(TB, 7); break;     \
    case 8: LF_RLS(TB, 8); break;     \
    default: LF_RLS(TB, 9); break;    \
  }
  if (slot_words(d) == 3) {
    LF_RLS_DEG(3)
  } else {
    LF_RLS_DEG(1)
  }
#undef LF_RLS_DEG
#undef LF_RLS
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const size_t len = (size_t)degree * d;
  hipLaunchKernelGGL(k_sum_partials, dim3((unsigned)len), dim3(256), 0, st, partial, nblk, len, evals);
  return hipGetLastError();
}
size_t round_lin_sparse_ppb(int d) {
  const int ns = d / slot_words(d);
  return RT / (ns < RT ? ns : RT);
}

hipError_t pair_sum(const uint64_t *E, size_t half, int d, uint64_t *out, hipStream_t st) {
  const size_t n = half * d;
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_pair_sum, dim3(blocks_of(n, 256)), dim3(256), 0, st, E, half, d, out);
  return hipGetLastError();
}

size_t mle_eval_partial_elems(int d, int nm) { return (size_t)64 * nm * d; }

hipError_t mle_dot(const uint64_t *mles, size_t stride, int nm, const uint64_t *eq, size_t n, int d,
                   uint64_t *partial, uint64_t *out, hipStream_t st) {
  if (!nm || !n) return hipSuccess;
  const int tb = slot_words(d), ns = d / tb;
  const int spb = ns < RT ? ns : RT, ppb = RT / spb;
  size_t sx = (n + ppb - 1) / ppb;
  const int nsplit = (int)(sx < 64 ? sx : 64);
  const dim3 grid((unsigned)nsplit, (unsigned)(ns / spb), (unsigned)nm);
  if (tb == 3)
    hipLaunchKernelGGL(k_mle_dot<3>, grid, dim3(RT), 0, st, mles, stride, eq, n, d, spb, nsplit, partial, nm);
  else
    hipLaunchKernelGGL(k_mle_dot<1>, grid, dim3(RT), 0, st, mles, stride, eq, n, d, spb, nsplit, partial, nm);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const size_t len = (size_t)nm * d;
  hipLaunchKernelGGL(k_sum_partials, dim3((unsigned)len), dim3(256), 0, st, partial, nsplit, len, out);
  return hipGetLastError();
}

hipError_t fhat_dot(const uint64_t *fc, size_t N, size_t wstride, int nw, const uint64_t *eq, size_t n, int d,
                    uint64_t *partial, uint64_t *out, hipStream_t st) {
  const int tb = slot_words(d), ns = d / tb, tau = tb == 3 ? 3 : 1, nm = nw * tau;
  if (!nw || !n) return hipSuccess;
  const int spb = ns < RT ? ns : RT, ppb = RT / spb;
  size_t sx = (n + ppb - 1) / ppb;
  const int nsplit = (int)(sx < 64 ? sx : 64);
  const dim3 grid((unsigned)nsplit, (unsigned)(ns / spb), (unsigned)nm);
  if (tb == 3)
    hipLaunchKernelGGL(k_fhat_dot<3>, grid, dim3(RT), 0, st, fc, N, wstride, eq, n, d, spb, nsplit, partial, nm);
  else
    hipLaunchKernelGGL(k_fhat_dot<1>, grid, dim3(RT), 0, st, fc, N, wstride, eq, n, d, spb, nsplit, partial, nm);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const size_t len = (size_t)nm * d;
  hipLaunchKernelGGL(k_sum_partials, dim3((unsigned)len), dim3(256), 0, st, partial, nsplit, len, out);
  return hipGetLastError();
}

hipError_t mle_lincomb(const uint64_t *mles, size_t stride, int nm, const uint64_t *coef, size_t n, int d,
                       uint64_t *io, hipStream_t st) {
  if (!nm || !n) return hipSuccess;
  const int tb = slot_words(d);
  const size_t nt = n * (size_t)(d / tb);
  if (tb == 3)
    hipLaunchKernelGGL(k_mle_lincomb<3>, dim3(blocks_of(nt, 256)), dim3(256), 0, st, mles, stride, nm, coef, n, d, io);
  else
    hipLaunchKernelGGL(k_mle_lincomb<1>, dim3(blocks_of(nt, 256)), dim3(256), 0, st, mles, stride, nm, coef, n, d, io);
  return hipGetLastError();
}

// ---------------------------------------------------------------- f_hat
// Witness::get_fhat (LF/arith.rs:273-297): MLE j of a witness holds, at point
// i < N, the NTT element whose slot s is coefficient j D + s of f_coeff[i] as a
// base-ring value (Phi_72: (c, 0, 0) in an Fq3 slot, D = 8 slots; X^d + 1:
// tau = 1, the coefficients themselves); points N .. 2^nv - 1 are zero (the
// reference's truncated MLE read as zero padding). One thread per output word.
__global__ void k_get_fhat(const uint64_t *f_coeff, size_t N, size_t wstride, int d, size_t npts, size_t per,
                           size_t total, uint64_t *out) {
  const size_t t0 = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (t0 >= total) return;
  const size_t wi = t0 / per, t = t0 - wi * per;  // witness wi, word t of its tau MLEs
  const uint64_t *fc = f_coeff + wi * wstride;
  const size_t w = t % d, ji = t / d, i = ji % npts;
  const int j = (int)(ji / npts);
  uint64_t v = 0;
  if (i < N) {
    if (d == 24)
      v = w % 3 == 0 ? fc[i * 24 + 8 * j + w / 3] : 0;
    else
      v = fc[i * d + w];
  }
  out[t0] = v;
}

// z_k = x_s[k] || w_ccs_k for nz instances (compute_mz_mles, decomposition.rs:229-256):
// out [nz][l1 + W][d] from x [nz][l1][d] and w [nz][W][d], one thread per word
__global__ void k_assemble_z(const uint64_t *x, const uint64_t *w, size_t l1, size_t W, int d, size_t total,
                             uint64_t *out) {
  const size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (t >= total) return;
  const size_t n = (l1 + W) * d, k = t / n, o = t - k * n;
  out[t] = o < l1 * d ? x[k * l1 * d + o] : w[k * W * d + o - l1 * d];
}

hipError_t get_fhat(const uint64_t *f_coeff, size_t N, int d, int nv, uint64_t *out, hipStream_t st, int nw,
                    size_t wstride) {
  const size_t npts = (size_t)1 << nv;
  if (N > npts || nw < 1) return hipErrorInvalidValue;
  const size_t per = (size_t)(d == 24 ? 3 : 1) * npts * d, total = per * nw;
  if (!total) return hipSuccess;
  hipLaunchKernelGGL(k_get_fhat, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, f_coeff, N, wstride, d, npts,
                     per, total, out);
  return hipGetLastError();
}

hipError_t assemble_z(const uint64_t *x, const uint64_t *w, int nz, size_t l1, size_t W, int d, uint64_t *out,
                      hipStream_t st) {
  const size_t total = (size_t)nz * (l1 + W) * d;
  if (!total) return hipSuccess;
  hipLaunchKernelGGL(k_assemble_z, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, x, w, l1, W, d, total, out);
  return hipGetLastError();
}

}  // namespace lfk
