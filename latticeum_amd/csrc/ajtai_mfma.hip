// ajtai_mfma.hip -- the Ajtai matrix-vector commitment on the i8 matrix cores.
//
// For X^d + 1 rings every NTT slot s is an independent GEMM over Z_p:
//   C_s[i][v] = sum_j A[i][j][s] * F_v[j][s]        (i < kappa <= 32, v < nvec <= 32)
// Each residue x is written as 8 signed base-256 digits (D8):
//   t = x <= 0x7F..7F ? x : x + 2^32 - 1;  digits = bytes of (t + 0x80..80) ^ 0x80..80
// so x == sum_k d_k 256^k (mod p), d_k in [-128, 127]. Then
//   C_s = sum_{t=0..14} 256^t * sum_{a+b=t} A_s^(a) F_s^(b)
// and each A_s^(a) F_s^(b) is one v_mfma_i32_32x32x32_i8 per 32 columns. The 15
// weight sums stay in i32 accumulators (<= 8 * 32 * 2^14 per chunk, so < 2^31
// over AJ_CPS chunks) and are folded mod p once per wave.
//
// Operands are stored in MFMA fragment order (lane map verified on gfx950 by
// tools/probe/probe_mfma_i8.hip): for slot s, 32-column chunk c, digit k, a
// 1 KiB tile where lane l (r = l & 31, h = l >> 5) holds element (r, 16h..16h+15)
// -- row r of A, or vector r of F -- as 16 bytes. The matrix is converted once
// when the scheme is created; the vectors are converted by k_to_frag per call.
#include "kernels.hpp"

namespace lfk {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

__device__ __forceinline__ uint64_t d8(uint64_t x) {
  const uint64_t t = x <= 0x7F7F7F7F7F7F7F7Full ? x : x + 0xFFFFFFFFull;
  return (t + 0x8080808080808080ull) ^ 0x8080808080808080ull;
}

// ---------------------------------------------------------------- to fragment order
// block = (16-slot block, 32-column chunk c, group of 8 rows). LDS tile
// [row][slot][column] of D8 words, rows padded to 34 words so the 16-B
// column reads of the emit phase are aligned. Rows >= nrows are never
// written: they only feed MFMA output columns (or rows) that are discarded.
constexpr int TF_S = 16, TF_R = 8, TF_J = 34;
__global__ void __launch_bounds__(256) k_to_frag(VecPtrs rows, int nrows, size_t N, int d, int nch,
                                                 uint4 *frag) {
  __shared__ uint64_t tile[TF_R * TF_S * TF_J];
  const int sb = blockIdx.x, c = blockIdx.y, r0 = blockIdx.z * TF_R, tid = threadIdx.x;
  // load: 8 rows x 32 columns x (16 slots = 128 B = 8 pieces of 16 B)
#pragma unroll
  for (int it = 0; it < TF_R * 32 * 8 / 256; it++) {
    const int p = it * 256 + tid;
    const int r = p >> 8, j = (p >> 3) & 31, q = p & 7;
    const size_t col = (size_t)c * 32 + j;
    ulonglong2 v = make_ulonglong2(0, 0);
    if (r0 + r < nrows && col < N)
      v = *reinterpret_cast<const ulonglong2 *>(rows.p[r0 + r] + col * d + (size_t)sb * TF_S + 2 * q);
    uint64_t *t = tile + (r * TF_S + 2 * q) * TF_J + j;
    t[0] = d8(v.x);
    t[TF_J] = d8(v.y);
  }
  __syncthreads();
  // emit: thread = (slot sl, half h, row r); lane (r, h) of the MFMA operand
  // holds columns 16h..16h+15 of one slot as 16 bytes per digit
  const int r = tid & 7, h = (tid >> 3) & 1, sl = tid >> 4;
  if (r0 + r >= nrows) return;
  const ulonglong2 *src = reinterpret_cast<const ulonglong2 *>(tile + (r * TF_S + sl) * TF_J + 16 * h);
  uint32_t lo[16], hi[16];
#pragma unroll
  for (int q = 0; q < 8; q++) {
    const ulonglong2 x = src[q];
    lo[2 * q] = (uint32_t)x.x;
    hi[2 * q] = (uint32_t)(x.x >> 32);
    lo[2 * q + 1] = (uint32_t)x.y;
    hi[2 * q + 1] = (uint32_t)(x.y >> 32);
  }
  const size_t s = (size_t)sb * TF_S + sl;
  uint4 *out = frag + ((s * nch + c) * 8) * 64 + r0 + r + 32 * h;
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
      out[(4 * half + bb) * 64] = make_uint4(dw0[0], dw0[1], dw0[2], dw0[3]);
      out[(4 * half + bb + 1) * 64] = make_uint4(dw1[0], dw1[1], dw1[2], dw1[3]);
    }
  }
}

// ---------------------------------------------------------------- the contraction
// one wave = one slot x one column split; one wave per SIMD (15 i32 32x32
// accumulators = 240 registers). Fragments of chunk c+1 load while chunk c's
// 64 MFMAs run.
constexpr int AJ_CPS = 320;  // chunks per split (i32 bound: < 512)
__global__ void __launch_bounds__(256, 1) k_ajtai_mfma(const uint4 *Af, const uint4 *Ff, int d, int nch,
                                                      int nvec, int kappa, uint64_t *partial) {
  const int lane = threadIdx.x & 63;
  const int gw = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int s = gw % d, js = gw / d;
  if (js >= (nch + AJ_CPS - 1) / AJ_CPS) return;
  const int c0 = js * AJ_CPS, c1 = min(nch, c0 + AJ_CPS);
  v16i acc[15];
#pragma unroll
  for (int t = 0; t < 15; t++) acc[t] = (v16i){0};
  if (c0 < c1) {
    const uint4 *pa = Af + ((size_t)s * nch * 8) * 64 + lane;
    const uint4 *pf = Ff + ((size_t)s * nch * 8) * 64 + lane;
    v4i a[8], b[8];
#pragma unroll
    for (int k = 0; k < 8; k++) {
      uint4 x = pa[((size_t)c0 * 8 + k) * 64], y = pf[((size_t)c0 * 8 + k) * 64];
      a[k] = (v4i){(int)x.x, (int)x.y, (int)x.z, (int)x.w};
      b[k] = (v4i){(int)y.x, (int)y.y, (int)y.z, (int)y.w};
    }
    for (int c = c0; c < c1; c++) {
      v4i an[8], bn[8];
      const int cn = c + 1 < c1 ? c + 1 : c;
#pragma unroll
      for (int k = 0; k < 8; k++) {
        uint4 x = pa[((size_t)cn * 8 + k) * 64], y = pf[((size_t)cn * 8 + k) * 64];
        an[k] = (v4i){(int)x.x, (int)x.y, (int)x.z, (int)x.w};
        bn[k] = (v4i){(int)y.x, (int)y.y, (int)y.z, (int)y.w};
      }
#pragma unroll
      for (int ka = 0; ka < 8; ka++)
#pragma unroll
        for (int kb = 0; kb < 8; kb++)
          acc[ka + kb] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[ka], b[kb], acc[ka + kb], 0, 0, 0);
#pragma unroll
      for (int k = 0; k < 8; k++) {
        a[k] = an[k];
        b[k] = bn[k];
      }
    }
  }
  // fold the weights: value = sum_t 2^(8t) acc_t  (mod p); D reg i of lane l is
  // row (i & 3) + 8 (i >> 2) + 4 (l >> 5), column (vector) l & 31
  const int v = lane & 31, h = lane >> 5;
#pragma unroll
  for (int i = 0; i < 16; i++) {
    uint64_t r = 0;
#pragma unroll
    for (int t = 0; t < 15; t++) {
      const int32_t x = acc[t][i];
      const uint64_t fx = x < 0 ? gl::P - (uint64_t)(-(int64_t)x) : (uint64_t)x;
      r = gl::add(r, gl::mul_pow2(fx, 8 * t));
    }
    const int row = (i & 3) + 8 * (i >> 2) + 4 * h;
    if (v < nvec && row < kappa)
      partial[(((size_t)js * nvec + v) * kappa + row) * d + s] = r;
  }
}

// ---------------------------------------------------------------- launchers
size_t frag_elems(size_t ncols, int d) {  // uint4 count of one fragment buffer
  const size_t nch = (ncols + 31) / 32;
  return (size_t)d * nch * 8 * 64;
}
int mfma_nsplit(size_t ncols) {
  const int nch = (int)((ncols + 31) / 32);
  return (nch + AJ_CPS - 1) / AJ_CPS;
}

hipError_t to_frag(const VecPtrs &rows, int nrows, size_t ncols, int d, uint4 *frag, hipStream_t st) {
  if (nrows < 1 || nrows > 32 || d % TF_S) return hipErrorInvalidValue;
  const int nch = (int)((ncols + 31) / 32);
  hipLaunchKernelGGL(k_to_frag, dim3(d / TF_S, nch, (nrows + TF_R - 1) / TF_R), dim3(256), 0, st, rows, nrows,
                     ncols, d, nch, frag);
  return hipGetLastError();
}

hipError_t ajtai_mfma(const uint4 *Af, size_t kappa, size_t ncols, int d, const VecPtrs &fv, int nvec,
                      uint4 *Ff, uint64_t *partial, uint64_t *cm, hipStream_t st, hipEvent_t ev0,
                      hipEvent_t ev1) {
  if (kappa > 32 || nvec < 1 || nvec > 32) return hipErrorInvalidValue;
  hipError_t e = to_frag(fv, nvec, ncols, d, Ff, st);
  if (e != hipSuccess) return e;
  const int nch = (int)((ncols + 31) / 32), nsplit = mfma_nsplit(ncols);
  if (ev0) (void)hipEventRecord(ev0, st);
  const size_t waves = (size_t)d * nsplit;
  hipLaunchKernelGGL(k_ajtai_mfma, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, st, Af, Ff, d, nch, nvec,
                     (int)kappa, partial);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  if (ev1) (void)hipEventRecord(ev1, st);
  return sum_planes(partial, nsplit, (size_t)nvec * kappa * d, cm, st);
}

}  // namespace lfk
