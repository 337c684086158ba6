// fold_coeff.hip -- f_0 = sum_i rho_i f_i (LF/nifs/folding.rs:258-268) for X^1024 + 1,
// in coefficient form on the i8 matrix cores.
//
// The 2K folded witnesses are the balanced digit planes of the two decomposed
// sides, f_i = NTT(D_i) with D_i in {-1, 0, 1}^1024 (b_small = 2), and the
// folding challenges are short: rho_i has coefficients in [-32, 32)
// (cyclotomic-rings rings/goldilocks.rs:41-67, get_rhos in folding/utils.rs:116-127).
// The NTT is a ring isomorphism, so f_0 = NTT(sum_i rho_i * D_i), * the
// negacyclic product, and
//   f0_coeff[c][e] = sum_i sum_j R_i[c][j] D_i[j][e],
//   R_i[c][j] = rho_i[c - j] (c >= j),  -rho_i[c - j + 1024] (c < j),
// an exact integer GEMM of i8 operands (|f0_coeff| <= 2K 1024 32 < 2^31):
// M = 1024 coefficients, N = elements, K = 2K x 1024. Canonicalised, it is
// Witness::from_f's f_coeff itself; f_0 and w_ccs follow from one forward
// transform per element (k_from_fcoeff_n32). Instead of the 2K NTT-form planes
// (E 2K N = 20 GB at W = 2^14) the fold reads one key byte per coefficient quad
// and plane (0.6 GB).
//
// R_i is Toeplitz: the 32 x 32 A tile of rows 32t.. and columns 32q.. depends
// only on t - q. A wave owns 8 row tiles; stepping q by one shifts its 8 tiles
// one diagonal, so it keeps them in an 8-slot register window and loads one new
// tile per 32-column step (16 bytes at a lane-dependent byte offset of the
// reversed table, assembled from 5 LDS dwords with v_alignbyte). The B operand
// (16 digits of one element) comes from 4 key bytes through a 256-entry LDS
// table: key = 4 magnitude bits | 4 sign bits -> the quad's 4 digit bytes.
//
// Used only when every rho_i has coefficients in [-127, 127] (k_rho_prep checks
// on the device); otherwise the flag it raises makes these kernels return at
// once and the NTT-form fold and Witness::from_f run instead (the same flag,
// the other way round), with no host synchronisation.
#include "digits.hpp"
#include "frag.hpp"
#include "kernels.hpp"
#include "ntt32.hpp"

namespace lfk {

namespace {
constexpr int FD = 1024;
constexpr int FC_KEYROW = 64;  // u32 per (element, plane): 256 key bytes

// bit b of x (b < 8) -> bit 4b
__device__ __forceinline__ uint32_t spread8(uint32_t x) {
  x &= 0xFFu;
  x = (x | (x << 12)) & 0x000F000Fu;
  x = (x | (x << 6)) & 0x03030303u;
  x = (x | (x << 3)) & 0x11111111u;
  return x;
}

// keys[(col K + k) 64 + h 32 + q] byte i = key of quad p = 8q + 4h + i (its
// coefficients 4p .. 4p + 3) in plane k: bit m = bit k of |x_(4p+m)|, bit 4 + m
// = its sign. From the fused decomposition's packed coefficients
// (k_pack_sm: smg[(col 16 + qq) 32 + rr] = sm(x[rr + 64 qq]) | sm(x[rr + 64 qq + 32]) << 16,
// sm = 15-bit magnitude | sign << 15). One thread per (col, h, 4 consecutive q):
// 128 B in, one 16-B row piece per plane out.
// nz[col] (when given): bit k = plane k of the column has a nonzero digit (the 16
// threads of a column are 16 consecutive lanes of one wave: OR by shuffles)
__global__ void __launch_bounds__(256) k_pack_keys(const uint32_t *smg, size_t ncol, int K, uint32_t *keys,
                                                   uint32_t *nz) {
  const size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (t >= (ncol * 16 + 63) / 64 * 64) return;  // whole waves stay (the shuffles below)
  const bool live_t = t < ncol * 16;
  const size_t col = live_t ? t >> 4 : 0;
  const int h = (int)(t >> 3) & 1, q0 = 4 * (int)(t & 7);
  // coefficient j = 32 q + 16 h + 4 i + m sits in word (qq = q / 2, rr = 16 h + 4 i + m), half q & 1
  uint32_t w[2][16];
#pragma unroll
  for (int a = 0; a < 2; a++) {
    const uint4 *src = reinterpret_cast<const uint4 *>(smg + col * 512 + (q0 / 2 + a) * 32 + 16 * h);
#pragma unroll
    for (int v = 0; v < 4; v++) {
      const uint4 x = src[v];
      w[a][4 * v] = x.x;
      w[a][4 * v + 1] = x.y;
      w[a][4 * v + 2] = x.z;
      w[a][4 * v + 3] = x.w;
    }
  }
  if (nz) {
    uint32_t m = 0;  // magnitude bits of every coefficient this thread holds
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
      for (int i = 0; i < 16; i++) m |= w[a][i] | (w[a][i] >> 16);
    m &= 0x7FFFu;
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) m |= __shfl_xor(m, o);
    if (live_t && (t & 15) == 0) nz[col] = m;
  }
  if (!live_t) return;
  // per quad: planes 0..7 (lo) and 8..15 (hi, plane 15 = the sign) bit-sliced, bit 4 (k % 8) + m
  uint32_t lo[16], hi[16];
#pragma unroll
  for (int qd = 0; qd < 4; qd++)
#pragma unroll
    for (int i = 0; i < 4; i++) {
      uint32_t L = 0, H = 0;
#pragma unroll
      for (int m = 0; m < 4; m++) {
        const uint32_t v = w[qd >> 1][4 * i + m] >> (16 * (qd & 1));
        L |= spread8(v) << m;
        H |= spread8(v >> 8) << m;
      }
      lo[4 * qd + i] = L;
      hi[4 * qd + i] = H;
    }
  uint4 *dst = reinterpret_cast<uint4 *>(keys + col * K * FC_KEYROW + 32 * h + q0);
  for (int k = 0; k < K; k++) {
    uint32_t o[4];
#pragma unroll
    for (int qd = 0; qd < 4; qd++) {
      uint32_t x = 0;
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const int u = 4 * qd + i;
        const uint32_t nib = (k < 8 ? lo[u] >> (4 * k) : hi[u] >> (4 * (k - 8))) & 0xFu;
        x |= (nib | ((hi[u] >> 28) << 4)) << (8 * i);
      }
      o[qd] = x;
    }
    dst[k * (FC_KEYROW / 4)] = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

// rho (2K NTT elements) -> coefficients (rc), reversed byte tables and the range
// flag in ONE launch: half-wave i inverts rho_i on the register 32 x 32 NTT
// (ntt32.hpp), then writes its coefficients and
//   tab[i][u + 1024] = rho_i[-u] (-1023 <= u <= 0), -rho_i[1024 - u] (1 <= u <= 1023), else 0.
// The blocks' ORs of "a coefficient is outside [-127, 127]" meet in sync[0]; the
// last block to finish (ticket sync[1]) publishes it to *bad and resets both, so
// sync is zero again for the next launch (no memset). It replaces a device copy,
// a memset, the 2K-element inverse transform and the table kernel (about 35 us
// of serialised launches per step at W = 464).
constexpr int RP_WAVES = 2;  // 4 rho per block: 2K = 30 is 8 blocks of one round each
__global__ void __launch_bounds__(64 * RP_WAVES) k_rho_prep(const uint64_t *rho, int nw, uint64_t *rc, uint8_t *tab,
                                                           int *bad, const uint64_t *mid_ig, int *sync) {
  __shared__ uint64_t lds_all[RP_WAVES * n32::WAVE_U64];
  __shared__ uint64_t mid[n32::MID_U64];
  __shared__ int any;
  n32::stage_mid(mid, mid_ig);
  if (threadIdx.x == 0) any = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, wib = threadIdx.x >> 6, r = lane & 31, h = lane >> 5;
  uint64_t *T = lds_all + wib * n32::WAVE_U64 + h * n32::HALF_U64;
  bool out = false;
  // every wave runs every round (wave-uniform)
  for (int i0 = 2 * RP_WAVES * blockIdx.x; i0 < nw; i0 += 2 * RP_WAVES * gridDim.x) {
    const int i = i0 + 2 * wib + h;
    const bool ok = i < nw;
    uint64_t v[32];
    n32::load_row32(rho + (size_t)(ok ? i : 0) * FD + r, v);  // slot input layout v[m2] = X[r + 32 m2]
    n32::inverse(v, mid, T, r);                                 // coefficient layout v[k] = x[r + 32 k]
    if (ok) {
      uint64_t *rci = rc + (size_t)i * FD + r;
      uint8_t *ti = tab + (size_t)i * FOLD_RT;
#pragma unroll
      for (int k = 0; k < 32; k++) {
        const int c = r + 32 * k;
        const int64_t sv = signed_rep(v[k]);
        out |= sv > 127 || sv < -127;
        rci[32 * k] = v[k];
        ti[1024 - c] = (uint8_t)(int8_t)sv;                      // u = -c
        if (c > 0) ti[2048 - c] = (uint8_t)(int8_t)(-sv);        // u = 1024 - c
      }
      // u = -1024 and u >= 1024: zero (positions 0 and 2048 .. FOLD_RT - 1)
      for (int o = 2048 + r; o < FOLD_RT; o += 32) ti[o] = 0;
      if (r == 0) ti[0] = 0;
    }
  }
  if (out) any = 1;  // every writer stores the same value
  __syncthreads();
  if (threadIdx.x == 0) {
    if (any) atomicOr(&sync[0], 1);
    __threadfence();
    if (atomicAdd(&sync[1], 1) == (int)gridDim.x - 1) {  // the last block: every block's flag is in
      *bad = atomicExch(&sync[0], 0);
      atomicExch(&sync[1], 0);
    }
  }
}

// 16 bytes of a rho table at byte offset o (any alignment): 5 dwords, v_alignbyte
__device__ __forceinline__ v4i tile_a(const uint8_t *ri, int o, int sh) {
  const uint32_t *p = reinterpret_cast<const uint32_t *>(ri + (o & ~3));
  const uint32_t d0 = p[0], d1 = p[1], d2 = p[2], d3 = p[3], d4 = p[4];
  v4i a;
  a[0] = (int)__builtin_amdgcn_alignbyte(d1, d0, sh);
  a[1] = (int)__builtin_amdgcn_alignbyte(d2, d1, sh);
  a[2] = (int)__builtin_amdgcn_alignbyte(d3, d2, sh);
  a[3] = (int)__builtin_amdgcn_alignbyte(d4, d3, sh);
  return a;
}

constexpr int FC_MAXW = 30;  // 2K <= 30
// A block (4 waves) owns 32 elements (MFMA columns) at a time; wave w the rows
// 256 w .. 256 w + 255 (row tiles t = 8 w + tt). Grid-stride over element tiles.
// ks_n > 1 (few elements: fewer 32-element tiles than the chip has block
// slots): task (tile, ks) sums only witnesses [ks nw / ks_n, (ks + 1) nw / ks_n)
// and writes its exact int32 partials to part[ks][e][1024]; k_fold_coeff_sum
// adds them up
// *bad (rho not short): with fb.frag the launch folds f_0 in NTT form from the
// operand rows instead (fold_frag_block, grid-stride; a separate gated launch of
// its (d / 16) nch blocks would wait for CU resources behind other streams' work
// even when it has nothing to do), else it returns and the NTT-form fold runs
__global__ void __launch_bounds__(256, 2) k_fold_coeff(const uint32_t *keys, const uint8_t *tab_g, const int *bad,
                                                      size_t N, int K, uint64_t *f0c, int ks_n, int32_t *part,
                                                      FoldFallback fb, int L, const uint32_t *nz) {
  __shared__ __attribute__((aligned(16))) uint8_t rt[FC_MAXW * FOLD_RT];
  __shared__ uint32_t lut[256];
  static_assert(FC_MAXW * FOLD_RT >= 512 * 9 * 8, "fold_frag_block's LDS fits the rho tables'");
  if (*bad) {
    if (fb.frag) {
      const size_t nvb = (size_t)(FD / 16) * fb.nch;
      for (size_t vb = blockIdx.x; vb < nvb; vb += gridDim.x)
        fold_frag_block(vb, fb.frag, fb.nch, fb.Lp, fb.Wp, fb.fr, fb.rho, FD, N, fb.f0,
                        reinterpret_cast<uint64_t *>(rt));
    }
    return;
  }
  const int nw = 2 * K, tid = threadIdx.x;
  for (int x = tid; x < nw * FOLD_RT / 16; x += blockDim.x)
    reinterpret_cast<uint4 *>(rt)[x] = reinterpret_cast<const uint4 *>(tab_g)[x];
  {
    const uint32_t m = tid & 15, s = tid >> 4;
    uint32_t v = 0;
#pragma unroll
    for (int i = 0; i < 4; i++)
      if ((m >> i) & 1) v |= ((s >> i) & 1 ? 0xFFu : 0x01u) << (8 * i);
    lut[tid] = v;
  }
  __syncthreads();
  const int lane = tid & 63, wv = tid >> 6, col = lane & 31, h = lane >> 5;
  const int sh = (-col) & 3;
  // A tile of diagonal dl = t - q for this lane: bytes o .. o + 15, o = obase - 32 dl
  const int obase = 1024 + 16 * h - col;
  // Tiles are limb-pure: tile (l, gt) holds elements (32 gt + col) L + l, so a
  // tile of the top limb (whose planes 4.. are zero for any balanced
  // decomposition of a field element) skips those planes' products; a plane is
  // skipped only when it is zero on all 32 of the tile's elements (nz: the
  // per-column plane masks of k_pack_keys), so any input stays exact.
  const size_t W = N / L, ntl = (W + 31) / 32, ntile = ntl * L;
  for (size_t task = blockIdx.x; task < ntile * ks_n; task += gridDim.x) {
    const size_t tile = task / ks_n;
    const int ks = (int)(task % ks_n), iq0 = 4 * (ks * nw / ks_n), iq1 = 4 * ((ks + 1) * nw / ks_n);
    const size_t grp = (tile % ntl) * 32 + col;
    const bool valid = grp < W;
    const size_t e = grp * L + tile / ntl, ee = valid ? e : 0;
    uint32_t live = nz ? (valid ? nz[ee] | (nz[N + ee] << K) : 0u) : 0xFFFFFFFFu;
#pragma unroll
    for (int o = 1; o < 32; o <<= 1) live |= __shfl_xor(live, o);  // the tile's 32 columns (both halves agree)
    live = __builtin_amdgcn_readfirstlane(live);
    // the next iq at or after iq whose plane is live (whole planes are skipped)
    auto next_live = [&](int iq) {
      while (iq < iq1 && !((live >> (iq >> 2)) & 1u)) iq = (iq & ~3) + 4;
      return iq;
    };
    const uint32_t *kb0 = keys + ee * K * FC_KEYROW + 32 * h, *kb1 = keys + (N + ee) * K * FC_KEYROW + 32 * h;
    v16i acc[8];
#pragma unroll
    for (int tt = 0; tt < 8; tt++)
#pragma unroll
      for (int i = 0; i < 16; i++) acc[tt][i] = 0;
    v4i A[8];
    // the key words of (plane i, q block qb): 8 dwords, one block ahead
    auto kaddr = [&](int iq) {
      const int i = iq >> 2, s = i >= K;
      return (s ? kb1 : kb0) + (i - s * K) * FC_KEYROW + 8 * (iq & 3);
    };
    uint4 kn0 = make_uint4(0, 0, 0, 0), kn1 = kn0;
    const int iqs = next_live(iq0);
    if (iqs < iq1) {
      const uint4 *p = reinterpret_cast<const uint4 *>(kaddr(iqs));
      kn0 = p[0];
      kn1 = p[1];
    }
    for (int iq = iqs; iq < iq1; iq = next_live(iq + 1)) {
      const int i = iq >> 2;
      const uint8_t *ri = rt + i * FOLD_RT;
      if ((iq & 3) == 0) {  // a new plane: slots 1..7 take diagonals 8 w + 1 .. 8 w + 7
#pragma unroll
        for (int tt = 1; tt < 8; tt++) A[tt] = tile_a(ri, obase - 32 * (8 * wv + tt), sh);
      }
      const uint32_t kw[8] = {kn0.x, kn0.y, kn0.z, kn0.w, kn1.x, kn1.y, kn1.z, kn1.w};
      {
        const int nx = next_live(iq + 1);
        const uint4 *p = reinterpret_cast<const uint4 *>(kaddr(nx < iq1 ? nx : iq));
        kn0 = p[0];
        kn1 = p[1];
      }
      const int q0 = 8 * (iq & 3);
#pragma unroll
      for (int qi = 0; qi < 8; qi++) {
        // slot (tt - q) & 7 holds diagonal 8 w + tt - q; the new one (tt = 0) goes to slot (-q) & 7
        A[(8 - qi) & 7] = tile_a(ri, obase - 32 * (8 * wv - (q0 + qi)), sh);
        v4i b;
        b[0] = (int)lut[kw[qi] & 0xFF];
        b[1] = (int)lut[(kw[qi] >> 8) & 0xFF];
        b[2] = (int)lut[(kw[qi] >> 16) & 0xFF];
        b[3] = (int)lut[kw[qi] >> 24];
#pragma unroll
        for (int tt = 0; tt < 8; tt++)
          acc[tt] = __builtin_amdgcn_mfma_i32_32x32x32_i8(A[(tt - qi) & 7], b, acc[tt], 0, 0, 0);
      }
    }
    if (valid && ks_n > 1) {
      int32_t *out = part + ((size_t)ks * N + e) * FD + 256 * wv + 4 * h;
#pragma unroll
      for (int tt = 0; tt < 8; tt++)
#pragma unroll
        for (int g = 0; g < 4; g++)
          *reinterpret_cast<v4i *>(out + 32 * tt + 8 * g) =
              (v4i){acc[tt][4 * g], acc[tt][4 * g + 1], acc[tt][4 * g + 2], acc[tt][4 * g + 3]};
    } else if (valid) {
      // lane (col, h), acc[tt][4 g + r]: row 32 (8 w + tt) + 8 g + 4 h + r of element e
      uint64_t *out = f0c + e * FD + 256 * wv + 4 * h;
      auto fe = [](int x) { return x < 0 ? (uint64_t)(int64_t)x + gl::P : (uint64_t)x; };
#pragma unroll
      for (int tt = 0; tt < 8; tt++)
#pragma unroll
        for (int g = 0; g < 4; g++) {
          ulonglong2 *o = reinterpret_cast<ulonglong2 *>(out + 32 * tt + 8 * g);
          o[0] = make_ulonglong2(fe(acc[tt][4 * g]), fe(acc[tt][4 * g + 1]));
          o[1] = make_ulonglong2(fe(acc[tt][4 * g + 2]), fe(acc[tt][4 * g + 3]));
        }
    }
  }
}
// f0c[e][c] = sum_ks part[ks][e][c] (exact: the full sum is the bounded one), canonical
__global__ void k_fold_coeff_sum(const int32_t *part, int ks_n, size_t n, const int *bad, uint64_t *f0c) {
  if (*bad) return;
  const size_t q = blockIdx.x * (size_t)blockDim.x + threadIdx.x;  // 4 coefficients
  if (q >= n / 4) return;
  v4i s = *reinterpret_cast<const v4i *>(part + 4 * q);
  for (int k = 1; k < ks_n; k++) s += *reinterpret_cast<const v4i *>(part + (size_t)k * n + 4 * q);
  auto fe = [](int x) { return x < 0 ? (uint64_t)(int64_t)x + gl::P : (uint64_t)x; };
  ulonglong2 *o = reinterpret_cast<ulonglong2 *>(f0c + 4 * q);
  o[0] = make_ulonglong2(fe(s[0]), fe(s[1]));
  o[1] = make_ulonglong2(fe(s[2]), fe(s[3]));
}
}  // namespace

// witness splits for N elements: enough (tile, split) tasks for two blocks per
// CU, the splits dividing the 2K witnesses evenly (1 at the bench's W = 2^14)
int fold_coeff_splits(size_t N, int K, int ncu) {
  const size_t ntile = (N + 31) / 32, cap = 2 * (size_t)ncu;
  int best = 1;
  for (int ks = 2; ks <= 2 * K; ks++)
    if ((2 * K) % ks == 0 && ntile * ks <= cap) best = ks;
  return best;
}

hipError_t fold_keys(const uint32_t *smg, size_t ncol, int K, uint32_t *keys, hipStream_t st, uint32_t *nz) {
  if (K < 1 || K > 15) return hipErrorInvalidValue;
  if (!ncol) return hipSuccess;
  hipLaunchKernelGGL(k_pack_keys, dim3((unsigned)((ncol * 16 + 255) / 256)), dim3(256), 0, st, smg, ncol, K, keys,
                     nz);
  return hipGetLastError();
}

hipError_t fold_rho_tables(const uint64_t *rho, int nw, uint64_t *rc, uint8_t *tab, int *bad,
                           const ring::NegaTables &inv, int *sync, hipStream_t st) {
  if (nw < 1 || nw > FC_MAXW || !inv.mid || !sync) return hipErrorInvalidValue;
  const int per = 2 * RP_WAVES;
  hipLaunchKernelGGL(k_rho_prep, dim3((nw + per - 1) / per), dim3(64 * RP_WAVES), 0, st, rho, nw, rc, tab, bad,
                     inv.mid, sync);
  return hipGetLastError();
}

hipError_t fold_coeff(const uint32_t *keys, const uint8_t *tab, const int *bad, size_t N, int K, uint64_t *f0c,
                      int ncu, hipStream_t st, int32_t *part, const FoldFallback *fb, int L, const uint32_t *nz) {
  FoldFallback fbv{};
  if (fb) fbv = *fb;
  if (K < 1 || 2 * K > FC_MAXW || ncu < 1 || L < 1 || N % L) return hipErrorInvalidValue;
  if (!N) return hipSuccess;
  const int ks_n = part ? fold_coeff_splits(N, K, ncu) : 1;
  const size_t ntile = (N / L + 31) / 32 * L;
  const size_t ntask = ntile * ks_n, cap = 2 * (size_t)ncu;  // two blocks per CU (LDS 63 KB, 256 registers)
  hipLaunchKernelGGL(k_fold_coeff, dim3((unsigned)(ntask < cap ? ntask : cap)), dim3(256), 0, st, keys, tab, bad, N,
                     K, f0c, ks_n, part, fbv, L, nz);
  if (ks_n > 1) {
    const size_t n = N * FD;
    hipLaunchKernelGGL(k_fold_coeff_sum, dim3((unsigned)((n / 4 + 255) / 256)), dim3(256), 0, st, part, ks_n, n, bad,
                       f0c);
  }
  return hipGetLastError();
}

}  // namespace lfk
