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
// over AJ_CPS chunks) and are folded mod p once per wave. A is in the D8 form
// above; the vectors F, written every step by several producers, are in the
// cheaper offset form (frag.hpp fenc: the bytes of x with their top bits
// flipped, standing for x - FOFF), and the epilogue adds FOFF sum_j a_j per
// (row, slot) back (`kr`, ajtai_rowsums; A is zero on the padding columns, so
// their F bytes do not matter).
//
// Operands are stored in MFMA fragment order (lane map verified on gfx950 by
// tools/probe/probe_mfma_i8.hip): lane l (r = l & 31, h = l >> 5) of the
// operand for slot s, 32-column chunk c, digit k holds element (r, 16h..16h+15)
// -- row r of A, or vector r of F -- as 16 bytes.
//  * A ("row-interleaved"): [s][c][k][lane] -- one 1 KiB tile per digit, so
//    each load instruction is one contiguous KiB. Built once per scheme.
//  * F ("vector-major"):    [s/4][c][r][h][k][s%4] -- one vector's pieces for
//    4 consecutive slots are 64 contiguous bytes, so a producer that emits one
//    vector at a time for consecutive slots (the fused decomposition,
//    kernels_n32.hip) writes whole 64-B segments; the 4 waves of a contraction
//    block take 4 consecutive slots and share every fetched line.
// Contraction order: the 32 columns of chunk c are the 16-column units
// u = 2c and 2c + 1; unit u = (G, l) = (u / Lp, u % Lp) holds limb l of the
// groups 16G .. 16G + 15 (column g Lp + l). With Lp = L (the gadget length)
// one unit is one limb of 16 consecutive groups, which is what a block of the
// fused decomposition holds at once; Lp = 1 is the natural column order. A and
// F use the same order, so the contraction is unchanged.
//
// Phi_72 (d = 24, the reference ring): a slot is an Fq3 = Fq[u]/(u^3 - 2^40)
// element, and a slot product is a product of degree-2 polynomials reduced mod
// u^3 - 2^40. Toom-3 turns the slot's 9 component products into 5 same-position
// products: both operands are evaluated at u in {0, 1, -1, 2, inf} when they are
// written in fragment order (5 "virtual slots" per slot, 40 per element), the
// contraction runs unchanged over the 40 virtual slots (each an independent GEMM
// over Z_p), and k_phi72_interp interpolates the sums
//   D(u) = sum_j a_j(u) b_j(u),  deg D = 4
// back to D's coefficients d0..d4 and reduces: c = (d0 + 2^40 d3, d1 + 2^40 d4, d2)
// (goldilocks/mod.rs:34-54 Fq3 multiplication, summed over the columns as
// matrix.rs:168-178 does).
#include <cstdlib>
#include <cstring>

#include "frag.hpp"
#include "kernels.hpp"

namespace lfk {

// virtual slots per element of the contraction: d for X^d + 1, 40 for Phi_72
int mfma_dim(int d) { return d == 24 ? 40 : d; }

// ---------------------------------------------------------------- to fragment order
FragGeom frag_geom(size_t ncols, int Lp) {
  FragGeom g;
  g.Lp = Lp;
  g.Wp = ncols / Lp;
  const size_t units = (g.Wp + 15) / 16 * Lp;
  g.nch = (int)((units + 1) / 2);
  return g;
}

// block = (16-slot block, 32-column chunk c, group of 8 rows). LDS tile
// [row][slot][column] of D8 words, rows padded to 34 words so the 16-B
// column reads of the emit phase are aligned. Rows >= nrows are never
// written: they only feed MFMA output columns (or rows) that are discarded.
// PHI72: d = 24, the element's 40 virtual slots (Toom-3 evaluations) are
// produced on the fly; dv = virtual slots per element (d, or 40 for PHI72).
// ONEROW (a single operand row, the commit of one witness): the tile's 8 "rows"
// are 8 consecutive chunks of that row instead, so no thread idles.
constexpr int TF_S = 16, TF_R = 8, TF_J = 34;
// virtual slots 16 SB .. 16 SB + 15 (those below 40) of one Phi_72 element
template <int SB>
__device__ __forceinline__ void phi72_evals(const uint64_t *e, uint64_t *ev) {
#pragma unroll
  for (int i = 0; i < TF_S; i++)
    if (SB * TF_S + i < 40) ev[i] = ring::phi72_eval(e, SB * TF_S + i);
}
// qd > 0: operand slot of slot s is (s % 4) qd + s / 4 (FragGeom::qperm, qd = d / 4)
__host__ __device__ __forceinline__ size_t op_slot(size_t s, int qd) { return qd ? (s & 3) * qd + (s >> 2) : s; }
template <bool VMAJOR, bool PHI72, bool ONEROW>
__global__ void __launch_bounds__(256) k_to_frag(VecPtrs rows, int rlo, int rhi, int d, int dv, int nch, int Lp,
                                                 size_t Wp, uint4 *frag, int qd) {
  __shared__ uint64_t tile[TF_R * TF_S * TF_J];
  const int sb = blockIdx.x, tid = threadIdx.x;
  const int c0 = ONEROW ? blockIdx.y * TF_R : blockIdx.y;
  const int r0 = ONEROW ? rlo : (rlo & ~(TF_R - 1)) + blockIdx.z * TF_R;
  if (PHI72) {
    // load: one thread per (row or chunk r, column j); the element's Fq3 slots
    // behind virtual slots 16 sb .. 16 sb + 15 are read once and evaluated in
    // registers (the slot block is uniform per launch block, so no divergence)
    const int r = tid >> 5, j = tid & 31;
    const int c = ONEROW ? c0 + r : c0, row = ONEROW ? r0 : r0 + r;
    bool ok;
    const size_t col = frag_column(c, j, Lp, Wp, ok);
    uint64_t ev[TF_S];
#pragma unroll
    for (int i = 0; i < TF_S; i++) ev[i] = 0;
    if (row >= rlo && row < rhi && c < nch && ok) {
      const uint64_t *e = rows.p[row] + col * d;
      if (sb == 0)
        phi72_evals<0>(e, ev);
      else if (sb == 1)
        phi72_evals<1>(e, ev);
      else
        phi72_evals<2>(e, ev);
    }
#pragma unroll
    for (int i = 0; i < TF_S; i++) tile[(r * TF_S + i) * TF_J + j] = VMAJOR ? fenc(ev[i]) : d8(ev[i]);
  } else {
    // load: 8 rows (or chunks) x 32 columns x (16 slots = 128 B = 8 pieces of 16 B)
#pragma unroll
    for (int it = 0; it < TF_R * 32 * 8 / 256; it++) {
      const int p = it * 256 + tid;
      const int r = p >> 8, j = (p >> 3) & 31, q = p & 7;
      const int c = ONEROW ? c0 + r : c0, row = ONEROW ? r0 : r0 + r;
      bool ok;
      const size_t col = frag_column(c, j, Lp, Wp, ok);
      ulonglong2 v = make_ulonglong2(0, 0);
      if (row >= rlo && row < rhi && c < nch && ok)
        v = *reinterpret_cast<const ulonglong2 *>(rows.p[row] + col * d + sb * TF_S + 2 * q);
      uint64_t *t = tile + (r * TF_S + 2 * q) * TF_J + j;
      t[0] = VMAJOR ? fenc(v.x) : d8(v.x);  // F rows in the offset form, A in D8
      t[TF_J] = VMAJOR ? fenc(v.y) : d8(v.y);
    }
  }
  __syncthreads();
  // emit: thread = (slot sl, half h, row r); lane (r, h) of the MFMA operand
  // holds columns 16h..16h+15 of one slot as 16 bytes per digit
  const int r = tid & 7, h = (tid >> 3) & 1, sl = tid >> 4;
  const int c = ONEROW ? c0 + r : c0, row = ONEROW ? r0 : r0 + r;
  if (row < rlo || row >= rhi || c >= nch || sb * TF_S + sl >= dv) return;
  const ulonglong2 *src = reinterpret_cast<const ulonglong2 *>(tile + (r * TF_S + sl) * TF_J + 16 * h);
  uint64_t x[16];
#pragma unroll
  for (int q = 0; q < 8; q++) {
    const ulonglong2 t = src[q];
    x[2 * q] = t.x;
    x[2 * q + 1] = t.y;
  }
  uint4 u[8];
  d8_transpose16(x, u);
  const size_t s = op_slot((size_t)sb * TF_S + sl, qd);
  if (VMAJOR) {
    uint4 *out = frag + fv_index(s, nch, c, row, h);
#pragma unroll
    for (int b = 0; b < 8; b++) out[4 * b] = u[b];
  } else {
    uint4 *out = frag + ((s * nch + c) * 8) * 64 + row + 32 * h;
#pragma unroll
    for (int b = 0; b < 8; b++) out[b * 64] = u[b];
  }
}

// ---------------------------------------------------------------- the contraction
// one wave = one slot x one column split; one wave per SIMD (15 i32 32x32
// accumulators = 240 registers). Fragments of chunk c+1 load while chunk c's
// 64 MFMAs run. A is row-interleaved, F vector-major (see the top of the file).
constexpr int AJ_CPS = 320;  // most chunks per split (i32 bound: < 512)
// The 4 waves of a block take 4 consecutive slots (same split). Both operands
// stream into LDS with global_load_lds_dwordx4 (no staging registers):
//  * A: each wave copies its 8 KiB (8 one-KiB tiles, lane order) per chunk;
//  * F: the 4 slots' pieces form one contiguous 32 KiB tile per chunk; the
//    block copies it in 32 one-KiB pieces, lane i of piece j taking global
//    piece 64 j + pi_j(i), pi_j(i) = i ^ (2 (j & 7) | (i >> 5 & 1)) (an
//    involution inside the KiB, so every copy stays one coalesced KiB); a wave
//    then reads its operand for digit k with 64 lanes over 16 distinct bank
//    groups per 16 lanes (conflict-free ds_read_b128).
typedef __attribute__((address_space(3))) void lds_void;
__device__ __forceinline__ int fl_pi(int j, int i) { return i ^ (((j & 7) << 1) | ((i >> 5) & 1)); }

// fold the weights: value = sum_t 2^(8t) acc_t  (mod p); D reg i of lane l is
// row (i & 3) + 8 (i >> 2) + 4 (l >> 5), column (vector) l & 31
// Exactly in int64 by quarters: S_j = sum_{t in 4j..4j+3} acc_t 2^(8(t-4j)),
// |S_j| < 2^57; value = S0 + S1 2^32 + S2 2^64 + S3 2^96
//                   == (S0 - S2 - S3) + (S1 + S2) 2^32   (2^64 == 2^32 - 1, 2^96 == -1)
// so: the ring slot the wave's results belong to
// kr (split 0 only): the offset form's correction FOFF sum_j a_j of the output's row and slot
__device__ __forceinline__ void mfma_epilogue(const v16i *acc, int lane, int kt, int kappa, int nvec, int d, int so,
                                              int js, int direct, const OutPtrs &dst, uint64_t *partial,
                                              const uint64_t *kr) {
  const int v = lane & 31, h = lane >> 5;
  auto fe = [](int64_t x) { return x < 0 ? (uint64_t)x + gl::P : (uint64_t)x; };  // |x| < 2^63 - p
#pragma unroll
  for (int i = 0; i < 16; i++) {
    int32_t x[15];
#pragma unroll
    for (int t = 0; t < 15; t++) x[t] = acc[t][i];
    // one output's 15 words at a time (the flush must not pull all 240 into VGPRs)
    asm volatile("" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]),
                 "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]), "+v"(x[13]), "+v"(x[14]));
    int64_t S[4] = {0, 0, 0, 0};
#pragma unroll
    for (int t = 0; t < 15; t++) S[t >> 2] += (int64_t)x[t] << (8 * (t & 3));
    uint64_t r = gl::add(fe(S[0] - S[2] - S[3]), gl::mul_pow2(fe(S[1] + S[2]), 32));
    const int row = 32 * kt + (i & 3) + 8 * (i >> 2) + 4 * h;
    if (v < nvec && row < kappa) {
      if (js == 0) r = gl::add(r, kr[(size_t)row * d + so]);
      if (direct)  // one column split: the result itself
        dst.p[v][(size_t)row * d + so] = r;
      else
        partial[(((size_t)js * nvec + v) * kappa + row) * d + so] = r;
    }
  }
}

// CPOL: cache policy of the operand copies (2 = nt: streaming, for operands far
// larger than the caches -- A and F are each read once per launch)
// kappa > 32: A is stored as 32-row tiles (tile_u4 uint4 each), and one wave
// contracts one tile; the tiles of one (slot quad, split) are the blocks
// i + 8 t of a group of 8 ktiles blocks. Blocks are dealt round-robin over the
// 8 XCDs, so those blocks run on the same XCD at about the same time and the
// second tile's F copies hit that XCD's L2 instead of HBM.
// The same contraction with A in registers ("ra"): a wave's A operand is its
// own (one slot per wave), so it needs no LDS. Each wave keeps DP chunks of A
// in flight in VGPRs (32 per chunk, next to the 240 accumulator AGPRs), and the
// 160 KiB of LDS hold DP chunks of F: per CU about 2 (DP - 1) x 32 KiB of
// copies stay outstanding instead of 96 KiB. Per chunk c: wait for this wave's
// A(c) and F(c) copies, barrier, issue F(c + DP - 1) into the buffer F(c - 1)
// left, read F(c), 64 MFMAs, issue A(c + DP) into A(c)'s registers. Issue
// order: A(c0) F(c0) A(c0+1) .. F(c0+DP-2) A(c0+DP-1), then per chunk F, A.
// waits and loads as asm: the compiler's own waitcnt insertion cannot see that
// A(c) has landed once F(c) has, and would wait for every copy in flight
template <int N>
__device__ __forceinline__ void vm_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
template <int DP>
__device__ __forceinline__ void vm_wait_chunk(int nf) {
  // ops issued after F(c): A(c+1) and DP - 2 (F, A) pairs
  switch (nf) {
    case 8: vm_wait<8 + (DP - 2) * 16>(); break;
    case 7: vm_wait<8 + (DP - 2) * 15>(); break;
    case 6: vm_wait<8 + (DP - 2) * 14>(); break;
    case 5: vm_wait<8 + (DP - 2) * 13>(); break;
    case 4: vm_wait<8 + (DP - 2) * 12>(); break;
    case 3: vm_wait<8 + (DP - 2) * 11>(); break;
    case 2: vm_wait<8 + (DP - 2) * 10>(); break;
    case 1: vm_wait<8 + (DP - 2) * 9>(); break;
    default: vm_wait<8 + (DP - 2) * 8>(); break;
  }
}
// before digit kb's products: the 8 F reads were issued in digit order and LDS
// returns in order, so 7 - kb of them may still be outstanding
__device__ __forceinline__ void lgkm_wait_digit(int kb) {
  switch (kb) {
    case 0: asm volatile("s_waitcnt lgkmcnt(7)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt lgkmcnt(6)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt lgkmcnt(5)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt lgkmcnt(4)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt lgkmcnt(3)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt lgkmcnt(2)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt lgkmcnt(1)" ::: "memory"); break;
    default: asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); break;
  }
}
template <int CPOL>
__device__ __forceinline__ v4i gload16(const v4i *p) {
  v4i r;
  if (CPOL == 2)
    asm volatile("global_load_dwordx4 %0, %1, off nt" : "=v"(r) : "v"(p) : "memory");
  else
    asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(r) : "v"(p) : "memory");
  return r;
}
// Several independent fold steps against the same A (nsteps > 1, StepOps): the
// blocks of one (slot quad, split, ktile) for the different steps are blocks
// i + 8 (t + ktiles st) of one group, so they run on the same XCD at about the
// same time and A is fetched from HBM once for all of them (the siblings hit
// that XCD's L2, or the MALL); each step contracts its own operand rows into its
// own outputs. CPA / CPF: cache policies of the A and F copies.
template <int CPA, int CPF, int DP>
__global__ void __launch_bounds__(256, 1) k_ajtai_mfma_ra(const uint4 *Af, const uint64_t *kr, StepOps so_, int nsteps,
                                                         int d, int nch,
                                                         int nvec, int kappa, int direct, int cps, int ktiles,
                                                         int nbase, size_t tile_u4, int qd) {
  static_assert(DP >= 3 && DP <= 5, "F buffers: DP x 32 KiB of LDS");
  __shared__ uint4 Fl[DP][32 * 64];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int per = 8 * ktiles * nsteps;
  const int grp = blockIdx.x / per, rem = blockIdx.x - grp * per;
  const int stp = rem / (8 * ktiles), rem2 = rem - stp * 8 * ktiles;
  const int kt = rem2 >> 3, bi = grp * 8 + (rem2 & 7);
  if (bi >= nbase) return;  // uniform over the block
  const uint4 *Ff = so_.Ff[stp];
  uint64_t *partial = so_.partial[stp];
  const OutPtrs &dst = so_.dst[stp];
  const int gw = bi * 4 + w;
  const int s = gw % d, js = gw / d;
  if (js >= (nch + cps - 1) / cps) return;  // uniform over the block
  const int c0 = js * cps, c1 = min(nch, c0 + cps);
  v16i acc[15];
#pragma unroll
  for (int t = 0; t < 15; t++) acc[t] = (v16i){0};
  const v4i *pa = reinterpret_cast<const v4i *>(Af + kt * tile_u4 + ((size_t)s * nch * 8) * 64 + lane);
  const uint4 *ft = Ff + (size_t)(s >> 2) * nch * FV_CHUNK;
  v4i ra[DP][8];
  auto load_a = [&](int c, v4i *dstr) {
#pragma unroll
    for (int k = 0; k < 8; k++) {
      dstr[k] = gload16<CPA>(pa + ((size_t)c * 8 + k) * 64);
    }
  };
  const int nf = __builtin_amdgcn_readfirstlane((nvec - w + 3) >> 2 < 8 ? (nvec - w + 3) >> 2 : 8);  // wave-uniform
  // Dead units (DeadUnits: pieces the decomposition did not write, zero): lane l
  // keeps the mask of chunk c0 + l + 64 m in dm[m], bit 2 q + h for this wave's
  // vector 4 q + w in unit 2 c + h; lanes 32 h .. 32 h + 31 copy half h of a
  // vector, and for a dead half they copy zero80's 0x80 bytes (the offset form of
  // 0) instead, so every chunk still issues the same copies (vm_wait_chunk's
  // counts hold) and the matrix-core work is unchanged; HBM reads of dead units
  // are gone. Read here, before any operand copy is in flight.
  constexpr int NDM = (AJ_CPS + 63) / 64;
  const DeadUnits du = so_.dead[stp];
  const bool has_dead = du.flags != nullptr && du.rows != 0;  // uniform
  uint32_t dm[NDM];
#pragma unroll
  for (int m = 0; m < NDM; m++) dm[m] = 0;
  if (has_dead) {
#pragma unroll
    for (int m = 0; m < NDM; m++) {
      const int c = c0 + lane + 64 * m;
      if (c < c1) {
        const uint4 *p = reinterpret_cast<const uint4 *>(du.flags + (size_t)c * 64);  // units 2c, 2c + 1
        const uint4 a0 = p[0], a1 = p[1], b0 = p[2], b1 = p[3];
        const uint32_t ua[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};  // dword q: rows 4 q .. 4 q + 3
        const uint32_t ub[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
        uint32_t bits = 0;
#pragma unroll
        for (int q = 0; q < 8; q++)
          if ((du.rows >> (4 * q + w)) & 1)
            bits |= (((ua[q] >> (8 * w)) & 1u) << (2 * q)) | (((ub[q] >> (8 * w)) & 1u) << (2 * q + 1));
        dm[m] = bits;
      }
    }
  }
  // c uniform. Each dm[m] is read with its own readlane and the word picked on
  // the scalar side: a per-lane select over dm[] made the compiler keep the
  // array in LDS, and that read's lgkmcnt(0) wait drained the chunk's 8 operand
  // reads before its first product.
  auto dead_mask = [&](int c) -> uint32_t {
    if (!has_dead) return 0u;
    const int ci = c - c0, m = ci >> 6, l = ci & 63;
    uint32_t r = __builtin_amdgcn_readlane(dm[0], l);
#pragma unroll
    for (int k = 1; k < NDM; k++) {
      const uint32_t x = __builtin_amdgcn_readlane(dm[k], l);
      r = m == k ? x : r;
    }
    return r;
  };
  const int hl = lane >> 5;
  const uint4 *z80 = so_.zero80 + (lane & 31);
  // (the source is selected as a uint4 pointer in place: a pointer handed to the
  // builtin through a lambda's return value makes clang drop the host-side kernel stub)
  auto stage_f = [&](int c, int buf) {
    const uint32_t dmask = dead_mask(c);
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const int j = 4 * q + w;
      const uint4 *src = ((dmask >> (2 * q + hl)) & 1u) ? z80 : ft + (size_t)c * FV_CHUNK + j * 64 + fl_pi(j, lane);
      if (q < nf) __builtin_amdgcn_global_load_lds((const void *)src, (lds_void *)&Fl[buf][j * 64], 16, 0, CPF);
    }
  };
  auto stage_f_piece = [&](int c, int buf, int q, uint32_t dmask) {
    const int j = 4 * q + w;
    const uint4 *src = ((dmask >> (2 * q + hl)) & 1u) ? z80 : ft + (size_t)c * FV_CHUNK + j * 64 + fl_pi(j, lane);
    __builtin_amdgcn_global_load_lds((const void *)src, (lds_void *)&Fl[buf][j * 64], 16, 0, CPF);
  };
  const int rh = 2 * (lane & 31) + (lane >> 5), fj = rh >> 1;
  int fpos[8];
#pragma unroll
  for (int k = 0; k < 8; k++) fpos[k] = fj * 64 + fl_pi(fj, (rh & 1) * 32 + k * 4 + w);
#pragma unroll
  for (int j = 0; j < DP; j++) {
    if (c0 + j < c1) load_a(c0 + j, ra[j]);
    if (j < DP - 1 && c0 + j < c1) stage_f(c0 + j, j);
  }
  for (int cb = c0; cb < c1; cb += DP) {
#pragma unroll
    for (int j = 0; j < DP; j++) {
      const int c = cb + j;
      if (c >= c1) continue;  // uniform (only in a split's last round)
      if (c + DP - 1 < c1)
        vm_wait_chunk<DP>(nf);
      else
        vm_wait<0>();
      __builtin_amdgcn_s_barrier();  // every wave's F(c) landed; every wave is done reading F(c - 1)
      v4i b[8];
      const uint32_t fbase = (uint32_t)(uintptr_t)&Fl[j][0];
      // the copies ride between the products instead of in front of them: F(c)
      // is read right after the barrier and each digit's 8 products wait only
      // for that digit; F(c + DP - 1)'s pieces follow the digit groups, and
      // A(c + DP)'s loads follow the last product reading that register
      // (the issue order F then A is unchanged, so vm_wait_chunk still holds)
#pragma unroll
      for (int k = 0; k < 8; k++) asm volatile("ds_read_b128 %0, %1" : "=v"(b[k]) : "v"(fbase + 16u * fpos[k]));
      const bool more_f = c + DP - 1 < c1, more_a = c + DP < c1;
      const int fb = (j + DP - 1) % DP;
      const uint32_t dmn = more_f ? dead_mask(c + DP - 1) : 0u;
#pragma unroll
      for (int kb = 0; kb < 8; kb++) {
        lgkm_wait_digit(kb);
        asm volatile("" : "+v"(b[kb]));
        if (kb == 0) {
#pragma unroll
          for (int k = 0; k < 8; k++) asm volatile("" : "+v"(ra[j][k]));
        }
        if (kb < 7) {
#pragma unroll
          for (int ka = 0; ka < 8; ka++)
            acc[ka + kb] = __builtin_amdgcn_mfma_i32_32x32x32_i8(ra[j][ka], b[kb], acc[ka + kb], 0, 0, 0);
          __builtin_amdgcn_sched_barrier(0);
          if (more_f && kb < nf) stage_f_piece(c + DP - 1, fb, kb, dmn);
          __builtin_amdgcn_sched_barrier(0);
        } else {
          if (more_f && nf == 8) stage_f_piece(c + DP - 1, fb, 7, dmn);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int ka = 0; ka < 8; ka++) {
            acc[ka + 7] = __builtin_amdgcn_mfma_i32_32x32x32_i8(ra[j][ka], b[7], acc[ka + 7], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
            if (more_a) ra[j][ka] = gload16<CPA>(pa + ((size_t)(c + DP) * 8 + ka) * 64);
            __builtin_amdgcn_sched_barrier(0);
          }
        }
      }
    }
  }
  const int so = qd ? (s % qd) * 4 + s / qd : s;
  mfma_epilogue(acc, lane, kt, kappa, nvec, d, so, js, direct, dst, partial, kr);
}

// ---------------------------------------------------------------- f_0 from the operand rows
// folding.rs:258-268 compute_f_0 when the step keeps the decomposed planes only
// as operand rows (offset form; the fused d = 1024 / 4096 decompositions with f_k = null): one
// block per fold_frag_block (frag.hpp). The packed-plane step runs the same
// blocks inside k_fold_coeff's launch instead (fold_coeff.hip).
// (8 columns per thread, 512 threads, 114 VGPRs: four waves per SIMD instead of two;
// configs[4]'s fold 1.34 -> 1.17 ms)
__global__ void __launch_bounds__(512) k_fold_frag(const uint4 *frag, int nch, int Lp, size_t Wp, FoldRows fr,
                                                  const uint64_t *rho, int d, size_t N, uint64_t *out,
                                                  const int *run_if, int qd) {
  if (run_if && !*run_if) return;  // uniform: the coefficient-form fold produced f_0
  __shared__ uint64_t red[512 * 9];  // [output (column, slot)][vector group], rows padded to 9
  fold_frag_block<8>(blockIdx.x, frag, nch, Lp, Wp, fr, rho, d, N, out, red, qd);
}

hipError_t fold_frag(const uint4 *frag, const FragGeom &g, const FoldRows &fr, const uint64_t *rho, int d, size_t N,
                     uint64_t *out, hipStream_t st, const int *run_if) {
  if (d == 24 || d % 16 || fr.n < 1 || fr.n > LF_MAX_VECS) return hipErrorInvalidValue;
  if (!N) return hipSuccess;
  const size_t nb = (size_t)(d / 16) * g.nch;
  hipLaunchKernelGGL(k_fold_frag, dim3((unsigned)nb), dim3(512), 0, st, frag, g.nch, g.Lp, g.Wp, fr, rho, d, N, out,
                     run_if, g.qperm ? d / 4 : 0);
  return hipGetLastError();
}

// Phi_72 epilogue: virtual-slot sums [nvec][kappa][40] -> Fq3 slots [kappa][24] per vector
__global__ void k_phi72_interp(const uint64_t *virt, int nvec, size_t kappa, OutPtrs out) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;  // (v, row, slot)
  if (i >= (size_t)nvec * kappa * 8) return;
  const int slot = (int)(i & 7);
  const size_t vr = i >> 3, v = vr / kappa, row = vr - v * kappa;
  const uint64_t *P = virt + vr * 40 + 5 * slot;
  constexpr uint64_t INV2 = 0x7FFFFFFF80000001ull, INV3 = 0xAAAAAAAA00000001ull;
  const uint64_t d0 = P[0], d4 = P[4];
  const uint64_t d2 = gl::sub(gl::sub(gl::mul(gl::add(P[1], P[2]), INV2), d0), d4);
  const uint64_t s1 = gl::mul(gl::sub(P[1], P[2]), INV2);  // d1 + d3
  const uint64_t u =  // d1 + 4 d3
      gl::mul(gl::sub(gl::sub(gl::sub(P[3], d0), gl::mul_pow2(d2, 2)), gl::mul_pow2(d4, 4)), INV2);
  const uint64_t d3 = gl::mul(gl::sub(u, s1), INV3), d1 = gl::sub(s1, d3);
  uint64_t *o = out.p[v] + row * 24 + 3 * slot;
  o[0] = gl::add(d0, gl::mul_pow2(d3, 40));
  o[1] = gl::add(d1, gl::mul_pow2(d4, 40));
  o[2] = d2;
}

// ---------------------------------------------------------------- row sums of A
// tmp[i][w] = sum_j A[i][j][w] mod p (thread per (row, word), lazy 3-word sums)
__global__ void k_rowsum(const uint64_t *A, size_t kappa, size_t ncols, int d, uint64_t *tmp) {
  const size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (t >= kappa * (size_t)d) return;
  const size_t i = t / d;
  const int w = (int)(t - i * d);
  const uint64_t *p = A + i * ncols * d + w;
  gl::Acc a;
  gl::acc_zero(a);
  for (size_t j = 0; j < ncols; j++) gl::acc_add(a, p[j * d]);
  tmp[t] = gl::acc_reduce(a);
}
// kr[i][so] = FOFF * (row sum at output slot so): the ring slot itself, or for
// Phi_72 the Toom-3 virtual slot (phi72_eval of the row sum, linear)
__global__ void k_rowsum_kr(const uint64_t *tmp, size_t kappa, int d, int dv, uint64_t *kr) {
  const size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (t >= kappa * (size_t)dv) return;
  const size_t i = t / dv;
  const int vs = (int)(t - i * dv);
  const uint64_t r = d == 24 ? ring::phi72_eval(tmp + i * 24, vs) : tmp[i * d + vs];
  kr[t] = gl::mul(FOFF, r);
}
size_t ajtai_rowsums_elems(size_t kappa, int d) { return kappa * (size_t)mfma_dim(d); }
hipError_t ajtai_rowsums(const uint64_t *A, size_t kappa, size_t ncols, int d, uint64_t *kr, uint64_t *tmp,
                         hipStream_t st) {
  const size_t n = kappa * (size_t)d, m = kappa * (size_t)mfma_dim(d);
  hipLaunchKernelGGL(k_rowsum, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, A, kappa, ncols, d, tmp);
  hipLaunchKernelGGL(k_rowsum_kr, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, st, tmp, kappa, d, mfma_dim(d),
                     kr);
  return hipGetLastError();
}

// ---------------------------------------------------------------- launchers
size_t frag_elems(const FragGeom &g, int d) { return (size_t)mfma_dim(d) * g.nch * 8 * 64; }  // uint4 per buffer
int mfma_ktiles(size_t kappa) { return (int)((kappa + 31) / 32); }
// chunks per column split: AJ_CPS for wide rings; for few virtual slots (Phi_72)
// enough splits that about 1024 waves run
int mfma_cps(const FragGeom &g, int d) {
  const int dv = mfma_dim(d);
  if (dv >= 256) return AJ_CPS;
  // about 1024 waves: Phi_72 at the zkvm shape, 4 streams, measured the same
  // at 1024 and 2048 waves and worse at 4096 / 8192 (one stream: 0.41 ms at
  // 1024 against 0.42, 0.44, 0.47; tools/gpu_p24w.sh)
  const int want = 1024 / dv > 1 ? 1024 / dv : 1;
  const int cps = (g.nch + want - 1) / want;
  return cps < 1 ? 1 : (cps > AJ_CPS ? AJ_CPS : cps);
}
int mfma_nsplit(const FragGeom &g, int d) {
  const int cps = mfma_cps(g, d);
  return (g.nch + cps - 1) / cps;
}
size_t mfma_scratch_elems(const FragGeom &g, int d, size_t kappa, int nvec) {
  const size_t dv = mfma_dim(d), nsplit = mfma_nsplit(g, d);
  return (nsplit > 1 ? nsplit : 0) * nvec * kappa * dv + (d == 24 ? (size_t)nvec * kappa * dv : 0);
}

// operand rows row0 .. row0 + nrows - 1 <- rows.p[0 .. nrows - 1]
hipError_t to_frag(const VecPtrs &rows, int nrows, int row0, const FragGeom &g, int d, bool vmajor, uint4 *frag,
                   hipStream_t st) {
  const int dv = mfma_dim(d);
  if (nrows < 1 || row0 < 0 || row0 + nrows > 32 || (d != 24 && d % TF_S)) return hipErrorInvalidValue;
  VecPtrs abs{};
  for (int i = 0; i < nrows; i++) abs.p[row0 + i] = rows.p[i];
  const int qd = g.qperm ? d / 4 : 0;
  const int rhi = row0 + nrows, ztiles = (rhi + TF_R - 1) / TF_R - row0 / TF_R;
  const dim3 grid((dv + TF_S - 1) / TF_S, g.nch, ztiles);
#define LF_TF(VM, PH) \
  hipLaunchKernelGGL((k_to_frag<VM, PH, false>), grid, dim3(256), 0, st, abs, row0, rhi, d, dv, g.nch, g.Lp, g.Wp, frag, \
                     qd)
  if (nrows == 1 && vmajor) {
    const dim3 grid1((dv + TF_S - 1) / TF_S, (g.nch + TF_R - 1) / TF_R, 1);
    if (d == 24)
      hipLaunchKernelGGL((k_to_frag<true, true, true>), grid1, dim3(256), 0, st, abs, row0, rhi, d, dv, g.nch, g.Lp,
                         g.Wp, frag, qd);
    else
      hipLaunchKernelGGL((k_to_frag<true, false, true>), grid1, dim3(256), 0, st, abs, row0, rhi, d, dv, g.nch, g.Lp,
                         g.Wp, frag, qd);
    return hipGetLastError();
  }
  if (d == 24) {
    if (vmajor)
      LF_TF(true, true);
    else
      LF_TF(false, true);
  } else if (vmajor) {
    LF_TF(true, false);
  } else {
    LF_TF(false, false);
  }
#undef LF_TF
  return hipGetLastError();
}

// nsteps independent steps against one A: step s contracts the operand rows
// Ff[s] into dst[s] (per vector), with partial[s] as its mfma_scratch_elems()
// scratch (split partial sums, then Phi_72's virtual-slot results)
hipError_t ajtai_mfma_steps(const uint4 *Af, const uint64_t *kr, size_t kappa, const FragGeom &g, int d, int nvec,
                            int nsteps,
                            const uint4 *const *Ff, uint64_t *const *partial, const OutPtrs *dst, hipStream_t st,
                            hipEvent_t ev0, hipEvent_t ev1, const DeadUnits *dead, const uint4 *zero80) {
  const int dv = mfma_dim(d);
  const int ktiles = mfma_ktiles(kappa);
  // zero80 (32 pieces of 0x80 bytes) is the copy source of the dead units'
  // operand pieces: required only when some step has dead-unit flags
  bool any_dead = false;
  for (int s = 0; dead && s < nsteps && s < LF_MAX_STEPS; s++) any_dead |= dead[s].flags != nullptr;
  if (!kr || (any_dead && !zero80) || kappa < 1 || ktiles > LF_MAX_KTILES || nvec < 1 || nvec > 32 || dv % 4 || nsteps < 1 ||
      nsteps > LF_MAX_STEPS)
    return hipErrorInvalidValue;
  const int nsplit = mfma_nsplit(g, d), cps = mfma_cps(g, d);
  // the contraction's own outputs: the results (X^d + 1), or Phi_72's virtual-slot sums
  StepOps so{};
  so.zero80 = zero80;
  for (int s = 0; s < nsteps; s++) {
    so.Ff[s] = Ff[s];
    so.partial[s] = partial[s];
    so.dst[s] = dst[s];
    if (dead && zero80) so.dead[s] = dead[s];  // dead units read the constant pieces
    if (d == 24) {
      uint64_t *virt = partial[s] + (nsplit > 1 ? (size_t)nsplit * nvec * kappa * dv : 0);
      for (int v = 0; v < nvec; v++) so.dst[s].p[v] = virt + (size_t)v * kappa * dv;
    }
  }
  if (ev0) (void)hipEventRecord(ev0, st);
  const size_t waves = (size_t)dv * nsplit;
  const int nbase = (int)((waves + 3) / 4);
  const dim3 grid((unsigned)((nbase + 7) / 8 * 8 * ktiles * nsteps));
  const size_t tile_u4 = frag_elems(g, d);
  // F is dv nch 8 KiB per step (A is as large for kappa = 32): streamed past the
  // caches when larger than they are; A too for one step, but not when several
  // steps share it. A in registers 4 chunks ahead (d = 1024, W = 2^14: 6.7-6.9 ms
  // against 7.0 for A staged through LDS and no better at 3 or 5 chunks,
  // DESIGN.md section 7)
  const bool big = (size_t)dv * g.nch * 8192 > STREAM_OUT_BYTES;
  const int qd = g.qperm ? d / 4 : 0, direct = nsplit == 1 ? 1 : 0;
#define LF_AJ(CA, CF)                                                                                     \
  hipLaunchKernelGGL((k_ajtai_mfma_ra<CA, CF, 4>), grid, dim3(256), 0, st, Af, kr, so, nsteps, dv, g.nch, nvec, \
                     (int)kappa, direct, cps, ktiles, nbase, tile_u4, qd)
  // batched: A cached so the sibling blocks hit it, F streamed (A/B on one box,
  // W = 2^14, 2 steps: 49.6 steps/s against 49.2 both streamed, 49.4 both
  // cached, 48.3 A streamed / F cached)
  if (big && nsteps == 1)
    LF_AJ(2, 2);
  else if (big)
    LF_AJ(0, 2);
  else
    LF_AJ(0, 0);
#undef LF_AJ
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  if (ev1) (void)hipEventRecord(ev1, st);
  for (int s = 0; s < nsteps; s++) {
    if (nsplit > 1) {
      e = sum_planes_to(partial[s], nsplit, kappa * (size_t)dv, nvec, so.dst[s], st);
      if (e != hipSuccess) return e;
    }
    if (d == 24) {
      const size_t n = (size_t)nvec * kappa * 8;
      hipLaunchKernelGGL(k_phi72_interp, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, so.dst[s].p[0], nvec,
                         kappa, dst[s]);
      e = hipGetLastError();
      if (e != hipSuccess) return e;
    }
  }
  return hipSuccess;
}

// partial: mfma_scratch_elems() u64 (split partial sums, then Phi_72's virtual-slot results)
hipError_t ajtai_mfma(const uint4 *Af, const uint64_t *kr, size_t kappa, const FragGeom &g, int d, const VecPtrs &fv,
                      int nvec,
                      bool f_ready, uint4 *Ff, uint64_t *partial, uint64_t *cm, hipStream_t st, hipEvent_t ev0,
                      hipEvent_t ev1, const OutPtrs *dst, const DeadUnits *dead, const uint4 *zero80) {
  if (nvec < 1 || nvec > 32 || (!cm && !dst)) return hipErrorInvalidValue;
  OutPtrs out{};
  for (int v = 0; v < nvec; v++) out.p[v] = cm ? cm + (size_t)v * kappa * d : dst->p[v];
  if (!f_ready) {
    hipError_t e = to_frag(fv, nvec, 0, g, d, true, Ff, st);
    if (e != hipSuccess) return e;
  }
  const uint4 *ff[1] = {Ff};
  uint64_t *pp[1] = {partial};
  return ajtai_mfma_steps(Af, kr, kappa, g, d, nvec, 1, ff, pp, &out, st, ev0, ev1, f_ready ? dead : nullptr, zero80);
}

}  // namespace lfk
