// kernels.hpp -- launcher declarations for kernels.hip (internal to the library).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "ring.hpp"

#define LF_MAX_VECS 32
#define LF_MAX_KTILES 4
#define LF_MAX_STEPS 8  // steps per batched contraction (lf_dev_fold_step_batch)

namespace lfk {

// table of up to LF_MAX_VECS device vectors, passed by value as a kernel argument
struct VecPtrs {
  const uint64_t *p[LF_MAX_VECS];
};
// destinations of up to LF_MAX_VECS output vectors
struct OutPtrs {
  uint64_t *p[LF_MAX_VECS];
};

// Dead operand pieces: a fused decomposition does not write the operand rows of a
// 16-column unit whose digit plane is zero on all 16 columns (the top limb's
// planes 4..K-1 of a balanced decomposition, plane K-1 of most units), and marks
// dead[u 32 + row] = 1 instead (0 when written); the flags are valid for the rows
// in `rows` only. Readers of those rows (the contraction, the operand-row folds)
// take the offset form of zero there.
struct DeadUnits {
  const uint8_t *flags = nullptr;  // [2 nch units][32 rows]
  uint32_t rows = 0;               // bit r: row r's flags are this step's
};
// per-step operands and destinations of a contraction over several independent steps
struct StepOps {
  const uint4 *Ff[LF_MAX_STEPS];
  uint64_t *partial[LF_MAX_STEPS];
  OutPtrs dst[LF_MAX_STEPS];
  DeadUnits dead[LF_MAX_STEPS];
  const uint4 *zero80 = nullptr;  // 32 operand pieces of 0x80 bytes (the offset form of 0) for dead units
};

hipError_t transform(uint64_t *data, size_t n, int d, bool fwd, const ring::NegaTables &tb,
                     hipStream_t st);
hipError_t slot_mul(const uint64_t *a, const uint64_t *b, uint64_t *out, size_t n, int d,
                    hipStream_t st);
hipError_t mont(uint64_t *x, size_t n, bool to, hipStream_t st);
// smg (d = 1024 only, may be null): also write the digits as the fused
// decomposition's packed sign|magnitude words ([W L][512] u32, k_pack_sm's layout),
// so that launch need not re-read f_coeff (the digits fit 15 bits when lb <= 15)
hipError_t from_w_ccs(const uint64_t *w_ccs, size_t W, int d, int lb, int L, uint64_t *f_coeff,
                      uint64_t *f, const ring::NegaTables &fwd, const ring::NegaTables &inv, int *err,
                      hipStream_t st, uint32_t *smg = nullptr);
// run_if (X^1024 + 1 and Phi_72): when given, the kernels do nothing unless *run_if != 0
// (the fallbacks of the coefficient-form fold, fold_coeff.hip)
hipError_t from_f(const uint64_t *f, size_t N, int d, int lb, int L, uint64_t *f_coeff,
                  uint64_t *w_ccs, const ring::NegaTables &inv, hipStream_t st, const int *run_if = nullptr);
// d = 24 with frag: planes 1..K-1 also written as i8-MFMA operand rows row0.. (Lp = L order, nch chunks)
hipError_t decompose_witness(const uint64_t *f_coeff, size_t N, int d, int lb, int L, int lbs, int K,
                             uint64_t *f_coeff_k, uint64_t *f_k, uint64_t *w_ccs_k,
                             const ring::NegaTables &fwd, int *err, hipStream_t st, uint4 *frag = nullptr,
                             int nch = 0, int row0 = 0);
int ajtai_nsplit(size_t ncols, int d, int nvec);
size_t ajtai_partial_elems(size_t kappa, size_t ncols, int d, int nvec);
hipError_t ajtai_commit(const uint64_t *A, size_t kappa, size_t ncols, int d, const VecPtrs &fv,
                        int nvec, uint64_t *partial, uint64_t *cm, hipStream_t st,
                        hipEvent_t ev0 = nullptr, hipEvent_t ev1 = nullptr);
hipError_t commit_y0(const uint64_t *cm, uint64_t *y, size_t kappa, int d, int lbs, int K,
                     hipStream_t st);
hipError_t fold(const uint64_t *rho, const VecPtrs &x, int nwit, size_t n, int d, uint64_t *out,
                hipStream_t st, const int *run_if = nullptr);
hipError_t p2_permute(uint64_t *states, size_t n, hipStream_t st, int rounds = 30);
hipError_t fill_uniform(uint64_t *out, size_t n, uint64_t seed, hipStream_t st);
hipError_t modp_sum(const uint64_t *in, int nparts, size_t len, uint64_t *out, hipStream_t st);

// rot_lin_combination: rho_coeff [n][d] (canonical), theta [n][tau d] (tau = 3 for d = 24, else 1) -> v0 [tau d]
hipError_t rot_lin(const uint64_t *rho_coeff, const uint64_t *theta, int n, int d, uint64_t *v0, hipStream_t st);
hipError_t limb_split(const uint64_t *x, size_t n, uint64_t *lo, uint64_t *hi, hipStream_t st);
hipError_t limb_join(const uint64_t *lo, const uint64_t *hi, size_t n, uint64_t *out, hipStream_t st);

hipError_t sum_planes(const uint64_t *partial, int nsplit, size_t len, uint64_t *out, hipStream_t st);
// out.p[v][r] = sum_s partial[s][v][r] for nvec vectors of len u64
hipError_t sum_planes_to(const uint64_t *partial, int nsplit, size_t len, int nvec, const OutPtrs &out,
                         hipStream_t st);
// the fold step's epilogue over the kappa d commitment slots, both sides:
// y_s[0] = cm_s - sum_{k>=1} 2^(k lbs) y_s[k] (decomposition.rs:183-200), then
// cm0 = sum_{s,k} rho_{sK+k} (.) y_s[k] (folding/utils.rs:470-476); X^d + 1 rings
hipError_t y0_cm0(const uint64_t *cm0s, const uint64_t *cm1s, uint64_t *y0, uint64_t *y1, const uint64_t *rho,
                  size_t kappa, int d, int lbs, int K, uint64_t *cm0, hipStream_t st);

// i8-MFMA Ajtai (ajtai_mfma.hip): negacyclic rings and Phi_72, nvec <= 32,
// kappa <= 32 LF_MAX_KTILES: A is stored as mfma_ktiles(kappa) tiles of 32 rows,
// frag_elems() uint4 each.
// Column (contraction) order: 16-column units u = (u / Lp, u % Lp) = limb l of
// groups 16G..16G+15; nch 32-column chunks.
struct FragGeom {
  int Lp;
  size_t Wp;
  int nch;
  // d = 4096: operand slot sigma(s) = (s % 4) d/4 + s / 4 (quarter-major, the
  // order kernels_n4k.hip produces slots in); the contraction maps it back
  int qperm = 0;
};
FragGeom frag_geom(size_t ncols, int Lp);
// d = 24 (Phi_72) contracts 40 virtual slots per element (Toom-3, ajtai_mfma.hip)
int mfma_dim(int d);
// whether ajtai_mfma gathers the vectors itself (no operand rows) for this geometry
size_t frag_elems(const FragGeom &g, int d);  // uint4 per fragment buffer (32 operand rows)
int mfma_ktiles(size_t kappa);
int mfma_nsplit(const FragGeom &g, int d);
// u64 of scratch ajtai_mfma needs (split partial sums, Phi_72 virtual-slot results)
size_t mfma_scratch_elems(const FragGeom &g, int d, size_t kappa, int nvec);
hipError_t to_frag(const VecPtrs &rows, int nrows, int row0, const FragGeom &g, int d, bool vmajor, uint4 *frag,
                   hipStream_t st);
// cm: contiguous [nvec][kappa d] results, or (cm == nullptr) per-vector destinations dst
// kr: FOFF times the row sums of A per (row, output slot), ajtai_rowsums (the
// vector operand rows are in the offset form, frag.hpp fenc)
hipError_t ajtai_rowsums(const uint64_t *A, size_t kappa, size_t ncols, int d, uint64_t *kr, uint64_t *tmp,
                         hipStream_t st);
size_t ajtai_rowsums_elems(size_t kappa, int d);  // u64 of kr; tmp needs kappa d
hipError_t ajtai_mfma(const uint4 *Af, const uint64_t *kr, size_t kappa, const FragGeom &g, int d, const VecPtrs &fv,
                      int nvec,
                      bool f_ready, uint4 *Ff, uint64_t *partial, uint64_t *cm, hipStream_t st,
                      hipEvent_t ev0 = nullptr, hipEvent_t ev1 = nullptr, const OutPtrs *dst = nullptr,
                      const DeadUnits *dead = nullptr, const uint4 *zero80 = nullptr);
// nsteps (<= LF_MAX_STEPS) independent steps in one pass over A: step s's operand
// rows Ff[s] (f_ready), scratch partial[s] (mfma_scratch_elems), results dst[s];
// dead[s] (may be null): step s's dead operand pieces, read as zero80's pieces
hipError_t ajtai_mfma_steps(const uint4 *Af, const uint64_t *kr, size_t kappa, const FragGeom &g, int d, int nvec,
                            int nsteps,
                            const uint4 *const *Ff, uint64_t *const *partial, const OutPtrs *dst, hipStream_t st,
                            hipEvent_t ev0 = nullptr, hipEvent_t ev1 = nullptr, const DeadUnits *dead = nullptr,
                            const uint4 *zero80 = nullptr);

// d = 1024 kernels on the register-resident 32 x 32 NTT (kernels_n32.hip)
// W below which from_w_ccs / from_f run one half-wave per (element, limb)
size_t witness_split_w();
// data = transform(src), in place when src is null
hipError_t transform_n32(uint64_t *data, size_t n, bool fwd, const ring::NegaTables &tb, hipStream_t st,
                         const uint64_t *src = nullptr);
hipError_t from_w_ccs_n32(const uint64_t *w_ccs, size_t W, int lb, int L, uint64_t *f_coeff, uint64_t *f,
                          const ring::NegaTables &fwd, const ring::NegaTables &inv, int *err, hipStream_t st,
                          uint32_t *smg = nullptr);
hipError_t from_f_n32(const uint64_t *f, size_t W, int lb, int L, uint64_t *f_coeff, uint64_t *w_ccs,
                      const ring::NegaTables &inv, hipStream_t st, const int *run_if = nullptr);
hipError_t decompose_n32(const uint64_t *f_coeff, size_t N, int lb, int L, int K, uint64_t *f_coeff_k,
                         uint64_t *f_k, uint64_t *w_ccs_k, const ring::NegaTables &fwd, int *err,
                         hipStream_t st);
// b_small = 2, d = 1024: decomposition of nside (<= 2) witnesses in one launch
// that also writes digit planes 1..K-1 of side s as i8-MFMA operand rows
// row0[s] .. row0[s] + K - 2 (vector-major, Lp = L order); smg[s]: N 512 u32
// for side s's packed coefficients (the caller's planes or scratch)
struct FusedSides {
  const uint64_t *f_coeff[2];
  // f_k may be null (d = 1024: the planes stay in the operand rows); d = 24: f_k and
  // f_coeff_k both null keeps the planes packed (the masks below are then required)
  uint64_t *f_coeff_k[2], *f_k[2], *w_ccs_k[2];
  int row0[2];                                   // operand row of plane 1 (planes 1 .. K-1 consecutive)
  int nside;
  int row_p0[2] = {-1, -1};                      // operand row of plane 0, or -1 (not written)
  uint2 *masks[2] = {nullptr, nullptr};          // d = 24, b_small = 2: digit masks [K][N] (nonzero, negative), or null
  uint32_t *smg[2] = {nullptr, nullptr};         // packed sign|magnitude words: d = 1024 fused [N][512], d = 24 [N][12];
                                                 // d = 4096 fused: [N][K][256] bytes (nibble | signs << 4)
  uint8_t *dead = nullptr;                       // d = 1024 fused: dead-unit flags of the rows written (DeadUnits)
  int prepacked = 0;                             // d = 1024 fused: bit s = side s's smg is already written
                                                 // (from_w_ccs wrote it; only side 1 may be)
};
// f_0 = sum_v rho_v f_v with every f_v read from the D8 operand rows (k_fold_frag)
struct FoldRows {
  int row[LF_MAX_VECS];   // operand row of vector v
  int rho[LF_MAX_VECS];   // its rho index
  int n;
  DeadUnits dead;         // units the decomposition left unwritten (zero)
};
hipError_t fold_frag(const uint4 *frag, const FragGeom &g, const FoldRows &fr, const uint64_t *rho, int d, size_t N,
                     uint64_t *out, hipStream_t st, const int *run_if = nullptr);
// sink: an 8 KiB device scratch row (stores of groups past W); ncu: the device's CU count
hipError_t decompose_fused(const FusedSides &sd, size_t N, int lb, int L, int K, const ring::NegaTables &fwd, uint4 *frag, int nch, int *err, uint64_t *sink, int ncu,
                           hipStream_t st);

// f_0 in coefficient form on the i8 matrix cores (fold_coeff.hip), X^1024 + 1, b_small = 2:
// keys [ncol = nside N][K][64] u32 from decompose_fused's packed coefficients (smg);
// rho (nw = 2K NTT elements) -> rc (nw 1024 u64 scratch, its coefficients) -> tab
// [nw][FOLD_RT] bytes, *bad = 1 if a coefficient is outside [-127, 127];
// fold_coeff writes f0c = the canonical coefficients of sum_i rho_i f_i unless *bad
constexpr int FOLD_RT = 2080;
// nz (may be null): [ncol] u32, bit k = plane k of the column has a nonzero digit
hipError_t fold_keys(const uint32_t *smg, size_t ncol, int K, uint32_t *keys, hipStream_t st, uint32_t *nz = nullptr);
// sync: two ints, zero before the first launch; every launch leaves them zero
hipError_t fold_rho_tables(const uint64_t *rho, int nw, uint64_t *rc, uint8_t *tab, int *bad,
                           const ring::NegaTables &inv, int *sync, hipStream_t st);
// part: fold_coeff_splits() N 1024 int32 of scratch for the witness-split partial
// sums when there are few elements (or null: no split)
int fold_coeff_splits(size_t N, int K, int ncu);
// fold_coeff's fallback for a rho that is not short (*bad): f_0 (NTT form) from the
// D8 operand rows in the same launch (the packed-plane step; frag == null: none)
struct FoldFallback {
  const uint4 *frag;
  int nch, Lp;
  size_t Wp;
  FoldRows fr;
  const uint64_t *rho;
  uint64_t *f0;
};
// L: the gadget length (elements g L + l; the tiles are limb-pure); nz: both sides'
// plane masks [2 N] from fold_keys (null: every plane is multiplied)
hipError_t fold_coeff(const uint32_t *keys, const uint8_t *tab, const int *bad, size_t N, int K, uint64_t *f0c,
                      int ncu, hipStream_t st, int32_t *part = nullptr, const FoldFallback *fb = nullptr, int L = 1,
                      const uint32_t *nz = nullptr);
// Witness::from_f given f's coefficients: f = NTT(f_coeff), w_ccs = recompose(f); gate: as
// fold_coeff. With inv, a set gate runs Witness::from_f of f instead (f_coeff = ICRT(f),
// w_ccs = recompose(f)) in the same launch: the NTT-form fold's fallback path
hipError_t from_fcoeff_n32(uint64_t *f_coeff, size_t W, int lb, int L, uint64_t *f, uint64_t *w_ccs,
                           const ring::NegaTables &fwd, const int *gate, hipStream_t st,
                           const ring::NegaTables *inv = nullptr);

// d = 24: both sides of a fold step in one launch (blockIdx.z = side); frag as decompose_witness
// *masks_written: whether the launch filled sd.masks (the wave-local kernel does);
// *dead_written: whether it left zero units unwritten and flagged them in sd.dead
// (the wave-local kernel with frag and sd.dead; the block kernel writes every row)
hipError_t decompose_phi72_sides(const FusedSides &sd, size_t N, int lb, int L, int lbs, int K, int *err,
                                 uint4 *frag, int nch, hipStream_t st, bool *masks_written = nullptr,
                                 bool *dead_written = nullptr);
// f_0 in coefficient form from the decomposition's digit masks (d = 24, b_small = 2):
// rho (2K NTT elements) -> rc [2K][25] packed 16-bit coefficient pairs, *bad = 1 if
// one is outside [-32, 32]; unless *bad: f0_coeff = sum_i rho_i * D_i, f0 = CRT(f0_coeff),
// w_ccs0 = recompose(f0) (folding.rs:258-268 then Witness::from_f, arith.rs:299-313)
hipError_t fold_phi72_rho(const uint64_t *rho, int nw, uint32_t *rc, int *bad, hipStream_t st);
hipError_t fold_phi72_coeff(const uint2 *masks0, const uint2 *masks1, const uint32_t *rc, const int *bad, size_t N,
                            int K, int L, int lb, uint64_t *f0_coeff, uint64_t *f0, uint64_t *w_ccs0, hipStream_t st);
// f_0 (NTT form) = CRT(sum_i ICRT(rho_i) * D_i) from the digit masks for any rho (run_if: only when *run_if != 0)
hipError_t fold_phi72_masks(const uint2 *masks0, const uint2 *masks1, const uint64_t *rho, int K, size_t N,
                            uint64_t *f0, const int *run_if, hipStream_t st);
// packed Phi_72 planes (n elements) -> f_coeff (digits mod p) and / or f = CRT(f_coeff)
hipError_t expand_phi72(const uint2 *planes, size_t n, uint64_t *fc, uint64_t *f, hipStream_t st);
// d = 1024: the fused decomposition's packed sign|magnitude words of N elements -> f_coeff_k [K][N]
hipError_t expand_sm(const uint32_t *smg, size_t N, int K, uint64_t *fck, hipStream_t st);
// d = 4096: the fused decomposition's packed bytes (N K 256 words) -> f_coeff_k [K][N][4096]
hipError_t expand_sm8(const uint32_t *sm8, size_t N, int K, uint64_t *fck, hipStream_t st);
// d = 4096, b_small = 2 (kernels_n4k.hip): sm4 holds nside N 1024 packed words; sink 4096 words.
// With frag (a scheme whose geometry has Lp = L and qperm), planes k >= 1 are also
// written as operand rows row0[side] + k - 1, as decompose_fused does for d = 1024.
hipError_t decompose_n4k(const FusedSides &sd, size_t N, int lb, int L, int K, uint64_t *sm4,
                         const ring::NegaTables &fwd, int *err, uint64_t *sink, int ncu, hipStream_t st,
                         uint4 *frag = nullptr, int nch = 0);

// d = 4096 Witness::from_f / from_w_ccs on the quarter transforms (kernels_n4k.hip)
hipError_t from_f_n4k(const uint64_t *f, size_t W, int lb, int L, uint64_t *f_coeff, uint64_t *w_ccs,
                      const ring::NegaTables &inv, hipStream_t st);
hipError_t from_w_ccs_n4k(const uint64_t *w_ccs, size_t W, int lb, int L, uint64_t *f_coeff, uint64_t *f,
                          const ring::NegaTables &fwd, const ring::NegaTables &inv, int *err, hipStream_t st);

// ---------------------------------------------------------------- sumcheck (sumcheck.hip)
// the multisets S_i of a CCS (linearization polynomial), by value as a kernel argument
constexpr int LF_MAX_MULTISETS = 64, LF_MAX_S = 512;
struct CombS {
  int q;
  int off[LF_MAX_MULTISETS + 1];
  short idx[LF_MAX_S];
};
int slot_words(int d);  // words of one NTT slot: 3 (Fq3, Phi_72) or 1
hipError_t eq_table(const uint64_t *r, int nv, int d, uint64_t *out, hipStream_t st);
// Witness::get_fhat: tau = d / slots MLEs of 2^nv points from N <= 2^nv coefficient elements
// nw witnesses wstride u64 apart -> nw consecutive groups of tau MLEs
hipError_t get_fhat(const uint64_t *f_coeff, size_t N, int d, int nv, uint64_t *out, hipStream_t st, int nw = 1,
                    size_t wstride = 0);
// z_k = x_k || w_k for nz instances: out [nz][l1 + W][d]
hipError_t assemble_z(const uint64_t *x, const uint64_t *w, int nz, size_t l1, size_t W, int d, uint64_t *out,
                      hipStream_t st);
// out[m][b] = in[m][2b] + r (in[m][2b+1] - in[m][2b]), b < half; r_base: slot_words(d) words
// ptrs (device, nm pointers, optional): MLE m at ptrs[m] instead of in + m in_stride
hipError_t mle_fix_first(const uint64_t *in, size_t in_stride, int nm, size_t half, int d, const uint64_t *r_base,
                         uint64_t *out, size_t out_stride, hipStream_t st, const uint64_t *const *ptrs = nullptr);
// nf: the f_hat MLEs the folding round may split over chunks (1 for linearization)
size_t round_partial_elems(int d, size_t half, int nevals, int nf);
hipError_t fold_weights(const uint64_t *mu, int nk, int tau, int d, uint64_t *w, hipStream_t st);
// evals [2 bsmall + 1][d]: the folding polynomial's round sums over `half` points;
// mles: 5 + nf MLEs at stride u64 apart; w: nf Horner weights
hipError_t round_folding(const uint64_t *mles, size_t stride, int nf, const uint64_t *w, int bsmall, size_t half, int d,
                         uint64_t *partial, uint64_t *evals, hipStream_t st);
// the folding round 0 (b_small = 2) with the 2K tau f_hat MLEs given by digit coefficient
// rows (fc0: the K witnesses of side 0, fc1 of side 1, wstride u64 apart, N elements):
// mles holds only the 5 general MLEs; evals [5][d]
hipError_t round_folding0_digits(const uint64_t *mles, size_t stride, const uint64_t *fc0, const uint64_t *fc1, int K,
                                size_t N, size_t wstride, int nf, const uint64_t *w, size_t half, int d,
                                uint64_t *partial, uint64_t *evals, hipStream_t st);
// those f_hat MLEs fixed by the first challenge (out: nf MLEs of half elements, out_stride apart)
hipError_t fix_fhat_digits(const uint64_t *fc0, const uint64_t *fc1, int K, size_t N, size_t wstride, int nf,
                           size_t half, int d, const uint64_t *r_base, uint64_t *out, size_t out_stride,
                           hipStream_t st);
// io[x] += sum_(k, j) coef[k tau + j] fhat_(k, j)[x] for the nw digit witnesses of fc (2^nv points)
hipError_t fhat_lincomb_digits(const uint64_t *fc, int nw, size_t N, size_t wstride, const uint64_t *coef, int nv,
                               int d, uint64_t *io, hipStream_t st);
hipError_t round_lin(const uint64_t *mles, size_t stride, int nm, const uint64_t *c, const CombS &cs, int degree,
                     size_t half, int d, uint64_t *partial, uint64_t *evals, hipStream_t st,
                     const uint64_t *const *ptrs = nullptr);
// evals [degree][d]: q(0 .. degree-1) of the linearization round with eq(beta) split
// off (E: eq over the unbound variables, half points); see k_round_lin_eq
hipError_t round_lin_eq(const uint64_t *mles, size_t stride, const uint64_t *E, const uint64_t *c, const CombS &cs,
                        int degree, size_t half, int d, uint64_t *partial, uint64_t *evals, hipStream_t st,
                        const uint64_t *const *ptrs = nullptr);
// round 0 of the split-eq linearization over the multisets' active points: block g
// runs multiset bms[g] on act[boff[g] .. bend[g]); evals [degree][d]
hipError_t round_lin_eq_sparse(const uint64_t *const *ptrs, const uint64_t *E, const uint64_t *c, const CombS &cs,
                               int degree, const uint32_t *act, const int *bms, const uint32_t *boff,
                               const uint32_t *bend, int nblk, int d, uint64_t *partial, uint64_t *evals,
                               hipStream_t st);
size_t round_lin_sparse_ppb(int d);  // points per block pass of round_lin_eq_sparse
// E_next[b] = E[2b] + E[2b+1] for b < half (whole ring elements)
hipError_t pair_sum(const uint64_t *E, size_t half, int d, uint64_t *out, hipStream_t st);
size_t mle_eval_partial_elems(int d, int nm);
// out[m] = sum_x eq[x] (.) mles[m][x], x < n
hipError_t mle_dot(const uint64_t *mles, size_t stride, int nm, const uint64_t *eq, size_t n, int d,
                   uint64_t *partial, uint64_t *out, hipStream_t st);
// out [nw][tau][d]: the f_hat MLEs of nw witnesses (f_coeff rows wstride u64 apart, N
// elements each) evaluated against the eq table, without materialising f_hat
hipError_t fhat_dot(const uint64_t *fc, size_t N, size_t wstride, int nw, const uint64_t *eq, size_t n, int d,
                    uint64_t *partial, uint64_t *out, hipStream_t st);
// io[x] += sum_m coef[m] (.) mles[m][x], x < n; coef [nm][d]
hipError_t mle_lincomb(const uint64_t *mles, size_t stride, int nm, const uint64_t *coef, size_t n, int d,
                       uint64_t *io, hipStream_t st);

// ---------------------------------------------------------------- width-8 Poseidon2 Merkle trees (merkle.hip)
hipError_t p2w8_permute(uint64_t *states, size_t n, hipStream_t st);
// nodes: merkle_nodes(nrows) x 4 digests (Plonky3's even-padded layers; 2 nrows - 1 for a
// power of two), leaves first, each level after the one below, root last
size_t merkle_nodes(size_t nrows);
hipError_t merkle_tree(const uint64_t *rows, size_t nrows, size_t width, uint64_t *nodes, hipStream_t st);
hipError_t hash_w8_rows(const uint64_t *rows, size_t nrows, size_t width, uint64_t *out, hipStream_t st);

// ---------------------------------------------------------------- sparse Mz products (mz.hip)
// the t CCS matrices (m x n, ring-element CSR) on the device, with the
// row-merged [M_0 | .. | M_(t-1)] and the per-matrix transposes as index arrays
// into the one value array
struct CcsDev {
  int d, t;
  size_t m, n;
  const uint64_t *rp;  // [t][m + 1], absolute offsets into col / val
  const uint32_t *col;
  const uint64_t *val;  // [nnz][d]
  const uint64_t *sval = nullptr;  // [nnz] when every entry is a scalar (v in every slot word 0, zero elsewhere)
  const uint64_t *svh = nullptr;   // sval in the row-merged order (svh[k] = sval[hidx[k]])
  const uint64_t *svc = nullptr;   // sval in the transposes' order (svc[k] = sval[cidx[k]])
  // ring-valued entries in the row-merged and transposes' orders (vh[k] = val[hidx[k]],
  // vc[k] = val[cidx[k]], d words each; null: those products gather through hidx / cidx)
  const uint64_t *vh = nullptr, *vc = nullptr;
  const uint64_t *hrp;  // [m + 1]
  const uint32_t *hcol;  // j n + col
  const uint32_t *hidx;  // value index
  const uint64_t *crp;  // [t][n + 1]
  const uint32_t *crow;
  const uint32_t *cidx;
};
size_t mz_scratch_elems(const CcsDev &M, int nz, int nv);
// out[k] = val[idx[k]] for k < nnz, d words each (CcsDev::vh / vc)
hipError_t gather_entries(const uint64_t *val, const uint32_t *idx, size_t nnz, int d, uint64_t *out, hipStream_t st);
// scratch words of one side of mz_challenged(_pair): the zeta powers, for d = 24 the
// matrix-core operand pieces, and y = sum_i zeta_i^(j+1) z_i ([t][n][d])
size_t mz_chall_elems(const CcsDev &M, int nz);
// out [nz][t][2^nv][d] = MLE(M_j z_i), zero-padded; z [nz][n][d]
// sel (device, optional): out holds the MLEs of matrices sel[0 .. nsel) in that order
hipError_t mz_mles(const CcsDev &M, const uint64_t *z, int nz, int nv, uint64_t *out, hipStream_t st,
                   const int *sel = nullptr, int nsel = 0);
// out [2^nv][d] = sum_i sum_j zeta_i^(j+1) MLE(M_j z_i)
// mz_challenged for two (z, zeta) at once over one pass of the row-merged matrix;
// scratch: 2 mz_chall_elems elements
hipError_t mz_challenged_pair(const CcsDev &M, const uint64_t *z0, const uint64_t *zeta0, const uint64_t *z1,
                              const uint64_t *zeta1, int nz, int nv, uint64_t *out0, uint64_t *out1,
                              uint64_t *scratch, hipStream_t st);
hipError_t mz_challenged(const CcsDev &M, const uint64_t *z, const uint64_t *zeta, int nz, int nv, uint64_t *out,
                         uint64_t *scratch, hipStream_t st);
// out [nz][t][d] = MLE(M_j z_i)(point)
// the evaluation route in two halves: w [t][n] = M_j^T eq (one point, any number of z
// sets), then out [nz][t] = w_j . z_i
hipError_t mz_weights(const CcsDev &M, const uint64_t *eq, uint64_t *w, hipStream_t st);
// partial (optional): mz_dots_partial_elems(M, nz) u64 of scratch for column splits
// when t nz blocks would not fill the chip
hipError_t mz_dots(const CcsDev &M, const uint64_t *w, const uint64_t *z, int nz, uint64_t *out, hipStream_t st,
                   uint64_t *partial = nullptr);
size_t mz_dots_partial_elems(const CcsDev &M, int nz);
hipError_t mz_evaluate(const CcsDev &M, const uint64_t *z, int nz, int nv, const uint64_t *point, uint64_t *out,
                       uint64_t *scratch, hipStream_t st);

}  // namespace lfk
