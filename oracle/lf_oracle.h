/*
 * lf_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C CPU restatement of the reference (Nesquiko/Latticeum) LatticeFold
 * commit+fold arithmetic. It is the parity checker for the HIP product path in
 * latticeum_amd/: only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it, and never as the thing measured or shipped.
 *
 * Parity pinning:
 *   - d = 24 (Phi_72 ring) restates the reference Rust line by line and is
 *     pinned by the reference's own known-answer tests (tests/golden/ KAT files).
 *   - d = 2^k negacyclic rings (X^d + 1) do not exist in the reference; they are
 *     this project's own convention and are pinned only by definition
 *     (schoolbook products, direct evaluation) -- "parity unpinned" vs reference.
 *   - The Poseidon2 permutation beyond initial MDS + external round 0, and the
 *     DuplexChallenger buffering, are "parity unpinned" (Plonky3 is absent).
 *
 * All values are canonical u64 in [0, p), p = 2^64 - 2^32 + 1 unless a
 * function says "Montgomery".
 */
#ifndef LF_ORACLE_H
#define LF_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- field (GL/mod.rs:16-27: modulus 18446744069414584321, generator 7) ---- */
uint64_t lfo_add(uint64_t a, uint64_t b);
uint64_t lfo_sub(uint64_t a, uint64_t b);
uint64_t lfo_mul(uint64_t a, uint64_t b);
uint64_t lfo_pow(uint64_t a, uint64_t e);
uint64_t lfo_inv(uint64_t a);
uint64_t lfo_to_mont(uint64_t a);   /* a * 2^64 mod p (ark-ff internal limb) */
uint64_t lfo_from_mont(uint64_t m); /* m * 2^-64 mod p */

/* ---- ring transforms, batched over n elements of d u64 each (AoS) ---- */
/* d == 24: Phi_72 CRT (GL/ntt.rs:135-228 + homogenize :326-334)
 * d == 2^k: negacyclic NTT, slot k = f(psi^(2k+1)), psi = 7^((p-1)/2d) */
void lfo_crt(uint64_t *elems, size_t n, int d);
void lfo_icrt(uint64_t *elems, size_t n, int d);
/* Phi_72 only: expose homogenize / dehomogenize (GL/ntt.rs:326-346) for KATs */
void lfo_phi72_homogenize(uint64_t *c24);
void lfo_phi72_dehomogenize(uint64_t *c24);
/* coefficient-form ring product (schoolbook + reduce):
 * d == 24 mod X^24 - X^12 + 1 (coeff_form.rs:54-67 + GL/mod.rs:75-98),
 * d == 2^k mod X^d + 1 */
void lfo_poly_mul(const uint64_t *a, const uint64_t *b, uint64_t *out, int d);
/* NTT-form slot-wise product (ntt_form.rs:159-175): Fq3 slots for d=24 */
void lfo_slot_mul(const uint64_t *a, const uint64_t *b, uint64_t *out, int d);

/* ---- balanced decomposition (SR/balanced_decomposition/mod.rs:62-103) ----
 * returns 0 on success, -1 if v needs more than len digits (reference panics) */
int lfo_decompose_balanced(uint64_t v, uint64_t b, int len, uint64_t *out);
/* GadgetDecompose for &[R] (mod.rs:163-175): n elements -> n*len elements,
 * digit k of coeff c of elem j -> out[(j*len + k)*d + c] */
int lfo_gadget_decompose(const uint64_t *in, size_t n, int d, uint64_t b, int len,
                         uint64_t *out);
/* GadgetRecompose (mod.rs:177-190), coordinate-wise Horner over u64 slots */
void lfo_gadget_recompose(const uint64_t *in, size_t n_out, int d, uint64_t b, int len,
                          uint64_t *out);

/* ---- Witness (LF/arith.rs:230-338) ----
 * from_w_ccs: w_ccs (W, NTT) -> f_coeff (W*L, coeff), f (W*L, NTT) */
int lfo_witness_from_w_ccs(const uint64_t *w_ccs, size_t W, int d, uint64_t B, int L,
                           uint64_t *f_coeff, uint64_t *f, int nthreads);
/* from_f: f (N, NTT) -> f_coeff (N), w_ccs (N/L) */
void lfo_witness_from_f(const uint64_t *f, size_t N, int d, uint64_t B, int L,
                        uint64_t *f_coeff, uint64_t *w_ccs, int nthreads);
/* get_fhat (LF/arith.rs:273-297) for d=24: tau=3 MLEs of N NTT elements whose
 * Fq3 slots are (coeff,0,0); out layout [tau][N][24] (no lnze truncation). */
void lfo_get_fhat_phi72(const uint64_t *f_coeff, size_t N, uint64_t *out);

/* ---- Ajtai (LF/commitment/commitment_scheme.rs:37-54, LA/matrix.rs:168-178) ----
 * A: kappa x ncols ring elements row-major; f: nvec vectors of ncols elems;
 * cm: nvec x kappa elems. Threads split over rows like rayon. */
void lfo_ajtai_commit(const uint64_t *A, size_t kappa, size_t ncols, int d,
                      const uint64_t *f, size_t nvec, uint64_t *cm, int nthreads);

/* ---- decomposition prover hot parts (LF/nifs/decomposition.rs:162-201) ----
 * decompose_witness: f_coeff (N, coeff) -> K witnesses via from_f_coeff:
 *   f_coeff_k [K][N], f_k [K][N], w_ccs_k [K][N/L] */
int lfo_decompose_witness(const uint64_t *f_coeff, size_t N, int d, uint64_t B, int L,
                          uint64_t b_small, int K, uint64_t *f_coeff_k, uint64_t *f_k,
                          uint64_t *w_ccs_k, int nthreads);
/* commit_witnesses y_0 fix-up: y[0] = cm - sum_{k>=1} b^k y[k]; y: [K][kappa] */
void lfo_commit_witnesses_y0(const uint64_t *cm, uint64_t *y, size_t kappa, int d,
                             uint64_t b_small, int K);

/* ---- folding (LF/nifs/folding.rs:258-268, folding/utils.rs:116-127,456-517) ---- */
/* short challenge (CR/rings/goldilocks.rs:41-67); generalised to 3d/4 bytes */
int lfo_short_challenge(const uint8_t *bytes, size_t nbytes, int d, uint64_t *coeffs);
/* f_0 = sum_i rho_i * f_i (NTT); rho: [nwit][d] NTT; f: [nwit][N][d] */
void lfo_fold_f0(const uint64_t *rho, const uint64_t *f, size_t nwit, size_t N, int d,
                 uint64_t *f0, int nthreads);
/* cm_0 = sum_i rho_i * cm_i; cm: [nwit][kappa][d] */
void lfo_fold_cm0(const uint64_t *rho, const uint64_t *cm, size_t nwit, size_t kappa, int d,
                  uint64_t *cm0);

/* rot_lin_combination (CR/rotation.rs:84-101): v_0 from rho_i (coefficient
 * form, [n][d]) and theta_i ([n][tau d] u64, tau = 3 for d = 24, 1 otherwise);
 * v0: tau d u64 */
void lfo_rot_lin_combination(const uint64_t *rho_coeff, const uint64_t *theta, size_t n, int d,
                             uint64_t *v0);
/* compute_x_s (LF/nifs/decomposition.rs:172-175): x (m NTT elems) -> x_s [K][m] */
int lfo_compute_x_s(const uint64_t *x, size_t m, int d, uint64_t B, int L, uint64_t b_small, int K,
                    uint64_t *x_s);

/* ---- Poseidon2 width 16 (ZK/poseidon2.rs:100-173, 243-268) ---- */
void lfo_p2_mds16(uint64_t *s);
void lfo_p2_permute(uint64_t *s);
void lfo_p2_permute_batch(uint64_t *states, size_t n, int nthreads);
/* hash_iter (ZK/poseidon2.rs:206-235): overwrite sponge, rate 12, out state[0..4] */
void lfo_p2_hash_iter(const uint64_t *in, size_t n, uint64_t out[4]);
/* PermutationIntermediateStates (ZK/poseidon2.rs:91-96): st = 31 x 16 words */
void lfo_p2_permute_states(uint64_t *s, uint64_t *st);
/* hash_iter's IntermediateStates: states [nperm][31][16]; returns nperm = ceil(n / 12) */
size_t lfo_p2_hash_iter_states(const uint64_t *in, size_t n, uint64_t out[4], uint64_t *states);

/* ---- width-8 Poseidon2 and Merkle trees (zkvm commitments.rs; parity unpinned: Plonky3 diag) ---- */
void lfo_p2w8_permute(uint64_t *s);
void lfo_p2w8_hash(const uint64_t *in, size_t n, uint64_t out[4]);
void lfo_p2w8_compress(const uint64_t a[4], const uint64_t b[4], uint64_t out[4]);
size_t lfo_merkle_nodes(size_t nrows);
void lfo_merkle_tree(const uint64_t *rows, size_t nrows, size_t width, uint64_t *nodes);

/* ---- transcript (ZK/fiat_shamir.rs) over DuplexChallenger<16,12> ---- */
typedef struct {
  uint64_t state[16];
  uint64_t inbuf[12];
  int nin;
  uint64_t outbuf[12];
  int nout;
} lfo_transcript;
void lfo_tr_init(lfo_transcript *t);
void lfo_tr_observe(lfo_transcript *t, uint64_t v);
uint64_t lfo_tr_sample(lfo_transcript *t);
/* absorb NTT ring elements (canonical in) as Montgomery limbs (fiat_shamir.rs:51-60) */
void lfo_tr_absorb_ring(lfo_transcript *t, const uint64_t *elems, size_t n, int d);
void lfo_tr_get_challenge(lfo_transcript *t, uint64_t out[3]);
void lfo_tr_squeeze_bytes(lfo_transcript *t, uint8_t *out, size_t n);

/* ---- multilinear sumcheck (8(f) rank 1): LF/utils/sumcheck*, PL/mle/dense.rs ----
 * ring elements in NTT form (d u64); MLEs over nv variables: 2^nv elements */
void lfo_eq_table(const uint64_t *r, int nv, int d, uint64_t *out);
void lfo_mle_fix_first(uint64_t *mle, size_t half, int d, const uint64_t *r);
void lfo_mle_evaluate(const uint64_t *mle, int nv, int d, const uint64_t *point, uint64_t *out);
typedef struct {
  int kind; /* 0 folding, 1 linearization */
  int nk, tau, bsmall;
  const uint64_t *mu;
  int q;
  const uint64_t *c;
  const int *S_off;
  const int *S_idx;
} lfo_comb;
void lfo_comb_eval(const lfo_comb *cb, const uint64_t *vals, int nm, int d, uint64_t *out);
void lfo_sumcheck_round(const lfo_comb *cb, const uint64_t *mles, int nm, int nv, int d, int degree,
                        uint64_t *evals);
void lfo_sumcheck_prove(lfo_transcript *t, const lfo_comb *cb, uint64_t *mles, int nm, int nv, int d, int degree,
                        uint64_t *proof, uint64_t *randomness);
int lfo_sumcheck_check(const uint64_t *proof, const uint64_t *randomness, int nv, int d, int degree,
                       const uint64_t *asserted_sum, uint64_t *expected_out);

/* ---- sparse Mz products: mat_vec_mul (LF/arith/utils.rs:52-65) over a CSR matrix of ring elements */
void lfo_spmv(const uint64_t *row_ptr, const uint32_t *col, const uint64_t *val, size_t nrows, int d,
              const uint64_t *z, uint64_t *y);

/* ---- seeded synthetic inputs: SplitMix64 stream, rejection to [0,p) ---- */
void lfo_fill_uniform(uint64_t *out, size_t n, uint64_t seed);
/* rows[0..nrows) of A f for A = lfo_fill_uniform(seed) as kappa x ncols x d
 * (generated on the fly, never stored): cm [nrows][d] */
void lfo_ajtai_rows_seeded(uint64_t seed, size_t ncols, int d, const uint64_t *f, const size_t *rows,
                           size_t nrows, uint64_t *cm, int nthreads);

#ifdef __cplusplus
}
#endif
#endif
