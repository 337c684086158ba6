/*
 * lf.h -- C ABI of latticeum_amd: the MI355X (gfx950) implementation of the
 * LatticeFold commit+fold hot path of Nesquiko/Latticeum.
 *
 * Reference interfaces replaced (paths under latticeum/crates/):
 *   stark-rings/crates/ring/src/cyclotomic_ring/ring_config.rs:11-35
 *       CyclotomicConfig::{crt_in_place, icrt_in_place}      -> lf_crt / lf_icrt
 *   stark-rings/crates/ring/src/cyclotomic_ring/crt.rs:10-45
 *       CRT::elementwise_crt / ICRT::elementwise_icrt          -> lf_crt / lf_icrt (batched)
 *   stark-rings/crates/ring/src/cyclotomic_ring/ntt_form.rs:159-189
 *       RqNTT Mul / MulUnchecked                               -> lf_ring_mul
 *   latticefold/src/commitment/commitment_scheme.rs:23-78
 *       AjtaiCommitmentScheme::{new, commit, commit_ntt, kappa, width}
 *                                                              -> lf_ajtai_*
 *   latticefold/src/arith.rs:230-338
 *       Witness::{from_w_ccs, from_f, from_f_coeff}            -> lf_witness_*
 *   latticefold/src/nifs/decomposition.rs:162-201
 *       decompose_witness / commit_witnesses                   -> lf_decompose_witness,
 *                                                                 lf_dev_commit_y0
 *   latticefold/src/nifs/folding.rs:258-268, folding/utils.rs:456-517
 *       compute_f_0 / cm_0                                     -> lf_dev_fold
 *       compute_v0_u0_x0_cm_0: u_0, x_0, v_0                   -> lf_fold_lcccs / lf_dev_fold_lcccs
 *   cyclotomic-rings/src/rotation.rs:84-101 rot_lin_combination -> lf_fold_lcccs (v_0)
 *   latticefold/src/nifs/decomposition.rs:172-175 compute_x_s  -> lf_compute_x_s / lf_dev_compute_x_s
 *   cyclotomic-rings/src/rings/goldilocks.rs:41-67
 *       short_challenge_from_random_bytes                      -> lf_short_challenge
 *   zkvm/src/poseidon2.rs:100-235
 *       WideZkVMPoseidon2Perm::permute_mut, hash_iter          -> lf_poseidon2_permute,
 *                                                                 lf_hash_iter
 *   zkvm/src/fiat_shamir.rs:20-114  Poseidon2Transcript         -> lf_transcript_*
 *   zkvm/src/main.rs:348-367  commit()                          -> lf_commit
 *   zkvm/src/main.rs:380-404  fold() (its commit+fold arithmetic) -> lf_fold_hot /
 *                                                                 lf_dev_fold_step,
 *                                                                 lf_dev_fold_step_batch
 *   zkvm/src/commitments.rs:192-340 vm_mem_comm, vm_mem_comm_with_opening, vm_code_comm
 *                                                              -> lf_vm_mem_comm, lf_dev_merkle_tree,
 *                                                                 lf_merkle_open, lf_vm_code_comm
 *   latticefold/src/nifs.rs:28-34 LFProof (ark CanonicalSerialize) -> lf_lfproof_serialize
 *       zkvm/src/main.rs:231-234 (serialized_size); the LCCCS layout (lf_lcccs_(de)serialize)
 *       is this project's own (the reference serialises no LCCCS)
 *   zkvm/src/zk_latticefold.rs:37-102 zk_latticefold_prove (fold())  -> lf_fold_prove
 *   zkvm/src/main.rs:305-344 initialize_accumulator's linearization  -> lf_linearize
 *   zkvm/src/zk_latticefold.rs:111-148 generate_verification_witness_vars -> lf_fold_replay
 *   zkvm/src/main.rs:121-219  the proving loop, sharded over GPUs (SURVEY.md 8(b)
 *       lf_fold_reduce_allranks; no reference analogue: rayon only)
 *                                                              -> lf_comm_*, lf_dev_fold_step_sharded,
 *                                                                 lf_fold_reduce_allranks
 *
 * Data: a ring element is d u64 (AoS). d = 24 is the reference's Goldilocks
 * ring Fq[X]/(X^24 - X^12 + 1); its NTT form is 8 Fq3 slots laid out
 * [s0.c0, s0.c1, s0.c2, s1.c0, ...] exactly as the reference's in-place CRT
 * (crt.rs:53-77). d in {16, 64, 256, 1024, 4096} selects Fq[X]/(X^d + 1)
 * (no reference analogue; NTT slot k = f(psi^(2k+1)), psi = 7^((p-1)/2d)).
 * Host-buffer calls take repr = LF_REPR_MONTGOMERY when the buffers are raw
 * ark-ff Fp64 limbs (zero-copy from Rust Vec<RqNTT>), LF_REPR_CANONICAL
 * otherwise. Device (lf_dev_*) calls are canonical and asynchronous on the
 * context stream; decomposition overflow is reported by lf_ctx_sync().
 *
 * Threading: a context is single-threaded (like the reference's &mut
 * transcript); distinct contexts may be used from distinct threads. Every
 * call runs on its context's device and restores the calling thread's current
 * device before it returns.
 */
#ifndef LATTICEUM_AMD_LF_H
#define LATTICEUM_AMD_LF_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct lf_ctx lf_ctx;
typedef struct lf_ajtai lf_ajtai;
typedef struct lf_transcript lf_transcript;
typedef struct lf_comm lf_comm;
typedef struct lf_ccs lf_ccs;

enum lf_status {
  LF_OK = 0,
  LF_ERR_INVALID_ARG = 1,
  LF_ERR_UNSUPPORTED_RING = 2,
  LF_ERR_WRONG_WITNESS_LENGTH = 3,    /* CommitmentError::WrongWitnessLength (commitment.rs:16-17) */
  LF_ERR_WRONG_COMMITMENT_LENGTH = 4, /* CommitmentError::WrongCommitmentLength (commitment.rs:19-20) */
  LF_ERR_WRONG_AJTAI_DIMENSIONS = 5,  /* CommitmentError::WrongAjtaiMatrixDimensions (:22-25) */
  LF_ERR_DECOMPOSITION_OVERFLOW = 6,  /* value needs more digits than padding (reference panics) */
  LF_ERR_INCORRECT_LENGTH = 7,        /* Decomposition/FoldingError::IncorrectLength (nifs/error.rs) */
  LF_ERR_CHALLENGE_BYTES = 8,         /* ChallengeSetError::TooFewBytes */
  LF_ERR_DEVICE = 9,                  /* HIP runtime error (see lf_ctx_last_error) */
  LF_ERR_OUT_OF_MEMORY = 10,
  LF_ERR_COMM = 11,                   /* RCCL error (see lf_ctx_last_error) */
  LF_ERR_VERIFICATION = 12,           /* lf_fold_verify rejected the proof (which check: lf_verify_check) */
  LF_ERR_UNSUPPORTED_CCS = 13         /* lf_prover_create: a multiset names the eq(beta) MLE (see lf_ctx_last_error) */
};
enum lf_repr { LF_REPR_CANONICAL = 0, LF_REPR_MONTGOMERY = 1 };

/* DecompositionParams (latticefold/src/decomposition_parameters.rs:11-20).
 * The device path needs B and b_small to be powers of two (GoldiLocksDP is). */
typedef struct {
  int d;
  uint64_t B;
  int L;
  uint64_t b_small;
  int K;
} lf_params;

/* zkvm GoldiLocksDP (zkvm/src/ccs.rs:26-34): B = 2^15, L = 5, B_SMALL = 2, K = 15 */
lf_params lf_goldilocks_dp(int d);

/* ------------------------------------------------------------ context */
int lf_ctx_create(int device, lf_ctx **out);
void lf_ctx_destroy(lf_ctx *ctx);
const char *lf_status_string(int status);
const char *lf_ctx_last_error(const lf_ctx *ctx);
/* records msg as the context's last error (for entry points that fail before any object exists) */
void lf_ctx_set_error(lf_ctx *ctx, const char *msg);
/* stream used by all work of this context (hipStream_t). A new context uses a
 * non-blocking stream of its own; NULL selects the HIP default (null) stream,
 * which is what torch's default current stream is. */
int lf_ctx_set_stream(lf_ctx *ctx, void *hip_stream);
void *lf_ctx_get_stream(const lf_ctx *ctx);
/* a non-blocking HIP stream of `device` whose kernels run only on the compute
 * units set in mask (nwords 32-bit words, bit i = CU i as the HIP runtime
 * numbers them), for lf_ctx_set_stream: a host can give concurrent step
 * streams disjoint parts of the chip. lf_stream_destroy releases it. */
int lf_stream_create_cu_mask(int device, const uint32_t *mask, int nwords, void **stream);
int lf_stream_destroy(void *stream);
/* compute units this context's stream may use (default: the device's): the
 * grid size of the persistent kernels (the fused decompositions, the
 * coefficient-form fold), so a context on a CU-masked stream fills its part
 * of the chip in one round */
int lf_ctx_set_cu_count(lf_ctx *ctx, int ncu);
/* stream on which lf_dev_fold_step_batch runs the batched contraction of the
 * steps it is called with when ctx is their first context (NULL, the default:
 * ctx's own stream). Every step stream's work before the contraction is
 * ordered before it and the work after it waits for it (HIP events; nothing
 * waits on the host), so with a CU-masked stream here and the step streams on
 * the remaining CUs one group's contraction runs beside the next group's
 * decompositions. The stream must be on ctx's device (LF_ERR_INVALID_ARG
 * otherwise) and outlive its use; the caller keeps ownership, and
 * lf_ctx_destroy waits for it before the context's buffers go. */
int lf_ctx_set_contract_stream(lf_ctx *ctx, void *hip_stream);
/* wait for the stream; returns LF_ERR_DECOMPOSITION_OVERFLOW (and clears it)
 * if any device decomposition since the last sync ran out of digits */
int lf_ctx_sync(lf_ctx *ctx);
/* pre-size internal scratch so no allocation happens inside timed/captured work */
int lf_ctx_reserve(lf_ctx *ctx, size_t kappa, size_t ncols, int d, int nvec);
/* kernel timing: HIP events recorded on the stream around every Ajtai matvec
 * kernel launch (the main kernel only, not its split-K reduction) */
int lf_ctx_kernel_timing(lf_ctx *ctx, int enable);
/* device ms summed over, and number of, timed Ajtai launches with nvec
 * vectors (nvec = 0: all) since timing was enabled; synchronises the stream */
int lf_ctx_kernel_stats(lf_ctx *ctx, int nvec, double *total_ms, long *count);
/* the same for the phases of lf_dev_fold_step (events on the stream around each) */
enum {
  LF_PHASE_FROM_W_CCS = 0, /* commit(z): Witness::from_w_ccs */
  LF_PHASE_DECOMPOSE = 1,  /* decompose_witness, one record per side (fused: + MFMA operand rows) */
  LF_PHASE_TO_FRAG = 2,    /* commit(z)'s f into MFMA operand order (fused path) */
  LF_PHASE_FOLD = 3,       /* f_0 = sum rho_i f_i */
  LF_PHASE_FROM_F = 4,     /* Witness::from_f(f_0) */
  LF_PHASE_COUNT = 5
};
int lf_ctx_phase_stats(lf_ctx *ctx, int phase, double *total_ms, long *count);
/* d = 1024: W below which Witness::from_w_ccs / from_f run one half-wave per
 * (element, limb) instead of one per element (a build constant, LF_SPLIT_W) */
size_t lf_witness_split_w(void);

/* ------------------------------------------------------------ host-buffer API (synchronous) */
int lf_crt(lf_ctx *ctx, uint64_t *elems, size_t n, int d, int repr);
int lf_icrt(lf_ctx *ctx, uint64_t *elems, size_t n, int d, int repr);
int lf_ring_mul(lf_ctx *ctx, const uint64_t *a, const uint64_t *b, uint64_t *out, size_t n, int d,
                int repr);

int lf_ajtai_create(lf_ctx *ctx, const uint64_t *A, size_t kappa, size_t ncols, int d, int repr,
                    lf_ajtai **out);
/* wraps a matrix already in device memory (canonical, AoS row-major); not copied */
int lf_ajtai_create_device(lf_ctx *ctx, const uint64_t *A_dev, size_t kappa, size_t ncols, int d,
                           lf_ajtai **out);
void lf_ajtai_destroy(lf_ajtai *aj);
size_t lf_ajtai_kappa(const lf_ajtai *aj);
size_t lf_ajtai_width(const lf_ajtai *aj);
int lf_ajtai_d(const lf_ajtai *aj);
/* 1 when the scheme keeps A in i8-MFMA fragment order (X^d+1 and Phi_72 rings, kappa <= 128;
 * the AoS matrix given to lf_ajtai_create_device is then no longer read and may
 * be freed), 0 when commitments run on the VALU from the AoS matrix */
int lf_ajtai_layout(const lf_ajtai *aj);
/* commit_ntt: f has f_len NTT elements (must equal width), cm receives kappa */
int lf_ajtai_commit(lf_ctx *ctx, const lf_ajtai *aj, const uint64_t *f, size_t f_len, uint64_t *cm,
                    int repr);

int lf_witness_from_w_ccs(lf_ctx *ctx, const lf_params *pr, const uint64_t *w_ccs, size_t W,
                          uint64_t *f_coeff, uint64_t *f, int repr);
int lf_witness_from_f(lf_ctx *ctx, const lf_params *pr, const uint64_t *f, size_t N,
                      uint64_t *f_coeff, uint64_t *w_ccs, int repr);
/* f_coeff (N) -> f_coeff_k [K][N], f_k [K][N], w_ccs_k [K][N/L] */
int lf_decompose_witness(lf_ctx *ctx, const lf_params *pr, const uint64_t *f_coeff, size_t N,
                         uint64_t *f_coeff_k, uint64_t *f_k, uint64_t *w_ccs_k, int repr);

/* zkvm commit(): z = [x_ccs (l) | 1 | w_ccs (W)] NTT elements; outputs the new
 * witness (f_coeff, f: W*L each) and the CCCS commitment cm (kappa). */
int lf_commit(lf_ctx *ctx, const lf_ajtai *aj, const lf_params *pr, const uint64_t *z, size_t z_len,
              size_t l, uint64_t *f_coeff, uint64_t *f, uint64_t *cm, int repr);

/* The commit+fold arithmetic of zkvm fold() for one step, given the folding
 * challenges rho (2K NTT elements, rho[2K-1] = ONE as get_rhos produces):
 *   decompose (acc, w_acc) and (cm_i, w_i) into K witnesses each, commit 2(K-1)
 *   of them, y_0 = cm - sum b^k y_k, f_0 = sum rho_i f_i, cm_0 = sum rho_i y_i,
 *   and Witness::from_f(f_0).
 * Outputs: y (2K x kappa), f0 / f0_coeff (N), w_ccs0 (N/L), cm0 (kappa). */
int lf_fold_hot(lf_ctx *ctx, const lf_ajtai *aj, const lf_params *pr, const uint64_t *acc_cm,
                const uint64_t *acc_f_coeff, const uint64_t *cm_i, const uint64_t *wi_f_coeff, size_t N,
                const uint64_t *rho, uint64_t *y, uint64_t *f0, uint64_t *f0_coeff, uint64_t *w_ccs0,
                uint64_t *cm0, int repr);

/* The rest of the folded LCCCS (compute_v0_u0_x0_cm_0, folding/utils.rs:456-517),
 * given the folding sumcheck's outputs (theta_s, eta_s) and rho:
 *   u0 = sum_i rho_i (.) eta_i           (t NTT elements; eta: [nwit][t])
 *   x0 = sum_i rho_i (.) (x_w || h)_i     (l1 = l + 1 elements; xwh: [nwit][l1])
 *   v0 = rot_lin_combination(rho_coeff, theta): rho_coeff [nwit][d] coefficient
 *        form, theta [nwit][tau] NTT elements, v0 tau elements (tau = 3 for
 *        d = 24, whose base ring is Fq3; 1 for X^d + 1)
 * t = 0 / l1 = 0 / theta = NULL skip that output. nwit <= 32. */
int lf_fold_lcccs(lf_ctx *ctx, int d, int nwit, const uint64_t *rho, const uint64_t *rho_coeff, const uint64_t *eta,
                  size_t t, const uint64_t *xwh, size_t l1, const uint64_t *theta, uint64_t *u0, uint64_t *x0,
                  uint64_t *v0, int repr);
/* compute_x_s: x = x_w || h (m NTT elements) -> x_s [K][m], the K decomposed
 * statements (decompose_big_vec_into_k_vec_and_compose_back) */
int lf_compute_x_s(lf_ctx *ctx, const lf_params *pr, const uint64_t *x, size_t m, uint64_t *x_s, int repr);

/* short_challenge_from_random_bytes: 3d/4 bytes -> d coefficients in [-32, 32) */
int lf_short_challenge(const uint8_t *bytes, size_t nbytes, int d, uint64_t *coeffs);
/* width-16 Poseidon2 permutation of n independent states (16 canonical u64 each) */
int lf_poseidon2_permute(lf_ctx *ctx, uint64_t *states, size_t n);

/* ------------------------------------------------------------ device-resident API (async) */
int lf_dev_crt(lf_ctx *ctx, uint64_t *elems, size_t n, int d);
int lf_dev_icrt(lf_ctx *ctx, uint64_t *elems, size_t n, int d);
int lf_dev_ring_mul(lf_ctx *ctx, const uint64_t *a, const uint64_t *b, uint64_t *out, size_t n, int d);
int lf_dev_to_montgomery(lf_ctx *ctx, uint64_t *x, size_t n);
int lf_dev_from_montgomery(lf_ctx *ctx, uint64_t *x, size_t n);
int lf_dev_witness_from_w_ccs(lf_ctx *ctx, const lf_params *pr, const uint64_t *w_ccs, size_t W,
                              uint64_t *f_coeff, uint64_t *f);
int lf_dev_witness_from_f(lf_ctx *ctx, const lf_params *pr, const uint64_t *f, size_t N,
                          uint64_t *f_coeff, uint64_t *w_ccs);
int lf_dev_decompose_witness(lf_ctx *ctx, const lf_params *pr, const uint64_t *f_coeff, size_t N,
                             uint64_t *f_coeff_k, uint64_t *f_k, uint64_t *w_ccs_k);
/* nvec (<= 32) vectors of width() NTT elements each -> cm [nvec][kappa] */
int lf_dev_ajtai_commit(lf_ctx *ctx, const lf_ajtai *aj, const uint64_t *const *f_vecs, int nvec,
                        uint64_t *cm);
/* y [K][kappa]: y[0] = cm - sum_{k>=1} b_small^k y[k] */
int lf_dev_commit_y0(lf_ctx *ctx, const lf_params *pr, const uint64_t *cm, uint64_t *y, size_t kappa);
/* out[j] = sum_{i<nwit} rho_i (.) x_i[j], j < n ring elements (nwit <= 32) */
int lf_dev_fold(lf_ctx *ctx, int d, const uint64_t *rho, const uint64_t *const *x, int nwit, size_t n,
                uint64_t *out);

/* device buffers of one commit+fold step (all canonical, caller-allocated) */
typedef struct {
  /* inputs */
  const uint64_t *w_ccs;       /* W: the new CCS witness (commit(z) input, NTT form) */
  const uint64_t *acc_cm;      /* kappa: accumulator commitment (LCCCS.cm) */
  const uint64_t *acc_f_coeff; /* N: accumulator witness f_coeff */
  const uint64_t *rho;         /* 2K NTT elements */
  /* outputs */
  uint64_t *f_coeff, *f;       /* N each: Witness::from_w_ccs(w_ccs) */
  uint64_t *cm;                /* kappa: CCCS.cm = A f */
  uint64_t *fk_coeff[2];       /* [K][N] per side (0 = accumulator, 1 = new instance) */
  uint64_t *fk[2];             /* [K][N]; both NULL on the fused X^1024+1 path: the decomposed planes then
                                * live only in the context's MFMA operand rows, which the fold reads
                                * (they are transient in the reference too: compute_f_0, folding.rs:258) */
  uint64_t *wk[2];             /* [K][W] */
  uint64_t *y[2];              /* [K][kappa] decomposition commitments */
  uint64_t *f0, *f0_coeff;     /* N each: folded witness */
  uint64_t *w_ccs0;            /* W */
  uint64_t *cm0;               /* kappa */
  /* b_small = 2 (optional, both sides or neither): the decomposed witnesses as
   * packed digit planes. d = 24: [K][N] u64, one per element and plane (bit i =
   * coefficient i is nonzero, bit 32 + i = it is -1). d = 1024 (the fused path):
   * N x 2 KiB, every coefficient's 16-bit sign|magnitude word, all K planes in
   * one (the decomposition's own packed input). With fk and fk_coeff all NULL
   * the planes are the decomposed witnesses' only form: the u64 rows (2 x 8 d B
   * per element and plane) are not written; lf_dev_expand_planes makes them.
   * d = 4096 (the fused path): N x K KiB, one byte per coefficient quad and plane
   * (bit b = the digit of coefficient a + 1024 b is nonzero, bit 4 + b = that
   * coefficient is negative; byte ((e K + k) 32 + r) 32 + j holds a = r + 32 j), and
   * f_0 is folded from the operand rows. */
  uint64_t *planes[2];
} lf_fold_step_bufs;
/* packed digit planes (lf_fold_step_bufs.planes) of N elements -> the Witness forms of
 * decompose_witness's outputs (decomposition.rs:162-167, arith.rs:324-338):
 * f_coeff_k [K][N] (digits mod p) and / or f_k [K][N] = CRT(f_coeff_k); either may be NULL */
int lf_dev_expand_planes(lf_ctx *ctx, const lf_params *pr, const uint64_t *planes, size_t N, uint64_t *f_coeff_k,
                         uint64_t *f_k);
/* commit(z) followed by the commit+fold arithmetic of fold(), all on device */
int lf_dev_fold_step(lf_ctx *ctx, const lf_ajtai *aj, const lf_params *pr, size_t W,
                     const lf_fold_step_bufs *b);
/* nsteps (<= 8) independent commit+fold steps against one Ajtai scheme (trace-batch
 * shard: independent witness / accumulator pairs, SURVEY.md 8(e) configs[3]), each
 * with its own context (stream) and buffers. Every step runs lf_dev_fold_step's
 * arithmetic on its own stream, except that their commitment contractions run
 * as ONE launch on ctx[0]'s stream, so A (kappa x width ring elements, 21.5 GB at
 * d = 1024, W = 2^14) is read from HBM once for all of them. Results are bit-exact
 * with nsteps calls of lf_dev_fold_step; the streams are ordered with events (no
 * host synchronisation). The contexts must be distinct and on aj's device. */
int lf_dev_fold_step_batch(lf_ctx *const *ctx, int nsteps, const lf_ajtai *aj, const lf_params *pr, size_t W,
                           const lf_fold_step_bufs *const *b);

/* A column-sharded step: rank r holds the columns of groups
 * [g_r, g_r + W_r) of the witness -- its w_ccs / acc_f_coeff shards, an Ajtai
 * scheme over A's matching columns, and shard-sized witness outputs -- plus the
 * full acc_cm and rho. The commitments are sums over columns, so each rank's
 * A_r f_r is a partial sum; after they are summed over ranks (mod p) every
 * rank finishes the step with the full y / cm / cm_0 and its own shard of
 * f_0, f_0 coefficients and w_ccs_0, bit-exact with the unsharded step.
 *   lf_dev_fold_step_partial: commit(z) + decompositions + the 1 + 2(K-1)
 *     partial commitments into partial[lf_fold_step_partial_len] (u64; order:
 *     commit(z)'s cm, then y_s[k], s = 0, 1, k = 1 .. K-1)
 *   lf_dev_fold_step_finish: given their sum over ranks, the rest of the step
 *   lf_dev_fold_step_sharded: partial, RCCL all-reduce mod p over `comm`, finish
 * Without an RCCL communicator (comm == NULL) the sharded step is lf_dev_fold_step. */
size_t lf_fold_step_partial_len(const lf_ajtai *aj, const lf_params *pr);
int lf_dev_fold_step_partial(lf_ctx *ctx, const lf_ajtai *aj, const lf_params *pr, size_t W,
                             const lf_fold_step_bufs *b, uint64_t *partial);
int lf_dev_fold_step_finish(lf_ctx *ctx, const lf_ajtai *aj, const lf_params *pr, size_t W,
                            const lf_fold_step_bufs *b, const uint64_t *partial_sum);
int lf_dev_fold_step_sharded(lf_ctx *ctx, const lf_ajtai *aj, const lf_params *pr, size_t W,
                             const lf_fold_step_bufs *b, lf_comm *comm);

/* ------------------------------------------------------------ communicators (RCCL over xGMI)
 * RCCL is resolved at run time (the copy already loaded in the process, else
 * librccl.so.1). A host creates one communicator per rank, either from a
 * unique id that rank 0 makes and the host distributes (128 bytes), or by
 * wrapping a caller-created ncclComm_t (not destroyed by lf_comm_destroy).
 * lf_comm_init with id == NULL and nranks == 1 makes a communicator without
 * RCCL (every exchange is then the identity). */
int lf_comm_unique_id(uint8_t *id, size_t len);
int lf_comm_init(lf_ctx *ctx, int nranks, int rank, const uint8_t *id, size_t len, lf_comm **out);
int lf_comm_wrap(lf_ctx *ctx, void *nccl_comm, lf_comm **out);
void lf_comm_destroy(lf_comm *comm);
int lf_comm_size(const lf_comm *comm);
int lf_comm_rank(const lf_comm *comm);
/* x <- sum over ranks of x (mod p), in place, on the context stream (32-bit
 * limbs over RCCL's u64 sum, joined mod p) */
int lf_comm_allreduce_modp(lf_ctx *ctx, lf_comm *comm, uint64_t *x, size_t n);
/* the accumulator exchange of independent per-rank step streams: cm_0 and f_0
 * summed over ranks mod p, in place (SURVEY.md 8(b) lf_fold_reduce_allranks) */
int lf_fold_reduce_allranks(lf_ctx *ctx, lf_comm *comm, uint64_t *cm0, size_t cm0_len, uint64_t *f0,
                            size_t f0_len);

int lf_dev_fold_lcccs(lf_ctx *ctx, int d, int nwit, const uint64_t *rho, const uint64_t *rho_coeff,
                      const uint64_t *eta, size_t t, const uint64_t *xwh, size_t l1, const uint64_t *theta,
                      uint64_t *u0, uint64_t *x0, uint64_t *v0);
int lf_dev_compute_x_s(lf_ctx *ctx, const lf_params *pr, const uint64_t *x, size_t m, uint64_t *x_s);

int lf_dev_poseidon2_permute(lf_ctx *ctx, uint64_t *states, size_t n);
/* the permutation stopped after its initial MDS and `rounds` (<= 30) rounds: the
 * 4 + 22 + 4 of poseidon2.rs:100-173 in order (debug entry: the reference's only
 * round vector, sages/inverse_mds.sage, pins the initial MDS and round 0) */
int lf_dev_poseidon2_permute_rounds(lf_ctx *ctx, uint64_t *states, size_t n, int rounds);
/* synthetic inputs: element i = SplitMix64(seed, i) re-mixed until < p */
int lf_dev_fill_uniform(lf_ctx *ctx, uint64_t *out, size_t n, uint64_t seed);
/* out[c] = sum_r in[r][c] mod p  (reduce of all-gathered accumulators) */
int lf_dev_modp_sum(lf_ctx *ctx, const uint64_t *in, int nparts, size_t len, uint64_t *out);

/* RCCL transport of field vectors: RCCL sums u64 modulo 2^64, so vectors are
 * all-reduced as 32-bit limbs (lo, hi as u64; <= 2^8 ranks) and joined mod p */
int lf_dev_limb_split(lf_ctx *ctx, const uint64_t *x, size_t n, uint64_t *lo, uint64_t *hi);
int lf_dev_limb_join(lf_ctx *ctx, const uint64_t *lo, const uint64_t *hi, size_t n, uint64_t *out);

/* ------------------------------------------------------------ multilinear sumcheck
 * latticefold/src/utils/sumcheck.rs:61-88 (prove_as_subprotocol),
 * utils/sumcheck/prover.rs:62-168 (prove_round), utils/sumcheck/utils.rs:140-210
 * (build_eq_x_r), poly/src/mle/dense.rs:107-199 (evaluate, fix_variables),
 * nifs/folding/utils.rs:196-331 and nifs/linearization/utils.rs:63-104 (the
 * two polynomials). MLEs are device buffers of 2^nv NTT ring elements each
 * (zero-padded), nm of them contiguous [nm][2^nv][d] unless a stride is given.
 * Challenges are base-ring elements (Fq3 for d = 24, Fq otherwise: 3 or 1
 * words) broadcast into every NTT slot. */
enum { LF_COMB_FOLDING = 0, LF_COMB_LINEARIZATION = 1 };
typedef struct {
  int kind;
  /* folding: MLEs [eq_r0, g0, eq_r1, g1, eq_beta, f_hat (nk instances x tau)];
   * mu: nk NTT elements on the device */
  int nk, tau, bsmall;
  const uint64_t *mu;
  /* linearization: MLEs [M_mles[j] for each i with c_i != 0, j in S_i] + [eq_beta];
   * c: q NTT elements on the device; S_off [q + 1], S_idx: host arrays. The
   * combination reads MLE position j for matrix index j, as the reference does. */
  int q;
  const uint64_t *c;
  const int *S_off;
  const int *S_idx;
} lf_comb;
int lf_dev_eq_table(lf_ctx *ctx, int d, const uint64_t *r, int nv, uint64_t *out);
/* Witness::get_fhat (latticefold/src/arith.rs:273-297): the f_hat MLEs of a
 * witness from its f_coeff [N][d] (N <= 2^nv): out [tau][2^nv][d], tau = 3 for
 * Phi_72 (slot s of MLE j is (f_coeff[i][8 j + s], 0, 0)), 1 for X^d + 1; the
 * points past N are zero (the reference truncates them; the MLE reads zero). */
int lf_dev_get_fhat(lf_ctx *ctx, int d, const uint64_t *f_coeff, size_t N, int nv, uint64_t *out);
/* out[m][b] = in[m][2b] + r (in[m][2b + 1] - in[m][2b]) for b < 2^(nv-1); r: base-ring words (host) */
int lf_dev_mle_fix_first(lf_ctx *ctx, int d, const uint64_t *in, size_t in_stride, int nm, int nv,
                         const uint64_t *r_base, uint64_t *out, size_t out_stride);
/* out[m] = mle_m(point) (nm NTT elements); point: nv NTT elements on the device */
int lf_dev_mle_evaluate(lf_ctx *ctx, int d, const uint64_t *mles, int nm, int nv, const uint64_t *point,
                        uint64_t *out);
/* the same from the point's eq table (2^nv NTT elements, lf_dev_eq_table) */
int lf_dev_mle_evaluate_eq(lf_ctx *ctx, int d, const uint64_t *mles, int nm, int nv, const uint64_t *eq,
                           uint64_t *out);
/* one prover round's message: evals[e] = sum_b comb(mle(2b) + e (mle(2b+1) - mle(2b))),
 * e <= degree (folding: degree = 2 bsmall) */
int lf_dev_sumcheck_round(lf_ctx *ctx, const lf_comb *comb, const uint64_t *mles, size_t stride, int nm, int nv,
                          int d, int degree, uint64_t *evals);
/* the whole prover with the Poseidon2 transcript: proof [nv][degree + 1][d]
 * and randomness [nv][1 or 3] in host memory; the MLEs are clobbered */
int lf_sumcheck_prove(lf_ctx *ctx, lf_transcript *t, const lf_comb *comb, uint64_t *mles, int nm, int nv, int d,
                      int degree, uint64_t *proof, uint64_t *randomness);
/* the same prover over MLEs that stay where they are: mles is a host array of nm
 * device pointers (one per MLE of 2^nv elements, repeats allowed), read in the first
 * round only and never written; work: a device buffer of nm x 2^(nv-2) elements for
 * the later rounds (the linearization sumcheck reads its Mz MLEs in place) */
int lf_sumcheck_prove_ptrs(lf_ctx *ctx, lf_transcript *t, const lf_comb *comb, const uint64_t *const *mles, int nm,
                           int nv, int d, int degree, uint64_t *work, uint64_t *proof, uint64_t *randomness);
/* the folding sumcheck (folding.rs:42-130 over folding/utils.rs:196-331, B_SMALL = 2) with
 * its 2K tau f_hat MLEs given as the decomposed witnesses' digit coefficient rows (fc0: the
 * K witnesses of side 0, fc1 of side 1, wstride u64 apart, N elements each; every value
 * 0, 1 or -1, as the decomposition guarantees) instead of materialised MLEs: mles5 holds
 * the 5 general MLEs [eq(r_0), g1, eq(r_1), g3, eq(beta)] (2^nv elements each); round 0
 * runs on the digits, the later rounds on the fixed MLEs in work (5 + 2K tau MLEs of
 * 2^(nv-2) elements) and the context scratch. The proof and randomness of lf_sumcheck_prove
 * over the materialised list. */
int lf_sumcheck_prove_fold_digits(lf_ctx *ctx, lf_transcript *t, const lf_comb *comb, const uint64_t *mles5,
                                  const uint64_t *fc0, const uint64_t *fc1, int K, size_t N, size_t wstride, int nv,
                                  int d, uint64_t *work, uint64_t *proof, uint64_t *randomness);
/* the linearization sumcheck (LFLinearizationProver::prove's, linearization.rs:153-197
 * over linearization/utils.rs:63-104) with eq(beta) given by beta itself: the proof and
 * randomness of lf_sumcheck_prove over [mles..., eq(beta)] (same transcript), with
 * eq(beta) split off each round (eq(beta_i, X) and eq over the unbound variables), so
 * the device evaluates a polynomial of one degree less. mles: nm device pointers as in
 * lf_sumcheck_prove_ptrs (S_idx < nm); beta: host [nv][d] broadcast base-ring values;
 * every multiset has fewer than `degree` entries; work: nm x 2^(nv-2) elements; evals
 * (device, nm ring elements, may be NULL): the MLEs at the challenge point (their
 * values after the last round's fix: MLE(M_j z)(r) for the linearization's u) */
int lf_sumcheck_prove_lin(lf_ctx *ctx, lf_transcript *t, const lf_comb *comb, const uint64_t *const *mles, int nm,
                          int nv, int d, int degree, const uint64_t *beta, uint64_t *work, uint64_t *proof,
                          uint64_t *randomness, uint64_t *evals);
/* lf_sumcheck_prove_lin whose first round visits, for multiset i, only the points
 * act[act_off[i] .. act_off[i + 1]) (act: device uint32 point indices b < 2^(nv-1);
 * act_off: host, q + 1 entries, act_off[0] = 0). The caller guarantees that at every
 * other point b some factor of S_i is zero on both rows 2b and 2b + 1, so the term is
 * zero at every evaluation point -- the zero short-cut of the reference's product
 * (linearization/utils.rs:86-104), decided once from the CCS rows (lf_ccs_row_live)
 * instead of per value. Same proof, randomness and evals as lf_sumcheck_prove_lin. */
int lf_sumcheck_prove_lin_sparse(lf_ctx *ctx, lf_transcript *t, const lf_comb *comb, const uint64_t *const *mles,
                                 int nm, int nv, int d, int degree, const uint64_t *beta, const uint32_t *act,
                                 const uint32_t *act_off, uint64_t *work, uint64_t *proof, uint64_t *randomness,
                                 uint64_t *evals);

/* ------------------------------------------------------------ sparse Mz products
 * CCS.M (latticefold/src/arith.rs:51-74): t matrices m x n of ring elements,
 * given as one CSR: row_ptr [t][m + 1] absolute offsets into col / val
 * (matrix j's entries follow matrix j-1's), col, val [nnz][d] (NTT form).
 *   lf_dev_mz_mles: calculate_Mz_mles / compute_mz_mles (mle_helpers.rs:137-146,
 *     nifs/decomposition.rs:229-256): out [nz][t][2^nv] = MLE(M_j z_i), mat_vec_mul
 *     (arith/utils.rs:52-65) zero-padded to 2^nv (to_mles_err)
 *   lf_dev_mz_challenged: calculate_challenged_mz_mle (nifs/folding.rs:208-234):
 *     out [2^nv] = sum_i sum_j zeta_i^(j+1) MLE(M_j z_i); zeta: nz NTT elements
 *   lf_dev_mz_evaluate: evaluate_mles of every MLE(M_j z_i) at point (compute_u_s,
 *     get_etas, compute_u): out [nz][t]; point: nv NTT elements
 * z: nz vectors [nz][n] (decomposed statement || w_ccs); all device buffers. */
int lf_ccs_create(lf_ctx *ctx, int d, int t, size_t m, size_t n, const uint64_t *row_ptr, const uint32_t *col,
                  const uint64_t *val, int repr, lf_ccs **out);
void lf_ccs_destroy(lf_ccs *M);
int lf_dev_mz_mles(lf_ctx *ctx, const lf_ccs *M, const uint64_t *z, int nz, int nv, uint64_t *out);
/* the MLEs of the selected matrices only, out[i] = MLE(M_sel[i] z) (sel: host, nsel
 * indices < t; one z) */
int lf_dev_mz_mles_sel(lf_ctx *ctx, const lf_ccs *M, const uint64_t *z, const int *sel, int nsel, int nv,
                       uint64_t *out);
int lf_dev_mz_challenged(lf_ctx *ctx, const lf_ccs *M, const uint64_t *z, const uint64_t *zeta, int nz, int nv,
                         uint64_t *out);
/* two lf_dev_mz_challenged at once (the folding prover's g1 and g3 parts, one per
 * decomposed side), reading the matrices' entries once for both */
int lf_dev_mz_challenged_pair(lf_ctx *ctx, const lf_ccs *M, const uint64_t *z0, const uint64_t *zeta0,
                              const uint64_t *z1, const uint64_t *zeta1, int nz, int nv, uint64_t *out0,
                              uint64_t *out1);
int lf_dev_mz_evaluate(lf_ctx *ctx, const lf_ccs *M, const uint64_t *z, int nz, int nv, const uint64_t *point,
                       uint64_t *out);
/* lf_dev_mz_evaluate in two halves, so one point's weights serve several z sets:
 * w [t][n] = M_j^T eq (eq: an eq table of 2^nv NTT elements, lf_dev_eq_table), then
 * out [nz][t] = w_j . z_i. lf_ccs_weights_len: the u64 of w. */
size_t lf_ccs_weights_len(const lf_ccs *M);
int lf_dev_mz_weights(lf_ctx *ctx, const lf_ccs *M, int nv, const uint64_t *eq, uint64_t *w);
int lf_dev_mz_dots(lf_ctx *ctx, const lf_ccs *M, const uint64_t *w, const uint64_t *z, int nz, uint64_t *out);

/* ------------------------------------------------------------ width-8 Poseidon2 commitments
 * zkvm/src/commitments.rs:192-340, over Poseidon2Goldilocks<8> (poseidon2.rs:31-49;
 * external constants crypto_consts.rs:9-96; internal diagonal = Plonky3
 * MATRIX_DIAG_8_GOLDILOCKS, not in the reference: parity unpinned). A row hash is
 * PaddingFreeSponge<8, rate 4, out 4>, a parent TruncatedPermutation<2, 4, 8> of its
 * children; trees follow Plonky3 MerkleTree::new over one matrix (git 33e58c7787f9,
 * not vendored): every layer below the root is padded to an even length with the
 * zero digest, so any height works.
 *   lf_dev_merkle_tree: vm_mem_comm_with_opening (:222-268; PAGE_COUNT rows of
 *     WORDS_PER_PAGE words) and vm_code_comm (:314-340; a width-1 matrix of the
 *     code's half-words, any height). nodes: lf_merkle_nodes_len(nrows) x 4 words on
 *     the device (2 nrows - 1 for a power of two), padded layers leaves first, root last
 *   lf_merkle_open: the sibling digest in every layer below the root (4 words each,
 *     host), leaves first: open_batch's opening_proof (log2(nrows) for a power of two)
 *   lf_vm_code_comm: vm_code_comm of `len` code bytes (host buffer) -> root
 *   lf_dev_hash_w8_rows: independent sponge hashes of nrows rows (the leaf layer)
 *   lf_hash_w8 / lf_vm_mem_comm (host, sequential): vm_mem_comm (:192-217) gives
 *     MerkleTree::new PAGE_COUNT one-row matrices, all of height 1, so its root is ONE
 *     sponge over all pages' words in page order -- a strictly sequential chain of
 *     nwords / 4 permutations that runs on the host (the device would run it on one
 *     8-lane group) */
int lf_dev_poseidon2_w8_permute(lf_ctx *ctx, uint64_t *states, size_t n);
size_t lf_merkle_nodes_len(size_t nrows);
int lf_dev_merkle_tree(lf_ctx *ctx, const uint64_t *rows, size_t nrows, size_t width, uint64_t *nodes);
int lf_merkle_open(lf_ctx *ctx, const uint64_t *nodes, size_t nrows, size_t index, uint64_t *path);
int lf_vm_code_comm(lf_ctx *ctx, const uint8_t *code, size_t len, uint64_t out4[4]);
int lf_dev_hash_w8_rows(lf_ctx *ctx, const uint64_t *rows, size_t nrows, size_t width, uint64_t *out);
void lf_hash_w8(const uint64_t *in, size_t n, uint64_t out4[4]);
int lf_vm_mem_comm(const uint32_t *words, size_t nwords, uint64_t out4[4]);

/* ------------------------------------------------------------ wire format
 * LFProof: ark-serialize 0.5 CanonicalSerialize as derived on the reference's
 * types (nifs.rs:28-34; compressed = uncompressed here): Fq = 8 bytes LE
 * canonical; an NTT ring element = its d slot words, no length; Vec<T> = u64 LE
 * length + items; structs = fields in declaration order. LCCCS: the reference
 * derives no CanonicalSerialize for it (arith.rs:193-194), so its layout is this
 * project's own, written by the same rules. repr describes the caller's words.
 * out == NULL (or too small: LF_ERR_INCORRECT_LENGTH) still returns the size. */
typedef struct {
  const uint64_t *elems; /* n ring elements (d words each) */
  size_t n;
} lf_ring_slice;
/* LCCCS { r, v, cm, u, x_w, h } (latticefold/src/arith.rs:192-206) */
typedef struct {
  int d;
  lf_ring_slice r, v, cm, u, x_w;
  const uint64_t *h; /* one ring element */
} lf_lcccs;
/* LFProof (latticefold/src/nifs.rs:28-34) */
typedef struct {
  const lf_ring_slice *u_s, *v_s, *x_s, *y_s; /* Vec<Vec<R>> and Vec<Commitment> */
  size_t n_u, n_v, n_x, n_y;
} lf_decomposition_proof;
typedef struct {
  int d;
  const uint64_t *lin_sumcheck; /* [lin_rounds][lin_evals] ring elements */
  size_t lin_rounds, lin_evals;
  lf_ring_slice lin_v, lin_u;
  lf_decomposition_proof dec[2]; /* decomposition_proof_l, decomposition_proof_r */
  const uint64_t *fold_sumcheck; /* [fold_rounds][fold_evals] */
  size_t fold_rounds, fold_evals;
  const lf_ring_slice *theta_s, *eta_s;
  size_t n_theta, n_eta;
} lf_lfproof;
int lf_lcccs_serialize(const lf_lcccs *acc, int repr, uint8_t *out, size_t cap, size_t *len);
/* parses into `buf` (buf_elems u64); `out` points into it */
int lf_lcccs_deserialize(const uint8_t *in, size_t len, int d, int repr, uint64_t *buf, size_t buf_elems,
                         lf_lcccs *out);
int lf_lfproof_serialize(const lf_lfproof *proof, int repr, uint8_t *out, size_t cap, size_t *len);

/* ------------------------------------------------------------ fold() end to end
 * zk_latticefold_prove (zkvm/src/zk_latticefold.rs:37-102), what fold()
 * (zkvm/src/main.rs:369-404) runs with a fresh Poseidon2 transcript:
 * absorb_public_input (:162-184), the linearization prover
 * (latticefold/src/nifs/linearization.rs:153-197), the decomposition provers of
 * (acc, w_acc) and of the linearized (cm_i, w_i) (nifs/decomposition.rs:33-88)
 * and the folding prover (nifs/folding.rs:42-130), in the reference's transcript
 * order. The witnesses stay in HBM; the LCCCS and the proof are host memory.
 *   lf_ccs_set_structure: the CCS's l (= |x_ccs|), degree (ccs.d), c (q NTT
 *     elements) and multisets S (S_off [q + 1], S_idx) -- CCS (arith.rs:51-74)
 *   lf_prover_create: device scratch for one (scheme, params, CCS) shape;
 *     the CCS must pass sanity_check (m = max((n - l - 1) L, m) rounded up to a
 *     power of two) with N = (n - l - 1) L rounding up to m as well; a multiset
 *     index equal to the number of Mz MLEs (the reference's eq(beta) position) is
 *     rejected with LF_ERR_UNSUPPORTED_CCS, a negative index or one past that
 *     position (malformed: the reference panics on it) with LF_ERR_INVALID_ARG;
 *     lf_ctx_last_error names the reason
 *   lf_fold_prove: -> the folded LCCCS, its witness (caller-allocated device
 *     buffers: f, f_coeff N elements, w_ccs W) and the LFProof (nifs.rs:28-34).
 *     repr describes every host buffer (acc, cm_i, x_ccs, out, proof).
 * Sizes: s = log2 m, tau = 3 (d = 24) or 1, t matrices, K = params K. */
typedef struct lf_prover lf_prover;
typedef struct {
  uint64_t *w_ccs;   /* W NTT elements */
  uint64_t *f;       /* N = W L NTT elements */
  uint64_t *f_coeff; /* N coefficient-form elements */
} lf_witness;
typedef struct {
  uint64_t *r;   /* s */
  uint64_t *v;   /* tau */
  uint64_t *cm;  /* kappa */
  uint64_t *u;   /* t */
  uint64_t *x_w; /* l */
  uint64_t *h;   /* 1 */
} lf_lcccs_mut;
typedef struct {
  uint64_t *lin_sumcheck;             /* [s][degree + 2] (linearization_sumcheck) */
  uint64_t *lin_v, *lin_u;            /* tau, t */
  uint64_t *u_s[2], *v_s[2];          /* [K][t], [K][tau]: decomposition_proof_l / _r */
  uint64_t *x_s[2], *y_s[2];          /* [K][l + 1], [K][kappa] */
  uint64_t *fold_sumcheck;            /* [s][2 b_small + 1] (pointshift_sumcheck_proof) */
  uint64_t *theta_s, *eta_s;          /* [2K][tau], [2K][t] */
} lf_lfproof_mut;
int lf_ccs_set_structure(lf_ctx *ctx, lf_ccs *M, size_t l, int degree, int q, const uint64_t *c, const int *S_off,
                         const int *S_idx, int repr);
int lf_ccs_shape(const lf_ccs *M, int *t, size_t *m, size_t *n, size_t *l, int *q, int *degree);
int lf_ccs_get_structure(const lf_ccs *M, uint64_t *c, int *S_off, int *S_idx);
const uint64_t *lf_ccs_c_device(const lf_ccs *M);
/* 1 if every entry of the matrices is a scalar (from_scalar: its value in word 0 of
 * every slot, zero elsewhere -- the zkvm's R1CS-derived matrices), which the Mz
 * products then read as one word per entry; else 0 */
int lf_ccs_is_scalar(const lf_ccs *M);
/* out[r] = 1 if row r of M_j holds an entry (so MLE(M_j z) may be nonzero there), else 0; m bytes */
int lf_ccs_row_live(const lf_ccs *M, int j, uint8_t *out);
/* tracing spans of lf_fold_prove (the reference's #[instrument] spans): wall ms per
 * phase, summed over calls since timing was (re)set; each phase ends with a
 * stream sync while timing is on */
enum {
  LF_SPAN_PUBLIC_INPUT = 0,           /* absorb_public_input */
  LF_SPAN_LINEARIZATION = 1,          /* beta, Mz, the degree-(d+1) sumcheck, v, u */
  LF_SPAN_DECOMPOSITION = 2,          /* x_s, decompose + commit_witnesses, v_s, u_s */
  LF_SPAN_DECOMPOSITION_TRANSCRIPT = 3, /* the 2K decomposed instances absorbed */
  LF_SPAN_FOLDING_MLES = 4,           /* alpha..beta, f_hat MLEs, challenged Mz, g, eq tables */
  LF_SPAN_FOLDING_SUMCHECK = 5,       /* the degree-2 b_small sumcheck */
  LF_SPAN_EVALUATIONS = 6,            /* theta_s, eta_s */
  LF_SPAN_FOLDING_TRANSCRIPT = 7,     /* theta_s, eta_s absorbed, get_rhos */
  LF_SPAN_FOLD = 8,                   /* CRT(rho), cm_0, f_0, from_f, v_0, u_0, x_0 */
  LF_SPAN_VARS = 9,                   /* lf_fold_prove_vars: the verification vars from the sample log */
  LF_SPAN_COUNT = 10
};
/* span_ms (LF_SPAN_COUNT, may be NULL) receives the sums so far; then timing is set to
 * `enable` and the sums are cleared */
int lf_prover_timing(lf_prover *prover, int enable, double *span_ms);
int lf_prover_create(lf_ctx *ctx, const lf_ajtai *aj, const lf_params *pr, const lf_ccs *ccs, lf_prover **out);
void lf_prover_destroy(lf_prover *prover);
const char *lf_prover_last_error(const lf_prover *prover);
/* LFLinearizationProver::prove of a CCCS (cm, x_ccs) with witness w on a fresh
 * transcript -- initialize_accumulator's accumulator (zkvm/src/main.rs:305-344):
 * the LCCCS {r, v, cm, u, x_ccs, ONE} and the linearization sumcheck [s][degree + 2] */
int lf_linearize(lf_prover *prover, const uint64_t *cm, const uint64_t *x_ccs, const lf_witness *w, lf_lcccs_mut *out,
                 uint64_t *lin_sumcheck, int repr);
int lf_fold_prove(lf_prover *prover, const lf_lcccs *acc, const lf_witness *w_acc, const uint64_t *cm_i,
                  const uint64_t *x_ccs, const lf_witness *w_i, lf_lcccs_mut *out, const lf_witness *w_out,
                  lf_lfproof_mut *proof, int repr);
/* the halves of the device fold step that fold() interleaves with its sumchecks:
 *   lf_dev_decompose_commit: decompose_witness + commit_witnesses of both sides
 *     (y_0 included), inputs acc_f_coeff, acc_cm, f_coeff and cm (the linearized instance)
 *   lf_dev_fold_combine: given rho, cm_0 / f_0 / Witness::from_f(f_0) (same context and buffers) */
int lf_dev_decompose_commit(lf_ctx *ctx, const lf_ajtai *aj, const lf_params *pr, size_t W,
                            const lf_fold_step_bufs *b);
int lf_dev_fold_combine(lf_ctx *ctx, const lf_ajtai *aj, const lf_params *pr, size_t W, const lf_fold_step_bufs *b);
/* evaluate_mles of the f_hat MLEs of nw witnesses straight from their f_coeff rows
 * (wstride u64 apart, 0 = N d): out [nw][tau] NTT elements; point: nv NTT elements */
int lf_dev_fhat_evaluate(lf_ctx *ctx, int d, const uint64_t *f_coeff, size_t N, size_t wstride, int nw, int nv,
                         const uint64_t *point, uint64_t *out);
/* the same with the point's eq table given (2^nv NTT elements, lf_dev_eq_table) */
int lf_dev_fhat_evaluate_eq(lf_ctx *ctx, int d, const uint64_t *f_coeff, size_t N, size_t wstride, int nw, int nv,
                            const uint64_t *eq, uint64_t *out);
/* io[x] += sum_m coef[m] (.) mles[m][x] over 2^nv points (stride 0 = 2^nv d) */
int lf_dev_mle_lincomb(lf_ctx *ctx, int d, const uint64_t *mles, size_t stride, int nm, int nv, const uint64_t *coef,
                       uint64_t *io);
int lf_ctx_device(const lf_ctx *ctx);

/* generate_verification_witness_vars (zkvm/src/zk_latticefold.rs:111-148): the
 * host replay of a fold() proof's transcript and the values the in-CCS folding
 * verifier consumes (collect_linearization_vars :204-345, collect_decomposition_vars
 * :393-432, collect_folding_vars :465-659). Phi_72 only (tau = 3). Every buffer is
 * caller-allocated host memory of NTT elements; sizes with s = log2 m, q multisets,
 * D1 = ccs degree + 2 (linearization evals), D2 = 2 b_small + 1 (folding evals). */
typedef struct {
  uint64_t *lin_beta;          /* s */
  uint64_t *lin_claimed_sums;  /* s + 1 (claim 0 first) */
  uint64_t *lin_subterms;      /* [s][D1] p_i L_i(r), i from D1 - 1 down */
  uint64_t *lin_point;         /* s (r) */
  uint64_t *lin_expected;      /* 1 */
  uint64_t *lin_inner;         /* 1: sum_i c_i prod_{j in S_i} u_j */
  uint64_t *lin_products;      /* q */
  uint64_t *lin_eq_xy, *lin_eq_factors; /* s, s (zk_eq_eval of (r, beta)) */
  uint64_t *lin_eq_sub;        /* s + 1 */
  uint64_t *alpha, *beta, *zeta, *mu; /* 2K, s, 2K, 2K */
  uint64_t *claim_g1_h1, *claim_g1_h2, *claim_g1_terms; /* 2K each */
  uint64_t *claim_g1;          /* 1 */
  uint64_t *claim_g3_h;        /* [2K][t - 1] Horner partials */
  uint64_t *claim_g3_terms;    /* 2K */
  uint64_t *claim_g3;          /* 1 */
  uint64_t *fold_claimed_sums; /* s + 1 */
  uint64_t *fold_subterms;     /* [s][D2] */
  uint64_t *fold_point;        /* s (r_0) */
  uint64_t *fold_expected;     /* 1 */
  uint64_t *should_equal_s;    /* 1 */
  uint64_t *rho;               /* 2K (NTT form) */
  uint64_t *final_cm, *final_u, *final_x; /* [2K][kappa], [2K][t], [2K][l + 1]: rho_i-weighted */
} lf_replay_vars;
/* the CCS shape the replay reads (host memory; no device handle, so the verifier
 * side runs without a GPU): t matrices of m rows, l public inputs, degree, the q
 * coefficients c (NTT elements) and multisets S (S_off [q + 1], S_idx) */
typedef struct {
  int t;
  size_t m, l;
  int degree, q;
  const uint64_t *c;
  const int *S_off, *S_idx;
} lf_ccs_desc;
/* the proof as lf_fold_prove wrote it (read only); repr describes every buffer, c included */
int lf_fold_replay(const lf_ccs_desc *ccs, const lf_params *pr, const lf_lcccs *acc, const uint64_t *cm_i,
                   const uint64_t *x_ccs, const lf_lfproof_mut *proof, lf_replay_vars *out, int repr);
/* the same replay with its challenges taken from the prover's sample log
 * (lf_prover_samples) instead of a second Poseidon2 pass: LF_ERR_INCORRECT_LENGTH
 * unless the replay draws exactly the logged samples.
 * PROVER-SIDE ONLY: the playback transcript drops every observe, so the vars are NOT
 * bound to the proof's messages -- any log of the right length is accepted. Feed it
 * only the log of the same prover's own lf_fold_prove call (what lf_fold_prove_vars
 * does); a received proof must go through lf_fold_replay or lf_fold_verify. */
int lf_fold_replay_samples(const lf_ccs_desc *ccs, const lf_params *pr, const lf_lcccs *acc, const uint64_t *cm_i,
                           const uint64_t *x_ccs, const lf_lfproof_mut *proof, const uint64_t *samples, size_t nsamples,
                           lf_replay_vars *out, int repr);
/* NIFSVerifier::verify (latticefold/src/nifs.rs:117-162) over the zkvm's public-input
 * absorption, as main.rs:408-426 (verify_folding, the `debug` feature) runs it after every
 * fold(): on the host, no device needed. LF_OK with the folded LCCCS in `out` (r s, v tau,
 * cm kappa, u t, x_w l, h 1), or LF_ERR_VERIFICATION with the failed check in *failed. */
enum lf_verify_check {
  LF_VERIFY_OK = 0,
  LF_VERIFY_LIN_SUMCHECK = 1,  /* a linearization sumcheck round: p(0) + p(1) != claim */
  LF_VERIFY_LIN_CLAIM = 2,     /* e(r, beta) sum c_i prod u_j != the sumcheck's final claim */
  LF_VERIFY_DEC_Y = 3,         /* sum_k b^k y_k != cm (either decomposition) */
  LF_VERIFY_DEC_V = 4,
  LF_VERIFY_DEC_U = 5,
  LF_VERIFY_DEC_X = 6,
  LF_VERIFY_FOLD_SUMCHECK = 7, /* a folding sumcheck round */
  LF_VERIFY_FOLD_CLAIM = 8     /* compute_sumcheck_claim_expected_value != the final claim */
};
int lf_fold_verify(const lf_ccs_desc *ccs, const lf_params *pr, const lf_lcccs *acc, const uint64_t *cm_i,
                   const uint64_t *x_ccs, const lf_lfproof_mut *proof, lf_lcccs_mut *out, int *failed, int repr);
/* every value the last lf_fold_prove sampled from its transcript (count returned, up to cap copied) */
size_t lf_prover_samples(const lf_prover *prover, uint64_t *out, size_t cap);
/* fold() then generate_verification_witness_vars (main.rs:175-185) in one call: lf_fold_prove,
 * then the vars from its own sample log (bit-exact with lf_fold_replay; Phi_72 only) */
int lf_fold_prove_vars(lf_prover *prover, const lf_lcccs *acc, const lf_witness *w_acc, const uint64_t *cm_i,
                       const uint64_t *x_ccs, const lf_witness *w_i, lf_lcccs_mut *out, const lf_witness *w_out,
                       lf_lfproof_mut *proof, lf_replay_vars *vars, int repr);

/* ------------------------------------------------------------ host transcript (sequential) */
lf_transcript *lf_transcript_new(void);
void lf_transcript_free(lf_transcript *t);
void lf_transcript_observe(lf_transcript *t, uint64_t v);
uint64_t lf_transcript_sample(lf_transcript *t);
/* Transcript::absorb of NTT ring elements: their base-field limbs observed as
 * ark Montgomery u64s (fiat_shamir.rs:51-60). repr describes `elems`. */
void lf_transcript_absorb_ring(lf_transcript *t, const uint64_t *elems, size_t n, int d, int repr);
void lf_transcript_get_challenge(lf_transcript *t, uint64_t out3[3]);
void lf_transcript_squeeze_bytes(lf_transcript *t, uint8_t *out, size_t n);
/* get_small_challenges: count short challenges in coefficient form (count x d) */
int lf_transcript_get_short_challenges(lf_transcript *t, int d, size_t count, uint64_t *coeffs);
/* WideZkVMPoseidon2::hash_iter (poseidon2.rs:206-235) */
void lf_hash_iter(const uint64_t *in, size_t n, uint64_t out4[4]);
/* sample log: lf_transcript_record starts (and clears) a log of every sampled value;
 * lf_transcript_samples copies up to cap of them and returns the count. A playback
 * transcript returns the logged samples in order and drops every observe, so a
 * transcript pass that absorbs the same messages in the same order (a verifier's
 * replay of a recorded proof) draws the same challenges without one permutation;
 * lf_transcript_playback_status: LF_OK iff exactly the logged samples were drawn.
 * A playback transcript binds nothing it observes: use it only to replay the
 * caller's own recorded transcript, never to check a proof received from elsewhere. */
void lf_transcript_record(lf_transcript *t);
size_t lf_transcript_samples(const lf_transcript *t, uint64_t *out, size_t cap);
lf_transcript *lf_transcript_new_playback(const uint64_t *samples, size_t n);
int lf_transcript_playback_status(const lf_transcript *t);

/* ------------------------------------------------------------ IVC step commitments (zkvm/src/commitments.rs)
 * hash_iter's second output, IntermediateStates (poseidon2.rs:199-202): one
 * PermutationIntermediateStates (:91-96) per permutation, LF_P2_STATES x 16
 * canonical words: after_initial_mds, after_ext_init_rounds[4],
 * after_internal_rounds[22], after_ext_terminal_rounds[4]. ivc.rs:24,63 carries the
 * ivc_step_comm's states into the next step's witness (ccs.rs:517-580 reads them). */
#define LF_P2_STATES 31
/* permutations hash_iter runs on n inputs: ceil(n / 12) (0 for an empty input) */
size_t lf_hash_iter_nperm(size_t n);
/* (digest, IntermediateStates): states [nperm][31][16] (NULL: digest only), cap >= nperm */
int lf_hash_iter_states(const uint64_t *in, size_t n, uint64_t out4[4], uint64_t *states, size_t cap);
/* ZkVmCommitter::acc_comm (commitments.rs:143-176): the LCCCS's r, v, cm, u, x_w, h
 * flattened (:349-361: every NTT element ICRT'd, each coefficient's ark Montgomery
 * limb taken as a Goldilocks value) and hashed with hash_iter. Phi_72 only (d = 24,
 * the zkvm's ring); repr describes acc's words. zkvm/src/main.rs:106,195 */
int lf_acc_comm(const lf_lcccs *acc, int repr, uint64_t out4[4]);
/* ZkVmCommitter::ivc_step_comm (commitments.rs:76-105): hash_iter of [i, state_0_comm,
 * state_i_comm, acc_comm] -- 13 elements, 2 permutations: states [2][31][16] or NULL.
 * zkvm/src/main.rs:107,196 */
int lf_ivc_step_comm(uint64_t i, const uint64_t state_0_comm[4], const uint64_t state_i_comm[4],
                     const uint64_t acc_comm[4], uint64_t out4[4], uint64_t *states);
/* ZkVmCommitter::state_i_comm (commitments.rs:107-141) given its parts (code_comm =
 * lf_vm_code_comm, regs_comm = lf_vm_regs_comm): hash_iter of the 17 elements */
int lf_state_i_comm(const uint64_t code_comm[4], uint64_t pc, const uint64_t memory_comm[4],
                    const uint64_t regs_comm[4], const uint64_t mem_ops_vec_comm[4], uint64_t out4[4]);
/* ZkVmCommitter::vm_regs_comm (commitments.rs:178-189): hash_iter of the registers */
int lf_vm_regs_comm(const uint32_t *regs, size_t n, uint64_t out4[4]);
/* ZkVmCommitter::vm_mem_ops_vec_comm (commitments.rs:290-307): the width-8
 * TruncatedPermutation of [previous_comm, (cycle, address, value, 0)] */
int lf_vm_mem_ops_vec_comm(const uint64_t prev[4], uint64_t cycle, uint32_t address, uint32_t value,
                           uint64_t out4[4]);

#ifdef __cplusplus
}
#endif
#endif
