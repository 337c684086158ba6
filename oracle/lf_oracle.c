/*
 * lf_oracle.c -- TEST INFRASTRUCTURE ONLY (see lf_oracle.h).
 *
 * CPU restatement of the reference LatticeFold commit+fold arithmetic. Each
 * function cites the reference file:line it follows (paths relative to
 * /root/reference/latticeum/crates/):
 *   GL = stark-rings/crates/ring/src/cyclotomic_ring/models/goldilocks
 *   SR = stark-rings/crates/ring/src
 *   LF = latticefold/src
 *   ZK = zkvm/src
 * Deliberately simple: u128 arithmetic, no vectorisation, pthreads only where
 * the reference uses rayon (so it doubles as the "port" CPU baseline).
 */
#include "lf_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned __int128 u128;
typedef __int128 i128;

#define P 0xFFFFFFFF00000001ull

/* ------------------------------------------------------------------ field */
uint64_t lfo_add(uint64_t a, uint64_t b) {
  u128 s = (u128)a + b;
  if (s >= P) s -= P;
  return (uint64_t)s;
}
uint64_t lfo_sub(uint64_t a, uint64_t b) { return a >= b ? a - b : (uint64_t)((u128)a + P - b); }
uint64_t lfo_mul(uint64_t a, uint64_t b) { return (uint64_t)(((u128)a * b) % P); }
static uint64_t neg(uint64_t a) { return a ? P - a : 0; }
uint64_t lfo_pow(uint64_t a, uint64_t e) {
  uint64_t r = 1;
  while (e) {
    if (e & 1) r = lfo_mul(r, a);
    a = lfo_mul(a, a);
    e >>= 1;
  }
  return r;
}
uint64_t lfo_inv(uint64_t a) { return lfo_pow(a, P - 2); }
/* ark-ff Fp64<MontBackend>: internal limb = a * R mod p, R = 2^64 mod p. */
uint64_t lfo_to_mont(uint64_t a) { return (uint64_t)((((u128)a) << 64) % P); }
uint64_t lfo_from_mont(uint64_t m) { return lfo_mul(m, lfo_inv(0xFFFFFFFFull)); }

/* --------------------------------------------------------- Fq3 (GL/mod.rs:34-54)
 * Fq[u]/(u^3 - NONRESIDUE), NONRESIDUE = 2^40 = 1099511627776. */
#define NR 1099511627776ull
static void fq3_mul(const uint64_t *a, const uint64_t *b, uint64_t *c) {
  uint64_t a0 = a[0], a1 = a[1], a2 = a[2], b0 = b[0], b1 = b[1], b2 = b[2];
  uint64_t c0 = lfo_add(lfo_mul(a0, b0), lfo_mul(NR, lfo_add(lfo_mul(a1, b2), lfo_mul(a2, b1))));
  uint64_t c1 = lfo_add(lfo_add(lfo_mul(a0, b1), lfo_mul(a1, b0)), lfo_mul(NR, lfo_mul(a2, b2)));
  uint64_t c2 = lfo_add(lfo_add(lfo_mul(a0, b2), lfo_mul(a1, b1)), lfo_mul(a2, b0));
  c[0] = c0;
  c[1] = c1;
  c[2] = c2;
}

/* ------------------------------------------ Phi_72 CRT (GL/ntt.rs:15-47, 135-346) */
static uint64_t W24[24]; /* ROOTS_OF_UNITY_24[i] = (2^40)^i  (GL/ntt.rs:15-40) */
static uint64_t KAPPA_C, EIGHT_INV, FOUR_INV;
static pthread_once_t once = PTHREAD_ONCE_INIT;
static void init_consts(void) {
  W24[0] = 1;
  for (int i = 1; i < 24; i++) W24[i] = lfo_mul(W24[i - 1], NR);
  /* GL/ntt.rs:42-43: the literal is 1/(2*ROOT[4] - 1) (its doc comment says 2*ROOT[4]-1;
   * the value is what the reference computes with, so the literal is used) */
  KAPPA_C = 12297829382473034411ull;
  EIGHT_INV = lfo_inv(8);
  FOUR_INV = lfo_inv(4);
}

/* GL/ntt.rs:348-437 -- isomorphisms between Fq[X]/(X^3 - w^k) and Fq3 */
void lfo_phi72_homogenize(uint64_t *c) { /* GL/ntt.rs:326-334 */
  uint64_t t;
  pthread_once(&once, init_consts);
  c[4] = neg(c[4]);                                  /* 13: c1 = -c1 */
  c[7] = lfo_mul(c[7], W24[2]);                      /* 7 */
  c[8] = lfo_mul(c[8], W24[4]);
  c[10] = lfo_mul(c[10], W24[6]);                    /* 19 */
  c[11] = lfo_mul(c[11], W24[12]);
  t = c[13];                                         /* 5 */
  c[13] = lfo_mul(c[14], W24[3]);
  c[14] = lfo_mul(t, W24[1]);
  t = c[16];                                         /* 17 */
  c[16] = lfo_mul(c[17], W24[11]);
  c[17] = lfo_mul(t, W24[5]);
  t = c[19];                                         /* 11 */
  c[19] = lfo_mul(c[20], W24[7]);
  c[20] = lfo_mul(t, W24[3]);
  t = c[22];                                         /* 23 */
  c[22] = lfo_mul(c[23], W24[15]);
  c[23] = lfo_mul(t, W24[7]);
}
void lfo_phi72_dehomogenize(uint64_t *c) { /* GL/ntt.rs:338-346 */
  uint64_t t;
  pthread_once(&once, init_consts);
  c[4] = neg(c[4]);
  c[7] = lfo_mul(c[7], W24[22]);
  c[8] = lfo_mul(c[8], W24[20]);
  c[10] = lfo_mul(c[10], W24[18]);
  c[11] = lfo_mul(c[11], W24[12]);
  t = c[13];
  c[13] = lfo_mul(c[14], W24[23]);
  c[14] = lfo_mul(t, W24[21]);
  t = c[16];
  c[16] = lfo_mul(c[17], W24[19]);
  c[17] = lfo_mul(t, W24[13]);
  t = c[19];
  c[19] = lfo_mul(c[20], W24[21]);
  c[20] = lfo_mul(t, W24[17]);
  t = c[22];
  c[22] = lfo_mul(c[23], W24[17]);
  c[23] = lfo_mul(t, W24[9]);
}

static void phi72_crt1(uint64_t *c) { /* GL/ntt.rs:135-228 */
  for (int i = 0; i < 12; i++) { /* f mod X^12 - zeta, X^12 - zeta^5 (:146-152) */
    uint64_t a = c[i], b = c[12 + i];
    uint64_t zb = lfo_mul(W24[4], b);
    c[i] = lfo_add(a, zb);
    c[12 + i] = lfo_sub(lfo_add(a, b), zb);
  }
  for (int i = 0; i < 6; i++) { /* :160-179 */
    uint64_t a = c[i], b = lfo_mul(W24[2], c[6 + i]);
    c[i] = lfo_add(a, b);
    c[6 + i] = lfo_sub(a, b);
    a = c[12 + i];
    b = lfo_mul(W24[10], c[18 + i]);
    c[12 + i] = lfo_add(a, b);
    c[18 + i] = lfo_sub(a, b);
  }
  static const int tw[4] = {1, 7, 5, 11}; /* :186-225 */
  for (int i = 0; i < 3; i++)
    for (int q = 0; q < 4; q++) {
      uint64_t a = c[6 * q + i], b = lfo_mul(W24[tw[q]], c[6 * q + 3 + i]);
      c[6 * q + i] = lfo_add(a, b);
      c[6 * q + 3 + i] = lfo_sub(a, b);
    }
  lfo_phi72_homogenize(c);
}

static void phi72_icrt1(uint64_t *c) { /* GL/ntt.rs:240-319 */
  lfo_phi72_dehomogenize(c);
  static const int tw[4] = {23, 17, 19, 13}; /* :250-285 */
  for (int i = 0; i < 3; i++)
    for (int q = 0; q < 4; q++) {
      uint64_t a = c[6 * q + i], b = c[6 * q + 3 + i];
      c[6 * q + i] = lfo_add(a, b);
      c[6 * q + 3 + i] = lfo_mul(W24[tw[q]], lfo_sub(a, b));
    }
  for (int i = 0; i < 6; i++) { /* :291-308 */
    uint64_t a = c[i], b = c[6 + i];
    c[i] = lfo_add(a, b);
    c[6 + i] = lfo_mul(W24[22], lfo_sub(a, b));
    a = c[12 + i];
    b = c[18 + i];
    c[12 + i] = lfo_add(a, b);
    c[18 + i] = lfo_mul(W24[14], lfo_sub(a, b));
  }
  for (int i = 0; i < 12; i++) { /* :311-318 */
    uint64_t a = c[i], b = c[12 + i];
    uint64_t kd = lfo_mul(KAPPA_C, lfo_sub(a, b));
    c[i] = lfo_mul(EIGHT_INV, lfo_sub(lfo_add(a, b), kd));
    c[12 + i] = lfo_mul(FOUR_INV, kd);
  }
}

/* ------------------------------------------- negacyclic X^d + 1 (own convention) */
static void nega_twiddles(int d, uint64_t *psi, uint64_t *psi_inv) {
  uint64_t g = lfo_pow(7, (P - 1) / (uint64_t)(2 * d));
  *psi = g;
  *psi_inv = lfo_inv(g);
}
/* in-place cyclic DFT of size d with root w, natural order in and out */
static void dft(uint64_t *a, int d, uint64_t w) {
  for (int i = 1, j = 0; i < d; i++) { /* bit reversal */
    int bit = d >> 1;
    for (; j & bit; bit >>= 1) j ^= bit;
    j ^= bit;
    if (i < j) {
      uint64_t t = a[i];
      a[i] = a[j];
      a[j] = t;
    }
  }
  for (int len = 2; len <= d; len <<= 1) {
    uint64_t wl = lfo_pow(w, (uint64_t)(d / len));
    for (int i = 0; i < d; i += len) {
      uint64_t x = 1;
      for (int k = 0; k < len / 2; k++) {
        uint64_t u = a[i + k], v = lfo_mul(a[i + k + len / 2], x);
        a[i + k] = lfo_add(u, v);
        a[i + k + len / 2] = lfo_sub(u, v);
        x = lfo_mul(x, wl);
      }
    }
  }
}
/* F[k] = sum_j f_j psi^((2k+1) j) */
static void nega_ntt1(uint64_t *a, int d) {
  uint64_t psi, psii;
  nega_twiddles(d, &psi, &psii);
  uint64_t x = 1;
  for (int j = 0; j < d; j++) {
    a[j] = lfo_mul(a[j], x);
    x = lfo_mul(x, psi);
  }
  dft(a, d, lfo_mul(psi, psi));
}
static void nega_intt1(uint64_t *a, int d) {
  uint64_t psi, psii;
  nega_twiddles(d, &psi, &psii);
  dft(a, d, lfo_mul(psii, psii));
  uint64_t dinv = lfo_inv((uint64_t)d), x = dinv;
  for (int j = 0; j < d; j++) {
    a[j] = lfo_mul(a[j], x);
    x = lfo_mul(x, psii);
  }
}

static int is_pow2(int d) { return d >= 2 && (d & (d - 1)) == 0; }

void lfo_crt(uint64_t *e, size_t n, int d) {
  pthread_once(&once, init_consts);
  for (size_t i = 0; i < n; i++) {
    if (d == 24)
      phi72_crt1(e + i * 24);
    else if (is_pow2(d))
      nega_ntt1(e + i * (size_t)d, d);
    else
      abort();
  }
}
void lfo_icrt(uint64_t *e, size_t n, int d) {
  pthread_once(&once, init_consts);
  for (size_t i = 0; i < n; i++) {
    if (d == 24)
      phi72_icrt1(e + i * 24);
    else if (is_pow2(d))
      nega_intt1(e + i * (size_t)d, d);
    else
      abort();
  }
}

/* SR/cyclotomic_ring/coeff_form.rs:54-67 schoolbook, then reduce:
 * d=24: GL/mod.rs:75-98 (X^24 = X^12 - 1); d=2^k: X^d = -1 */
void lfo_poly_mul(const uint64_t *a, const uint64_t *b, uint64_t *out, int d) {
  uint64_t *t = calloc((size_t)2 * d, sizeof(uint64_t));
  for (int i = 0; i < d; i++)
    for (int j = 0; j < d; j++) t[i + j] = lfo_add(t[i + j], lfo_mul(a[i], b[j]));
  if (d == 24) {
    for (int i = 0; i < 12; i++) t[i] = lfo_sub(lfo_sub(t[i], t[24 + i]), t[36 + i]);
    for (int i = 12; i < 24; i++) t[i] = lfo_add(t[i], t[12 + i]);
  } else {
    for (int i = 0; i < d; i++) t[i] = lfo_sub(t[i], t[d + i]);
  }
  memcpy(out, t, sizeof(uint64_t) * (size_t)d);
  free(t);
}

/* SR/cyclotomic_ring/ntt_form.rs:159-175 (zero short-cut is value-neutral) */
void lfo_slot_mul(const uint64_t *a, const uint64_t *b, uint64_t *out, int d) {
  if (d == 24) {
    for (int s = 0; s < 8; s++) fq3_mul(a + 3 * s, b + 3 * s, out + 3 * s);
  } else {
    for (int s = 0; s < d; s++) out[s] = lfo_mul(a[s], b[s]);
  }
}
static void slot_mul_acc(const uint64_t *a, const uint64_t *b, uint64_t *acc, int d) {
  if (d == 24) {
    uint64_t t[3];
    for (int s = 0; s < 8; s++) {
      fq3_mul(a + 3 * s, b + 3 * s, t);
      for (int c = 0; c < 3; c++) acc[3 * s + c] = lfo_add(acc[3 * s + c], t[c]);
    }
  } else {
    for (int s = 0; s < d; s++) acc[s] = lfo_add(acc[s], lfo_mul(a[s], b[s]));
  }
}

/* ------------------------------------ balanced decomposition (SR/balanced_decomposition)
 * signed representative: fq_convertible.rs:22-34; digits: mod.rs:62-103;
 * rounded_div: linear_algebra/src/ops.rs:64-80; back to Fq: fq_convertible.rs:38-49 */
static i128 signed_rep(uint64_t v) {
  const uint64_t qh = (P - 1) / 2;
  return v > qh ? (i128)v - (i128)P : (i128)v;
}
static uint64_t from_signed(i128 x) {
  if (x < 0) {
    i128 r = x % (i128)P;
    return (uint64_t)(r + (i128)P) % P; /* Fp::from(r + q) */
  }
  return (uint64_t)(x % (i128)P);
}
static i128 rounded_div(i128 dividend, i128 divisor) {
  if ((dividend ^ divisor) >= 0) return (dividend + divisor / 2) / divisor;
  return (dividend - divisor / 2) / divisor;
}
int lfo_decompose_balanced(uint64_t v, uint64_t bu, int len, uint64_t *out) {
  if (bu < 2 || (bu & 1)) return -2;
  i128 curr = signed_rep(v), b = (i128)bu, bh = b / 2;
  int i = 0;
  for (;;) {
    i128 rem = curr % b; /* Rust % truncates like C */
    if (i >= len) return -1; /* the reference indexes out of bounds and panics */
    if ((rem < 0 ? -rem : rem) <= bh) {
      out[i] = from_signed(rem);
      curr /= b;
    } else {
      out[i] = from_signed(rem < 0 ? rem + b : rem - b);
      i128 carry = rounded_div(rem, b);
      curr = curr / b + carry;
    }
    i++;
    if (curr == 0) break;
  }
  for (; i < len; i++) out[i] = 0;
  return 0;
}

int lfo_gadget_decompose(const uint64_t *in, size_t n, int d, uint64_t b, int len,
                         uint64_t *out) {
  uint64_t dig[64];
  if (len > 64) return -2;
  for (size_t j = 0; j < n; j++)
    for (int c = 0; c < d; c++) { /* coeff_form.rs:593-605 */
      if (lfo_decompose_balanced(in[j * d + c], b, len, dig)) return -1;
      for (int k = 0; k < len; k++) out[(j * len + k) * d + c] = dig[k];
    }
  return 0;
}

void lfo_gadget_recompose(const uint64_t *in, size_t n_out, int d, uint64_t b, int len,
                          uint64_t *out) {
  for (size_t j = 0; j < n_out; j++)
    for (int c = 0; c < d; c++) { /* recompose(): Horner from the top digit */
      uint64_t r = 0;
      for (int k = len - 1; k >= 0; k--) r = lfo_add(lfo_mul(r, b % P), in[(j * len + k) * d + c]);
      out[j * d + c] = r;
    }
}

/* --------------------------------------------------------------- threading */
typedef struct {
  void (*fn)(void *, size_t, size_t);
  void *arg;
  size_t lo, hi;
} job_t;
static void *job_run(void *p) {
  job_t *j = p;
  j->fn(j->arg, j->lo, j->hi);
  return NULL;
}
static void parallel_for(size_t n, int nthreads, void (*fn)(void *, size_t, size_t), void *arg) {
  if (nthreads <= 1 || n < 2) {
    fn(arg, 0, n);
    return;
  }
  if ((size_t)nthreads > n) nthreads = (int)n;
  pthread_t th[256];
  job_t jobs[256];
  if (nthreads > 256) nthreads = 256;
  for (int t = 0; t < nthreads; t++) {
    jobs[t].fn = fn;
    jobs[t].arg = arg;
    jobs[t].lo = n * (size_t)t / (size_t)nthreads;
    jobs[t].hi = n * (size_t)(t + 1) / (size_t)nthreads;
    pthread_create(&th[t], NULL, job_run, &jobs[t]);
  }
  for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
}

/* ------------------------------------------------------ Witness (LF/arith.rs) */
typedef struct {
  const uint64_t *in;
  uint64_t *fc, *f;
  int d, L;
  uint64_t B;
  int err;
} wit_arg;
static void wit_from_w_ccs_range(void *p, size_t lo, size_t hi) {
  wit_arg *a = p;
  int d = a->d;
  uint64_t *tmp = malloc(sizeof(uint64_t) * (size_t)d);
  for (size_t j = lo; j < hi; j++) {
    memcpy(tmp, a->in + j * d, sizeof(uint64_t) * (size_t)d);
    lfo_icrt(tmp, 1, d); /* ICRT::elementwise_icrt (:232) */
    if (lfo_gadget_decompose(tmp, 1, d, a->B, a->L, a->fc + j * a->L * d)) a->err = 1;
  }
  free(tmp);
  /* f = CRT(f_coeff) (:238) -- the reference's CRT loop is sequential */
  memcpy(a->f + lo * a->L * d, a->fc + lo * a->L * d, sizeof(uint64_t) * (hi - lo) * a->L * d);
  lfo_crt(a->f + lo * a->L * d, (hi - lo) * a->L, d);
}
int lfo_witness_from_w_ccs(const uint64_t *w_ccs, size_t W, int d, uint64_t B, int L,
                           uint64_t *f_coeff, uint64_t *f, int nthreads) {
  wit_arg a = {w_ccs, f_coeff, f, d, L, B, 0};
  parallel_for(W, nthreads, wit_from_w_ccs_range, &a);
  return a.err ? -1 : 0;
}

typedef struct {
  const uint64_t *f;
  uint64_t *fc, *w;
  int d, L;
  uint64_t B;
} from_f_arg;
static void from_f_range(void *p, size_t lo, size_t hi) {
  from_f_arg *a = p;
  int d = a->d, L = a->L;
  memcpy(a->fc + lo * L * d, a->f + lo * L * d, sizeof(uint64_t) * (hi - lo) * L * d);
  lfo_icrt(a->fc + lo * L * d, (hi - lo) * L, d); /* LF/arith.rs:300 */
  lfo_gadget_recompose(a->f + lo * L * d, hi - lo, d, a->B, L, a->w + lo * d); /* :305 */
}
void lfo_witness_from_f(const uint64_t *f, size_t N, int d, uint64_t B, int L,
                        uint64_t *f_coeff, uint64_t *w_ccs, int nthreads) {
  from_f_arg a = {f, f_coeff, w_ccs, d, L, B};
  parallel_for(N / (size_t)L, nthreads, from_f_range, &a);
}

void lfo_get_fhat_phi72(const uint64_t *f_coeff, size_t N, uint64_t *out) {
  /* LF/arith.rs:273-297: fhat[j][i] slot s = (f_i.coeff[8j + s], 0, 0) */
  for (int j = 0; j < 3; j++)
    for (size_t i = 0; i < N; i++)
      for (int s = 0; s < 8; s++) {
        uint64_t *o = out + ((size_t)j * N + i) * 24 + 3 * s;
        o[0] = f_coeff[i * 24 + 8 * j + s];
        o[1] = 0;
        o[2] = 0;
      }
}

/* --------------------------------------------------------------- Ajtai commit */
typedef struct {
  const uint64_t *A, *f;
  uint64_t *cm;
  size_t kappa, ncols, nvec;
  int d;
} ajtai_arg;
static void ajtai_rows(void *p, size_t lo, size_t hi) {
  ajtai_arg *a = p;
  int d = a->d;
  for (size_t v = 0; v < a->nvec; v++)
    for (size_t i = lo; i < hi; i++) { /* LA/matrix.rs:174-176: row . v */
      uint64_t *acc = a->cm + (v * a->kappa + i) * d;
      memset(acc, 0, sizeof(uint64_t) * (size_t)d);
      for (size_t j = 0; j < a->ncols; j++)
        slot_mul_acc(a->A + (i * a->ncols + j) * d, a->f + (v * a->ncols + j) * d, acc, d);
    }
}
void lfo_ajtai_commit(const uint64_t *A, size_t kappa, size_t ncols, int d, const uint64_t *f,
                      size_t nvec, uint64_t *cm, int nthreads) {
  ajtai_arg a = {A, f, cm, kappa, ncols, nvec, d};
  parallel_for(kappa, nthreads, ajtai_rows, &a);
}

/* ------------------------------------------- decomposition (LF/nifs/decomposition.rs) */
typedef struct {
  const uint64_t *fc;
  uint64_t *fck, *fk, *wk;
  size_t N;
  int d, L, K;
  uint64_t B, bs;
  int err;
} dec_arg;
static void dec_range(void *p, size_t lo, size_t hi) {
  dec_arg *a = p;
  int d = a->d, L = a->L, K = a->K;
  size_t N = a->N;
  uint64_t dig[64];
  /* decompose_B_vec_into_k_vec (decomposition/utils.rs:45-49): per element,
   * per coefficient, K balanced base-b_small digits; transpose to K vectors */
  for (size_t j = lo * L; j < hi * L; j++)
    for (int c = 0; c < d; c++) {
      if (lfo_decompose_balanced(a->fc[j * d + c], a->bs, K, dig)) a->err = 1;
      for (int k = 0; k < K; k++) a->fck[((size_t)k * N + j) * d + c] = dig[k];
    }
  /* Witness::from_f_coeff (LF/arith.rs:324-338) per k: f = CRT, w_ccs = recompose */
  for (int k = 0; k < K; k++) {
    uint64_t *fk = a->fk + (size_t)k * N * d, *fck = a->fck + (size_t)k * N * d;
    memcpy(fk + lo * L * d, fck + lo * L * d, sizeof(uint64_t) * (hi - lo) * L * d);
    lfo_crt(fk + lo * L * d, (hi - lo) * L, d);
    lfo_gadget_recompose(fk + lo * L * d, hi - lo, d, a->B, L,
                         a->wk + ((size_t)k * (N / L) + lo) * d);
  }
}
int lfo_decompose_witness(const uint64_t *f_coeff, size_t N, int d, uint64_t B, int L,
                          uint64_t b_small, int K, uint64_t *f_coeff_k, uint64_t *f_k,
                          uint64_t *w_ccs_k, int nthreads) {
  dec_arg a = {f_coeff, f_coeff_k, f_k, w_ccs_k, N, d, L, K, B, b_small, 0};
  parallel_for(N / (size_t)L, nthreads, dec_range, &a);
  return a.err ? -1 : 0;
}

void lfo_commit_witnesses_y0(const uint64_t *cm, uint64_t *y, size_t kappa, int d,
                             uint64_t b_small, int K) {
  /* LF/nifs/decomposition.rs:183-200: b_sum = fold_rev((acc + y_i) * b), y_0 = cm - b_sum */
  size_t n = kappa * (size_t)d;
  for (size_t c = 0; c < n; c++) {
    uint64_t acc = 0;
    for (int k = K - 1; k >= 1; k--) acc = lfo_mul(lfo_add(acc, y[(size_t)k * n + c]), b_small);
    y[c] = lfo_sub(cm[c], acc);
  }
}

/* ---------------------------------------------------------------------- folding */
int lfo_short_challenge(const uint8_t *bs, size_t nbytes, int d, uint64_t *coeffs) {
  /* CR/rings/goldilocks.rs:41-67: 3 bytes -> 4 coefficients of 6 bits, minus 32 */
  if (d % 4 != 0 || nbytes != (size_t)(3 * d / 4)) return -1;
  for (int i = 0; i < d / 4; i++) {
    int x[4];
    x[0] = (bs[3 * i] & 0x3f) - 32;
    x[1] = (((bs[3 * i] & 0xc0) >> 6) | ((bs[3 * i + 1] & 0x0f) << 2)) - 32;
    x[2] = (((bs[3 * i + 1] & 0xf0) >> 4) | ((bs[3 * i + 2] & 0x03) << 4)) - 32;
    x[3] = ((bs[3 * i + 2] & 0xfc) >> 2) - 32;
    for (int k = 0; k < 4; k++) coeffs[4 * i + k] = x[k] < 0 ? P - (uint64_t)(-x[k]) : (uint64_t)x[k];
  }
  return 0;
}

typedef struct {
  const uint64_t *rho, *f;
  uint64_t *f0;
  size_t nwit, N;
  int d;
} fold_arg;
static void fold_range(void *p, size_t lo, size_t hi) {
  fold_arg *a = p;
  int d = a->d;
  for (size_t j = lo; j < hi; j++) {
    uint64_t *acc = a->f0 + j * d;
    memset(acc, 0, sizeof(uint64_t) * (size_t)d);
    for (size_t i = 0; i < a->nwit; i++) /* LF/nifs/folding.rs:258-268 */
      slot_mul_acc(a->rho + i * d, a->f + (i * a->N + j) * d, acc, d);
  }
}
void lfo_fold_f0(const uint64_t *rho, const uint64_t *f, size_t nwit, size_t N, int d,
                 uint64_t *f0, int nthreads) {
  fold_arg a = {rho, f, f0, nwit, N, d};
  parallel_for(N, nthreads, fold_range, &a);
}
void lfo_fold_cm0(const uint64_t *rho, const uint64_t *cm, size_t nwit, size_t kappa, int d,
                  uint64_t *cm0) {
  fold_arg a = {rho, cm, cm0, nwit, kappa, d}; /* folding/utils.rs:470-476 */
  fold_range(&a, 0, kappa);
}

/* ---------------------------------------- the rest of the folded LCCCS
 * rot (GL/mod.rs:138-149 for Phi_72; X^d = -1 for the negacyclic rings):
 * multiply a coefficient vector by X in place */
static void rot1(uint64_t *c, int d) {
  const uint64_t last = c[d - 1];
  for (int i = d - 1; i > 0; i--) c[i] = c[i - 1];
  c[0] = neg(last);
  if (d == 24) c[12] = lfo_add(c[12], last); /* X^24 = X^12 - 1 */
}
/* rot_lin_combination (CR/rotation.rs:84-101) with rot_sum (:45-63):
 * v_0 = sum_i RotSum(rho_i, flatten(theta_i)); flatten reinterprets the tau
 * NTT elements of theta_i as d base-ring values b_r (Phi_72: Fq3 triples, tau
 * = 3; X^d + 1: Fq, tau = 1); RotSum(a, b)_j = sum_r b_r coeff_j(X^r a);
 * the result is promoted back to tau NTT elements (the same u64 layout). */
void lfo_rot_lin_combination(const uint64_t *rho_coeff, const uint64_t *theta, size_t n, int d,
                             uint64_t *v0) {
  const int comp = d == 24 ? 3 : 1; /* base-ring components per value */
  uint64_t *x = malloc(sizeof(uint64_t) * (size_t)d);
  memset(v0, 0, sizeof(uint64_t) * (size_t)d * comp);
  for (size_t i = 0; i < n; i++) {
    memcpy(x, rho_coeff + i * d, sizeof(uint64_t) * (size_t)d); /* X^0 rho first (traits.rs:72-84) */
    const uint64_t *b = theta + i * (size_t)d * comp;
    for (int r = 0; r < d; r++) {
      for (int j = 0; j < d; j++)
        for (int c = 0; c < comp; c++)
          v0[j * comp + c] = lfo_add(v0[j * comp + c], lfo_mul(b[r * comp + c], x[j]));
      rot1(x, d);
    }
  }
  free(x);
}

/* compute_x_s (LF/nifs/decomposition.rs:172-175) ->
 * decompose_big_vec_into_k_vec_and_compose_back (decomposition/utils.rs:12-42):
 * ICRT, gadget_decompose(B, L), decompose_to_vec(b_small, K) and transpose,
 * recompose each L-chunk with B, CRT. x: m NTT elements; x_s: [K][m] */
int lfo_compute_x_s(const uint64_t *x, size_t m, int d, uint64_t B, int L, uint64_t b_small, int K,
                    uint64_t *x_s) {
  uint64_t *coeff = malloc(sizeof(uint64_t) * m * d);
  uint64_t *gad = malloc(sizeof(uint64_t) * m * L * d);
  uint64_t dig[64];
  int rc = 0;
  memcpy(coeff, x, sizeof(uint64_t) * m * d);
  lfo_icrt(coeff, m, d);
  if (lfo_gadget_decompose(coeff, m, d, B, L, gad)) rc = -1;
  for (size_t j = 0; j < m && !rc; j++)
    for (int c = 0; c < d; c++) {
      uint64_t acc[64];
      for (int k = 0; k < K; k++) acc[k] = 0;
      for (int l = L - 1; l >= 0; l--) { /* recompose(chunk, B): Horner over the L digits */
        if (lfo_decompose_balanced(gad[(j * L + l) * d + c], b_small, K, dig)) rc = -1;
        for (int k = 0; k < K; k++) acc[k] = lfo_add(lfo_mul(acc[k], B % P), dig[k]);
      }
      for (int k = 0; k < K; k++) x_s[((size_t)k * m + j) * d + c] = acc[k];
    }
  if (!rc) lfo_crt(x_s, (size_t)K * m, d);
  free(coeff);
  free(gad);
  return rc;
}

/* --------------------------------------------- Poseidon2-16 (ZK/poseidon2.rs) */
#include "p2_consts.inc"
static const uint64_t EXT_INIT[64] = LF_P2_EXT_INIT;
static const uint64_t EXT_TERM[64] = LF_P2_EXT_TERM;
static const uint64_t INTERNAL[22] = LF_P2_INTERNAL;
static const uint64_t DIAG_M1[16] = LF_P2_DIAG_M1;

static uint64_t sbox(uint64_t x, uint64_t rc) { /* Plonky3 add_rc_and_sbox_generic: (x+rc)^7 */
  uint64_t y = lfo_add(x, rc), y2 = lfo_mul(y, y), y4 = lfo_mul(y2, y2);
  return lfo_mul(lfo_mul(y4, y2), y);
}
void lfo_p2_mds16(uint64_t *s) { /* ZK/poseidon2.rs:243-268, MDSMat4 (sages/initial_mds.sage:27-31) */
  for (int c = 0; c < 16; c += 4) {
    uint64_t x0 = s[c], x1 = s[c + 1], x2 = s[c + 2], x3 = s[c + 3];
    uint64_t t = lfo_add(lfo_add(x0, x1), lfo_add(x2, x3));
    s[c + 0] = lfo_add(t, lfo_add(x0, lfo_add(x1, x1)));           /* 2 3 1 1 */
    s[c + 1] = lfo_add(t, lfo_add(x1, lfo_add(x2, x2)));           /* 1 2 3 1 */
    s[c + 2] = lfo_add(t, lfo_add(x2, lfo_add(x3, x3)));           /* 1 1 2 3 */
    s[c + 3] = lfo_add(t, lfo_add(x3, lfo_add(x0, x0)));           /* 3 1 1 2 */
  }
  for (int k = 0; k < 4; k++) {
    uint64_t sum = lfo_add(lfo_add(s[k], s[4 + k]), lfo_add(s[8 + k], s[12 + k]));
    for (int j = k; j < 16; j += 4) s[j] = lfo_add(s[j], sum);
  }
}
void lfo_p2_permute(uint64_t *s) { /* ZK/poseidon2.rs:100-173 */
  lfo_p2_mds16(s);
  for (int r = 0; r < 4; r++) {
    for (int i = 0; i < 16; i++) s[i] = sbox(s[i], EXT_INIT[16 * r + i]);
    lfo_p2_mds16(s);
  }
  for (int r = 0; r < 22; r++) {
    s[0] = sbox(s[0], INTERNAL[r]);
    uint64_t sum = 0; /* Plonky3 matmul_internal: s_i = s_i * diag_m1_i + sum */
    for (int i = 0; i < 16; i++) sum = lfo_add(sum, s[i]);
    for (int i = 0; i < 16; i++) s[i] = lfo_add(lfo_mul(s[i], DIAG_M1[i]), sum);
  }
  for (int r = 0; r < 4; r++) {
    for (int i = 0; i < 16; i++) s[i] = sbox(s[i], EXT_TERM[16 * r + i]);
    lfo_p2_mds16(s);
  }
}
/* WideZkVMPoseidon2Perm::permute_mut's PermutationIntermediateStates
 * (ZK/poseidon2.rs:91-96, 100-173): st[0] after the initial MDS (:131-132),
 * st[1..4] after each initial external round (:134-146), st[5..26] after each
 * internal round (:150-154), st[27..30] after each terminal external round (:157-169) */
void lfo_p2_permute_states(uint64_t *s, uint64_t *st) {
  lfo_p2_mds16(s);
  memcpy(st, s, 16 * sizeof(uint64_t));
  for (int r = 0; r < 4; r++) {
    for (int i = 0; i < 16; i++) s[i] = sbox(s[i], EXT_INIT[16 * r + i]);
    lfo_p2_mds16(s);
    memcpy(st + 16 * (1 + r), s, 16 * sizeof(uint64_t));
  }
  for (int r = 0; r < 22; r++) {
    s[0] = sbox(s[0], INTERNAL[r]);
    uint64_t sum = 0;
    for (int i = 0; i < 16; i++) sum = lfo_add(sum, s[i]);
    for (int i = 0; i < 16; i++) s[i] = lfo_add(lfo_mul(s[i], DIAG_M1[i]), sum);
    memcpy(st + 16 * (5 + r), s, 16 * sizeof(uint64_t));
  }
  for (int r = 0; r < 4; r++) {
    for (int i = 0; i < 16; i++) s[i] = sbox(s[i], EXT_TERM[16 * r + i]);
    lfo_p2_mds16(s);
    memcpy(st + 16 * (27 + r), s, 16 * sizeof(uint64_t));
  }
}
/* hash_iter returning IntermediateStates (ZK/poseidon2.rs:206-235): one 31 x 16
 * record per permutation, in order; returns the number of permutations */
size_t lfo_p2_hash_iter_states(const uint64_t *in, size_t n, uint64_t out[4], uint64_t *states) {
  uint64_t s[16] = {0};
  size_t pos = 0, np = 0;
  for (;;) {
    int i;
    for (i = 0; i < 12; i++) {
      if (pos < n) {
        s[i] = in[pos++];
      } else {
        if (i != 0) lfo_p2_permute_states(s, states + 31 * 16 * np++);
        goto done;
      }
    }
    lfo_p2_permute_states(s, states + 31 * 16 * np++);
  }
done:
  memcpy(out, s, 4 * sizeof(uint64_t));
  return np;
}
static void p2_range(void *p, size_t lo, size_t hi) {
  uint64_t *st = p;
  for (size_t i = lo; i < hi; i++) lfo_p2_permute(st + 16 * i);
}
void lfo_p2_permute_batch(uint64_t *states, size_t n, int nthreads) {
  parallel_for(n, nthreads, p2_range, states);
}
void lfo_p2_hash_iter(const uint64_t *in, size_t n, uint64_t out[4]) {
  uint64_t s[16] = {0}; /* ZK/poseidon2.rs:210-234 */
  size_t pos = 0;
  for (;;) {
    int i;
    for (i = 0; i < 12; i++) {
      if (pos < n) {
        s[i] = in[pos++];
      } else {
        if (i != 0) lfo_p2_permute(s);
        goto done;
      }
    }
    lfo_p2_permute(s);
  }
done:
  memcpy(out, s, 4 * sizeof(uint64_t));
}

/* ------------------------- DuplexChallenger<Goldilocks, Perm, 16, 12> (Plonky3; unpinned) */
void lfo_tr_init(lfo_transcript *t) { memset(t, 0, sizeof(*t)); }
static void duplexing(lfo_transcript *t) {
  for (int i = 0; i < t->nin; i++) t->state[i] = t->inbuf[i]; /* overwrite mode */
  t->nin = 0;
  lfo_p2_permute(t->state);
  memcpy(t->outbuf, t->state, 12 * sizeof(uint64_t));
  t->nout = 12;
}
void lfo_tr_observe(lfo_transcript *t, uint64_t v) {
  t->nout = 0; /* buffered output is invalidated */
  t->inbuf[t->nin++] = v % P;
  if (t->nin == 12) duplexing(t);
}
uint64_t lfo_tr_sample(lfo_transcript *t) {
  if (t->nin > 0 || t->nout == 0) duplexing(t);
  return t->outbuf[--t->nout]; /* pops from the end */
}
void lfo_tr_absorb_ring(lfo_transcript *t, const uint64_t *e, size_t n, int d) {
  /* ZK/fiat_shamir.rs:51-60: each NTT slot's base-field limbs, as raw ark
   * Montgomery u64s, observed in order */
  for (size_t i = 0; i < n * (size_t)d; i++) lfo_tr_observe(t, lfo_to_mont(e[i]));
}
void lfo_tr_get_challenge(lfo_transcript *t, uint64_t out[3]) {
  for (int i = 0; i < 3; i++) out[i] = lfo_tr_sample(t); /* fiat_shamir.rs:69-86 */
  for (int i = 0; i < 3; i++) lfo_tr_observe(t, out[i]);
}
void lfo_tr_squeeze_bytes(lfo_transcript *t, uint8_t *out, size_t n) {
  while (n > 0) { /* fiat_shamir.rs:88-102: canonical little-endian bytes */
    uint64_t v = lfo_tr_sample(t);
    size_t take = n < 8 ? n : 8;
    for (size_t i = 0; i < take; i++) *out++ = (uint8_t)(v >> (8 * i));
    n -= take;
  }
}

/* ----------------------------------------------------------- synthetic inputs */
static uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
void lfo_fill_uniform(uint64_t *out, size_t n, uint64_t seed) {
  /* element i = SplitMix64 output for counter i, re-mixed until < p
   * (index-addressable, so the device generator reproduces it exactly) */
  const uint64_t G = 0x9e3779b97f4a7c15ull;
  for (size_t i = 0; i < n; i++) {
    uint64_t x = mix64(seed + (uint64_t)(i + 1) * G);
    while (x >= P) x = mix64(x + G);
    out[i] = x;
  }
}

static uint64_t uniform_at(uint64_t seed, uint64_t i) { /* element i of lfo_fill_uniform(seed) */
  const uint64_t G = 0x9e3779b97f4a7c15ull;
  uint64_t x = mix64(seed + (i + 1) * G);
  while (x >= P) x = mix64(x + G);
  return x;
}

/* Ajtai rows of a matrix that exists only as lfo_fill_uniform(seed) of
 * kappa x ncols x d (row-major, as bench.py / the device fill make it): the
 * same product as lfo_ajtai_commit (LA/matrix.rs:168-178), with A generated on
 * the fly, so rows of a 21.5 GB matrix can be checked without a host copy. */
typedef struct {
  uint64_t seed;
  size_t ncols, nchunk;
  int d;
  const uint64_t *f;
  const size_t *rows;
  uint64_t *part; /* [nrows][nchunk][d] */
} seeded_arg;
static void seeded_range(void *p, size_t lo, size_t hi) {
  seeded_arg *a = p;
  const int d = a->d;
  uint64_t *e = malloc(sizeof(uint64_t) * (size_t)d);
  for (size_t job = lo; job < hi; job++) {
    const size_t ri = job / a->nchunk, ch = job % a->nchunk, row = a->rows[ri];
    const size_t j0 = a->ncols * ch / a->nchunk, j1 = a->ncols * (ch + 1) / a->nchunk;
    uint64_t *acc = a->part + job * (size_t)d;
    memset(acc, 0, sizeof(uint64_t) * (size_t)d);
    for (size_t j = j0; j < j1; j++) {
      const uint64_t base = ((uint64_t)row * a->ncols + j) * (uint64_t)d;
      for (int c = 0; c < d; c++) e[c] = uniform_at(a->seed, base + c);
      slot_mul_acc(e, a->f + j * (size_t)d, acc, d);
    }
  }
  free(e);
}
void lfo_ajtai_rows_seeded(uint64_t seed, size_t ncols, int d, const uint64_t *f, const size_t *rows,
                           size_t nrows, uint64_t *cm, int nthreads) {
  pthread_once(&once, init_consts);
  const size_t nchunk = (size_t)(nthreads > 0 ? nthreads : 1) * 4;
  uint64_t *part = malloc(sizeof(uint64_t) * nrows * nchunk * (size_t)d);
  seeded_arg a = {seed, ncols, nchunk, d, f, rows, part};
  parallel_for(nrows * nchunk, nthreads, seeded_range, &a);
  for (size_t r = 0; r < nrows; r++)
    for (int c = 0; c < d; c++) {
      uint64_t v = 0;
      for (size_t ch = 0; ch < nchunk; ch++) v = lfo_add(v, part[(r * nchunk + ch) * (size_t)d + c]);
      cm[r * (size_t)d + c] = v;
    }
  free(part);
}

/* ================================================ multilinear sumcheck (8(f) rank 1)
 * Ring elements in NTT form (d u64: Phi_72's 8 Fq3 slots, or d Fq slots);
 * an MLE over nv variables is 2^nv ring elements, zero-padded (the reference's
 * DenseMultilinearExtension reads missing trailing entries as zero:
 * PL/mle/dense.rs:397-418). Challenges are base-ring elements (Fq3 for
 * Phi_72, Fq otherwise) broadcast into every slot (ntt_form.rs:689-692). */
static int base_deg(int d) { return d == 24 ? 3 : 1; }
static void ring_add(const uint64_t *a, const uint64_t *b, uint64_t *c, int d) {
  for (int i = 0; i < d; i++) c[i] = lfo_add(a[i], b[i]);
}
static void ring_sub(const uint64_t *a, const uint64_t *b, uint64_t *c, int d) {
  for (int i = 0; i < d; i++) c[i] = lfo_sub(a[i], b[i]);
}
static int ring_is_zero(const uint64_t *a, int d) {
  for (int i = 0; i < d; i++)
    if (a[i]) return 0;
  return 1;
}
/* scalar (a base-ring element of base_deg(d) components) into every slot */
static void ring_from_base(const uint64_t *v, int d, uint64_t *out) {
  const int t = base_deg(d);
  for (int i = 0; i < d; i++) out[i] = v[i % t];
}

/* build_eq_x_r (LF/utils/sumcheck/utils.rs:140-210): eq[x] = prod_k (x_k ? r_k : 1 - r_k),
 * x_0 the least significant bit; built from r[nv-1] down as the reference's recursion */
void lfo_eq_table(const uint64_t *r, int nv, int d, uint64_t *out) {
  size_t len = 2;
  uint64_t *tmp = malloc(sizeof(uint64_t) * (size_t)d);
  uint64_t *buf = malloc(sizeof(uint64_t) * ((size_t)d << nv));
  const uint64_t *rl = r + (size_t)(nv - 1) * d;
  for (int i = 0; i < d; i++) buf[i] = lfo_sub((d == 24 && i % 3) ? 0 : 1, rl[i]); /* ONE - r */
  memcpy(buf + d, rl, sizeof(uint64_t) * (size_t)d);
  for (int k = nv - 2; k >= 0; k--) {
    const uint64_t *rk = r + (size_t)k * d;
    for (size_t i = len; i-- > 0;) { /* res[2i] = b_i - r_k b_i, res[2i+1] = r_k b_i */
      uint64_t *bi = buf + i * d;
      lfo_slot_mul(rk, bi, tmp, d);
      ring_sub(bi, tmp, buf + 2 * i * d, d);
      memcpy(buf + (2 * i + 1) * d, tmp, sizeof(uint64_t) * (size_t)d);
    }
    len *= 2;
  }
  memcpy(out, buf, sizeof(uint64_t) * ((size_t)d << nv));
  free(buf);
  free(tmp);
}

/* fix_variables with one point (PL/mle/dense.rs:171-199): mle[b] = left + r (right - left),
 * b < half; the zero short-cut is value-neutral */
void lfo_mle_fix_first(uint64_t *mle, size_t half, int d, const uint64_t *r) {
  uint64_t *a = malloc(sizeof(uint64_t) * (size_t)d), *t = malloc(sizeof(uint64_t) * (size_t)d);
  for (size_t b = 0; b < half; b++) {
    const uint64_t *left = mle + 2 * b * d, *right = mle + (2 * b + 1) * d;
    ring_sub(right, left, a, d);
    if (!ring_is_zero(a, d)) {
      lfo_slot_mul(r, a, t, d);
      ring_add(left, t, mle + b * d, d);
    } else {
      memmove(mle + b * d, left, sizeof(uint64_t) * (size_t)d);
    }
  }
  free(a);
  free(t);
}

/* DenseMultilinearExtension::evaluate (dense.rs:107-113): fix every variable */
void lfo_mle_evaluate(const uint64_t *mle, int nv, int d, const uint64_t *point, uint64_t *out) {
  uint64_t *m = malloc(sizeof(uint64_t) * ((size_t)d << nv));
  memcpy(m, mle, sizeof(uint64_t) * ((size_t)d << nv));
  for (int i = 0; i < nv; i++) lfo_mle_fix_first(m, (size_t)1 << (nv - 1 - i), d, point + (size_t)i * d);
  memcpy(out, m, sizeof(uint64_t) * (size_t)d);
  free(m);
}

/* the sumcheck polynomials' combination functions (lfo_comb, lf_oracle.h):
 * kind 0: folding (folding/utils.rs:278-331): 2K instances of tau f_hat MLEs, B_SMALL, mu [nk][d];
 * kind 1: linearization (linearization/utils.rs:86-104): q multisets, c [q][d], S_off [q+1], S_idx */

static void comb_eval(const lfo_comb *cb, const uint64_t *vals, int d, uint64_t *out) {
  uint64_t *t0 = malloc(sizeof(uint64_t) * (size_t)d), *t1 = malloc(sizeof(uint64_t) * (size_t)d);
  uint64_t *t2 = malloc(sizeof(uint64_t) * (size_t)d), *inter = malloc(sizeof(uint64_t) * (size_t)d);
  if (cb->kind == 0) {
    /* result = v0 v1 + v2 v3 (eq_r * (g1 + g3) of both halves) */
    lfo_slot_mul(vals, vals + d, out, d);
    lfo_slot_mul(vals + 2 * d, vals + 3 * d, t0, d);
    ring_add(out, t0, out, d);
    for (int k = 0; k < cb->nk; k++) {
      const uint64_t *mu = cb->mu + (size_t)k * d;
      memset(inter, 0, sizeof(uint64_t) * (size_t)d);
      for (int dd = cb->tau - 1; dd >= 0; dd--) {
        const uint64_t *f = vals + (size_t)(5 + k * cb->tau + dd) * d;
        if (ring_is_zero(f, d)) {
          if (!ring_is_zero(inter, d)) {
            lfo_slot_mul(inter, mu, t0, d);
            memcpy(inter, t0, sizeof(uint64_t) * (size_t)d);
          }
          continue;
        }
        memcpy(t1, vals + 4 * d, sizeof(uint64_t) * (size_t)d); /* eval = eq_beta */
        lfo_slot_mul(f, f, t2, d);                                /* f^2 */
        for (int b = 1; b < cb->bsmall; b++) {
          uint64_t m[4096];
          const uint64_t bb = (uint64_t)b * (uint64_t)b;
          for (int i = 0; i < d; i++) m[i] = lfo_sub(t2[i], (d == 24 && i % 3) ? 0 : bb); /* f^2 - b^2 */
          if (ring_is_zero(m, d)) {
            memset(t1, 0, sizeof(uint64_t) * (size_t)d);
            break;
          }
          lfo_slot_mul(t1, m, t0, d);
          memcpy(t1, t0, sizeof(uint64_t) * (size_t)d);
        }
        lfo_slot_mul(t1, f, t0, d); /* eval *= f_i */
        ring_add(inter, t0, inter, d);
        lfo_slot_mul(inter, mu, t0, d);
        memcpy(inter, t0, sizeof(uint64_t) * (size_t)d);
      }
      ring_add(out, inter, out, d);
    }
  } else {
    memset(out, 0, sizeof(uint64_t) * (size_t)d);
    for (int i = 0; i < cb->q; i++) {
      const uint64_t *c = cb->c + (size_t)i * d;
      if (ring_is_zero(c, d)) continue;
      memcpy(t1, c, sizeof(uint64_t) * (size_t)d);
      int skip = 0;
      for (int s = cb->S_off[i]; s < cb->S_off[i + 1]; s++) {
        const uint64_t *v = vals + (size_t)cb->S_idx[s] * d; /* vals[j], j the matrix index */
        if (ring_is_zero(v, d)) {
          skip = 1;
          break;
        }
        lfo_slot_mul(t1, v, t0, d);
        memcpy(t1, t0, sizeof(uint64_t) * (size_t)d);
      }
      if (!skip) ring_add(out, t1, out, d);
    }
    (void)t2;
  }
  free(t0);
  free(t1);
  free(t2);
  free(inter);
}
/* the combination function at one point of the sumcheck domain: vals [nm][d] -> out */
void lfo_comb_eval(const lfo_comb *cb, const uint64_t *vals, int nm, int d, uint64_t *out) {
  if (cb->kind == 1) { /* eq is the last MLE: result * vals[last] */
    uint64_t *t = malloc(sizeof(uint64_t) * (size_t)d);
    comb_eval(cb, vals, d, t);
    lfo_slot_mul(t, vals + (size_t)(nm - 1) * d, out, d);
    free(t);
  } else {
    comb_eval(cb, vals, d, out);
  }
}

/* IPForMLSumcheck::prove_round's sum (LF/utils/sumcheck/prover.rs:93-167):
 * evals[e] = sum_b comb(v_b(e)), v_b(e) = mle[2b] + e (mle[2b+1] - mle[2b]), e <= degree;
 * mles [nm][2^nv][d] */
void lfo_sumcheck_round(const lfo_comb *cb, const uint64_t *mles, int nm, int nv, int d, int degree,
                        uint64_t *evals) {
  const size_t n = (size_t)1 << nv, half = n / 2;
  uint64_t *v0 = malloc(sizeof(uint64_t) * (size_t)nm * d), *v1 = malloc(sizeof(uint64_t) * (size_t)nm * d);
  uint64_t *st = malloc(sizeof(uint64_t) * (size_t)nm * d), *v = malloc(sizeof(uint64_t) * (size_t)nm * d);
  uint64_t *le = malloc(sizeof(uint64_t) * (size_t)d);
  memset(evals, 0, sizeof(uint64_t) * (size_t)(degree + 1) * d);
  for (size_t b = 0; b < half; b++) {
    for (int m = 0; m < nm; m++) {
      memcpy(v0 + (size_t)m * d, mles + ((size_t)m * n + 2 * b) * d, sizeof(uint64_t) * (size_t)d);
      memcpy(v1 + (size_t)m * d, mles + ((size_t)m * n + 2 * b + 1) * d, sizeof(uint64_t) * (size_t)d);
    }
    lfo_comb_eval(cb, v0, nm, d, le);
    ring_add(evals, le, evals, d);
    lfo_comb_eval(cb, v1, nm, d, le);
    ring_add(evals + d, le, evals + d, d);
    for (int m = 0; m < nm; m++) ring_sub(v1 + (size_t)m * d, v0 + (size_t)m * d, st + (size_t)m * d, d);
    memcpy(v, v1, sizeof(uint64_t) * (size_t)nm * d);
    for (int e = 2; e <= degree; e++) {
      for (int m = 0; m < nm; m++) ring_add(v + (size_t)m * d, st + (size_t)m * d, v + (size_t)m * d, d);
      lfo_comb_eval(cb, v, nm, d, le);
      ring_add(evals + (size_t)e * d, le, evals + (size_t)e * d, d);
    }
  }
  free(v0);
  free(v1);
  free(st);
  free(v);
  free(le);
}

/* MLSumcheck::prove_as_subprotocol (LF/utils/sumcheck.rs:61-88) with the
 * Poseidon2 transcript: absorb nvars, degree; per round the prover message
 * (degree + 1 ring elements) is absorbed, the challenge (a base-ring element:
 * fiat_shamir.rs:69-86 for Fq3; one sample for Fq) sampled and absorbed as a
 * broadcast ring element, and every MLE's first variable fixed to it.
 * mles are consumed (fixed in place). proof [nv][degree+1][d], randomness [nv][tau]. */
void lfo_sumcheck_prove(lfo_transcript *t, const lfo_comb *cb, uint64_t *mles, int nm, int nv, int d, int degree,
                        uint64_t *proof, uint64_t *randomness) {
  const int tb = base_deg(d);
  uint64_t *scal = calloc((size_t)d, sizeof(uint64_t)), *rr = malloc(sizeof(uint64_t) * (size_t)d);
  uint64_t *work = malloc(sizeof(uint64_t) * (size_t)nm * ((size_t)d << nv));
  memcpy(work, mles, sizeof(uint64_t) * (size_t)nm * ((size_t)d << nv));
  uint64_t sv[3] = {(uint64_t)nv, 0, 0};
  ring_from_base(sv, d, scal); /* R::from(nvars as u128) */
  lfo_tr_absorb_ring(t, scal, 1, d);
  sv[0] = (uint64_t)degree;
  ring_from_base(sv, d, scal);
  lfo_tr_absorb_ring(t, scal, 1, d);
  for (int i = 0; i < nv; i++) {
    const int cur = nv - i; /* variables left */
    const size_t n = (size_t)1 << cur;
    /* the MLEs of this round are the first 2^cur entries of each (stride 2^nv) */
    uint64_t *tmp = malloc(sizeof(uint64_t) * (size_t)nm * n * d);
    for (int m = 0; m < nm; m++)
      memcpy(tmp + (size_t)m * n * d, work + (size_t)m * ((size_t)d << nv), sizeof(uint64_t) * n * d);
    uint64_t *msg = proof + (size_t)i * (degree + 1) * d;
    lfo_sumcheck_round(cb, tmp, nm, cur, d, degree, msg);
    free(tmp);
    lfo_tr_absorb_ring(t, msg, (size_t)degree + 1, d);
    uint64_t *ch = randomness + (size_t)i * tb;
    if (tb == 3) {
      lfo_tr_get_challenge(t, ch);
    } else {
      ch[0] = lfo_tr_sample(t);
      lfo_tr_observe(t, ch[0]);
    }
    ring_from_base(ch, d, rr);
    lfo_tr_absorb_ring(t, rr, 1, d);
    for (int m = 0; m < nm; m++) lfo_mle_fix_first(work + (size_t)m * ((size_t)d << nv), n / 2, d, rr);
  }
  memcpy(mles, work, sizeof(uint64_t) * (size_t)nm * ((size_t)d << nv));
  free(work);
  free(scal);
  free(rr);
}

/* the verifier's check (LF/utils/sumcheck/verifier.rs:100-129) with
 * interpolate_uni_poly (:143-222) as plain Lagrange interpolation at 0..degree:
 * p(0) + p(1) = expected each round, expected <- p(r). Returns 0 and the final
 * expected evaluation, or -1 - round when a round's sum is wrong. */
int lfo_sumcheck_check(const uint64_t *proof, const uint64_t *randomness, int nv, int d, int degree,
                       const uint64_t *asserted_sum, uint64_t *expected_out) {
  const int tb = base_deg(d);
  uint64_t *exp = malloc(sizeof(uint64_t) * (size_t)d), *s = malloc(sizeof(uint64_t) * (size_t)d);
  uint64_t *rr = malloc(sizeof(uint64_t) * (size_t)d), *acc = malloc(sizeof(uint64_t) * (size_t)d);
  uint64_t *w = malloc(sizeof(uint64_t) * (size_t)d), *t = malloc(sizeof(uint64_t) * (size_t)d);
  memcpy(exp, asserted_sum, sizeof(uint64_t) * (size_t)d);
  int rc = 0;
  for (int i = 0; i < nv && !rc; i++) {
    const uint64_t *ev = proof + (size_t)i * (degree + 1) * d;
    ring_add(ev, ev + d, s, d);
    if (memcmp(s, exp, sizeof(uint64_t) * (size_t)d)) {
      rc = -1 - i;
      break;
    }
    ring_from_base(randomness + (size_t)i * tb, d, rr);
    memset(acc, 0, sizeof(uint64_t) * (size_t)d);
    for (int k = 0; k <= degree; k++) { /* L_k(r) = prod_{j != k} (r - j) / (k - j) */
      uint64_t num[4096];
      uint64_t one[3] = {1, 0, 0};
      ring_from_base(one, d, num);
      uint64_t den = 1;
      for (int j = 0; j <= degree; j++) {
        if (j == k) continue;
        uint64_t jj[3] = {(uint64_t)j, 0, 0}, tmp[4096];
        ring_from_base(jj, d, tmp);
        ring_sub(rr, tmp, tmp, d);
        lfo_slot_mul(num, tmp, w, d);
        memcpy(num, w, sizeof(uint64_t) * (size_t)d);
        den = lfo_mul(den, k > j ? (uint64_t)(k - j) : P - (uint64_t)(j - k));
      }
      const uint64_t dinv = lfo_inv(den);
      for (int c = 0; c < d; c++) num[c] = lfo_mul(num[c], dinv);
      lfo_slot_mul(num, ev + (size_t)k * d, t, d);
      ring_add(acc, t, acc, d);
    }
    memcpy(exp, acc, sizeof(uint64_t) * (size_t)d);
  }
  memcpy(expected_out, exp, sizeof(uint64_t) * (size_t)d);
  free(exp);
  free(s);
  free(rr);
  free(acc);
  free(w);
  free(t);
  return rc;
}

/* ================================================ sparse Mz products (8(f) rank 2)
 * mat_vec_mul (LF/arith/utils.rs:52-65): y[r] = sum over row r's (value, col)
 * of value (.) z[col]; CSR: row_ptr [nrows + 1], col, val [nnz][d] */
void lfo_spmv(const uint64_t *row_ptr, const uint32_t *col, const uint64_t *val, size_t nrows, int d,
              const uint64_t *z, uint64_t *y) {
  for (size_t r = 0; r < nrows; r++) {
    uint64_t *acc = y + r * (size_t)d;
    memset(acc, 0, sizeof(uint64_t) * (size_t)d);
    for (uint64_t k = row_ptr[r]; k < row_ptr[r + 1]; k++)
      slot_mul_acc(val + k * (size_t)d, z + (size_t)col[k] * d, acc, d);
  }
}

/* ================================================ width-8 Poseidon2 Merkle trees (8(f) rank 3)
 * Poseidon2Goldilocks<8> (zkvm/src/poseidon2.rs:31-49, Plonky3 p3-poseidon2 at
 * git 33e58c7, not vendored): the width-16 round structure above with the
 * width-8 external constants (crypto_consts.rs:9-96), the same 22 internal
 * constants, MDS light on two 4-chunks, and Plonky3's MATRIX_DIAG_8_GOLDILOCKS
 * (restated; parity unpinned: no reference vector exists) */
static const uint64_t EXT8_INIT[32] = LF_P2W8_EXT_INIT;
static const uint64_t EXT8_TERM[32] = LF_P2W8_EXT_TERM;
static const uint64_t DIAG8_M1[8] = LF_P2W8_DIAG_M1;
static void mds8(uint64_t *s) {
  for (int c = 0; c < 8; c += 4) {
    uint64_t x0 = s[c], x1 = s[c + 1], x2 = s[c + 2], x3 = s[c + 3];
    uint64_t t = lfo_add(lfo_add(x0, x1), lfo_add(x2, x3));
    s[c + 0] = lfo_add(t, lfo_add(x0, lfo_add(x1, x1)));
    s[c + 1] = lfo_add(t, lfo_add(x1, lfo_add(x2, x2)));
    s[c + 2] = lfo_add(t, lfo_add(x2, lfo_add(x3, x3)));
    s[c + 3] = lfo_add(t, lfo_add(x3, lfo_add(x0, x0)));
  }
  for (int k = 0; k < 4; k++) {
    uint64_t sum = lfo_add(s[k], s[4 + k]);
    s[k] = lfo_add(s[k], sum);
    s[4 + k] = lfo_add(s[4 + k], sum);
  }
}
void lfo_p2w8_permute(uint64_t *s) {
  mds8(s);
  for (int r = 0; r < 4; r++) {
    for (int i = 0; i < 8; i++) s[i] = sbox(s[i], EXT8_INIT[8 * r + i]);
    mds8(s);
  }
  for (int r = 0; r < 22; r++) {
    s[0] = sbox(s[0], INTERNAL[r]);
    uint64_t sum = 0;
    for (int i = 0; i < 8; i++) sum = lfo_add(sum, s[i]);
    for (int i = 0; i < 8; i++) s[i] = lfo_add(lfo_mul(s[i], DIAG8_M1[i]), sum);
  }
  for (int r = 0; r < 4; r++) {
    for (int i = 0; i < 8; i++) s[i] = sbox(s[i], EXT8_TERM[8 * r + i]);
    mds8(s);
  }
}
/* PaddingFreeSponge<perm, 8, rate 4, out 4>::hash_iter: overwrite mode, permute
 * on a partial final block, no padding (the structure of poseidon2.rs:210-234) */
void lfo_p2w8_hash(const uint64_t *in, size_t n, uint64_t out[4]) {
  uint64_t s[8] = {0};
  size_t pos = 0;
  for (;;) {
    int i;
    for (i = 0; i < 4; i++) {
      if (pos < n) {
        s[i] = in[pos++];
      } else {
        if (i != 0) lfo_p2w8_permute(s);
        goto done;
      }
    }
    lfo_p2w8_permute(s);
  }
done:
  memcpy(out, s, 4 * sizeof(uint64_t));
}
/* TruncatedPermutation<perm, 2, 4, 8>::compress: permute(a || b)[0..4] */
void lfo_p2w8_compress(const uint64_t a[4], const uint64_t b[4], uint64_t out[4]) {
  uint64_t s[8];
  memcpy(s, a, 32);
  memcpy(s + 4, b, 32);
  lfo_p2w8_permute(s);
  memcpy(out, s, 32);
}
/* MerkleTreeMmcs::commit of one RowMajorMatrix of nrows (a power of two) rows
 * (commitments.rs:192-262): leaf = hash(row), parent = compress(left, right).
 * nodes: every level's digests concatenated, leaves first, root last
 * ((2 nrows - 1) x 4 words) */
/* Plonky3 MerkleTree::new over one matrix (p3-merkle-tree merkle_tree.rs,
 * git 33e58c7787f9, not vendored: restated): first_digest_layer hashes every
 * row and pads the layer to an even length with the zero digest (a single row
 * is the root); every next layer compresses pairs and pads to an even length
 * again (compress: next_len_padded = prev == 2 ? 1 : (prev / 2 + 1) & ~1).
 * Called with PAGE_COUNT rows by vm_mem_comm_with_opening
 * (ZK/commitments.rs:222-240) and with the code half-words by vm_code_comm
 * (:314-340). nodes: the padded layers, leaves first, root last. */
size_t lfo_merkle_nodes(size_t nrows) {
  size_t n = nrows <= 1 ? 1 : nrows + nrows % 2, tot = n;
  while (n > 1) {
    n = n == 2 ? 1 : ((n / 2 + 1) & ~(size_t)1);
    tot += n;
  }
  return tot;
}
void lfo_merkle_tree(const uint64_t *rows, size_t nrows, size_t width, uint64_t *nodes) {
  size_t n = nrows <= 1 ? 1 : nrows + nrows % 2, off = 0;
  for (size_t i = 0; i < nrows; i++) lfo_p2w8_hash(rows + i * width, width, nodes + 4 * i);
  memset(nodes + 4 * nrows, 0, 32 * (n - nrows));
  while (n > 1) {
    const size_t nn = n == 2 ? 1 : ((n / 2 + 1) & ~(size_t)1);
    for (size_t i = 0; i < n / 2; i++)
      lfo_p2w8_compress(nodes + 4 * (off + 2 * i), nodes + 4 * (off + 2 * i + 1), nodes + 4 * (off + n + i));
    memset(nodes + 4 * (off + n + n / 2), 0, 32 * (nn - n / 2));
    off += n;
    n = nn;
  }
}
