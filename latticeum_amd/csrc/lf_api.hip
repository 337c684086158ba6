// lf_api.hip -- the extern "C" boundary (include/lf.h): context, twiddle
// tables, host-buffer wrappers, the device-resident commit+fold step, and the
// host-side transcript. No CPU compute fallback exists: every ring/commit/fold
// operation runs on the GPU, and creating a context fails loudly without one.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>  // types only: the RCCL entry points are resolved at run time (rccl())

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "../../include/lf.h"
#include "gl.hpp"
#include "kernels.hpp"

namespace {

struct Tables {
  uint64_t *mem = nullptr;  // 4*d u64: fwd twist | fwd roots | inv twist | inv roots
  ring::NegaTables fwd{}, inv{};
};

struct TimedLaunch {
  hipEvent_t a, b;
  int nvec;       // Ajtai launches: vectors per launch; phases: -1 - LF_PHASE_*
  int count = 1;  // steps the launch covers (a batched contraction: every step's share)
};

}  // namespace

struct lf_ctx {
  int device = 0;
  hipStream_t own = nullptr, cur = nullptr;
  int *d_err = nullptr;
  int *d_sync = nullptr;        // two ints, zero between launches (k_rho_prep's cross-block flag)
  std::string last_error;
  std::map<int, Tables> tables;
  uint64_t *scratch = nullptr;  // Ajtai split partial sums
  size_t scratch_elems = 0;
  uint64_t *ybuf = nullptr;     // batched commitments before they are scattered to y / cm
  size_t ybuf_elems = 0;
  uint4 *frag = nullptr;        // vectors in MFMA fragment order (ajtai_mfma.hip)
  size_t frag_elems = 0;
  uint32_t *smg = nullptr;      // packed coefficients for the fused decomposition
  size_t smg_elems = 0;
  size_t smg_sides_n = 0;       // N when smg_side holds both sides of the last fused d = 1024 fold_commit, else 0
  uint32_t *smg_side[2] = {nullptr, nullptr};  // those packed words: the caller's planes, or smg
  size_t masks24_n = 0;         // N when masks24 hold both sides' Phi_72 digit masks of the last fold_commit, else 0
  const uint2 *masks24[2] = {nullptr, nullptr};  // in fkeys or the caller's lf_fold_step_bufs.planes
  uint32_t *fkeys = nullptr;    // coefficient-form fold: digit keys [2 N][K][64] (fold_coeff.hip)
  size_t fkeys_elems = 0;
  uint64_t *faux = nullptr;     // coefficient-form fold: rho coefficients, byte tables, the not-short flag
  int32_t *fpart = nullptr;     // coefficient-form fold with few elements: per witness-split partial sums
  size_t fpart_elems = 0;
  size_t faux_elems = 0;
  uint64_t *sink = nullptr;     // 32 KiB row the fused decompositions store work past the end into
  uint8_t *dead = nullptr;      // dead-unit flags of the operand rows (lfk::DeadUnits) [2 nch][32]
  size_t dead_elems = 0;
  uint4 *zero80 = nullptr;      // 32 operand pieces of 0x80 bytes: the offset form of 0 (dead units)
  lfk::DeadUnits dead_units{};  // the last fused decomposition's flags (what the readers of c->frag honour)
  int ncu = 0;                  // compute units of `device`
  uint64_t *stage = nullptr;    // sharded step: the partial commitments [nvec][kappa d]
  size_t stage_elems = 0;
  uint64_t *limb = nullptr;     // RCCL transport: [lo | hi] 32-bit limbs of a field vector
  size_t limb_elems = 0;
  uint64_t *tmp = nullptr;      // small intermediates (compute_x_s)
  size_t tmp_elems = 0;
  uint64_t *sc = nullptr;       // sumcheck: fixed MLEs of the next round, round partial sums, weights
  size_t sc_elems = 0;
  uint64_t *ptrs = nullptr;     // lf_sumcheck_prove_ptrs: the MLE pointer table
  size_t ptrs_elems = 0;
  int *sel = nullptr;           // lf_dev_mz_mles_sel: the selected matrices
  size_t sel_elems = 0;
  uint64_t *hmsg = nullptr;     // pinned host staging of the sumcheck round messages
  size_t hmsg_elems = 0;
  lfk::FoldRows fold_rows{};    // a step without f_k buffers: where its 2K planes sit in the operand rows
  bool fold_from_frag = false;
  bool frag_fallback = false;   // packed d = 1024 planes: fold_rows serve the not-short-rho fallback
  bool timing = false;
  hipEvent_t join = nullptr;    // lf_dev_fold_step_batch: this stream's point to wait for / be waited on
  hipStream_t contract = nullptr;  // lf_ctx_set_contract_stream: where batched contractions led by this context run
  hipEvent_t cjoin = nullptr;   // the end of the last such contraction
  std::vector<TimedLaunch> pending;
  std::map<int, std::pair<double, long>> stats;  // nvec -> (ms, count)
};

// restores the calling thread's device on scope exit (also for destructors)
struct DevGuardBase {
  int prev = -1;
  explicit DevGuardBase(int dev) {
    int cur = -1;
    if (dev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != dev && hipSetDevice(dev) == hipSuccess) prev = cur;
  }
  ~DevGuardBase() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

struct lf_ajtai {
  int device = 0;
  const uint64_t *A = nullptr;
  uint4 *Af = nullptr;  // A in i8-MFMA fragment order, mfma_ktiles(kappa) tiles of 32 rows
  uint64_t *kr = nullptr;  // FOFF x row sums of A per (row, output slot): lfk::ajtai_rowsums
  lfk::FragGeom geom{};  // contraction order of the fragments (ajtai_mfma.hip)
  bool owned = false;
  size_t kappa = 0, ncols = 0;
  int d = 0;
};

// the CCS matrices on the device (lf_ccs_create), plus the structure the
// linearization needs (lf_ccs_set_structure): l, the degree, c and S
struct lf_ccs {
  int device = 0;
  lfk::CcsDev dev{};
  std::vector<void *> bufs;
  bool structured = false;
  size_t l = 0;
  int degree = 0;
  std::vector<uint64_t> c;     // q NTT elements, canonical
  std::vector<int> S_off, S_idx;
  std::vector<uint8_t> live;   // [t][m]: row r of M_j holds an entry
  uint64_t *c_dev = nullptr;   // in bufs
  size_t c_dev_elems = 0;
  ~lf_ccs() {  // every device buffer, also on a failed lf_ccs_create
    DevGuardBase g(device);
    for (void *p : bufs) (void)hipFree(p);
  }
};

// a communicator for the accumulator exchange (RCCL over xGMI)
struct lf_comm {
  ncclComm_t comm = nullptr;
  bool owned = false;
  int nranks = 1, rank = 0;
};

namespace {

// Every entry point runs on its context's device and restores the caller's
// current device afterwards, so contexts on different GPUs can be used from
// one thread (lf.h threading contract).
struct DevGuard {
  int prev = -1;
  explicit DevGuard(int dev) {
    int cur = -1;
    if (dev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != dev && hipSetDevice(dev) == hipSuccess) prev = cur;
  }
  explicit DevGuard(const lf_ctx *c);
  ~DevGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};
DevGuard::DevGuard(const lf_ctx *c) : DevGuard(c ? c->device : -1) {}

int fail(lf_ctx *c, int code, const std::string &msg) {
  if (c) c->last_error = msg;
  return code;
}

#define LF_HIP(ctx, call)                                                                         \
  do {                                                                                            \
    hipError_t e_ = (call);                                                                       \
    if (e_ != hipSuccess)                                                                         \
      return fail((ctx), e_ == hipErrorOutOfMemory ? LF_ERR_OUT_OF_MEMORY : LF_ERR_DEVICE,        \
                  std::string(#call) + ": " + hipGetErrorString(e_));                            \
  } while (0)

#define LF_TRY(expr)          \
  do {                        \
    int r_ = (expr);          \
    if (r_ != LF_OK) return r_; \
  } while (0)

bool ring_ok(int d) { return d == 24 || d == 16 || d == 64 || d == 256 || d == 1024 || d == 4096; }

int log2_exact(uint64_t v) {
  if (v < 2 || (v & (v - 1))) return -1;
  int l = 0;
  while ((1ull << l) != v) l++;
  return l;
}

int check_params(lf_ctx *c, const lf_params *pr, int &lb, int &lbs) {
  if (!pr) return fail(c, LF_ERR_INVALID_ARG, "null params");
  if (!ring_ok(pr->d)) return fail(c, LF_ERR_UNSUPPORTED_RING, "unsupported ring degree");
  lb = log2_exact(pr->B);
  lbs = log2_exact(pr->b_small);
  if (lb < 1 || lb > 62 || lbs < 1 || lbs > 62 || pr->L < 1 || pr->K < 1 || pr->L > 8 || pr->K > 64)
    return fail(c, LF_ERR_INVALID_ARG, "device path needs power-of-two B, b_small and L<=8, K<=64");
  return LF_OK;
}

// negacyclic twiddle tables for degree d (built on the host once per context)
int get_tables(lf_ctx *c, int d, Tables *&out) {
  auto it = c->tables.find(d);
  if (it != c->tables.end()) {
    out = &it->second;
    return LF_OK;
  }
  Tables t;
  if (d != 24) {
    // d = 1024: the 32 x 32 NTT middle factors (fwd, inv); d = 4096: those of its
    // 1024-point sub-transforms, then the radix-4 twists (fwd, inv) and the digit
    // butterfly table (kernels_n4k.hip)
    const size_t extra = d == 1024 ? 2048 : d == 4096 ? 2048 + 2 * 4096 + 1024 : 0;
    // d = 1024: then the D8 byte planes of zeta^((2 m1 + 1) j2) for the matrix-core stage 1 (1024 u64);
    // d = 4096: the quarters' stage-1 planes Z''_m0 (4 x 4096 u64) and middle factors (4 x 1024)
    const size_t az_off = 4 * (size_t)d + extra;
    std::vector<uint64_t> h(az_off + (d == 1024 ? 1024 : d == 4096 ? 4 * 4096 + 4 * 1024 : 0));
    const uint64_t psi = gl::pow(7, (gl::P - 1) / (2 * (uint64_t)d));
    const uint64_t psi_inv = gl::inv(psi), w = gl::mul(psi, psi), w_inv = gl::mul(psi_inv, psi_inv);
    const uint64_t dinv = gl::inv((uint64_t)d);
    uint64_t a = 1, b = 1, x = dinv, y = 1;
    for (int j = 0; j < d; j++) {
      h[j] = a;                // psi^j
      h[d + j] = b;            // w^j
      h[2 * d + j] = x;        // d^-1 psi^-j
      h[3 * d + j] = y;        // w^-j
      a = gl::mul(a, psi);
      b = gl::mul(b, w);
      x = gl::mul(x, psi_inv);
      y = gl::mul(y, w_inv);
    }
    // ring.hpp stockham4: omega^(d/4) is the shift 2^48
    if (h[d + d / 4] != gl::mul_pow2(1, 48) || h[3 * d + d / 4] != gl::mul_pow2(1, 144))
      return fail(c, LF_ERR_DEVICE, "unexpected 4th root of unity");
    if (extra) {
      // the 1024-point transform's root: psi itself (d = 1024) or psi^4 (d = 4096)
      const uint64_t p1 = d == 1024 ? psi : gl::pow(psi, 4), p1_inv = gl::inv(p1), q1inv = gl::inv(1024);
      // ntt32.hpp relies on p1^32 = 2^39 and p1^64 = 2^78 (shift-only 32-point stages)
      if (gl::pow(p1, 32) != gl::mul_pow2(1, 39) || gl::pow(p1, 64) != gl::mul_pow2(1, 78))
        return fail(c, LF_ERR_DEVICE, "unexpected root of unity for the 32 x 32 NTT");
      auto brv5 = [](int i) { return ((i & 1) << 4) | ((i & 2) << 2) | (i & 4) | ((i & 8) >> 2) | ((i & 16) >> 4); };
      for (int r = 0; r < 32; r++)
        for (int i = 0; i < 32; i++) {
          // forward: p1^((2 brv5(i) + 1) r);  inverse: 1024^-1 p1^-((2r + 1) brv5(i))
          h[4 * d + r * 32 + i] = gl::pow(p1, (uint64_t)(2 * brv5(i) + 1) * r);
          h[4 * d + 1024 + r * 32 + i] = gl::mul(q1inv, gl::pow(p1_inv, (uint64_t)(2 * r + 1) * brv5(i)));
        }
      if (d == 1024) {
        // az[t][m1][j2] = signed byte t of D8(zeta^((2 m1 + 1) j2)), zeta = p1^32 (frag.hpp d8)
        int8_t *az = reinterpret_cast<int8_t *>(h.data() + az_off);
        const uint64_t zeta = gl::pow(p1, 32);
        for (int m1 = 0; m1 < 32; m1++)
          for (int j2 = 0; j2 < 32; j2++) {
            const uint64_t x = gl::pow(zeta, (uint64_t)(2 * m1 + 1) * j2);
            const uint64_t tt = x <= 0x7F7F7F7F7F7F7F7Full ? x : x + 0xFFFFFFFFull;
            const uint64_t dd = (tt + 0x8080808080808080ull) ^ 0x8080808080808080ull;
            for (int b = 0; b < 8; b++) az[(b * 32 + m1) * 32 + j2] = (int8_t)(uint8_t)(dd >> (8 * b));
          }
      }
      if (d == 4096) {
        // kernels_n4k.hip relies on psi^1024 = 2^120 (the radix-4 butterflies are shifts)
        if (gl::pow(psi, 1024) != gl::mul_pow2(1, 120)) return fail(c, LF_ERR_DEVICE, "unexpected 8th root of unity");
        uint64_t *tf = h.data() + 4 * d + 2048, *ti = tf + 4096, *zt = ti + 4096;
        const uint64_t inv4 = gl::inv(4);
        for (int m0 = 0; m0 < 4; m0++) {
          const uint64_t s = gl::pow(psi, (uint64_t)((2 * m0 - 3 + 8192) % 8192));  // psi^(2 m0 - 3)
          const uint64_t s_inv = gl::inv(s);
          uint64_t f = 1, g = inv4;
          for (int ai = 0; ai < 1024; ai++) {
            tf[m0 * 1024 + ai] = f;  // psi^((2 m0 - 3) a)
            ti[m0 * 1024 + ai] = g;  // 4^-1 psi^-((2 m0 - 3) a)
            f = gl::mul(f, s);
            g = gl::mul(g, s_inv);
          }
          for (int idx = 0; idx < 256; idx++) {  // sum_b d_b 2^(120 b (2 m0 + 1)), d_b = +-bit_b
            uint64_t z = 0;
            for (int bb = 0; bb < 4; bb++) {
              if (!((idx >> bb) & 1)) continue;
              const uint64_t cb = gl::mul_pow2(1, (120 * bb * (2 * m0 + 1)) % 192);
              z = (idx >> (4 + bb)) & 1 ? gl::sub(z, cb) : gl::add(z, cb);
            }
            zt[m0 * 256 + idx] = z;
          }
        }
        // stage 1 of quarter m0 as one ternary i8 product (tools/ntt4096_mx_model.py): with
        // a = j1 + 32 j2 the twist psi^((2 m0 - 3) a) = s^j1 s^(32 j2), so
        //   Z''_m0[m1][32 b + j2] = zeta^((2 m1 + 1) j2) s^(32 j2) 2^(120 b (2 m0 + 1))
        //   midq[m0][j1][i] = p1^((2 brv5(i) + 1) j1) s^j1
        int8_t *zq = reinterpret_cast<int8_t *>(h.data() + az_off);
        uint64_t *mq = h.data() + az_off + 4 * 4096;
        const uint64_t zeta = gl::pow(p1, 32);
        for (int m0 = 0; m0 < 4; m0++) {
          const uint64_t s = gl::pow(psi, (uint64_t)((2 * m0 - 3 + 8192) % 8192));
          const uint64_t s32 = gl::pow(s, 32);
          for (int m1 = 0; m1 < 32; m1++)
            for (int b = 0; b < 4; b++)
              for (int j2 = 0; j2 < 32; j2++) {
                const uint64_t cb = gl::mul_pow2(1, (120 * b * (2 * m0 + 1)) % 192);
                const uint64_t x = gl::mul(gl::mul(gl::pow(zeta, (uint64_t)(2 * m1 + 1) * j2), gl::pow(s32, j2)), cb);
                const uint64_t tt = x <= 0x7F7F7F7F7F7F7F7Full ? x : x + 0xFFFFFFFFull;
                const uint64_t dd = (tt + 0x8080808080808080ull) ^ 0x8080808080808080ull;
                for (int t = 0; t < 8; t++)
                  zq[(((size_t)m0 * 8 + t) * 32 + m1) * 128 + 32 * b + j2] = (int8_t)(uint8_t)(dd >> (8 * t));
              }
          for (int j1 = 0; j1 < 32; j1++) {
            const uint64_t sj = gl::pow(s, j1);
            for (int i = 0; i < 32; i++) mq[(size_t)m0 * 1024 + j1 * 32 + i] = gl::mul(h[4 * d + j1 * 32 + i], sj);
          }
        }
      }
    }
    LF_HIP(c, hipMalloc(&t.mem, h.size() * 8));
    LF_HIP(c, hipMemcpy(t.mem, h.data(), h.size() * 8, hipMemcpyHostToDevice));
    // d = 1024 / 4096 run the register-resident 32 x 32 NTT kernels (kernels_n32.hip, kernels_n4k.hip)
    const bool n32 = extra != 0;
    t.fwd = {t.mem, t.mem + d, n32 ? t.mem + 4 * d : nullptr};
    if (d == 1024) t.fwd.az = t.mem + az_off;
    t.inv = {t.mem + 2 * d, t.mem + 3 * d, n32 ? t.mem + 4 * d + 1024 : nullptr};
    if (n32 && d == 4096) {
      t.fwd.tw4 = t.mem + 4 * d + 2048;
      t.inv.tw4 = t.fwd.tw4 + 4096;
      t.fwd.ztab = t.inv.tw4 + 4096;
      t.fwd.zq = t.mem + az_off;
      t.fwd.midq = t.mem + az_off + 4 * 4096;
    }
  }
  out = &(c->tables[d] = t);
  return LF_OK;
}

template <class T>
int grow(lf_ctx *c, T *&buf, size_t &have, size_t need) {
  if (need <= have) return LF_OK;
  if (buf) {
    LF_HIP(c, hipStreamSynchronize(c->cur));
    LF_HIP(c, hipFree(buf));
    buf = nullptr;
    have = 0;
  }
  LF_HIP(c, hipMalloc((void **)&buf, need * sizeof(T)));
  have = need;
  return LF_OK;
}
int reserve(lf_ctx *c, size_t elems) { return grow(c, c->scratch, c->scratch_elems, elems); }
// the dead-unit flags: zeroed when (re)allocated, so a padding unit that no
// decomposition writes (unit 2c + 1 when nblk L is odd) reads as live, never as
// uninitialised memory
int grow_dead(lf_ctx *c, size_t need) {
  if (need <= c->dead_elems) return LF_OK;
  LF_TRY(grow(c, c->dead, c->dead_elems, need));
  LF_HIP(c, hipMemsetAsync(c->dead, 0, need, c->cur));
  return LF_OK;
}
// a round message back through pinned memory (a pageable destination costs an extra
// staging copy per round)
int pinned(lf_ctx *c, size_t elems) {
  if (elems > c->hmsg_elems) {
    if (c->hmsg) LF_HIP(c, hipHostFree(c->hmsg));
    c->hmsg = nullptr;
    c->hmsg_elems = 0;
    LF_HIP(c, hipHostMalloc((void **)&c->hmsg, elems * 8, hipHostMallocDefault));
    c->hmsg_elems = elems;
  }
  return LF_OK;
}
int download_msg(lf_ctx *c, uint64_t *dst, const uint64_t *src, size_t elems) {
  LF_TRY(pinned(c, elems));
  LF_HIP(c, hipMemcpyAsync(c->hmsg, src, elems * 8, hipMemcpyDeviceToHost, c->cur));
  LF_HIP(c, hipStreamSynchronize(c->cur));
  memcpy(dst, c->hmsg, elems * 8);
  return LF_OK;
}

bool use_mfma(int d, size_t kappa) {
  // kappa > 32 LF_MAX_KTILES (A tiles of 32 rows): the VALU contraction (k_ajtai_phi72 / k_ajtai_nega)
  return (d == 24 || d % 16 == 0) && lfk::mfma_ktiles(kappa) <= LF_MAX_KTILES;
}

// RAII device buffer for the synchronous host API
struct DevBuf {
  uint64_t *p = nullptr;
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
};
int dev_alloc(lf_ctx *c, DevBuf &b, size_t elems) {
  LF_HIP(c, hipMalloc(&b.p, (elems ? elems : 1) * 8));
  return LF_OK;
}
int upload(lf_ctx *c, DevBuf &b, const uint64_t *h, size_t elems, int repr) {
  LF_TRY(dev_alloc(c, b, elems));
  if (elems) {
    LF_HIP(c, hipMemcpyAsync(b.p, h, elems * 8, hipMemcpyHostToDevice, c->cur));
    if (repr == LF_REPR_MONTGOMERY) LF_HIP(c, lfk::mont(b.p, elems, false, c->cur));
  }
  return LF_OK;
}
int download(lf_ctx *c, uint64_t *h, DevBuf &b, size_t elems, int repr) {
  if (!elems) return LF_OK;
  if (repr == LF_REPR_MONTGOMERY) LF_HIP(c, lfk::mont(b.p, elems, true, c->cur));
  LF_HIP(c, hipMemcpyAsync(h, b.p, elems * 8, hipMemcpyDeviceToHost, c->cur));
  return LF_OK;
}
int check_repr(lf_ctx *c, int repr) {
  if (repr != LF_REPR_CANONICAL && repr != LF_REPR_MONTGOMERY)
    return fail(c, LF_ERR_INVALID_ARG, "repr must be LF_REPR_CANONICAL or LF_REPR_MONTGOMERY");
  return LF_OK;
}

// fragment column order: units of 16 groups at one limb for the GoldiLocksDP
// gadget length L = 5 (what the fused decomposition emits), else natural order
lfk::FragGeom ajtai_geom(size_t ncols) { return lfk::frag_geom(ncols, ncols % 5 == 0 ? 5 : 1); }

size_t partial_elems(const lf_ajtai *aj, int nvec) {
  if (aj->Af) return lfk::mfma_scratch_elems(aj->geom, aj->d, aj->kappa, nvec);
  return lfk::ajtai_partial_elems(aj->kappa, aj->ncols, aj->d, nvec);
}

// cm[v] = A f_v for nvec vectors, on the matrix cores when the scheme has fragments
int ajtai_launch(lf_ctx *c, const lf_ajtai *aj, const uint64_t *const *vecs, int nvec, uint64_t *cm) {
  if (nvec < 1 || nvec > LF_MAX_VECS) return fail(c, LF_ERR_INVALID_ARG, "nvec must be in [1, 32]");
  lfk::VecPtrs vp{};
  for (int v = 0; v < nvec; v++) vp.p[v] = vecs[v];
  LF_TRY(reserve(c, partial_elems(aj, nvec)));
  if (aj->Af)
    LF_TRY(grow(c, c->frag, c->frag_elems, lfk::frag_elems(aj->geom, aj->d)));
  hipEvent_t a = nullptr, b = nullptr;
  if (c->timing) {
    LF_HIP(c, hipEventCreate(&a));
    LF_HIP(c, hipEventCreate(&b));
  }
  if (aj->Af)
    LF_HIP(c, lfk::ajtai_mfma(aj->Af, aj->kr, aj->kappa, aj->geom, aj->d, vp, nvec, false, c->frag, c->scratch, cm,
                              c->cur, a, b, nullptr, nullptr, c->zero80));
  else
    LF_HIP(c, lfk::ajtai_commit(aj->A, aj->kappa, aj->ncols, aj->d, vp, nvec, c->scratch, cm, c->cur, a, b));
  if (c->timing) c->pending.push_back({a, b, nvec});
  return LF_OK;
}

// build the MFMA fragment copy of A (scheme creation): 32-row tiles
int ajtai_prepare(lf_ctx *c, lf_ajtai *aj) {
  if (!use_mfma(aj->d, aj->kappa)) return LF_OK;
  aj->geom = ajtai_geom(aj->ncols);
  aj->geom.qperm = aj->d == 4096;  // the slot order kernels_n4k.hip produces
  const size_t n = lfk::frag_elems(aj->geom, aj->d);
  const int ktiles = lfk::mfma_ktiles(aj->kappa);
  LF_HIP(c, hipMalloc((void **)&aj->Af, n * ktiles * sizeof(uint4)));
  for (int t = 0; t < ktiles; t++) {
    lfk::VecPtrs rows{};
    const int r0 = 32 * t, nr = (int)std::min<size_t>(32, aj->kappa - r0);
    for (int i = 0; i < nr; i++) rows.p[i] = aj->A + (size_t)(r0 + i) * aj->ncols * aj->d;
    LF_HIP(c, lfk::to_frag(rows, nr, 0, aj->geom, aj->d, false, aj->Af + n * t, c->cur));
  }
  // the offset form's correction per (row, output slot)
  uint64_t *tmp = nullptr;
  LF_HIP(c, hipMalloc((void **)&aj->kr, lfk::ajtai_rowsums_elems(aj->kappa, aj->d) * sizeof(uint64_t)));
  LF_HIP(c, hipMalloc((void **)&tmp, aj->kappa * (size_t)aj->d * sizeof(uint64_t)));
  const hipError_t e = lfk::ajtai_rowsums(aj->A, aj->kappa, aj->ncols, aj->d, aj->kr, tmp, c->cur);
  const hipError_t e2 = hipStreamSynchronize(c->cur);
  (void)hipFree(tmp);
  LF_HIP(c, e);
  LF_HIP(c, e2);
  return LF_OK;
}

int drain_timing(lf_ctx *c) {
  if (c->pending.empty()) return LF_OK;
  LF_HIP(c, hipStreamSynchronize(c->cur));
  for (auto &t : c->pending) {
    float ms = 0;
    LF_HIP(c, hipEventElapsedTime(&ms, t.a, t.b));
    auto &s = c->stats[t.nvec];  // nvec < 0: a phase
    s.first += ms;
    s.second += t.count;
    (void)hipEventDestroy(t.a);
    (void)hipEventDestroy(t.b);
  }
  c->pending.clear();
  return LF_OK;
}

// The commit+fold arithmetic of fold() on device buffers. When `commit_f` is
// given (the fused device step), commit(z)'s A.f rides in the same pass over A
// as the 2(K-1) decomposition commitments (29 vectors, one read of A) and its
// result lands in `commit_cm`, which is then cm_i.
// events around one step phase (lf_ctx_phase_stats); no-op unless timing is on
struct PhaseTimer {
  lf_ctx *c;
  int phase;
  hipEvent_t a = nullptr;
  PhaseTimer(lf_ctx *ctx, int ph) : c(ctx), phase(ph) {
    if (c->timing && hipEventCreate(&a) == hipSuccess) (void)hipEventRecord(a, c->cur);
  }
  ~PhaseTimer() {
    hipEvent_t b = nullptr;
    if (a && hipEventCreate(&b) == hipSuccess) {
      (void)hipEventRecord(b, c->cur);
      c->pending.push_back({a, b, -1 - phase});
    }
  }
};

// The commit+fold arithmetic of fold() on device buffers, in two halves so a
// column-sharded step can all-reduce the commitments between them:
//  fold_commit: decompose_witness of both sides (decomposition.rs:162-167) and
//    the 2(K-1) commitments of commit_witnesses (:178-201), plus -- when
//    `commit_f` is given (the device step) -- commit(z)'s A.f in the same pass
//    over A (29 vectors, one read of A). Result v goes to dst[v]: commit(z)'s
//    cm first, then y_s[k], s = 0, 1, k = 1 .. K-1.
//  fold_finish: y_0 = cm - sum b^k y_k of both sides, cm_0 = sum rho_i y_i,
//    f_0 = sum rho_i f_i (folding.rs:258-268, folding/utils.rs:470-476) and
//    Witness::from_f(f_0) (arith.rs:299-313).
// d = 4096 with b_small = 2: the register-transform decomposition (kernels_n4k.hip),
// all sides in one launch; the packed coefficients go to the smg scratch
bool n4k_ok(const Tables *t, int d, int lbs, int K) { return d == 4096 && lbs == 1 && K <= 15 && t->fwd.tw4; }
int decompose_n4k_sides(lf_ctx *c, const Tables *t, int nside, const uint64_t *const *fc, uint64_t *const *fck,
                        uint64_t *const *fk, uint64_t *const *wk, size_t N, int lb, int L, int K,
                        uint4 *frag = nullptr, int nch = 0, const int *row0 = nullptr, const int *row_p0 = nullptr,
                        uint64_t *const *planes = nullptr, uint8_t *dead = nullptr) {
  // packed digits: one u64 per 4 coefficients, or (fused) one byte per 4 coefficients and
  // plane -- into the caller's planes when given (the packed step's decomposed witnesses)
  const bool own = !(frag && planes && planes[0]);
  if (own) LF_TRY(grow(c, c->smg, c->smg_elems, (size_t)nside * N * (frag ? (size_t)K * 256 : 2048)));
  c->smg_sides_n = 0;
  lfk::FusedSides sd{};
  sd.nside = nside;
  sd.dead = frag ? dead : nullptr;
  for (int s = 0; s < nside; s++) {
    sd.f_coeff[s] = fc[s];
    sd.f_coeff_k[s] = fck[s];
    sd.f_k[s] = fk[s];
    sd.w_ccs_k[s] = wk[s];
    sd.row0[s] = row0 ? row0[s] : 0;
    sd.row_p0[s] = row_p0 ? row_p0[s] : -1;
    if (!own) sd.smg[s] = reinterpret_cast<uint32_t *>(planes[s]);
  }
  LF_HIP(c, lfk::decompose_n4k(sd, N, lb, L, K, own ? reinterpret_cast<uint64_t *>(c->smg) : nullptr, t->fwd, c->d_err,
                               c->sink, c->ncu, c->cur, frag, nch));
  return LF_OK;
}

int fold_nvec(const lf_params *pr, bool commit_f) { return (commit_f ? 1 : 0) + 2 * (pr->K - 1); }

// a fused step's contraction left for lf_dev_fold_step_batch to launch with other steps'
struct Deferred {
  const uint4 *Ff = nullptr;
  uint64_t *partial = nullptr;
  lfk::OutPtrs dst{};
  lfk::DeadUnits dead{};
  const uint4 *zero80 = nullptr;
  int nvec = 0;
  bool set = false;
};

int fold_commit(lf_ctx *c, const lf_ajtai *aj, const lf_params *pr, int lb, int lbs, size_t W,
                const lf_fold_step_bufs *b, const uint64_t *wi_f_coeff, const uint64_t *commit_f,
                const lfk::OutPtrs &dst, Deferred *defer = nullptr, const uint32_t *prepacked1 = nullptr) {
  // prepacked1: the buffer into which step_commit's from_w_ccs has just written
  // side 1's sign|magnitude words (fused d = 1024 path), or null. It is an
  // argument, not context state, so a failed step cannot leave it set for a
  // later call.
  const int d = pr->d, L = pr->L, K = pr->K;
  const size_t N = W * (size_t)L, kappa = aj->kappa;
  const int extra = commit_f ? 1 : 0, nvec = fold_nvec(pr, commit_f != nullptr);
  if (2 * K > LF_MAX_VECS || nvec > LF_MAX_VECS) return fail(c, LF_ERR_INVALID_ARG, "2K must be <= 32");
  if (aj->ncols != N) return fail(c, LF_ERR_WRONG_WITNESS_LENGTH, "witness length != Ajtai width");
  Tables *t;
  LF_TRY(get_tables(c, d, t));
  const uint64_t *fc_side[2] = {b->acc_f_coeff, wi_f_coeff};
  const size_t kd = kappa * (size_t)d;
  // fused path (d = 1024, b_small = 2, fragment order grouped by this L): the
  // decomposition writes its digit planes straight into the MFMA operand buffer
  const bool fused = aj->Af && aj->geom.Lp == L && d == 1024 && lbs == 1 && K <= 15 && t->fwd.mid;
  // Phi_72 (d = 24): each side's decomposition writes its planes as operand rows (kernels.hip)
  const bool fused24 = aj->Af && aj->geom.Lp == L && d == 24 && L <= 5;
  // d = 4096 (kernels_n4k.hip): the same, with the quarter-major operand slots
  const bool fused4k = aj->Af && aj->geom.Lp == L && aj->geom.qperm && n4k_ok(t, d, lbs, K);
  // without f_k buffers the planes exist only as operand rows (planes 1..K-1
  // of each side as usual, plane 0 in rows extra + 2(K-1) + s) and fold_finish
  // reads f_0's inputs from there (k_fold_frag)
  const bool no_fk = !b->fk[0] && !b->fk[1];
  c->fold_from_frag = false;
  c->masks24_n = 0;
  c->frag_fallback = false;
  c->dead_units = lfk::DeadUnits{};
  c->fold_rows.dead = lfk::DeadUnits{};
  if (b->planes[0] || b->planes[1]) {
    if (!(fused24 || fused || fused4k) || lbs != 1 || !b->planes[0] || !b->planes[1])
      return fail(c, LF_ERR_INVALID_ARG,
                  "packed planes: d = 24 or the fused d = 1024 / 4096 paths, b_small = 2, both sides");
  }
  // X^1024 + 1 without f_k / f_coeff_k: the planes stay packed (the fused
  // decomposition's sign|magnitude words), f_0 comes from the coefficient-form
  // fold, whose fallback for a rho that is not short reads the operand rows
  const bool packed1024 = no_fk && fused && !b->fk_coeff[0] && !b->fk_coeff[1];
  // Phi_72 without f_k / f_coeff_k: the decomposed witnesses stay packed (digit masks)
  const bool packed24 = no_fk && fused24;
  if (packed24) {
    if (lbs != 1) return fail(c, LF_ERR_INVALID_ARG, "packed Phi_72 planes need b_small = 2");
    if (b->fk_coeff[0] || b->fk_coeff[1])
      return fail(c, LF_ERR_INVALID_ARG, "Phi_72: f_k and f_coeff_k are both given or both NULL");
  } else if (no_fk) {
    if (!fused && !fused4k)
      return fail(c, LF_ERR_INVALID_ARG, "f_k buffers may be omitted only on the fused X^1024+1 / X^4096+1 paths");
    if (fused4k && (b->fk_coeff[0] || b->fk_coeff[1]) && !(b->fk_coeff[0] && b->fk_coeff[1]))
      return fail(c, LF_ERR_INVALID_ARG, "f_coeff_k: both sides or neither");
    if (fused && !packed1024 && (!b->fk_coeff[0] || !b->fk_coeff[1]))
      return fail(c, LF_ERR_INVALID_ARG, "f_coeff_k: both sides or neither");
    if (extra + 2 * (K - 1) + 2 > LF_MAX_VECS) return fail(c, LF_ERR_INVALID_ARG, "too many operand rows");
    lfk::FoldRows &fr = c->fold_rows;
    fr.n = 2 * K;
    for (int s2 = 0; s2 < 2; s2++)
      for (int k = 0; k < K; k++) {
        fr.row[s2 * K + k] = k > 0 ? extra + s2 * (K - 1) + k - 1 : extra + 2 * (K - 1) + s2;
        fr.rho[s2 * K + k] = s2 * K + k;
      }
    // packed planes fold in coefficient form with the rows as the fallback
    c->fold_from_frag = !packed1024;
    c->frag_fallback = packed1024;
  } else if (!b->fk[0] || !b->fk[1]) {
    return fail(c, LF_ERR_INVALID_ARG, "f_k: both sides or neither");
  }
  if (fused || fused24 || fused4k) {
    LF_TRY(grow(c, c->frag, c->frag_elems, lfk::frag_elems(aj->geom, d)));
    if (fused4k) {
      // without f_k, plane 0 of each side gets an operand row too and f_0 is folded
      // from the rows (fold_finish: k_fold_frag over the quarter-major slots)
      const int row0[2] = {extra, extra + K - 1};
      const int row_p0[2] = {no_fk ? extra + 2 * (K - 1) : -1, no_fk ? extra + 2 * (K - 1) + 1 : -1};
      // dead units (operand rows left unwritten where a unit's plane is zero), as at d = 1024
      LF_TRY(grow_dead(c, (size_t)aj->geom.nch * 64));
      uint32_t rows = 0;
      for (int s = 0; s < 2; s++) {
        for (int k = 1; k < K; k++) rows |= 1u << (row0[s] + k - 1);
        if (row_p0[s] >= 0) rows |= 1u << row_p0[s];
      }
      c->dead_units.flags = c->dead;
      c->dead_units.rows = rows;
      c->fold_rows.dead = c->dead_units;
      PhaseTimer pt(c, LF_PHASE_DECOMPOSE);  // both sides in one launch
      LF_TRY(decompose_n4k_sides(c, t, 2, fc_side, b->fk_coeff, b->fk, b->wk, N, lb, L, K, c->frag, aj->geom.nch,
                                 row0, row_p0, b->planes, c->dead));
    } else if (fused) {
      // the packed words go straight into the caller's planes when given
      if (!b->planes[0]) LF_TRY(grow(c, c->smg, c->smg_elems, 2 * N * 512));
      lfk::FusedSides sd{};
      sd.nside = 2;
      // dead units: the planes' rows are written only where a unit's plane is nonzero
      LF_TRY(grow_dead(c, (size_t)aj->geom.nch * 64));
      sd.dead = c->dead;
      uint32_t rows = 0;
      for (int s = 0; s < 2; s++) {
        sd.f_coeff[s] = fc_side[s];
        sd.f_coeff_k[s] = b->fk_coeff[s];
        sd.f_k[s] = b->fk[s];
        sd.w_ccs_k[s] = b->wk[s];
        sd.row0[s] = extra + s * (K - 1);
        sd.row_p0[s] = no_fk ? extra + 2 * (K - 1) + s : -1;
        sd.smg[s] = b->planes[0] ? reinterpret_cast<uint32_t *>(b->planes[s]) : c->smg + (size_t)s * N * 512;
        c->smg_side[s] = sd.smg[s];
        for (int k = 1; k < K; k++) rows |= 1u << (sd.row0[s] + k - 1);
        if (sd.row_p0[s] >= 0) rows |= 1u << sd.row_p0[s];
      }
      c->dead_units.flags = c->dead;
      c->dead_units.rows = rows;
      c->fold_rows.dead = c->dead_units;
      // side 1's words, when step_commit's from_w_ccs wrote them into this very buffer
      sd.prepacked = prepacked1 && prepacked1 == sd.smg[1] && wi_f_coeff == b->f_coeff ? 2 : 0;
      PhaseTimer pt(c, LF_PHASE_DECOMPOSE);  // both sides in one launch
      LF_HIP(c, lfk::decompose_fused(sd, N, lb, L, K, t->fwd, c->frag, aj->geom.nch, c->d_err,
                                     c->sink, c->ncu, c->cur));
      c->smg_sides_n = N;  // fold_finish's coefficient-form fold reads the digits from here
    } else {
      lfk::FusedSides sd{};
      sd.nside = 2;
      // b_small = 2: the digit masks for fold_finish's coefficient-form fold,
      // into the caller's planes if given, else the context's scratch
      const bool want_masks = lbs == 1;
      if (want_masks && !b->planes[0]) LF_TRY(grow(c, c->fkeys, c->fkeys_elems, 2 * 2 * (size_t)K * N));
      LF_TRY(grow(c, c->smg, c->smg_elems, 2 * N * 12));  // the coefficients as 16-bit sign|magnitude
      // dead units (the wave-local b_small = 2 kernel flags the zero planes' rows)
      LF_TRY(grow_dead(c, (size_t)aj->geom.nch * 64));
      sd.dead = lbs == 1 ? c->dead : nullptr;
      uint32_t rows = 0;
      for (int s = 0; s < 2; s++) {
        sd.f_coeff[s] = fc_side[s];
        sd.f_coeff_k[s] = b->fk_coeff[s];
        sd.f_k[s] = b->fk[s];
        sd.w_ccs_k[s] = b->wk[s];
        sd.row0[s] = extra + s * (K - 1);
        for (int k = 1; k < K; k++) rows |= 1u << (sd.row0[s] + k - 1);
        sd.smg[s] = c->smg + (size_t)s * N * 12;
        if (want_masks)
          sd.masks[s] = b->planes[s] ? reinterpret_cast<uint2 *>(b->planes[s])
                                     : reinterpret_cast<uint2 *>(c->fkeys) + (size_t)s * K * N;
        c->masks24[s] = sd.masks[s];
      }
      PhaseTimer pt(c, LF_PHASE_DECOMPOSE);  // both sides in one launch
      bool masks = false, dead = false;
      LF_HIP(c, lfk::decompose_phi72_sides(sd, N, lb, L, lbs, K, c->d_err, c->frag, aj->geom.nch, c->cur, &masks,
                                           &dead));
      if (packed24 && !masks) return fail(c, LF_ERR_INVALID_ARG, "packed Phi_72 planes need the wave-local decomposition");
      c->masks24_n = masks ? N : 0;
      if (dead) {  // the wave-local kernel ran: its flags are this step's
        c->dead_units.flags = c->dead;
        c->dead_units.rows = rows;
      }
    }
    lfk::VecPtrs vp{};
    if (commit_f) {
      PhaseTimer pt(c, LF_PHASE_TO_FRAG);
      vp.p[0] = commit_f;
      LF_HIP(c, lfk::to_frag(vp, 1, 0, aj->geom, d, true, c->frag, c->cur));
    }
    LF_TRY(reserve(c, partial_elems(aj, nvec)));
    if (defer) {  // the caller contracts this step together with others (one pass over A)
      defer->Ff = c->frag;
      defer->partial = c->scratch;
      defer->dst = dst;
      defer->dead = c->dead_units;
      defer->zero80 = c->zero80;
      defer->nvec = nvec;
      defer->set = true;
      return LF_OK;
    }
    hipEvent_t ea = nullptr, eb = nullptr;
    if (c->timing) {
      LF_HIP(c, hipEventCreate(&ea));
      LF_HIP(c, hipEventCreate(&eb));
    }
    LF_HIP(c, lfk::ajtai_mfma(aj->Af, aj->kr, kappa, aj->geom, d, vp, nvec, true, c->frag, c->scratch, nullptr, c->cur,
                              ea, eb, &dst, &c->dead_units, c->zero80));
    if (c->timing) c->pending.push_back({ea, eb, nvec});
    return LF_OK;
  }
  if (n4k_ok(t, d, lbs, K)) {
    PhaseTimer pt(c, LF_PHASE_DECOMPOSE);  // both sides in one launch
    LF_TRY(decompose_n4k_sides(c, t, 2, fc_side, b->fk_coeff, b->fk, b->wk, N, lb, L, K));
  } else {
    for (int s = 0; s < 2; s++) {
      PhaseTimer pt(c, LF_PHASE_DECOMPOSE);
      LF_HIP(c, lfk::decompose_witness(fc_side[s], N, d, lb, L, lbs, K, b->fk_coeff[s], b->fk[s], b->wk[s], t->fwd,
                                       c->d_err, c->cur));
    }
  }
  // commit_witnesses: 2(K-1) commitments sharing one pass over A (decomposition.rs:185-188)
  std::vector<const uint64_t *> vecs;
  if (commit_f) vecs.push_back(commit_f);
  for (int s = 0; s < 2; s++)
    for (int k = 1; k < K; k++) vecs.push_back(b->fk[s] + (size_t)k * N * d);
  LF_TRY(grow(c, c->ybuf, c->ybuf_elems, (size_t)nvec * kd));
  LF_TRY(ajtai_launch(c, aj, vecs.data(), nvec, c->ybuf));
  for (int v = 0; v < nvec; v++)
    if (dst.p[v] != c->ybuf + v * kd)
      LF_HIP(c, hipMemcpyAsync(dst.p[v], c->ybuf + v * kd, kd * 8, hipMemcpyDeviceToDevice, c->cur));
  return LF_OK;
}

// destinations of fold_commit's results in the step buffers
lfk::OutPtrs fold_dst(const lf_params *pr, const lf_fold_step_bufs *b, size_t kd, uint64_t *commit_cm) {
  lfk::OutPtrs dst{};
  const int extra = commit_cm ? 1 : 0;
  if (commit_cm) dst.p[0] = commit_cm;
  for (int s = 0; s < 2; s++)
    for (int k = 1; k < pr->K; k++) dst.p[extra + s * (pr->K - 1) + k - 1] = b->y[s] + (size_t)k * kd;
  return dst;
}


int fold_finish(lf_ctx *c, const lf_ajtai *aj, const lf_params *pr, int lb, int lbs, size_t W,
                const lf_fold_step_bufs *b, const uint64_t *cm_i) {
  const int d = pr->d, L = pr->L, K = pr->K;
  const size_t N = W * (size_t)L, kappa = aj->kappa;
  Tables *t;
  LF_TRY(get_tables(c, d, t));
  // y_0 of both sides and cm_0 = sum rho_i y_i in one pass (the y_s[k >= 1] are in place)
  LF_HIP(c, lfk::y0_cm0(b->acc_cm, cm_i, b->y[0], b->y[1], b->rho, kappa, d, lbs, K, b->cm0, c->cur));
  // X^1024 + 1 after the fused decomposition: f_0 in coefficient form on the
  // matrix cores from the digits (fold_coeff.hip), then f_0 and w_ccs by one
  // forward transform per element. If a rho is not short the device flag `bad`
  // turns those kernels off and the NTT-form fold and from_f on.
  if (c->smg_sides_n == N && N && d == 1024 && lbs == 1 && K <= 15 && !c->fold_from_frag && t->fwd.mid &&
      t->inv.mid) {
    const int nw = 2 * K;
    const size_t tab_u64 = ((size_t)nw * lfk::FOLD_RT + 7) / 8, aux = (size_t)nw * 1024 + tab_u64 + 1;
    // the digit keys [2 N][K][64] u32, then each column's plane mask [2 N] u32
    LF_TRY(grow(c, c->fkeys, c->fkeys_elems, 2 * N * (size_t)K * 64 + 2 * N));
    uint32_t *nz = c->fkeys + 2 * N * (size_t)K * 64;
    LF_TRY(grow(c, c->faux, c->faux_elems, aux));
    uint64_t *rc = c->faux;
    uint8_t *tab = reinterpret_cast<uint8_t *>(c->faux + (size_t)nw * 1024);
    int *bad = reinterpret_cast<int *>(c->faux + aux - 1);
    {
      PhaseTimer pt(c, LF_PHASE_FOLD);
      for (int s = 0; s < 2; s++)
        LF_HIP(c, lfk::fold_keys(c->smg_side[s], N, K, c->fkeys + (size_t)s * N * K * 64, c->cur, nz + (size_t)s * N));
      LF_HIP(c, lfk::fold_rho_tables(b->rho, nw, rc, tab, bad, t->inv, c->d_sync, c->cur));
      const int ks_n = lfk::fold_coeff_splits(N, K, c->ncu);
      if (ks_n > 1) LF_TRY(grow(c, c->fpart, c->fpart_elems, (size_t)ks_n * N * 1024));
      if (c->frag_fallback) {
        // packed planes: the fallback (f_0 in NTT form from the operand rows) runs
        // inside the same launch when the flag is set (no separate gated launch)
        lfk::FoldFallback fb{};
        fb.frag = c->frag;
        fb.nch = aj->geom.nch;
        fb.Lp = aj->geom.Lp;
        fb.Wp = aj->geom.Wp;
        fb.fr = c->fold_rows;
        fb.rho = b->rho;
        fb.f0 = b->f0;
        LF_HIP(c, lfk::fold_coeff(c->fkeys, tab, bad, N, K, b->f0_coeff, c->ncu, c->cur,
                                  ks_n > 1 ? c->fpart : nullptr, &fb, L, nz));
      } else {
        LF_HIP(c, lfk::fold_coeff(c->fkeys, tab, bad, N, K, b->f0_coeff, c->ncu, c->cur,
                                  ks_n > 1 ? c->fpart : nullptr, nullptr, L, nz));
        lfk::VecPtrs fx{};
        for (int s = 0; s < 2; s++)
          for (int k = 0; k < K; k++) fx.p[s * K + k] = b->fk[s] + (size_t)k * N * d;
        LF_HIP(c, lfk::fold(b->rho, fx, nw, N, d, b->f0, c->cur, bad));
      }
    }
    // f_0 and w_ccs from f_0's coefficients, or (flag set) Witness::from_f of the
    // NTT-form f_0, in one launch
    PhaseTimer pt(c, LF_PHASE_FROM_F);
    LF_HIP(c, lfk::from_fcoeff_n32(b->f0_coeff, W, lb, L, b->f0, b->w_ccs0, t->fwd, bad, c->cur, &t->inv));
    return LF_OK;
  }
  // Phi_72 after the wave-local decomposition: f_0 in coefficient form from its
  // digit masks, then f_0 = CRT and w_ccs_0 (kernels.hip k_fold_coeff_phi72); a
  // rho that is not short raises `bad`, which turns that kernel off and the
  // NTT-form fold and Witness::from_f on
  if (c->masks24_n == N && N && d == 24 && lbs == 1 && !c->fold_from_frag) {
    const uint2 *m0 = c->masks24[0], *m1 = c->masks24[1];
    if (!b->fk[0]) {
      // the planes are packed: the fallback for a rho that is not short folds
      // f_0 from the masks in Z_p, then Witness::from_f
      const int nw = 2 * K;
      LF_TRY(grow(c, c->faux, c->faux_elems, (size_t)nw * 13 + 1));
      uint32_t *rc = reinterpret_cast<uint32_t *>(c->faux);
      int *bad = reinterpret_cast<int *>(c->faux + (size_t)nw * 13);
      {
        PhaseTimer pt(c, LF_PHASE_FOLD);
        LF_HIP(c, lfk::fold_phi72_rho(b->rho, nw, rc, bad, c->cur));
        LF_HIP(c, lfk::fold_phi72_coeff(m0, m1, rc, bad, N, K, L, lb, b->f0_coeff, b->f0, b->w_ccs0, c->cur));
        LF_HIP(c, lfk::fold_phi72_masks(m0, m1, b->rho, K, N, b->f0, bad, c->cur));
      }
      PhaseTimer pt(c, LF_PHASE_FROM_F);
      LF_HIP(c, lfk::from_f(b->f0, N, d, lb, L, b->f0_coeff, b->w_ccs0, t->inv, c->cur, bad));
      return LF_OK;
    }
    const int nw = 2 * K;
    LF_TRY(grow(c, c->faux, c->faux_elems, (size_t)nw * 13 + 1));
    uint32_t *rc = reinterpret_cast<uint32_t *>(c->faux);  // 25 packed words per witness
    int *bad = reinterpret_cast<int *>(c->faux + (size_t)nw * 13);
    {
      PhaseTimer pt(c, LF_PHASE_FOLD);
      LF_HIP(c, lfk::fold_phi72_rho(b->rho, nw, rc, bad, c->cur));
      LF_HIP(c, lfk::fold_phi72_coeff(m0, m1, rc, bad, N, K, L, lb, b->f0_coeff, b->f0, b->w_ccs0, c->cur));
      lfk::VecPtrs fx{};
      for (int s = 0; s < 2; s++)
        for (int k = 0; k < K; k++) fx.p[s * K + k] = b->fk[s] + (size_t)k * N * d;
      LF_HIP(c, lfk::fold(b->rho, fx, nw, N, d, b->f0, c->cur, bad));
    }
    PhaseTimer pt(c, LF_PHASE_FROM_F);
    LF_HIP(c, lfk::from_f(b->f0, N, d, lb, L, b->f0_coeff, b->w_ccs0, t->inv, c->cur, bad));
    return LF_OK;
  }
  if (c->fold_from_frag) {  // the planes are only in the operand rows (fold_commit)
    PhaseTimer pt(c, LF_PHASE_FOLD);
    LF_HIP(c, lfk::fold_frag(c->frag, aj->geom, c->fold_rows, b->rho, d, N, b->f0, c->cur));
  } else {
    lfk::VecPtrs fx{};
    for (int s = 0; s < 2; s++)
      for (int k = 0; k < K; k++) fx.p[s * K + k] = b->fk[s] + (size_t)k * N * d;
    PhaseTimer pt(c, LF_PHASE_FOLD);
    LF_HIP(c, lfk::fold(b->rho, fx, 2 * K, N, d, b->f0, c->cur));
  }
  PhaseTimer pt(c, LF_PHASE_FROM_F);
  LF_HIP(c, lfk::from_f(b->f0, N, d, lb, L, b->f0_coeff, b->w_ccs0, t->inv, c->cur));
  return LF_OK;
}

// ---------------------------------------------------------------- RCCL (resolved at run time)
// The library does not link RCCL: the entry points are looked up in the RCCL
// already loaded into the process (torch's, whose communicators a caller may
// hand over through lf_comm_wrap) or else in librccl.so.1.
struct Rccl {
  bool ok = false;
  std::string err;
  ncclResult_t (*getUniqueId)(ncclUniqueId *) = nullptr;
  ncclResult_t (*commInitRank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*commDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*commCount)(const ncclComm_t, int *) = nullptr;
  ncclResult_t (*commUserRank)(const ncclComm_t, int *) = nullptr;
  ncclResult_t (*allReduce)(const void *, void *, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                            hipStream_t) = nullptr;
  const char *(*errorString)(ncclResult_t) = nullptr;
};
const Rccl &rccl() {
  static const Rccl r = [] {
    Rccl x;
    void *h = nullptr;
    for (const char *name : {"librccl.so.1", "librccl.so"})
      if (!h) h = dlopen(name, RTLD_NOW | RTLD_NOLOAD);
    for (const char *name : {"librccl.so.1", "librccl.so"})
      if (!h) h = dlopen(name, RTLD_NOW | RTLD_GLOBAL);
    if (!h) {
      x.err = "RCCL (librccl.so.1) not found";
      return x;
    }
    x.getUniqueId = (decltype(x.getUniqueId))dlsym(h, "ncclGetUniqueId");
    x.commInitRank = (decltype(x.commInitRank))dlsym(h, "ncclCommInitRank");
    x.commDestroy = (decltype(x.commDestroy))dlsym(h, "ncclCommDestroy");
    x.commCount = (decltype(x.commCount))dlsym(h, "ncclCommCount");
    x.commUserRank = (decltype(x.commUserRank))dlsym(h, "ncclCommUserRank");
    x.allReduce = (decltype(x.allReduce))dlsym(h, "ncclAllReduce");
    x.errorString = (decltype(x.errorString))dlsym(h, "ncclGetErrorString");
    x.ok = x.getUniqueId && x.commInitRank && x.commDestroy && x.commCount && x.commUserRank && x.allReduce &&
           x.errorString;
    if (!x.ok) x.err = "RCCL entry points missing";
    return x;
  }();
  return r;
}
#define LF_NCCL(ctx, call)                                                                       \
  do {                                                                                          \
    ncclResult_t r_ = (call);                                                                    \
    if (r_ != ncclSuccess)                                                                       \
      return fail((ctx), LF_ERR_COMM, std::string(#call) + ": " + rccl().errorString(r_));       \
  } while (0)

// x <- sum over the communicator's ranks of x, mod p, on the context stream:
// RCCL's integer sum is mod 2^64, so the vector travels as 32-bit limbs
// (exact for < 2^32 ranks) and is folded back into the field afterwards
int allreduce_modp(lf_ctx *c, lf_comm *cm, uint64_t *x, size_t n) {
  if (!cm || !cm->comm || !n) return LF_OK;  // one rank without a communicator: the sum is x
  if (!rccl().ok) return fail(c, LF_ERR_COMM, rccl().err);
  LF_TRY(grow(c, c->limb, c->limb_elems, 2 * n));
  LF_HIP(c, lfk::limb_split(x, n, c->limb, c->limb + n, c->cur));
  LF_NCCL(c, rccl().allReduce(c->limb, c->limb, 2 * n, ncclUint64, ncclSum, cm->comm, c->cur));
  LF_HIP(c, lfk::limb_join(c->limb, c->limb + n, n, x, c->cur));
  return LF_OK;
}

}  // namespace

extern "C" {

lf_params lf_goldilocks_dp(int d) {
  lf_params p;
  p.d = d;
  p.B = 1ull << 15;
  p.L = 5;
  p.b_small = 2;
  p.K = 15;
  return p;
}

const char *lf_status_string(int s) {
  switch (s) {
    case LF_OK: return "ok";
    case LF_ERR_INVALID_ARG: return "invalid argument";
    case LF_ERR_UNSUPPORTED_RING: return "unsupported ring degree";
    case LF_ERR_WRONG_WITNESS_LENGTH: return "wrong length of the witness";
    case LF_ERR_WRONG_COMMITMENT_LENGTH: return "wrong length of the commitment";
    case LF_ERR_WRONG_AJTAI_DIMENSIONS: return "Ajtai matrix has wrong dimensions";
    case LF_ERR_DECOMPOSITION_OVERFLOW: return "balanced decomposition ran out of digits";
    case LF_ERR_INCORRECT_LENGTH: return "incorrect length";
    case LF_ERR_CHALLENGE_BYTES: return "wrong number of challenge bytes";
    case LF_ERR_DEVICE: return "HIP device error";
    case LF_ERR_OUT_OF_MEMORY: return "out of device memory";
    case LF_ERR_COMM: return "RCCL communicator error";
    case LF_ERR_VERIFICATION: return "the folding proof does not verify";
    case LF_ERR_UNSUPPORTED_CCS: return "unsupported CCS structure";
  }
  return "unknown status";
}

int lf_ctx_create(int device, lf_ctx **out) {
  if (!out) return LF_ERR_INVALID_ARG;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0 || device < 0 || device >= n) {
    fprintf(stderr, "latticeum_amd: no HIP device %d available (count=%d)\n", device, n);
    return LF_ERR_DEVICE;
  }
  auto c = std::make_unique<lf_ctx>();
  c->device = device;
  DevGuard g(device);
  if (hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking) != hipSuccess) return LF_ERR_DEVICE;
  c->cur = c->own;
  if (hipMalloc(&c->d_err, sizeof(int)) != hipSuccess) return LF_ERR_OUT_OF_MEMORY;
  if (hipMemset(c->d_err, 0, sizeof(int)) != hipSuccess) return LF_ERR_DEVICE;
  if (hipMalloc(&c->d_sync, 2 * sizeof(int)) != hipSuccess) return LF_ERR_OUT_OF_MEMORY;
  if (hipMemset(c->d_sync, 0, 2 * sizeof(int)) != hipSuccess) return LF_ERR_DEVICE;
  if (hipMalloc(&c->sink, 4096 * sizeof(uint64_t)) != hipSuccess) return LF_ERR_OUT_OF_MEMORY;
  if (hipMalloc(&c->zero80, 32 * sizeof(uint4)) != hipSuccess) return LF_ERR_OUT_OF_MEMORY;
  if (hipMemset(c->zero80, 0x80, 32 * sizeof(uint4)) != hipSuccess) return LF_ERR_DEVICE;
  if (hipDeviceGetAttribute(&c->ncu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || c->ncu < 1)
    return LF_ERR_DEVICE;
  *out = c.release();
  return LF_OK;
}

void lf_ctx_destroy(lf_ctx *c) {
  if (!c) return;
  DevGuard g(c);
  (void)hipStreamSynchronize(c->cur);
  // a batched contraction this context led on the caller's contract stream reads its buffers
  if (c->contract) (void)hipStreamSynchronize(c->contract);
  c->contract = nullptr;
  for (auto &t : c->pending) {
    (void)hipEventDestroy(t.a);
    (void)hipEventDestroy(t.b);
  }
  for (auto &kv : c->tables)
    if (kv.second.mem) (void)hipFree(kv.second.mem);
  if (c->scratch) (void)hipFree(c->scratch);
  if (c->ybuf) (void)hipFree(c->ybuf);
  if (c->frag) (void)hipFree(c->frag);
  if (c->smg) (void)hipFree(c->smg);
  if (c->fkeys) (void)hipFree(c->fkeys);
  if (c->faux) (void)hipFree(c->faux);
  if (c->fpart) (void)hipFree(c->fpart);
  if (c->sink) (void)hipFree(c->sink);
  if (c->dead) (void)hipFree(c->dead);
  if (c->zero80) (void)hipFree(c->zero80);
  if (c->stage) (void)hipFree(c->stage);
  if (c->limb) (void)hipFree(c->limb);
  if (c->tmp) (void)hipFree(c->tmp);
  if (c->sc) (void)hipFree(c->sc);
  if (c->ptrs) (void)hipFree(c->ptrs);
  if (c->sel) (void)hipFree(c->sel);
  if (c->hmsg) (void)hipHostFree(c->hmsg);
  if (c->join) (void)hipEventDestroy(c->join);
  if (c->cjoin) (void)hipEventDestroy(c->cjoin);
  if (c->d_err) (void)hipFree(c->d_err);
  if (c->d_sync) (void)hipFree(c->d_sync);
  if (c->own) (void)hipStreamDestroy(c->own);
  delete c;
}

const char *lf_ctx_last_error(const lf_ctx *c) { return c ? c->last_error.c_str() : ""; }
void lf_ctx_set_error(lf_ctx *c, const char *msg) {
  if (c) c->last_error = msg ? msg : "";
}

size_t lf_witness_split_w(void) { return lfk::witness_split_w(); }

int lf_ctx_device(const lf_ctx *c) { return c ? c->device : -1; }

int lf_ctx_set_stream(lf_ctx *c, void *s) {
  if (!c) return LF_ERR_INVALID_ARG;
  c->cur = (hipStream_t)s;  // NULL = the HIP default (null) stream, e.g. torch's default stream
  return LF_OK;
}
void *lf_ctx_get_stream(const lf_ctx *c) { return c ? (void *)c->cur : nullptr; }

int lf_stream_create_cu_mask(int device, const uint32_t *mask, int nwords, void **stream) {
  if (!mask || nwords < 1 || !stream) return LF_ERR_INVALID_ARG;
  *stream = nullptr;
  DevGuard g(device);
  hipStream_t s = nullptr;
  if (hipExtStreamCreateWithCUMask(&s, (uint32_t)nwords, mask) != hipSuccess) return LF_ERR_DEVICE;
  *stream = (void *)s;
  return LF_OK;
}
int lf_ctx_set_contract_stream(lf_ctx *c, void *s) {
  if (!c) return LF_ERR_INVALID_ARG;
  if (s) {  // the caller keeps ownership; it must be a stream of this context's device
    hipDevice_t dev = -1;
    if (hipStreamGetDevice((hipStream_t)s, &dev) != hipSuccess)
      return fail(c, LF_ERR_INVALID_ARG, "contract stream: not a valid stream");
    if (dev != c->device) return fail(c, LF_ERR_INVALID_ARG, "contract stream is on another device");
  }
  c->contract = (hipStream_t)s;
  return LF_OK;
}
int lf_ctx_set_cu_count(lf_ctx *c, int ncu) {
  if (!c || ncu < 1) return LF_ERR_INVALID_ARG;
  c->ncu = ncu;
  return LF_OK;
}
int lf_stream_destroy(void *stream) {
  if (!stream) return LF_ERR_INVALID_ARG;
  return hipStreamDestroy((hipStream_t)stream) == hipSuccess ? LF_OK : LF_ERR_DEVICE;
}

int lf_ctx_sync(lf_ctx *c) {
  DevGuard g(c);
  if (!c) return LF_ERR_INVALID_ARG;
  LF_HIP(c, hipStreamSynchronize(c->cur));
  int e = 0;
  LF_HIP(c, hipMemcpy(&e, c->d_err, sizeof(int), hipMemcpyDeviceToHost));
  if (e) {
    LF_HIP(c, hipMemset(c->d_err, 0, sizeof(int)));
    return fail(c, LF_ERR_DECOMPOSITION_OVERFLOW, "a coefficient needed more digits than padding_size");
  }
  return LF_OK;
}

int lf_ctx_reserve(lf_ctx *c, size_t kappa, size_t ncols, int d, int nvec) {
  DevGuard g(c);
  if (!c || !ring_ok(d) || nvec < 1 || nvec > LF_MAX_VECS) return LF_ERR_INVALID_ARG;
  Tables *t;
  LF_TRY(get_tables(c, d, t));
  lf_ajtai probe;
  probe.kappa = kappa;
  probe.ncols = ncols;
  probe.d = d;
  if (use_mfma(d, kappa)) {
    probe.Af = reinterpret_cast<uint4 *>(1);  // sizing only
    probe.geom = ajtai_geom(ncols);
    probe.geom.qperm = d == 4096;
    LF_TRY(grow(c, c->frag, c->frag_elems, lfk::frag_elems(probe.geom, d)));
  }
  LF_TRY(reserve(c, partial_elems(&probe, nvec)));
  return grow(c, c->ybuf, c->ybuf_elems, (size_t)nvec * kappa * d);
}

int lf_ctx_kernel_timing(lf_ctx *c, int enable) {
  DevGuard g(c);
  if (!c) return LF_ERR_INVALID_ARG;
  LF_TRY(drain_timing(c));
  c->timing = enable != 0;
  c->stats.clear();
  return LF_OK;
}

int lf_ctx_phase_stats(lf_ctx *c, int phase, double *ms, long *count) {
  DevGuard g(c);
  if (!c || !ms || !count || phase < 0 || phase >= LF_PHASE_COUNT) return LF_ERR_INVALID_ARG;
  LF_TRY(drain_timing(c));
  auto it = c->stats.find(-1 - phase);
  *ms = it == c->stats.end() ? 0.0 : it->second.first;
  *count = it == c->stats.end() ? 0 : it->second.second;
  return LF_OK;
}

int lf_ctx_kernel_stats(lf_ctx *c, int nvec, double *ms, long *count) {
  DevGuard g(c);
  if (!c || !ms || !count) return LF_ERR_INVALID_ARG;
  LF_TRY(drain_timing(c));
  *ms = 0;
  *count = 0;
  for (auto &kv : c->stats)
    if (kv.first > 0 && (nvec == 0 || kv.first == nvec)) {
      *ms += kv.second.first;
      *count += kv.second.second;
    }
  return LF_OK;
}

// ---------------------------------------------------------------- host-buffer API
static int xform_host(lf_ctx *c, uint64_t *e, size_t n, int d, int repr, bool fwd) {
  DevGuard g(c);
  if (!c || (!e && n)) return LF_ERR_INVALID_ARG;
  LF_TRY(check_repr(c, repr));
  if (!ring_ok(d)) return fail(c, LF_ERR_UNSUPPORTED_RING, "unsupported ring degree");
  Tables *t;
  LF_TRY(get_tables(c, d, t));
  DevBuf b;
  LF_TRY(upload(c, b, e, n * d, repr));
  LF_HIP(c, lfk::transform(b.p, n, d, fwd, fwd ? t->fwd : t->inv, c->cur));
  LF_TRY(download(c, e, b, n * d, repr));
  return lf_ctx_sync(c);
}
int lf_crt(lf_ctx *c, uint64_t *e, size_t n, int d, int repr) { return xform_host(c, e, n, d, repr, true); }
int lf_icrt(lf_ctx *c, uint64_t *e, size_t n, int d, int repr) { return xform_host(c, e, n, d, repr, false); }

int lf_ring_mul(lf_ctx *c, const uint64_t *a, const uint64_t *b, uint64_t *out, size_t n, int d, int repr) {
  DevGuard g(c);
  if (!c || ((!a || !b || !out) && n)) return LF_ERR_INVALID_ARG;
  LF_TRY(check_repr(c, repr));
  if (!ring_ok(d)) return fail(c, LF_ERR_UNSUPPORTED_RING, "unsupported ring degree");
  DevBuf da, db, dout;
  LF_TRY(upload(c, da, a, n * d, repr));
  LF_TRY(upload(c, db, b, n * d, repr));
  LF_TRY(dev_alloc(c, dout, n * d));
  LF_HIP(c, lfk::slot_mul(da.p, db.p, dout.p, n, d, c->cur));
  LF_TRY(download(c, out, dout, n * d, repr));
  return lf_ctx_sync(c);
}

int lf_ajtai_create(lf_ctx *c, const uint64_t *A, size_t kappa, size_t ncols, int d, int repr,
                    lf_ajtai **out) {
  DevGuard g(c);
  if (!c || !A || !out || !kappa || !ncols) return LF_ERR_INVALID_ARG;
  LF_TRY(check_repr(c, repr));
  if (!ring_ok(d)) return fail(c, LF_ERR_UNSUPPORTED_RING, "unsupported ring degree");
  DevBuf b;
  LF_TRY(upload(c, b, A, kappa * ncols * d, repr));
  LF_TRY(lf_ctx_sync(c));
  auto *aj = new lf_ajtai;
  aj->device = c->device;
  aj->A = b.p;
  b.p = nullptr;
  aj->owned = true;
  aj->kappa = kappa;
  aj->ncols = ncols;
  aj->d = d;
  int rc = ajtai_prepare(c, aj);
  if (rc != LF_OK) {
    lf_ajtai_destroy(aj);
    return rc;
  }
  *out = aj;
  return LF_OK;
}

int lf_ajtai_create_device(lf_ctx *c, const uint64_t *A_dev, size_t kappa, size_t ncols, int d,
                           lf_ajtai **out) {
  DevGuard g(c);
  if (!c || !A_dev || !out || !kappa || !ncols) return LF_ERR_INVALID_ARG;
  if (!ring_ok(d)) return fail(c, LF_ERR_UNSUPPORTED_RING, "unsupported ring degree");
  auto *aj = new lf_ajtai;
  aj->device = c->device;
  aj->A = A_dev;
  aj->kappa = kappa;
  aj->ncols = ncols;
  aj->d = d;
  int rc = ajtai_prepare(c, aj);
  if (rc != LF_OK) {
    lf_ajtai_destroy(aj);
    return rc;
  }
  *out = aj;
  return LF_OK;
}

void lf_ajtai_destroy(lf_ajtai *aj) {
  if (!aj) return;
  DevGuard g(aj->device);
  if (aj->owned) (void)hipFree((void *)aj->A);
  if (aj->Af) (void)hipFree(aj->Af);
  if (aj->kr) (void)hipFree(aj->kr);
  delete aj;
}
size_t lf_ajtai_kappa(const lf_ajtai *aj) { return aj ? aj->kappa : 0; }
size_t lf_ajtai_width(const lf_ajtai *aj) { return aj ? aj->ncols : 0; }
int lf_ajtai_d(const lf_ajtai *aj) { return aj ? aj->d : 0; }
int lf_ajtai_layout(const lf_ajtai *aj) { return aj && aj->Af ? 1 : 0; }

int lf_ajtai_commit(lf_ctx *c, const lf_ajtai *aj, const uint64_t *f, size_t f_len, uint64_t *cm, int repr) {
  DevGuard g(c);
  if (!c || !aj || !f || !cm) return LF_ERR_INVALID_ARG;
  LF_TRY(check_repr(c, repr));
  if (f_len != aj->ncols)  // commitment_scheme.rs:38-43
    return fail(c, LF_ERR_WRONG_WITNESS_LENGTH, "Wrong length of the witness");
  DevBuf df, dcm;
  LF_TRY(upload(c, df, f, f_len * aj->d, repr));
  LF_TRY(dev_alloc(c, dcm, aj->kappa * aj->d));
  const uint64_t *v = df.p;
  LF_TRY(ajtai_launch(c, aj, &v, 1, dcm.p));
  LF_TRY(download(c, cm, dcm, aj->kappa * aj->d, repr));
  return lf_ctx_sync(c);
}

int lf_witness_from_w_ccs(lf_ctx *c, const lf_params *pr, const uint64_t *w, size_t W, uint64_t *fc,
                          uint64_t *f, int repr) {
  DevGuard g(c);
  if (!c || (!w && W) || !fc || !f) return LF_ERR_INVALID_ARG;
  LF_TRY(check_repr(c, repr));
  int lb, lbs;
  LF_TRY(check_params(c, pr, lb, lbs));
  const int d = pr->d;
  const size_t N = W * pr->L;
  DevBuf dw, dfc, df;
  LF_TRY(upload(c, dw, w, W * d, repr));
  LF_TRY(dev_alloc(c, dfc, N * d));
  LF_TRY(dev_alloc(c, df, N * d));
  LF_TRY(lf_dev_witness_from_w_ccs(c, pr, dw.p, W, dfc.p, df.p));
  LF_TRY(download(c, fc, dfc, N * d, repr));
  LF_TRY(download(c, f, df, N * d, repr));
  return lf_ctx_sync(c);
}

int lf_witness_from_f(lf_ctx *c, const lf_params *pr, const uint64_t *f, size_t N, uint64_t *fc,
                      uint64_t *w, int repr) {
  DevGuard g(c);
  if (!c || (!f && N) || !fc || !w) return LF_ERR_INVALID_ARG;
  LF_TRY(check_repr(c, repr));
  int lb, lbs;
  LF_TRY(check_params(c, pr, lb, lbs));
  if (N % pr->L) return fail(c, LF_ERR_INCORRECT_LENGTH, "N must be a multiple of L");
  const int d = pr->d;
  DevBuf df, dfc, dw;
  LF_TRY(upload(c, df, f, N * d, repr));
  LF_TRY(dev_alloc(c, dfc, N * d));
  LF_TRY(dev_alloc(c, dw, N / pr->L * d));
  LF_TRY(lf_dev_witness_from_f(c, pr, df.p, N, dfc.p, dw.p));
  LF_TRY(download(c, fc, dfc, N * d, repr));
  LF_TRY(download(c, w, dw, N / pr->L * d, repr));
  return lf_ctx_sync(c);
}

int lf_decompose_witness(lf_ctx *c, const lf_params *pr, const uint64_t *fc, size_t N, uint64_t *fck,
                         uint64_t *fk, uint64_t *wk, int repr) {
  DevGuard g(c);
  if (!c || (!fc && N) || !fck || !fk || !wk) return LF_ERR_INVALID_ARG;
  LF_TRY(check_repr(c, repr));
  int lb, lbs;
  LF_TRY(check_params(c, pr, lb, lbs));
  if (N % pr->L) return fail(c, LF_ERR_INCORRECT_LENGTH, "N must be a multiple of L");
  const int d = pr->d, K = pr->K;
  DevBuf dfc, dfck, dfk, dwk;
  LF_TRY(upload(c, dfc, fc, N * d, repr));
  LF_TRY(dev_alloc(c, dfck, K * N * d));
  LF_TRY(dev_alloc(c, dfk, K * N * d));
  LF_TRY(dev_alloc(c, dwk, K * (N / pr->L) * d));
  LF_TRY(lf_dev_decompose_witness(c, pr, dfc.p, N, dfck.p, dfk.p, dwk.p));
  LF_TRY(download(c, fck, dfck, K * N * d, repr));
  LF_TRY(download(c, fk, dfk, K * N * d, repr));
  LF_TRY(download(c, wk, dwk, K * (N / pr->L) * d, repr));
  return lf_ctx_sync(c);
}

int lf_commit(lf_ctx *c, const lf_ajtai *aj, const lf_params *pr, const uint64_t *z, size_t z_len, size_t l,
              uint64_t *fc, uint64_t *f, uint64_t *cm, int repr) {
  DevGuard g(c);
  if (!c || !aj || !z || !fc || !f || !cm) return LF_ERR_INVALID_ARG;
  LF_TRY(check_repr(c, repr));
  int lb, lbs;
  LF_TRY(check_params(c, pr, lb, lbs));
  if (pr->d != aj->d) return fail(c, LF_ERR_INVALID_ARG, "params ring != Ajtai ring");
  if (z_len < l + 1) return fail(c, LF_ERR_INCORRECT_LENGTH, "z shorter than l + 1");
  const int d = pr->d;
  const size_t W = z_len - l - 1, N = W * pr->L;  // main.rs:354-355: w_ccs = z[l+1..]
  if (N != aj->ncols) return fail(c, LF_ERR_WRONG_WITNESS_LENGTH, "Wrong length of the witness");
  DevBuf dw, dfc, df, dcm;
  LF_TRY(upload(c, dw, z + (l + 1) * d, W * d, repr));
  LF_TRY(dev_alloc(c, dfc, N * d));
  LF_TRY(dev_alloc(c, df, N * d));
  LF_TRY(dev_alloc(c, dcm, aj->kappa * d));
  LF_TRY(lf_dev_witness_from_w_ccs(c, pr, dw.p, W, dfc.p, df.p));
  const uint64_t *v = df.p;
  LF_TRY(ajtai_launch(c, aj, &v, 1, dcm.p));
  LF_TRY(download(c, fc, dfc, N * d, repr));
  LF_TRY(download(c, f, df, N * d, repr));
  LF_TRY(download(c, cm, dcm, aj->kappa * d, repr));
  return lf_ctx_sync(c);
}

int lf_fold_hot(lf_ctx *c, const lf_ajtai *aj, const lf_params *pr, const uint64_t *acc_cm,
                const uint64_t *acc_fc, const uint64_t *cm_i, const uint64_t *wi_fc, size_t N,
                const uint64_t *rho, uint64_t *y, uint64_t *f0, uint64_t *f0c, uint64_t *w0, uint64_t *cm0,
                int repr) {
  DevGuard g(c);
  if (!c || !aj || !acc_cm || !acc_fc || !cm_i || !wi_fc || !rho || !y || !f0 || !f0c || !w0 || !cm0)
    return LF_ERR_INVALID_ARG;
  LF_TRY(check_repr(c, repr));
  int lb, lbs;
  LF_TRY(check_params(c, pr, lb, lbs));
  if (pr->d != aj->d) return fail(c, LF_ERR_INVALID_ARG, "params ring != Ajtai ring");
  if (N % pr->L) return fail(c, LF_ERR_INCORRECT_LENGTH, "N must be a multiple of L");
  const int d = pr->d, K = pr->K;
  const size_t W = N / pr->L, kd = aj->kappa * d;
  DevBuf dacm, dafc, dcmi, dwfc, drho, dfck[2], dfk[2], dwk[2], dy, df0, df0c, dw0, dcm0;
  LF_TRY(upload(c, dacm, acc_cm, kd, repr));
  LF_TRY(upload(c, dafc, acc_fc, N * d, repr));
  LF_TRY(upload(c, dcmi, cm_i, kd, repr));
  LF_TRY(upload(c, dwfc, wi_fc, N * d, repr));
  LF_TRY(upload(c, drho, rho, 2 * (size_t)K * d, repr));
  for (int s = 0; s < 2; s++) {
    LF_TRY(dev_alloc(c, dfck[s], K * N * d));
    LF_TRY(dev_alloc(c, dfk[s], K * N * d));
    LF_TRY(dev_alloc(c, dwk[s], K * W * d));
  }
  LF_TRY(dev_alloc(c, dy, 2 * K * kd));
  LF_TRY(dev_alloc(c, df0, N * d));
  LF_TRY(dev_alloc(c, df0c, N * d));
  LF_TRY(dev_alloc(c, dw0, W * d));
  LF_TRY(dev_alloc(c, dcm0, kd));
  lf_fold_step_bufs b{};
  b.acc_cm = dacm.p;
  b.acc_f_coeff = dafc.p;
  b.rho = drho.p;
  for (int s = 0; s < 2; s++) {
    b.fk_coeff[s] = dfck[s].p;
    b.fk[s] = dfk[s].p;
    b.wk[s] = dwk[s].p;
    b.y[s] = dy.p + (size_t)s * K * kd;
  }
  b.f0 = df0.p;
  b.f0_coeff = df0c.p;
  b.w_ccs0 = dw0.p;
  b.cm0 = dcm0.p;
  LF_TRY(fold_commit(c, aj, pr, lb, lbs, W, &b, dwfc.p, nullptr, fold_dst(pr, &b, kd, nullptr)));
  LF_TRY(fold_finish(c, aj, pr, lb, lbs, W, &b, dcmi.p));
  LF_TRY(download(c, y, dy, 2 * K * kd, repr));
  LF_TRY(download(c, f0, df0, N * d, repr));
  LF_TRY(download(c, f0c, df0c, N * d, repr));
  LF_TRY(download(c, w0, dw0, W * d, repr));
  LF_TRY(download(c, cm0, dcm0, kd, repr));
  return lf_ctx_sync(c);
}

int lf_short_challenge(const uint8_t *bs, size_t nbytes, int d, uint64_t *coeffs) {
  // cyclotomic-rings rings/goldilocks.rs:41-67 (3 bytes -> 4 six-bit coefficients - 32)
  if (!bs || !coeffs || d % 4) return LF_ERR_INVALID_ARG;
  if (nbytes != (size_t)(3 * d / 4)) return LF_ERR_CHALLENGE_BYTES;
  for (int i = 0; i < d / 4; i++) {
    int x[4];
    x[0] = (bs[3 * i] & 0x3f) - 32;
    x[1] = (((bs[3 * i] & 0xc0) >> 6) | ((bs[3 * i + 1] & 0x0f) << 2)) - 32;
    x[2] = (((bs[3 * i + 1] & 0xf0) >> 4) | ((bs[3 * i + 2] & 0x03) << 4)) - 32;
    x[3] = ((bs[3 * i + 2] & 0xfc) >> 2) - 32;
    for (int k = 0; k < 4; k++) coeffs[4 * i + k] = x[k] < 0 ? gl::P - (uint64_t)(-x[k]) : (uint64_t)x[k];
  }
  return LF_OK;
}

int lf_poseidon2_permute(lf_ctx *c, uint64_t *states, size_t n) {
  DevGuard g(c);
  if (!c || (!states && n)) return LF_ERR_INVALID_ARG;
  DevBuf b;
  LF_TRY(upload(c, b, states, 16 * n, LF_REPR_CANONICAL));
  LF_HIP(c, lfk::p2_permute(b.p, n, c->cur));
  LF_TRY(download(c, states, b, 16 * n, LF_REPR_CANONICAL));
  return lf_ctx_sync(c);
}

// ---------------------------------------------------------------- device API
int lf_dev_crt(lf_ctx *c, uint64_t *e, size_t n, int d) {
  DevGuard g(c);
  if (!c || (!e && n)) return LF_ERR_INVALID_ARG;
  if (!ring_ok(d)) return fail(c, LF_ERR_UNSUPPORTED_RING, "unsupported ring degree");
  Tables *t;
  LF_TRY(get_tables(c, d, t));
  LF_HIP(c, lfk::transform(e, n, d, true, t->fwd, c->cur));
  return LF_OK;
}
int lf_dev_icrt(lf_ctx *c, uint64_t *e, size_t n, int d) {
  DevGuard g(c);
  if (!c || (!e && n)) return LF_ERR_INVALID_ARG;
  if (!ring_ok(d)) return fail(c, LF_ERR_UNSUPPORTED_RING, "unsupported ring degree");
  Tables *t;
  LF_TRY(get_tables(c, d, t));
  LF_HIP(c, lfk::transform(e, n, d, false, t->inv, c->cur));
  return LF_OK;
}
int lf_dev_ring_mul(lf_ctx *c, const uint64_t *a, const uint64_t *b, uint64_t *out, size_t n, int d) {
  DevGuard g(c);
  if (!c) return LF_ERR_INVALID_ARG;
  if (!ring_ok(d)) return fail(c, LF_ERR_UNSUPPORTED_RING, "unsupported ring degree");
  LF_HIP(c, lfk::slot_mul(a, b, out, n, d, c->cur));
  return LF_OK;
}
int lf_dev_to_montgomery(lf_ctx *c, uint64_t *x, size_t n) {
  DevGuard g(c);
  if (!c) return LF_ERR_INVALID_ARG;
  LF_HIP(c, lfk::mont(x, n, true, c->cur));
  return LF_OK;
}
int lf_dev_from_montgomery(lf_ctx *c, uint64_t *x, size_t n) {
  DevGuard g(c);
  if (!c) return LF_ERR_INVALID_ARG;
  LF_HIP(c, lfk::mont(x, n, false, c->cur));
  return LF_OK;
}
int lf_dev_witness_from_w_ccs(lf_ctx *c, const lf_params *pr, const uint64_t *w, size_t W, uint64_t *fc,
                              uint64_t *f) {
  DevGuard g(c);
  if (!c) return LF_ERR_INVALID_ARG;
  int lb, lbs;
  LF_TRY(check_params(c, pr, lb, lbs));
  Tables *t;
  LF_TRY(get_tables(c, pr->d, t));
  LF_HIP(c, lfk::from_w_ccs(w, W, pr->d, lb, pr->L, fc, f, t->fwd, t->inv, c->d_err, c->cur));
  return LF_OK;
}
int lf_dev_witness_from_f(lf_ctx *c, const lf_params *pr, const uint64_t *f, size_t N, uint64_t *fc,
                          uint64_t *w) {
  DevGuard g(c);
  if (!c) return LF_ERR_INVALID_ARG;
  int lb, lbs;
  LF_TRY(check_params(c, pr, lb, lbs));
  if (N % pr->L) return fail(c, LF_ERR_INCORRECT_LENGTH, "N must be a multiple of L");
  Tables *t;
  LF_TRY(get_tables(c, pr->d, t));
  LF_HIP(c, lfk::from_f(f, N, pr->d, lb, pr->L, fc, w, t->inv, c->cur));
  return LF_OK;
}
int lf_dev_decompose_witness(lf_ctx *c, const lf_params *pr, const uint64_t *fc, size_t N, uint64_t *fck,
                             uint64_t *fk, uint64_t *wk) {
  DevGuard g(c);
  if (!c) return LF_ERR_INVALID_ARG;
  int lb, lbs;
  LF_TRY(check_params(c, pr, lb, lbs));
  if (N % pr->L) return fail(c, LF_ERR_INCORRECT_LENGTH, "N must be a multiple of L");
  Tables *t;
  LF_TRY(get_tables(c, pr->d, t));
  if (n4k_ok(t, pr->d, lbs, pr->K) && N % pr->L == 0)
    return decompose_n4k_sides(c, t, 1, &fc, &fck, &fk, &wk, N, lb, pr->L, pr->K);
  LF_HIP(c, lfk::decompose_witness(fc, N, pr->d, lb, pr->L, lbs, pr->K, fck, fk, wk, t->fwd, c->d_err, c->cur));
  return LF_OK;
}
int lf_dev_ajtai_commit(lf_ctx *c, const lf_ajtai *aj, const uint64_t *const *vecs, int nvec, uint64_t *cm) {
  DevGuard g(c);
  if (!c || !aj || !vecs || !cm) return LF_ERR_INVALID_ARG;
  return ajtai_launch(c, aj, vecs, nvec, cm);
}
int lf_dev_commit_y0(lf_ctx *c, const lf_params *pr, const uint64_t *cm, uint64_t *y, size_t kappa) {
  DevGuard g(c);
  if (!c) return LF_ERR_INVALID_ARG;
  int lb, lbs;
  LF_TRY(check_params(c, pr, lb, lbs));
  LF_HIP(c, lfk::commit_y0(cm, y, kappa, pr->d, lbs, pr->K, c->cur));
  return LF_OK;
}
int lf_dev_fold(lf_ctx *c, int d, const uint64_t *rho, const uint64_t *const *x, int nwit, size_t n,
                uint64_t *out) {
  DevGuard g(c);
  if (!c || !rho || !x || !out || nwit < 1 || nwit > LF_MAX_VECS) return LF_ERR_INVALID_ARG;
  if (!ring_ok(d)) return fail(c, LF_ERR_UNSUPPORTED_RING, "unsupported ring degree");
  lfk::VecPtrs vp{};
  for (int i = 0; i < nwit; i++) vp.p[i] = x[i];
  LF_HIP(c, lfk::fold(rho, vp, nwit, n, d, out, c->cur));
  return LF_OK;
}

// commit(z) (zkvm main.rs:348-367): Witness::from_w_ccs; its A f is batched
// with the decomposition commitments of fold() in a single pass over A
static int step_check(lf_ctx *c, const lf_ajtai *aj, const lf_params *pr, size_t W, const lf_fold_step_bufs *b,
                      int &lb, int &lbs) {
  if (!c || !aj || !b) return LF_ERR_INVALID_ARG;
  LF_TRY(check_params(c, pr, lb, lbs));
  if (pr->d != aj->d) return fail(c, LF_ERR_INVALID_ARG, "params ring != Ajtai ring");
  if (W * (size_t)pr->L != aj->ncols) return fail(c, LF_ERR_WRONG_WITNESS_LENGTH, "W*L != Ajtai width");
  return LF_OK;
}
static int step_commit(lf_ctx *c, const lf_ajtai *aj, const lf_params *pr, size_t W, const lf_fold_step_bufs *b,
                       int lb, int lbs, const lfk::OutPtrs &dst, Deferred *defer = nullptr) {
  uint32_t *smg1 = nullptr;
  {
    PhaseTimer pt(c, LF_PHASE_FROM_W_CCS);
    // the fused X^1024 + 1 decomposition that fold_commit runs next packs both
    // sides' digits into sign|magnitude words; the new witness's (side 1) are
    // written here, by the kernel that makes its digits, instead of re-read
    Tables *t;
    LF_TRY(get_tables(c, pr->d, t));
    const int L = pr->L, K = pr->K, d = pr->d;
    const size_t N = W * (size_t)L;
    const bool fused = aj->Af && aj->geom.Lp == L && d == 1024 && lbs == 1 && K <= 15 && t->fwd.mid &&
                       t->inv.mid && lb <= K && aj->ncols == N && (!b->planes[0]) == (!b->planes[1]);
    if (fused) {
      if (!b->planes[0]) LF_TRY(grow(c, c->smg, c->smg_elems, 2 * N * 512));
      smg1 = b->planes[1] ? reinterpret_cast<uint32_t *>(b->planes[1]) : c->smg + N * 512;
    }
    if (!b->w_ccs || !b->f_coeff || !b->f) return fail(c, LF_ERR_INVALID_ARG, "null step buffer");
    LF_HIP(c, lfk::from_w_ccs(b->w_ccs, W, d, lb, L, b->f_coeff, b->f, t->fwd, t->inv, c->d_err, c->cur, smg1));
  }
  return fold_commit(c, aj, pr, lb, lbs, W, b, b->f_coeff, b->f, dst, defer, smg1);
}

int lf_dev_fold_lcccs(lf_ctx *c, int d, int nwit, const uint64_t *rho, const uint64_t *rho_coeff, const uint64_t *eta,
                      size_t t, const uint64_t *xwh, size_t l1, const uint64_t *theta, uint64_t *u0, uint64_t *x0,
                      uint64_t *v0) {
  if (!c || nwit < 1 || nwit > LF_MAX_VECS || !rho) return LF_ERR_INVALID_ARG;
  DevGuard g(c);
  if (!ring_ok(d)) return fail(c, LF_ERR_UNSUPPORTED_RING, "unsupported ring degree");
  if ((t && (!eta || !u0)) || (l1 && (!xwh || !x0)) || (!rho_coeff != !theta) || (theta && !v0))
    return fail(c, LF_ERR_INVALID_ARG, "missing buffer");
  lfk::VecPtrs ve{}, vx{};
  for (int i = 0; i < nwit; i++) {
    ve.p[i] = eta + (size_t)i * t * d;
    vx.p[i] = xwh + (size_t)i * l1 * d;
  }
  // u_0 = sum rho_i eta_i (folding/utils.rs:478-496), x_0 = sum rho_i (x_w || h)_i (:498-514)
  if (t) LF_HIP(c, lfk::fold(rho, ve, nwit, t, d, u0, c->cur));
  if (l1) LF_HIP(c, lfk::fold(rho, vx, nwit, l1, d, x0, c->cur));
  // v_0 = rot_lin_combination(rho_s_coeff, theta_s) (:466)
  if (theta) LF_HIP(c, lfk::rot_lin(rho_coeff, theta, nwit, d, v0, c->cur));
  return LF_OK;
}

int lf_fold_lcccs(lf_ctx *c, int d, int nwit, const uint64_t *rho, const uint64_t *rho_coeff, const uint64_t *eta,
                  size_t t, const uint64_t *xwh, size_t l1, const uint64_t *theta, uint64_t *u0, uint64_t *x0,
                  uint64_t *v0, int repr) {
  if (!c || nwit < 1 || nwit > LF_MAX_VECS || !rho) return LF_ERR_INVALID_ARG;
  DevGuard g(c);
  LF_TRY(check_repr(c, repr));
  if (!ring_ok(d)) return fail(c, LF_ERR_UNSUPPORTED_RING, "unsupported ring degree");
  const size_t tau = d == 24 ? 3 : 1, n = (size_t)nwit;
  DevBuf drho, drc, deta, dx, dth, du, dx0, dv;
  LF_TRY(upload(c, drho, rho, n * d, repr));
  if (t) {
    LF_TRY(upload(c, deta, eta, n * t * d, repr));
    LF_TRY(dev_alloc(c, du, t * d));
  }
  if (l1) {
    LF_TRY(upload(c, dx, xwh, n * l1 * d, repr));
    LF_TRY(dev_alloc(c, dx0, l1 * d));
  }
  if (theta) {
    LF_TRY(upload(c, drc, rho_coeff, n * d, repr));
    LF_TRY(upload(c, dth, theta, n * tau * d, repr));
    LF_TRY(dev_alloc(c, dv, tau * d));
  }
  LF_TRY(lf_dev_fold_lcccs(c, d, nwit, drho.p, drc.p, deta.p, t, dx.p, l1, dth.p, du.p, dx0.p, dv.p));
  if (t) LF_TRY(download(c, u0, du, t * d, repr));
  if (l1) LF_TRY(download(c, x0, dx0, l1 * d, repr));
  if (theta) LF_TRY(download(c, v0, dv, tau * d, repr));
  return lf_ctx_sync(c);
}

// compute_x_s = w_ccs_k of decompose_witness(Witness::from_w_ccs(x).f_coeff):
// gadget_decompose(ICRT(x)), its b_small digit planes, each plane recomposed
// over the L limbs with B and CRT'd -- decompose_big_vec_into_k_vec_and_compose_back
// (decomposition/utils.rs:12-42), the same arithmetic (CRT is linear)
int lf_dev_compute_x_s(lf_ctx *c, const lf_params *pr, const uint64_t *x, size_t m, uint64_t *x_s) {
  if (!c || (!x && m) || (!x_s && m)) return LF_ERR_INVALID_ARG;
  DevGuard g(c);
  int lb, lbs;
  LF_TRY(check_params(c, pr, lb, lbs));
  if (!m) return LF_OK;
  const int d = pr->d, L = pr->L, K = pr->K;
  const size_t N = m * L;
  LF_TRY(grow(c, c->tmp, c->tmp_elems, (2 + 2 * (size_t)K) * N * d));
  uint64_t *fc = c->tmp, *f = fc + N * d, *fck = f + N * d, *fk = fck + (size_t)K * N * d;
  LF_TRY(lf_dev_witness_from_w_ccs(c, pr, x, m, fc, f));
  return lf_dev_decompose_witness(c, pr, fc, N, fck, fk, x_s);
}

int lf_compute_x_s(lf_ctx *c, const lf_params *pr, const uint64_t *x, size_t m, uint64_t *x_s, int repr) {
  if (!c || (!x && m) || (!x_s && m)) return LF_ERR_INVALID_ARG;
  DevGuard g(c);
  LF_TRY(check_repr(c, repr));
  int lb, lbs;
  LF_TRY(check_params(c, pr, lb, lbs));
  DevBuf dx, ds;
  LF_TRY(upload(c, dx, x, m * pr->d, repr));
  LF_TRY(dev_alloc(c, ds, (size_t)pr->K * m * pr->d));
  LF_TRY(lf_dev_compute_x_s(c, pr, dx.p, m, ds.p));
  LF_TRY(download(c, x_s, ds, (size_t)pr->K * m * pr->d, repr));
  return lf_ctx_sync(c);
}

// ---------------------------------------------------------------- multilinear sumcheck
static int comb_check(lf_ctx *c, const lf_comb *cb, int nm, int d, int degree, lfk::CombS *cs) {
  if (!cb) return fail(c, LF_ERR_INVALID_ARG, "null combination");
  if (cb->kind == LF_COMB_FOLDING) {
    if (!cb->mu || cb->nk < 1 || cb->tau < 1 || cb->bsmall < 1 || cb->bsmall > 4 || nm != 5 + cb->nk * cb->tau ||
        (degree >= 0 && degree != 2 * cb->bsmall))
      return fail(c, LF_ERR_INVALID_ARG, "folding sumcheck: 5 + nk tau MLEs, degree 2 B_SMALL, B_SMALL <= 4");
    return LF_OK;
  }
  if (cb->kind != LF_COMB_LINEARIZATION || !cb->c || !cb->S_off || !cb->S_idx || cb->q < 1 ||
      cb->q > lfk::LF_MAX_MULTISETS || degree < 1 || degree > 9)
    return fail(c, LF_ERR_INVALID_ARG, "linearization sumcheck: 1 <= q <= 64 multisets, degree <= 9");
  cs->q = cb->q;
  for (int i = 0; i <= cb->q; i++) cs->off[i] = cb->S_off[i];
  if (cs->off[0] != 0 || cs->off[cb->q] > lfk::LF_MAX_S)
    return fail(c, LF_ERR_INVALID_ARG, "linearization sumcheck: at most 512 multiset entries");
  for (int i = 0; i < cs->off[cb->q]; i++) {
    if (cb->S_idx[i] < 0 || cb->S_idx[i] >= nm - 1) return fail(c, LF_ERR_INVALID_ARG, "multiset index out of range");
    cs->idx[i] = (short)cb->S_idx[i];
  }
  return LF_OK;
}
static int comb_degree(const lf_comb *cb, int degree) { return cb->kind == LF_COMB_FOLDING ? 2 * cb->bsmall : degree; }

int lf_dev_eq_table(lf_ctx *c, int d, const uint64_t *r, int nv, uint64_t *out) {
  if (!c || !r || !out || nv < 1) return LF_ERR_INVALID_ARG;
  DevGuard g(c);
  if (!ring_ok(d)) return fail(c, LF_ERR_UNSUPPORTED_RING, "unsupported ring degree");
  LF_HIP(c, lfk::eq_table(r, nv, d, out, c->cur));
  return LF_OK;
}

int lf_dev_get_fhat(lf_ctx *c, int d, const uint64_t *f_coeff, size_t N, int nv, uint64_t *out) {
  if (!c || !out || (N && !f_coeff) || nv < 0 || nv > 40) return LF_ERR_INVALID_ARG;
  DevGuard g(c);
  if (!ring_ok(d)) return fail(c, LF_ERR_UNSUPPORTED_RING, "unsupported ring degree");
  if (N > ((size_t)1 << nv)) return fail(c, LF_ERR_INCORRECT_LENGTH, "N exceeds 2^nv");
  LF_HIP(c, lfk::get_fhat(f_coeff, N, d, nv, out, c->cur));
  return LF_OK;
}

int lf_dev_fhat_evaluate(lf_ctx *c, int d, const uint64_t *f_coeff, size_t N, size_t wstride, int nw, int nv,
                         const uint64_t *point, uint64_t *out) {
  if (!c || !point || !out || nw < 0 || nv < 1 || (nw && N && !f_coeff)) return LF_ERR_INVALID_ARG;
  DevGuard g(c);
  if (!ring_ok(d)) return fail(c, LF_ERR_UNSUPPORTED_RING, "unsupported ring degree");
  const size_t n = (size_t)1 << nv;
  if (N > n) return fail(c, LF_ERR_INCORRECT_LENGTH, "N exceeds 2^nv");
  const int tau = d == 24 ? 3 : 1;
  LF_TRY(grow(c, c->sc, c->sc_elems, n * d + lfk::mle_eval_partial_elems(d, nw * tau)));
  LF_HIP(c, lfk::eq_table(point, nv, d, c->sc, c->cur));
  LF_HIP(c, lfk::fhat_dot(f_coeff, N, wstride ? wstride : N * d, nw, c->sc, n, d, c->sc + n * d, out, c->cur));
  return LF_OK;
}

int lf_dev_fhat_evaluate_eq(lf_ctx *c, int d, const uint64_t *f_coeff, size_t N, size_t wstride, int nw, int nv,
                            const uint64_t *eq, uint64_t *out) {
  if (!c || !eq || !out || nw < 0 || nv < 1 || (nw && N && !f_coeff)) return LF_ERR_INVALID_ARG;
  DevGuard g(c);
  if (!ring_ok(d)) return fail(c, LF_ERR_UNSUPPORTED_RING, "unsupported ring degree");
  const size_t n = (size_t)1 << nv;
  if (N > n) return fail(c, LF_ERR_INCORRECT_LENGTH, "N exceeds 2^nv");
  const int tau = d == 24 ? 3 : 1;
  LF_TRY(grow(c, c->sc, c->sc_elems, lfk::mle_eval_partial_elems(d, nw * tau)));
  LF_HIP(c, lfk::fhat_dot(f_coeff, N, wstride ? wstride : N * d, nw, eq, n, d, c->sc, out, c->cur));
  return LF_OK;
}

int lf_dev_mle_lincomb(lf_ctx *c, int d, const uint64_t *mles, size_t stride, int nm, int nv, const uint64_t *coef,
                       uint64_t *io) {
  if (!c || !io || nm < 0 || nv < 0 || (nm && (!mles || !coef))) return LF_ERR_INVALID_ARG;
  DevGuard g(c);
  if (!ring_ok(d)) return fail(c, LF_ERR_UNSUPPORTED_RING, "unsupported ring degree");
  const size_t n = (size_t)1 << nv;
  LF_HIP(c, lfk::mle_lincomb(mles, stride ? stride : n * d, nm, coef, n, d, io, c->cur));
  return LF_OK;
}

int lf_dev_mle_fix_first(lf_ctx *c, int d, const uint64_t *in, size_t in_stride, int nm, int nv,
                         const uint64_t *r_base, uint64_t *out, size_t out_stride) {
  if (!c || !in || !out || !r_base || nm < 1 || nv < 1) return LF_ERR_INVALID_ARG;
  DevGuard g(c);
  if (!ring_ok(d)) return fail(c, LF_ERR_UNSUPPORTED_RING, "unsupported ring degree");
  LF_HIP(c, lfk::mle_fix_first(in, in_stride, nm, (size_t)1 << (nv - 1), d, r_base, out, out_stride, c->cur));
  return LF_OK;
}

int lf_dev_mle_evaluate_eq(lf_ctx *c, int d, const uint64_t *mles, int nm, int nv, const uint64_t *eq, uint64_t *out) {
  if (!c || !mles || !eq || !out || nm < 1 || nv < 1) return LF_ERR_INVALID_ARG;
  DevGuard g(c);
  if (!ring_ok(d)) return fail(c, LF_ERR_UNSUPPORTED_RING, "unsupported ring degree");
  const size_t n = (size_t)1 << nv;
  LF_TRY(grow(c, c->sc, c->sc_elems, lfk::mle_eval_partial_elems(d, nm)));
  LF_HIP(c, lfk::mle_dot(mles, n * d, nm, eq, n, d, c->sc, out, c->cur));
  return LF_OK;
}

int lf_dev_mle_evaluate(lf_ctx *c, int d, const uint64_t *mles, int nm, int nv, const uint64_t *point, uint64_t *out) {
  if (!c || !mles || !point || !out || nm < 1 || nv < 1) return LF_ERR_INVALID_ARG;
  DevGuard g(c);
  if (!ring_ok(d)) return fail(c, LF_ERR_UNSUPPORTED_RING, "unsupported ring degree");
  const size_t n = (size_t)1 << nv;
  LF_TRY(grow(c, c->sc, c->sc_elems, n * d + lfk::mle_eval_partial_elems(d, nm)));
  LF_HIP(c, lfk::eq_table(point, nv, d, c->sc, c->cur));
  LF_HIP(c, lfk::mle_dot(mles, n * d, nm, c->sc, n, d, c->sc + n * d, out, c->cur));
  return LF_OK;
}

int lf_dev_sumcheck_round(lf_ctx *c, const lf_comb *cb, const uint64_t *mles, size_t stride, int nm, int nv, int d,
                          int degree, uint64_t *evals) {
  if (!c || !mles || !evals || nv < 1) return LF_ERR_INVALID_ARG;
  DevGuard g(c);
  if (!ring_ok(d)) return fail(c, LF_ERR_UNSUPPORTED_RING, "unsupported ring degree");
  lfk::CombS cs;
  LF_TRY(comb_check(c, cb, nm, d, cb && cb->kind == LF_COMB_FOLDING ? -1 : degree, &cs));
  const int deg = comb_degree(cb, degree);
  const size_t half = (size_t)1 << (nv - 1);
  const size_t part = lfk::round_partial_elems(d, half, deg + 1, cb->kind == LF_COMB_FOLDING ? cb->nk * cb->tau : cb->q);
  const size_t wlen = cb->kind == LF_COMB_FOLDING ? (size_t)cb->nk * cb->tau * d : 0;
  LF_TRY(grow(c, c->sc, c->sc_elems, part + wlen));
  if (cb->kind == LF_COMB_FOLDING) {
    uint64_t *w = c->sc + part;
    LF_HIP(c, lfk::fold_weights(cb->mu, cb->nk, cb->tau, d, w, c->cur));
    LF_HIP(c, lfk::round_folding(mles, stride, cb->nk * cb->tau, w, cb->bsmall, half, d, c->sc, evals, c->cur));
  } else {
    LF_HIP(c, lfk::round_lin(mles, stride, nm, cb->c, cs, deg, half, d, c->sc, evals, c->cur));
  }
  return LF_OK;
}

// MLSumcheck::prove_as_subprotocol (sumcheck.rs:61-88). Round 0 reads the MLEs at
// `mles` (stride 2^nv d) or, with ptrs (device array of nm pointers), wherever
// those point; every round fixes them into the next buffer: the context scratch
// (2^(nv-1) points) and `alt` (2^(nv-2) points; the input itself when ptrs is null)
// the folding polynomial's f_hat MLEs as digit coefficient rows (lf_sumcheck_prove_fold_digits)
struct DigitFhat {
  const uint64_t *fc0, *fc1;
  int K;
  size_t N, wstride;
};
static int sumcheck_run(lf_ctx *c, lf_transcript *t, const lf_comb *cb, const lfk::CombS &cs, const uint64_t *mles,
                        const uint64_t *const *ptrs, uint64_t *alt, int nm, int nv, int d, int degree, uint64_t *proof,
                        uint64_t *randomness, const DigitFhat *dg = nullptr) {
  const int tb = lfk::slot_words(d), nev = degree + 1;
  const size_t n = (size_t)1 << nv;
  // scratch: the MLEs fixed by the first challenge, the round's partial sums, the
  // evaluations, the weights; the partial sums of every round fit the largest
  // round's (chunks only split the small ones)
  const int nfc = cb->kind == LF_COMB_FOLDING ? cb->nk * cb->tau : cb->q;  // the chunked sum (f_hat MLEs / multisets)
  size_t part = 0;
  for (size_t h = n / 2; h >= 1; h /= 2) part = std::max(part, lfk::round_partial_elems(d, h, nev, nfc));
  const size_t fixed = (size_t)nm * (n / 2) * d;
  const size_t wlen = cb->kind == LF_COMB_FOLDING ? (size_t)cb->nk * cb->tau * d : 0;
  LF_TRY(grow(c, c->sc, c->sc_elems, fixed + part + (size_t)nev * d + wlen));
  uint64_t *buf = c->sc, *partial = buf + fixed, *ev = partial + part, *w = ev + (size_t)nev * d;
  if (wlen) LF_HIP(c, lfk::fold_weights(cb->mu, cb->nk, cb->tau, d, w, c->cur));
  // absorb R::from(nvars), R::from(degree)
  std::vector<uint64_t> scal(d, 0);
  for (int i = 0; i < d; i += tb) scal[i] = (uint64_t)nv;
  lf_transcript_absorb_ring(t, scal.data(), 1, d, LF_REPR_CANONICAL);
  for (int i = 0; i < d; i += tb) scal[i] = (uint64_t)degree;
  lf_transcript_absorb_ring(t, scal.data(), 1, d, LF_REPR_CANONICAL);
  const uint64_t *cur = mles;
  const uint64_t *const *cptrs = ptrs;
  size_t stride = n * d;
  for (int i = 0; i < nv; i++) {
    const size_t half = n >> (i + 1);
    uint64_t *msg = proof + (size_t)i * nev * d;
    if (dg && i == 0)  // round 0 straight from the digits (cur: the 5 general MLEs)
      LF_HIP(c, lfk::round_folding0_digits(cur, stride, dg->fc0, dg->fc1, dg->K, dg->N, dg->wstride, cb->nk * cb->tau, w,
                                           half, d, partial, ev, c->cur));
    else if (cb->kind == LF_COMB_FOLDING)
      LF_HIP(c, lfk::round_folding(cur, stride, cb->nk * cb->tau, w, cb->bsmall, half, d, partial, ev, c->cur));
    else
      LF_HIP(c, lfk::round_lin(cur, stride, nm, cb->c, cs, degree, half, d, partial, ev, c->cur, cptrs));
    LF_TRY(download_msg(c, msg, ev, (size_t)nev * d));
    // prover message absorbed, challenge sampled (fiat_shamir.rs:69-86; one sample for Fq) and absorbed
    lf_transcript_absorb_ring(t, msg, (size_t)nev, d, LF_REPR_CANONICAL);
    uint64_t *ch = randomness + (size_t)i * tb;
    if (tb == 3) {
      lf_transcript_get_challenge(t, ch);
    } else {
      ch[0] = lf_transcript_sample(t);
      lf_transcript_observe(t, ch[0]);
    }
    for (int k = 0; k < d; k++) scal[k] = ch[k % tb];
    lf_transcript_absorb_ring(t, scal.data(), 1, d, LF_REPR_CANONICAL);
    // fix_variables(r) of every MLE (prover.rs:75-78), into the other buffer
    if (half >= 1 && i + 1 < nv) {
      uint64_t *dst = (i % 2 == 0) ? buf : alt;
      if (dg && i == 0) {  // the 5 general MLEs, then the f_hat ones from the digits
        LF_HIP(c, lfk::mle_fix_first(cur, stride, 5, half, d, ch, dst, half * d, c->cur, cptrs));
        LF_HIP(c, lfk::fix_fhat_digits(dg->fc0, dg->fc1, dg->K, dg->N, dg->wstride, nm - 5, half, d, ch,
                                       dst + 5 * half * d, half * d, c->cur));
      } else {
        LF_HIP(c, lfk::mle_fix_first(cur, stride, nm, half, d, ch, dst, half * d, c->cur, cptrs));
      }
      cur = dst;
      cptrs = nullptr;
      stride = half * d;
    }
  }
  return LF_OK;
}

int lf_sumcheck_prove_fold_digits(lf_ctx *c, lf_transcript *t, const lf_comb *cb, const uint64_t *mles5,
                                  const uint64_t *fc0, const uint64_t *fc1, int K, size_t N, size_t wstride, int nv,
                                  int d, uint64_t *work, uint64_t *proof, uint64_t *randomness) {
  if (!c || !t || !cb || !mles5 || !fc0 || !fc1 || !work || !proof || !randomness || nv < 1 || K < 1)
    return LF_ERR_INVALID_ARG;
  DevGuard g(c);
  if (!ring_ok(d)) return fail(c, LF_ERR_UNSUPPORTED_RING, "unsupported ring degree");
  const int tau = d == 24 ? 3 : 1;
  if (cb->kind != LF_COMB_FOLDING || cb->bsmall != 2 || cb->nk != 2 * K || cb->tau != tau || N > ((size_t)1 << nv))
    return fail(c, LF_ERR_INVALID_ARG, "fold_digits: a folding combination with B_SMALL = 2 over 2K witnesses");
  lfk::CombS cs;
  const int nm = 5 + cb->nk * cb->tau;
  LF_TRY(comb_check(c, cb, nm, d, 4, &cs));
  const DigitFhat dg{fc0, fc1, K, N, wstride};
  return sumcheck_run(c, t, cb, cs, mles5, nullptr, work, nm, nv, d, 4, proof, randomness, &dg);
}

int lf_sumcheck_prove(lf_ctx *c, lf_transcript *t, const lf_comb *cb, uint64_t *mles, int nm, int nv, int d,
                      int degree, uint64_t *proof, uint64_t *randomness) {
  if (!c || !t || !mles || !proof || !randomness || nv < 1 || nm < 1) return LF_ERR_INVALID_ARG;
  DevGuard g(c);
  if (!ring_ok(d)) return fail(c, LF_ERR_UNSUPPORTED_RING, "unsupported ring degree");
  lfk::CombS cs;
  LF_TRY(comb_check(c, cb, nm, d, degree, &cs));
  return sumcheck_run(c, t, cb, cs, mles, nullptr, mles, nm, nv, d, degree, proof, randomness);
}

int lf_sumcheck_prove_ptrs(lf_ctx *c, lf_transcript *t, const lf_comb *cb, const uint64_t *const *mles, int nm, int nv,
                           int d, int degree, uint64_t *work, uint64_t *proof, uint64_t *randomness) {
  if (!c || !t || !mles || !work || !proof || !randomness || nv < 1 || nm < 1) return LF_ERR_INVALID_ARG;
  DevGuard g(c);
  if (!ring_ok(d)) return fail(c, LF_ERR_UNSUPPORTED_RING, "unsupported ring degree");
  for (int m = 0; m < nm; m++)
    if (!mles[m]) return fail(c, LF_ERR_INVALID_ARG, "null MLE pointer");
  lfk::CombS cs;
  LF_TRY(comb_check(c, cb, nm, d, degree, &cs));
  // the pointer table on the device, behind the scratch the rounds use
  LF_TRY(grow(c, c->ptrs, c->ptrs_elems, (size_t)nm));
  LF_HIP(c, hipMemcpyAsync(c->ptrs, mles, (size_t)nm * sizeof(uint64_t), hipMemcpyHostToDevice, c->cur));
  return sumcheck_run(c, t, cb, cs, nullptr, reinterpret_cast<const uint64_t *const *>(c->ptrs), work, nm, nv, d,
                      degree, proof, randomness);
}

// The linearization sumcheck over [mles..., eq(beta)] with eq(beta) split off
// (lfk::round_lin_eq): round i sums q_i(e) = sum_b E_i[b] inner(e, b) for e < degree
// on the device, E_i = eq(beta_(i+1) ..) over the unbound variables (E_0 an eq table,
// then pair sums); the host extrapolates q_i(degree) (q_i has degree < degree:
// q(n) = sum_(k<n) (-1)^(n-1-k) C(n, k) q(k)) and forms the message
//   p_i(e) = P_i eq(beta_i, e) q_i(e),  P_i = prod_(k<i) eq(beta_k, r_k),
// the same field elements as the unsplit round sums, so the transcript is the same.
static int sumcheck_run_lin(lf_ctx *c, lf_transcript *t, const lf_comb *cb, const lfk::CombS &cs,
                            const uint64_t *const *ptrs, uint64_t *alt, int nm, int nv, int d, int degree,
                            const uint64_t *beta, uint64_t *proof, uint64_t *randomness, uint64_t *evals,
                            const uint32_t *act = nullptr, const uint32_t *act_off = nullptr) {
  const int tb = lfk::slot_words(d), nev = degree + 1, nq = degree, ns = d / tb;
  const size_t n = (size_t)1 << nv;
  size_t part = 0;
  for (size_t h = n / 2; h >= 1; h /= 2) part = std::max(part, lfk::round_partial_elems(d, h, nq, cb->q));
  // sparse round 0: block g runs multiset bms[g] over act[boff[g] .. bend[g]), about 8
  // points per thread
  std::vector<uint32_t> blk;  // bms | boff | bend
  int nblk = 0;
  if (act) {
    const uint32_t per = (uint32_t)lfk::round_lin_sparse_ppb(d) * 8;
    std::vector<uint32_t> bms, bo, be;
    for (int i = 0; i < cs.q; i++)
      for (uint32_t p = act_off[i]; p < act_off[i + 1]; p += per) {
        bms.push_back((uint32_t)i);
        bo.push_back(p);
        be.push_back(std::min(p + per, act_off[i + 1]));
      }
    nblk = (int)bms.size();
    blk = bms;
    blk.insert(blk.end(), bo.begin(), bo.end());
    blk.insert(blk.end(), be.begin(), be.end());
    part = std::max(part, (size_t)nblk * nq * d);
  }
  const size_t fixed = (size_t)nm * (n / 2) * d, blk_elems = (blk.size() + 1) / 2;
  // scratch: fixed MLEs | partial sums | q | E tables (n/2 + n/4 + .. + 1 < n elements) | beta | blocks
  LF_TRY(grow(c, c->sc, c->sc_elems, fixed + part + (size_t)nq * d + n * d + (size_t)nv * d + blk_elems));
  uint64_t *buf = c->sc, *partial = buf + fixed, *qd = partial + part, *Et = qd + (size_t)nq * d,
           *bd = Et + n * d, *bk = bd + (size_t)nv * d;
  LF_HIP(c, hipMemcpyAsync(bd, beta, (size_t)nv * d * 8, hipMemcpyHostToDevice, c->cur));
  if (nblk) {  // through the pinned staging, grown here so no round frees it under the copy
    LF_TRY(pinned(c, std::max(blk_elems, (size_t)nq * d)));
    memcpy(c->hmsg, blk.data(), blk.size() * 4);
    LF_HIP(c, hipMemcpyAsync(bk, c->hmsg, blk.size() * 4, hipMemcpyHostToDevice, c->cur));
  }
  if (nv > 1) {
    LF_HIP(c, lfk::eq_table(bd + d, nv - 1, d, Et, c->cur));
  } else {
    std::vector<uint64_t> one(d, 0);
    for (int k = 0; k < d; k += tb) one[k] = 1;
    LF_HIP(c, hipMemcpyAsync(Et, one.data(), (size_t)d * 8, hipMemcpyHostToDevice, c->cur));
    LF_HIP(c, hipStreamSynchronize(c->cur));
  }
  // (-1)^(nq-1-k) C(nq, k): q(nq) from q(0 .. nq-1)
  std::vector<uint64_t> wext(nq);
  for (int k = 0; k < nq; k++) {
    uint64_t b = 1;
    for (int j = 0; j < k; j++) b = b * (uint64_t)(nq - j) / (uint64_t)(j + 1);
    wext[k] = (nq - 1 - k) % 2 ? gl::neg(b % gl::P) : b % gl::P;
  }
  auto bmul = [tb](const uint64_t *a, const uint64_t *b, uint64_t *o) {
    if (tb == 3) {
      uint64_t r[3];
      gl::fq3_mul(a, b, r);
      o[0] = r[0], o[1] = r[1], o[2] = r[2];
    } else {
      o[0] = gl::mul(a[0], b[0]);
    }
  };
  // eq(beta, x) = (1 - beta) + x (2 beta - 1) for a base-ring x
  auto eqv = [tb](const uint64_t *be, const uint64_t *x, uint64_t *o) {
    uint64_t a[3] = {0, 0, 0}, s[3] = {0, 0, 0};
    for (int w = 0; w < tb; w++) {
      a[w] = gl::neg(be[w]);
      s[w] = gl::add(be[w], be[w]);
    }
    a[0] = gl::add(a[0], 1);
    s[0] = gl::sub(s[0], 1);
    uint64_t m[3];
    if (tb == 3) {
      gl::fq3_mul(s, x, m);
    } else {
      m[0] = gl::mul(s[0], x[0]);
    }
    for (int w = 0; w < tb; w++) o[w] = gl::add(a[w], m[w]);
  };
  std::vector<uint64_t> scal(d, 0);
  for (int i = 0; i < d; i += tb) scal[i] = (uint64_t)nv;
  lf_transcript_absorb_ring(t, scal.data(), 1, d, LF_REPR_CANONICAL);
  for (int i = 0; i < d; i += tb) scal[i] = (uint64_t)degree;
  lf_transcript_absorb_ring(t, scal.data(), 1, d, LF_REPR_CANONICAL);
  std::vector<uint64_t> qh((size_t)nq * d);
  uint64_t pfx[3] = {1, 0, 0};
  const uint64_t *cur = nullptr;
  const uint64_t *const *cptrs = ptrs;
  size_t stride = 0;
  uint64_t *E = Et;
  for (int i = 0; i < nv; i++) {
    const size_t half = n >> (i + 1);
    uint64_t *msg = proof + (size_t)i * nev * d;
    if (i == 0 && act) {
      if (nblk) {
        const uint32_t *b32 = reinterpret_cast<const uint32_t *>(bk);
        LF_HIP(c, lfk::round_lin_eq_sparse(cptrs, E, cb->c, cs, degree, act, reinterpret_cast<const int *>(b32),
                                           b32 + nblk, b32 + 2 * nblk, nblk, d, partial, qd, c->cur));
      } else {
        LF_HIP(c, hipMemsetAsync(qd, 0, (size_t)nq * d * 8, c->cur));
      }
    } else {
      LF_HIP(c, lfk::round_lin_eq(cur, stride, E, cb->c, cs, degree, half, d, partial, qd, c->cur, cptrs));
    }
    LF_TRY(download_msg(c, qh.data(), qd, (size_t)nq * d));
    const uint64_t *be = beta + (size_t)i * d;  // slot 0 holds the base-ring value
    for (int e = 0; e < nev; e++) {
      uint64_t x[3] = {(uint64_t)e, 0, 0}, ev[3], f[3];
      eqv(be, x, ev);
      bmul(pfx, ev, f);
      for (int s = 0; s < ns; s++) {
        uint64_t qv[3] = {0, 0, 0};
        if (e < nq) {
          for (int w = 0; w < tb; w++) qv[w] = qh[(size_t)e * d + s * tb + w];
        } else {
          for (int k = 0; k < nq; k++)
            for (int w = 0; w < tb; w++) qv[w] = gl::add(qv[w], gl::mul(wext[k], qh[(size_t)k * d + s * tb + w]));
        }
        bmul(f, qv, msg + (size_t)e * d + s * tb);
      }
    }
    lf_transcript_absorb_ring(t, msg, (size_t)nev, d, LF_REPR_CANONICAL);
    uint64_t *ch = randomness + (size_t)i * tb;
    if (tb == 3) {
      lf_transcript_get_challenge(t, ch);
    } else {
      ch[0] = lf_transcript_sample(t);
      lf_transcript_observe(t, ch[0]);
    }
    for (int k = 0; k < d; k++) scal[k] = ch[k % tb];
    lf_transcript_absorb_ring(t, scal.data(), 1, d, LF_REPR_CANONICAL);
    {
      uint64_t ev[3], np[3];
      eqv(be, ch, ev);
      bmul(pfx, ev, np);
      for (int w = 0; w < tb; w++) pfx[w] = np[w];
    }
    if (i + 1 == nv && evals)  // the MLEs at the whole challenge point (the prover's final values)
      LF_HIP(c, lfk::mle_fix_first(cur, stride, nm, half, d, ch, evals, d, c->cur, cptrs));
    if (i + 1 < nv) {
      uint64_t *dst = (i % 2 == 0) ? buf : alt;
      LF_HIP(c, lfk::mle_fix_first(cur, stride, nm, half, d, ch, dst, half * d, c->cur, cptrs));
      LF_HIP(c, lfk::pair_sum(E, half / 2, d, E + half * d, c->cur));
      E += half * d;
      cur = dst;
      cptrs = nullptr;
      stride = half * d;
    }
  }
  return LF_OK;
}

int lf_sumcheck_prove_lin(lf_ctx *c, lf_transcript *t, const lf_comb *cb, const uint64_t *const *mles, int nm, int nv,
                          int d, int degree, const uint64_t *beta, uint64_t *work, uint64_t *proof,
                          uint64_t *randomness, uint64_t *evals) {
  if (!c || !t || !mles || !beta || !work || !proof || !randomness || nv < 1 || nm < 1) return LF_ERR_INVALID_ARG;
  DevGuard g(c);
  if (!ring_ok(d)) return fail(c, LF_ERR_UNSUPPORTED_RING, "unsupported ring degree");
  for (int m = 0; m < nm; m++)
    if (!mles[m]) return fail(c, LF_ERR_INVALID_ARG, "null MLE pointer");
  if (cb && cb->kind != LF_COMB_LINEARIZATION)
    return fail(c, LF_ERR_INVALID_ARG, "lf_sumcheck_prove_lin: a linearization combination");
  lfk::CombS cs;
  LF_TRY(comb_check(c, cb, nm + 1, d, degree, &cs));  // the list with eq(beta) last
  for (int i = 0; i < cs.q; i++)
    if (cs.off[i + 1] - cs.off[i] > degree - 1)
      return fail(c, LF_ERR_INVALID_ARG, "linearization sumcheck: a multiset of degree or more factors");
  LF_TRY(grow(c, c->ptrs, c->ptrs_elems, (size_t)nm));
  LF_HIP(c, hipMemcpyAsync(c->ptrs, mles, (size_t)nm * sizeof(uint64_t), hipMemcpyHostToDevice, c->cur));
  return sumcheck_run_lin(c, t, cb, cs, reinterpret_cast<const uint64_t *const *>(c->ptrs), work, nm, nv, d, degree,
                          beta, proof, randomness, evals);
}

int lf_sumcheck_prove_lin_sparse(lf_ctx *c, lf_transcript *t, const lf_comb *cb, const uint64_t *const *mles, int nm,
                                 int nv, int d, int degree, const uint64_t *beta, const uint32_t *act,
                                 const uint32_t *act_off, uint64_t *work, uint64_t *proof, uint64_t *randomness,
                                 uint64_t *evals) {
  if (!c || !t || !cb || !mles || !beta || !act || !act_off || !work || !proof || !randomness || nv < 1 || nm < 1)
    return LF_ERR_INVALID_ARG;
  DevGuard g(c);
  if (!ring_ok(d)) return fail(c, LF_ERR_UNSUPPORTED_RING, "unsupported ring degree");
  for (int m = 0; m < nm; m++)
    if (!mles[m]) return fail(c, LF_ERR_INVALID_ARG, "null MLE pointer");
  if (cb->kind != LF_COMB_LINEARIZATION)
    return fail(c, LF_ERR_INVALID_ARG, "lf_sumcheck_prove_lin_sparse: a linearization combination");
  lfk::CombS cs;
  LF_TRY(comb_check(c, cb, nm + 1, d, degree, &cs));
  for (int i = 0; i < cs.q; i++) {
    if (cs.off[i + 1] - cs.off[i] > degree - 1)
      return fail(c, LF_ERR_INVALID_ARG, "linearization sumcheck: a multiset of degree or more factors");
    if (act_off[i + 1] < act_off[i] || act_off[i + 1] - act_off[i] > ((size_t)1 << (nv - 1)))
      return fail(c, LF_ERR_INVALID_ARG, "sparse linearization: act_off must not decrease, at most 2^(nv-1) points each");
  }
  if (act_off[0] != 0) return fail(c, LF_ERR_INVALID_ARG, "sparse linearization: act_off[0] must be 0");
  LF_TRY(grow(c, c->ptrs, c->ptrs_elems, (size_t)nm));
  LF_HIP(c, hipMemcpyAsync(c->ptrs, mles, (size_t)nm * sizeof(uint64_t), hipMemcpyHostToDevice, c->cur));
  return sumcheck_run_lin(c, t, cb, cs, reinterpret_cast<const uint64_t *const *>(c->ptrs), work, nm, nv, d, degree,
                          beta, proof, randomness, evals, act, act_off);
}

// ---------------------------------------------------------------- sparse Mz products
void lf_ccs_destroy(lf_ccs *M) { delete M; }

int lf_ccs_shape(const lf_ccs *M, int *t, size_t *m, size_t *n, size_t *l, int *q, int *degree) {
  if (!M) return LF_ERR_INVALID_ARG;
  if (t) *t = M->dev.t;
  if (m) *m = M->dev.m;
  if (n) *n = M->dev.n;
  if (l) *l = M->l;
  if (q) *q = M->structured ? (int)M->S_off.size() - 1 : 0;
  if (degree) *degree = M->degree;
  return M->structured ? LF_OK : LF_ERR_INVALID_ARG;
}

int lf_ccs_get_structure(const lf_ccs *M, uint64_t *cc, int *S_off, int *S_idx) {
  if (!M || !M->structured) return LF_ERR_INVALID_ARG;
  if (cc) std::copy(M->c.begin(), M->c.end(), cc);
  if (S_off) std::copy(M->S_off.begin(), M->S_off.end(), S_off);
  if (S_idx) std::copy(M->S_idx.begin(), M->S_idx.end(), S_idx);
  return LF_OK;
}

const uint64_t *lf_ccs_c_device(const lf_ccs *M) { return M ? M->c_dev : nullptr; }

int lf_ccs_is_scalar(const lf_ccs *M) { return M && M->dev.sval ? 1 : 0; }

int lf_ccs_row_live(const lf_ccs *M, int j, uint8_t *out) {
  if (!M || !out || j < 0 || j >= M->dev.t) return LF_ERR_INVALID_ARG;
  std::copy(M->live.begin() + (size_t)j * M->dev.m, M->live.begin() + (size_t)(j + 1) * M->dev.m, out);
  return LF_OK;
}

int lf_ccs_set_structure(lf_ctx *c, lf_ccs *M, size_t l, int degree, int q, const uint64_t *cc, const int *S_off,
                         const int *S_idx, int repr) {
  if (!c || !M || q < 1 || !cc || !S_off || !S_idx || degree < 1) return LF_ERR_INVALID_ARG;
  DevGuard g(c);
  LF_TRY(check_repr(c, repr));
  const int d = M->dev.d;
  if (l + 1 > M->dev.n) return fail(c, LF_ERR_INVALID_ARG, "CCS: l + 1 > n");
  if (S_off[0] != 0) return fail(c, LF_ERR_INVALID_ARG, "CCS: S_off[0] must be 0");
  for (int i = 0; i < q; i++) {
    if (S_off[i + 1] < S_off[i]) return fail(c, LF_ERR_INVALID_ARG, "CCS: S_off must not decrease");
    if (S_off[i + 1] - S_off[i] > degree) return fail(c, LF_ERR_INVALID_ARG, "CCS: a multiset exceeds the degree");
  }
  for (int k = 0; k < S_off[q]; k++)
    if (S_idx[k] < 0 || S_idx[k] >= M->dev.t) return fail(c, LF_ERR_INVALID_ARG, "CCS: multiset index out of range");
  M->c.assign(cc, cc + (size_t)q * d);
  if (repr == LF_REPR_MONTGOMERY)
    for (auto &x : M->c) x = gl::from_mont(x);
  M->S_off.assign(S_off, S_off + q + 1);
  M->S_idx.assign(S_idx, S_idx + S_off[q]);
  M->l = l;
  M->degree = degree;
  if (!M->c_dev || M->c_dev_elems < (size_t)q * d) {
    void *p = nullptr;
    LF_HIP(c, hipMalloc(&p, (size_t)q * d * 8));
    M->bufs.push_back(p);
    M->c_dev = (uint64_t *)p;
    M->c_dev_elems = (size_t)q * d;
  }
  LF_HIP(c, hipMemcpyAsync(M->c_dev, M->c.data(), (size_t)q * d * 8, hipMemcpyHostToDevice, c->cur));
  LF_HIP(c, hipStreamSynchronize(c->cur));
  M->structured = true;
  return LF_OK;
}

// the largest pair of reordered ring-valued entry copies lf_ccs_create keeps (CcsDev::vh / vc)
constexpr size_t CCS_REORDER_BYTES = (size_t)16 << 30;

int lf_ccs_create(lf_ctx *c, int d, int t, size_t m, size_t n, const uint64_t *row_ptr, const uint32_t *col,
                  const uint64_t *val, int repr, lf_ccs **out) {
  if (!c || !out || t < 1 || !m || !n || !row_ptr) return LF_ERR_INVALID_ARG;
  DevGuard g(c);
  LF_TRY(check_repr(c, repr));
  if (!ring_ok(d)) return fail(c, LF_ERR_UNSUPPORTED_RING, "unsupported ring degree");
  *out = nullptr;
  const size_t nnz = row_ptr[(size_t)t * (m + 1) - 1];
  if (nnz >= (1ull << 32) || (nnz && (!col || !val)) || (size_t)t * n >= (1ull << 32))
    return fail(c, LF_ERR_INVALID_ARG, "CCS: nnz and t n must fit 32-bit indices");
  for (int j = 0; j < t; j++) {
    const uint64_t *rp = row_ptr + (size_t)j * (m + 1);
    for (size_t r = 0; r < m; r++)
      if (rp[r] > rp[r + 1]) return fail(c, LF_ERR_INVALID_ARG, "CCS: row offsets must not decrease");
    if (j && rp[0] != row_ptr[(size_t)j * (m + 1) - 1]) return fail(c, LF_ERR_INVALID_ARG, "CCS: matrices must be contiguous");
  }
  for (size_t k = 0; k < nnz; k++)
    if (col[k] >= n) return fail(c, LF_ERR_INVALID_ARG, "CCS: column index out of range");
  // the row-merged matrix (SparseMatrix::hconcat) and the per-matrix transposes
  std::vector<uint64_t> hrp(m + 1, 0), crp((size_t)t * (n + 1), 0);
  std::vector<uint32_t> hcol(nnz), hidx(nnz), crow(nnz), cidx(nnz);
  for (int j = 0; j < t; j++)
    for (size_t r = 0; r < m; r++) hrp[r + 1] += row_ptr[(size_t)j * (m + 1) + r + 1] - row_ptr[(size_t)j * (m + 1) + r];
  for (size_t r = 0; r < m; r++) hrp[r + 1] += hrp[r];
  {
    std::vector<uint64_t> fill(hrp.begin(), hrp.end() - 1);
    for (size_t r = 0; r < m; r++)
      for (int j = 0; j < t; j++)
        for (uint64_t k = row_ptr[(size_t)j * (m + 1) + r]; k < row_ptr[(size_t)j * (m + 1) + r + 1]; k++) {
          hcol[fill[r]] = (uint32_t)(j * n + col[k]);
          hidx[fill[r]++] = (uint32_t)k;
        }
  }
  for (int j = 0; j < t; j++) {
    uint64_t *cp = crp.data() + (size_t)j * (n + 1);
    const uint64_t *rp = row_ptr + (size_t)j * (m + 1);
    for (uint64_t k = rp[0]; k < rp[m]; k++) cp[col[k] + 1]++;
    cp[0] = rp[0];
    for (size_t q = 0; q < n; q++) cp[q + 1] += cp[q];
    std::vector<uint64_t> fill(cp, cp + n);
    for (size_t r = 0; r < m; r++)
      for (uint64_t k = rp[r]; k < rp[r + 1]; k++) {
        crow[fill[col[k]]] = (uint32_t)r;
        cidx[fill[col[k]]++] = (uint32_t)k;
      }
  }
  auto M = std::make_unique<lf_ccs>();
  M->device = c->device;
  M->live.resize((size_t)t * m);
  for (int j = 0; j < t; j++)
    for (size_t r = 0; r < m; r++)
      M->live[(size_t)j * m + r] = row_ptr[(size_t)j * (m + 1) + r + 1] > row_ptr[(size_t)j * (m + 1) + r];
  auto put = [&](const void *h, size_t bytes, void **dst) -> int {
    LF_HIP(c, hipMalloc(dst, bytes ? bytes : 8));
    M->bufs.push_back(*dst);
    if (bytes) LF_HIP(c, hipMemcpyAsync(*dst, h, bytes, hipMemcpyHostToDevice, c->cur));
    return LF_OK;
  };
  void *p;
  lfk::CcsDev &D = M->dev;
  D.d = d;
  D.t = t;
  D.m = m;
  D.n = n;
  LF_TRY(put(row_ptr, (size_t)t * (m + 1) * 8, &p));
  D.rp = (const uint64_t *)p;
  LF_TRY(put(col, nnz * 4, &p));
  D.col = (const uint32_t *)p;
  LF_TRY(put(val, nnz * d * 8, &p));
  D.val = (const uint64_t *)p;
  if (repr == LF_REPR_MONTGOMERY && nnz) LF_HIP(c, lfk::mont((uint64_t *)p, nnz * d, false, c->cur));
  {  // every entry a scalar (its value in word 0 of each slot, zero elsewhere: from_scalar,
     // ntt_form.rs:689-692)? then the products read one word per entry (CcsDev::sval)
    const int tb = lfk::slot_words(d);
    bool scalar = nnz > 0;
    for (size_t k = 0; k < nnz && scalar; k++) {
      const uint64_t *v = val + k * d;
      for (int w = 0; w < d; w++)
        if (v[w] != (w % tb == 0 ? v[0] : 0)) {
          scalar = false;
          break;
        }
    }
    if (scalar) {
      // also in the row-merged and transposed orders, so those products read them
      // sequentially instead of gathering one word per entry through hidx / cidx
      std::vector<uint64_t> sv(nnz), sh(nnz), sc(nnz);
      for (size_t k = 0; k < nnz; k++) sv[k] = val[k * d];
      for (size_t k = 0; k < nnz; k++) {
        sh[k] = sv[hidx[k]];
        sc[k] = sv[cidx[k]];
      }
      const uint64_t **dst[3] = {&D.sval, &D.svh, &D.svc};
      const std::vector<uint64_t> *src[3] = {&sv, &sh, &sc};
      for (int q = 0; q < 3; q++) {
        LF_TRY(put(src[q]->data(), nnz * 8, &p));
        *dst[q] = (const uint64_t *)p;
        if (repr == LF_REPR_MONTGOMERY) LF_HIP(c, lfk::mont((uint64_t *)p, nnz, false, c->cur));
      }
      LF_HIP(c, hipStreamSynchronize(c->cur));  // the host vectors go out of scope
    }
  }
  LF_TRY(put(hrp.data(), hrp.size() * 8, &p));
  D.hrp = (const uint64_t *)p;
  LF_TRY(put(hcol.data(), nnz * 4, &p));
  D.hcol = (const uint32_t *)p;
  LF_TRY(put(hidx.data(), nnz * 4, &p));
  D.hidx = (const uint32_t *)p;
  LF_TRY(put(crp.data(), crp.size() * 8, &p));
  D.crp = (const uint64_t *)p;
  LF_TRY(put(crow.data(), nnz * 4, &p));
  D.crow = (const uint32_t *)p;
  LF_TRY(put(cidx.data(), nnz * 4, &p));
  D.cidx = (const uint32_t *)p;
  // ring-valued entries: copies in the row-merged and transposes' orders, so the
  // challenged pass and the Mz weights read their values sequentially instead of
  // gathering d words per entry through hidx / cidx (at the zkvm's shape 2 x 3.15 GB;
  // above CCS_REORDER_BYTES the gathers stay)
  if (!D.sval && nnz && 2 * nnz * d * 8 <= CCS_REORDER_BYTES) {
    const uint32_t *ix[2] = {D.hidx, D.cidx};
    const uint64_t **dst[2] = {&D.vh, &D.vc};
    for (int q = 0; q < 2; q++) {
      LF_HIP(c, hipMalloc(&p, nnz * d * 8));
      M->bufs.push_back(p);
      LF_HIP(c, lfk::gather_entries(D.val, ix[q], nnz, d, (uint64_t *)p, c->cur));
      *dst[q] = (const uint64_t *)p;
    }
  }
  LF_HIP(c, hipStreamSynchronize(c->cur));  // the host vectors go out of scope
  *out = M.release();
  return LF_OK;
}

static int mz_check(lf_ctx *c, const lf_ccs *M, int nz, int nv) {
  if (!M || nz < 1 || nv < 1) return fail(c, LF_ERR_INVALID_ARG, "CCS products: null matrices or no vectors");
  if (M->device != c->device) return fail(c, LF_ERR_INVALID_ARG, "CCS matrices live on another device");
  if (M->dev.m > ((size_t)1 << nv)) return fail(c, LF_ERR_INVALID_ARG, "MLE too short for m rows (to_mles_err)");
  return LF_OK;
}

int lf_dev_mz_mles(lf_ctx *c, const lf_ccs *M, const uint64_t *z, int nz, int nv, uint64_t *out) {
  if (!c || !z || !out) return LF_ERR_INVALID_ARG;
  DevGuard g(c);
  LF_TRY(mz_check(c, M, nz, nv));
  LF_HIP(c, lfk::mz_mles(M->dev, z, nz, nv, out, c->cur));
  return LF_OK;
}

int lf_dev_mz_mles_sel(lf_ctx *c, const lf_ccs *M, const uint64_t *z, const int *sel, int nsel, int nv,
                       uint64_t *out) {
  if (!c || !z || !out || (!sel && nsel) || nsel < 0) return LF_ERR_INVALID_ARG;
  DevGuard g(c);
  LF_TRY(mz_check(c, M, 1, nv));
  for (int i = 0; i < nsel; i++)
    if (sel[i] < 0 || sel[i] >= M->dev.t) return fail(c, LF_ERR_INVALID_ARG, "matrix index out of range");
  if (!nsel) return LF_OK;
  LF_TRY(grow(c, c->sel, c->sel_elems, (size_t)nsel));
  LF_HIP(c, hipMemcpyAsync(c->sel, sel, (size_t)nsel * sizeof(int), hipMemcpyHostToDevice, c->cur));
  LF_HIP(c, lfk::mz_mles(M->dev, z, 1, nv, out, c->cur, c->sel, nsel));
  return LF_OK;
}

int lf_dev_mz_challenged(lf_ctx *c, const lf_ccs *M, const uint64_t *z, const uint64_t *zeta, int nz, int nv,
                         uint64_t *out) {
  if (!c || !z || !zeta || !out) return LF_ERR_INVALID_ARG;
  DevGuard g(c);
  LF_TRY(mz_check(c, M, nz, nv));
  LF_TRY(grow(c, c->tmp, c->tmp_elems, lfk::mz_scratch_elems(M->dev, nz, nv)));
  LF_HIP(c, lfk::mz_challenged(M->dev, z, zeta, nz, nv, out, c->tmp, c->cur));
  return LF_OK;
}

int lf_dev_mz_challenged_pair(lf_ctx *c, const lf_ccs *M, const uint64_t *z0, const uint64_t *zeta0,
                              const uint64_t *z1, const uint64_t *zeta1, int nz, int nv, uint64_t *out0,
                              uint64_t *out1) {
  if (!c || !z0 || !zeta0 || !z1 || !zeta1 || !out0 || !out1) return LF_ERR_INVALID_ARG;
  DevGuard g(c);
  LF_TRY(mz_check(c, M, nz, nv));
  const lfk::CcsDev &D = M->dev;
  LF_TRY(grow(c, c->tmp, c->tmp_elems, 2 * lfk::mz_chall_elems(D, nz)));
  LF_HIP(c, lfk::mz_challenged_pair(D, z0, zeta0, z1, zeta1, nz, nv, out0, out1, c->tmp, c->cur));
  return LF_OK;
}

int lf_dev_mz_evaluate(lf_ctx *c, const lf_ccs *M, const uint64_t *z, int nz, int nv, const uint64_t *point,
                       uint64_t *out) {
  if (!c || !z || !point || !out) return LF_ERR_INVALID_ARG;
  DevGuard g(c);
  LF_TRY(mz_check(c, M, nz, nv));
  LF_TRY(grow(c, c->tmp, c->tmp_elems, lfk::mz_scratch_elems(M->dev, nz, nv)));
  LF_HIP(c, lfk::mz_evaluate(M->dev, z, nz, nv, point, out, c->tmp, c->cur));
  return LF_OK;
}

int lf_dev_mz_weights(lf_ctx *c, const lf_ccs *M, int nv, const uint64_t *eq, uint64_t *w) {
  if (!c || !eq || !w) return LF_ERR_INVALID_ARG;
  DevGuard g(c);
  LF_TRY(mz_check(c, M, 1, nv));
  LF_HIP(c, lfk::mz_weights(M->dev, eq, w, c->cur));
  return LF_OK;
}

int lf_dev_mz_dots(lf_ctx *c, const lf_ccs *M, const uint64_t *w, const uint64_t *z, int nz, uint64_t *out) {
  if (!c || !M || !w || !z || !out || nz < 1) return LF_ERR_INVALID_ARG;
  DevGuard g(c);
  LF_TRY(grow(c, c->tmp, c->tmp_elems, lfk::mz_dots_partial_elems(M->dev, nz)));
  LF_HIP(c, lfk::mz_dots(M->dev, w, z, nz, out, c->cur, c->tmp));
  return LF_OK;
}

size_t lf_ccs_weights_len(const lf_ccs *M) { return M ? (size_t)M->dev.t * M->dev.n * M->dev.d : 0; }

// ---------------------------------------------------------------- width-8 Poseidon2 Merkle trees
int lf_dev_poseidon2_w8_permute(lf_ctx *c, uint64_t *states, size_t n) {
  if (!c || (!states && n)) return LF_ERR_INVALID_ARG;
  DevGuard g(c);
  LF_HIP(c, lfk::p2w8_permute(states, n, c->cur));
  return LF_OK;
}

size_t lf_merkle_nodes_len(size_t nrows) { return nrows ? lfk::merkle_nodes(nrows) : 0; }

int lf_dev_merkle_tree(lf_ctx *c, const uint64_t *rows, size_t nrows, size_t width, uint64_t *nodes) {
  if (!c || !rows || !nodes || !width || !nrows)
    return c ? fail(c, LF_ERR_INVALID_ARG, "Merkle tree: at least one row of width >= 1") : LF_ERR_INVALID_ARG;
  DevGuard g(c);
  LF_HIP(c, lfk::merkle_tree(rows, nrows, width, nodes, c->cur));
  return LF_OK;
}

int lf_dev_hash_w8_rows(lf_ctx *c, const uint64_t *rows, size_t nrows, size_t width, uint64_t *out) {
  if (!c || (nrows && (!out || (width && !rows)))) return LF_ERR_INVALID_ARG;
  DevGuard g(c);
  LF_HIP(c, lfk::hash_w8_rows(rows, nrows, width, out, c->cur));
  return LF_OK;
}

int lf_merkle_open(lf_ctx *c, const uint64_t *nodes, size_t nrows, size_t index, uint64_t *path) {
  if (!c || !nodes || !path || !nrows || index >= nrows) return LF_ERR_INVALID_ARG;
  DevGuard g(c);
  // the sibling of the node on the path in every padded layer below the root,
  // leaves first (open_batch's opening_proof; a zero digest where the layer was padded)
  size_t off = 0, n = nrows <= 1 ? 1 : nrows + nrows % 2, i = index, k = 0;
  while (n > 1) {
    LF_HIP(c, hipMemcpyAsync(path + 4 * k, nodes + 4 * (off + (i ^ 1)), 32, hipMemcpyDeviceToHost, c->cur));
    off += n;
    n = n == 2 ? 1 : ((n / 2 + 1) & ~(size_t)1);
    i /= 2;
    k++;
  }
  LF_HIP(c, hipStreamSynchronize(c->cur));
  return LF_OK;
}

int lf_vm_code_comm(lf_ctx *c, const uint8_t *code, size_t len, uint64_t out4[4]) {
  if (!c || !out4 || (len && !code)) return LF_ERR_INVALID_ARG;
  if (!len) return fail(c, LF_ERR_INVALID_ARG, "vm_code_comm: empty code (the reference asserts)");
  DevGuard g(c);
  // little-endian 16-bit half-words, an odd last byte padded with zero (commitments.rs:316-328)
  const size_t nh = (len + 1) / 2;
  std::vector<uint64_t> hw(nh);
  for (size_t i = 0; i < nh; i++) hw[i] = code[2 * i] | (2 * i + 1 < len ? (uint64_t)code[2 * i + 1] << 8 : 0);
  DevBuf dr, dn;
  LF_TRY(upload(c, dr, hw.data(), nh, LF_REPR_CANONICAL));
  const size_t nn = lfk::merkle_nodes(nh);
  LF_TRY(dev_alloc(c, dn, 4 * nn));
  LF_HIP(c, lfk::merkle_tree(dr.p, nh, 1, dn.p, c->cur));
  LF_HIP(c, hipMemcpyAsync(out4, dn.p + 4 * (nn - 1), 32, hipMemcpyDeviceToHost, c->cur));
  LF_HIP(c, hipStreamSynchronize(c->cur));
  return LF_OK;
}

int lf_dev_expand_planes(lf_ctx *c, const lf_params *pr, const uint64_t *planes, size_t N, uint64_t *fck,
                         uint64_t *fk) {
  if (!c) return LF_ERR_INVALID_ARG;
  DevGuard g(c);
  int lb, lbs;
  LF_TRY(check_params(c, pr, lb, lbs));
  const int d = pr->d, K = pr->K;
  if (!planes && N) return fail(c, LF_ERR_INVALID_ARG, "planes is NULL");
  if (lbs != 1) return fail(c, LF_ERR_INVALID_ARG, "packed planes need b_small = 2");
  if (d == 24) {  // [K][N] digit masks
    LF_HIP(c, lfk::expand_phi72(reinterpret_cast<const uint2 *>(planes), (size_t)K * N, fck, fk, c->cur));
    return LF_OK;
  }
  if ((d != 1024 && d != 4096) || K > 15) return fail(c, LF_ERR_UNSUPPORTED_RING, "packed planes: d = 24, 1024 or 4096");
  if (!fck && !fk) return LF_OK;
  // sign|magnitude words (d = 4096: the digit bytes) -> f_coeff_k, then f_k = NTT(f_coeff_k)
  // (CRT::elementwise_crt)
  uint64_t *dst = fck ? fck : fk;
  if (d == 1024)
    LF_HIP(c, lfk::expand_sm(reinterpret_cast<const uint32_t *>(planes), N, K, dst, c->cur));
  else
    LF_HIP(c, lfk::expand_sm8(reinterpret_cast<const uint32_t *>(planes), N, K, dst, c->cur));
  if (fk) {
    if (fck) LF_HIP(c, hipMemcpyAsync(fk, fck, (size_t)K * N * d * 8, hipMemcpyDeviceToDevice, c->cur));
    LF_TRY(lf_dev_crt(c, fk, (size_t)K * N, d));
  }
  return LF_OK;
}

int lf_dev_fold_step(lf_ctx *c, const lf_ajtai *aj, const lf_params *pr, size_t W, const lf_fold_step_bufs *b) {
  DevGuard g(c);
  int lb, lbs;
  LF_TRY(step_check(c, aj, pr, W, b, lb, lbs));
  LF_TRY(step_commit(c, aj, pr, W, b, lb, lbs, fold_dst(pr, b, aj->kappa * (size_t)pr->d, b->cm)));
  return fold_finish(c, aj, pr, lb, lbs, W, b, b->cm);
}

// nsteps independent steps (one context, stream and buffer set each): every
// step's commit and decompositions on its own stream, one contraction of all of
// them on ctx[0]'s stream (ajtai_mfma_steps: A read from HBM once), then every
// step's fold_finish on its own stream again. Events order the streams; nothing
// waits on the host.
int lf_dev_fold_step_batch(lf_ctx *const *cs, int nsteps, const lf_ajtai *aj, const lf_params *pr, size_t W,
                           const lf_fold_step_bufs *const *bs) {
  if (!cs || !bs || !aj || nsteps < 1 || nsteps > LF_MAX_STEPS || !cs[0]) return LF_ERR_INVALID_ARG;
  lf_ctx *c0 = cs[0];
  for (int s = 0; s < nsteps; s++) {
    if (!cs[s] || !bs[s]) return fail(c0, LF_ERR_INVALID_ARG, "null context or step buffers");
    if (cs[s]->device != aj->device) return fail(c0, LF_ERR_INVALID_ARG, "every context must be on the scheme's device");
    for (int t = 0; t < s; t++)
      if (cs[t] == cs[s]) return fail(c0, LF_ERR_INVALID_ARG, "each step needs its own context");
  }
  if (nsteps == 1) return lf_dev_fold_step(c0, aj, pr, W, bs[0]);
  DevGuard g(c0);
  int lb = 0, lbs = 0;
  for (int s = 0; s < nsteps; s++) LF_TRY(step_check(cs[s], aj, pr, W, bs[s], lb, lbs));
  const size_t kd = aj->kappa * (size_t)pr->d;
  Deferred dfr[LF_MAX_STEPS];
  for (int s = 0; s < nsteps; s++) {
    DevGuard gs(cs[s]);
    LF_TRY(step_commit(cs[s], aj, pr, W, bs[s], lb, lbs, fold_dst(pr, bs[s], kd, bs[s]->cm), &dfr[s]));
  }
  // steps whose path has no fragments contracted on their own already
  const uint4 *ff[LF_MAX_STEPS];
  uint64_t *pp[LF_MAX_STEPS];
  lfk::OutPtrs dd[LF_MAX_STEPS];
  lfk::DeadUnits du[LF_MAX_STEPS];
  int n = 0, nvec = 0;
  for (int s = 0; s < nsteps; s++) {
    if (!dfr[s].set) continue;
    ff[n] = dfr[s].Ff;
    pp[n] = dfr[s].partial;
    dd[n] = dfr[s].dst;
    du[n] = dfr[s].dead;
    nvec = dfr[s].nvec;
    n++;
  }
  for (int s = 0; s < nsteps; s++)
    if (!cs[s]->join) LF_HIP(cs[s], hipEventCreateWithFlags(&cs[s]->join, hipEventDisableTiming));
  if (n) {
    // the contraction runs on c0's stream, or on c0's contraction stream when one
    // is set (lf_ctx_set_contract_stream: e.g. a CU-masked stream beside the step
    // streams' CUs), after every step stream's decomposition
    const hipStream_t cst = c0->contract ? c0->contract : c0->cur;
    for (int s = c0->contract ? 0 : 1; s < nsteps; s++) {
      LF_HIP(c0, hipEventRecord(cs[s]->join, cs[s]->cur));
      LF_HIP(c0, hipStreamWaitEvent(cst, cs[s]->join, 0));
    }
    hipEvent_t ea = nullptr, eb = nullptr;
    if (c0->timing) {
      LF_HIP(c0, hipEventCreate(&ea));
      LF_HIP(c0, hipEventCreate(&eb));
    }
    LF_HIP(c0, lfk::ajtai_mfma_steps(aj->Af, aj->kr, aj->kappa, aj->geom, pr->d, nvec, n, ff, pp, dd, cst, ea, eb, du,
                                     c0->zero80));
    if (c0->timing) c0->pending.push_back({ea, eb, nvec, n});
    if (c0->contract) {
      if (!c0->cjoin) LF_HIP(c0, hipEventCreateWithFlags(&c0->cjoin, hipEventDisableTiming));
      LF_HIP(c0, hipEventRecord(c0->cjoin, cst));
      for (int s = 0; s < nsteps; s++) LF_HIP(cs[s], hipStreamWaitEvent(cs[s]->cur, c0->cjoin, 0));
    } else {
      LF_HIP(c0, hipEventRecord(c0->join, c0->cur));
      for (int s = 1; s < nsteps; s++) LF_HIP(cs[s], hipStreamWaitEvent(cs[s]->cur, c0->join, 0));
    }
  }
  for (int s = 0; s < nsteps; s++) {
    DevGuard gs(cs[s]);
    LF_TRY(fold_finish(cs[s], aj, pr, lb, lbs, W, bs[s], bs[s]->cm));
  }
  return LF_OK;
}

size_t lf_fold_step_partial_len(const lf_ajtai *aj, const lf_params *pr) {
  return aj && pr ? (size_t)fold_nvec(pr, true) * aj->kappa * pr->d : 0;
}

int lf_dev_fold_step_partial(lf_ctx *c, const lf_ajtai *aj, const lf_params *pr, size_t W,
                             const lf_fold_step_bufs *b, uint64_t *partial) {
  DevGuard g(c);
  int lb, lbs;
  LF_TRY(step_check(c, aj, pr, W, b, lb, lbs));
  if (!partial) return fail(c, LF_ERR_INVALID_ARG, "null partial buffer");
  const size_t kd = aj->kappa * (size_t)pr->d;
  lfk::OutPtrs dst{};
  for (int v = 0; v < fold_nvec(pr, true); v++) dst.p[v] = partial + v * kd;
  return step_commit(c, aj, pr, W, b, lb, lbs, dst);
}

int lf_dev_fold_step_finish(lf_ctx *c, const lf_ajtai *aj, const lf_params *pr, size_t W,
                            const lf_fold_step_bufs *b, const uint64_t *partial_sum) {
  DevGuard g(c);
  int lb, lbs;
  LF_TRY(step_check(c, aj, pr, W, b, lb, lbs));
  if (!partial_sum) return fail(c, LF_ERR_INVALID_ARG, "null partial sum");
  const size_t kd = aj->kappa * (size_t)pr->d;
  const lfk::OutPtrs dst = fold_dst(pr, b, kd, b->cm);
  for (int v = 0; v < fold_nvec(pr, true); v++)
    LF_HIP(c, hipMemcpyAsync(dst.p[v], partial_sum + v * kd, kd * 8, hipMemcpyDeviceToDevice, c->cur));
  return fold_finish(c, aj, pr, lb, lbs, W, b, b->cm);
}

// the decomposition half of fold() without commit(z): both sides' decompose_witness
// and commit_witnesses (decomposition.rs:162-201), y_0 included; inputs
// acc_f_coeff / acc_cm (accumulator) and f_coeff / cm (the linearized instance)
int lf_dev_decompose_commit(lf_ctx *c, const lf_ajtai *aj, const lf_params *pr, size_t W,
                            const lf_fold_step_bufs *b) {
  DevGuard g(c);
  int lb, lbs;
  LF_TRY(step_check(c, aj, pr, W, b, lb, lbs));
  if (!b->acc_f_coeff || !b->f_coeff || !b->acc_cm || !b->cm || !b->y[0] || !b->y[1] || !b->wk[0] || !b->wk[1])
    return fail(c, LF_ERR_INVALID_ARG, "decompose_commit: missing buffer");
  const size_t kd = aj->kappa * (size_t)pr->d;
  LF_TRY(fold_commit(c, aj, pr, lb, lbs, W, b, b->f_coeff, nullptr, fold_dst(pr, b, kd, nullptr)));
  for (int s = 0; s < 2; s++)
    LF_HIP(c, lfk::commit_y0(s ? b->cm : b->acc_cm, b->y[s], aj->kappa, pr->d, lbs, pr->K, c->cur));
  return LF_OK;
}

// the folding half, given rho: cm_0, f_0 and Witness::from_f(f_0) (folding.rs:112-122);
// right after lf_dev_decompose_commit on the same context and buffers
int lf_dev_fold_combine(lf_ctx *c, const lf_ajtai *aj, const lf_params *pr, size_t W, const lf_fold_step_bufs *b) {
  DevGuard g(c);
  int lb, lbs;
  LF_TRY(step_check(c, aj, pr, W, b, lb, lbs));
  if (!b->rho || !b->f0 || !b->f0_coeff || !b->w_ccs0 || !b->cm0) return fail(c, LF_ERR_INVALID_ARG, "fold_combine: missing buffer");
  return fold_finish(c, aj, pr, lb, lbs, W, b, b->cm);
}

int lf_dev_fold_step_sharded(lf_ctx *c, const lf_ajtai *aj, const lf_params *pr, size_t W,
                             const lf_fold_step_bufs *b, lf_comm *cm) {
  DevGuard g(c);
  int lb, lbs;
  LF_TRY(step_check(c, aj, pr, W, b, lb, lbs));
  if (!cm || !cm->comm) return lf_dev_fold_step(c, aj, pr, W, b);
  const size_t len = lf_fold_step_partial_len(aj, pr);
  LF_TRY(grow(c, c->stage, c->stage_elems, len));
  LF_TRY(lf_dev_fold_step_partial(c, aj, pr, W, b, c->stage));
  LF_TRY(allreduce_modp(c, cm, c->stage, len));
  return lf_dev_fold_step_finish(c, aj, pr, W, b, c->stage);
}

// ---------------------------------------------------------------- communicators
int lf_comm_unique_id(uint8_t *id, size_t len) {
  if (!id || len != NCCL_UNIQUE_ID_BYTES) return LF_ERR_INVALID_ARG;
  if (!rccl().ok) return LF_ERR_COMM;
  ncclUniqueId u;
  if (rccl().getUniqueId(&u) != ncclSuccess) return LF_ERR_COMM;
  memcpy(id, u.internal, NCCL_UNIQUE_ID_BYTES);
  return LF_OK;
}

int lf_comm_init(lf_ctx *c, int nranks, int rank, const uint8_t *id, size_t len, lf_comm **out) {
  if (!c || !out || nranks < 1 || rank < 0 || rank >= nranks || (nranks > 1 && !id) ||
      (id && len != NCCL_UNIQUE_ID_BYTES))
    return LF_ERR_INVALID_ARG;
  DevGuard g(c);
  *out = nullptr;
  auto cm = std::make_unique<lf_comm>();
  cm->nranks = nranks;
  cm->rank = rank;
  if (id) {  // one rank with an id still makes a (trivial) RCCL communicator
    if (!rccl().ok) return fail(c, LF_ERR_COMM, rccl().err);
    ncclUniqueId u;
    memcpy(u.internal, id, NCCL_UNIQUE_ID_BYTES);
    LF_NCCL(c, rccl().commInitRank(&cm->comm, nranks, u, rank));
    cm->owned = true;
  }
  *out = cm.release();
  return LF_OK;
}

int lf_comm_wrap(lf_ctx *c, void *nccl_comm, lf_comm **out) {
  if (!c || !nccl_comm || !out) return LF_ERR_INVALID_ARG;
  DevGuard g(c);
  if (!rccl().ok) return fail(c, LF_ERR_COMM, rccl().err);
  auto cm = std::make_unique<lf_comm>();
  cm->comm = (ncclComm_t)nccl_comm;
  LF_NCCL(c, rccl().commCount(cm->comm, &cm->nranks));
  LF_NCCL(c, rccl().commUserRank(cm->comm, &cm->rank));
  *out = cm.release();
  return LF_OK;
}

void lf_comm_destroy(lf_comm *cm) {
  if (!cm) return;
  if (cm->owned && cm->comm && rccl().ok) (void)rccl().commDestroy(cm->comm);
  delete cm;
}
int lf_comm_size(const lf_comm *cm) { return cm ? cm->nranks : 0; }
int lf_comm_rank(const lf_comm *cm) { return cm ? cm->rank : -1; }

int lf_comm_allreduce_modp(lf_ctx *c, lf_comm *cm, uint64_t *x, size_t n) {
  if (!c || !cm || (!x && n)) return LF_ERR_INVALID_ARG;
  DevGuard g(c);
  return allreduce_modp(c, cm, x, n);
}

int lf_fold_reduce_allranks(lf_ctx *c, lf_comm *cm, uint64_t *cm0, size_t cm0_len, uint64_t *f0, size_t f0_len) {
  if (!c || !cm) return LF_ERR_INVALID_ARG;
  DevGuard g(c);
  LF_TRY(allreduce_modp(c, cm, cm0, cm0_len));
  return allreduce_modp(c, cm, f0, f0_len);
}

int lf_dev_poseidon2_permute(lf_ctx *c, uint64_t *states, size_t n) {
  DevGuard g(c);
  if (!c) return LF_ERR_INVALID_ARG;
  LF_HIP(c, lfk::p2_permute(states, n, c->cur));
  return LF_OK;
}

int lf_dev_poseidon2_permute_rounds(lf_ctx *c, uint64_t *states, size_t n, int rounds) {
  if (!c || (!states && n) || rounds < 0 || rounds > 30) return LF_ERR_INVALID_ARG;
  DevGuard g(c);
  LF_HIP(c, lfk::p2_permute(states, n, c->cur, rounds));
  return LF_OK;
}
int lf_dev_fill_uniform(lf_ctx *c, uint64_t *out, size_t n, uint64_t seed) {
  DevGuard g(c);
  if (!c) return LF_ERR_INVALID_ARG;
  LF_HIP(c, lfk::fill_uniform(out, n, seed, c->cur));
  return LF_OK;
}
int lf_dev_modp_sum(lf_ctx *c, const uint64_t *in, int nparts, size_t len, uint64_t *out) {
  DevGuard g(c);
  if (!c || nparts < 1) return LF_ERR_INVALID_ARG;
  LF_HIP(c, lfk::modp_sum(in, nparts, len, out, c->cur));
  return LF_OK;
}

int lf_dev_limb_split(lf_ctx *c, const uint64_t *x, size_t n, uint64_t *lo, uint64_t *hi) {
  DevGuard g(c);
  if (!c) return LF_ERR_INVALID_ARG;
  LF_HIP(c, lfk::limb_split(x, n, lo, hi, c->cur));
  return LF_OK;
}
int lf_dev_limb_join(lf_ctx *c, const uint64_t *lo, const uint64_t *hi, size_t n, uint64_t *out) {
  DevGuard g(c);
  if (!c) return LF_ERR_INVALID_ARG;
  LF_HIP(c, lfk::limb_join(lo, hi, n, out, c->cur));
  return LF_OK;
}

}  // extern "C"
