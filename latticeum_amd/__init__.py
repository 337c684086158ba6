"""latticeum_amd -- MI355X-native LatticeFold commit+fold hot path.

Thin Python view of the C ABI (include/lf.h). The names follow the reference
(Nesquiko/Latticeum): ``AjtaiCommitmentScheme`` (latticefold
commitment_scheme.rs), ``Witness.from_w_ccs / from_f`` (latticefold arith.rs),
``commit`` / ``fold`` (zkvm main.rs:348,380), ``Poseidon2Transcript``
(zkvm fiat_shamir.rs). Every operation runs through the HIP library; there is
no CPU fallback, and constructing a ``Context`` fails without a GPU.

Host arrays are numpy uint64 in AoS layout (``[n, d]`` ring elements). Device
arrays are torch int64 tensors on a HIP device (bit patterns of u64).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from ._lib import LfComb, LfFoldStepBufs, LfParams, load

P = (1 << 64) - (1 << 32) + 1
REPR_CANONICAL = 0
REPR_MONTGOMERY = 1
SUPPORTED_D = (24, 16, 64, 256, 1024, 4096)


class LfError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"lf error {code}: {msg}")
        self.code = code


def goldilocks_dp(d: int = 24) -> LfParams:
    """zkvm GoldiLocksDP (zkvm/src/ccs.rs:26-34): B=2^15, L=5, B_SMALL=2, K=15."""
    return load().lf_goldilocks_dp(d)


def _u64(a) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a, dtype=np.uint64))


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


def _dptr(t) -> int:
    """device pointer of a torch tensor (or a raw int)."""
    return t if isinstance(t, int) else t.data_ptr()


class Context:
    """One HIP device + stream (lf_ctx). Not thread-safe; one per thread."""

    def __init__(self, device: int = 0):
        self.lib = load()
        h = C.c_void_p()
        rc = self.lib.lf_ctx_create(device, C.byref(h))
        if rc != 0:
            raise LfError(rc, f"lf_ctx_create(device={device}) failed: "
                              f"{self.lib.lf_status_string(rc).decode()}")
        self.h = h
        self.device = device

    def close(self):
        if getattr(self, "h", None):
            self.lib.lf_ctx_destroy(self.h)  # synchronises the current stream first
            self.h = None
        for st in getattr(self, "_masked", []):
            self.lib.lf_stream_destroy(st)
        self._masked = []

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def check(self, rc: int):
        if rc != 0:
            msg = self.lib.lf_ctx_last_error(self.h).decode() or self.lib.lf_status_string(rc).decode()
            raise LfError(rc, msg)

    # ---------------------------------------------------------------- stream / timing
    def set_stream(self, hip_stream: int | None):
        self.check(self.lib.lf_ctx_set_stream(self.h, hip_stream))

    def sync(self):
        self.check(self.lib.lf_ctx_sync(self.h))

    def use_cu_mask(self, cus):
        """run this context's work on a stream of its own restricted to the
        compute units `cus` (iterable of CU indices); lf_stream_create_cu_mask"""
        cus = list(cus)
        st = self.cu_mask_stream(cus)
        self.set_stream(st)
        self.check(self.lib.lf_ctx_set_cu_count(self.h, len(set(cus))))
        return st

    def set_contract_stream(self, hip_stream: int | None):
        """where dev_fold_step_batch led by this context runs the group's
        contraction (lf_ctx_set_contract_stream; None: this context's stream)"""
        self.check(self.lib.lf_ctx_set_contract_stream(self.h, hip_stream))

    def cu_mask_stream(self, cus):
        """a stream of this context's device restricted to the compute units
        `cus`, released with the context (lf_stream_create_cu_mask)"""
        cus = list(cus)
        words = (max(cus) // 32 + 1) if cus else 1
        mask = (C.c_uint32 * words)()
        for i in cus:
            mask[i // 32] |= 1 << (i % 32)
        st = C.c_void_p()
        rc = self.lib.lf_stream_create_cu_mask(self.device, mask, words, C.byref(st))
        if rc != 0:
            raise LfError(rc, "lf_stream_create_cu_mask")
        self._masked = getattr(self, "_masked", []) + [st.value]
        return st.value

    def reserve(self, kappa: int, ncols: int, d: int, nvec: int):
        self.check(self.lib.lf_ctx_reserve(self.h, kappa, ncols, d, nvec))

    def kernel_timing(self, enable: bool):
        self.check(self.lib.lf_ctx_kernel_timing(self.h, int(enable)))

    def kernel_stats(self, nvec: int = 0):
        ms, cnt = C.c_double(), C.c_long()
        self.check(self.lib.lf_ctx_kernel_stats(self.h, nvec, C.byref(ms), C.byref(cnt)))
        return ms.value, cnt.value

    PHASES = ("from_w_ccs", "decompose", "to_frag", "fold", "from_f")  # lf.h LF_PHASE_*

    def phase_stats(self, phase: str):
        ms, cnt = C.c_double(), C.c_long()
        self.check(self.lib.lf_ctx_phase_stats(self.h, self.PHASES.index(phase), C.byref(ms), C.byref(cnt)))
        return ms.value, cnt.value

    # ---------------------------------------------------------------- host-buffer API
    def crt(self, elems, d: int, repr: int = REPR_CANONICAL) -> np.ndarray:
        x = _u64(elems).copy()
        self.check(self.lib.lf_crt(self.h, _ptr(x), x.size // d, d, repr))
        return x

    def icrt(self, elems, d: int, repr: int = REPR_CANONICAL) -> np.ndarray:
        x = _u64(elems).copy()
        self.check(self.lib.lf_icrt(self.h, _ptr(x), x.size // d, d, repr))
        return x

    def ring_mul(self, a, b, d: int, repr: int = REPR_CANONICAL) -> np.ndarray:
        a, b = _u64(a), _u64(b)
        out = np.empty_like(a)
        self.check(self.lib.lf_ring_mul(self.h, _ptr(a), _ptr(b), _ptr(out), a.size // d, d, repr))
        return out

    def witness_from_w_ccs(self, w_ccs, params: LfParams, repr: int = REPR_CANONICAL):
        w = _u64(w_ccs)
        d, L = params.d, params.L
        W = w.size // d
        fc = np.empty(W * L * d, np.uint64)
        f = np.empty(W * L * d, np.uint64)
        self.check(self.lib.lf_witness_from_w_ccs(self.h, C.byref(params), _ptr(w), W, _ptr(fc), _ptr(f), repr))
        return fc, f

    def witness_from_f(self, f, params: LfParams, repr: int = REPR_CANONICAL):
        x = _u64(f)
        d, L = params.d, params.L
        N = x.size // d
        fc = np.empty(N * d, np.uint64)
        w = np.empty((N // L) * d, np.uint64)
        self.check(self.lib.lf_witness_from_f(self.h, C.byref(params), _ptr(x), N, _ptr(fc), _ptr(w), repr))
        return fc, w

    def dev_decompose_witness(self, params: LfParams, f_coeff, N: int, f_coeff_k, f_k, w_ccs_k):
        """decompose_witness on device buffers: f_coeff [N] -> [K][N], [K][N], [K][N / L]"""
        self.check(self.lib.lf_dev_decompose_witness(self.h, C.byref(params), _dptr(f_coeff), N, _dptr(f_coeff_k),
                                                     _dptr(f_k), _dptr(w_ccs_k)))

    def decompose_witness(self, f_coeff, params: LfParams, repr: int = REPR_CANONICAL):
        x = _u64(f_coeff)
        d, L, K = params.d, params.L, params.K
        N = x.size // d
        fck = np.empty(K * N * d, np.uint64)
        fk = np.empty(K * N * d, np.uint64)
        wk = np.empty(K * (N // L) * d, np.uint64)
        self.check(self.lib.lf_decompose_witness(self.h, C.byref(params), _ptr(x), N, _ptr(fck),
                                                 _ptr(fk), _ptr(wk), repr))
        return fck, fk, wk

    def commit(self, scheme: "AjtaiCommitmentScheme", z, l: int, params: LfParams,
               repr: int = REPR_CANONICAL):
        """zkvm commit() (main.rs:348-367): returns (f_coeff, f, cm)."""
        zz = _u64(z)
        d = params.d
        N = scheme.width
        fc = np.empty(N * d, np.uint64)
        f = np.empty(N * d, np.uint64)
        cm = np.empty(scheme.kappa * d, np.uint64)
        self.check(self.lib.lf_commit(self.h, scheme.h, C.byref(params), _ptr(zz), zz.size // d, l,
                                      _ptr(fc), _ptr(f), _ptr(cm), repr))
        return fc, f, cm

    def fold_hot(self, scheme: "AjtaiCommitmentScheme", params: LfParams, acc_cm, acc_f_coeff,
                 cm_i, wi_f_coeff, rho, repr: int = REPR_CANONICAL) -> dict:
        """commit+fold arithmetic of zkvm fold() for one step (see lf.h lf_fold_hot)."""
        d, K, L = params.d, params.K, params.L
        a_cm, a_fc, c_i, w_fc, r = map(_u64, (acc_cm, acc_f_coeff, cm_i, wi_f_coeff, rho))
        N = a_fc.size // d
        kd = scheme.kappa * d
        out = {
            "y": np.empty(2 * K * kd, np.uint64), "f0": np.empty(N * d, np.uint64),
            "f0_coeff": np.empty(N * d, np.uint64), "w_ccs0": np.empty((N // L) * d, np.uint64),
            "cm0": np.empty(kd, np.uint64),
        }
        self.check(self.lib.lf_fold_hot(
            self.h, scheme.h, C.byref(params), _ptr(a_cm), _ptr(a_fc), _ptr(c_i), _ptr(w_fc), N,
            _ptr(r), _ptr(out["y"]), _ptr(out["f0"]), _ptr(out["f0_coeff"]), _ptr(out["w_ccs0"]),
            _ptr(out["cm0"]), repr))
        return out

    def fold_lcccs(self, d: int, rho, rho_coeff=None, eta=None, xwh=None, theta=None,
                   repr: int = REPR_CANONICAL) -> dict:
        """u_0, x_0, v_0 of the folded LCCCS (compute_v0_u0_x0_cm_0,
        folding/utils.rs:456-517): rho [nwit][d]; eta [nwit][t]; xwh [nwit][l+1];
        theta [nwit][tau] with its rho_coeff [nwit][d] (tau = 3 for d = 24, else 1)"""
        r = _u64(rho)
        nwit = r.size // d
        tau = 3 if d == 24 else 1
        e = _u64(eta) if eta is not None else None
        x = _u64(xwh) if xwh is not None else None
        th = _u64(theta) if theta is not None else None
        rc = _u64(rho_coeff) if rho_coeff is not None else None
        t = e.size // (nwit * d) if e is not None else 0
        l1 = x.size // (nwit * d) if x is not None else 0
        out = {"u0": np.empty(t * d, np.uint64), "x0": np.empty(l1 * d, np.uint64),
               "v0": np.empty(tau * d if th is not None else 0, np.uint64)}
        p = lambda a: _ptr(a) if a is not None else None
        self.check(self.lib.lf_fold_lcccs(self.h, d, nwit, _ptr(r), p(rc), p(e), t, p(x), l1, p(th),
                                          _ptr(out["u0"]), _ptr(out["x0"]), _ptr(out["v0"]), repr))
        return out

    def compute_x_s(self, x, params: LfParams, repr: int = REPR_CANONICAL) -> np.ndarray:
        """compute_x_s (decomposition.rs:172-175): x_w || h -> [K][m] decomposed statements"""
        xx = _u64(x)
        m = xx.size // params.d
        out = np.empty(params.K * m * params.d, np.uint64)
        self.check(self.lib.lf_compute_x_s(self.h, C.byref(params), _ptr(xx), m, _ptr(out), repr))
        return out

    def poseidon2_permute(self, states) -> np.ndarray:
        s = _u64(states).copy()
        self.check(self.lib.lf_poseidon2_permute(self.h, _ptr(s), s.size // 16))
        return s

    # ---------------------------------------------------------------- device API (torch tensors)
    def dev_crt(self, t, d: int):
        self.check(self.lib.lf_dev_crt(self.h, _dptr(t), t.numel() // d, d))

    def dev_icrt(self, t, d: int):
        self.check(self.lib.lf_dev_icrt(self.h, _dptr(t), t.numel() // d, d))

    def dev_fill_uniform(self, t, seed: int):
        self.check(self.lib.lf_dev_fill_uniform(self.h, _dptr(t), t.numel(), seed))

    def dev_ajtai_commit(self, scheme: "AjtaiCommitmentScheme", vecs, cm):
        arr = (C.c_void_p * len(vecs))(*[_dptr(v) for v in vecs])
        self.check(self.lib.lf_dev_ajtai_commit(self.h, scheme.h, arr, len(vecs), _dptr(cm)))

    def dev_fold_step(self, scheme: "AjtaiCommitmentScheme", params: LfParams, W: int,
                      bufs: LfFoldStepBufs):
        self.check(self.lib.lf_dev_fold_step(self.h, scheme.h, C.byref(params), W, C.byref(bufs)))

    def dev_fold_step_batch(self, others, scheme: "AjtaiCommitmentScheme", params: LfParams, W: int, bufs):
        """len(bufs) independent steps: step 0 on this context, step i on others[i - 1]
        (each its own stream); their contractions share one pass over A (lf.h)"""
        ctxs = [self] + list(others)
        if len(ctxs) != len(bufs):
            raise ValueError("one context per step")
        ch = (C.c_void_p * len(ctxs))(*[c.h for c in ctxs])
        bh = (C.c_void_p * len(bufs))(*[C.cast(C.byref(b), C.c_void_p) for b in bufs])
        self.check(self.lib.lf_dev_fold_step_batch(ch, len(ctxs), scheme.h, C.byref(params), W, bh))

    def fold_step_partial_len(self, scheme: "AjtaiCommitmentScheme", params: LfParams) -> int:
        return self.lib.lf_fold_step_partial_len(scheme.h, C.byref(params))

    def dev_fold_step_partial(self, scheme, params: LfParams, W: int, bufs: LfFoldStepBufs, partial):
        """column-sharded step, first half: partial commitments of this rank's columns (lf.h)"""
        self.check(self.lib.lf_dev_fold_step_partial(self.h, scheme.h, C.byref(params), W, C.byref(bufs),
                                                     _dptr(partial)))

    def dev_fold_step_finish(self, scheme, params: LfParams, W: int, bufs: LfFoldStepBufs, partial_sum):
        """column-sharded step, second half, given the partial commitments summed over ranks"""
        self.check(self.lib.lf_dev_fold_step_finish(self.h, scheme.h, C.byref(params), W, C.byref(bufs),
                                                    _dptr(partial_sum)))

    def dev_fold_step_sharded(self, scheme, params: LfParams, W: int, bufs: LfFoldStepBufs,
                              comm: "Communicator | None"):
        self.check(self.lib.lf_dev_fold_step_sharded(self.h, scheme.h, C.byref(params), W, C.byref(bufs),
                                                     comm.h if comm is not None else None))

    def dev_limb_split(self, x, lo, hi):
        self.check(self.lib.lf_dev_limb_split(self.h, _dptr(x), x.numel(), _dptr(lo), _dptr(hi)))

    def dev_limb_join(self, lo, hi, out):
        self.check(self.lib.lf_dev_limb_join(self.h, _dptr(lo), _dptr(hi), out.numel(), _dptr(out)))

    # ---------------------------------------------------------------- multilinear sumcheck
    def dev_eq_table(self, d: int, r, nv: int, out):
        self.check(self.lib.lf_dev_eq_table(self.h, d, _dptr(r), nv, _dptr(out)))

    def dev_expand_planes(self, params: LfParams, planes, N: int, f_coeff_k=None, f_k=None):
        """packed digit planes of N elements (lf_fold_step_bufs.planes) -> f_coeff_k and / or
        f_k = CRT(f_coeff_k), [K][N] each"""
        self.check(self.lib.lf_dev_expand_planes(self.h, C.byref(params), _dptr(planes), N,
                                                 _dptr(f_coeff_k) if f_coeff_k is not None else None,
                                                 _dptr(f_k) if f_k is not None else None))

    def dev_get_fhat(self, d, f_coeff, N, nv, out):
        """Witness::get_fhat on the device: out [tau][2^nv][d] from f_coeff [N][d]"""
        self.check(self.lib.lf_dev_get_fhat(self.h, d, _dptr(f_coeff), N, nv, _dptr(out)))

    def dev_mle_evaluate(self, d: int, mles, nm: int, nv: int, point, out):
        self.check(self.lib.lf_dev_mle_evaluate(self.h, d, _dptr(mles), nm, nv, _dptr(point), _dptr(out)))

    def dev_mle_fix_first(self, d: int, src, src_stride: int, nm: int, nv: int, r_base, out, out_stride: int):
        r = _u64(r_base)
        self.check(self.lib.lf_dev_mle_fix_first(self.h, d, _dptr(src), src_stride, nm, nv, _ptr(r), _dptr(out),
                                                 out_stride))

    def dev_sumcheck_round(self, comb: "Comb", mles, stride: int, nm: int, nv: int, d: int, degree: int, evals):
        self.check(self.lib.lf_dev_sumcheck_round(self.h, C.byref(comb.s), _dptr(mles), stride, nm, nv, d, degree,
                                                  _dptr(evals)))

    def sumcheck_prove(self, transcript: "Poseidon2Transcript", comb: "Comb", mles, nm: int, nv: int, d: int,
                       degree: int):
        """MLSumcheck::prove_as_subprotocol on the device (mles is clobbered):
        returns (proof [nv][degree+1][d], randomness [nv][tau]) as numpy"""
        tau = 3 if d == 24 else 1
        proof = np.zeros(nv * (degree + 1) * d, np.uint64)
        rnd = np.zeros(nv * tau, np.uint64)
        self.check(self.lib.lf_sumcheck_prove(self.h, transcript.h, C.byref(comb.s), _dptr(mles), nm, nv, d,
                                              degree, _ptr(proof), _ptr(rnd)))
        return proof, rnd

    def sumcheck_prove_fold_digits(self, transcript: "Poseidon2Transcript", comb: "Comb", mles5, fc0, fc1, K: int,
                                   N: int, wstride: int, nv: int, d: int, work):
        """the folding sumcheck with its f_hat MLEs as digit coefficient rows
        (lf_sumcheck_prove_fold_digits): the proof and randomness of sumcheck_prove over
        [mles5..., get_fhat of the 2K witnesses]"""
        tau = 3 if d == 24 else 1
        proof = np.zeros(nv * 5 * d, np.uint64)
        rnd = np.zeros(nv * tau, np.uint64)
        self.check(self.lib.lf_sumcheck_prove_fold_digits(self.h, transcript.h, C.byref(comb.s), _dptr(mles5), _dptr(fc0),
                                                          _dptr(fc1), K, N, wstride, nv, d, _dptr(work), _ptr(proof),
                                                          _ptr(rnd)))
        return proof, rnd

    def sumcheck_prove_lin(self, transcript: "Poseidon2Transcript", comb: "Comb", mles, nv: int, d: int,
                           degree: int, beta, work, evals=None):
        """the linearization sumcheck with eq(beta) split off (lf_sumcheck_prove_lin): mles a
        list of device tensors (one MLE of 2^nv elements each, read only), beta [nv][d] host
        values; the proof and randomness of sumcheck_prove over [mles..., eq(beta)]; evals
        (device, len(mles) d, optional) receives the MLEs at the challenge point"""
        tau = 3 if d == 24 else 1
        proof = np.zeros(nv * (degree + 1) * d, np.uint64)
        rnd = np.zeros(nv * tau, np.uint64)
        ptrs = (C.c_void_p * len(mles))(*[_dptr(m) for m in mles])
        b = _u64(beta)
        self.check(self.lib.lf_sumcheck_prove_lin(self.h, transcript.h, C.byref(comb.s), ptrs, len(mles), nv, d,
                                                  degree, _ptr(b), _dptr(work), _ptr(proof), _ptr(rnd),
                                                  _dptr(evals) if evals is not None else None))
        return proof, rnd

    def sumcheck_prove_lin_sparse(self, transcript: "Poseidon2Transcript", comb: "Comb", mles, nv: int, d: int,
                                  degree: int, beta, act, act_off, work, evals=None):
        """sumcheck_prove_lin with round 0 over each multiset's active points only
        (lf_sumcheck_prove_lin_sparse): act a device int32 tensor of point indices,
        act_off (host, q + 1) each multiset's range in it"""
        tau = 3 if d == 24 else 1
        proof = np.zeros(nv * (degree + 1) * d, np.uint64)
        rnd = np.zeros(nv * tau, np.uint64)
        ptrs = (C.c_void_p * len(mles))(*[_dptr(m) for m in mles])
        b = _u64(beta)
        off = np.ascontiguousarray(act_off, dtype=np.uint32)
        self.check(self.lib.lf_sumcheck_prove_lin_sparse(self.h, transcript.h, C.byref(comb.s), ptrs, len(mles), nv,
                                                         d, degree, _ptr(b), _dptr(act), off.ctypes.data,
                                                         _dptr(work), _ptr(proof), _ptr(rnd),
                                                         _dptr(evals) if evals is not None else None))
        return proof, rnd

    # ---------------------------------------------------------------- width-8 Merkle trees
    def dev_poseidon2_w8_permute(self, t):
        self.check(self.lib.lf_dev_poseidon2_w8_permute(self.h, _dptr(t), t.numel() // 8))

    def dev_merkle_tree(self, rows, nrows: int, width: int, nodes):
        """matrix [nrows][width] -> merkle_nodes_len(nrows) x 4 digests (Plonky3's even-padded
        layers), root last"""
        self.check(self.lib.lf_dev_merkle_tree(self.h, _dptr(rows), nrows, width, _dptr(nodes)))

    def merkle_open(self, nodes, nrows: int, index: int) -> np.ndarray:
        path = np.zeros(4 * max(1, merkle_depth(nrows)), np.uint64)
        self.check(self.lib.lf_merkle_open(self.h, _dptr(nodes), nrows, index, _ptr(path)))
        return path[:4 * merkle_depth(nrows)]

    def dev_hash_w8_rows(self, rows, nrows: int, width: int, out):
        """independent width-8 sponge hashes of nrows rows -> out [nrows][4]"""
        self.check(self.lib.lf_dev_hash_w8_rows(self.h, _dptr(rows), nrows, width, _dptr(out)))

    def vm_code_comm(self, code: bytes) -> np.ndarray:
        """zkvm vm_code_comm (commitments.rs:314-340): Merkle root over the code's half-words"""
        out = np.zeros(4, np.uint64)
        buf = (C.c_uint8 * len(code)).from_buffer_copy(code)
        self.check(self.lib.lf_vm_code_comm(self.h, buf, len(code), _ptr(out)))
        return out

    def dev_poseidon2_permute(self, t):
        self.check(self.lib.lf_dev_poseidon2_permute(self.h, _dptr(t), t.numel() // 16))

    def dev_modp_sum(self, inp, nparts: int, length: int, out):
        self.check(self.lib.lf_dev_modp_sum(self.h, _dptr(inp), nparts, length, _dptr(out)))


class Communicator:
    """lf_comm: an RCCL communicator of one rank, for the accumulator exchange
    (lf.h lf_comm_*). Built from a 128-byte unique id that rank 0 creates
    (``Communicator.unique_id()``) and the host distributes, or by wrapping a
    caller-created ncclComm_t (``Communicator.wrap``)."""

    ID_BYTES = 128

    def __init__(self, ctx: Context, nranks: int, rank: int, uid: bytes | None = None, *, _handle=None):
        self.ctx, self.lib = ctx, ctx.lib
        if _handle is not None:
            self.h = _handle
        else:
            h = C.c_void_p()
            if uid is None:  # one rank without RCCL
                ctx.check(self.lib.lf_comm_init(ctx.h, nranks, rank, None, 0, C.byref(h)))
            else:
                buf = np.frombuffer(bytes(uid), np.uint8).copy()
                ctx.check(self.lib.lf_comm_init(ctx.h, nranks, rank, _ptr(buf), buf.size, C.byref(h)))
            self.h = h
        self.size = self.lib.lf_comm_size(self.h)
        self.rank = self.lib.lf_comm_rank(self.h)

    @staticmethod
    def unique_id() -> bytes:
        lib = load()
        buf = np.zeros(Communicator.ID_BYTES, np.uint8)
        rc = lib.lf_comm_unique_id(_ptr(buf), buf.size)
        if rc:
            raise LfError(rc, "lf_comm_unique_id: " + lib.lf_status_string(rc).decode())
        return buf.tobytes()

    @classmethod
    def wrap(cls, ctx: Context, nccl_comm: int) -> "Communicator":
        h = C.c_void_p()
        ctx.check(ctx.lib.lf_comm_wrap(ctx.h, nccl_comm, C.byref(h)))
        return cls(ctx, 0, 0, _handle=h)

    def allreduce_modp(self, t):
        """t <- sum over ranks of t (mod p), in place on the context stream"""
        self.ctx.check(self.lib.lf_comm_allreduce_modp(self.ctx.h, self.h, _dptr(t), t.numel()))

    def fold_reduce_allranks(self, cm0, f0):
        self.ctx.check(self.lib.lf_fold_reduce_allranks(self.ctx.h, self.h, _dptr(cm0), cm0.numel(),
                                                        _dptr(f0), f0.numel()))

    def close(self):
        if getattr(self, "h", None):
            self.lib.lf_comm_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Comb:
    """lf_comb: the combination function of a sumcheck polynomial (lf.h)."""

    def __init__(self, s: LfComb, keep):
        self.s, self._keep = s, keep

    @classmethod
    def folding(cls, mu_dev, nk: int, tau: int, bsmall: int = 2) -> "Comb":
        """the folding polynomial (folding/utils.rs:196-331); mu: nk NTT elements on the device"""
        return cls(LfComb(kind=0, nk=nk, tau=tau, bsmall=bsmall, mu=_dptr(mu_dev)), [mu_dev])

    @classmethod
    def linearization(cls, c_dev, S) -> "Comb":
        """the linearization polynomial (linearization/utils.rs:63-104); c: q NTT
        elements on the device; S: q lists of matrix indices"""
        off = np.zeros(len(S) + 1, np.int32)
        off[1:] = np.cumsum([len(x) for x in S])
        idx = np.array([j for x in S for j in x] or [0], np.int32)
        return cls(LfComb(kind=1, q=len(S), c=_dptr(c_dev), S_off=_ptr(off), S_idx=_ptr(idx)), [c_dev, off, idx])


class CCSMatrices:
    """CCS.M on the device (lf_ccs): t sparse m x n matrices of ring elements,
    given as (row_ptr, col, val) per matrix (row_ptr relative to that matrix)."""

    def __init__(self, ctx: Context, d: int, m: int, n: int, mats, repr: int = REPR_CANONICAL):
        self.ctx, self.lib = ctx, ctx.lib
        rps, cols, vals, base = [], [], [], 0
        for rp, col, val in mats:
            rp = np.asarray(rp, np.uint64)
            rps.append(rp + np.uint64(base))
            base += int(rp[-1])
            cols.append(np.asarray(col, np.uint32))
            vals.append(_u64(val))
        row_ptr = np.ascontiguousarray(np.concatenate(rps))
        col = np.ascontiguousarray(np.concatenate(cols)) if base else np.zeros(1, np.uint32)
        val = np.ascontiguousarray(np.concatenate(vals)) if base else np.zeros(d, np.uint64)
        h = C.c_void_p()
        ctx.check(self.lib.lf_ccs_create(ctx.h, d, len(mats), m, n, _ptr(row_ptr), _ptr(col), _ptr(val), repr,
                                         C.byref(h)))
        self.h, self.d, self.t, self.m, self.n = h, d, len(mats), m, n

    def mz_mles(self, z, nz: int, nv: int, out):
        self.ctx.check(self.lib.lf_dev_mz_mles(self.ctx.h, self.h, _dptr(z), nz, nv, _dptr(out)))

    def mz_mles_sel(self, z, sel, nv: int, out):
        """the MLEs of the selected matrices only (lf_dev_mz_mles_sel): out[i] = MLE(M_sel[i] z)"""
        s = np.ascontiguousarray(np.asarray(sel, np.int32))
        self.ctx.check(self.lib.lf_dev_mz_mles_sel(self.ctx.h, self.h, _dptr(z), _ptr(s), len(s), nv, _dptr(out)))

    @property
    def scalar(self) -> bool:
        """every entry a scalar (lf_ccs_is_scalar): the products read one word per entry"""
        return bool(self.lib.lf_ccs_is_scalar(self.h))

    def row_live(self, j: int, m: int):
        """which rows of M_j hold an entry (lf_ccs_row_live): m bools"""
        out = np.zeros(m, np.uint8)
        self.ctx.check(self.lib.lf_ccs_row_live(self.h, j, out.ctypes.data))
        return out.astype(bool)

    def mz_challenged(self, z, zeta, nz: int, nv: int, out):
        self.ctx.check(self.lib.lf_dev_mz_challenged(self.ctx.h, self.h, _dptr(z), _dptr(zeta), nz, nv, _dptr(out)))

    def mz_challenged_pair(self, z0, zeta0, z1, zeta1, nz: int, nv: int, out0, out1):
        """two challenged Mz MLEs over one pass of the matrices (lf_dev_mz_challenged_pair)"""
        self.ctx.check(self.lib.lf_dev_mz_challenged_pair(self.ctx.h, self.h, _dptr(z0), _dptr(zeta0), _dptr(z1),
                                                          _dptr(zeta1), nz, nv, _dptr(out0), _dptr(out1)))

    def mz_evaluate(self, z, nz: int, nv: int, point, out):
        self.ctx.check(self.lib.lf_dev_mz_evaluate(self.ctx.h, self.h, _dptr(z), nz, nv, _dptr(point), _dptr(out)))

    def __del__(self):
        try:
            if self.h:
                self.lib.lf_ccs_destroy(self.h)
                self.h = None
        except Exception:
            pass


class Prover:
    """fold() end to end (lf_fold_prove, zk_latticefold_prove): device scratch for one
    (scheme, params, CCS) shape. The CCS gets its structure (l, degree, c, S) here."""

    def __init__(self, ctx: Context, scheme: "AjtaiCommitmentScheme", params: LfParams, ccs: CCSMatrices, l: int,
                 degree: int, c, S, repr: int = REPR_CANONICAL):
        self.ctx, self.lib, self.pr, self.ccs, self.scheme = ctx, ctx.lib, params, ccs, scheme
        c = _u64(c)
        off = np.zeros(len(S) + 1, np.int32)
        off[1:] = np.cumsum([len(x) for x in S])
        idx = np.array([j for x in S for j in x] or [0], np.int32)
        ctx.check(self.lib.lf_ccs_set_structure(ctx.h, ccs.h, l, degree, len(S), _ptr(c), _ptr(off), _ptr(idx), repr))
        h = C.c_void_p()
        self.lib.lf_ctx_set_error(ctx.h, b"")  # so a message read below is this call's
        rc = self.lib.lf_prover_create(ctx.h, scheme.h, C.byref(params), ccs.h, C.byref(h))
        if rc:
            msg = self.lib.lf_ctx_last_error(ctx.h).decode()
            raise LfError(rc, msg or "lf_prover_create: " + self.lib.lf_status_string(rc).decode())
        self.h = h
        self.d, self.l, self.t, self.degree = params.d, l, ccs.t, degree
        self.s = ccs.m.bit_length() - 1
        self.tau = 3 if params.d == 24 else 1
        self.kappa = scheme.kappa
        self.c, self.S = c, [list(x) for x in S]

    def replay(self, acc: dict, cm_i, x_ccs, proof: dict, repr: int = REPR_CANONICAL) -> dict:
        """the verifier-variable replay (fold_replay) of a proof this prover wrote"""
        return fold_replay(self.pr, self.t, self.ccs.m, self.l, self.degree, self.c, self.S, self.kappa, acc, cm_i,
                           x_ccs, proof, repr)

    def fold_prove(self, acc: dict, w_acc: dict, cm_i, x_ccs, w_i: dict, w_out: dict, repr: int = REPR_CANONICAL,
                   vars: bool = False):
        """acc: {r, v, cm, u, x_w, h} host arrays; w_*: {w_ccs, f, f_coeff} device tensors.
        Returns (folded LCCCS dict, LFProof dict) as host arrays; w_out is filled.
        vars=True: lf_fold_prove_vars, returning (LCCCS, LFProof, verification vars) with
        the vars replayed from the call's own sample log (keys as fold_replay's)."""
        from ._lib import REPLAY_FIELDS, LfLcccs, LfLcccsMut, LfLfproofMut, LfReplayVars, LfRingSlice, LfWitness
        d, s, tau, t, l, K, kappa = self.d, self.s, self.tau, self.t, self.l, self.pr.K, self.kappa
        keep = {k: _u64(v) for k, v in acc.items()}
        sl = lambda a: LfRingSlice(a.ctypes.data, a.size // d)
        A = LfLcccs(d, sl(keep["r"]), sl(keep["v"]), sl(keep["cm"]), sl(keep["u"]), sl(keep["x_w"]),
                    keep["h"].ctypes.data)
        wit = lambda w: LfWitness(_dptr(w["w_ccs"]), _dptr(w["f"]), _dptr(w["f_coeff"]))
        out = {"r": np.zeros(s * d, np.uint64), "v": np.zeros(tau * d, np.uint64),
               "cm": np.zeros(kappa * d, np.uint64), "u": np.zeros(t * d, np.uint64),
               "x_w": np.zeros(max(l, 1) * d, np.uint64), "h": np.zeros(d, np.uint64)}
        pf = {"lin_sumcheck": np.zeros(s * (self.degree + 2) * d, np.uint64), "lin_v": np.zeros(tau * d, np.uint64),
              "lin_u": np.zeros(t * d, np.uint64),
              "u_s": [np.zeros(K * t * d, np.uint64) for _ in range(2)],
              "v_s": [np.zeros(K * tau * d, np.uint64) for _ in range(2)],
              "x_s": [np.zeros(K * (l + 1) * d, np.uint64) for _ in range(2)],
              "y_s": [np.zeros(K * kappa * d, np.uint64) for _ in range(2)],
              "fold_sumcheck": np.zeros(s * (2 * self.pr.b_small + 1) * d, np.uint64),
              "theta_s": np.zeros(2 * K * tau * d, np.uint64), "eta_s": np.zeros(2 * K * t * d, np.uint64)}
        O_ = LfLcccsMut(*[out[k].ctypes.data for k in ("r", "v", "cm", "u", "x_w", "h")])
        PM = LfLfproofMut()
        for k in ("lin_sumcheck", "lin_v", "lin_u", "fold_sumcheck", "theta_s", "eta_s"):
            setattr(PM, k, pf[k].ctypes.data)
        for k in ("u_s", "v_s", "x_s", "y_s"):
            for side in range(2):
                getattr(PM, k)[side] = pf[k][side].ctypes.data
        cm = _u64(cm_i)
        xc = _u64(x_ccs) if l else np.zeros(1, np.uint64)
        wa, wi, wo = wit(w_acc), wit(w_i), wit(w_out)
        if vars:
            vout = {k: np.zeros(n * d, np.uint64) for k, n in replay_sizes(self.pr, self.t, self.ccs.m, l, self.degree,
                                                                           len(self.S), kappa).items()}
            V = LfReplayVars(*[vout[k].ctypes.data for k in REPLAY_FIELDS])
            rc = self.lib.lf_fold_prove_vars(self.h, C.byref(A), C.byref(wa), cm.ctypes.data, xc.ctypes.data,
                                             C.byref(wi), C.byref(O_), C.byref(wo), C.byref(PM), C.byref(V), repr)
        else:
            rc = self.lib.lf_fold_prove(self.h, C.byref(A), C.byref(wa), cm.ctypes.data, xc.ctypes.data, C.byref(wi),
                                        C.byref(O_), C.byref(wo), C.byref(PM), repr)
        if rc:
            raise LfError(rc, self.lib.lf_prover_last_error(self.h).decode() or self.lib.lf_status_string(rc).decode())
        out["x_w"] = out["x_w"][:l * d]
        return (out, pf, vout) if vars else (out, pf)

    def samples(self) -> np.ndarray:
        """every value the last fold_prove sampled from its transcript, in order"""
        n = self.lib.lf_prover_samples(self.h, None, 0)
        out = np.zeros(max(n, 1), np.uint64)
        self.lib.lf_prover_samples(self.h, out.ctypes.data, n)
        return out[:n]

    SPANS = ("public_input", "linearization", "decomposition", "decomposition_transcript", "folding_mles",
             "folding_sumcheck", "evaluations", "folding_transcript", "fold", "vars")

    def timing(self, enable: bool) -> dict:
        """the fold() phase spans (ms, summed) since the last call; then timing on/off"""
        ms = np.zeros(len(self.SPANS), np.float64)
        self.lib.lf_prover_timing(self.h, int(enable), ms.ctypes.data)
        return dict(zip(self.SPANS, ms.tolist()))

    def linearize(self, cm, x_ccs, w: dict, repr: int = REPR_CANONICAL):
        """initialize_accumulator's LFLinearizationProver::prove on a fresh transcript:
        -> (LCCCS dict, linearization sumcheck messages)"""
        from ._lib import LfLcccsMut, LfWitness
        d, s, tau, t, l = self.d, self.s, self.tau, self.t, self.l
        out = {"r": np.zeros(s * d, np.uint64), "v": np.zeros(tau * d, np.uint64),
               "cm": np.zeros(self.kappa * d, np.uint64), "u": np.zeros(t * d, np.uint64),
               "x_w": np.zeros(max(l, 1) * d, np.uint64), "h": np.zeros(d, np.uint64)}
        sc = np.zeros(s * (self.degree + 2) * d, np.uint64)
        O_ = LfLcccsMut(*[out[k].ctypes.data for k in ("r", "v", "cm", "u", "x_w", "h")])
        cm, xc = _u64(cm), (_u64(x_ccs) if l else np.zeros(1, np.uint64))
        wi = LfWitness(_dptr(w["w_ccs"]), _dptr(w["f"]), _dptr(w["f_coeff"]))
        rc = self.lib.lf_linearize(self.h, cm.ctypes.data, xc.ctypes.data, C.byref(wi), C.byref(O_), sc.ctypes.data,
                                   repr)
        if rc:
            raise LfError(rc, self.lib.lf_prover_last_error(self.h).decode() or self.lib.lf_status_string(rc).decode())
        out["x_w"] = out["x_w"][:l * d]
        return out, sc

    def __del__(self):
        try:
            if self.h:
                self.lib.lf_prover_destroy(self.h)
                self.h = None
        except Exception:
            pass


def replay_sizes(params: LfParams, t: int, m: int, l: int, degree: int, q: int, kappa: int) -> dict:
    """NTT elements of every lf_replay_vars field"""
    K, bs, s = params.K, params.b_small, m.bit_length() - 1
    return {"lin_beta": s, "lin_claimed_sums": s + 1, "lin_subterms": s * (degree + 2), "lin_point": s,
            "lin_expected": 1, "lin_inner": 1, "lin_products": q, "lin_eq_xy": s, "lin_eq_factors": s,
            "lin_eq_sub": s + 1, "alpha": 2 * K, "beta": s, "zeta": 2 * K, "mu": 2 * K, "claim_g1_h1": 2 * K,
            "claim_g1_h2": 2 * K, "claim_g1_terms": 2 * K, "claim_g1": 1, "claim_g3_h": 2 * K * (t - 1),
            "claim_g3_terms": 2 * K, "claim_g3": 1, "fold_claimed_sums": s + 1, "fold_subterms": s * (2 * bs + 1),
            "fold_point": s, "fold_expected": 1, "should_equal_s": 1, "rho": 2 * K, "final_cm": 2 * K * kappa,
            "final_u": 2 * K * t, "final_x": 2 * K * (l + 1)}


def fold_replay(params: LfParams, t: int, m: int, l: int, degree: int, c, S, kappa: int, acc: dict, cm_i, x_ccs,
                proof: dict, repr: int = REPR_CANONICAL, samples=None) -> dict:
    """generate_verification_witness_vars (zkvm/src/zk_latticefold.rs:111-148) on the
    host: replays a fold() proof (the dict Prover.fold_prove returns) and returns the
    in-CCS verifier's values, keyed as oracle/nifs.py fold_replay names them, each a
    flat u64 array of NTT elements. Phi_72 only; no GPU involved. samples: the
    prover's sample log (lf_fold_replay_samples: no second Poseidon2 pass).
    samples is for the prover's OWN proof only: the playback drops every observe,
    so the vars are not bound to the proof's messages. A proof received from
    elsewhere must be replayed with samples=None (or checked with fold_verify)."""
    from ._lib import REPLAY_FIELDS, LfCcsDesc, LfLcccs, LfLfproofMut, LfReplayVars, LfRingSlice
    lib, d, K, bs = load(), params.d, params.K, params.b_small
    s, q = m.bit_length() - 1, len(S)
    c = _u64(c)
    off = np.zeros(q + 1, np.int32)
    off[1:] = np.cumsum([len(x) for x in S])
    idx = np.array([j for x in S for j in x] or [0], np.int32)
    desc = LfCcsDesc(t, m, l, degree, q, c.ctypes.data, off.ctypes.data, idx.ctypes.data)
    keep = {k: _u64(v) for k, v in acc.items()}
    sl = lambda a: LfRingSlice(a.ctypes.data, a.size // d)
    A = LfLcccs(d, sl(keep["r"]), sl(keep["v"]), sl(keep["cm"]), sl(keep["u"]), sl(keep["x_w"]), keep["h"].ctypes.data)
    pf = {k: (_u64(v) if not isinstance(v, list) else [_u64(x) for x in v]) for k, v in proof.items()}
    PM = LfLfproofMut()
    for k in ("lin_sumcheck", "lin_v", "lin_u", "fold_sumcheck", "theta_s", "eta_s"):
        setattr(PM, k, pf[k].ctypes.data)
    for k in ("u_s", "v_s", "x_s", "y_s"):
        for side in range(2):
            getattr(PM, k)[side] = pf[k][side].ctypes.data
    sizes = replay_sizes(params, t, m, l, degree, q, kappa)
    out = {k: np.zeros(sizes[k] * d, np.uint64) for k in REPLAY_FIELDS}
    V = LfReplayVars(*[out[k].ctypes.data for k in REPLAY_FIELDS])
    cm, xc = _u64(cm_i), (_u64(x_ccs) if l else np.zeros(1, np.uint64))
    if samples is None:
        rc = lib.lf_fold_replay(C.byref(desc), C.byref(params), C.byref(A), cm.ctypes.data, xc.ctypes.data,
                                C.byref(PM), C.byref(V), repr)
    else:
        sm = _u64(samples) if len(samples) else np.zeros(1, np.uint64)
        rc = lib.lf_fold_replay_samples(C.byref(desc), C.byref(params), C.byref(A), cm.ctypes.data, xc.ctypes.data,
                                        C.byref(PM), sm.ctypes.data, len(samples), C.byref(V), repr)
    if rc:
        raise LfError(rc, "lf_fold_replay: " + lib.lf_status_string(rc).decode())
    return out


VERIFY_CHECKS = {1: "linearization sumcheck", 2: "linearization evaluation claim", 3: "decomposition recompose y",
                 4: "decomposition recompose v", 5: "decomposition recompose u", 6: "decomposition recompose x",
                 7: "folding sumcheck", 8: "folding evaluation claim"}


class VerificationError(LfError):
    def __init__(self, check: int):
        super().__init__(12, VERIFY_CHECKS.get(check, str(check)))
        self.check = check


def fold_verify(params: LfParams, t: int, m: int, l: int, degree: int, c, S, kappa: int, acc: dict, cm_i, x_ccs,
                proof: dict, repr: int = REPR_CANONICAL) -> dict:
    """NIFSVerifier::verify of a fold() proof (lf_fold_verify; zkvm main.rs:408-426): the
    folded LCCCS dict {r, v, cm, u, x_w, h}, or VerificationError naming the failed check.
    Host only (Phi_72)."""
    from ._lib import LfCcsDesc, LfLcccs, LfLcccsMut, LfLfproofMut, LfRingSlice
    lib, d = load(), params.d
    s, q = m.bit_length() - 1, len(S)
    c = _u64(c)
    off = np.zeros(q + 1, np.int32)
    off[1:] = np.cumsum([len(x) for x in S])
    idx = np.array([j for x in S for j in x] or [0], np.int32)
    desc = LfCcsDesc(t, m, l, degree, q, c.ctypes.data, off.ctypes.data, idx.ctypes.data)
    keep = {k: _u64(v) for k, v in acc.items()}
    sl = lambda a: LfRingSlice(a.ctypes.data, a.size // d)
    A = LfLcccs(d, sl(keep["r"]), sl(keep["v"]), sl(keep["cm"]), sl(keep["u"]), sl(keep["x_w"]), keep["h"].ctypes.data)
    pf = {k: (_u64(v) if not isinstance(v, list) else [_u64(x) for x in v]) for k, v in proof.items()}
    PM = LfLfproofMut()
    for k in ("lin_sumcheck", "lin_v", "lin_u", "fold_sumcheck", "theta_s", "eta_s"):
        setattr(PM, k, pf[k].ctypes.data)
    for k in ("u_s", "v_s", "x_s", "y_s"):
        for side in range(2):
            getattr(PM, k)[side] = pf[k][side].ctypes.data
    tau = 3 if d == 24 else 1
    out = {"r": np.zeros(s * d, np.uint64), "v": np.zeros(tau * d, np.uint64), "cm": np.zeros(kappa * d, np.uint64),
           "u": np.zeros(t * d, np.uint64), "x_w": np.zeros(max(l, 1) * d, np.uint64), "h": np.zeros(d, np.uint64)}
    O_ = LfLcccsMut(*[out[k].ctypes.data for k in ("r", "v", "cm", "u", "x_w", "h")])
    cm, xc = _u64(cm_i), (_u64(x_ccs) if l else np.zeros(1, np.uint64))
    failed = C.c_int(0)
    rc = lib.lf_fold_verify(C.byref(desc), C.byref(params), C.byref(A), cm.ctypes.data, xc.ctypes.data, C.byref(PM),
                            C.byref(O_), C.byref(failed), repr)
    if rc == 12:
        raise VerificationError(failed.value)
    if rc:
        raise LfError(rc, "lf_fold_verify: " + lib.lf_status_string(rc).decode())
    out["x_w"] = out["x_w"][:l * d]
    return out


def witness_split_w() -> int:
    """W below which the d = 1024 witness kernels split elements by limb (lf.h)."""
    return load().lf_witness_split_w()


class AjtaiCommitmentScheme:
    """latticefold commitment_scheme.rs:17-78 -- kappa x n Ajtai matrix (NTT form)."""

    def __init__(self, ctx: Context, matrix=None, *, kappa: int | None = None, ncols: int | None = None,
                 d: int | None = None, device_tensor=None, repr: int = REPR_CANONICAL):
        self.ctx = ctx
        h = C.c_void_p()
        if device_tensor is not None:
            self._keep = device_tensor
            ctx.check(ctx.lib.lf_ajtai_create_device(ctx.h, _dptr(device_tensor), kappa, ncols, d, C.byref(h)))
        else:
            m = _u64(matrix)
            kappa, ncols, d = (m.shape if m.ndim == 3 else (kappa, ncols, d))
            ctx.check(ctx.lib.lf_ajtai_create(ctx.h, _ptr(m), kappa, ncols, d, repr, C.byref(h)))
        self.h = h
        self.kappa, self.width, self.d = kappa, ncols, d
        # with the MFMA layout the scheme owns a fragment-order copy of A, so the
        # caller's AoS device matrix is no longer read (lf_ajtai_layout == 1)
        self.layout = ctx.lib.lf_ajtai_layout(h)
        if self.layout == 1:
            self._keep = None

    def commit_ntt(self, f, repr: int = REPR_CANONICAL) -> np.ndarray:
        x = _u64(f)
        cm = np.empty(self.kappa * self.d, np.uint64)
        self.ctx.check(self.ctx.lib.lf_ajtai_commit(self.ctx.h, self.h, _ptr(x), x.size // self.d,
                                                    _ptr(cm), repr))
        return cm

    commit = commit_ntt

    def __del__(self):
        try:
            if self.h:
                self.ctx.lib.lf_ajtai_destroy(self.h)
                self.h = None
        except Exception:
            pass


class Poseidon2Transcript:
    """zkvm fiat_shamir.rs:20-114 (host-side sequential sponge)."""

    def __init__(self):
        self.lib = load()
        self.h = self.lib.lf_transcript_new()

    def __del__(self):
        try:
            self.lib.lf_transcript_free(self.h)
        except Exception:
            pass

    def observe(self, v: int):
        self.lib.lf_transcript_observe(self.h, v)

    def sample(self) -> int:
        return self.lib.lf_transcript_sample(self.h)

    def absorb_ring(self, elems, d: int, repr: int = REPR_CANONICAL):
        x = _u64(elems)
        self.lib.lf_transcript_absorb_ring(self.h, _ptr(x), x.size // d, d, repr)

    def get_challenge(self):
        out = np.zeros(3, np.uint64)
        self.lib.lf_transcript_get_challenge(self.h, _ptr(out))
        return out

    def squeeze_bytes(self, n: int) -> bytes:
        out = np.zeros(n, np.uint8)
        self.lib.lf_transcript_squeeze_bytes(self.h, _ptr(out), n)
        return out.tobytes()

    def get_short_challenges(self, d: int, count: int) -> np.ndarray:
        out = np.zeros(count * d, np.uint64)
        rc = self.lib.lf_transcript_get_short_challenges(self.h, d, count, _ptr(out))
        if rc:
            raise LfError(rc, "get_short_challenges")
        return out


def short_challenge(bs: bytes, d: int = 24) -> np.ndarray:
    """cyclotomic-rings goldilocks.rs:41-67."""
    lib = load()
    b = np.frombuffer(bytes(bs), np.uint8).copy()
    out = np.zeros(d, np.uint64)
    rc = lib.lf_short_challenge(_ptr(b), b.size, d, _ptr(out))
    if rc:
        raise LfError(rc, lib.lf_status_string(rc).decode())
    return out


def hash_iter(vals) -> np.ndarray:
    """zkvm poseidon2.rs:206-235 WideZkVMPoseidon2::hash_iter."""
    x = _u64(vals) if len(vals) else np.zeros(1, np.uint64)
    out = np.zeros(4, np.uint64)
    load().lf_hash_iter(_ptr(x), len(vals), _ptr(out))
    return out


def _chk(rc: int, what: str):
    if rc:
        raise LfError(rc, f"{what}: " + load().lf_status_string(rc).decode())


def hash_iter_states(vals) -> tuple[np.ndarray, np.ndarray]:
    """hash_iter with its IntermediateStates (zkvm poseidon2.rs:199-235):
    (digest, states [nperm][31][16])"""
    lib = load()
    x = _u64(vals) if len(vals) else np.zeros(1, np.uint64)
    k = lib.lf_hash_iter_nperm(len(vals))
    out = np.zeros(4, np.uint64)
    st = np.zeros((max(k, 1), 31, 16), np.uint64)
    _chk(lib.lf_hash_iter_states(_ptr(x), len(vals), _ptr(out), _ptr(st), k), "lf_hash_iter_states")
    return out, st[:k]


def acc_comm(acc: dict, d: int = 24, repr: int = REPR_CANONICAL) -> np.ndarray:
    """ZkVmCommitter::acc_comm (zkvm commitments.rs:143-176) of an LCCCS dict
    {r, v, cm, u, x_w, h} (the dicts Prover.fold_prove / linearize return)"""
    from ._lib import LfLcccs, LfRingSlice
    keep = {k: _u64(acc[k]) for k in ("r", "v", "cm", "u", "x_w", "h")}
    sl = lambda a: LfRingSlice(a.ctypes.data if a.size else None, a.size // d)
    A = LfLcccs(d, sl(keep["r"]), sl(keep["v"]), sl(keep["cm"]), sl(keep["u"]), sl(keep["x_w"]), keep["h"].ctypes.data)
    out = np.zeros(4, np.uint64)
    _chk(load().lf_acc_comm(C.byref(A), repr, _ptr(out)), "lf_acc_comm")
    return out


def ivc_step_comm(i: int, state_0_comm, state_i_comm, accc) -> tuple[np.ndarray, np.ndarray]:
    """ZkVmCommitter::ivc_step_comm (commitments.rs:76-105): (digest, states [2][31][16])"""
    a, b, c = _u64(state_0_comm), _u64(state_i_comm), _u64(accc)
    out = np.zeros(4, np.uint64)
    st = np.zeros((2, 31, 16), np.uint64)
    _chk(load().lf_ivc_step_comm(int(i) % P, _ptr(a), _ptr(b), _ptr(c), _ptr(out), _ptr(st)), "lf_ivc_step_comm")
    return out, st


def state_i_comm(code_comm, pc: int, memory_comm, regs_comm, mem_ops_vec_comm) -> np.ndarray:
    """ZkVmCommitter::state_i_comm (commitments.rs:107-141) from its parts"""
    parts = [_u64(x) for x in (code_comm, memory_comm, regs_comm, mem_ops_vec_comm)]
    out = np.zeros(4, np.uint64)
    _chk(load().lf_state_i_comm(_ptr(parts[0]), int(pc) % P, _ptr(parts[1]), _ptr(parts[2]), _ptr(parts[3]),
                                _ptr(out)), "lf_state_i_comm")
    return out


def vm_regs_comm(regs) -> np.ndarray:
    """ZkVmCommitter::vm_regs_comm (commitments.rs:178-189)"""
    r = np.ascontiguousarray(np.asarray(regs, dtype=np.uint32))
    out = np.zeros(4, np.uint64)
    _chk(load().lf_vm_regs_comm(r.ctypes.data if r.size else None, r.size, _ptr(out)), "lf_vm_regs_comm")
    return out


def vm_mem_ops_vec_comm(prev, cycle: int, address: int, value: int) -> np.ndarray:
    """ZkVmCommitter::vm_mem_ops_vec_comm (commitments.rs:290-307)"""
    pv = _u64(prev)
    out = np.zeros(4, np.uint64)
    _chk(load().lf_vm_mem_ops_vec_comm(_ptr(pv), int(cycle) % P, address & 0xFFFFFFFF, value & 0xFFFFFFFF,
                                       _ptr(out)), "lf_vm_mem_ops_vec_comm")
    return out


def merkle_nodes_len(nrows: int) -> int:
    """digests in a tree over nrows rows (Plonky3's even-padded layers)"""
    return load().lf_merkle_nodes_len(nrows)


def merkle_depth(nrows: int) -> int:
    """layers below the root (the length of an opening path)"""
    n, k = (1 if nrows <= 1 else nrows + nrows % 2), 0
    while n > 1:
        n, k = (1 if n == 2 else (n // 2 + 1) & ~1), k + 1
    return k


def hash_w8(vals) -> np.ndarray:
    """PaddingFreeSponge<Poseidon2Goldilocks<8>, 8, 4, 4>::hash_iter (host)"""
    x = np.ascontiguousarray(np.asarray(vals, dtype=np.uint64)) if len(vals) else np.zeros(1, np.uint64)
    out = np.zeros(4, np.uint64)
    load().lf_hash_w8(_ptr(x), len(vals), _ptr(out))
    return out


def vm_mem_comm(words) -> np.ndarray:
    """zkvm vm_mem_comm (commitments.rs:192-217): one width-8 sponge over every page's u32 words"""
    w = np.ascontiguousarray(np.asarray(words, dtype=np.uint32))
    out = np.zeros(4, np.uint64)
    lib = load()
    rc = lib.lf_vm_mem_comm(w.ctypes.data if w.size else None, w.size, _ptr(out))
    if rc:
        raise LfError(rc, lib.lf_status_string(rc).decode())
    return out


__all__ = ["Context", "AjtaiCommitmentScheme", "Communicator", "Comb", "CCSMatrices", "Prover", "witness_split_w", "Poseidon2Transcript",
           "LfParams", "LfFoldStepBufs", "merkle_nodes_len", "merkle_depth", "hash_w8", "vm_mem_comm",
           "LfError", "goldilocks_dp", "short_challenge", "hash_iter", "hash_iter_states", "acc_comm",
           "ivc_step_comm", "state_i_comm", "vm_regs_comm", "vm_mem_ops_vec_comm", "fold_verify",
           "VerificationError", "P", "REPR_CANONICAL",
           "REPR_MONTGOMERY", "load"]
