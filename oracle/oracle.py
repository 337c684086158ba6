"""ctypes wrapper over oracle/liblf_oracle.so -- TEST INFRASTRUCTURE ONLY.

The C oracle (oracle/lf_oracle.c) is a CPU restatement of the reference's
LatticeFold commit+fold arithmetic, used as the parity checker for the HIP
product path. Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg may import this module. Arrays are numpy uint64 in AoS layout
(element-major, d u64 per ring element), canonical values in [0, p).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from pathlib import Path

import numpy as np

P = (1 << 64) - (1 << 32) + 1
_DIR = Path(__file__).resolve().parent
_LIB = _DIR / "liblf_oracle.so"
_lib = None

u64p = np.ctypeslib.ndpointer(dtype=np.uint64, flags="C_CONTIGUOUS")
u8p = np.ctypeslib.ndpointer(dtype=np.uint8, flags="C_CONTIGUOUS")
SZ, I, U64 = C.c_size_t, C.c_int, C.c_uint64


def build() -> Path:
    """Compile the oracle with its own Makefile (gcc only)."""
    subprocess.run(["make", "-s", "-C", str(_DIR)], check=True)
    return _LIB


class Transcript(C.Structure):
    _fields_ = [("state", U64 * 16), ("inbuf", U64 * 12), ("nin", I),
                ("outbuf", U64 * 12), ("nout", I)]


class Comb(C.Structure):
    _fields_ = [("kind", I), ("nk", I), ("tau", I), ("bsmall", I), ("mu", C.c_void_p), ("q", I),
                ("c", C.c_void_p), ("S_off", C.c_void_p), ("S_idx", C.c_void_p)]


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not _LIB.exists():
        build()
    L = C.CDLL(str(_LIB))
    sig = {
        "lfo_add": (U64, [U64, U64]), "lfo_sub": (U64, [U64, U64]),
        "lfo_mul": (U64, [U64, U64]), "lfo_pow": (U64, [U64, U64]),
        "lfo_inv": (U64, [U64]), "lfo_to_mont": (U64, [U64]), "lfo_from_mont": (U64, [U64]),
        "lfo_crt": (None, [u64p, SZ, I]), "lfo_icrt": (None, [u64p, SZ, I]),
        "lfo_phi72_homogenize": (None, [u64p]), "lfo_phi72_dehomogenize": (None, [u64p]),
        "lfo_poly_mul": (None, [u64p, u64p, u64p, I]),
        "lfo_slot_mul": (None, [u64p, u64p, u64p, I]),
        "lfo_decompose_balanced": (I, [U64, U64, I, u64p]),
        "lfo_gadget_decompose": (I, [u64p, SZ, I, U64, I, u64p]),
        "lfo_gadget_recompose": (None, [u64p, SZ, I, U64, I, u64p]),
        "lfo_witness_from_w_ccs": (I, [u64p, SZ, I, U64, I, u64p, u64p, I]),
        "lfo_witness_from_f": (None, [u64p, SZ, I, U64, I, u64p, u64p, I]),
        "lfo_get_fhat_phi72": (None, [u64p, SZ, u64p]),
        "lfo_ajtai_commit": (None, [u64p, SZ, SZ, I, u64p, SZ, u64p, I]),
        "lfo_decompose_witness": (I, [u64p, SZ, I, U64, I, U64, I, u64p, u64p, u64p, I]),
        "lfo_commit_witnesses_y0": (None, [u64p, u64p, SZ, I, U64, I]),
        "lfo_short_challenge": (I, [u8p, SZ, I, u64p]),
        "lfo_fold_f0": (None, [u64p, u64p, SZ, SZ, I, u64p, I]),
        "lfo_fold_cm0": (None, [u64p, u64p, SZ, SZ, I, u64p]),
        "lfo_p2_mds16": (None, [u64p]), "lfo_p2_permute": (None, [u64p]),
        "lfo_p2_permute_batch": (None, [u64p, SZ, I]),
        "lfo_p2_hash_iter": (None, [u64p, SZ, u64p]),
        "lfo_p2_permute_states": (None, [u64p, u64p]),
        "lfo_p2_hash_iter_states": (SZ, [u64p, SZ, u64p, u64p]),
        "lfo_tr_init": (None, [C.POINTER(Transcript)]),
        "lfo_tr_observe": (None, [C.POINTER(Transcript), U64]),
        "lfo_tr_sample": (U64, [C.POINTER(Transcript)]),
        "lfo_tr_absorb_ring": (None, [C.POINTER(Transcript), u64p, SZ, I]),
        "lfo_tr_get_challenge": (None, [C.POINTER(Transcript), u64p]),
        "lfo_tr_squeeze_bytes": (None, [C.POINTER(Transcript), u8p, SZ]),
        "lfo_fill_uniform": (None, [u64p, SZ, U64]),
        "lfo_ajtai_rows_seeded": (None, [U64, SZ, I, u64p, u64p, SZ, u64p, I]),
        "lfo_rot_lin_combination": (None, [u64p, u64p, SZ, I, u64p]),
        "lfo_eq_table": (None, [u64p, I, I, u64p]),
        "lfo_p2w8_permute": (None, [u64p]),
        "lfo_p2w8_hash": (None, [u64p, SZ, u64p]),
        "lfo_p2w8_compress": (None, [u64p, u64p, u64p]),
        "lfo_merkle_tree": (None, [u64p, SZ, SZ, u64p]),
        "lfo_merkle_nodes": (SZ, [SZ]),
        "lfo_spmv": (None, [u64p, np.ctypeslib.ndpointer(dtype=np.uint32, flags="C_CONTIGUOUS"), u64p, SZ, I,
                            u64p, u64p]),
        "lfo_mle_fix_first": (None, [u64p, SZ, I, u64p]),
        "lfo_mle_evaluate": (None, [u64p, I, I, u64p, u64p]),
        "lfo_comb_eval": (None, [C.POINTER(Comb), u64p, I, I, u64p]),
        "lfo_sumcheck_round": (None, [C.POINTER(Comb), u64p, I, I, I, I, u64p]),
        "lfo_sumcheck_prove": (None, [C.POINTER(Transcript), C.POINTER(Comb), u64p, I, I, I, I, u64p, u64p]),
        "lfo_sumcheck_check": (I, [u64p, u64p, I, I, I, u64p, u64p]),
        "lfo_compute_x_s": (I, [u64p, SZ, I, U64, I, U64, I, u64p]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def _u64(a) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a, dtype=np.uint64))


def nthreads_default() -> int:
    # os.cpu_count() is the whole machine on the GPU box; its CPU share is 16
    return int(os.environ.get("LF_ORACLE_THREADS", min(16, os.cpu_count() or 1)))


# ---------------------------------------------------------------- ring ops
def crt(elems, d: int) -> np.ndarray:
    x = _u64(elems).copy()
    lib().lfo_crt(x, x.size // d, d)
    return x


def icrt(elems, d: int) -> np.ndarray:
    x = _u64(elems).copy()
    lib().lfo_icrt(x, x.size // d, d)
    return x


def poly_mul(a, b, d: int) -> np.ndarray:
    out = np.zeros(d, np.uint64)
    lib().lfo_poly_mul(_u64(a), _u64(b), out, d)
    return out


def slot_mul(a, b, d: int) -> np.ndarray:
    out = np.zeros(d, np.uint64)
    lib().lfo_slot_mul(_u64(a), _u64(b), out, d)
    return out


def decompose_balanced(v: int, b: int, length: int):
    out = np.zeros(length, np.uint64)
    rc = lib().lfo_decompose_balanced(v, b, length, out)
    if rc:
        raise ValueError(f"decompose_balanced failed rc={rc}")
    return out


def gadget_decompose(elems, d: int, b: int, length: int) -> np.ndarray:
    x = _u64(elems)
    n = x.size // d
    out = np.zeros(n * length * d, np.uint64)
    if lib().lfo_gadget_decompose(x, n, d, b, length, out):
        raise ValueError("gadget_decompose: value needs more digits than padding_size")
    return out


def gadget_recompose(elems, d: int, b: int, length: int) -> np.ndarray:
    x = _u64(elems)
    n_out = x.size // (d * length)
    out = np.zeros(n_out * d, np.uint64)
    lib().lfo_gadget_recompose(x, n_out, d, b, length, out)
    return out


def witness_from_w_ccs(w_ccs, d: int, B: int, L: int, nthreads: int | None = None):
    x = _u64(w_ccs)
    W = x.size // d
    fc = np.zeros(W * L * d, np.uint64)
    f = np.zeros(W * L * d, np.uint64)
    if lib().lfo_witness_from_w_ccs(x, W, d, B, L, fc, f, nthreads or nthreads_default()):
        raise ValueError("from_w_ccs: decomposition overflow")
    return fc, f


def witness_from_f(f, d: int, B: int, L: int, nthreads: int | None = None):
    x = _u64(f)
    N = x.size // d
    fc = np.zeros(N * d, np.uint64)
    w = np.zeros((N // L) * d, np.uint64)
    lib().lfo_witness_from_f(x, N, d, B, L, fc, w, nthreads or nthreads_default())
    return fc, w


def get_fhat_phi72(f_coeff) -> np.ndarray:
    x = _u64(f_coeff)
    N = x.size // 24
    out = np.zeros(3 * N * 24, np.uint64)
    lib().lfo_get_fhat_phi72(x, N, out)
    return out


def ajtai_commit(A, kappa: int, ncols: int, d: int, f, nvec: int = 1,
                 nthreads: int | None = None) -> np.ndarray:
    cm = np.zeros(nvec * kappa * d, np.uint64)
    lib().lfo_ajtai_commit(_u64(A), kappa, ncols, d, _u64(f), nvec, cm,
                           nthreads or nthreads_default())
    return cm


def decompose_witness(f_coeff, d: int, B: int, L: int, b_small: int, K: int,
                      nthreads: int | None = None):
    x = _u64(f_coeff)
    N = x.size // d
    fck = np.zeros(K * N * d, np.uint64)
    fk = np.zeros(K * N * d, np.uint64)
    wk = np.zeros(K * (N // L) * d, np.uint64)
    if lib().lfo_decompose_witness(x, N, d, B, L, b_small, K, fck, fk, wk,
                                   nthreads or nthreads_default()):
        raise ValueError("decompose_witness: coefficient exceeds b_small^K range")
    return fck, fk, wk


def commit_witnesses_y0(cm, y, kappa: int, d: int, b_small: int, K: int) -> np.ndarray:
    yy = _u64(y).copy()
    lib().lfo_commit_witnesses_y0(_u64(cm), yy, kappa, d, b_small, K)
    return yy


def short_challenge(bs: bytes, d: int) -> np.ndarray:
    out = np.zeros(d, np.uint64)
    if lib().lfo_short_challenge(np.frombuffer(bytes(bs), np.uint8).copy(), len(bs), d, out):
        raise ValueError("short_challenge: wrong byte count")
    return out


def fold_f0(rho, f, nwit: int, N: int, d: int, nthreads: int | None = None) -> np.ndarray:
    out = np.zeros(N * d, np.uint64)
    lib().lfo_fold_f0(_u64(rho), _u64(f), nwit, N, d, out, nthreads or nthreads_default())
    return out


def fold_cm0(rho, cm, nwit: int, kappa: int, d: int) -> np.ndarray:
    out = np.zeros(kappa * d, np.uint64)
    lib().lfo_fold_cm0(_u64(rho), _u64(cm), nwit, kappa, d, out)
    return out


def tau(d: int) -> int:
    """NTT elements per f_hat evaluation / theta_i: the base ring's degree over Fq"""
    return 3 if d == 24 else 1


def rot_lin_combination(rho_coeff, theta, d: int) -> np.ndarray:
    r = _u64(rho_coeff)
    n = r.size // d
    out = np.zeros(tau(d) * d, np.uint64)
    lib().lfo_rot_lin_combination(r, _u64(theta), n, d, out)
    return out


def compute_x_s(x, d: int, B: int, L: int, b_small: int, K: int) -> np.ndarray:
    xx = _u64(x)
    m = xx.size // d
    out = np.zeros(K * m * d, np.uint64)
    if lib().lfo_compute_x_s(xx, m, d, B, L, b_small, K, out):
        raise ValueError("compute_x_s: decomposition overflow")
    return out


# ---------------------------------------------------------------- multilinear sumcheck
class SumcheckComb:
    """the combination function (lfo_comb): keeps its arrays alive"""

    def __init__(self, kind, nk=0, tau=0, bsmall=2, mu=None, c=None, S=None):
        self.keep = []
        mu_p = c_p = off_p = idx_p = None
        if mu is not None:
            mu = _u64(mu)
            self.keep.append(mu)
            mu_p = mu.ctypes.data
        q = 0
        if S is not None:
            c = _u64(c)
            off = np.zeros(len(S) + 1, np.int32)
            off[1:] = np.cumsum([len(x) for x in S])
            idx = np.array([j for x in S for j in x] or [0], np.int32)
            self.keep += [c, off, idx]
            c_p, off_p, idx_p, q = c.ctypes.data, off.ctypes.data, idx.ctypes.data, len(S)
        self.s = Comb(kind, nk, tau, bsmall, mu_p, q, c_p, off_p, idx_p)

    @classmethod
    def folding(cls, mu, nk, tau, bsmall=2):
        return cls(0, nk=nk, tau=tau, bsmall=bsmall, mu=mu)

    @classmethod
    def linearization(cls, c, S):
        return cls(1, c=c, S=S)


def eq_table(r, nv: int, d: int) -> np.ndarray:
    out = np.zeros((d << nv), np.uint64)
    lib().lfo_eq_table(_u64(r), nv, d, out)
    return out


def mle_evaluate(mle, nv: int, d: int, point) -> np.ndarray:
    out = np.zeros(d, np.uint64)
    lib().lfo_mle_evaluate(_u64(mle), nv, d, _u64(point), out)
    return out


def comb_eval(comb: SumcheckComb, vals, nm: int, d: int) -> np.ndarray:
    out = np.zeros(d, np.uint64)
    lib().lfo_comb_eval(C.byref(comb.s), _u64(vals), nm, d, out)
    return out


def sumcheck_round(comb: SumcheckComb, mles, nm: int, nv: int, d: int, degree: int) -> np.ndarray:
    out = np.zeros((degree + 1) * d, np.uint64)
    lib().lfo_sumcheck_round(C.byref(comb.s), _u64(mles), nm, nv, d, degree, out)
    return out


def sumcheck_prove(t: Transcript, comb: SumcheckComb, mles, nm: int, nv: int, d: int, degree: int):
    m = _u64(mles).copy()
    tau = 3 if d == 24 else 1
    proof = np.zeros(nv * (degree + 1) * d, np.uint64)
    rnd = np.zeros(nv * tau, np.uint64)
    lib().lfo_sumcheck_prove(C.byref(t), C.byref(comb.s), m, nm, nv, d, degree, proof, rnd)
    return proof, rnd


def sumcheck_check(proof, randomness, nv: int, d: int, degree: int, asserted_sum):
    out = np.zeros(d, np.uint64)
    rc = lib().lfo_sumcheck_check(_u64(proof), _u64(randomness), nv, d, degree, _u64(asserted_sum), out)
    return rc, out


# ---------------------------------------------------------------- sparse Mz products
def spmv(row_ptr, col, val, d: int, z) -> np.ndarray:
    """mat_vec_mul (LF/arith/utils.rs:52-65)"""
    rp = _u64(row_ptr)
    out = np.zeros((rp.size - 1) * d, np.uint64)
    lib().lfo_spmv(rp, np.ascontiguousarray(col, np.uint32), _u64(val), rp.size - 1, d, _u64(z), out)
    return out


def mz_mles(mats, z, nv: int, d: int) -> np.ndarray:
    """calculate_Mz_mles / compute_mz_mles (mle_helpers.rs:137-146): MLE(M_j z)
    for every matrix, zero-padded to 2^nv; mats: [(row_ptr, col, val)]"""
    out = []
    for rp, col, val in mats:
        y = spmv(rp, col, val, d, z)
        pad = np.zeros((1 << nv) * d, np.uint64)
        pad[:y.size] = y
        out.append(pad)
    return np.concatenate(out)


def mz_challenged(mats, zs, zetas, nv: int, d: int) -> np.ndarray:
    """calculate_challenged_mz_mle (folding.rs:208-234): for each instance i, Horner
    over the matrices in reverse (mle += M_j z_i; mle *= zeta_i), summed over i"""
    n = 1 << nv
    total = np.zeros(n * d, np.uint64)
    for z, zeta in zip(zs, zetas):
        ms = mz_mles(mats, z, nv, d).reshape(len(mats), n * d)
        mle = np.zeros(n * d, np.uint64)
        for j in reversed(range(len(mats))):
            mle = np.array([(int(a) + int(b)) % P for a, b in zip(mle, ms[j])], np.uint64)
            mle = np.concatenate([slot_mul(mle[x * d:(x + 1) * d], zeta, d) for x in range(n)])
        total = np.array([(int(a) + int(b)) % P for a, b in zip(total, mle)], np.uint64)
    return total


# ---------------------------------------------------------------- width-8 Poseidon2 Merkle trees
def p2w8_permute(state) -> np.ndarray:
    s = _u64(state).copy()
    lib().lfo_p2w8_permute(s)
    return s


def p2w8_hash(vals) -> np.ndarray:
    out = np.zeros(4, np.uint64)
    v = _u64(vals) if len(vals) else np.zeros(1, np.uint64)
    lib().lfo_p2w8_hash(v, len(vals), out)
    return out


def p2w8_compress(a, b) -> np.ndarray:
    out = np.zeros(4, np.uint64)
    lib().lfo_p2w8_compress(_u64(a), _u64(b), out)
    return out


def merkle_nodes(nrows: int) -> int:
    """digests in the padded layers of a tree over nrows rows (2 nrows - 1 for a power of two)"""
    return lib().lfo_merkle_nodes(nrows)


def merkle_tree(rows, nrows: int, width: int) -> np.ndarray:
    out = np.zeros(merkle_nodes(nrows) * 4, np.uint64)
    lib().lfo_merkle_tree(_u64(rows), nrows, width, out)
    return out


def broadcast(base, d: int) -> np.ndarray:
    """a base-ring element (tau words) in every NTT slot"""
    b = _u64(base)
    return np.tile(b, d // b.size)


# ---------------------------------------------------------------- Poseidon2
def p2_mds16(s) -> np.ndarray:
    x = _u64(s).copy()
    lib().lfo_p2_mds16(x)
    return x


def p2_permute(states, nthreads: int = 1) -> np.ndarray:
    x = _u64(states).copy()
    lib().lfo_p2_permute_batch(x, x.size // 16, nthreads)
    return x


def p2_hash_iter(vals) -> np.ndarray:
    out = np.zeros(4, np.uint64)
    x = _u64(vals) if len(vals) else np.zeros(1, np.uint64)
    lib().lfo_p2_hash_iter(x, len(vals), out)
    return out


def p2_permute_states(state) -> tuple[np.ndarray, np.ndarray]:
    """one permutation and its PermutationIntermediateStates (ZK/poseidon2.rs:91-96):
    (final state, 31 x 16 captured states)"""
    x = _u64(state).copy()
    st = np.zeros((31, 16), np.uint64)
    lib().lfo_p2_permute_states(x, st)
    return x, st


def p2_hash_iter_states(vals) -> tuple[np.ndarray, np.ndarray]:
    """hash_iter (ZK/poseidon2.rs:206-235): (digest, IntermediateStates as [nperm][31][16])"""
    n = len(vals)
    out = np.zeros(4, np.uint64)
    x = _u64(vals) if n else np.zeros(1, np.uint64)
    st = np.zeros((max(1, -(-n // 12)), 31, 16), np.uint64)
    k = lib().lfo_p2_hash_iter_states(x, n, out, st)
    return out, st[:k]


# ---------------------------------------------------------------- zkvm step commitments (ZK/commitments.rs)
def flatten_mont(elems, d: int = 24) -> np.ndarray:
    """commitments.rs:343-361 flatten(): ICRT every NTT element (ICRT::icrt), then each
    coefficient's ark limb `fq.0.0[0]` -- its Montgomery form -- as a Plonky3
    Goldilocks (from_u64). Canonical NTT elements in, Montgomery limbs out."""
    c = icrt(elems, d) if len(elems) else np.zeros(0, np.uint64)
    return np.array([to_mont(int(v)) for v in c], np.uint64)


def acc_comm(acc: dict, d: int = 24) -> np.ndarray:
    """ZkVmCommitter::acc_comm (commitments.rs:143-176): r, v, cm, u, x_w, h flattened
    in that order and hashed with hash_iter; acc holds canonical NTT elements"""
    parts = [flatten_mont(_u64(acc[k]).ravel(), d) for k in ("r", "v", "cm", "u", "x_w", "h")]
    return p2_hash_iter(np.concatenate(parts))


def ivc_step_comm(i: int, state0, state_i, accc) -> tuple[np.ndarray, np.ndarray]:
    """ZkVmCommitter::ivc_step_comm (commitments.rs:76-105): hash_iter of
    [i, state_0_comm, state_i_comm, acc_comm] (13 elements, 2 permutations)"""
    vals = [int(i) % P] + [int(x) for x in state0] + [int(x) for x in state_i] + [int(x) for x in accc]
    return p2_hash_iter_states(vals)


def state_i_comm(code_comm, pc: int, memory_comm, regs_comm, mem_ops_vec_comm) -> np.ndarray:
    """ZkVmCommitter::state_i_comm (commitments.rs:107-141), given code_comm and regs_comm"""
    vals = [int(x) for x in code_comm] + [int(pc) % P] + [int(x) for x in memory_comm] + \
           [int(x) for x in regs_comm] + [int(x) for x in mem_ops_vec_comm]
    return p2_hash_iter(vals)


def vm_regs_comm(regs) -> np.ndarray:
    """ZkVmCommitter::vm_regs_comm (commitments.rs:178-189): hash_iter of the 32 u32 registers"""
    return p2_hash_iter([int(r) & 0xFFFFFFFF for r in regs])


def vm_mem_ops_vec_comm(prev, cycle: int, address: int, value: int) -> np.ndarray:
    """ZkVmCommitter::vm_mem_ops_vec_comm (commitments.rs:290-307): TruncatedPermutation<8>
    compress of [prev, (cycle, address, value, 0)]"""
    return p2w8_compress(_u64(prev), _u64([cycle % P, address & 0xFFFFFFFF, value & 0xFFFFFFFF, 0]))


def new_transcript() -> Transcript:
    t = Transcript()
    lib().lfo_tr_init(C.byref(t))
    return t


def fill_uniform(n: int, seed: int) -> np.ndarray:
    out = np.zeros(n, np.uint64)
    lib().lfo_fill_uniform(out, n, seed)
    return out


def ajtai_rows_seeded(seed: int, ncols: int, d: int, f, rows, nthreads: int | None = None) -> np.ndarray:
    """rows of A f with A = fill_uniform(kappa * ncols * d, seed) generated on the fly"""
    r = np.ascontiguousarray(np.asarray(rows, dtype=np.uint64))
    out = np.zeros(r.size * d, np.uint64)
    lib().lfo_ajtai_rows_seeded(seed, ncols, d, _u64(f), r, r.size, out, nthreads or nthreads_default())
    return out


def to_mont(a: int) -> int:
    return lib().lfo_to_mont(a)


def from_mont(a: int) -> int:
    return lib().lfo_from_mont(a)
