"""The wire format of the accumulator and the folding proof (include/lf.h
lf_lcccs_* / lf_lfproof_serialize): ark-serialize 0.5 CanonicalSerialize of
the reference's types (latticefold/src/nifs.rs:28-34, arith.rs:192-206).
Host-side byte layouts; numpy uint64 ring elements of d words each."""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import LfDecompositionProof, LfLcccs, LfLfproof, LfRingSlice, load

REPR_CANONICAL, REPR_MONTGOMERY = 0, 1


class LfError(RuntimeError):
    pass


def _slice(a, d, keep):
    a = np.ascontiguousarray(np.asarray(a, np.uint64)).ravel()
    keep.append(a)
    return LfRingSlice(a.ctypes.data_as(C.c_void_p) if a.size else None, a.size // d)


def _slices(vs, d, keep):
    arr = (LfRingSlice * max(1, len(vs)))(*[_slice(v, d, keep) for v in vs])
    keep.append(arr)
    return C.cast(arr, C.c_void_p), len(vs)


def _run(fn, *args):
    n = C.c_size_t()
    rc = fn(*args, None, 0, C.byref(n))
    if rc not in (0, 7):
        raise LfError(f"serialize rc={rc}")
    buf = (C.c_uint8 * max(1, n.value))()
    rc = fn(*args, buf, n.value, C.byref(n))
    if rc:
        raise LfError(f"serialize rc={rc}")
    return bytes(buf)[:n.value]


def serialize_lcccs(d, r, v, cm, u, x_w, h, repr=REPR_CANONICAL) -> bytes:
    keep = []
    acc = LfLcccs(d, _slice(r, d, keep), _slice(v, d, keep), _slice(cm, d, keep), _slice(u, d, keep),
                  _slice(x_w, d, keep), None)
    hh = np.ascontiguousarray(np.asarray(h, np.uint64))
    acc.h = hh.ctypes.data_as(C.c_void_p)
    return _run(load().lf_lcccs_serialize, C.byref(acc), repr)


def deserialize_lcccs(data: bytes, d: int, repr=REPR_CANONICAL) -> dict:
    raw = np.frombuffer(bytes(data), np.uint8).copy()
    buf = np.zeros(max(1, raw.size // 8 + d), np.uint64)
    out = LfLcccs()
    rc = load().lf_lcccs_deserialize(raw.ctypes.data_as(C.c_void_p), raw.size, d, repr,
                                     buf.ctypes.data_as(C.c_void_p), buf.size, C.byref(out))
    if rc:
        raise LfError(f"deserialize rc={rc}")
    base = buf.ctypes.data

    def take(s):
        off = (s.elems - base) // 8 if s.elems else 0
        return buf[off:off + s.n * d].copy()
    res = {k: take(getattr(out, k)) for k in ("r", "v", "cm", "u", "x_w")}
    off = (out.h - base) // 8
    res["h"] = buf[off:off + d].copy()
    return res


def serialize_lfproof(d, lin_sumcheck, lin_rounds, lin_evals, lin_v, lin_u, dec, fold_sumcheck, fold_rounds,
                      fold_evals, theta_s, eta_s, repr=REPR_CANONICAL) -> bytes:
    """dec: two dicts with u_s, v_s, x_s, y_s (lists of ring-element arrays)"""
    keep = []
    p = LfLfproof()
    p.d = d
    ls = np.ascontiguousarray(np.asarray(lin_sumcheck, np.uint64))
    fs = np.ascontiguousarray(np.asarray(fold_sumcheck, np.uint64))
    keep += [ls, fs]
    p.lin_sumcheck, p.lin_rounds, p.lin_evals = ls.ctypes.data_as(C.c_void_p), lin_rounds, lin_evals
    p.lin_v, p.lin_u = _slice(lin_v, d, keep), _slice(lin_u, d, keep)
    for s in range(2):
        dp = LfDecompositionProof()
        dp.u_s, dp.n_u = _slices(dec[s]["u_s"], d, keep)
        dp.v_s, dp.n_v = _slices(dec[s]["v_s"], d, keep)
        dp.x_s, dp.n_x = _slices(dec[s]["x_s"], d, keep)
        dp.y_s, dp.n_y = _slices(dec[s]["y_s"], d, keep)
        p.dec[s] = dp
    p.fold_sumcheck, p.fold_rounds, p.fold_evals = fs.ctypes.data_as(C.c_void_p), fold_rounds, fold_evals
    p.theta_s, p.n_theta = _slices(theta_s, d, keep)
    p.eta_s, p.n_eta = _slices(eta_s, d, keep)
    return _run(load().lf_lfproof_serialize, C.byref(p), repr)
