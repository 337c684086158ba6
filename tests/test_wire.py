"""The wire format against a plain restatement of
ark-serialize 0.5's derived CanonicalSerialize (u64 LE lengths, 8-byte LE
canonical field elements, fields in declaration order): LCCCS round trips,
Montgomery-limb input, the LFProof layout, and its size at the zkvm's shape.
The reference holds no serialized bytes, so the format is pinned by its
definition only (parity unpinned against reference bytes)."""
import struct

import numpy as np
import pytest

import oracle as O
from latticeum_amd import wire

P = O.P


def ark_vec(elems, d):
    e = np.asarray(elems, np.uint64).ravel()
    return struct.pack("<Q", e.size // d) + b"".join(struct.pack("<Q", int(x)) for x in e)


def ark_vecvec(vs, d):
    return struct.pack("<Q", len(vs)) + b"".join(ark_vec(v, d) for v in vs)


def rnd(n, seed):
    return O.fill_uniform(n, seed)


@pytest.mark.parametrize("d", [24, 16])
def test_lcccs_layout_and_round_trip(d):
    f = {"r": rnd(17 * d, 1), "v": rnd(3 * d, 2), "cm": rnd(32 * d, 3), "u": rnd(125 * d, 4), "x_w": rnd(4 * d, 5)}
    h = rnd(d, 6)
    b = wire.serialize_lcccs(d, f["r"], f["v"], f["cm"], f["u"], f["x_w"], h)
    want = b"".join(ark_vec(f[k], d) for k in ("r", "v", "cm", "u", "x_w")) + b"".join(
        struct.pack("<Q", int(x)) for x in h)
    assert b == want
    back = wire.deserialize_lcccs(b, d)
    for k in f:
        assert np.array_equal(back[k], f[k])
    assert np.array_equal(back["h"], h)
    # Montgomery limbs in (a Rust caller's memory) -> canonical bytes out, and back
    mont = {k: np.array([O.to_mont(int(x)) for x in v], np.uint64) for k, v in f.items()}
    hm = np.array([O.to_mont(int(x)) for x in h], np.uint64)
    bm = wire.serialize_lcccs(d, mont["r"], mont["v"], mont["cm"], mont["u"], mont["x_w"], hm, repr=wire.REPR_MONTGOMERY)
    assert bm == b
    backm = wire.deserialize_lcccs(b, d, repr=wire.REPR_MONTGOMERY)
    assert np.array_equal(backm["u"], mont["u"])


def test_lcccs_rejects_bad_bytes():
    d = 24
    b = wire.serialize_lcccs(d, rnd(d, 1), [], [], [], [], rnd(d, 2))
    with pytest.raises(wire.LfError):
        wire.deserialize_lcccs(b[:-1], d)  # truncated
    bad = bytearray(b)
    bad[8:16] = struct.pack("<Q", P)  # a non-canonical field element
    with pytest.raises(wire.LfError):
        wire.deserialize_lcccs(bytes(bad), d)


def test_lfproof_layout_zkvm_shape():
    """LFProof at the zkvm's shape: linearization sumcheck 17 rounds x (d_ccs + 2 = 9)
    evaluations, v (tau = 3), u (t = 125); two decomposition proofs with K = 15 u_s
    (125 each), v_s (3), x_s (l + 1 = 5), y_s (kappa = 32); the folding sumcheck 17 x 5,
    theta_s 30 x 3, eta_s 30 x 125"""
    d, K, t, kappa = 24, 15, 125, 32
    ls, fs = rnd(17 * 9 * d, 10), rnd(17 * 5 * d, 11)
    lv, lu = rnd(3 * d, 12), rnd(t * d, 13)
    dec = [{"u_s": [rnd(t * d, 20 + s * 100 + i) for i in range(K)],
            "v_s": [rnd(3 * d, 40 + s * 100 + i) for i in range(K)],
            "x_s": [rnd(5 * d, 60 + s * 100 + i) for i in range(K)],
            "y_s": [rnd(kappa * d, 80 + s * 100 + i) for i in range(K)]} for s in range(2)]
    th = [rnd(3 * d, 300 + i) for i in range(2 * K)]
    et = [rnd(t * d, 400 + i) for i in range(2 * K)]
    b = wire.serialize_lfproof(d, ls, 17, 9, lv, lu, dec, fs, 17, 5, th, et)
    want = (ark_vecvec([ls[r * 9 * d:(r + 1) * 9 * d] for r in range(17)], d) + ark_vec(lv, d) + ark_vec(lu, d))
    for s in range(2):
        want += b"".join(ark_vecvec(dec[s][k], d) for k in ("u_s", "v_s", "x_s", "y_s"))
    want += ark_vecvec([fs[r * 5 * d:(r + 1) * 5 * d] for r in range(17)], d) + ark_vecvec(th, d) + ark_vecvec(et, d)
    assert b == want
    elems = 17 * 9 + 3 + t + 2 * K * (t + 3 + 5 + kappa) + 17 * 5 + 2 * K * 3 + 2 * K * t
    lens = (1 + 17) + 2 + 2 * (4 + 4 * K) + (1 + 17) + (1 + 2 * K) * 2
    assert len(b) == elems * d * 8 + lens * 8
