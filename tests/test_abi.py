"""C-ABI checks that need no GPU: the library loads, exports every symbol
include/lf.h declares, and its host-only logic (short challenges, transcript,
hash_iter) matches the oracle / reference KATs."""
import json
import re
from pathlib import Path

import numpy as np
import pytest

import latticeum_amd as LA
import oracle as O
from latticeum_amd import _lib

ROOT = Path(__file__).resolve().parents[1]
KATS = json.loads((ROOT / "tests/golden/reference_kats.json").read_text())


def header_symbols():
    txt = (ROOT / "include/lf.h").read_text()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(lf_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_header_symbol():
    lib = _lib.load()
    syms = header_symbols()
    assert len(syms) >= 50
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    # and the Python binding declares a signature for each of them
    assert sorted(_lib.SIGNATURES) == syms


def test_goldilocks_dp():
    p = LA.goldilocks_dp(24)
    assert (p.d, p.B, p.L, p.b_small, p.K) == (24, 1 << 15, 5, 2, 15)


def test_short_challenge_kat():
    k = KATS["short_challenge"]
    assert [int(x) for x in LA.short_challenge(bytes(k["bytes"]), 24)] == k["coeffs"]
    with pytest.raises(LA.LfError):
        LA.short_challenge(bytes(17), 24)


def test_short_challenge_nega_matches_oracle():
    rng = np.random.default_rng(3)
    bs = rng.integers(0, 256, 768, dtype=np.uint8).tobytes()
    assert np.array_equal(LA.short_challenge(bs, 1024), O.short_challenge(bs, 1024))


@pytest.mark.parametrize("n", [0, 1, 11, 12, 13, 24, 25, 182 * 24])
def test_hash_iter_matches_oracle(n):
    vals = O.fill_uniform(max(n, 1), 1000 + n)[:n]
    assert np.array_equal(LA.hash_iter(vals), O.p2_hash_iter(vals))


@pytest.mark.parametrize("fill", ["p-1", "max", "edges"])
def test_hash_iter_edge_values_match_oracle(fill):
    """the host permutation keeps its state weakly reduced (transcript.cpp):
    inputs at the top of the field and of u64 (canonicalised on absorption), and
    a mix of 0, 1, p-1, 2^63 and 2^64-1, against the oracle's canonical one"""
    P = (1 << 64) - (1 << 32) + 1
    n = 12 * 40 + 5
    if fill == "p-1":
        vals = np.full(n, P - 1, np.uint64)
    elif fill == "max":
        vals = np.full(n, (1 << 64) - 1, np.uint64)
    else:
        edge = np.array([0, 1, P - 1, P - 2, 1 << 63, (1 << 64) - 1, (1 << 32) - 1, 1 << 32], np.uint64)
        vals = edge[np.arange(n) % len(edge)]
    canon = np.where(vals >= np.uint64(P), vals - np.uint64(P), vals).astype(np.uint64)
    assert np.array_equal(LA.hash_iter(vals), O.p2_hash_iter(canon))


def test_transcript_matches_oracle():
    t = LA.Poseidon2Transcript()
    o = O.new_transcript()
    L = O.lib()
    import ctypes as C
    elems = O.fill_uniform(24 * 7, 42)
    t.absorb_ring(elems, 24)
    L.lfo_tr_absorb_ring(C.byref(o), elems, 7, 24)
    ch = t.get_challenge()
    och = np.zeros(3, np.uint64)
    L.lfo_tr_get_challenge(C.byref(o), och)
    assert np.array_equal(ch, och)
    for v in [5, 6, 7]:
        t.observe(v)
        L.lfo_tr_observe(C.byref(o), v)
    b = t.squeeze_bytes(18)
    ob = np.zeros(18, np.uint8)
    L.lfo_tr_squeeze_bytes(C.byref(o), ob, 18)
    assert b == ob.tobytes()
    # absorbs that start mid-block and end mid-block, between observes and samples
    for k, (pre, nel, dd) in enumerate([(5, 3, 24), (0, 1, 24), (11, 2, 16), (0, 5, 16), (7, 1, 1024)]):
        for v in range(pre):
            t.observe(100 + v)
            L.lfo_tr_observe(C.byref(o), 100 + v)
        x = O.fill_uniform(nel * dd, 50 + k)
        t.absorb_ring(x, dd)
        L.lfo_tr_absorb_ring(C.byref(o), x, nel, dd)
        assert t.sample() == L.lfo_tr_sample(C.byref(o)), k
    # Montgomery-repr absorb is the same stream as canonical absorb
    t1, t2 = LA.Poseidon2Transcript(), LA.Poseidon2Transcript()
    t1.absorb_ring(elems, 24)
    t2.absorb_ring(np.array([O.to_mont(int(x)) for x in elems], np.uint64), 24, LA.REPR_MONTGOMERY)
    assert t1.sample() == t2.sample()


def test_short_challenges_from_transcript():
    t = LA.Poseidon2Transcript()
    rhos = t.get_short_challenges(24, 29).reshape(29, 24)
    P = LA.P
    signed = np.where(rhos > (P - 1) // 2, rhos.astype(object) - P, rhos.astype(object))
    assert all(-32 <= int(x) < 32 for x in signed.ravel())


def test_context_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(LA.LfError):
        LA.Context(0)
