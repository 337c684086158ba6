"""The zkvm's IVC step commitments (zkvm/src/commitments.rs, poseidon2.rs:91-235) on
the host side of the C ABI against the oracle's composition:

  * hash_iter's IntermediateStates (31 captured states per permutation), whose
    first two records (after the initial MDS, after external round 0) are pinned
    by the reference's own Poseidon2 vector P3 (sages/inverse_mds.sage:29-76);
  * acc_comm over an LCCCS at the zkvm's shape (r 17, v 3, cm 32, u 125, x_w 4,
    h 1: 182 ring elements -> 4,368 Montgomery limbs -> 364 permutations), in
    both representations;
  * ivc_step_comm (13 elements, 2 permutations, states kept), state_i_comm,
    vm_regs_comm and vm_mem_ops_vec_comm.
The full permutation itself is parity unpinned (no 16 -> 16 KAT in the
reference), so beyond P3 these are equalities with the restated oracle."""
import json
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))

import latticeum_amd as LA  # noqa: E402
import oracle as O  # noqa: E402

KATS = json.loads((ROOT / "tests/golden/reference_kats.json").read_text())
ZKVM_LCCCS = {"r": 17, "v": 3, "cm": 32, "u": 125, "x_w": 4, "h": 1}  # ccs.rs:43-67, LCCCS arith.rs:192-206


def lcccs(seed, shape=ZKVM_LCCCS, d=24):
    return {k: O.fill_uniform(n * d, seed + i) for i, (k, n) in enumerate(shape.items())}


@pytest.mark.parametrize("n", [0, 1, 11, 12, 13, 24, 25, 100, 4368])
def test_hash_iter_states_match_oracle(n):
    v = O.fill_uniform(n, 0x4C46_0100 + n)
    dg, st = LA.hash_iter_states(v)
    odg, ost = O.p2_hash_iter_states(v)
    assert st.shape == (-(-n // 12), 31, 16) == ost.shape
    assert np.array_equal(dg, odg) and np.array_equal(st, ost)
    assert np.array_equal(dg, LA.hash_iter(v))
    if n:  # the last record is the final state, whose first 4 words are the digest
        assert np.array_equal(st[-1, -1, :4], dg)


def test_captured_states_pinned_by_p3():
    """P3 (inverse_mds.sage): v with v[12..16) = 0 is exactly the state hash_iter
    permutes for the input v[0..12); its after_initial_mds record must be MDS16(v)
    and its after_ext_init_rounds[0] record MDS16((MDS16(v) + consts_0)^7)."""
    k = KATS["poseidon2"]["P3_round0"]
    v = [int(x) for x in k["input"]]
    assert len(v) == 16 and v[12:] == [0, 0, 0, 0]
    _, st = LA.hash_iter_states(v[:12])
    assert [int(x) for x in st[0, 0]] == [int(x) for x in O.p2_mds16(v)]
    assert [int(x) for x in st[0, 1]] == k["mds_sbox_mds"]
    _, ost = O.p2_permute_states(v)
    assert np.array_equal(st[0], ost)


def test_states_follow_the_round_structure():
    """after_internal_rounds[r] differ from the previous record only through the
    internal layer: state_i = s_i diag_i + sum (s_0 S-boxed first); checked on the
    host from consecutive records with the oracle's field ops"""
    _, st = LA.hash_iter_states(O.fill_uniform(12, 7))
    P = LA.P
    txt = (ROOT / "oracle/p2_consts.inc").read_text()
    nums = lambda name: [int(x, 16) for x in txt.split(name)[1].split("}")[0].replace("{", "").replace(
        "ull", "").replace("\\", "").replace(",", " ").split() if x.startswith("0x")]
    internal, diag = nums("LF_P2_INTERNAL"), nums("LF_P2_DIAG_M1")
    for r in range(22):
        s = [int(x) for x in st[0, 4 + r]]
        s[0] = pow((s[0] + internal[r]) % P, 7, P)
        tot = sum(s) % P
        assert [int(x) for x in st[0, 5 + r]] == [(s[i] * diag[i] + tot) % P for i in range(16)]


@pytest.mark.parametrize("repr_", [LA.REPR_CANONICAL, LA.REPR_MONTGOMERY])
def test_acc_comm_zkvm_shape(repr_):
    acc = lcccs(0x4C46_0200)
    want = O.acc_comm(acc)
    if repr_ == LA.REPR_MONTGOMERY:
        acc = {k: np.array([O.to_mont(int(x)) for x in v], np.uint64) for k, v in acc.items()}
    assert np.array_equal(LA.acc_comm(acc, repr=repr_), want)
    # 182 ring elements -> 4,368 limbs -> 364 permutations
    assert sum(ZKVM_LCCCS.values()) * 24 == 4368 and LA.load().lf_hash_iter_nperm(4368) == 364


def test_acc_comm_hashes_montgomery_limbs_of_the_coefficients():
    """flatten (commitments.rs:349-361) hashes fq.0.0[0], the ark Montgomery limb of
    each ICRT coefficient: an LCCCS whose only nonzero element is h = ONE (NTT form
    of 1) flattens to [R, 0, ..., 0] at h's position"""
    shape = {"r": 1, "v": 1, "cm": 1, "u": 1, "x_w": 1, "h": 1}
    acc = {k: np.zeros(24, np.uint64) for k in shape}
    acc["h"] = O.crt(np.array([1] + [0] * 23, np.uint64), 24)
    flat = np.zeros(6 * 24, np.uint64)
    flat[5 * 24] = (1 << 64) % LA.P  # R = 2^64 mod p = 2^32 - 1
    assert np.array_equal(LA.acc_comm(acc), O.p2_hash_iter(flat))


def test_acc_comm_rejects_other_rings():
    acc = lcccs(1, {"r": 1, "v": 1, "cm": 1, "u": 1, "x_w": 1, "h": 1}, d=16)
    with pytest.raises(LA.LfError):
        LA.acc_comm(acc, d=16)


def test_ivc_step_comm_and_state_parts():
    s0, si, ac = O.fill_uniform(4, 1), O.fill_uniform(4, 2), O.fill_uniform(4, 3)
    for i in (0, 1, 17, 99):
        dg, st = LA.ivc_step_comm(i, s0, si, ac)
        odg, ost = O.ivc_step_comm(i, s0, si, ac)
        assert st.shape == (2, 31, 16)  # ccs.rs:520 asserts two permutations
        assert np.array_equal(dg, odg) and np.array_equal(st, ost)
    code, mem, regs, ops = (O.fill_uniform(4, 10 + k) for k in range(4))
    assert np.array_equal(LA.state_i_comm(code, 0x1000, mem, regs, ops),
                          O.state_i_comm(code, 0x1000, mem, regs, ops))
    r = np.random.default_rng(5).integers(0, 1 << 32, 32, dtype=np.uint64).astype(np.uint32)
    assert np.array_equal(LA.vm_regs_comm(r), O.vm_regs_comm(r))
    prev = np.zeros(4, np.uint64)  # ZERO_GOLDILOCKS_COMM, the chain's start (main.rs:95)
    for cyc, addr, val in ((0, 0x604, 1), (7, 0xFFFFFFFC, 0xDEADBEEF)):
        got = LA.vm_mem_ops_vec_comm(prev, cyc, addr, val)
        assert np.array_equal(got, O.vm_mem_ops_vec_comm(prev, cyc, addr, val))
        prev = got


def test_hash_iter_states_capacity_checked():
    lib = LA.load()
    x = O.fill_uniform(25, 1)
    out = np.zeros(4, np.uint64)
    st = np.zeros((2, 31, 16), np.uint64)
    assert lib.lf_hash_iter_states(x.ctypes.data, 25, out.ctypes.data, st.ctypes.data, 2) != 0  # needs 3
    assert lib.lf_hash_iter_states(x.ctypes.data, 25, out.ctypes.data, None, 0) == 0
    assert np.array_equal(out, O.p2_hash_iter(x))


def test_permutation_avx512_and_scalar_agree():
    """the host permutation's AVX-512 form (selected at run time) and its scalar form
    (LATTICEUM_AMD_P2_SCALAR=1, in a child process) give the same hash_iter digests and
    transcript samples, on random and extreme inputs, both equal to the oracle's"""
    import subprocess
    import os
    rng = np.random.default_rng(9)
    xs = [rng.integers(0, LA.P, 12 * 40 + 5, dtype=np.uint64),
          np.full(100, LA.P - 1, np.uint64), np.zeros(13, np.uint64)]
    code = ("import sys, numpy as np; sys.path.insert(0, %r); import latticeum_amd as LA\n"
            "rng = np.random.default_rng(9)\n"
            "xs = [rng.integers(0, LA.P, 12 * 40 + 5, dtype=np.uint64), np.full(100, LA.P - 1, np.uint64), "
            "np.zeros(13, np.uint64)]\n"
            "print(' '.join(str(int(v)) for x in xs for v in LA.hash_iter(x)))\n") % str(ROOT)
    outs = []
    for flag in ("0", "1"):
        env = dict(os.environ, LATTICEUM_AMD_P2_SCALAR=flag)
        r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr
        outs.append(r.stdout.split())
    assert outs[0] == outs[1]
    want = [str(int(v)) for x in xs for v in O.p2_hash_iter(x)]
    assert outs[0] == want
