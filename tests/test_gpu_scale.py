"""GPU parity at the benchmarked sizes.

bench.py times one commit+fold step at d=1024, W=2^14, kappa=32 (BASELINE.json
configs[2]) and the configs[4] ring d=4096 with kappa=64. At those sizes the
kernels run other instantiations than at oracle-friendly sizes (streaming
stores and copies above 4 GiB per launch, >2^32-element offsets, the 21.5 GB
fragment matrix, kappa tiles), so this file runs bench.py's own Workload and
checks its outputs against the oracle:

* whole vectors where the oracle is cheap (Witness::from_w_ccs of both sides);
* sampled 16-group blocks of every per-element output (every output element
  depends only on its own element or group): the K digit witnesses of both
  sides, f_0, Witness::from_f(f_0);
* commitment rows against an oracle Ajtai that generates A from its seed on
  the fly (no host copy of the matrix): commit(z)'s cm, the accumulator's cm,
  and y_k rows of both sides;
* y_0 and cm_0 recomputed on the host from the device's y and cm.

It also runs the full 2^16-polynomial d=1024 NTT batch (configs[1]) and the
witness kernels past their grid-stride cap.
"""
import numpy as np
import pytest

import latticeum_amd as LA
import oracle as O

import bench

pytestmark = pytest.mark.gpu
P = LA.P


def host(t):
    return t.cpu().numpy().view(np.uint64)


def blocks_to_groups(W, nblk_pick):
    nblk = (W + 15) // 16
    groups = []
    for B in sorted(set(b % nblk for b in nblk_pick)):
        groups.extend(range(16 * B, min(W, 16 * B + 16)))
    return np.array(groups)


class _LeanPlanes:
    """The packed digit planes (d = 1024 / 4096: column-major, one fixed-size
    record per element) expanded a column block at a time, so a check never holds
    a side's K x N u64 rows (20 GB per step at W = 2^14) beside bench.py's
    8-stream workload (about 240 of the 288 GB)."""

    def __init__(self, wl, planes, block=8192):
        self.wl, self.planes, self.block = wl, planes, block
        K, d = wl.pr.K, wl.d
        self.per_col = 256 if d == 1024 else K * 128  # int64 words per element (lf.h planes layout)

    def _expand(self, s, c0, n):
        import torch
        wl = self.wl
        K, d = wl.pr.K, wl.d
        p = self.planes[s]
        fck, fk = (torch.empty(K * n * d, dtype=torch.int64, device=p.device) for _ in range(2))
        wl.ctxs[0].dev_expand_planes(wl.pr, p.data_ptr() + 8 * c0 * self.per_col, n, fck, fk)
        wl.ctxs[0].sync()
        return fck.view(K, n, d), fk.view(K, n, d)

    def full_planes(self, s, ks):
        """host f_k rows of planes `ks` over all N columns: {k: [N d] u64}"""
        N, d = self.wl.N, self.wl.d
        out = {k: np.empty(N * d, np.uint64) for k in ks}
        for c0 in range(0, N, self.block):
            n = min(self.block, N - c0)
            _, fk = self._expand(s, c0, n)
            for k in ks:
                out[k][c0 * d:(c0 + n) * d] = host(fk[k].contiguous()).ravel()
            del fk
        return out

    def cols(self, s, groups):
        """host (f_coeff_k, f_k) [K][len(cols)][d] of the columns of `groups` (whole 16-group blocks)"""
        L = self.wl.pr.L
        fcs, fks = [], []
        blocks = sorted(set(int(g) // 16 for g in groups))
        for B in blocks:
            g0, g1 = 16 * B, min(self.wl.W, 16 * B + 16)
            fck, fk = self._expand(s, g0 * L, (g1 - g0) * L)
            fcs.append(host(fck.contiguous()).reshape(fck.shape))
            fks.append(host(fk.contiguous()).reshape(fk.shape))
        return np.concatenate(fcs, axis=1), np.concatenate(fks, axis=1)


def check_workload(wl, seed_w, picks, cm_rows, y_rows, stream=0, lean_expand=False):
    """bench.Workload `wl` has run its steps on step stream `stream`; compare the
    outputs against the oracle. lean_expand: expand packed planes column block
    by column block (HBM-tight workloads)."""
    import torch
    d, W, kappa, pr = wl.d, wl.W, wl.kappa, wl.pr
    K, L, N = pr.K, pr.L, wl.N
    keep = wl.keeps[stream]
    seed_w += 104729 * stream  # bench.Workload's per-stream w_ccs seed
    torch.cuda.synchronize()
    # commit(z) side: Witness::from_w_ccs of the whole vector
    w_ccs = O.fill_uniform(W * d, seed_w)
    assert np.array_equal(host(keep["w_ccs"]), w_ccs)
    fc1, f1 = O.witness_from_w_ccs(w_ccs, d, pr.B, L)
    assert np.array_equal(host(keep["f_coeff"]), fc1), "from_w_ccs f_coeff"
    assert np.array_equal(host(keep["f"]), f1), "from_w_ccs f"
    # accumulator side: a previous witness built the reference way
    fc0, f0acc = O.witness_from_w_ccs(O.fill_uniform(W * d, bench.SEED_ACC), d, pr.B, L)
    assert np.array_equal(host(keep["acc_f_coeff"]), fc0), "accumulator f_coeff"
    # commitments: rows of A f with A generated from its seed
    cm = host(keep["cm"]).reshape(kappa, d)
    acc_cm = host(keep["acc_cm"]).reshape(kappa, d)
    got = O.ajtai_rows_seeded(bench.SEED_A, N, d, f1, cm_rows).reshape(len(cm_rows), d)
    assert np.array_equal(cm[cm_rows], got), "commit(z) cm rows"
    got = O.ajtai_rows_seeded(bench.SEED_A, N, d, f0acc, cm_rows[:2]).reshape(2, d)
    assert np.array_equal(acc_cm[cm_rows[:2]], got), "accumulator cm rows"
    # rho: 29 decoded short challenges + ONE, NTT form (as bench.Workload makes them)
    rng = np.random.default_rng(bench.SEED_RHO)
    rc = [O.short_challenge(rng.integers(0, 256, 3 * d // 4, dtype=np.uint8).tobytes(), d) for _ in range(2 * K - 1)]
    one = np.zeros(d, np.uint64)
    one[0] = 1
    rho = O.crt(np.concatenate(rc + [one]), d)
    assert np.array_equal(host(keep["rho"]), rho)
    # y rows of both sides: the decomposition's own operand rows through the contraction
    y = [host(t).reshape(K, kappa, d) for t in keep["y"]]
    fk_dev, fck_dev = keep["fk"], keep["fk_coeff"]
    lean = None  # packed planes expanded column block by column block (bench.py's 8-stream HBM footprint)
    if keep.get("planes", [None])[0] is not None and fk_dev[0] is None:
        if lean_expand and d in (1024, 4096):
            lean = _LeanPlanes(wl, keep["planes"])
        else:
            # the step kept its planes packed: the u64 rows as lf_dev_expand_planes makes them
            fk_dev, fck_dev = [], []
            for s in range(2):
                fck, fk = (torch.empty(K * N * d, dtype=torch.int64, device=keep["f"].device) for _ in range(2))
                wl.ctxs[0].dev_expand_planes(pr, keep["planes"][s], N, fck, fk)
                fk_dev.append(fk)
                fck_dev.append(fck)
            wl.ctxs[0].sync()
    elif fk_dev[0] is None:
        # the step kept its planes only as operand rows: decompose both sides
        # again through the standalone entry (parity-tested on its own)
        fk_dev = []
        for s, src in ((0, keep["acc_f_coeff"]), (1, keep["f_coeff"])):
            fck, fk, wk = (torch.empty(n, dtype=torch.int64, device=src.device) for n in (K * N * d, K * N * d,
                                                                                          K * W * d))
            wl.ctxs[0].dev_decompose_witness(pr, src, N, fck, fk, wk)
            wl.ctxs[0].sync()
            assert torch.equal(fck, keep["fk_coeff"][s]) and torch.equal(wk, keep["wk"][s]), f"side {s}"
            del fck, wk
            fk_dev.append(fk)
    if lean is not None:
        want_k = {s: sorted({k for s2, k, _ in y_rows if s2 == s}) for s in range(2)}
        planes_k = {s: lean.full_planes(s, want_k[s]) for s in range(2) if want_k[s]}
    for s, k, row in y_rows:
        fk = planes_k[s][k] if lean is not None else host(fk_dev[s][k * N * d:(k + 1) * N * d])
        got = O.ajtai_rows_seeded(bench.SEED_A, N, d, fk, [row])
        assert np.array_equal(y[s][k, row], got), f"y side {s} k {k} row {row}"
    # y_0 = cm - sum 2^k y_k and cm_0 = sum rho_i y_i, recomputed from the device's y
    for s, c in ((0, acc_cm), (1, cm)):
        yy = y[s].copy()
        yy[0] = 0
        want = O.commit_witnesses_y0(c.ravel(), yy.ravel(), kappa, d, pr.b_small, K).reshape(K, kappa, d)
        assert np.array_equal(y[s][0], want[0]), f"y_0 side {s}"
    cm0 = O.fold_cm0(rho, np.concatenate([y[0].ravel(), y[1].ravel()]), 2 * K, kappa, d)
    assert np.array_equal(host(keep["cm0"]), cm0), "cm_0"
    # sampled groups: digit witnesses, f_0, from_f(f_0)
    groups = blocks_to_groups(W, picks)
    cols = (groups[:, None] * L + np.arange(L)[None, :]).ravel()
    ng = len(groups)
    fks = []
    for s, fc in ((0, fc0), (1, fc1)):
        sub = fc.reshape(N, d)[cols].ravel()
        ofck, ofk, owk = O.decompose_witness(sub, d, pr.B, L, pr.b_small, K)
        ofck, ofk, owk = ofck.reshape(K, -1, d), ofk.reshape(K, -1, d), owk.reshape(K, ng, d)
        if lean is not None:
            lfck, lfk = lean.cols(s, groups)
            assert np.array_equal(lfck, ofck), f"f_coeff_k side {s}"
            assert np.array_equal(lfk, ofk), f"f_k side {s}"
        rows = (("w_ccs_k", keep["wk"][s], owk, groups),) if lean is not None else \
            (("f_coeff_k", fck_dev[s], ofck, cols), ("f_k", fk_dev[s], ofk, cols), ("w_ccs_k", keep["wk"][s], owk, groups))
        for name, got_t, want, idx in rows:
            n_per = N if name != "w_ccs_k" else W
            g = got_t.view(K, n_per, d)[:, torch.from_numpy(idx).to(got_t.device)]
            assert np.array_equal(host(g.contiguous()).reshape(K, len(idx), d), want), f"{name} side {s}"
        fks.append(ofk.reshape(K, len(cols) * d))
    of0 = O.fold_f0(rho, np.concatenate(fks).ravel(), 2 * K, len(cols), d)
    f0 = keep["f0"].view(N, d)
    idx = torch.from_numpy(cols).to(f0.device)
    gf0 = host(f0[idx].contiguous()).ravel()
    assert np.array_equal(gf0, of0), "f_0"
    ofc, ow = O.witness_from_f(gf0, d, pr.B, L)
    assert np.array_equal(host(keep["f0_coeff"].view(N, d)[idx].contiguous()).ravel(), ofc), "f_0 coeff"
    gidx = torch.from_numpy(groups).to(f0.device)
    assert np.array_equal(host(keep["w_ccs0"].view(W, d)[gidx].contiguous()).ravel(), ow), "w_ccs_0"


def run_workload(d, W, kappa, streams=1, batch=0, packed=None, steps=None):
    """bench.Workload after `steps` steps (default: one per stream), run the way
    bench.py runs its timed steps (Workload.run: whole groups, a partial last group
    as one smaller batch)"""
    import torch
    wl = bench.Workload(LA, torch, 0, 0, d, W, kappa, streams, batch=batch, packed=packed)
    try:
        wl.run(streams if steps is None else steps)
        wl.sync()
        return wl
    except Exception:
        wl.close()
        raise


def test_fold_step_bench_shape_d1024():
    """bench.py's default workload shape: d=1024, W=2^14, kappa=32 (streaming-store
    decomposition, nt-copy contraction over the 21.5 GB fragment matrix)"""
    import torch
    wl = run_workload(1024, 1 << 14, 32)
    try:
        assert wl.sch.layout == 1
        nblk = (wl.W + 15) // 16
        check_workload(wl, bench.SEED_W, [0, 1, nblk // 2, nblk - 1], [0, 1, 15, 16, 30, 31],
                       [(0, 1, 0), (1, 14, 31), (1, 7, 16), (0, 14, 5)])
    finally:
        wl.close()
        del wl
        torch.cuda.empty_cache()


@pytest.mark.parametrize("streams", [2, 4])
def test_fold_step_bench_shape_d1024_batched(streams):
    """smaller groups than bench.py's default (8 streams, test below): 2 and 4
    step streams in one batch, the steps' contractions one launch over the
    21.5 GB fragment matrix (A with the default cache policy, the operand rows
    streamed); every step against the oracle"""
    import torch
    wl = run_workload(1024, 1 << 14, 32, streams=streams, batch=streams)
    try:
        assert wl.batch and wl.group == streams
        nblk = (wl.W + 15) // 16
        for st in range(streams):
            check_workload(wl, bench.SEED_W, [st, nblk // 3, nblk - 1 - st], [0, 17, 31],
                           [(0, 1, 3), (1, 14, 30), (st % 2, 9 + st, 16)], stream=st)
    finally:
        wl.close()
        del wl
        torch.cuda.empty_cache()


def test_fold_step_bench_headline_schedule():
    """the headline's exact timed instance: bench.py's defaults (8 step streams,
    --batch 8) at d=1024, W=2^14, kappa=32, run through bench.py's 20-step
    schedule -- two 8-step contraction launches (k_ajtai_mfma_ra<0, 2, 4> with
    nsteps = 8 over the 21.5 GB fragment matrix) and a trailing 4-step batch.
    Every one of the 8 streams against the oracle (streams 0-3 last ran in the
    4-step batch, 4-7 in the second 8-step launch). The packed planes are expanded
    a column block at a time: the workload holds about 240 of the 288 GB.
    Reference: decompose_witness + commit_witnesses
    (latticefold/src/nifs/decomposition.rs:162-201) and the Ajtai mat-vec
    (stark-rings/crates/linear_algebra/src/matrix.rs:168-178), as the oracle
    restates them."""
    import torch
    wl = run_workload(1024, 1 << 14, 32, streams=8, batch=8, steps=20)
    try:
        assert wl.batch and wl.group == 8 and wl.packed
        nblk = (wl.W + 15) // 16
        for st in range(8):
            check_workload(wl, bench.SEED_W, [st, nblk // 2 + st, nblk - 1 - st], [0, 31],
                           [(st % 2, 1 + st, 7), (1 - st % 2, 14 - st, 24)], stream=st, lean_expand=True)
    finally:
        wl.close()
        del wl
        torch.cuda.empty_cache()


def test_fold_step_w464_bench_pairs():
    """the W=464 line (SURVEY 8(d)'s byte-equivalent shape) as bench.py times it:
    4 step streams in groups of 2 (each pair one contraction launch, the pairs
    taking turns), 8 steps; every stream against the oracle"""
    import torch
    wl = run_workload(1024, 464, 32, streams=4, batch=2, steps=8)
    try:
        assert wl.batch and wl.group == 2
        nblk = (wl.W + 15) // 16
        for st in range(4):
            check_workload(wl, bench.SEED_W, [0, st + 5, nblk - 1], [0, 1, 16, 31],
                           [(0, 1, st), (1, 14, 31 - st), (st % 2, 3 + st, 16)], stream=st)
    finally:
        wl.close()
        del wl
        torch.cuda.empty_cache()


def test_fold_step_configs4_bench_pair():
    """configs[4]'s line as bench.py times it: d=4096, W=1024, kappa=64, 2 step
    streams whose contractions are one launch (batch 2), 20 steps; both streams
    against the oracle"""
    import torch
    wl = run_workload(4096, 1024, 64, streams=2, batch=2, steps=20)
    try:
        assert wl.batch and wl.group == 2 and wl.packed
        nblk = (wl.W + 15) // 16
        for st in range(2):
            check_workload(wl, bench.SEED_W, [st, nblk // 2, nblk - 1], [0, 31, 32, 63],
                           [(0, 1, 5 + st), (1, 14, 63 - st), (st, 3, 33)], stream=st)
    finally:
        wl.close()
        del wl
        torch.cuda.empty_cache()


def test_fold_step_reference_ring_zkvm_shape_batched():
    """the reference ring line of bench.py: four step streams, one contraction
    launch for the four steps (the first and the last checked)"""
    import torch
    wl = run_workload(24, 19763, 32, streams=4, batch=4)
    try:
        assert wl.batch and wl.group == 4
        nblk = (wl.W + 15) // 16
        for st in (0, 3):
            check_workload(wl, bench.SEED_W, [st, nblk // 2, nblk - 1], [0, 16, 31],
                           [(0, 1, 0), (1, 14, 31), (st % 2, 7, 16)], stream=st)
    finally:
        wl.close()
        del wl
        torch.cuda.empty_cache()


def test_fold_step_reference_ring_zkvm_shape():
    """the reference ring Phi_72 (d=24) at the real zkvm step shape, bench.py's
    reference_ring workload: W = 19 763 (1 236 units of 16 groups, the last
    with 3 live groups), kappa = 32, the wave-local decomposition with the
    decomposed witnesses kept as packed digit planes (bench.Workload's d = 24 default)"""
    import torch
    wl = run_workload(24, 19763, 32)
    try:
        assert wl.sch.layout == 1
        nblk = (wl.W + 15) // 16
        check_workload(wl, bench.SEED_W, [0, 1, nblk // 2, nblk - 1], [0, 1, 15, 16, 30, 31],
                       [(0, 1, 0), (1, 14, 31), (1, 7, 16), (0, 14, 5)])
    finally:
        wl.close()
        del wl
        torch.cuda.empty_cache()


@pytest.mark.parametrize("packed", [True, False])
def test_fold_step_configs4_d4096_kappa64(packed):
    """BASELINE configs[4]'s ring: d=4096 with kappa=64 (two 32-row MFMA tiles);
    packed (the bench's default): digit bytes instead of u64 f_k / f_coeff_k rows,
    f_0 folded from the quarter-major operand rows"""
    import torch
    wl = run_workload(4096, 1024, 64, packed=packed)
    try:
        assert wl.sch.layout == 1
        nblk = (wl.W + 15) // 16
        check_workload(wl, bench.SEED_W, [0, nblk // 3, nblk - 1], [0, 31, 32, 63],
                       [(0, 1, 0), (1, 14, 63), (1, 3, 33)])
    finally:
        wl.close()
        del wl
        torch.cuda.empty_cache()


def test_ntt_full_batch_configs1():
    """configs[1]: 2^16 polynomials x d=1024 -- forward against the oracle on
    sampled polynomials (including past the kernel's grid-stride cap of 32768
    half-waves), inverse(forward) = identity on the whole batch"""
    import torch
    ctx = LA.Context(0)
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    d, n = 1024, 1 << 16
    x = torch.empty(n * d, dtype=torch.int64, device="cuda")
    ctx.dev_fill_uniform(x, 0x4C460001)
    orig = x.clone()
    ctx.dev_crt(x, d)
    ctx.sync()
    picks = [0, 1, 32767, 32768, 32769, 50000, n - 1]
    xs = host(orig.view(n, d)[picks].contiguous()).ravel()
    assert np.array_equal(host(x.view(n, d)[picks].contiguous()).ravel(), O.crt(xs, d))
    y = x.clone()
    ctx.dev_icrt(y, d)
    ctx.sync()
    assert torch.equal(y, orig)
    # the inverse alone against the oracle
    assert np.array_equal(host(y.view(n, d)[picks].contiguous()).ravel(), xs)
    ctx.dev_icrt(orig, d)
    ctx.sync()
    assert np.array_equal(host(orig.view(n, d)[picks].contiguous()).ravel(), O.icrt(xs, d))
    ctx.close()


def test_witness_kernels_past_grid_stride_cap():
    """d=1024 from_w_ccs / from_f cap their grids at 4096 blocks (32768
    half-waves): W = 40000 runs the grid-stride loop's second iteration"""
    import torch
    ctx = LA.Context(0)
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    d, W = 1024, 40000
    pr = LA.goldilocks_dp(d)
    L = pr.L
    i64 = dict(dtype=torch.int64, device="cuda")
    w = torch.empty(W * d, **i64)
    ctx.dev_fill_uniform(w, 77)
    fc, f = torch.empty(W * L * d, **i64), torch.empty(W * L * d, **i64)
    ctx.check(ctx.lib.lf_dev_witness_from_w_ccs(ctx.h, LA._lib.C.byref(pr), w.data_ptr(), W, fc.data_ptr(),
                                                f.data_ptr()))
    f_in = torch.empty(W * L * d, **i64)
    ctx.dev_fill_uniform(f_in, 78)
    fc2, w2 = torch.empty(W * L * d, **i64), torch.empty(W * d, **i64)
    ctx.check(ctx.lib.lf_dev_witness_from_f(ctx.h, LA._lib.C.byref(pr), f_in.data_ptr(), W * L, fc2.data_ptr(),
                                            w2.data_ptr()))
    ctx.sync()
    for j in (0, 32767, 32768, 32769, 36000, W - 1):
        wj = host(w[j * d:(j + 1) * d])
        ofc, of = O.witness_from_w_ccs(wj, d, pr.B, L)
        assert np.array_equal(host(fc[j * L * d:(j + 1) * L * d]), ofc), j
        assert np.array_equal(host(f[j * L * d:(j + 1) * L * d]), of), j
        ofc2, ow2 = O.witness_from_f(host(f_in[j * L * d:(j + 1) * L * d]), d, pr.B, L)
        assert np.array_equal(host(fc2[j * L * d:(j + 1) * L * d]), ofc2), j
        assert np.array_equal(host(w2[j * d:(j + 1) * d]), ow2), j
    ctx.close()
