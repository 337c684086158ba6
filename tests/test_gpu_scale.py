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


def check_workload(wl, seed_w, picks, cm_rows, y_rows, stream=0):
    """bench.Workload `wl` has run one step on step stream `stream`; compare it
    against the oracle."""
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
    if keep.get("planes", [None])[0] is not None and fk_dev[0] is None:
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
    for s, k, row in y_rows:
        fk = host(fk_dev[s][k * N * d:(k + 1) * N * d])
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
        for name, got_t, want, idx in (("f_coeff_k", fck_dev[s], ofck, cols), ("f_k", fk_dev[s], ofk, cols),
                                       ("w_ccs_k", keep["wk"][s], owk, groups)):
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


def run_workload(d, W, kappa, streams=1, batch=0, packed=None):
    import torch
    wl = bench.Workload(LA, torch, 0, 0, d, W, kappa, streams, batch=batch, packed=packed)
    try:
        wl.run(streams)
        wl.sync()
        return wl
    except Exception:
        wl.close()
        raise


def test_fold_step_bench_shape_d1024():
    """bench.py's default workload: d=1024, W=2^14, kappa=32 (streaming-store
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
    """bench.py's default (4 step streams, one batch) and the pairs form: the
    steps' contractions are one launch over the 21.5 GB fragment matrix (A with
    the default cache policy, the operand rows streamed: the instance only this
    size runs); every step against the oracle"""
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
