"""Benchmark: LatticeFold commit + fold steps per second on MI355X.

A step = zkvm commit(z) (Witness::from_w_ccs + Ajtai A.f) followed by the
commit+fold arithmetic of fold(): decompose accumulator and new witness into
K=15 witnesses each, 28 batched Ajtai commitments, y_0 fix-ups, f_0 / cm_0 linear
fold with 30 short challenges, Witness::from_f(f_0). Inputs are synthetic
(seeded SplitMix64, SURVEY.md §8d seeds) and resident in HBM before timing.

Default workload (BASELINE.json configs[2], "Ajtai commit + single LatticeFold
step on 2^14 synthetic CCS witnesses", at the metric's d=1024): ring
Fq[X]/(X^1024+1), w_ccs = 2^14 ring elements, kappa = 32, B=2^15, L=5, K=15.

Multi-GPU (torchrun, one rank per GPU): independent steps per rank (weak
scaling); at the end of the timed batch the ranks' folded accumulators
(cm_0, f_0) are reduced mod p over RCCL (latticeum_amd.dist).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

SEED_W = 0x4C460003
SEED_A = 0x4C460004
SEED_RHO = 0x4C460005
SEED_ACC = 0x4C460006
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--d", type=int, default=1024)
    ap.add_argument("--w", type=int, default=1 << 14, help="w_ccs length W (ring elements)")
    ap.add_argument("--kappa", type=int, default=32)
    ap.add_argument("--streams", type=int, default=1, help="concurrent step streams per GPU")
    ap.add_argument("--no-small-shape", dest="small", action="store_false", default=True,
                    help="skip the W=464 / d=24 multi-stream measurements and the NTT / Poseidon2 timings "
                         "reported beside the default workload")
    ap.add_argument("--cpu-baseline", dest="cpu", action="store_true", default=True)
    ap.add_argument("--no-cpu-baseline", dest="cpu", action="store_false")
    ap.add_argument("--cpu-w", type=int, default=0, help="W of the CPU baseline sample (0 = auto)")
    ap.add_argument("--cpu-threads", type=int, default=0)
    return ap.parse_args()


def algorithmic_bytes(d, W, kappa, L=5, K=15):
    """SURVEY.md §8d bytes/step and the algorithmic bytes of one launch of each
    step phase (inputs read once + outputs written once)."""
    E, N = 8 * d, W * L
    step = (E * (W + 3 * N + kappa * N + kappa) + 2 * E * (N + K * (2 * N + W))
            + E * (kappa * N + 2 * (K - 1) * N + 2 * (K - 1) * kappa) + E * (2 * K * N + N)
            + E * (2 * N + W))
    nvec = 2 * (K - 1) + 1  # commit(z)'s A.f rides in the decomposition-commitment pass
    # i8-MFMA operand bytes per element: 8 signed bytes per slot; d = 24 (Phi_72)
    # contracts 40 virtual slots (Toom-3 evaluations of its 8 Fq3 slots)
    F = 8 * (40 if d == 24 else d)
    sides = 1 if d == 24 else 2  # the d = 1024 decomposition runs both sides in one launch
    phases = {
        # f_coeff in; f_k_coeff, f_k (K N each), w_ccs_k (K W), K-1 planes as i8-MFMA operand rows out
        "decompose": sides * (E * (N + 2 * K * N + K * W) + F * (K - 1) * N),
        # A and the 29 vectors in operand form, and the 29 kappa-element results
        "ajtai": F * (kappa * N + nvec * N) + E * nvec * kappa,
        "fold": E * (2 * K * N + N),
        "from_w_ccs": E * (W + 2 * N),
        "from_f": E * (2 * N + W),
        "to_frag": E * N + F * N,
    }
    return step, phases


def load_traffic(d, W, kappa):
    """PMC-measured HBM bytes per launch (profiles/pmc_traffic.json, written by
    tools/prof_summary.py traffic from separate FETCH_SIZE / WRITE_SIZE passes of
    this same configuration); {} when absent or for another configuration."""
    f = ROOT / "profiles" / "pmc_traffic.json"
    try:
        doc = json.loads(f.read_text())
    except (OSError, ValueError):
        return {}
    if doc.get("config") != {"d": d, "W": W, "kappa": kappa}:
        return {}
    t = {k: v["hbm_bytes_per_launch"] for k, v in doc.get("kernels", {}).items()}
    # a kernel launched as one template instance (k_decompose_fused<true>,
    # k_ajtai_mfma<2>) is looked up by its plain name too
    for k in list(t):
        base = k.split("<")[0]
        if base != k and base not in t and sum(x.split("<")[0] == base for x in t) == 1:
            t[base] = t[k]
    if "k_decompose_fused" in t and "k_pack_sm" in t:  # the decompose phase launches both
        t["k_decompose_fused"] += t["k_pack_sm"]
    return t


def cpu_baseline(d, W_full, kappa, cpu_w, threads):
    """Time the oracle's restatement of the same step on host cores (bounded sample)."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle as O

    B, L, bs, K = 1 << 15, 5, 2, 15
    W = cpu_w
    N = W * L
    A = O.fill_uniform(kappa * N * d, SEED_A)
    w_ccs = O.fill_uniform(W * d, SEED_W)
    acc_fc, acc_f = O.witness_from_w_ccs(O.fill_uniform(W * d, SEED_ACC), d, B, L, threads)
    acc_cm = O.ajtai_commit(A, kappa, N, d, acc_f, 1, threads)
    rho = O.crt(O.fill_uniform(2 * K * d, SEED_RHO), d)
    t0 = time.perf_counter()
    fc, f = O.witness_from_w_ccs(w_ccs, d, B, L, threads)
    cm = O.ajtai_commit(A, kappa, N, d, f, 1, threads)
    sides = [O.decompose_witness(x, d, B, L, bs, K, threads) for x in (acc_fc, fc)]
    vecs = np.concatenate([s[1].reshape(K, N * d)[1:] for s in sides]).ravel()
    ycat = O.ajtai_commit(A, kappa, N, d, vecs, 2 * (K - 1), threads).reshape(2, K - 1, kappa * d)
    ys = []
    for s, c in enumerate((acc_cm, cm)):
        y = np.zeros((K, kappa * d), np.uint64)
        y[1:] = ycat[s]
        ys.append(O.commit_witnesses_y0(c, y.ravel(), kappa, d, bs, K))
    f0 = O.fold_f0(rho, np.concatenate([s[1] for s in sides]), 2 * K, N, d, threads)
    O.fold_cm0(rho, np.concatenate(ys), 2 * K, kappa, d)
    O.witness_from_f(f0, d, B, L, threads)
    dt = time.perf_counter() - t0
    steps_per_s = 1.0 / (dt * W_full / W)  # every stage is linear in W
    return {"value": steps_per_s, "unit": "fold-steps/s", "cores": threads, "kind": "port",
            "sample": f"1 full step at W={W} (1/{W_full // W} of W={W_full}), d={d}, kappa={kappa}, "
                      f"{dt:.2f} s on {threads} threads; scaled linearly in W"}


class Workload:
    """One fold-step workload resident in HBM: the Ajtai scheme, the accumulator
    side and rho (shared, read-only), and `streams` independent step streams,
    each an lf context on its own HIP stream with its own w_ccs and outputs."""

    def __init__(self, LA, torch, local, rank, d, W, kappa, streams):
        self.LA, self.torch = LA, torch
        self.d, self.W, self.kappa = d, W, kappa
        self.pr = pr = LA.goldilocks_dp(d)
        K, L = pr.K, pr.L
        self.N = N = W * L
        i64 = dict(dtype=torch.int64, device=f"cuda:{local}")
        z = lambda n: torch.empty(n, **i64)
        ctx = LA.Context(local)
        ctx.set_stream(torch.cuda.current_stream().cuda_stream)
        A = z(kappa * N * d)
        ctx.dev_fill_uniform(A, SEED_A)
        self.sch = sch = LA.AjtaiCommitmentScheme(ctx, device_tensor=A, kappa=kappa, ncols=N, d=d)
        if sch.layout == 1:  # the scheme keeps A in MFMA fragment order; drop the AoS copy
            del A
            torch.cuda.empty_cache()
        # accumulator side: a previous witness built the reference way (from_w_ccs + commit)
        acc_w = z(W * d)
        ctx.dev_fill_uniform(acc_w, SEED_ACC)
        acc_fc, acc_f, acc_cm = z(N * d), z(N * d), z(kappa * d)
        ctx.check(ctx.lib.lf_dev_witness_from_w_ccs(ctx.h, LA._lib.C.byref(pr), acc_w.data_ptr(), W,
                                                    acc_fc.data_ptr(), acc_f.data_ptr()))
        ctx.dev_ajtai_commit(sch, [acc_f], acc_cm)
        del acc_w, acc_f
        # rho: 29 short challenges from seeded bytes (CR/rings/goldilocks.rs:41-67) + ONE, NTT form
        rng = np.random.default_rng(SEED_RHO)
        rc = [LA.short_challenge(rng.integers(0, 256, 3 * d // 4, dtype=np.uint8).tobytes(), d)
              for _ in range(2 * K - 1)]
        one = np.zeros(d, np.uint64)
        one[0] = 1
        rho = torch.from_numpy(np.concatenate(rc + [one]).view(np.int64)).to(f"cuda:{local}")
        ctx.dev_crt(rho, d)
        self.ctxs, self.keeps, self.bufs, self.streams = [], [], [], []
        for i in range(streams):
            c = ctx if i == 0 else LA.Context(local)
            if i > 0:
                st = torch.cuda.Stream()
                c.set_stream(st.cuda_stream)
                self.streams.append(st)
            w_ccs = z(W * d)
            c.dev_fill_uniform(w_ccs, SEED_W + 7919 * rank + 104729 * i)
            keep = {
                "w_ccs": w_ccs, "acc_cm": acc_cm, "acc_f_coeff": acc_fc, "rho": rho,
                "f_coeff": z(N * d), "f": z(N * d), "cm": z(kappa * d),
                "fk_coeff": [z(K * N * d) for _ in range(2)], "fk": [z(K * N * d) for _ in range(2)],
                "wk": [z(K * W * d) for _ in range(2)], "y": [z(K * kappa * d) for _ in range(2)],
                "f0": z(N * d), "f0_coeff": z(N * d), "w_ccs0": z(W * d), "cm0": z(kappa * d),
            }
            bufs = LA.LfFoldStepBufs()
            for k, v in keep.items():
                if isinstance(v, list):
                    for s in range(2):
                        getattr(bufs, k)[s] = v[s].data_ptr()
                else:
                    setattr(bufs, k, v.data_ptr())
            c.reserve(kappa, N, d, 2 * (K - 1) + 1)
            self.ctxs.append(c)
            self.keeps.append(keep)
            self.bufs.append(bufs)
        torch.cuda.synchronize()

    def run(self, steps):
        """`steps` fold steps, round-robin over the step streams (asynchronous)"""
        S = len(self.ctxs)
        for i in range(steps):
            self.ctxs[i % S].dev_fold_step(self.sch, self.pr, self.W, self.bufs[i % S])

    def sync(self):
        for c in self.ctxs:
            c.sync()  # surfaces any decomposition overflow

    def close(self):
        self.sync()
        self.sch = None
        self.keeps, self.bufs = [], []
        for c in self.ctxs:
            c.close()
        self.ctxs = []


def extra_shape(LA, torch, LD, pg, local, rank, world, d, W, kappa, S, steps, warmup, what):
    """Another commit+fold workload with S concurrent step streams per GPU,
    reported beside the default one (not as `value`): SURVEY.md §8d's
    byte-equivalent shape (d = 1024, W = 464), whose per-GPU rate the north-star
    target (1e4 steps/s on 8 GPUs) is about, and the reference's own ring at the
    real zkvm shape (d = 24, W = 19 763; the bit-exact-vs-reference path)."""
    wl = Workload(LA, torch, local, rank, d, W, kappa, S)
    wl.run(warmup)
    torch.cuda.synchronize()
    LD.barrier(pg)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    wl.run(steps)
    torch.cuda.synchronize()
    LD.barrier(pg)
    dt = LD.max_over_ranks(pg, time.perf_counter() - t0)
    wl.close()
    torch.cuda.empty_cache()
    value = world * steps / dt
    step_bytes, _ = algorithmic_bytes(d, W, kappa)
    return {"workload": f"commit+fold step, {what}, w_ccs W={W}, kappa={kappa}, {S} concurrent step streams per GPU",
            "d": d, "W": W, "streams": S, "value": value, "unit": "fold-steps/s", "n_gpus": world, "steps": steps,
            "ms_per_step_per_gpu": dt / steps * 1e3, "hbm_gbs_step_algorithmic": step_bytes * value / world / 1e9}


def side_ops(LA, torch, local):
    """BASELINE.json configs[1] (batched d = 1024 NTT/INTT of 2^16 polynomials)
    and the Poseidon2 batch of configs[4] (2^20 states), device time per launch."""
    ctx = LA.Context(local)
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)

    def ev_ms(fn, reps=10):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps

    out = {}
    d, n = 1024, 1 << 16
    x = torch.empty(n * d, dtype=torch.int64, device=f"cuda:{local}")
    ctx.dev_fill_uniform(x, SEED_W - 2)
    by = 2 * n * d * 8
    for name, fn in (("fwd", lambda: ctx.dev_crt(x, d)), ("inv", lambda: ctx.dev_icrt(x, d))):
        ms = ev_ms(fn)
        out[f"ntt_{name}"] = {"npoly": n, "d": d, "ms": ms, "polys_per_s": n / ms * 1e3,
                              "achieved_gbs": by / ms / 1e6, "frac_hbm": by / ms / 1e6 / HBM_PEAK_GBS}
    del x
    m = 1 << 20
    st = torch.empty(16 * m, dtype=torch.int64, device=f"cuda:{local}")
    ctx.dev_fill_uniform(st, 0x4C460007)
    ms = ev_ms(lambda: ctx.dev_poseidon2_permute(st))
    out["poseidon2_w16"] = {"states": m, "ms": ms, "perms_per_s": m / ms * 1e3}
    del st
    ctx.sync()
    ctx.close()
    torch.cuda.empty_cache()
    return out


def main():
    args = parse()
    import torch
    import latticeum_amd as LA
    from latticeum_amd import dist as LD

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    torch.cuda.set_device(local)
    pg = LD.init(world)

    d, W, kappa = args.d, args.w, args.kappa
    wl = Workload(LA, torch, local, rank, d, W, kappa, args.streams)
    pr, sch = wl.pr, wl.sch
    K, L, N = pr.K, pr.L, wl.N
    ctx, keep, bufs = wl.ctxs[0], wl.keeps[0], wl.bufs[0]

    wl.run(args.warmup)
    wl.sync()
    reducer = LD.AccumulatorReducer(ctx, world, [keep["cm0"], keep["f0"]]) if world > 1 else None

    ctx.kernel_timing(True)  # HIP events on the stream around every phase (lf_ctx_phase_stats)
    LD.barrier(pg)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    wl.run(args.steps)
    if reducer is not None:
        reducer.reduce()  # RCCL reduce of the folded accumulators (once per timed batch)
    torch.cuda.synchronize()
    LD.barrier(pg)
    dt = time.perf_counter() - t0
    ctx.sync()  # surfaces any decomposition overflow
    dt_max = LD.max_over_ranks(pg, dt)
    nvec = 2 * (K - 1) + 1
    ms_b, n_b = ctx.kernel_stats(nvec)
    timed = {"ajtai": (ms_b, n_b)}
    for ph in ("from_w_ccs", "decompose", "to_frag", "fold", "from_f"):
        timed[ph] = ctx.phase_stats(ph)
    ctx.kernel_timing(False)

    step_bytes, ph_bytes = algorithmic_bytes(d, W, kappa, L, K)
    if d == 24:
        kernel_of = {"decompose": "k_decompose_phi72", "ajtai": "k_ajtai_mfma" if sch.layout == 1 else "k_ajtai_phi72",
                     "fold": "k_fold_phi72", "from_w_ccs": "k_from_w_ccs_phi72", "from_f": "k_from_f_phi72",
                     "to_frag": "k_to_frag<true, true, true>"}
    else:
        small = W < 4096  # kernels_n32.hip SPLIT_W: one half-wave per (element, limb)
        kernel_of = {"decompose": "k_decompose_fused",
                     "ajtai": "k_ajtai_mfma" if sch.layout == 1 else "k_ajtai_nega", "fold": "k_fold_nega",
                     "from_w_ccs": "k_from_w_ccs_split" if small else "k_from_w_ccs_n32",
                     "from_f": "k_from_f_split" if small else "k_from_f_n32", "to_frag": "k_to_frag<true, false, true>"}
    traffic = load_traffic(d, W, kappa)
    phases = {}
    for ph, (ms, cnt) in timed.items():
        if not cnt:
            continue
        avg = ms / cnt
        gbs = ph_bytes[ph] / (avg * 1e-3) / 1e9
        phases[ph] = {"kernel": kernel_of[ph], "avg_launch_ms": avg, "launches_per_step": cnt / args.steps,
                      "ms_per_step": ms / args.steps, "algorithmic_bytes_per_launch": ph_bytes[ph],
                      "achieved_gbs": gbs, "frac_hbm": gbs / HBM_PEAK_GBS,
                      "traffic_bytes_per_launch": traffic.get(kernel_of[ph])}
    dom = max(phases, key=lambda k: phases[k]["ms_per_step"]) if phases else None
    out = None
    if rank == 0:
        cpu = None
        if args.cpu and world == 1:
            threads = args.cpu_threads or min(16, os.cpu_count() or 1)
            cpu_w = args.cpu_w or max(1, min(W, 64 if d >= 1024 else 2048))
            cpu = cpu_baseline(d, W, kappa, cpu_w, threads)
        value = world * args.steps / dt_max
        out = {
            "metric": "fold-steps/sec (Ajtai commit+fold) at d=1024",
            "value": value, "unit": "fold-steps/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": dt_max / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u64 (Goldilocks mod-p integer)",
            "data": "synthetic (seeded SplitMix64 inputs, random Ajtai matrix)",
            "config": {"workload": f"commit+fold step, X^{d}+1 ring, w_ccs W={W}, N={N}, kappa={kappa}, "
                                   f"B=2^15 L=5 K=15, 29 Ajtai products in one pass over A",
                       "d": d, "W": W, "N": N, "kappa": kappa,
                       "parallelism": f"{world} independent step streams (weak)"},
            "hbm_gbs_step_algorithmic": step_bytes * value / world / 1e9,
            # the dominant phase by device time per step; every phase below (HIP events
            # on the launch stream, inside the timed region)
            "roofline": None if dom is None else {
                "kernel": phases[dom]["kernel"], "phase": dom, "bound": "hbm",
                "achieved": phases[dom]["achieved_gbs"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": phases[dom]["frac_hbm"], "traffic": phases[dom]["traffic_bytes_per_launch"],
                "avg_launch_ms": phases[dom]["avg_launch_ms"],
                "bytes_per_launch": phases[dom]["algorithmic_bytes_per_launch"]},
            "phases": phases,
            "cpu_baseline": cpu,
        }
    del ctx, keep, bufs, reducer, sch
    wl.close()
    del wl
    torch.cuda.empty_cache()
    if args.small and args.d == 1024:
        small = extra_shape(LA, torch, LD, pg, local, rank, world, 1024, 464, args.kappa, 4, 256, 16,
                            "X^1024+1 ring (byte-equivalent to the real zkvm step)")
        ref = extra_shape(LA, torch, LD, pg, local, rank, world, 24, 19763, 32, 4, 128, 8,
                          "the reference ring Phi_72 = X^24 - X^12 + 1 at the real zkvm shape")
        ops = side_ops(LA, torch, local)
        if out is not None:
            out["small_shape"] = small
            out["reference_ring"] = ref
            out["side_ops"] = ops
    if out is not None:
        print(json.dumps(out), flush=True)
    LD.finalize(pg)
    return out


if __name__ == "__main__":
    main()
