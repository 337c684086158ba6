"""Check a bench line's per-phase launch times against the rocprofv3 kernel trace
of the same run (every roofline.avg_launch_ms and phase average
within 5 % of a committed summary).

usage: python tools/check_profile.py <bench log or json> <stats.windows.json>

bench.py wraps each workload's serialized phase pass in a roctx range
(roofline.profile_window); tools/prof_summary.py stats keeps the kernels inside
each range. Per phase, the trace figure is (the phase kernel's launches plus the
helper kernels the phase launches with it: the digit packing of the fused
decompositions, the key packing of the coefficient fold) / the phase kernel's
launches, against the line's avg_launch_ms (the launch time for a batched
contraction, which the context records once per step it covers). A phase agrees
when the two are within 5 % or within EVENT_US (the HIP event records around a
phase of a few tens of microseconds).
"""
import json
import os
import sys

# every kernel a phase's HIP-event pair brackets (lf_api.hip fold_commit / fold_finish),
# by base name; the primary kernel (launched once per phase record) comes first
PHASE_KERNELS = {
    "decompose": ("k_decompose_fused", "k_decompose_phi72_w", "k_decompose_n4k_mx", "k_decompose_n4k_fused", "k_decompose_n4k",
                  "k_pack_sm", "k_pack_sm24", "k_pack_sm8", "k_pack_sm4", "k_expand_sm"),
    "fold": ("k_fold_coeff", "k_fold_coeff_phi72", "k_fold_nega", "k_fold_frag", "k_fold_coeff_sum", "k_pack_keys",
             "k_rho_prep", "k_rho_phi72", "k_fold_phi72_masks"),
    "from_f": ("k_from_fcoeff_n32", "k_from_fcoeff_split", "k_from_f_phi72", "k_from_f_n4k", "k_from_f_n32",
               "k_from_f_split"),
    "from_w_ccs": ("k_from_w_ccs_n32", "k_from_w_ccs_digits", "k_from_w_ccs_phi72", "k_from_w_ccs_n4k", "k_xform_n32"),
    "to_frag": ("k_to_frag",),
    "ajtai": ("k_ajtai_mfma_ra",),
}
EVENT_US = 8.0  # a phase's two HIP event records on the stream add a few us around short phases


def line_of(path):
    """the bench record of a log or json: the printed line names the detail file
    holding the full record (per-phase times of every workload); follow it"""
    txt = open(path).read()
    for ln in reversed(txt.splitlines()):
        ln = ln.strip()
        if ln.startswith("{") and '"metric"' in ln:
            rec = json.loads(ln)
            det = rec.get("detail")
            if det and os.path.exists(det):
                return json.load(open(det))
            return rec
    raise SystemExit(f"no bench line in {path}")


def base(k):
    return k.split(" grid=")[0].split("<")[0].replace("lfk::", "")


def check(workload, wins, tol=0.05):
    roof = workload.get("roofline") or {}
    win = wins.get(roof.get("profile_window"))
    rows, ok = [], True
    if win is None:
        return [f"  no window {roof.get('profile_window')!r} in the trace"], False
    ks = win["kernels"]
    for ph, p in workload["phases"].items():
        kb = base(p["kernel"])
        prim = [k for k in ks if base(k) == kb]
        if not prim:
            rows.append(f"  {ph:10s} {p['kernel']}: not in the window")
            ok = False
            continue
        main = max(prim, key=lambda k: ks[k]["avg_us"] * ks[k]["launches"])
        n = ks[main]["launches"]
        if ph == "ajtai":  # the contraction kernel alone (its split-K sum is outside the phase)
            members = [main]
        else:
            members = [k for k in ks if base(k) in PHASE_KERNELS.get(ph, (kb,))]
        tot = sum(ks[k]["avg_us"] * ks[k]["launches"] for k in members)
        trace_ms = tot / n / 1e3
        line_ms = p.get("launch_ms", p["avg_launch_ms"])
        r = line_ms / trace_ms if trace_ms else float("inf")
        good = abs(r - 1) <= tol or abs(line_ms - trace_ms) * 1e3 <= EVENT_US
        ok &= good
        names = "+".join(base(k) for k in members)
        rows.append(f"  {ph:10s} line {line_ms:9.4f} ms  trace {trace_ms:9.4f} ms  ratio {r:.3f}  "
                    f"diff {(line_ms - trace_ms) * 1e3:+6.1f} us{'' if good else '  <-- off'}  [{names}]")
    return rows, ok


def main():
    b = line_of(sys.argv[1])
    wins = json.load(open(sys.argv[2]))
    allok = True
    for key in (None, "reference_ring", "small_shape", "configs4_d4096_kappa64"):
        w = b if key is None else b.get(key)
        if not w or "phases" not in w:
            continue
        rows, ok = check(w, wins)
        allok &= ok
        print(f"{key or 'headline'}: window {w['roofline'].get('profile_window')!r}, {'OK' if ok else 'MISMATCH'}")
        print("\n".join(rows))
    sys.exit(0 if allok else 1)


if __name__ == "__main__":
    main()
