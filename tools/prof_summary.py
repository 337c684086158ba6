"""Summarise rocprofv3 outputs into profiles/ (committed evidence).

usage:
  python tools/prof_summary.py stats  <prof_dir> <out.md>
  python tools/prof_summary.py traffic <fetch_dir> <write_dir> <out.json> [d W kappa]

`traffic` follows MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE come from
separate --pmc passes (TCC slot limits); both are in KiB; on gfx950 FETCH_SIZE
reports 1/2 of the bytes of a wide coalesced streaming read, so it is doubled.
"""
import csv
import glob
import json
import os
import subprocess
import sys
from collections import defaultdict

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from bench import kernel_source_hash  # noqa: E402  (the hash bench.py checks before using a PMC file)


def find(dirname, suffix):
    hits = sorted(glob.glob(os.path.join(dirname, "**", f"*{suffix}"), recursive=True))
    if not hits:
        raise SystemExit(f"no *{suffix} under {dirname}")
    return hits[0]


def grid(r):
    if "Grid_Size_X" in r:
        return f"{r['Grid_Size_X']}x{r.get('Grid_Size_Y', 1)}x{r.get('Grid_Size_Z', 1)}"
    return str(r.get("Grid_Size", "?"))


def short(name):
    n = name.replace("(anonymous namespace)::", "").split("(")[0]
    return n.replace("void ", "").strip()


def marker_windows(prof_dir, prefix="phase_pass"):
    """roctx ranges bench.py pushes around each workload's serialized phase pass
    (rocprofv3 --marker-trace): {name: [(start_ns, end_ns), ...]}"""
    hits = sorted(glob.glob(os.path.join(prof_dir, "**", "*marker_api_trace.csv"), recursive=True))
    wins = defaultdict(list)
    for f in hits:
        for r in csv.DictReader(open(f)):
            name = next((v for v in r.values() if isinstance(v, str) and v.startswith(prefix)), None)
            if name is not None:
                wins[name].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    return wins


def window_table(trace, lo, hi):
    """per kernel (and grid for the contraction): launches, avg us inside [lo, hi],
    and the window's largest number of kernels in flight at once (1 = serialized)"""
    inside = [t for t in trace if int(t["Start_Timestamp"]) >= lo and int(t["End_Timestamp"]) <= hi]
    by = defaultdict(list)
    ev = []
    for t in inside:
        s, e = int(t["Start_Timestamp"]), int(t["End_Timestamp"])
        key = short(t["Kernel_Name"]) + (f" grid={grid(t)}" if "ajtai" in t["Kernel_Name"] else "")
        by[key].append((e - s) / 1e3)
        ev += [(s, 1), (e, -1)]
    conc = cur = 0
    for _, dlt in sorted(ev, key=lambda x: (x[0], x[1])):
        cur += dlt
        conc = max(conc, cur)
    return by, conc


def stats(prof_dir, out_md):
    rows = list(csv.DictReader(open(find(prof_dir, "kernel_stats.csv"))))
    trace = list(csv.DictReader(open(find(prof_dir, "kernel_trace.csv"))))
    lines = []
    side = {}
    for name, spans in sorted(marker_windows(prof_dir).items()):
        lo, hi = min(s for s, _ in spans), max(e for _, e in spans)
        by, conc = window_table(trace, lo, hi)
        lines += [f"## window `{name}` (roctx range, {(hi - lo) / 1e6:.2f} ms; at most {conc} kernel(s) in flight)",
                  "", "| kernel | launches | avg us | total ms |", "|---|---|---|---|"]
        tot = sum(sum(v) for v in by.values())
        for k, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
            lines.append(f"| `{k}` | {len(v)} | {sum(v) / len(v):.1f} | {sum(v) / 1e3:.2f} |")
        lines += [f"| (all) | {sum(len(v) for v in by.values())} | | {tot / 1e3:.2f} |", ""]
        side[name] = {"window_ms": (hi - lo) / 1e6, "max_in_flight": conc,
                      "kernels": {k: {"launches": len(v), "avg_us": sum(v) / len(v)} for k, v in by.items()}}
    if side:
        json.dump(side, open(os.path.splitext(out_md)[0] + ".windows.json", "w"), indent=1)
        lines += ["## whole process (every stream; concurrent launches stretch each other's durations)", ""]
    lines += ["| kernel | calls | avg us | total ms | % |", "|---|---|---|---|---|"]
    for r in rows:
        lines.append(f"| `{short(r['Name'])}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | "
                     f"{float(r['TotalDurationNs']) / 1e6:.2f} | {float(r['Percentage']):.2f} |")
    # per-grid breakdown of the Ajtai kernel (batched vs single launches differ in grid)
    by = defaultdict(list)
    for t in trace:
        if "ajtai" in t["Kernel_Name"]:
            key = (short(t["Kernel_Name"]), grid(t))
            by[key].append((int(t["End_Timestamp"]) - int(t["Start_Timestamp"])) / 1e3)
    if by:
        lines += ["", "| Ajtai launch kind (kernel, grid) | launches | avg us |", "|---|---|---|"]
        for (k, g), v in sorted(by.items()):
            lines.append(f"| `{k}` grid={g} | {len(v)} | {sum(v) / len(v):.1f} |")
    open(out_md, "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


def counter_per_dispatch(d, counter):
    f = find(d, "counter_collection.csv")
    out = defaultdict(float)
    meta = {}
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] != counter:
            continue
        did = r["Dispatch_Id"]
        out[did] += float(r["Counter_Value"])
        meta[did] = (short(r["Kernel_Name"]).replace("lfk::", ""), grid(r))
    return out, meta


def traffic(fetch_dir, write_dir, out_json, config):
    """Per kernel (the grid that moves the most bytes, e.g. the f-fold rather
    than the cm-fold): HBM bytes per launch = (2 FETCH_SIZE + WRITE_SIZE) KiB."""
    fetch, mf = counter_per_dispatch(fetch_dir, "FETCH_SIZE")
    write, mw = counter_per_dispatch(write_dir, "WRITE_SIZE")
    acc = defaultdict(lambda: {"fetch_kib": [], "write_kib": []})
    for did, v in fetch.items():
        acc[mf[did]]["fetch_kib"].append(v)
    for did, v in write.items():
        acc[mw[did]]["write_kib"].append(v)
    kernels = {}
    for (name, g), r in acc.items():
        if not r["fetch_kib"] or not r["write_kib"]:
            continue
        fk = sum(r["fetch_kib"]) / len(r["fetch_kib"])
        wk = sum(r["write_kib"]) / len(r["write_kib"])
        e = {"grid": g, "launches": len(r["fetch_kib"]), "fetch_kib_raw": fk, "write_kib": wk,
             "hbm_bytes_per_launch": (2 * fk + wk) * 1024}
        if name not in kernels or e["hbm_bytes_per_launch"] > kernels[name]["hbm_bytes_per_launch"]:
            kernels[name] = e
    try:
        rev = subprocess.run(["git", "rev-parse", "--short", "HEAD"], capture_output=True, text=True).stdout.strip()
    except Exception:
        rev = "?"
    doc = {"config": config, "kernels": kernels, "git": rev, "src_hash": kernel_source_hash(),
           "method": "separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of bench.py; bytes = "
                     "(2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE counts 1/2 of wide streaming "
                     "reads, MI355X_MICROARCH.md §HBM)"}
    json.dump(doc, open(out_json, "w"), indent=1)
    print(json.dumps(doc, indent=1))


def sq(sq_dir, out_json, config, simds=1024, xcds=8):
    """Per kernel: the VALU pipes' busy fraction from one SQ pass,
    SQ_ACTIVE_INST_VALU (quad-cycles) x 4 / (SIMDs x GRBM_GUI_ACTIVE / XCDs)
    (GRBM_GUI_ACTIVE is summed over the XCDs), averaged over launches; with
    SQ_VALU_MFMA_BUSY_CYCLES in the pass also the matrix pipes' busy fraction
    (that counter counts cycles, summed over the SIMDs) and the clock."""
    per = {}
    for c in ("SQ_ACTIVE_INST_VALU", "SQ_INSTS_VALU", "GRBM_GUI_ACTIVE", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY",
              "SQ_WAIT_INST_ANY", "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_WAIT_INST_LDS"):
        try:
            vals, meta = counter_per_dispatch(sq_dir, c)
        except SystemExit:
            continue
        for did, v in vals.items():
            per.setdefault(did, {"name": meta[did][0]})[c] = v
    acc = defaultdict(list)
    for did, r in per.items():
        if r.get("GRBM_GUI_ACTIVE") and "SQ_ACTIVE_INST_VALU" in r:
            cyc = r["GRBM_GUI_ACTIVE"] / xcds
            acc[r["name"]].append({"valu_busy": 4 * r["SQ_ACTIVE_INST_VALU"] / (simds * cyc),
                                   "valu_insts_per_cu_cycle": r["SQ_INSTS_VALU"] / (simds / 4 * cyc),
                                   "cycles": cyc,
                                   "wait_issue_frac": r["SQ_WAIT_INST_ANY"] / max(r["SQ_WAVE_CYCLES"], 1),
                                   "wait_cnt_frac": r["SQ_WAIT_ANY"] / max(r["SQ_WAVE_CYCLES"], 1),
                                   **({"mfma_busy": r["SQ_VALU_MFMA_BUSY_CYCLES"] / (simds * cyc)}
                                      if "SQ_VALU_MFMA_BUSY_CYCLES" in r else {}),
                                   **({"wait_lds_frac": r["SQ_WAIT_INST_LDS"] / max(r["SQ_WAVE_CYCLES"], 1)}
                                      if "SQ_WAIT_INST_LDS" in r else {})})
    kernels = {k: {f: sum(x[f] for x in v) / len(v) for f in v[0]} | {"launches": len(v)} for k, v in acc.items()}
    counters = sorted({c for r in per.values() for c in r if c != "name"})
    doc = {"config": config, "kernels": kernels, "src_hash": kernel_source_hash(),
           "method": f"one rocprofv3 --pmc pass ({' '.join(counters)}); "
                     "valu_busy = 4 SQ_ACTIVE_INST_VALU / (1024 SIMDs x GRBM_GUI_ACTIVE / 8); "
                     "mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)"}
    json.dump(doc, open(out_json, "w"), indent=1)
    print(json.dumps(doc, indent=1))


def _config(argv, pos):
    """--config '<json>' anywhere in argv, else d W kappa at argv[pos:pos + 3]"""
    if "--config" in argv:
        return json.loads(argv[argv.index("--config") + 1])
    d, W, kappa = (int(x) for x in argv[pos:pos + 3]) if len(argv) >= pos + 3 else (1024, 16384, 32)
    return {"d": d, "W": W, "kappa": kappa}


if __name__ == "__main__":
    if sys.argv[1] == "stats":
        stats(sys.argv[2], sys.argv[3])
    elif sys.argv[1] == "traffic":
        traffic(sys.argv[2], sys.argv[3], sys.argv[4], _config(sys.argv, 5))
    elif sys.argv[1] == "sq":
        sq(sys.argv[2], sys.argv[3], _config(sys.argv, 4))
