"""Summarise a rocprofv3 kernel trace of tools/fold_prof.py: per kernel, the
launches and device time per fold() (the folds are counted by k_round_lin_eq_sparse,
launched once per fold), split at the first fold so the setup (CCS upload, A
conversion) is kept apart. usage: python tools/fold_trace_summary.py <prof_dir>"""
import csv
import glob
import sys
from collections import defaultdict


def main(d):
    f = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    starts = [int(r["Start_Timestamp"]) for r in rows if "k_round_lin_eq_sparse" in r["Kernel_Name"]]
    if not starts:
        raise SystemExit("no fold() found")
    t0 = starts[0] - 50_000_000  # 50 ms before the first sparse round: the fold's own Mz work starts earlier
    nf = len(starts)
    tot = defaultdict(lambda: [0, 0.0])
    setup = defaultdict(lambda: [0, 0.0])
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
        acc = tot if s >= t0 else setup
        acc[name][0] += 1
        acc[name][1] += (e - s) / 1e6
    span = (int(rows[-1]["End_Timestamp"]) - t0) / 1e6
    print(f"{nf} folds; trace span from the first fold {span:.1f} ms ({span / nf:.2f} ms per fold)")
    print("| kernel | launches per fold | device ms per fold |\n|---|---|---|")
    busy = 0.0
    for k, (n, ms) in sorted(tot.items(), key=lambda kv: -kv[1][1]):
        busy += ms
        print(f"| `{k}` | {n / nf:.1f} | {ms / nf:.3f} |")
    print(f"| (all) | | {busy / nf:.2f} |")
    print("setup:", {k: (n, round(ms, 1)) for k, (n, ms) in sorted(setup.items(), key=lambda kv: -kv[1][1])[:6]})


if __name__ == "__main__":
    main(sys.argv[1])
