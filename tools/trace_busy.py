"""Kernel-trace occupancy of a roctx range: per kernel total / count / mean, the
union of busy time, time with k kernels in flight, and the longest idle gaps.
usage: python tools/trace_busy.py DIR [range-name]"""
import csv
import glob
import sys
from collections import defaultdict


def rows(path):
    with open(path) as f:
        yield from csv.DictReader(f)


def main():
    d = sys.argv[1]
    name = sys.argv[2] if len(sys.argv) > 2 else "timed_steps"
    kt = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
    mk = glob.glob(f"{d}/**/*marker_api_trace.csv", recursive=True)
    lo, hi = 0, 1 << 63
    for m in (rows(mk[0]) if mk else []):
        if m.get("Function") == name:
            lo, hi = int(m["Start_Timestamp"]), int(m["End_Timestamp"])
    ev = []
    tot = defaultdict(lambda: [0.0, 0])
    for r in rows(kt):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if s < lo or e > hi:
            continue
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
        ev.append((s, e, k))
        tot[k][0] += (e - s) / 1e3
        tot[k][1] += 1
    ev.sort()
    t0, t1 = ev[0][0], max(e for _, e, _ in ev)
    span = (t1 - t0) / 1e3
    pts = sorted([(s, 1) for s, _, _ in ev] + [(e, -1) for _, e, _ in ev])
    depth, last, hist, gaps = 0, t0, defaultdict(float), []
    for t, dlt in pts:
        hist[depth] += (t - last) / 1e3
        if depth == 0 and t > last:
            gaps.append(((t - last) / 1e3, last))
        depth += dlt
        last = t
    print(f"range {name}: {len(ev)} kernels over {span:.1f} us")
    for k, v in sorted(tot.items(), key=lambda kv: -kv[1][0]):
        print(f"  {k[:60]:60s} n={v[1]:5d} total={v[0]:9.1f} us mean={v[0] / v[1]:8.2f} us")
    print("  in flight: " + ", ".join(f"{k}: {v / span:.3f}" for k, v in sorted(hist.items())))
    gaps.sort(reverse=True)
    print("  idle total %.1f us, largest gaps (us): %s" % (sum(g for g, _ in gaps),
                                                       [round(g, 1) for g, _ in gaps[:10]]))


if __name__ == "__main__":
    main()
