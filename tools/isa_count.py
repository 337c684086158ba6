#!/usr/bin/env python3
"""Static instruction mix per kernel of a gfx950 device assembly file.

  hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only -S x.hip -o x.s
  python tools/isa_count.py x.s [kernel-substring ...]

Counts VALU (v_*, minus the v_mfma/v_readlane/v_writelane classes listed
apart), SALU, LDS, global/buffer memory and s_nop per kernel body. A static
count: the hot kernels here are fully unrolled per loop iteration, so the body
count tracks the per-unit issue count closely enough to compare variants
before spending GPU time on them.
"""
import re
import sys
from collections import Counter


def kernels(path):
    cur, body = None, []
    for line in open(path):
        m = re.match(r"^(_Z\S+):\s*(;.*)?$", line)
        if m and cur is None:
            cur, body = m.group(1), []
            continue
        if cur is not None:
            if line.startswith(".Lfunc_end"):
                yield cur, body
                cur = None
            else:
                body.append(line)


def mix(body):
    c = Counter()
    for line in body:
        s = line.strip()
        if not s or s.startswith((";", ".")) or s.endswith(":"):
            continue
        op = s.split()[0]
        if op.startswith("v_mfma"):
            c["mfma"] += 1
        elif op.startswith("v_cndmask"):
            c["valu"] += 1
            c["cndmask"] += 1
        elif op.startswith("v_"):
            c["valu"] += 1
        elif op == "s_nop":
            c["nop"] += 1
        elif op.startswith("s_waitcnt"):
            c["wait"] += 1
        elif op.startswith("s_"):
            c["salu"] += 1
        elif op.startswith("ds_"):
            c["lds"] += 1
        elif op.startswith(("global_", "buffer_", "flat_", "scratch_")):
            c["vmem"] += 1
            if op.startswith("scratch_") or "spill" in s:
                c["scratch"] += 1
    return c


def main():
    path, pats = sys.argv[1], sys.argv[2:]
    for name, body in kernels(path):
        if pats and not any(p in name for p in pats):
            continue
        c = mix(body)
        keys = ("valu", "cndmask", "salu", "nop", "lds", "vmem", "scratch", "mfma", "wait")
        print(f"{name[:70]:70s} " + " ".join(f"{k}={c[k]}" for k in keys))


if __name__ == "__main__":
    main()
