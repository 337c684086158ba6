"""Host checks of the device field helpers in latticeum_amd/csrc/gl.hpp that have no
oracle counterpart: gl::from_x_y32, the exact reduction of X + Y 2^32 for signed
|X|, |Y| < 2^62 that the i8-MFMA epilogues end in (mz.hip k_zcomb_mfma), against
Python's integers -- random pairs over every magnitude and the edge values. The
header is compiled for the host with ROCm's clang (its __builtin_addc); the test
is skipped where that compiler is absent."""
import os
import subprocess
import tempfile
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
CLANG = "/opt/rocm/lib/llvm/bin/clang++"
P = (1 << 64) - (1 << 32) + 1

DRIVER = r"""
#include "gl.hpp"
#include <cstdio>
#include <cstdlib>
static unsigned long long s = 0x4C46u;
static unsigned long long nxt() {  // SplitMix64
  unsigned long long z = (s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
static long long pick() {
  const int sh = (int)(nxt() % 63);  // magnitudes 0 .. 2^62 - 1
  const long long m = sh ? (long long)(nxt() >> (64 - sh)) : 0;
  return (nxt() & 1) ? -m : m;
}
int main(int argc, char **argv) {
  const long long L = (1ll << 62) - 1;
  const long long edge[] = {0, 1, -1, L, -L, 1ll << 32, -(1ll << 32), (1ll << 32) - 1, -((1ll << 32) - 1),
                            1ll << 48, -(1ll << 48), 0x7FFFFFFF, -0x80000000ll, 0xFFFFFFFF00000001ll >> 2};
  for (long long a : edge)
    for (long long b : edge) printf("%lld %lld %llu\n", a, b, (unsigned long long)gl::from_x_y32(a, b));
  const int n = atoi(argv[1]);
  for (int i = 0; i < n; i++) {
    const long long x = pick(), y = pick();
    printf("%lld %lld %llu\n", x, y, (unsigned long long)gl::from_x_y32(x, y));
  }
  return 0;
}
"""


def test_from_x_y32_matches_integers():
    if not os.path.exists(CLANG):
        pytest.skip("ROCm clang++ not present")
    with tempfile.TemporaryDirectory() as td:
        src, exe = Path(td) / "xy.cpp", Path(td) / "xy"
        src.write_text(DRIVER)
        r = subprocess.run([CLANG, "-O2", "-std=c++17", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
                            f"-I{ROOT / 'latticeum_amd/csrc'}", "-x", "c++", str(src), "-o", str(exe)],
                           capture_output=True, text=True)
        if r.returncode != 0:
            pytest.skip(f"host build of gl.hpp failed: {r.stderr[-300:]}")
        out = subprocess.run([str(exe), "200000"], capture_output=True, text=True, check=True).stdout.split("\n")
    rows = [ln.split() for ln in out if ln]
    assert len(rows) == 14 * 14 + 200000
    for x, y, v in rows:
        want = (int(x) + (int(y) << 32)) % P
        assert int(v) == want, (x, y, v)
