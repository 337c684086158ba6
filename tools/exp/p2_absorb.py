"""host transcript cost: absorbing ring elements (lf_transcript_absorb_ring, d = 24) vs
the raw permutations behind it (lf_hash_iter at rate 12): us per permutation"""
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import latticeum_amd as LA  # noqa: E402

n = 8000  # ring elements: 16 000 permutations
x = np.random.default_rng(1).integers(0, 1 << 63, n * 24, dtype=np.uint64)
for _ in range(3):
    t = LA.Poseidon2Transcript()
    t0 = time.perf_counter()
    t.absorb_ring(x, 24)
    t.sample()
    a = time.perf_counter() - t0
    t0 = time.perf_counter()
    LA.hash_iter(x)
    b = time.perf_counter() - t0
    print(f"absorb {a / (n * 2) * 1e6:.3f} us/perm   hash_iter {b / (n * 2) * 1e6:.3f} us/perm")
