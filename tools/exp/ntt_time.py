"""time the batched d = 1024 NTT / INTT (bench.py side_ops' workload): 2^16 polynomials"""
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import torch  # noqa: E402
import bench  # noqa: E402
import latticeum_amd as LA  # noqa: E402

for _ in range(3):
    o = bench.side_ops(LA, torch, 0)
    print(round(o["ntt_fwd"]["ms"], 4), round(o["ntt_inv"]["ms"], 4), flush=True)
