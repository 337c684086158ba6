"""Profile driver for the 8(f) kernels: one folding-sumcheck prove and the
sparse CCS products at the zkvm shapes (bench.next_rows without the CPU leg)."""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

import bench  # noqa: E402
import latticeum_amd as LA  # noqa: E402

if __name__ == "__main__":
    print(json.dumps(bench.next_rows(LA, torch, 0, None)))
