"""BASELINE configs[1] (2^16 d = 1024 NTT / INTT) and configs[4]'s Poseidon2 batch
(2^20 width-16 states) alone, as bench.side_ops times them: the program the
side-op PMC passes profile (tools/gpu_pmc_side.sh), so their counters come from
these launches at these sizes."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

import bench  # noqa: E402
import latticeum_amd as LA  # noqa: E402

if __name__ == "__main__":
    torch.cuda.set_device(0)
    print(json.dumps(bench.side_ops(LA, torch, 0)), flush=True)
