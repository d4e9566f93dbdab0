"""Standalone k_resize4 time on a batch of 256 336x336 q90 4:2:0 JPEGs (one
batch in flight), whose resize fits 16 waves per CU in LDS: the occupancy
study of DESIGN.md §4 (LDT_LIBRARY selects the build). GPU box only."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "lance-distributed-training_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import ldt_amd  # noqa: E402
from ldt_amd import _lib, synth  # noqa: E402

n, side = 256, int(os.environ.get("SIDE", "336"))
cells = [synth.encode(synth.field(side, side, 100 + k), quality=90, subsampling=2) for k in range(n)]
rb = ldt_amd.ResidentBatch(cells, np.arange(n), device=torch.device("cuda", 0))
pipe = ldt_amd.DecodePipeline(depth=1, device=torch.device("cuda", 0), profile=True)
for _ in range(3):
    pipe.decode(rb)
torch.cuda.synchronize()
pipe.stage_times(reset=True)
for _ in range(10):
    pipe.decode(rb)
torch.cuda.synchronize()
st = pipe.stage_times(reset=True)
pipe.check()
print(side, {k: round(v[0] / max(v[1], 1), 4) for k, v in st.items()})
