"""Diagnostic: how much of the standalone stage time the 3-deep pipeline hides
at c2's shape (256 x 512x512 4:2:0) as the JPEG quality (stream size, so
k_huff_image's LDS window) varies: a smaller window leaves room for a resize
workgroup beside the Huffman decoder of another batch."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "lance-distributed-training_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import ldt_amd  # noqa: E402
from ldt_amd import synth  # noqa: E402

for q in (90, 75, 50):
    batches = []
    for k in range(2):
        cells = [synth.encode(synth.field(512, 512, k * 100003 + i, 6.0), quality=q, subsampling="4:2:0")
                 for i in range(256)]
        batches.append(ldt_amd.ResidentBatch(cells, np.arange(256) % 101))
    kb = max(len(c) for c in cells) / 1024
    pipe = ldt_amd.DecodePipeline(depth=3)
    for k in range(10):
        pipe.decode(batches[k % 2])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(60):
        pipe.decode(batches[k % 2])
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / 60 * 1e3
    solo = ldt_amd.DecodePipeline(depth=1, profile=True)
    for k in range(3):
        solo.decode(batches[k % 2])
    torch.cuda.synchronize()
    solo.stage_times(reset=True)
    for k in range(6):
        solo.decode(batches[k % 2])
    torch.cuda.synchronize()
    st = {k: v[0] / max(v[1], 1) for k, v in solo.stage_times(reset=True).items()}
    tot = sum(v for k, v in st.items() if k != "h2d")
    print(f"q{q}: max cell {kb:.1f} KB; pipelined {ms:.3f} ms/step ({256 / ms * 1e3:,.0f} img/s); standalone "
          f"{ {k: round(v, 3) for k, v in st.items()} } sum {tot:.3f} ms; hidden {1 - ms / tot:.0%}", flush=True)
