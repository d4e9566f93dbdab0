"""Diagnostic: raw resize diff pattern vs the oracle."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "lance-distributed-training_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import torch, ldt_amd
from oracle import oracle
for (h, w) in ((300, 200), (224, 224), (40, 1000), (1024, 1024), (500, 333)):
    x = np.random.RandomState(1).randint(0, 256, size=(2, h, w, 3), dtype=np.uint8)
    for dev in (False, True):
        t = torch.from_numpy(x)
        if dev: t = t.cuda()
        out = ldt_amd.resize_raw(t, h, w, normalize=False).cpu().numpy()
        exp = oracle.raw_to_tensor(x[0])
        d = np.abs(out[0] - exp)
        bad = np.argwhere(d > 0)
        print((h, w), "dev" if dev else "host", "maxdiff", d.max(), "nbad", len(bad), bad[:6].tolist(), flush=True)
