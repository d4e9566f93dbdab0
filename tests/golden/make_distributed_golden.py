"""Golden vectors for the map-style DistributedSampler row:
torch 2.10's own torch.utils.data.DistributedSampler (the reference's
lance_map_style.py:58 sampler, in-container) run here; sha256 of the int64
index vector per case. Regenerate: python tests/golden/make_distributed_golden.py"""
import hashlib
import json
import os

import numpy as np
import torch
from torch.utils.data import DistributedSampler

CASES = []
for n in (0, 1, 2, 7, 101, 1000, 75750):  # 75,750 = FOOD101 train rows
    for W in (1, 2, 3, 8):
        for drop_last in (False, True):
            for shuffle in (True, False):
                CASES.append(dict(n=n, W=W, drop_last=drop_last, shuffle=shuffle, seed=0, epoch=0))
CASES += [dict(n=75750, W=8, drop_last=False, shuffle=True, seed=s, epoch=e)
          for s, e in ((42, 3), (-5, 1), (2**40 + 7, 0), (2**63 - 1, 1))]
CASES += [dict(n=1281167, W=8, drop_last=False, shuffle=True, seed=0, epoch=1)]  # ImageNet-1k train


def run(c):
    out = []
    for r in range(c["W"]):
        s = DistributedSampler(range(c["n"]), num_replicas=c["W"], rank=r, shuffle=c["shuffle"],
                               seed=c["seed"], drop_last=c["drop_last"])
        s.set_epoch(c["epoch"])
        idx = np.asarray(list(s), np.int64)
        out.append(dict(count=len(idx), sha256=hashlib.sha256(idx.tobytes()).hexdigest(),
                        head=idx[:4].tolist()))
    return out


if __name__ == "__main__":
    res = [dict(case=c, ranks=run(c)) for c in CASES]
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "distributed.json")
    json.dump(dict(torch=torch.__version__, cases=res), open(path, "w"), indent=0)
    print(path, len(res))
