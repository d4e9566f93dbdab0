"""End-to-end probe of the map-style path:
the reference's lance_map_style.py loop — SafeLanceDataset + DistributedSampler
+ get_safe_loader(batch_size=128, num_workers=8, collate_fn=...) — over an
Arrow dataset of FOOD101-shaped JPEGs, with

  gpu           ldt_amd.collate_fn + ldt_amd.DistributedSampler (workers fetch
                rows and pack them into one RecordBatch; decode + sampler
                indices on the GPU)
  gpu_prefetch  the same with make_collate_fn(prefetch=2)
  ref  the reference recipe: PIL collate_fn (lance_map_style.py:21-44) in the
       8 workers + torch's DistributedSampler

Both iterate the same epoch after one warm epoch; prints one JSON line.
    python tools/mapstyle_probe.py [--rows 4096] [--workers 8]
"""
import argparse
import json
import os
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "lance-distributed-training_amd"), REPO):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import pyarrow as pa  # noqa: E402
import torch  # noqa: E402


def epoch(loader, device_out):
    t0 = time.perf_counter()
    n = 0
    for b in loader:
        img = b["image"]
        if device_out:
            assert img.is_cuda
        n += img.shape[0]
    torch.cuda.synchronize()
    return n, time.perf_counter() - t0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=4096)
    ap.add_argument("--workers", type=int, default=8)
    args = ap.parse_args()
    import ldt_amd
    from ldt_amd import synth
    from oracle import oracle  # the reference recipe (checker side)

    cells, labels = synth.food101_like(args.rows, seed=11)
    tmp = tempfile.mkdtemp()
    path = os.path.join(tmp, "food.arrow")
    ldt_amd.write_dataset(pa.table({"image": pa.array(cells, pa.binary()),
                                    "label": pa.array(labels, pa.int64())}), path, max_rows_per_file=1024)
    ds = ldt_amd.SafeLanceDataset(path)
    res = {"probe": "mapstyle", "rows": args.rows, "batch": 128, "num_workers": args.workers,
           "bytes_per_img": round(float(np.mean([len(c) for c in cells])), 1)}
    for mode in ("gpu", "gpu_prefetch", "ref"):
        if mode.startswith("gpu"):
            smp = ldt_amd.DistributedSampler(ds, num_replicas=1, rank=0, seed=3)
            collate = ldt_amd.collate_fn if mode == "gpu" else ldt_amd.make_collate_fn(prefetch=2)
        else:
            smp = torch.utils.data.DistributedSampler(ds, num_replicas=1, rank=0, seed=3)
            collate = oracle.pil_collate_fn
        loader = ldt_amd.get_safe_loader(ds, batch_size=128, sampler=smp, num_workers=args.workers,
                                         collate_fn=collate, persistent_workers=True)
        smp.set_epoch(0)
        epoch(loader, mode != "ref")  # warm: worker start-up, contexts
        smp.set_epoch(1)
        n, dt = epoch(loader, mode != "ref")
        res[f"{mode}_img_s"] = round(n / dt, 1)
    res["gpu_over_ref"] = round(res["gpu_img_s"] / res["ref_img_s"], 2)
    res["gpu_prefetch_over_ref"] = round(res["gpu_prefetch_img_s"] / res["ref_img_s"], 2)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
