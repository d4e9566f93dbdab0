"""Worker for tests/test_gpu_dist.py: one rank of the reference's iterable DDP
setup (lance_iterable.py:61-69, :80) on the GPU box — gloo process group, both
ranks on cuda:0, LanceDataset + ShardedFragmentSampler(pad=True) with the
device shard kernel (no stand-ins) + decode_tensor_image."""
import os
import sys


def run(rank, world, port, uri, outdir, check_every=7):
    here = os.path.dirname(os.path.abspath(__file__))
    repo = os.path.dirname(here)
    for p in (os.path.join(repo, "lance-distributed-training_amd"), repo, here):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import hashlib
    import json

    import numpy as np
    import torch
    import torch.distributed as dist

    import ldt_amd
    from ldt_amd import LanceDataset, ShardedFragmentSampler
    from oracle import oracle

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ds = ldt_amd.dataset(uri)
    sampler = ShardedFragmentSampler(rank=rank, world_size=world, pad=True)
    loader = LanceDataset(ds, batch_size=8, sampler=sampler, to_tensor_fn=ldt_amd.decode_tensor_image)
    labels, bad = [], []
    for k, b in enumerate(loader):
        lbl = b["label"].cpu().numpy()
        labels.append(lbl.tolist())
        if k % check_every == 0:  # every check_every-th batch image by image vs the oracle
            rows = ds.take(lbl.tolist(), ["image"]).column("image").to_pylist()
            img = b["image"].cpu().numpy()
            for j, cell in enumerate(rows):
                if hashlib.sha256(img[j].tobytes()).hexdigest() != \
                        hashlib.sha256(oracle.jpeg_to_tensor(cell).tobytes()).hexdigest():
                    bad.append(int(lbl[j]))
    with open(os.path.join(outdir, f"gpu_rank{rank}.json"), "w") as f:
        json.dump({"batches": len(labels), "labels": labels, "bad": bad}, f)
    dist.barrier()
    dist.destroy_process_group()
