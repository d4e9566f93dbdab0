"""Worker for tests/test_gpu_fullbatch.py's config-shaped dataset legs: one
rank of the reference's iterable loop (lance_iterable.py:53-72, :80) on the GPU
box — gloo process group, every rank on cuda:0, LanceDataset + the config's
sampler (ShardedBatchSampler for configs[2], ShardedFragmentSampler(pad=True)
for configs[3]) + the pipelined copying to_tensor_fn (make_to_tensor_fn), batch
128. Row r of the dataset holds cell r % 128 of the fixture batch and label r;
every decoded image is compared with the fixture's oracle sha256 of its cell."""
import os
import sys


def run(rank, world, port, uri, outdir, kind, exp_path, batch=128):
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

    with open(exp_path) as f:
        exp = json.load(f)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    if kind == "fragment":
        sampler = ldt_amd.ShardedFragmentSampler(rank=rank, world_size=world, pad=True)
    else:
        sampler = ldt_amd.ShardedBatchSampler(rank=rank, world_size=world)
    fn = ldt_amd.make_to_tensor_fn()
    loader = ldt_amd.LanceDataset(uri, batch_size=batch, sampler=sampler, to_tensor_fn=fn)
    labels, bad = [], []
    for b in loader:
        lbl = b["label"].cpu().numpy()
        img = b["image"].cpu().numpy()
        labels.append(lbl.tolist())
        for j, r in enumerate(lbl.tolist()):
            if hashlib.sha256(np.ascontiguousarray(img[j]).tobytes()).hexdigest() != exp[r % len(exp)]:
                bad.append(int(r))
    fn.check()
    with open(os.path.join(outdir, f"fb_{kind}_rank{rank}.json"), "w") as f:
        json.dump({"batches": len(labels), "labels": labels, "bad": bad}, f)
    dist.barrier()
    dist.destroy_process_group()
