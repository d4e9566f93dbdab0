"""End-to-end probe for SURVEY.md §8f row 2 (decode overlapped with the
training step): the reference's training loop (lance_iterable.py:100-116:
.to(device), zero_grad, forward, CrossEntropy, backward, SGD step,
loss.item() every step) fed three ways from the same Arrow dataset of
FOOD101-shaped JPEGs through LanceDataset + ShardedBatchSampler (rank 0 of 1):

  train_only  the step on one pre-decoded batch (upper bound, no input path)
  sync        to_tensor_fn = decode_tensor_image (decode, then the step)
  prefetch    to_tensor_fn = make_to_tensor_fn(prefetch=2): batches k+1, k+2
              decode on side streams while step k runs

Model: ResNet-50 (torchvision's layout — bottlenecks [3, 4, 6, 3], 101
classes — written out here because torchvision is not installed; random
init), fp32 as in the reference. Prints one JSON line.
    python tools/train_overlap.py [--batch 128] [--steps 12]
"""
import argparse
import json
import os
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "lance-distributed-training_amd"))

import numpy as np  # noqa: E402
import pyarrow as pa  # noqa: E402
import torch  # noqa: E402
import torch.nn as nn  # noqa: E402


class Bottleneck(nn.Module):
    def __init__(self, cin, width, stride):
        super().__init__()
        cout = width * 4
        self.c1 = nn.Conv2d(cin, width, 1, bias=False)
        self.b1 = nn.BatchNorm2d(width)
        self.c2 = nn.Conv2d(width, width, 3, stride, 1, bias=False)
        self.b2 = nn.BatchNorm2d(width)
        self.c3 = nn.Conv2d(width, cout, 1, bias=False)
        self.b3 = nn.BatchNorm2d(cout)
        self.down = None
        if stride != 1 or cin != cout:
            self.down = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False), nn.BatchNorm2d(cout))

    def forward(self, x):
        r = x if self.down is None else self.down(x)
        y = torch.relu(self.b1(self.c1(x)))
        y = torch.relu(self.b2(self.c2(y)))
        return torch.relu(self.b3(self.c3(y)) + r)


def resnet50(num_classes=101):
    layers = [nn.Conv2d(3, 64, 7, 2, 3, bias=False), nn.BatchNorm2d(64), nn.ReLU(inplace=True),
              nn.MaxPool2d(3, 2, 1)]
    cin = 64
    for width, blocks, stride in ((64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2)):
        for b in range(blocks):
            layers.append(Bottleneck(cin, width, stride if b == 0 else 1))
            cin = width * 4
    layers += [nn.AdaptiveAvgPool2d(1), nn.Flatten(), nn.Linear(cin, num_classes)]
    return nn.Sequential(*layers)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--steps", type=int, default=12)
    args = ap.parse_args()
    import ldt_amd
    from ldt_amd import synth

    dev = torch.device("cuda:0")
    B, K = args.batch, args.steps
    cells, labels = synth.food101_like(B * 4, seed=3)
    tmp = tempfile.mkdtemp()
    tbl = pa.table({"image": pa.array(cells, pa.binary()), "label": pa.array(labels, pa.int64())})
    ds_path = os.path.join(tmp, "food.arrow")
    ldt_amd.write_dataset(tbl, ds_path, max_rows_per_file=12500)

    model = resnet50().to(dev)
    opt = torch.optim.SGD(model.parameters(), lr=0.01)
    loss_fn = nn.CrossEntropyLoss()

    def step(batch):
        images = batch["image"].to(dev)
        lbl = batch["label"].to(dev)
        opt.zero_grad()
        loss = loss_fn(model(images), lbl)
        loss.backward()
        opt.step()
        return loss.item()

    def batches(fn, k):
        # epochs of the 4-batch dataset until k batches were consumed
        while True:
            ds = ldt_amd.LanceDataset(ds_path, batch_size=B, to_tensor_fn=fn,
                                      sampler=ldt_amd.ShardedBatchSampler(rank=0, world_size=1))
            for b in ds:
                yield b
                k -= 1
                if k == 0:
                    return

    def timed(it, k):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        n = 0
        for b in it:
            step(b)
            n += 1
        torch.cuda.synchronize()
        assert n == k
        return (time.perf_counter() - t0) / k * 1e3

    fixed = ldt_amd.decode_tensor_image(next(iter(batches(None, 1))), device=dev)
    for _ in range(3):  # warm-up: MIOpen kernel selection, allocator
        step(fixed)
    res = {}
    res["train_only_ms"] = timed(iter([fixed] * K), K)
    res["sync_ms"] = timed(batches(ldt_amd.decode_tensor_image, K), K)
    pf = ldt_amd.make_to_tensor_fn(depth=3, device=dev, prefetch=2)
    for b in batches(pf, 3):  # warm the pipeline's contexts
        step(b)
    res["prefetch_ms"] = timed(batches(pf, K), K)
    # the input path alone (host RecordBatch -> tensors), synchronous
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for b in batches(ldt_amd.decode_tensor_image, K):
        pass
    torch.cuda.synchronize()
    res["decode_only_ms"] = (time.perf_counter() - t0) / K * 1e3
    out = {"probe": "train_overlap", "model": "resnet50 (fp32, random init, 101 classes)", "batch": B,
           "steps": K, "data": "FOOD101-shaped synthetic JPEG (q75 4:2:0) via LanceDataset + ShardedBatchSampler"}
    out.update({k: round(v, 3) for k, v in res.items()})
    out["train_img_s_prefetch"] = round(B / res["prefetch_ms"] * 1e3, 1)
    out["overlap_hidden_frac"] = round((res["sync_ms"] - res["prefetch_ms"]) / max(1e-9, res["decode_only_ms"]), 3)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
