"""Diagnostic (not a test): per-image max abs diff vs the oracle for both
resize implementations on the golden images and config batches."""
import json, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "lance-distributed-training_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import numpy as np, pyarrow as pa
import ldt_amd
from ldt_amd import _lib, synth
from oracle import oracle
G = os.path.join(os.path.dirname(__file__), "..", "..", "tests", "golden")
man = json.load(open(os.path.join(G, "manifest.json")))
ctx = _lib.get_context(0)
def batch(cells):
    return pa.RecordBatch.from_arrays([pa.array(cells, pa.binary()), pa.array(np.arange(len(cells)), pa.int64())],
                                      names=["image", "label"])
for impl in (2, 0):
    ctx.set_option(_lib.OPT_RESIZE_IMPL, impl)
    bad = []
    for e in man["images"]:
        b = open(os.path.join(G, e["file"]), "rb").read()
        img = ldt_amd.decode_tensor_image(batch([b]))["image"].cpu().numpy()[0]
        d = np.abs(img - oracle.jpeg_to_tensor(b))
        if d.max() > 0:
            ch, yy, xx = np.unravel_index(np.argmax(d), d.shape)
            bad.append((e["name"], round(float(d.max()) * 255, 1), int(np.count_nonzero(d)), (int(ch), int(yy), int(xx))))
    print("impl", impl, "bad:", bad, flush=True)
    cells, labels = synth.q90_512(8, seed=3)
    img = ldt_amd.decode_tensor_image(batch(cells))["image"].cpu().numpy()
    print("impl", impl, "q90", [round(float(np.abs(img[k] - oracle.jpeg_to_tensor(cells[k])).max()) * 255, 1) for k in range(8)], flush=True)
