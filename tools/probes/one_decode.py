"""Diagnostic: decode a few c2 images once (smallest GPU repro)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "lance-distributed-training_amd"))
import ldt_amd  # noqa: E402
from ldt_amd import synth  # noqa: E402

cells, labels = synth.q90_512(4, seed=1)
out = ldt_amd.decode_tensor_image(synth.arrow_batch(cells, labels), device="cuda:0")
print("ok", out["image"].shape, float(out["image"].mean()))
