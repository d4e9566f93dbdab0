"""Debug probe: the c2 corrupt-entropy fuzz trials of
tests/test_gpu_parity.py::test_corrupt_entropy_data_is_contained, reporting per
trial the status of the corrupt row and where a valid neighbour differs from
the oracle (block coordinates), decoding each batch twice."""
import os
import sys

import numpy as np
import pyarrow as pa

R = os.path.join(os.path.dirname(__file__), "..", "..")
sys.path.insert(0, os.path.join(R, "lance-distributed-training_amd"))
sys.path.insert(0, R)
import ldt_amd  # noqa: E402
from ldt_amd import synth  # noqa: E402
from oracle import oracle  # noqa: E402


def batch(cells):
    return pa.RecordBatch.from_arrays([pa.array(cells, pa.binary()), pa.array(np.arange(len(cells)), pa.int64())],
                                      names=["image", "label"])


def sos_end(b):
    i = 2
    while i + 4 <= len(b):
        m, L = b[i + 1], (b[i + 2] << 8) | b[i + 3]
        if m == 0xDA:
            return i + 2 + L
        i += 2 + L


base = synth.encode(synth.field(512, 512, 5, 6.0), quality=90)
good = synth.encode(synth.field(300, 200, 8, 6.0))
exp = oracle.jpeg_to_tensor(good)
rng = np.random.default_rng(1)
s0 = sos_end(base)
for trial in range(12):
    b = bytearray(base)
    mode = trial % 4
    for _ in range(int(rng.integers(1, 8))):
        p = int(rng.integers(s0, len(b) - 2))
        if mode == 0:
            b[p] ^= 1 << int(rng.integers(0, 8))
        elif mode == 1:
            b[p] = int(rng.integers(0, 256))
        elif mode == 2:
            b[p:p + 2] = bytes([0xFF, int(rng.choice([0x00, 0xD0, 0xD3, 0xD9, 0xC4, 0xFF]))])
        else:
            del b[p:p + int(rng.integers(1, 64))]
    for rep in range(2):
        try:
            out = ldt_amd.decode_tensor_image(batch([good, bytes(b), good]))["image"].cpu().numpy()
        except ldt_amd.ImageDecodeError as e:
            print(trial, rep, "error rows", e.rows, flush=True)
            continue
        for k in (0, 2):
            d = np.abs(out[k] - exp)
            if d.max() > 0:
                ys, xs = np.nonzero(d.max(0))
                print(trial, rep, "row", k, "max", d.max(), "n", len(ys), "y", ys.min(), ys.max(), "x", xs.min(), xs.max(),
                      flush=True)
        print(trial, rep, "ok" if all(np.array_equal(out[k], exp) for k in (0, 2)) else "DIFF", flush=True)
    alone = ldt_amd.decode_tensor_image(batch([good]))["image"].cpu().numpy()
    print(trial, "good alone after:", np.array_equal(alone[0], exp), flush=True)
