"""Full c2 and c1 batches decoded with LDT_OPT_RESIZE_IMPL 1 (32-bit staging) and 0 (packed 16-bit, the default) must give
identical tensors (tools/r4_resizepk.sh)."""
import sys

import numpy as np

sys.path.insert(0, "lance-distributed-training_amd")
import pyarrow as pa  # noqa: E402

import ldt_amd  # noqa: E402
from ldt_amd import _lib, synth  # noqa: E402


def main():
    ctx = _lib.get_context(0)
    for name, (cells, labels) in (("c2", synth.q90_512(256, seed=3)), ("c1", synth.food101_like(128, seed=4))):
        b = pa.RecordBatch.from_arrays([pa.array(cells, pa.binary()), pa.array(np.asarray(labels, np.int64))],
                                       names=["image", "label"])
        out = {}
        for impl in (1, 0):
            ctx.set_option(_lib.OPT_RESIZE_IMPL, impl)
            out[impl] = ldt_amd.decode_tensor_image(b)["image"].cpu().numpy()
        ctx.set_option(_lib.OPT_RESIZE_IMPL, 0)
        assert np.array_equal(out[1], out[0]), name
        print(name, "impl 0 (packed) == impl 1 (32-bit) on", len(cells), "images")


if __name__ == "__main__":
    main()
