"""Generate the committed golden fixtures for the batch-decode hot path.

The expected outputs come from the reference arithmetic itself as it exists
in this container — Pillow 12.2.0 (libjpeg-turbo 3.1.4.1) for
``Image.open(BytesIO(b)).convert("RGB")`` and ``.resize((224, 224), BILINEAR)``
(what torchvision's ``Resize((224,224))`` calls for PIL input), then the
torchvision ``to_tensor`` recipe (``float32 / 255``, CHW) and ``Normalize``
restated in numpy (torchvision is absent). Reference call sites:
``lance_iterable.py:28-50``, ``lance_map_style.py:21-44``. The reference's
own Python files cannot be imported (pylance/torchvision absent, an ordinary
ModuleNotFoundError — SURVEY.md §8c), so the fixtures pin the third-party
arithmetic they call.

Sampler vectors follow README.md:140-155 / 257-271 (FOOD101 fragments
[12500 x 6, 750], B = 128, W = 1, 2, 4, 8); see oracle/oracle.py.

Run:  python tests/golden/make_golden.py   (writes tests/golden/*)
"""
from __future__ import annotations

import hashlib
import io
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "lance-distributed-training_amd"))
sys.path.insert(0, REPO)

from PIL import Image, features  # noqa: E402

from ldt_amd import synth  # noqa: E402  (seeded fields + PIL encoder only)
from oracle import oracle  # noqa: E402  (sampler restatement)

MEAN = np.asarray((0.485, 0.456, 0.406), np.float32)[:, None, None]
STD = np.asarray((0.229, 0.224, 0.225), np.float32)[:, None, None]


def sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


CASES = [
    # name, H, W, save kwargs, noise
    ("food_384x512_q75", 384, 512, {}, 20),
    ("food_512x384_q75", 512, 384, {}, 20),
    ("food_512x512_q75", 512, 512, {}, 20),
    ("c2_512x512_q90", 512, 512, dict(quality=90, subsampling="4:2:0"), 20),
    ("c4_375x500_q90_rst", 375, 500, dict(quality=90, restart_marker_rows=1), 20),
    ("c4_250x333_q90_rstblk", 250, 333, dict(quality=90, restart_marker_blocks=5), 20),
    ("odd_13x17", 13, 17, {}, 20),
    ("tiny_1x1", 1, 1, {}, 20),
    ("tiny_3x5", 3, 5, {}, 20),
    ("tiny_4x4", 4, 4, {}, 20),
    ("tiny_5x5", 5, 5, {}, 20),
    ("tiny_2x9", 2, 9, {}, 20),
    ("strip_1x200", 1, 200, {}, 20),
    ("strip_200x1", 200, 1, {}, 20),
    ("exact_224x224", 224, 224, {}, 20),
    ("up_100x150", 100, 150, {}, 20),
    ("s444_100x300", 100, 300, dict(subsampling="4:4:4"), 20),
    ("s422_33x65", 33, 65, dict(subsampling="4:2:2"), 20),
    ("big_768x1024_q95", 768, 1024, dict(quality=95), 12),
    ("q100_64x64", 64, 64, dict(quality=100), 30),
    ("noisy_256x256_q50", 256, 256, dict(quality=50), 60),
    ("flat_96x96", 96, 96, {}, 0),
    # progressive (SOF2, libjpeg jpeg_simple_progression: spectral selection +
    # successive approximation, EOB runs)
    ("prog_64x80", 64, 80, dict(progressive=True), 20),
    ("prog_375x500_q90", 375, 500, dict(quality=90, progressive=True), 20),
    ("prog_13x17", 13, 17, dict(progressive=True), 20),
    ("prog_1x200", 1, 200, dict(progressive=True), 20),
    ("prog_s444_100x300", 100, 300, dict(subsampling="4:4:4", progressive=True), 20),
    ("prog_s422_33x65", 33, 65, dict(subsampling="4:2:2", progressive=True), 20),
    ("prog_rst_250x333_q90", 250, 333, dict(quality=90, progressive=True, restart_marker_blocks=5), 20),
    ("prog_q100_64x64", 64, 64, dict(quality=100, progressive=True), 30),
]


def pil_expected(b: bytes):
    im = Image.open(io.BytesIO(b)).convert("RGB")
    rgb = np.asarray(im, np.uint8)
    rs = np.asarray(im.resize((224, 224), Image.BILINEAR), np.uint8)
    t = rs.transpose(2, 0, 1).astype(np.float32) / np.float32(255)
    tn = (t - MEAN) / STD
    return rgb, rs, t, tn


def _cmyk(rgb) -> bytes:
    """4-component (CMYK, Adobe) JPEG: Pillow decodes it, the build reports
    LDT_IMG_UNSUPPORTED (ldt.h)."""
    b = io.BytesIO()
    Image.fromarray(rgb).convert("CMYK").save(b, format="JPEG")
    return b.getvalue()


def main():
    jdir = os.path.join(HERE, "jpeg")
    os.makedirs(jdir, exist_ok=True)
    manifest = {
        "generator": "tests/golden/make_golden.py",
        "pillow": Image.__version__ if hasattr(Image, "__version__") else "",
        "libjpeg_turbo": features.version_feature("libjpeg_turbo"),
        "images": [],
        "bad": [],
    }
    import PIL

    manifest["pillow"] = PIL.__version__
    for i, (name, h, w, kw, noise) in enumerate(CASES):
        if name.startswith("tiny") or name.startswith("strip") or name == "flat_96x96":
            img = synth.field(h, w, 1000 + i, noise)
        else:
            img = synth.field(h, w, 1000 + i, noise)
        if name == "flat_96x96":
            img[:] = (40, 200, 90)
        b = synth.encode(img, **kw)
        with open(os.path.join(jdir, name + ".jpg"), "wb") as f:
            f.write(b)
        rgb, rs, t, tn = pil_expected(b)
        manifest["images"].append({
            "name": name, "file": f"jpeg/{name}.jpg", "height": rgb.shape[0], "width": rgb.shape[1],
            "bytes": len(b), "label": (7 * i) % 101,
            "sha256_rgb": sha(rgb), "sha256_resized_u8": sha(rs),
            "sha256_tensor_f32": sha(t), "sha256_tensor_norm_f32": sha(tn),
        })
    # gray (mode L -> convert("RGB") replicates)
    g = synth.field(77, 91, 4242)[..., 0]
    b = io.BytesIO()
    Image.fromarray(g).save(b, format="JPEG")
    b = b.getvalue()
    with open(os.path.join(jdir, "gray_77x91.jpg"), "wb") as f:
        f.write(b)
    rgb, rs, t, tn = pil_expected(b)
    manifest["images"].append({"name": "gray_77x91", "file": "jpeg/gray_77x91.jpg", "height": 77, "width": 91,
                               "bytes": len(b), "label": 100, "sha256_rgb": sha(rgb),
                               "sha256_resized_u8": sha(rs), "sha256_tensor_f32": sha(t),
                               "sha256_tensor_norm_f32": sha(tn)})
    b = io.BytesIO()
    Image.fromarray(g).save(b, format="JPEG", progressive=True)
    b = b.getvalue()
    with open(os.path.join(jdir, "prog_gray_77x91.jpg"), "wb") as f:
        f.write(b)
    rgb, rs, t, tn = pil_expected(b)
    manifest["images"].append({"name": "prog_gray_77x91", "file": "jpeg/prog_gray_77x91.jpg", "height": 77,
                               "width": 91, "bytes": len(b), "label": 99, "sha256_rgb": sha(rgb),
                               "sha256_resized_u8": sha(rs), "sha256_tensor_f32": sha(t),
                               "sha256_tensor_norm_f32": sha(tn)})
    # bad inputs: PIL raises on each
    good = open(os.path.join(jdir, "food_384x512_q75.jpg"), "rb").read()
    bad = {
        "bad_truncated": good[: len(good) // 2],
        "bad_not_jpeg": b"\x89PNG\r\n\x1a\n" + bytes(range(200)),
        "bad_cmyk": _cmyk(synth.field(64, 80, 5)),
        "bad_empty": b"",
    }
    for name, data in bad.items():
        with open(os.path.join(jdir, name + ".bin"), "wb") as f:
            f.write(data)
        try:
            pil_expected(data)
            raised = False
        except Exception:
            raised = True
        manifest["bad"].append({"name": name, "file": f"jpeg/{name}.bin", "pil_raises": raised,
                                "expect_status": {"bad_truncated": 3, "bad_not_jpeg": 1,
                                                  "bad_cmyk": 2, "bad_empty": 1}[name]})
    # raw HWC (config 5 path) small fixture
    raw = np.random.RandomState(5).randint(0, 256, size=(2, 300, 200, 3), dtype=np.uint8)
    exp = []
    for k in range(2):
        rs = np.asarray(Image.fromarray(raw[k]).resize((224, 224), Image.BILINEAR), np.uint8)
        t = rs.transpose(2, 0, 1).astype(np.float32) / np.float32(255)
        exp.append({"sha256_tensor_f32": sha(t), "sha256_tensor_norm_f32": sha((t - MEAN) / STD)})
    np.savez_compressed(os.path.join(HERE, "raw_small.npz"), hwc=raw)
    manifest["raw"] = {"file": "raw_small.npz", "expected": exp}
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)

    # sampler vectors
    frags = synth.FOOD101_FRAGMENTS
    sv = {"fragments": frags, "batch_size": 128, "num_rows": sum(frags), "sharded_batch": {}, "sharded_fragment": {}}
    for W in (1, 2, 4, 8):
        sb, sf = [], []
        for r in range(W):
            rngs = np.asarray(oracle.sharded_batch_ranges(sum(frags), 128, r, W), np.int64).reshape(-1, 2)
            sb.append({"count": int(len(rngs)), "first": rngs[0].tolist() if len(rngs) else None,
                       "last": rngs[-1].tolist() if len(rngs) else None, "sha256": sha(rngs)})
            recs = np.asarray(oracle.sharded_fragment_batches(frags, 128, r, W, pad=False), np.int64).reshape(-1, 5)
            prec = np.asarray(oracle.sharded_fragment_batches(frags, 128, r, W, pad=True), np.int64).reshape(-1, 5)
            sf.append({"count": int(len(recs)), "padded_count": int(len(prec)), "sha256": sha(recs),
                       "sha256_padded": sha(prec)})
        sv["sharded_batch"][str(W)] = sb
        sv["sharded_fragment"][str(W)] = sf
    with open(os.path.join(HERE, "sampler.json"), "w") as f:
        json.dump(sv, f, indent=1)
    print("wrote", len(manifest["images"]), "images,", len(manifest["bad"]), "bad inputs")


if __name__ == "__main__":
    main()
