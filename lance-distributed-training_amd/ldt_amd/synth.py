"""Seeded synthetic inputs of the shapes BASELINE.json's configs name.

Stand-in for the reference's input producer (``create_datasets/
classification.py:13-63``): FOOD101 cannot be downloaded offline, so images
are seeded smooth fields + Gaussian noise (sigma 6: 22 KiB per FOOD101-shaped
q75 image, 65 KiB per 512x512 q90 image, matching SURVEY.md §6 probe sizes), encoded exactly as the reference
encodes them — ``img.save(buffer, format="JPEG")`` (``:27-29``), i.e. Pillow
defaults: quality 75, 4:2:0, baseline, standard Huffman tables, no restart
markers — unless a config asks otherwise (q90, restart markers).
Labels are ``i % 101`` (FOOD101 has 101 classes), int64.
"""
from __future__ import annotations

import io
from typing import List, Sequence, Tuple

import numpy as np

FOOD101_SHAPES = ((384, 512), (512, 384), (512, 512))  # (H, W), FOOD101 max side 512
FOOD101_FRAGMENTS = [12500] * 6 + [750]                 # 75,750 rows, max_rows_per_file=12500


def field(h: int, w: int, seed: int, noise: float = 20.0) -> np.ndarray:
    """Seeded uint8 HWC image: 3 sinusoid fields + Gaussian noise."""
    r = np.random.RandomState(seed)
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float32)
    img = np.empty((h, w, 3), np.float32)
    for c in range(3):
        fx, fy, ph = r.uniform(0.004, 0.05), r.uniform(0.004, 0.05), r.uniform(0, 6.28)
        img[..., c] = 128 + 90 * np.sin(xx * fx + yy * fy + ph) + 25 * np.cos(xx * fy * 1.7 - yy * fx * 0.6)
    img += r.normal(0, noise, img.shape).astype(np.float32)
    return np.clip(img, 0, 255).astype(np.uint8)


def _pmap(fn, n: int) -> list:
    """[fn(0), ..., fn(n-1)] on a thread pool (Pillow's encoder and numpy's
    large-array kernels release the GIL); each item is seeded by its index, so
    the result does not depend on the threads."""
    if n < 16:
        return [fn(i) for i in range(n)]
    import os
    from concurrent.futures import ThreadPoolExecutor

    with ThreadPoolExecutor(max(1, min(8, os.cpu_count() or 1))) as ex:
        return list(ex.map(fn, range(n)))


def encode(img: np.ndarray, **save_kwargs) -> bytes:
    from PIL import Image

    b = io.BytesIO()
    Image.fromarray(img).save(b, format="JPEG", **save_kwargs)
    return b.getvalue()


def food101_like(n: int, seed: int = 0, noise: float = 6.0) -> Tuple[List[bytes], np.ndarray]:
    """Config 1/3: FOOD101-shaped, PIL defaults (q75 4:2:0, no DRI)."""
    def one(i):
        h, w = FOOD101_SHAPES[(seed + i) % 3]
        return encode(field(h, w, seed * 100003 + i, noise))

    return _pmap(one, n), np.arange(n, dtype=np.int64) % 101


def q90_512(n: int, seed: int = 0, noise: float = 6.0,
            progressive: bool = False) -> Tuple[List[bytes], np.ndarray]:
    """Config 2: 512x512 baseline, 4:2:0, quality 90, no DRI (progressive=True:
    the same images as SOF2, libjpeg's default progression script)."""
    cells = _pmap(lambda i: encode(field(512, 512, seed * 100003 + i, noise), quality=90, subsampling="4:2:0",
                                   progressive=progressive), n)
    return cells, np.arange(n, dtype=np.int64) % 101


def imagenet_like(n: int, seed: int = 0, noise: float = 6.0) -> Tuple[List[bytes], np.ndarray]:
    """Config 4: variable ~500x375 (W in [333,500], H in [250,500]), q90, restart every MCU row."""
    r = np.random.RandomState(seed + 7)
    dims = [(int(r.randint(333, 501)), int(r.randint(250, 501))) for _ in range(n)]
    cells = _pmap(lambda i: encode(field(dims[i][1], dims[i][0], seed * 100003 + i, noise), quality=90,
                                   restart_marker_rows=1), n)
    return cells, np.arange(n, dtype=np.int64) % 1000


def raw_hwc(n: int, h: int = 1024, w: int = 1024, seed: int = 0) -> np.ndarray:
    """Config 5: raw uint8 HWC cells (seeded uniform)."""
    return np.random.RandomState(seed).randint(0, 256, size=(n, h, w, 3), dtype=np.uint8)


def raw_hwc_one(h: int, w: int, seed: int) -> np.ndarray:
    """One raw uint8 HWC cell (seeded uniform), for full-batch parity runs
    that build a large batch image by image."""
    return np.random.RandomState(seed).randint(0, 256, size=(h, w, 3), dtype=np.uint8)


def arrow_batch(cells: Sequence[bytes], labels) -> "pa.RecordBatch":
    import pyarrow as pa

    return pa.RecordBatch.from_arrays([pa.array(list(cells), type=pa.binary()),
                                       pa.array(np.asarray(labels, np.int64), type=pa.int64())],
                                      names=["image", "label"])
