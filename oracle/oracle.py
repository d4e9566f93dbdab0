"""TEST INFRASTRUCTURE ONLY — the CPU oracle for the batch-decode hot path.

Imported only by ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg, and only as the CHECKER / CPU baseline. The product
package (``lance-distributed-training_amd/ldt_amd``) never imports this module.

Contents
--------
* ctypes bindings to ``liborc.so`` (``jpeg_oracle.c``): a plain-C restatement
  of libjpeg-turbo 3.1.4.1's baseline decode (as Pillow 12.2.0 drives it),
  Pillow's BILINEAR ``Resample.c`` and torchvision's ``to_tensor``/``Normalize``.
  Reference call sites: ``lance_iterable.py:28-50``, ``lance_map_style.py:21-44``.
* ``pil_decode_tensor_image`` / ``pil_collate_fn``: the reference transform run
  through Pillow itself (torchvision is absent here, so its two PIL-path steps,
  ``F_pil.resize`` -> ``img.resize(size[::-1], BILINEAR)`` and ``to_tensor``, are
  restated in numpy/torch). This is the reference CPU path used as the timed
  baseline (``cpu_baseline.kind == "port"``).
* Sampler restatements (pure Python, small): ``ShardedBatchSampler`` per
  ``README.md:257-271``; ``ShardedFragmentSampler`` per ``README.md:140-155``
  plus this build's documented ``pad=True`` rule (parity unpinned: pylance's
  rule is not in the reference or this container — SURVEY.md §8c).
"""
from __future__ import annotations

import ctypes
import functools
import io
import math
import os
from typing import List, Sequence

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

MEAN = (0.485, 0.456, 0.406)  # lance_iterable.py:31 (commented-out Normalize)
STD = (0.229, 0.224, 0.225)


def build() -> str:
    """Compile liborc.so with gcc (no GPU needed)."""
    import subprocess

    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return os.path.join(_HERE, "liborc.so")


def lib() -> ctypes.CDLL:
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liborc.so")
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        f32p = ctypes.POINTER(ctypes.c_float)
        ip = ctypes.POINTER(ctypes.c_int)
        L.orc_jpeg_info.argtypes = [u8p, ctypes.c_size_t, ip, ip, ip]
        L.orc_decode_rgb.argtypes = [u8p, ctypes.c_size_t, u8p, ctypes.c_int]
        L.orc_decode_planes_out.argtypes = [u8p, ctypes.c_size_t, u8p, ctypes.c_long, ip]
        L.orc_resize_rgb.argtypes = [u8p, ctypes.c_int, ctypes.c_int, u8p, ctypes.c_int, ctypes.c_int]
        L.orc_to_tensor.argtypes = [u8p, ctypes.c_int, ctypes.c_int, f32p, f32p, f32p]
        L.orc_to_tensor.restype = None
        L.orc_jpeg_to_tensor.argtypes = [u8p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, f32p, f32p, f32p]
        L.orc_raw_to_tensor.argtypes = [u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, f32p, f32p, f32p]
        L.orc_resample_coeffs.argtypes = [ctypes.c_int, ctypes.c_int, ip, ctypes.POINTER(ctypes.c_int32), ctypes.c_int]
        _LIB = L
    return _LIB


def _u8(buf) -> "ctypes.POINTER(ctypes.c_uint8)":
    return ctypes.cast(ctypes.c_char_p(bytes(buf)) if isinstance(buf, (bytes, bytearray)) else buf,
                       ctypes.POINTER(ctypes.c_uint8))


def _ptr(a: np.ndarray, t=ctypes.c_uint8):
    return a.ctypes.data_as(ctypes.POINTER(t))


class OracleError(ValueError):
    pass


def jpeg_info(data: bytes):
    w, h, nc = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    a = np.frombuffer(data, np.uint8)
    rc = lib().orc_jpeg_info(_ptr(a), len(data), ctypes.byref(w), ctypes.byref(h), ctypes.byref(nc))
    if rc:
        raise OracleError(f"orc_jpeg_info rc={rc}")
    return w.value, h.value, nc.value


def decode_rgb(data: bytes) -> np.ndarray:
    """Image.open(BytesIO(data)).convert('RGB') as uint8 [H, W, 3]."""
    w, h, _ = jpeg_info(data)
    out = np.empty((h, w, 3), np.uint8)
    a = np.frombuffer(data, np.uint8)
    rc = lib().orc_decode_rgb(_ptr(a), len(data), _ptr(out), w * h)
    if rc:
        raise OracleError(f"orc_decode_rgb rc={rc}")
    return out


def resize_rgb(rgb: np.ndarray, oh: int = 224, ow: int = 224) -> np.ndarray:
    rgb = np.ascontiguousarray(rgb, np.uint8)
    h, w, _ = rgb.shape
    out = np.empty((oh, ow, 3), np.uint8)
    rc = lib().orc_resize_rgb(_ptr(rgb), w, h, _ptr(out), ow, oh)
    if rc:
        raise OracleError(f"orc_resize_rgb rc={rc}")
    return out


def resample_coeffs(in_size: int, out_size: int):
    cap = out_size * (2 * ((in_size + out_size - 1) // out_size) + 3) + 64
    bounds = np.zeros(2 * out_size, np.int32)
    kk = np.zeros(cap, np.int32)
    ks = lib().orc_resample_coeffs(in_size, out_size, _ptr(bounds, ctypes.c_int), _ptr(kk, ctypes.c_int32), cap)
    return ks, bounds.reshape(out_size, 2), kk[: ks * out_size].reshape(out_size, ks)


def _norm_ptrs(normalize):
    if not normalize:
        return None, None, None
    mean = np.asarray(normalize[0] if isinstance(normalize, tuple) else MEAN, np.float32)
    std = np.asarray(normalize[1] if isinstance(normalize, tuple) else STD, np.float32)
    return (mean, std), _ptr(mean, ctypes.c_float), _ptr(std, ctypes.c_float)


def jpeg_to_tensor(data: bytes, oh: int = 224, ow: int = 224, normalize=None) -> np.ndarray:
    """Oracle for one row of decode_tensor_image: float32 [3, oh, ow]."""
    keep, mp, sp = _norm_ptrs(normalize)
    out = np.empty((3, oh, ow), np.float32)
    a = np.frombuffer(data, np.uint8)
    rc = lib().orc_jpeg_to_tensor(_ptr(a), len(data), oh, ow, mp, sp, _ptr(out, ctypes.c_float))
    if rc:
        raise OracleError(f"orc_jpeg_to_tensor rc={rc}")
    return out


def raw_to_tensor(hwc: np.ndarray, oh: int = 224, ow: int = 224, normalize=None) -> np.ndarray:
    keep, mp, sp = _norm_ptrs(normalize)
    hwc = np.ascontiguousarray(hwc, np.uint8)
    h, w, _ = hwc.shape
    out = np.empty((3, oh, ow), np.float32)
    rc = lib().orc_raw_to_tensor(_ptr(hwc), h, w, oh, ow, mp, sp, _ptr(out, ctypes.c_float))
    if rc:
        raise OracleError(f"orc_raw_to_tensor rc={rc}")
    return out


def decode_batch(images: Sequence[bytes], labels: Sequence[int], normalize=None):
    """Oracle for decode_tensor_image / collate_fn on a whole batch (numpy)."""
    imgs = np.stack([jpeg_to_tensor(b, normalize=normalize) for b in images]) if len(images) else \
        np.zeros((0, 3, 224, 224), np.float32)
    return imgs, np.asarray(list(labels), dtype=np.int64)


# --------------------------------------------------------------------------
# The reference recipe through Pillow itself (lance_map_style.py:21-44).
# --------------------------------------------------------------------------

def pil_image_to_tensor(b: bytes, normalize=None) -> np.ndarray:
    from PIL import Image

    img = Image.open(io.BytesIO(b)).convert("RGB")          # lance_map_style.py:36
    img = img.resize((224, 224), Image.BILINEAR)            # transforms.Resize((224,224)) :30
    a = np.asarray(img, dtype=np.uint8)                     # to_tensor :31
    t = a.transpose(2, 0, 1).astype(np.float32) / np.float32(255)
    if normalize:
        m = np.asarray(MEAN, np.float32)[:, None, None]
        s = np.asarray(STD, np.float32)[:, None, None]
        t = (t - m) / s
    return t


def pil_collate_fn(batch_of_dicts):
    """The reference collate_fn (lance_map_style.py:21-44), torch output."""
    import torch

    images = [torch.from_numpy(pil_image_to_tensor(item["image"])) for item in batch_of_dicts]
    labels = [item["label"] for item in batch_of_dicts]
    return {"image": torch.stack(images), "label": torch.tensor(labels, dtype=torch.long)}


def pil_decode_tensor_image(batch, **kwargs):
    """The reference to_tensor_fn (lance_iterable.py:38-50), torch output."""
    return pil_collate_fn(batch.to_pylist())


# --------------------------------------------------------------------------
# Sampler index restatements.
# --------------------------------------------------------------------------

def sharded_batch_ranges(num_rows: int, batch_size: int, rank: int, world_size: int):
    """ShardedBatchSampler (README.md:257-271): batch k = [k*B, min(k*B+B, N)),
    rank r takes k = r, r+W, r+2W, ...  Returns list of (start, end)."""
    nb = (num_rows + batch_size - 1) // batch_size
    return [(k * batch_size, min(k * batch_size + batch_size, num_rows)) for k in range(rank, nb, world_size)]


def fragment_batches(fragment_rows: Sequence[int], batch_size: int):
    """All batches of a dataset read fragment by fragment (fragment.to_batches(B)):
    list of (fragment_id, start_in_fragment, end_in_fragment, global_start)."""
    out = []
    base = 0
    for f, n in enumerate(fragment_rows):
        s = 0
        while s < n:
            e = min(s + batch_size, n)
            out.append((f, s, e, base + s))
            s = e
        base += n
    return out


def sharded_fragment_batches(fragment_rows: Sequence[int], batch_size: int, rank: int,
                             world_size: int, pad: bool = False):
    """ShardedFragmentSampler (README.md:140-155): rank r reads fragments
    r, r+W, ...; batches never cross a fragment. With pad=True every rank yields
    max-over-ranks batches; this build's padding rule (documented in DESIGN.md,
    parity unpinned vs pylance): a short rank re-yields its own batches
    cyclically from its first one; a rank that owns no rows re-yields the
    global batch list cyclically starting at global batch index ``rank``.
    Returns list of (fragment_id, start, end, global_start, is_pad)."""
    own = []
    for f in range(rank, len(fragment_rows), world_size):
        for (ff, s, e, g) in fragment_batches(fragment_rows, batch_size):
            if ff == f:
                own.append((ff, s, e, g, 0))
    if not pad:
        return own
    counts = []
    for r in range(world_size):
        c = 0
        for f in range(r, len(fragment_rows), world_size):
            c += (fragment_rows[f] + batch_size - 1) // batch_size
        counts.append(c)
    target = max(counts) if counts else 0
    res = list(own)
    if len(own) == 0:
        allb = fragment_batches(fragment_rows, batch_size)
        if not allb:
            return res
        i = 0
        while len(res) < target:
            (ff, s, e, g) = allb[(rank + i) % len(allb)]
            res.append((ff, s, e, g, 1))
            i += 1
    else:
        i = 0
        while len(res) < target:
            (ff, s, e, g, _) = own[i % len(own)]
            res.append((ff, s, e, g, 1))
            i += 1
    return res


# ---------------------------------------------------------------------------
# Map-style DistributedSampler (lance_map_style.py:58 -> torch 2.10
# torch/utils/data/distributed.py:94-141). Pinned against torch itself in
# tests/test_oracle.py (torch.randperm / DistributedSampler are in-container).
# ---------------------------------------------------------------------------
def mt19937_u32(seed: int, count: int) -> np.ndarray:
    """MT19937 32-bit outputs (torch CPUGeneratorImpl::random(): the engine is
    seeded with the low 32 bits of the 64-bit seed). Vectorised twist."""
    N, M = 624, 397
    st = np.zeros(N, np.uint64)
    v = seed & 0xFFFFFFFF
    st[0] = v
    for j in range(1, N):
        v = (1812433253 * (v ^ (v >> 30)) + j) & 0xFFFFFFFF
        st[j] = v
    st = st.astype(np.uint32)
    out = np.empty(max(count, 0), np.uint32)
    pos = 0
    mag = np.array([0, 0x9908B0DF], np.uint32)
    while pos < count:
        new = np.empty(N, np.uint32)
        k = np.arange(N - M)
        y = (st[k] & 0x80000000) | (st[k + 1] & 0x7FFFFFFF)
        new[k] = st[k + M] ^ (y >> 1) ^ mag[y & 1]
        k = np.arange(N - M, 2 * (N - M))
        y = (st[k] & 0x80000000) | (st[k + 1] & 0x7FFFFFFF)
        new[k] = new[k - (N - M)] ^ (y >> 1) ^ mag[y & 1]
        k = np.arange(2 * (N - M), N)
        nxt = np.where(k + 1 < N, st[np.minimum(k + 1, N - 1)], new[0])
        y = (st[k] & 0x80000000) | (nxt & 0x7FFFFFFF)
        new[k] = new[k - (N - M)] ^ (y >> 1) ^ mag[y & 1]
        st = new
        y = st.copy()
        y ^= y >> 11
        y ^= (y << 7) & 0x9D2C5680
        y ^= (y << 15) & 0xEFC60000
        y ^= y >> 18
        take = min(N, count - pos)
        out[pos:pos + take] = y[:take]
        pos += take
    return out


@functools.lru_cache(maxsize=8)
def randperm(n: int, seed: int) -> np.ndarray:
    """torch.randperm(n, generator=manual_seed(seed)) for n < 2^32/20: forward
    Fisher-Yates, z = mt() % (n - i), swap(r[i], r[i + z]) (ATen randperm_cpu)."""
    r = np.arange(n, dtype=np.int64)
    z = mt19937_u32(seed, n - 1).astype(np.int64)
    for i in range(n - 1):
        k = i + int(z[i] % (n - i))
        r[i], r[k] = r[k], r[i]
    r.setflags(write=False)
    return r


def distributed_num_samples(n: int, num_replicas: int, drop_last: bool) -> int:
    """distributed.py:94-102."""
    if drop_last and n % num_replicas != 0:
        return max(0, math.ceil((n - num_replicas) / num_replicas))
    return math.ceil(n / num_replicas)


def distributed_indices(n: int, num_replicas: int, rank: int, shuffle: bool = True,
                        seed: int = 0, epoch: int = 0, drop_last: bool = False) -> List[int]:
    """DistributedSampler.__iter__ (distributed.py:107-141)."""
    base = randperm(n, (seed + epoch) % (1 << 64)) if shuffle else np.arange(n, dtype=np.int64)
    ns = distributed_num_samples(n, num_replicas, drop_last)
    total = ns * num_replicas
    if total == 0:
        return []
    p = (rank + np.arange(ns, dtype=np.int64) * num_replicas) % n
    return base[p].tolist()
