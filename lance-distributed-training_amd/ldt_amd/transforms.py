"""Drop-in replacements for the reference's batch transforms.

* ``decode_tensor_image(batch, **kwargs)`` — the iterable ``to_tensor_fn``
  (reference ``lance_iterable.py:38-50``, registered with
  ``LanceDataset(..., to_tensor_fn=decode_tensor_image)`` at ``:53-59``).
* ``collate_fn(batch_of_dicts)`` — the map-style ``collate_fn``
  (reference ``lance_map_style.py:21-44``, passed to ``get_safe_loader`` at
  ``:60-69``).

Both return ``{"image": float32[N,3,224,224], "label": int64[N]}`` exactly
like the reference (PIL ``open -> convert("RGB") -> Resize((224,224)) ->
ToTensor -> stack``), bit-exact, except that the tensors are already on the
GPU (``cuda:{LOCAL_RANK}``), so the consumer's ``.to(device)``
(``lance_iterable.py:108-109``) is a no-op. All arithmetic runs in libldt.so's
gfx950 kernels; Python only hands over Arrow buffer addresses.

Inside a torch DataLoader worker (``num_workers > 0``: lance_map_style.py:60-69
with 8 spawn workers, lance_iterable.py:71-72 under ``--no_ddp``) the workers
never touch the GPU. There the plug-ins return a ``DeviceBatch``: the batch's
compressed cells packed into shared-memory tensors, which the DataLoader moves
to the main process. The GPU decode then runs in the main process — in the
DataLoader's pin-memory thread when ``pin_memory=True`` (so it overlaps the
training step), otherwise when the batch is first indexed. Decoded tensors are
``DeviceTensor``s, whose ``pin_memory()`` is the identity, so
``pin_memory=True`` also works when the collate runs in the main process.
"""
from __future__ import annotations

import ctypes
import os
from typing import Iterable, Optional, Sequence, Tuple

import numpy as np
import pyarrow as pa
import torch

from . import _lib
from ._lib import ImageDecodeError, Norm

IMAGENET_MEAN = (0.485, 0.456, 0.406)  # lance_iterable.py:31 (commented out there)
IMAGENET_STD = (0.229, 0.224, 0.225)

_OUT = 224


def default_device() -> torch.device:
    """cuda:{LOCAL_RANK} as the reference training loop picks (lance_iterable.py:83)."""
    if not torch.cuda.is_available():
        raise RuntimeError("ldt_amd needs a HIP device (MI355X); no CPU fallback exists")
    return torch.device("cuda", int(os.environ.get("LOCAL_RANK", torch.cuda.current_device())))


def _norm_struct(normalize) -> Optional[Norm]:
    if not normalize:
        return None
    if normalize is True:
        mean, std = IMAGENET_MEAN, IMAGENET_STD
    else:
        mean, std = normalize
    n = Norm()
    for c in range(3):
        n.mean[c] = float(mean[c])
        n.std[c] = float(std[c])
    return n


def _column(batch, name: str):
    if isinstance(batch, pa.RecordBatch):
        return batch.column(batch.schema.get_field_index(name))
    if isinstance(batch, pa.Table):
        col = batch.column(name)
        return col.combine_chunks() if col.num_chunks != 1 else col.chunk(0)
    raise TypeError(f"expected pyarrow.RecordBatch, got {type(batch).__name__}")


def _labels_buffer(batch, label_column: str):
    """(address, offset, keepalive) of an int64 label column, or None."""
    if label_column is None:
        return None
    names = batch.schema.names
    if label_column not in names:
        return None
    lab = _column(batch, label_column)
    if lab.null_count:
        raise ValueError(f"null values in label column {label_column!r}")
    if lab.type != pa.int64():
        lab = lab.cast(pa.int64())
    bufs = lab.buffers()
    return bufs[1].address, lab.offset, lab


class _Decoder:
    def __init__(self, device: torch.device):
        self.device = device
        self.ctx = _lib.get_context(device.index)


_decoders: dict = {}


def _decoder(device) -> _Decoder:
    dev = torch.device(device) if device is not None else default_device()
    if dev.type != "cuda":
        raise ValueError(f"ldt_amd decodes on a HIP device, got {dev}")
    if dev.index is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    d = _decoders.get(dev.index)
    if d is None:
        d = _Decoder(dev)
        _decoders[dev.index] = d
    return d


def decode_arrow(images: pa.Array, labels=None, *, device=None, normalize=None,
                 stream: Optional[torch.cuda.Stream] = None, ctx=None, out=None, out_lbl=None):
    """Decode an Arrow ``binary``/``large_binary`` array of JPEG cells.

    ``labels``: optional (address, offset, keepalive) as from ``_labels_buffer``
    or an int64 sequence. ``ctx``: a libldt context (default: the device's
    shared one). Returns (image float32[N,3,224,224], label int64[N] or None).
    The host cells are only borrowed for the call (copied into the context's
    pinned ring, then sent to HBM on ``stream``).
    """
    if isinstance(images, pa.ChunkedArray):
        images = images.combine_chunks()
    dec = _decoder(device)
    ctx = ctx or dec.ctx
    n = len(images)
    if out is None:
        out = torch.empty((n, 3, _OUT, _OUT), dtype=torch.float32, device=dec.device)
    lbl_keep = None
    if labels is not None and not isinstance(labels, tuple):
        arr = np.ascontiguousarray(np.asarray(labels, dtype=np.int64))
        lbl_keep = arr
        labels = (arr.ctypes.data, 0, arr)
    if labels is not None and out_lbl is None:
        out_lbl = torch.empty((n,), dtype=torch.int64, device=dec.device)
    elif labels is None:
        out_lbl = None
    if n == 0:
        return out, out_lbl
    t = images.type
    if t == pa.binary() or t == pa.string():
        fn = ctx.lib.ldt_decode_batch
    elif t == pa.large_binary() or t == pa.large_string():
        fn = ctx.lib.ldt_decode_batch_large
    else:
        raise TypeError(f"image column must be binary or large_binary, got {t}")
    bufs = images.buffers()
    validity = bufs[0].address if (bufs[0] is not None and images.null_count) else None
    offsets, data = bufs[1], bufs[2]
    data_addr = data.address if data is not None else None
    if data_addr is None:
        # all-empty cells: give the library a valid pointer
        lbl_dummy = np.zeros(8, np.uint8)
        data_addr = lbl_dummy.ctypes.data
    status = np.zeros(n, np.int32)
    norm = _norm_struct(normalize)
    s = stream if stream is not None else torch.cuda.current_stream(dec.device)
    with ctx.lock:
        rc = fn(ctx.handle, data_addr, offsets.address, images.offset, n, validity,
                labels[0] if labels is not None else None,
                labels[1] if labels is not None else 0,
                out.data_ptr(), out_lbl.data_ptr() if out_lbl is not None else None,
                ctypes.byref(norm) if norm is not None else None,
                s.cuda_stream, status.ctypes.data)
    del lbl_keep
    if rc == _lib.LDT_ERR_IMAGE:
        bad = {int(i): int(status[i]) for i in np.nonzero(status)[0]}
        raise ImageDecodeError(bad)
    ctx.check(rc, "ldt_decode_batch")
    return out, out_lbl


class DeviceTensor(torch.Tensor):
    """A decoded batch tensor on the GPU. Behaves as a plain ``torch.Tensor``
    (ops on it return plain tensors); its ``pin_memory()`` returns itself, so
    a DataLoader with ``pin_memory=True`` (lance_map_style.py:67) passes the
    device tensors through instead of failing to pin them (torch pins dense
    CPU tensors only)."""

    __torch_function__ = torch._C._disabled_torch_function_impl

    def pin_memory(self, device=None):
        return self


def _as_device_batch(img: torch.Tensor, lbl: Optional[torch.Tensor]) -> dict:
    out = {"image": img.as_subclass(DeviceTensor)}
    if lbl is not None:
        out["label"] = lbl.as_subclass(DeviceTensor)
    return out


def _in_worker() -> bool:
    """True inside a torch DataLoader worker process."""
    return torch.utils.data.get_worker_info() is not None


def _shm_uint8(nbytes: int) -> torch.Tensor:
    t = torch.empty((nbytes,), dtype=torch.uint8)
    t.share_memory_()  # the DataLoader then sends a handle, not the bytes
    return t


def _pack_list(images: Sequence, labels) -> dict:
    """Worker side: a list of JPEG ``bytes`` (None = null cell) packed into one
    shared-memory byte tensor + int64 offsets (one copy per cell)."""
    n = len(images)
    lens = np.fromiter((0 if b is None else len(b) for b in images), dtype=np.int64, count=n)
    offs = np.zeros(n + 1, np.int64)
    np.cumsum(lens, out=offs[1:])
    data = _shm_uint8(int(offs[-1]))
    buf = data.numpy()
    for i, b in enumerate(images):
        if b:
            buf[offs[i]:offs[i + 1]] = np.frombuffer(b, dtype=np.uint8)
    packed = {"offsets": torch.from_numpy(offs), "data": data}
    if any(b is None for b in images):
        packed["valid"] = torch.from_numpy(np.fromiter((b is not None for b in images), dtype=np.bool_, count=n))
    if labels is not None:
        packed["label"] = torch.from_numpy(np.ascontiguousarray(np.asarray(labels, dtype=np.int64)))
    return packed


def _pack_arrow(images: pa.Array, labels) -> dict:
    """Worker side: an Arrow ``binary``/``large_binary`` column (any offset)
    packed like ``_pack_list`` with one memcpy of its data range."""
    if isinstance(images, pa.ChunkedArray):
        images = images.combine_chunks()
    n = len(images)
    bufs = images.buffers()
    odt = np.int64 if pa.types.is_large_binary(images.type) or pa.types.is_large_string(images.type) else np.int32
    offs = np.frombuffer(bufs[1], dtype=odt, count=n + 1, offset=images.offset * np.dtype(odt).itemsize)
    offs = offs.astype(np.int64)
    lo, hi = int(offs[0]), int(offs[-1])
    data = _shm_uint8(hi - lo)
    if hi > lo:
        data.numpy()[:] = np.frombuffer(bufs[2], dtype=np.uint8, count=hi - lo, offset=lo)
    packed = {"offsets": torch.from_numpy(offs - lo), "data": data}
    if images.null_count:
        packed["valid"] = torch.from_numpy(np.asarray(images.is_valid().to_numpy(zero_copy_only=False), np.bool_))
    if labels is not None:
        packed["label"] = torch.from_numpy(np.ascontiguousarray(labels, dtype=np.int64))
    return packed


def _unpack(packed: dict) -> Tuple[pa.Array, Optional[np.ndarray]]:
    """Main-process side: a ``large_binary`` Arrow array over the shared
    tensors (no copy) and the labels."""
    offs = packed["offsets"].numpy()
    n = len(offs) - 1
    valid = None
    if "valid" in packed:
        valid = pa.array(packed["valid"].numpy()).buffers()[1]
    data = packed["data"].numpy()
    arr = pa.Array.from_buffers(pa.large_binary(), n, [valid, pa.py_buffer(offs), pa.py_buffer(data)])
    lab = packed["label"].numpy() if "label" in packed else None
    return arr, lab


class DeviceBatch:
    """What ``collate_fn`` / ``decode_tensor_image`` return inside a DataLoader
    worker: the batch's compressed cells in shared memory, decoded on the GPU
    in the main process on first use.

    Indexing (``batch["image"]``, ``batch["label"]``), ``keys()``/``items()``
    and ``pin_memory()`` trigger the decode; ``pin_memory()`` — called by the
    DataLoader's pin-memory thread when ``pin_memory=True`` — returns the plain
    ``{"image", "label"}`` dict. Deliberately not a ``Mapping``: torch's
    ``pin_memory`` would otherwise pin the values one by one instead of calling
    ``pin_memory()`` on the batch. Decode errors raise ``ImageDecodeError``
    where the decode runs (re-raised in the main thread by the DataLoader when
    it runs in the pin-memory thread)."""

    __slots__ = ("_packed", "_device", "_normalize", "_out")

    def __init__(self, packed: dict, device=None, normalize=None):
        self._packed = packed
        self._device = None if device is None else str(device)
        self._normalize = normalize
        self._out = None

    def decode(self) -> dict:
        if self._out is None:
            arr, lab = _unpack(self._packed)
            img, lbl = decode_arrow(arr, lab, device=self._device, normalize=self._normalize)
            self._out = _as_device_batch(img, lbl)
            self._packed = None
        return self._out

    def pin_memory(self, device=None) -> dict:
        return self.decode()

    def __getitem__(self, key):
        return self.decode()[key]

    def __contains__(self, key) -> bool:
        return key in self.decode()

    def __iter__(self):
        return iter(self.decode())

    def __len__(self) -> int:
        return len(self.decode())

    def keys(self):
        return self.decode().keys()

    def values(self):
        return self.decode().values()

    def items(self):
        return self.decode().items()

    def get(self, key, default=None):
        return self.decode().get(key, default)

    def __repr__(self) -> str:
        state = "decoded" if self._out is not None else f"{len(self._packed['offsets']) - 1} cells pending"
        return f"DeviceBatch({state})"


def decode_tensor_image(batch, **kwargs):
    """to_tensor_fn: ``pa.RecordBatch`` -> ``{"image", "label"}`` (lance_iterable.py:38-50).

    Unknown keyword arguments from LanceDataset are accepted and ignored, as
    the reference's ``**kwargs`` does. Optional keywords of this build:
    ``image_column`` ("image"), ``label_column`` ("label"), ``device``,
    ``normalize`` (False; True = ImageNet mean/std, lance_iterable.py:31).
    In a DataLoader worker it returns a ``DeviceBatch`` (decoded in the main
    process).
    """
    image_column = kwargs.get("image_column", "image")
    label_column = kwargs.get("label_column", "label")
    images = _column(batch, image_column)
    if _in_worker():
        labels = None
        if label_column is not None and label_column in batch.schema.names:
            lab = _column(batch, label_column)
            if lab.null_count:
                raise ValueError(f"null values in label column {label_column!r}")
            labels = lab.to_numpy(zero_copy_only=False)
        return DeviceBatch(_pack_arrow(images, labels), kwargs.get("device"), kwargs.get("normalize"))
    lab = _labels_buffer(batch, label_column)
    img, lbl = decode_arrow(images, lab, device=kwargs.get("device"),
                            normalize=kwargs.get("normalize"), stream=kwargs.get("stream"))
    return _as_device_batch(img, lbl)


def collate_fn(batch_of_dicts, *, device=None, normalize=None):
    """collate_fn: list of ``{"image": bytes, "label": int}`` -> stacked tensors
    (lance_map_style.py:21-44). The bytes are packed into one buffer (zero-copy
    of the Python ``bytes`` objects is impossible; this is the one host copy)
    and decoded on the GPU — in a DataLoader worker, packed into shared memory
    and returned as a ``DeviceBatch`` for the main process to decode. A
    ``pa.RecordBatch`` is accepted too."""
    if isinstance(batch_of_dicts, pa.RecordBatch):
        return decode_tensor_image(batch_of_dicts, device=device, normalize=normalize)
    images = [item["image"] for item in batch_of_dicts]
    labels = [item["label"] for item in batch_of_dicts] if batch_of_dicts and "label" in batch_of_dicts[0] \
        else None
    if _in_worker():
        return DeviceBatch(_pack_list(images, labels), device, normalize)
    arr = pa.array(images, type=pa.binary())
    img, lbl = decode_arrow(arr, labels, device=device, normalize=normalize)
    return _as_device_batch(img, lbl)


def make_collate_fn(device=None, normalize=None):
    """A picklable collate_fn bound to a device / Normalize setting (for
    ``DataLoader(collate_fn=...)`` with spawn workers)."""
    return _BoundCollate(device, normalize)


class _BoundCollate:
    def __init__(self, device, normalize):
        self.device = None if device is None else str(device)
        self.normalize = normalize

    def __call__(self, batch_of_dicts):
        return collate_fn(batch_of_dicts, device=self.device, normalize=self.normalize)


def resize_raw(hwc, height: int, width: int, *, device=None, normalize=True):
    """Config 5: raw uint8 HWC cells -> Resize(224,224) [+Normalize] -> float32[N,3,224,224].

    ``hwc`` is a uint8 torch tensor [N, H, W, 3] (host or device) or an Arrow
    ``binary`` / ``fixed_size_binary(H*W*3)`` array of cells."""
    dec = _decoder(device)
    ctx = dec.ctx
    keep = None
    if isinstance(hwc, torch.Tensor):
        if hwc.dtype != torch.uint8 or hwc.dim() != 4 or tuple(hwc.shape[1:]) != (height, width, 3):
            raise ValueError("expected uint8 [N, H, W, 3]")
        t = hwc.contiguous()
        keep = t
        n = t.shape[0]
        ptr, is_dev, stride = t.data_ptr(), 1 if t.is_cuda else 0, height * width * 3
    else:
        arr = hwc.combine_chunks() if isinstance(hwc, pa.ChunkedArray) else hwc
        n = len(arr)
        bufs = arr.buffers()
        cell = height * width * 3
        if pa.types.is_fixed_size_binary(arr.type):
            if arr.type.byte_width != cell:
                raise ValueError("fixed_size_binary width != H*W*3")
            ptr = bufs[1].address + arr.offset * cell
        else:
            offs = np.frombuffer(bufs[1], dtype=np.int64 if pa.types.is_large_binary(arr.type) else np.int32,
                                 count=len(arr) + 1 + arr.offset)[arr.offset:]
            if np.any(np.diff(offs) != cell):
                raise ValueError("every raw cell must be H*W*3 bytes")
            ptr = bufs[2].address + int(offs[0])
        is_dev, stride = 0, cell
        keep = arr
    out = torch.empty((n, 3, _OUT, _OUT), dtype=torch.float32, device=dec.device)
    if n == 0:
        return out
    norm = _norm_struct(normalize)
    s = torch.cuda.current_stream(dec.device)
    with ctx.lock:
        rc = ctx.lib.ldt_resize_raw(ctx.handle, ptr, is_dev, n, height, width, stride,
                                    out.data_ptr(), ctypes.byref(norm) if norm is not None else None,
                                    s.cuda_stream)
    ctx.check(rc, "ldt_resize_raw")
    del keep
    return out


def _parse_cpulist(s: str):
    out = set()
    for part in s.split(","):
        part = part.strip()
        if not part:
            continue
        a, _, b = part.partition("-")
        out.update(range(int(a), int(b or a) + 1))
    return out


def bind_numa(device=None):
    """Restrict the calling thread (and the threads and processes it starts
    later) to the CPUs local to `device`'s NUMA node, within its current
    affinity — `numactl --cpunodebind` for one rank. Host buffers the thread
    allocates afterwards (Arrow batches read in it) then land on the GPU's
    node by first touch, so the copy pool (bound there, ldt_host_info) reads
    them locally: from a remote node its copy runs at the inter-socket link's
    ~48 GB/s instead of ~170 GB/s. Returns the CPUs now allowed
    (unchanged if the GPU's local CPUs are unknown or outside the affinity)."""
    import os

    info = _decoder(device).ctx.host_info()
    cur = os.sched_getaffinity(0)
    local = _parse_cpulist(info.get("local_cpulist", "")) & cur
    if local and local != cur:
        os.sched_setaffinity(0, local)
        return local
    return cur


def _host_range(obj):
    """(address, size) of the host bytes behind a pa.Buffer, the data buffer of
    a binary/large_binary/fixed_size_binary pa.Array / ChunkedArray chunk, or
    a numpy array."""
    if isinstance(obj, pa.ChunkedArray):
        if obj.num_chunks != 1:
            raise ValueError("register one chunk at a time")
        obj = obj.chunk(0)
    if isinstance(obj, pa.Array):
        bufs = obj.buffers()
        obj = bufs[1] if pa.types.is_fixed_size_binary(obj.type) else bufs[2]
    if isinstance(obj, pa.Buffer):
        return obj.address, obj.size
    if isinstance(obj, np.ndarray):
        return obj.ctypes.data, obj.nbytes
    raise TypeError(f"cannot register {type(obj).__name__}")


_registered: dict = {}


def register_host(obj, device=None):
    """Page-lock the host bytes of `obj` in place (ldt_register_host), so that
    every later decode of cells inside them copies to HBM by DMA without the
    memcpy into the pinned ring: for a memory-mapped Arrow IPC / Lance
    fragment, register the `image` column's data buffer once. The bytes must
    stay alive until unregister_host(obj). Returns the registered (address,
    size)."""
    addr, size = _host_range(obj)
    if size == 0 or addr in _registered:
        return addr, size
    dec = _decoder(device)
    dec.ctx.check(dec.ctx.lib.ldt_register_host(dec.ctx.handle, addr, size), "ldt_register_host")
    _registered[addr] = (size, obj, dec)  # keeps `obj` alive while registered
    return addr, size


def unregister_host(obj):
    """Undo register_host (waits for the device first)."""
    addr, _ = _host_range(obj)
    ent = _registered.pop(addr, None)
    if ent is None:
        return
    dec = ent[2]
    dec.ctx.check(dec.ctx.lib.ldt_unregister_host(dec.ctx.handle, addr), "ldt_unregister_host")


class ResidentBatch:
    """A batch of JPEG cells staged once into HBM (bench / pre-staged loaders).

    ``decode()`` runs the full decode path with the compressed bytes already
    resident, so a timed loop measures the GPU path, not PCIe."""

    def __init__(self, cells: Sequence[bytes], labels: Iterable[int] | None = None, *, device=None):
        dec = _decoder(device)
        self.dec = dec
        self.n = len(cells)
        lens = np.fromiter((len(c) for c in cells), dtype=np.int64, count=self.n)
        self.offsets = np.zeros(self.n + 1, np.int64)
        np.cumsum(lens, out=self.offsets[1:])
        self.host = np.frombuffer(b"".join(cells), dtype=np.uint8).copy() if self.n else np.zeros(1, np.uint8)
        self.dev = torch.from_numpy(self.host).to(dec.device)
        self.labels = None if labels is None else np.ascontiguousarray(np.asarray(list(labels), np.int64))
        self.bytes = int(self.offsets[-1])

    def decode(self, out=None, out_lbl=None, normalize=None, *, ctx=None, stream=None):
        """Decode on `stream` (default: the current stream) with context `ctx`
        (default: the device's shared context)."""
        ctx = ctx or self.dec.ctx
        s = stream or torch.cuda.current_stream(self.dec.device)
        if out is None:
            out = torch.empty((self.n, 3, _OUT, _OUT), dtype=torch.float32, device=self.dec.device)
        if self.labels is not None and out_lbl is None:
            out_lbl = torch.empty((self.n,), dtype=torch.int64, device=self.dec.device)
        status = np.zeros(self.n, np.int32)
        norm = _norm_struct(normalize)
        rc = ctx.lib.ldt_decode_batch_resident(
            ctx.handle, self.host.ctypes.data, self.dev.data_ptr(), self.offsets.ctypes.data, self.n,
            self.labels.ctypes.data if self.labels is not None else None,
            out.data_ptr(), out_lbl.data_ptr() if out_lbl is not None else None,
            ctypes.byref(norm) if norm is not None else None, s.cuda_stream, status.ctypes.data)
        if rc == _lib.LDT_ERR_IMAGE:
            raise ImageDecodeError({int(i): int(status[i]) for i in np.nonzero(status)[0]})
        ctx.check(rc, "ldt_decode_batch_resident")
        return out, out_lbl


def slot_streams(depth: int, queues: int, env: Optional[str] = None) -> Tuple[int, bool]:
    """DecodePipeline's stream plan for ``depth`` slots on a process with
    ``queues`` HIP hardware queues per priority (GPU_MAX_HW_QUEUES): returns
    (slots on high-priority streams, cells' DMA on the slots' own streams).

    Normal priority while the slots and the consumer's stream fit the queues;
    deeper pipelines put up to ``queues`` slots on high-priority streams (their
    own queues) and the rest beside the consumer. The copy stream needs a
    normal queue of its own beside normal slots, and beside high-priority slots
    it measured slower when normal slots share the pool too (c2p depth 6: host
    input 35k vs 50k at depth 7 with the DMA on the slots' streams).
    ``env`` (LDT_SLOT_PRIORITY) "0"/"1" forces every slot's priority."""
    if env is not None:
        n_high = depth if int(env) else 0
    else:
        n_high = 0 if depth + 1 <= queues else min(depth, queues)
    n_normal = depth - n_high
    slot_dma = (n_normal + 2 > queues or n_high > 0) if n_normal else (n_high > queues)
    return n_high, slot_dma


# Batches in flight for progressive (SOF2) datasets: make_to_tensor_fn(depth=
# PROGRESSIVE_DEPTH). A c2p batch spends ~13 ms in k_prog, so several must be
# in flight. At 5 (4 slots on high-priority streams, 1 beside the consumer) the
# rate is the same in a clean process and in a DDP process in the reference's
# order (62k img/s both); at 7 the clean rate is 5% higher but the DDP order
# costs 23% (three normal-priority slots share queues with the comm and
# consumer streams, whose per-step waits then block them). DESIGN.md §6.
PROGRESSIVE_DEPTH = 5

_slot_stream_sets: dict = {}  # (device index, priority) -> [torch.cuda.Stream]


def _slot_stream(dev, priority: int, i: int):
    """The device's process-wide slot stream i of `priority` (0 normal, -1
    high), created on first request: DecodePipelines share them (a process's
    pipelines decode one after another; two used at once serialise on the
    shared slots, still in order)."""
    lst = _slot_stream_sets.setdefault((dev.index, priority), [])
    while len(lst) <= i:
        lst.append(torch.cuda.Stream(dev, priority=priority))
    return lst[i]


class DecodePipeline:
    """`depth` batches in flight: each slot owns a libldt context (its own HBM
    workspace and pinned staging ring) and a HIP stream. ``decode(batch)``
    enqueues on the next slot's stream without waiting for the caller's stream
    and makes the caller's current stream wait for the result, so the
    latency-bound Huffman stages of one batch overlap the resize/IDCT of the
    previous one — the GPU-side analogue of the reference DataLoader's
    prefetching workers (lance_map_style.py:137, num_workers=8).

    ``adaptive=True`` (``depth`` 3, what ``make_to_tensor_fn()`` builds):
    the batches in flight follow each call's batch size, with the process's
    four hardware queues held by the consumer's stream and the three slot
    streams throughout. A host batch of at least 8 MB of encoded cells takes
    slots 0 and 1 in turn with its DMA on slot 2's stream (two in flight, the
    transfer overlapping the previous batches' kernels); smaller batches and
    resident ones rotate over all three slots with the DMA on the slot's own
    stream (three in flight: a batch of 128 small images does not fill the
    GPU). DESIGN.md §7a.

    Errors are asynchronous: every decode gets its context's ticket
    (ldt_last_ticket), and ``check()`` waits for every unchecked batch and
    raises ImageDecodeError with its failing rows (per-image status, as
    ldt_fetch_status_ticket reports). ``check_slot(i)`` checks slot i's
    batches older than its most recent one — a batch two uses of the slot ago,
    long finished — so checking before each reuse never waits for the batch
    just enqueued."""

    def __init__(self, depth: int = 2, device=None, profile: bool = False, adaptive: bool = False):
        from collections import deque

        self.dec = _decoder(device)
        self.depth = 3 if adaptive else max(1, int(depth))
        self.adaptive = bool(adaptive)
        self.ctxs = [_lib.Context(self.dec.device.index) for _ in range(self.depth)]
        for c in self.ctxs:
            c.set_option(_lib.OPT_SYNC_STATUS, 0)
            if profile:
                c.set_option(_lib.OPT_PROFILE, 1)
        # the cells' DMA of host batches goes on the device's copy stream when
        # the process has a hardware queue for it beside the slots' streams and
        # the consumer's (otherwise two streams would share a queue and the
        # slots' kernels serialise): else on the slot's own stream
        # slot streams: normal priority while the slots and the consumer's
        # stream fit the process's hardware queues (GPU_MAX_HW_QUEUES, 4 by
        # default); deeper pipelines (progressive batches take ~15 ms each, so
        # they want 4 in flight) take high-priority streams, which ROCm serves
        # from their own set of queues, so no slot shares a queue with the
        # consumer's stream (a shared queue serialises the slots: measured
        # c2p depth 4: 26k img/s on normal streams vs 44k). LDT_SLOT_PRIORITY
        # = 0 / 1 forces either.
        n_high, slot_dma = slot_streams(self.depth, _lib.hw_queues(), os.environ.get("LDT_SLOT_PRIORITY"))
        if self.adaptive:
            env = os.environ.get("LDT_SLOT_PRIORITY")
            n_high, slot_dma = (self.depth if env is not None and int(env) else 0), True
        self.high_priority = n_high > 0
        if slot_dma:
            for c in self.ctxs:
                c.set_option(_lib.OPT_COPY_MODE, 1)
        # the slot streams are taken at the first decode (see _streams_now)
        self._n_high = n_high
        self._streams = None
        self._copy_mode = [1 if slot_dma else 0] * self.depth
        self._k_large = self._k_small = 0
        self.pending = [deque() for _ in range(self.depth)]  # per slot: (ticket, n), oldest first
        self.last_ticket = None  # (slot, ticket) of the most recent decode
        self.k = 0

    @property
    def streams(self):
        """The slots' HIP streams (taken at the first decode)."""
        return self._streams_now()

    def _streams_now(self):
        """Slot i's stream is the device's process-wide slot stream i of its
        priority (_slot_stream), taken at the first decode rather than at
        construction. The HIP runtime maps a process's streams onto
        GPU_MAX_HW_QUEUES hardware queues per priority in the order they
        come to it, and a slot whose queue also carries a stream the process
        made afterwards lost up to 30% (tools/probes/stream_env.py, DESIGN.md
        §6): pipelines built before a DDP process group and model (the
        reference's order, lance_iterable.py:78-95) run their first batch
        after them, and every pipeline of the process shares the same few
        slot streams instead of adding new ones that the runtime would place
        on the queues of the live pipeline's slots."""
        if self._streams is None:
            st = [_slot_stream(self.dec.device, -1, i) if i < self._n_high
                  else _slot_stream(self.dec.device, 0, i - self._n_high) for i in range(self.depth)]
            self._streams = st
            # adaptive: slots 0 and 1 DMA large batches on slot 2's stream
            if self.adaptive:
                for c in self.ctxs[:2]:
                    c.set_copy_stream(st[2])
        return self._streams

    def decode(self, batch, normalize=None, image_column: str = "image", label_column: str = "label",
               wait: bool = True):
        """Enqueue one batch: a ``ResidentBatch`` (cells already in HBM) or a
        host ``pa.RecordBatch`` as LanceDataset yields it (its buffers are
        copied into the slot's pinned ring during the call, then to HBM
        asynchronously on the slot's stream).

        ``wait=True``: torch's current stream waits for the result now;
        returns ``(image, label)``. ``wait=False``: nothing waits yet; returns
        ``(image, label, ready)`` and the consumer calls ``ready()`` on the
        stream that will use the tensors, so work enqueued there in between
        (a training step) overlaps this decode (see ``prefetch``)."""
        if self.adaptive:
            large = not isinstance(batch, ResidentBatch) and \
                auto_host_depth(_cell_bytes(batch, image_column)) == 2
            if large:
                slot = self._k_large % 2
                self._k_large += 1
            else:
                slot = self._k_small % 3
                self._k_small += 1
            mode = 0 if large else 1
            if self._copy_mode[slot] != mode:
                self.ctxs[slot].set_option(_lib.OPT_COPY_MODE, mode)
                self._copy_mode[slot] = mode
        else:
            slot = self.k % self.depth
        # the slot's context holds the status of its last two calls: check the
        # older one before this call replaces it (it finished long ago)
        self.check_slot(slot)
        self.k += 1
        s = self.streams[slot]
        cur = torch.cuda.current_stream(self.dec.device)
        if isinstance(batch, ResidentBatch):
            n, has_lbl = batch.n, batch.labels is not None
        else:
            images = _column(batch, image_column)
            lab = _labels_buffer(batch, label_column)
            n, has_lbl = len(images), lab is not None
        with torch.cuda.stream(s):
            out = torch.empty((n, 3, _OUT, _OUT), dtype=torch.float32, device=self.dec.device)
            lbl = torch.empty((n,), dtype=torch.int64, device=self.dec.device) if has_lbl else None
        ctx = self.ctxs[slot]
        before = ctx.lib.ldt_last_ticket(ctx.handle)
        if isinstance(batch, ResidentBatch):
            batch.decode(out, lbl, normalize, ctx=ctx, stream=s)
        else:
            decode_arrow(images, lab, device=self.dec.device, normalize=normalize, stream=s,
                         ctx=ctx, out=out, out_lbl=lbl)
        t = ctx.lib.ldt_last_ticket(ctx.handle)
        self.last_ticket = (slot, t) if t != before else None
        if t != before:
            self.pending[slot].append((t, n))
        if wait:
            cur.wait_stream(s)
            out.record_stream(cur)
            if lbl is not None:
                lbl.record_stream(cur)
            return out, lbl
        ev = torch.cuda.Event()
        ev.record(s)

        def ready():
            use = torch.cuda.current_stream(self.dec.device)
            use.wait_event(ev)
            out.record_stream(use)
            if lbl is not None:
                lbl.record_stream(use)

        return out, lbl, ready

    def prefetch(self, batches, ahead: int = 2, normalize=None, image_column: str = "image",
                 label_column: str = "label"):
        """Iterate ``batches`` (host RecordBatches or ResidentBatches) yielding
        ``{"image", "label"}`` dicts, with the decode of the next ``ahead``
        batches enqueued before each yield: while the consumer's step k runs on
        torch's stream, batches k+1..k+ahead decode on the slots' streams
        (decode overlapped with the training step, so
        ``.to(device)`` at lance_iterable.py:108-109 is a no-op). A batch's
        per-image status is checked before it is yielded: ImageDecodeError is
        raised instead of yielding a batch with a failed row."""
        from collections import deque

        ahead = max(0, min(int(ahead), self.depth - 1))
        q = deque()

        def emit():
            img, lbl, ready, tk = q.popleft()
            # the batch itself is checked before it is yielded, so a bad row
            # raises here (as PIL would) instead of reaching the consumer; it
            # waits only for this batch, enqueued `ahead` batches ago
            if tk is not None:
                self.check_ticket(*tk)
            ready()
            return _as_device_batch(img, lbl)

        for b in batches:
            q.append(self.decode(b, normalize=normalize, image_column=image_column,
                                 label_column=label_column, wait=False) + (self.last_ticket,))
            if len(q) > ahead:
                yield emit()
        while q:
            yield emit()
        self.check()

    def stage_times(self, reset: bool = False):
        tot: dict = {}
        for c in self.ctxs:
            for k, (ms, n) in c.stage_times(reset=reset).items():
                a = tot.get(k, (0.0, 0))
                tot[k] = (a[0] + ms, a[1] + n)
        return tot

    def host_times(self, reset: bool = False):
        """Host phase times summed over the slots' contexts (LDT_OPT_HOST_TIMING)."""
        tot: dict = {}
        calls = 0
        for c in self.ctxs:
            us, n = c.host_times(reset=reset)
            calls += n
            for k, v in us.items():
                tot[k] = tot.get(k, 0.0) + v
        return tot, calls

    def set_option(self, opt: int, value: int):
        for c in self.ctxs:
            c.set_option(opt, value)

    def _ticket_status(self, i: int, ticket: int, n: int) -> dict:
        c = self.ctxs[i]
        st = np.zeros(n, np.int32)
        rc = c.lib.ldt_fetch_status_ticket(c.handle, ticket, st.ctypes.data, n)
        if rc != _lib.LDT_ERR_IMAGE:
            c.check(rc, "ldt_fetch_status_ticket")
        return {int(j): int(st[j]) for j in np.nonzero(st)[0]}

    def check_ticket(self, i: int, ticket: int):
        """Wait for slot i's batch `ticket` (if still unchecked); raise
        ImageDecodeError on failures."""
        p = self.pending[i]
        for j, (t, n) in enumerate(p):
            if t == ticket:
                del p[j]
                bad = self._ticket_status(i, t, n)
                if bad:
                    raise ImageDecodeError(bad)
                return

    def check_slot(self, i: int):
        """Check slot i's batches older than its most recent one (they finished
        long ago: the slot's context has been used since); raise
        ImageDecodeError on failures. Called before the slot is reused, so the
        context's two held statuses are never overwritten unchecked."""
        p = self.pending[i]
        while len(p) > 1:
            t, n = p.popleft()
            bad = self._ticket_status(i, t, n)
            if bad:
                raise ImageDecodeError(bad)

    def check(self):
        """Wait for every unchecked batch; raise ImageDecodeError with the
        failing rows of all of them."""
        bad = {}
        for i in range(self.depth):
            p = self.pending[i]
            while p:
                t, n = p.popleft()
                bad.update(self._ticket_status(i, t, n))
        if bad:
            raise ImageDecodeError(bad)


# make_to_tensor_fn(depth=None): batches with fewer cell bytes than this run 3
# deep (DMA on the slot streams), larger ones 2 deep beside the copy stream
# (profiles/r4/host_depth_ab_r4hd.txt: 3.3 MB batches of 128 +10% at depth 3,
# 17 MB batches of 256 steady only at depth 2)
AUTO_DEPTH_SMALL_BYTES = 8 << 20


def auto_host_depth(cell_bytes: int) -> int:
    """Batches in flight that make_to_tensor_fn(depth=None) (an adaptive
    DecodePipeline) runs a host batch of `cell_bytes` bytes of encoded cells
    at: 2 (its DMA on a stream of its own) from AUTO_DEPTH_SMALL_BYTES on, 3
    below."""
    return 3 if 0 < cell_bytes < AUTO_DEPTH_SMALL_BYTES else 2


def _cell_bytes(batch, col: str) -> int:
    """Encoded bytes of a host RecordBatch's image cells (0 if unknown)."""
    try:
        if col not in batch.schema.names:
            return 0
        col_ = batch.column(col)  # a Table's column stays chunked here
        # a chunked column: the chunks' byte spans summed (no combine_chunks copy)
        chunks = col_.chunks if isinstance(col_, pa.ChunkedArray) else [col_]
        tot = 0
        for arr in chunks:
            if pa.types.is_fixed_size_binary(arr.type):
                tot += len(arr) * arr.type.byte_width
                continue
            if len(arr) == 0:
                continue
            dt = np.int64 if pa.types.is_large_binary(arr.type) else np.int32
            o = np.frombuffer(arr.buffers()[1], dtype=dt)
            tot += int(o[arr.offset + len(arr)] - o[arr.offset])
        return tot
    except Exception:  # not a host binary column: keep the default
        return 0


def make_to_tensor_fn(depth: Optional[int] = None, device=None, normalize=None, prefetch: int = 0,
                      register: bool = False, register_cap: int = 8, **fixed):
    """A pipelined ``to_tensor_fn`` for ``LanceDataset(..., to_tensor_fn=...)``
    (lance_iterable.py:53-59): each call enqueues its RecordBatch on one of
    `depth` contexts/streams and returns at once, so batch k+1's host copy and
    kernels overlap batch k's. The tensors are ready on torch's current stream
    (it waits for the slot's stream). Per-image errors are reported
    asynchronously: by ``fn.check()``, and at the latest when the slot is
    reused a second time (2 * `depth` calls later, when that batch finished
    long ago, so the check never stalls the host) — unlike the synchronous
    ``decode_tensor_image``.

    ``depth=None`` (the default): the batches in flight follow each call's
    batch (``DecodePipeline(adaptive=True)``): 2 with the DMA on a stream of
    its own for batches of at least 8 MB of encoded cells (c2-shaped batches
    of 256), 3 with the DMA on the slot's stream below that (FOOD101-shaped
    batches of 128), ``auto_host_depth``. With
    ``register=True`` it means 3 (registered sources: DESIGN.md §8).

    ``prefetch=k`` (k < depth): ``LanceDataset`` iterates through
    ``fn.iterate`` instead, enqueueing the next k batches before yielding each
    one, so their decode overlaps the consumer's training step.

    ``register=True``: the first batch seen from each underlying `image` data
    buffer page-locks that whole buffer in place (``register_host``), so the
    batches sliced from a memory-mapped fragment reach HBM by DMA without a
    host memcpy. Only for long-lived buffers (a mapped dataset), not for
    batches built anew each step. At most ``register_cap`` buffers stay
    registered by this function (least recently used ones are unregistered),
    and a buffer the driver refuses to lock (memlock limit, overlapping
    registration) switches the function to the copying path instead of
    raising (ldt.h: such a range stays on the copying path)."""
    from collections import OrderedDict

    # (registered sources have no size-independent best depth: LanceDataset
    # over registered c2 fragments 436-475k img/s at depth 3 vs 297-308k at 2,
    # two alternating registered c2 batches 389k at 3 vs 572-583k at 2;
    # profiles/r4/dataset_depth_ab_r4dd.txt: 3 for them)
    if depth is None and register:
        depth = 3
    pipe = DecodePipeline(depth=depth or 3, device=device, adaptive=depth is None)
    image_column = fixed.get("image_column", "image")
    owned: "OrderedDict[int, object]" = OrderedDict()  # registrations made here, LRU order
    reg_on = [bool(register)]
    # churn guard: unregistering synchronises the device, so a loader that hands
    # out fresh buffers every batch (instead of slices of mapped fragments)
    # must not evict on every call; `evictions` holds the batch numbers of the
    # recent evictions
    seen = [0]  # batches offered to maybe_register (to_tensor_fn and the fn.iterate path)
    evictions: list = []

    def maybe_register(batch, col):
        seen[0] += 1
        if not reg_on[0] or not isinstance(batch, pa.RecordBatch):
            return
        arr = _column(batch, col)
        addr, size = _host_range(arr)
        if size == 0:
            return
        if addr in owned:
            owned.move_to_end(addr)
            return
        if addr in _registered:  # registered by the caller: theirs to manage
            return
        try:
            register_host(arr, device=device)
        except _lib.LdtError:
            reg_on[0] = False  # copying path from here on
            return
        owned[addr] = arr
        cap = max(1, int(register_cap))
        while len(owned) > cap:
            _, old = owned.popitem(last=False)
            unregister_host(old)
            evictions.append(seen[0])
        # more evictions than the cap within 4 x cap batches: the buffers do not
        # repeat, so registration cannot amortise; the copying path from here
        # on (the ranges still registered are released at once)
        while evictions and evictions[0] < seen[0] - 4 * cap:
            evictions.pop(0)
        if len(evictions) > cap:
            reg_on[0] = False
            release()

    def to_tensor_fn(batch, **kwargs):
        maybe_register(batch, kwargs.get("image_column", image_column))
        img, lbl = pipe.decode(batch, normalize=kwargs.get("normalize", normalize),
                               image_column=kwargs.get("image_column", fixed.get("image_column", "image")),
                               label_column=kwargs.get("label_column", fixed.get("label_column", "label")))
        return _as_device_batch(img, lbl)

    def release():
        """Unregister the buffers this function registered (waits for the device)."""
        while owned:
            _, old = owned.popitem(last=False)
            unregister_host(old)

    to_tensor_fn.check = pipe.check
    to_tensor_fn.registering = lambda: reg_on[0]
    to_tensor_fn.pipeline = pipe
    to_tensor_fn.release = release
    to_tensor_fn.prefetch = max(0, min(int(prefetch), pipe.depth - 1))
    def registered(batches):
        for b in batches:
            maybe_register(b, image_column)
            yield b

    to_tensor_fn.iterate = lambda batches: pipe.prefetch(
        registered(batches), ahead=to_tensor_fn.prefetch, normalize=normalize,
        image_column=fixed.get("image_column", "image"), label_column=fixed.get("label_column", "label"))
    return to_tensor_fn
