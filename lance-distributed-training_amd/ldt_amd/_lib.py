"""ctypes binding of libldt.so (include/ldt.h) and the per-device context.

This is the Python side of the C-ABI boundary: the same stub a maintainer of
the reference would add. It owns no compute: every decode,
resize and shard computation runs in the gfx950 kernels of libldt.so. If the
library is missing or cannot be loaded, importing the product raises — there
is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  (must load torch's HIP runtime before libldt.so)


def hw_queues() -> int:
    """Hardware queues per process the HIP runtime uses (ROCclr's
    GPU_MAX_HW_QUEUES, default 4): streams beyond it share a queue."""
    try:
        return int(os.environ.get("GPU_MAX_HW_QUEUES", "4"))
    except ValueError:
        return 4

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libldt.so")

LDT_OK = 0
LDT_ERR_ARG = -1
LDT_ERR_HIP = -2
LDT_ERR_NOMEM = -3
LDT_ERR_IMAGE = -4

IMG_OK = 0
IMG_NOT_JPEG = 1
IMG_UNSUPPORTED = 2
IMG_CORRUPT = 3
IMG_TOO_LARGE = 4
IMG_NULL = 5
IMG_STATUS_TEXT = {
    IMG_NOT_JPEG: "cannot identify image file (not a baseline JPEG)",
    IMG_UNSUPPORTED: "unsupported JPEG (arithmetic/lossless/12-bit/CMYK/multi-scan sequential)",
    IMG_CORRUPT: "image file is truncated or corrupt",
    IMG_TOO_LARGE: "image dimensions exceed LDT_MAX_DIM",
    IMG_NULL: "null image cell",
}

OPT_SYNC_STATUS = 1
OPT_HUFF_MODE = 2
OPT_SUBSEQ_BITS = 3
OPT_PROFILE = 4
OPT_RESIZE_IMPL = 5
OPT_SYNC_WARM = 7
OPT_COPY_THREADS = 8
OPT_HOST_TIMING = 9
OPT_RESIZE_WAVES_PCT = 10
OPT_FUSED_DESTUFF = 11
OPT_COPY_MODE = 12
OPT_COPY_BIND = 13
OPT_COPY_NT = 14
OPT_RESIZE_WG_WAVES = 15
OPT_DEBUG_COUNTERS = 16
OPT_HUFF_WINDOW = 17

STAGES = ("h2d", "destuff", "huffman", "idct", "resize")
HOST_PHASES = ("slot", "parse", "plan", "copy_join", "launch", "status", "copy_wake", "copy_span")

# Every symbol include/ldt.h declares (checked by tests/test_abi.py).
EXPORTED = (
    "ldt_create", "ldt_destroy", "ldt_last_error", "ldt_set_option", "ldt_set_copy_stream", "ldt_version",
    "ldt_decode_batch", "ldt_decode_batch_large", "ldt_decode_batch_resident",
    "ldt_register_host", "ldt_unregister_host", "ldt_fetch_status", "ldt_last_ticket", "ldt_fetch_status_ticket",
    "ldt_stage_times", "ldt_host_times", "ldt_host_info", "ldt_resize_raw", "ldt_shard_ranges",
    "ldt_shard_fragments", "ldt_distributed_indices", "ldt_debug_counters",
)


class LdtError(RuntimeError):
    """A libldt call failed (argument, HIP runtime or allocation error)."""


class ImageDecodeError(ValueError, OSError):
    """One or more rows could not be decoded.

    Subclasses OSError so code written against the reference (PIL raises
    UnidentifiedImageError / OSError from Image.open at lance_iterable.py:42)
    keeps working, and ValueError per SURVEY.md §8b. ``rows`` maps row index ->
    LDT_IMG_* status. Also constructible from a message string alone, which is
    how torch's DataLoader re-raises an exception caught in a worker or in the
    pin-memory thread (``ExceptionWrapper.reraise``)."""

    def __init__(self, rows):
        if isinstance(rows, str):
            self.rows = {}
            super().__init__(rows)
            return
        self.rows = dict(rows)
        first = sorted(self.rows)[:8]
        desc = "; ".join(f"row {i}: {IMG_STATUS_TEXT.get(self.rows[i], self.rows[i])}" for i in first)
        more = "" if len(self.rows) <= 8 else f" (+{len(self.rows) - 8} more)"
        super().__init__(f"{len(self.rows)} image(s) failed to decode: {desc}{more}")


class Norm(ctypes.Structure):
    _fields_ = [("mean", ctypes.c_float * 3), ("std", ctypes.c_float * 3)]


_lib = None
_lib_lock = threading.Lock()


def load_library(path: str | None = None) -> ctypes.CDLL:
    """Load libldt.so and declare its signatures. Raises if it is missing."""
    global _lib
    with _lib_lock:
        if _lib is not None:
            return _lib
        p = path or os.environ.get("LDT_LIBRARY") or LIB_PATH  # override: experiment builds
        if not os.path.exists(p):
            raise ImportError(
                f"libldt.so not found at {p}: build it with `make -C lance-distributed-training_amd` "
                "or __graft_entry__.build(); the HIP path has no CPU fallback")
        L = ctypes.CDLL(p)
        vp, i64, i32, sz = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_size_t
        L.ldt_create.argtypes = [i32, sz, i32]
        L.ldt_create.restype = vp
        L.ldt_destroy.argtypes = [vp]
        L.ldt_destroy.restype = None
        L.ldt_last_error.argtypes = [vp]
        L.ldt_last_error.restype = ctypes.c_char_p
        L.ldt_set_option.argtypes = [vp, i32, i64]
        L.ldt_set_copy_stream.argtypes = [vp, vp]
        L.ldt_version.argtypes = []
        L.ldt_version.restype = ctypes.c_char_p
        L.ldt_decode_batch.argtypes = [vp, vp, vp, i64, i64, vp, vp, i64, vp, vp, vp, vp, vp]
        L.ldt_decode_batch_large.argtypes = [vp, vp, vp, i64, i64, vp, vp, i64, vp, vp, vp, vp, vp]
        L.ldt_decode_batch_resident.argtypes = [vp, vp, vp, vp, i64, vp, vp, vp, vp, vp, vp]
        L.ldt_fetch_status.argtypes = [vp, vp, vp, i64]
        L.ldt_last_ticket.argtypes = [vp]
        L.ldt_last_ticket.restype = i64
        L.ldt_fetch_status_ticket.argtypes = [vp, i64, vp, i64]
        L.ldt_stage_times.argtypes = [vp, vp, vp, i32]
        L.ldt_host_times.argtypes = [vp, vp, vp, i32]
        L.ldt_host_info.argtypes = [vp, ctypes.c_char_p, sz]
        L.ldt_resize_raw.argtypes = [vp, vp, i32, i64, i32, i32, i64, vp, vp, vp]
        L.ldt_shard_ranges.argtypes = [vp, i64, i64, i32, i32, vp, i64, vp, vp]
        L.ldt_shard_fragments.argtypes = [vp, vp, i32, i64, i32, i32, i64, vp, i64, vp, vp, vp]
        L.ldt_distributed_indices.argtypes = [vp, i64, i32, i32, i32, ctypes.c_uint64, i32, vp, i64,
                                              vp, vp]
        L.ldt_debug_resample_coeffs.argtypes = [vp, i32, i32, vp, vp, vp]
        L.ldt_debug_counters.argtypes = [vp, vp, vp]
        L.ldt_debug_last_resize.argtypes = [vp]
        L.ldt_debug_last_resize.restype = ctypes.c_int
        L.ldt_register_host.argtypes = [vp, vp, sz]
        L.ldt_unregister_host.argtypes = [vp, vp]
        for name in ("ldt_set_option", "ldt_set_copy_stream", "ldt_decode_batch", "ldt_decode_batch_large", "ldt_register_host",
                     "ldt_unregister_host",
                     "ldt_decode_batch_resident", "ldt_fetch_status", "ldt_fetch_status_ticket", "ldt_resize_raw", "ldt_stage_times", "ldt_host_times", "ldt_host_info",
                     "ldt_shard_ranges", "ldt_shard_fragments", "ldt_distributed_indices",
                     "ldt_debug_resample_coeffs",
                     "ldt_debug_counters"):
            getattr(L, name).restype = ctypes.c_int
        _lib = L
        return L


class Context:
    """One libldt context per (process, device) — ldt.h threading contract."""

    def __init__(self, device: int):
        self.lib = load_library()
        self.device = int(device)
        self.handle = self.lib.ldt_create(self.device, 0, 0)
        if not self.handle:
            raise LdtError(f"ldt_create(device={device}) failed (no HIP device?)")
        self.lock = threading.Lock()

    def check(self, rc: int, what: str) -> None:
        if rc == LDT_OK:
            return
        msg = self.lib.ldt_last_error(self.handle).decode(errors="replace")
        raise LdtError(f"{what} failed (rc={rc}): {msg}")

    def set_option(self, opt: int, value: int) -> None:
        self.check(self.lib.ldt_set_option(self.handle, opt, int(value)), "ldt_set_option")

    def set_copy_stream(self, stream) -> None:
        """The stream (a torch.cuda.Stream, or None for the library's own)
        this context's host cells go to HBM on under LDT_OPT_COPY_MODE 0."""
        self.check(self.lib.ldt_set_copy_stream(self.handle, stream.cuda_stream if stream is not None else None),
                   "ldt_set_copy_stream")

    def stage_times(self, reset: bool = False):
        """{stage: (total_ms, launches)} from LDT_OPT_PROFILE events."""
        import numpy as np

        ms = np.zeros(len(STAGES), np.float64)
        cnt = np.zeros(len(STAGES), np.int64)
        self.check(self.lib.ldt_stage_times(self.handle, ms.ctypes.data, cnt.ctypes.data, int(reset)),
                   "ldt_stage_times")
        return {k: (float(ms[i]), int(cnt[i])) for i, k in enumerate(STAGES)}

    def host_times(self, reset: bool = False):
        """({phase: total_us}, calls) from LDT_OPT_HOST_TIMING."""
        import numpy as np

        us = np.zeros(len(HOST_PHASES), np.float64)
        calls = ctypes.c_int64(0)
        self.check(self.lib.ldt_host_times(self.handle, us.ctypes.data, ctypes.byref(calls), int(reset)),
                   "ldt_host_times")
        return {k: float(us[i]) for i, k in enumerate(HOST_PHASES)}, int(calls.value)

    def debug_counters(self, stream=None):
        """The parallel Huffman decoder's 16 counters of the last batch
        (LDT_OPT_DEBUG_COUNTERS = 1; layout in ldt.h), as a list of ints."""
        import numpy as np

        out = np.zeros(16, np.int32)
        self.check(self.lib.ldt_debug_counters(self.handle, out.ctypes.data,
                                               stream.cuda_stream if stream is not None else None),
                   "ldt_debug_counters")
        return out.tolist()

    def host_info(self) -> dict:
        """The host copy placement (ldt_host_info): copy threads and their
        CPUs, the GPU's NUMA node, the cgroup quota, local rank/world."""
        import json

        buf = ctypes.create_string_buffer(4096)
        self.check(self.lib.ldt_host_info(self.handle, buf, len(buf)), "ldt_host_info")
        return json.loads(buf.value.decode())

    def __del__(self):
        h = getattr(self, "handle", None)
        if h:
            try:
                self.lib.ldt_destroy(h)
            except Exception:
                pass
            self.handle = None


_contexts: dict = {}
_ctx_lock = threading.Lock()


def get_context(device: int) -> Context:
    with _ctx_lock:
        ctx = _contexts.get(device)
        if ctx is None:
            ctx = Context(device)
            _contexts[device] = ctx
        return ctx


def version() -> str:
    return load_library().ldt_version().decode()
