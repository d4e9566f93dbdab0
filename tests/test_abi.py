"""CPU tests of the C-ABI boundary: libldt.so loads (after torch, sharing its
HIP runtime) and exports every entry point include/ldt.h declares."""
import ctypes
import os
import re

import pytest

from conftest import REPO, has_gpu


def declared_symbols():
    src = open(os.path.join(REPO, "include", "ldt.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(ldt_[a-z_]+)\s*\(", src)))


def test_header_declares_expected_entry_points():
    syms = declared_symbols()
    for s in ("ldt_create", "ldt_destroy", "ldt_decode_batch", "ldt_decode_batch_large",
              "ldt_decode_batch_resident", "ldt_resize_raw", "ldt_shard_ranges", "ldt_shard_fragments"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    import ldt_amd
    from ldt_amd import _lib

    L = _lib.load_library()
    for s in declared_symbols():
        assert hasattr(L, s), f"libldt.so does not export {s}"
    assert set(_lib.EXPORTED) == set(declared_symbols())
    assert ldt_amd.version().startswith("ldt ")


def test_library_is_gfx950_code_object():
    data = open(os.path.join(REPO, "lance-distributed-training_amd", "ldt_amd", "libldt.so"), "rb").read()
    assert b"gfx950" in data


@pytest.mark.skipif(has_gpu(), reason="checks the no-device error path")
def test_no_device_fails_loudly():
    from ldt_amd import _lib

    L = _lib.load_library()
    assert L.ldt_create(0, 0, 0) is None
    with pytest.raises(_lib.LdtError):
        _lib.Context(0)
    import pyarrow as pa
    from ldt_amd import decode_tensor_image
    rb = pa.RecordBatch.from_arrays([pa.array([b"x"], pa.binary()), pa.array([1], pa.int64())], ["image", "label"])
    with pytest.raises(RuntimeError):
        decode_tensor_image(rb)


def test_null_context_is_rejected():
    from ldt_amd import _lib

    L = _lib.load_library()
    assert L.ldt_set_option(None, 1, 0) == _lib.LDT_ERR_ARG
    assert L.ldt_decode_batch(None, None, None, 0, 0, None, None, 0, None, None, None, None, None) == _lib.LDT_ERR_ARG
