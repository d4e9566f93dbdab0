"""CPU tests of the DataLoader-worker side of the plug-ins (no GPU needed).

The reference runs its collate_fn in 8 spawn workers with pin_memory=True
(lance_map_style.py:60-69) and, under --no_ddp, its to_tensor_fn inside 8
spawn workers of a DataLoader over LanceDataset (lance_iterable.py:71-72).
In a worker the plug-ins must not touch the GPU: they return a DeviceBatch
whose packed cells travel through shared memory. These tests check what the
workers hand back (bytes, labels, order, one yield per batch); the decode of
those batches is checked against the oracle by the -m gpu tests.
"""
import collections.abc

import numpy as np
import pyarrow as pa
import pytest
import torch
from torch.utils.data import DataLoader

from ldt_amd import transforms


def _cells(n):
    return [bytes([(7 * i) % 256]) * (3 + (i * 13) % 41) for i in range(n)]


@pytest.fixture()
def cell_ds(tmp_path):
    from ldt_amd import write_dataset

    cells = _cells(57)
    tbl = pa.table({"image": pa.array(cells, pa.binary()), "label": pa.array(np.arange(57) * 3, pa.int64())})
    return write_dataset(tbl, str(tmp_path / "ds"), max_rows_per_file=20), cells


def test_pack_roundtrip_list_and_arrow():
    cells = _cells(9)
    cells[4] = None
    arr, lab = transforms._unpack(transforms._pack_list(cells, list(range(9))))
    assert arr.to_pylist() == cells and lab.tolist() == list(range(9))
    a = pa.array(_cells(12), pa.binary()).slice(3, 7)
    arr, lab = transforms._unpack(transforms._pack_arrow(a, np.arange(7)))
    assert arr.to_pylist() == a.to_pylist() and arr.type == pa.large_binary()
    big = pa.array(_cells(5), pa.large_binary()).slice(1, 3)
    assert transforms._unpack(transforms._pack_arrow(big, None))[0].to_pylist() == big.to_pylist()


def test_device_batch_is_not_a_mapping():
    # torch's pin_memory() must call DeviceBatch.pin_memory() rather than
    # recurse into a Mapping's values
    b = transforms.DeviceBatch(transforms._pack_list(_cells(2), [0, 1]))
    assert not isinstance(b, collections.abc.Mapping) and hasattr(b, "pin_memory")
    assert "2 cells pending" in repr(b)


def test_device_tensor_pin_memory_is_identity():
    from torch.utils.data._utils.pin_memory import pin_memory

    t = torch.arange(6.0).as_subclass(transforms.DeviceTensor)
    out = pin_memory({"image": t})
    assert out["image"] is t
    assert type(t + 1) is torch.Tensor  # ops give plain tensors


def test_map_style_collate_in_spawn_workers(cell_ds):
    """collate_fn in stock DataLoader spawn workers (the reference's
    get_safe_loader arguments, lance_map_style.py:60-69) returns DeviceBatches
    carrying exactly the rows' bytes and labels, in sampler order."""
    from ldt_amd import SafeLanceDataset, collate_fn

    ds, cells = cell_ds
    sds = SafeLanceDataset(ds.uri)
    dl = DataLoader(sds, batch_size=8, shuffle=False, num_workers=2, collate_fn=collate_fn,
                    pin_memory=False, persistent_workers=True, multiprocessing_context="spawn")
    got_cells, got_labels = [], []
    for b in dl:
        assert isinstance(b, transforms.DeviceBatch)
        arr, lab = transforms._unpack(b._packed)
        got_cells += arr.to_pylist()
        got_labels += lab.tolist()
    assert got_cells == cells and got_labels == list(np.arange(57) * 3)


def test_iterable_lance_dataset_workers_yield_each_batch_once(cell_ds):
    """LanceDataset in a DataLoader with spawn workers and batch_size=None
    (lance_iterable.py:71-72): every sampler batch is yielded once, in the
    sampler's order, and to_tensor_fn's worker result carries its cells."""
    from ldt_amd import FullScanSampler, LanceDataset, decode_tensor_image

    ds, cells = cell_ds
    ref = [rb.column(1).to_pylist() for rb in LanceDataset(ds, batch_size=6, sampler=FullScanSampler())]
    lds = LanceDataset(ds, batch_size=6, sampler=FullScanSampler())
    dl = DataLoader(lds, num_workers=3, batch_size=None, multiprocessing_context="spawn")
    assert [rb.column(1).to_pylist() for rb in dl] == ref
    lds = LanceDataset(ds, batch_size=6, sampler=FullScanSampler(), to_tensor_fn=decode_tensor_image)
    dl = DataLoader(lds, num_workers=2, batch_size=None, multiprocessing_context="spawn")
    got = []
    for b in dl:
        assert isinstance(b, transforms.DeviceBatch)
        arr, lab = transforms._unpack(b._packed)
        got.append(lab.tolist())
        assert arr.to_pylist() == [cells[i // 3] for i in lab.tolist()]
    assert got == ref


class _ProtocolSampler:
    """A sampler that only follows the pylance call protocol
    sampler(dataset, batch_size=...) -> RecordBatches (no read plan)."""

    def __call__(self, dataset, *args, batch_size=128, columns=None, **kwargs):
        for f in dataset.get_fragments():
            yield from f.to_batches(batch_size, columns)


def test_protocol_sampler_runs_in_spawn_workers(cell_ds):
    """A sampler without this build's read plan still pickles with the
    dataset; the workers run it and yield every batch once, in order."""
    from ldt_amd import LanceDataset

    ds, _ = cell_ds
    ref = [rb.column(1).to_pylist() for rb in LanceDataset(ds, batch_size=6, sampler=_ProtocolSampler())]
    lds = LanceDataset(ds, batch_size=6, sampler=_ProtocolSampler())
    dl = DataLoader(lds, num_workers=3, batch_size=None, multiprocessing_context="spawn")
    assert [rb.column(1).to_pylist() for rb in dl] == ref


def test_filter_with_workers_raises(cell_ds):
    """A filter the shim cannot apply must not be dropped silently in workers."""
    import pickle

    from ldt_amd import FullScanSampler, LanceDataset

    ds, _ = cell_ds
    lds = LanceDataset(ds, batch_size=6, sampler=FullScanSampler(), filter="label > 3")
    with pytest.raises(NotImplementedError):
        pickle.dumps(lds)


def test_forked_worker_refuses_device_planning(cell_ds):
    """Under fork the worker would run the device plan kernels (and pad=True's
    collective) in the child: it raises instead."""
    from ldt_amd import FullScanSampler, LanceDataset

    ds, _ = cell_ds
    lds = LanceDataset(ds, batch_size=6, sampler=FullScanSampler())
    dl = DataLoader(lds, num_workers=1, batch_size=None, multiprocessing_context="fork")
    with pytest.raises(RuntimeError, match="spawn"):
        list(dl)
