"""Arrow-backed stand-in for the pylance dataset classes the reference uses.

pylance is not installed in this image, so this module
provides the minimum the hot path's callers need, with the same names and
call shapes as the reference's imports:

* ``write_dataset(data, uri, max_rows_per_file=...)`` — fragments of at most
  ``max_rows_per_file`` rows, like ``lance.write_dataset`` at
  ``create_datasets/classification.py:55-61`` (FOOD101: [12500 x 6, 750]).
  Fragments are Arrow IPC files, memory-mapped on read (zero-copy buffers
  that ``to_tensor_fn`` hands to libldt.so by address).
* ``LanceDataset(path, batch_size, to_tensor_fn=..., sampler=...)`` — the
  iterable dataset of ``lance_iterable.py:53-59``.
* ``SafeLanceDataset(uri)`` + ``get_safe_loader(...)`` — the map-style pair of
  ``lance_map_style.py:54,60-69``; ``get_safe_loader`` is a stock DataLoader.
  With ``num_workers > 0`` the workers only fetch and pack rows; the GPU
  decode runs in the main process (``ldt_amd.transforms.DeviceBatch``).

It is I/O plumbing, not the accelerated path: the storage engine is out of
scope.
"""
from __future__ import annotations

import json
import os
from typing import Iterable, List, Optional, Sequence, Union

import numpy as np
import pyarrow as pa
import pyarrow.ipc as ipc
import torch
from torch.utils.data import DataLoader, Dataset, IterableDataset

_META = "_ldt_dataset.json"


def write_dataset(data: Union[pa.Table, Iterable[pa.RecordBatch]], uri: str, schema: Optional[pa.Schema] = None,
                  mode: str = "overwrite", max_rows_per_file: int = 1024 * 1024) -> "ArrowDataset":
    if mode != "overwrite" and os.path.exists(os.path.join(uri, _META)):
        raise FileExistsError(uri)
    os.makedirs(uri, exist_ok=True)
    for f in os.listdir(uri):
        if f.endswith(".arrow") or f == _META:
            os.remove(os.path.join(uri, f))
    if isinstance(data, pa.Table):
        schema = schema or data.schema
        batches = data.to_batches()
    else:
        batches = data
    rows: List[int] = []
    writer = None
    cur = 0

    def _open():
        nonlocal writer, cur
        path = os.path.join(uri, f"fragment-{len(rows):06d}.arrow")
        writer = ipc.new_file(path, schema)
        rows.append(0)
        cur = 0

    for rb in batches:
        if schema is None:
            schema = rb.schema
        off = 0
        while off < rb.num_rows:
            if writer is None or cur == max_rows_per_file:
                if writer is not None:
                    writer.close()
                _open()
            take = min(max_rows_per_file - cur, rb.num_rows - off)
            writer.write_batch(rb.slice(off, take))
            cur += take
            rows[-1] += take
            off += take
    if writer is not None:
        writer.close()
    with open(os.path.join(uri, _META), "w") as f:
        json.dump({"fragments": rows, "schema": schema.to_string() if schema is not None else ""}, f)
    return ArrowDataset(uri)


class Fragment:
    def __init__(self, path: str, fid: int, rows: int):
        self.path, self.fragment_id, self._rows = path, fid, rows
        self._table = None

    def _tbl(self) -> pa.Table:
        if self._table is None:
            src = pa.memory_map(self.path, "r")
            self._table = ipc.open_file(src).read_all()
        return self._table

    def count_rows(self) -> int:
        return self._rows

    def read_slice(self, start: int, end: int, columns=None) -> pa.RecordBatch:
        t = self._tbl().slice(start, end - start)
        if columns is not None:
            t = t.select(columns)
        return t.combine_chunks().to_batches()[0] if t.num_rows else pa.RecordBatch.from_pylist([], schema=t.schema)

    def to_batches(self, batch_size: int, columns=None):
        for s in range(0, self._rows, batch_size):
            yield self.read_slice(s, min(s + batch_size, self._rows), columns)


class ArrowDataset:
    """Fragmented Arrow dataset on disk (the storage the samplers walk)."""

    def __init__(self, uri: str):
        with open(os.path.join(uri, _META)) as f:
            meta = json.load(f)
        self.uri = uri
        self._frags = [Fragment(os.path.join(uri, f"fragment-{i:06d}.arrow"), i, r)
                       for i, r in enumerate(meta["fragments"])]
        self._starts = np.concatenate([[0], np.cumsum([f.count_rows() for f in self._frags])]).astype(np.int64)

    def get_fragments(self) -> List[Fragment]:
        return list(self._frags)

    def count_rows(self) -> int:
        return int(self._starts[-1])

    @property
    def schema(self) -> pa.Schema:
        return self._frags[0]._tbl().schema

    def read_range(self, start: int, end: int, columns=None) -> pa.RecordBatch:
        """Rows [start, end) in dataset order (may span fragments)."""
        parts = []
        f = int(np.searchsorted(self._starts, start, side="right") - 1)
        pos = start
        while pos < end:
            fs, fe = int(self._starts[f]), int(self._starts[f + 1])
            e = min(end, fe)
            parts.append(self._frags[f].read_slice(pos - fs, e - fs, columns))
            pos = e
            f += 1
        if len(parts) == 1:
            return parts[0]
        return pa.Table.from_batches(parts).combine_chunks().to_batches()[0]

    def take(self, indices: Sequence[int], columns=None) -> pa.Table:
        """Rows at `indices` (dataset order), in the given order: one vectorised
        Table.take per fragment touched, then the original order restored."""
        idx = np.asarray(indices, dtype=np.int64)
        if idx.size == 0:
            t = self.schema.empty_table()
            return t.select(columns) if columns is not None else t
        if idx.min() < 0 or idx.max() >= self.count_rows():
            raise IndexError("row index out of range")
        frag = np.searchsorted(self._starts, idx, side="right") - 1
        parts, pos = [], []
        for fid in np.unique(frag):
            sel = np.nonzero(frag == fid)[0]
            t = self._frags[int(fid)]._tbl()
            if columns is not None:
                t = t.select(columns)
            parts.append(t.take(pa.array(idx[sel] - self._starts[fid])))
            pos.append(sel)
        tbl = pa.concat_tables(parts) if len(parts) > 1 else parts[0]
        if len(parts) > 1:
            tbl = tbl.take(pa.array(np.argsort(np.concatenate(pos), kind="stable")))
        return tbl


def dataset(uri: str) -> ArrowDataset:
    return ArrowDataset(uri)


class LanceDataset(IterableDataset):
    """Iterable dataset calling ``to_tensor_fn`` once per RecordBatch
    (pylance LanceDataset as used at lance_iterable.py:53-59)."""

    def __init__(self, dataset, batch_size: int, *args, columns=None, filter=None, sampler=None,
                 to_tensor_fn=None, batch_readahead: int = 16, **kwargs):
        super().__init__()
        self.dataset = dataset if isinstance(dataset, ArrowDataset) else ArrowDataset(dataset)
        self.batch_size = int(batch_size)
        self.columns, self.filter = columns, filter
        self.sampler = sampler
        self.to_tensor_fn = to_tensor_fn
        self.batch_readahead = batch_readahead

    def _sampler(self):
        from .sampler import FullScanSampler

        return self.sampler or FullScanSampler()

    def __getstate__(self):
        # Pickled for DataLoader workers (spawn) in the main process: the
        # sampler's batch plan is computed here, where the device kernels and
        # the process group (pad=True's all_reduce) live, and the workers only
        # read rows. Each worker w then yields plan batches w, w+nw, ... in
        # order, which the DataLoader's round-robin turns back into the
        # sampler's order. A sampler without a read plan (any object following
        # the pylance protocol sampler(dataset, batch_size=...)) runs in the
        # workers instead.
        if self.filter is not None:
            raise NotImplementedError("filter is not supported by the dataset shim")
        state = dict(self.__dict__)
        sampler = self._sampler()
        if hasattr(sampler, "read_plan"):
            state["_worker_plan"] = sampler.read_plan(self.dataset, self.batch_size)
        return state

    def __iter__(self):
        from torch.utils.data import get_worker_info

        from .sampler import read_planned

        info = get_worker_info()
        fn = self.to_tensor_fn
        if info is not None:
            if self.filter is not None:
                raise NotImplementedError("filter is not supported by the dataset shim")
            plan = getattr(self, "_worker_plan", None)
            sampler = self._sampler()
            if plan is None and hasattr(sampler, "read_plan"):
                # not pickled (fork start method): this build's samplers plan on
                # the GPU (and pad=True runs a collective), which a forked child
                # must not touch
                raise RuntimeError("LanceDataset workers need multiprocessing_context='spawn' with this "
                                   "build's samplers (the batch plan runs device kernels in the main process)")
            if plan is None:
                # a protocol sampler has no read plan to shard before reading:
                # every worker runs it whole and keeps its own share, so the
                # rows are read num_workers times (the decode is not repeated)
                if info.id == 0 and info.num_workers > 1:
                    import warnings

                    warnings.warn(f"{type(sampler).__name__} has no read_plan: each of the {info.num_workers} "
                                  "workers reads every batch and keeps 1/num_workers of them", RuntimeWarning)
                batches = sampler(self.dataset, batch_size=self.batch_size, columns=self.columns,
                                  batch_readahead=self.batch_readahead)
                for k, rb in enumerate(batches):
                    if k % info.num_workers == info.id:
                        yield fn(rb) if fn is not None else rb
                return
            for desc in plan[info.id::info.num_workers]:
                rb = read_planned(self.dataset, desc, self.columns)
                yield fn(rb) if fn is not None else rb
            return
        batches = self._sampler()(self.dataset, batch_size=self.batch_size, columns=self.columns,
                                  filter=self.filter, batch_readahead=self.batch_readahead)
        if fn is not None and getattr(fn, "prefetch", 0) > 0:
            # make_to_tensor_fn(prefetch=k): decode k batches ahead on side streams
            yield from fn.iterate(batches)
            return
        for rb in batches:
            yield fn(rb) if fn is not None else rb


class SafeLanceDataset(Dataset):
    """Map-style dataset yielding ``{"image": bytes, "label": int}`` rows
    (pylance SafeLanceDataset as used at lance_map_style.py:54)."""

    def __init__(self, uri: str, columns=None):
        self.uri = uri
        self.columns = columns
        self._ds = None
        self._n = ArrowDataset(uri).count_rows()

    def _d(self) -> ArrowDataset:
        if self._ds is None:  # opened lazily per worker process
            self._ds = ArrowDataset(self.uri)
        return self._ds

    def __len__(self) -> int:
        return self._n

    def __getitem__(self, i: int):
        return self._d().take([int(i)], self.columns).to_pylist()[0]

    def __getitems__(self, indices):
        return self._d().take(list(indices), self.columns).to_pylist()


def get_safe_loader(dataset, batch_size: int, sampler=None, shuffle: bool = False, num_workers: int = 0,
                    collate_fn=None, pin_memory: bool = False, persistent_workers: bool = False, **kwargs):
    """``lance.torch.data.get_safe_loader`` stand-in (lance_map_style.py:60-69):
    a stock ``torch.utils.data.DataLoader`` with spawn workers. The GPU
    ``collate_fn`` needs no special casing: in the workers it packs the rows
    into shared memory and the decode runs in the main process (see
    ``ldt_amd.transforms.DeviceBatch``)."""
    mp_ctx = kwargs.pop("multiprocessing_context", "spawn" if num_workers > 0 else None)
    return DataLoader(dataset, batch_size=batch_size, sampler=sampler, shuffle=shuffle if sampler is None else False,
                      num_workers=num_workers, collate_fn=collate_fn, pin_memory=pin_memory,
                      persistent_workers=persistent_workers if num_workers > 0 else False,
                      multiprocessing_context=mp_ctx, **kwargs)
