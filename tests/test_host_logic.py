"""CPU tests of the host-side logic around the kernels: the Arrow dataset
shim, sampler iteration (with the oracle standing in for the index kernel,
as the checker), error reporting."""
import os

import numpy as np
import pyarrow as pa
import pytest

from oracle import oracle


def _frag_compute(rows, B, r, W, pad_to):
    recs = oracle.sharded_fragment_batches(rows, B, r, W, pad=False)
    local = len(recs)
    if pad_to is not None and pad_to >= 0:
        full = oracle.sharded_fragment_batches(rows, B, r, W, pad=True)
        # oracle pads to max-over-ranks; trim/extend semantics identical when pad_to == max
        assert pad_to >= local
        recs = full[:pad_to] if len(full) >= pad_to else full
    return recs, local


@pytest.fixture()
def small_ds(tmp_path):
    from ldt_amd import write_dataset

    n = 1000
    tbl = pa.table({"image": pa.array([bytes([i % 251]) * (1 + i % 7) for i in range(n)], pa.binary()),
                    "label": pa.array(np.arange(n) % 101, pa.int64())})
    return write_dataset(tbl, str(tmp_path / "ds"), max_rows_per_file=300), n


def test_write_dataset_fragments(small_ds):
    ds, n = small_ds
    assert [f.count_rows() for f in ds.get_fragments()] == [300, 300, 300, 100]
    assert ds.count_rows() == n
    rb = ds.read_range(250, 380)  # spans two fragments
    assert rb.num_rows == 130 and rb.column(1).to_pylist() == list(np.arange(250, 380) % 101)


def test_sharded_batch_sampler_iteration(small_ds):
    from ldt_amd import ShardedBatchSampler

    ds, n = small_ds
    seen = []
    for r in range(3):
        s = ShardedBatchSampler(r, 3, compute=oracle.sharded_batch_ranges)
        for rb in s(ds, batch_size=64):
            seen += rb.column(1).to_pylist()
    assert sorted(seen) == sorted(list(np.arange(n) % 101))


def test_sharded_fragment_sampler_iteration(small_ds):
    from ldt_amd import ShardedFragmentSampler

    ds, n = small_ds
    counts = []
    for r in range(3):
        s = ShardedFragmentSampler(r, 3, compute=_frag_compute)
        bs = list(s(ds, batch_size=128))
        counts.append(len(bs))
        assert all(b.num_rows <= 128 for b in bs)
    assert counts == [3 + 1, 3, 3]  # rank 0 owns fragments 0 and 3


def test_lance_dataset_iterates_to_tensor_fn(small_ds):
    from ldt_amd import FullScanSampler, LanceDataset

    ds, n = small_ds
    calls = []
    lds = LanceDataset(ds, batch_size=100, sampler=FullScanSampler(),
                       to_tensor_fn=lambda b, **kw: calls.append(b.num_rows) or b.num_rows)
    assert sum(lds) == n and calls[:3] == [100, 100, 100]


def test_safe_dataset_rows(small_ds, tmp_path):
    from ldt_amd import SafeLanceDataset, get_safe_loader

    ds, n = small_ds
    sds = SafeLanceDataset(ds.uri)
    assert len(sds) == n and sds[5]["label"] == 5
    got = sds.__getitems__([1, 999])
    assert [g["label"] for g in got] == [1, 999 % 101]
    dl = get_safe_loader(sds, batch_size=10, collate_fn=lambda rows: [r["label"] for r in rows])
    first = next(iter(dl))
    assert first == list(range(10))


def test_image_decode_error_is_oserror_and_valueerror():
    from ldt_amd import ImageDecodeError

    e = ImageDecodeError({3: 1, 0: 3})
    assert isinstance(e, OSError) and isinstance(e, ValueError)
    assert "row 0" in str(e) and "row 3" in str(e)


def _dist_compute(n, W, r, shuffle, seed, drop_last):
    # the oracle stands in for the device kernel (checker only)
    return np.asarray(oracle.distributed_indices(n, W, r, shuffle, seed, 0, drop_last), np.int64)


@pytest.mark.parametrize("n,W,drop_last", [(10, 3, False), (10, 3, True), (1, 4, False), (1, 4, True),
                                           (257, 8, False), (0, 2, False)])
def test_distributed_sampler_host_logic_matches_torch(n, W, drop_last):
    """ldt_amd.DistributedSampler: constructor, num_samples, set_epoch and
    iteration order identical to torch's (distributed.py:66-157)."""
    from torch.utils.data import DistributedSampler as TorchDS

    from ldt_amd import DistributedSampler

    ds = list(range(n))
    for r in range(W):
        for shuffle in (True, False):
            a = DistributedSampler(ds, num_replicas=W, rank=r, shuffle=shuffle, seed=5, drop_last=drop_last,
                                   compute=_dist_compute)
            b = TorchDS(ds, num_replicas=W, rank=r, shuffle=shuffle, seed=5, drop_last=drop_last)
            for ep in (0, 2):
                a.set_epoch(ep)
                b.set_epoch(ep)
                assert len(a) == len(b) and a.total_size == b.total_size
                assert list(a) == list(b)


def test_distributed_sampler_rank_errors():
    from ldt_amd import DistributedSampler

    with pytest.raises(ValueError):
        DistributedSampler(range(5), num_replicas=2, rank=2)
    with pytest.raises(ValueError):
        DistributedSampler(range(5), num_replicas=2, rank=-1)


def test_image_decode_error_survives_dataloader_reraise():
    """torch re-raises worker / pin-thread exceptions as exc_type(message)."""
    from torch._utils import ExceptionWrapper

    from ldt_amd import ImageDecodeError

    try:
        raise ImageDecodeError({1: 3})
    except ImageDecodeError:
        w = ExceptionWrapper(where="in pin memory thread for device 0")
    with pytest.raises(ImageDecodeError, match="row 1"):
        w.reraise()


def test_fused_destuff_classification_matches_per_byte_rules(tmp_path):
    """The fused destuff's 0xFF-driven classification (ldt_device.hpp
    ds_classify16_ff, used by k_huff_image) equals the per-byte rules of the
    k_destuff_* kernels (ds_classify16) on 2M random marker-heavy cases:
    compiled as host code with hipcc, no GPU needed."""
    import os
    import shutil
    import subprocess

    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = tmp_path / "ds_classify_check"
    subprocess.run([hipcc, "-O2", "-std=c++17", "-w",
                    "-I", os.path.join(root, "lance-distributed-training_amd", "csrc"),
                    os.path.join(root, "tools", "checks", "ds_classify_check.cpp"), "-o", str(exe)],
                   check=True, timeout=300)
    r = subprocess.run([str(exe), "2000000"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 mismatches" in r.stdout


def test_slot_stream_plan():
    """DecodePipeline's stream plan (transforms.slot_streams): normal streams
    while the slots + the consumer's stream fit the hardware queues, high
    priority for deeper pipelines (up to one pool of queues), the cells' DMA on
    the slots' streams whenever the copy stream would share a queue."""
    from ldt_amd.transforms import slot_streams

    assert slot_streams(2, 4) == (0, False)   # c2 host legs: copy stream
    assert slot_streams(3, 4) == (0, True)    # c2 resident: 3 slots + consumer + copy > 4
    assert slot_streams(4, 4) == (4, False)   # all high priority, copy stream beside the consumer
    assert slot_streams(5, 4) == (4, True)    # progressive default: 4 high + 1 normal
    assert slot_streams(7, 4) == (4, True)    # 4 high + 3 normal: DMA on the slots
    assert slot_streams(8, 4) == (4, True)
    assert slot_streams(6, 8) == (0, False)   # 6 slots + consumer + copy stream fit 8 queues
    assert slot_streams(7, 8) == (0, True)
    assert slot_streams(3, 4, "1") == (3, False)
    assert slot_streams(7, 4, "0") == (0, True)


def test_auto_host_depth_from_cell_bytes():
    """make_to_tensor_fn(depth=None) picks 3 in flight for batches under 8 MB
    of encoded cells and 2 above (profiles/r4/host_depth_ab_r4hd.txt); the
    cell bytes of a sliced binary / large_binary / fixed-size column are the
    slice's value bytes, not its whole buffer's."""
    from ldt_amd.transforms import AUTO_DEPTH_SMALL_BYTES, _cell_bytes, auto_host_depth

    assert auto_host_depth(3_300_000) == 3          # FOOD101-shaped batch of 128
    assert auto_host_depth(17_000_000) == 2         # c2 batch of 256
    assert auto_host_depth(AUTO_DEPTH_SMALL_BYTES) == 2
    assert auto_host_depth(0) == 2                  # unknown (not a host column)
    cells = [bytes([k % 251]) * (100 + 7 * k) for k in range(40)]
    for t in (pa.binary(), pa.large_binary()):
        rb = pa.RecordBatch.from_arrays([pa.array(cells, t), pa.array(np.arange(40, dtype=np.int64))],
                                        names=["image", "label"])
        assert _cell_bytes(rb, "image") == sum(map(len, cells))
        sl = rb.slice(5, 20)
        assert _cell_bytes(sl, "image") == sum(map(len, cells[5:25]))
    fx = pa.RecordBatch.from_arrays([pa.array([b"x" * 48] * 9, pa.binary(48))], names=["image"])
    assert _cell_bytes(fx.slice(2, 5), "image") == 5 * 48
    assert _cell_bytes(fx, "missing") == 0
    # a Table's chunked column: the chunks' spans, no combine
    tb = pa.Table.from_batches([pa.RecordBatch.from_arrays([pa.array(cells[:15], pa.binary())], names=["image"]),
                                pa.RecordBatch.from_arrays([pa.array(cells[15:], pa.binary())], names=["image"])])
    assert tb.column("image").num_chunks == 2
    assert _cell_bytes(tb, "image") == sum(map(len, cells))


class _FakePipeline:
    """DecodePipeline stand-in for host-logic tests (no GPU): records decodes."""

    def __init__(self, depth=2, device=None, profile=False, adaptive=False):
        self.depth = depth
        self.k = 0
        self.ctxs = []

    def set_option(self, opt, value):
        pass

    def check_slot(self, i):
        pass

    def check(self):
        pass

    def decode(self, batch, **kw):
        self.k += 1
        return None, None

    def prefetch(self, batches, ahead=2, **kw):
        for b in batches:
            self.k += 1
            yield {"image": b}


def test_register_churn_guard_counts_prefetch_batches(monkeypatch):
    """make_to_tensor_fn(register=True): the churn guard counts batches on the
    fn.iterate (prefetch) path too, so a loop cycling over more mapped buffers
    than register_cap, each serving many batches, keeps registering (ADVICE r4:
    the guard's window never slid on that path and switched registration off
    after cap+1 evictions), while buffers that never repeat switch it off."""
    from ldt_amd import transforms as T

    regs = []
    monkeypatch.setattr(T, "DecodePipeline", _FakePipeline)
    monkeypatch.setattr(T, "register_host", lambda arr, device=None: regs.append(T._host_range(arr)[0]))
    monkeypatch.setattr(T, "unregister_host", lambda arr: None)
    monkeypatch.setattr(T, "_as_device_batch", lambda img, lbl: {"image": img})
    frags = [pa.RecordBatch.from_arrays([pa.array([bytes([f]) * 64] * 400, pa.binary())], names=["image"])
             for f in range(5)]
    # 5 fragments, cap 2: every fragment change evicts, but each serves 20 batches
    order = [frags[(k // 20) % 5].slice((k % 20) * 10, 10) for k in range(400)]
    for use_iterate in (True, False):
        regs.clear()
        fn = T.make_to_tensor_fn(depth=2, register=True, register_cap=2, prefetch=1)
        if use_iterate:
            assert sum(1 for _ in fn.iterate(order)) == 400
        else:
            for b in order:
                fn(b)
        assert fn.registering(), use_iterate
        assert len(regs) == 20  # one registration per fragment visit
    # fresh buffers every batch: no reuse, registration switches off
    fn = T.make_to_tensor_fn(depth=2, register=True, register_cap=2, prefetch=1)
    fresh = [pa.RecordBatch.from_arrays([pa.array([bytes([k % 251]) * 64] * 10, pa.binary())], names=["image"])
             for k in range(40)]
    assert sum(1 for _ in fn.iterate(fresh)) == 40
    assert not fn.registering()


def test_progressive_depth_default_agrees_with_bench():
    """bench.py's progressive legs run at ldt_amd.PROGRESSIVE_DEPTH (it sets
    its own copy before importing torch)."""
    import re

    import ldt_amd
    from conftest import REPO

    src = open(os.path.join(REPO, "bench.py")).read()
    m = re.search(r"^    PROG_DEPTH = (\d+)", src, re.M)
    assert m and int(m.group(1)) == ldt_amd.PROGRESSIVE_DEPTH == 5
