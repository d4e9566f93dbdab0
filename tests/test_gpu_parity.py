"""GPU parity tests: the HIP path through the C-ABI vs the oracle / golden
vectors. Bar: bit-exact (the whole path is integer + an exact float32 LUT),
which is stricter than north_star's max-abs <= 2/255 tolerance; the
tolerance check is kept as a second assertion so a regression reports its size.
"""
import hashlib

import numpy as np
import pyarrow as pa
import pytest

from conftest import GOLDEN, read_golden
from oracle import oracle

pytestmark = pytest.mark.gpu

TOL = 2.0 / 255.0  # north_star: max abs <= 2/255 per channel


def sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def _batch(cells, labels=None, large=False):
    t = pa.large_binary() if large else pa.binary()
    labels = np.arange(len(cells), dtype=np.int64) if labels is None else np.asarray(labels, np.int64)
    return pa.RecordBatch.from_arrays([pa.array(list(cells), type=t), pa.array(labels, pa.int64())],
                                      names=["image", "label"])


def _check(got, exp, what=""):
    got = np.asarray(got)
    diff = np.abs(got.astype(np.float64) - exp.astype(np.float64))
    assert diff.max() <= TOL, f"{what}: max abs {diff.max()} > 2/255 (mean {diff.mean()})"
    assert np.array_equal(got, exp), f"{what}: not bit-exact (max abs {diff.max()}, mean {diff.mean()}, " \
                                     f"{np.count_nonzero(diff)} elems differ)"


def test_golden_images_bit_exact(manifest):
    import ldt_amd

    ents = manifest["images"]
    cells = [read_golden(e["file"]) for e in ents]
    labels = [e["label"] for e in ents]
    out = ldt_amd.decode_tensor_image(_batch(cells, labels))
    img = out["image"].cpu().numpy()
    assert out["image"].dtype.__str__() == "torch.float32" and out["image"].is_contiguous()
    assert out["label"].cpu().numpy().tolist() == labels
    for k, e in enumerate(ents):
        if sha(img[k]) != e["sha256_tensor_f32"]:
            _check(img[k], oracle.jpeg_to_tensor(cells[k]), e["name"])
        assert sha(img[k]) == e["sha256_tensor_f32"], e["name"]
    nrm = ldt_amd.decode_tensor_image(_batch(cells, labels), normalize=True)["image"].cpu().numpy()
    for k, e in enumerate(ents):
        assert sha(nrm[k]) == e["sha256_tensor_norm_f32"], e["name"]


def test_each_golden_image_alone(manifest):
    import ldt_amd

    for e in manifest["images"]:
        b = read_golden(e["file"])
        img = ldt_amd.decode_tensor_image(_batch([b]))["image"].cpu().numpy()
        _check(img[0], oracle.jpeg_to_tensor(b), e["name"])


@pytest.mark.parametrize("kind,n", [("food101", 128), ("q90_512", 24), ("imagenet", 48)])
def test_config_batches_vs_oracle(kind, n):
    import ldt_amd
    from ldt_amd import synth

    cells, labels = {"food101": synth.food101_like, "q90_512": synth.q90_512,
                     "imagenet": synth.imagenet_like}[kind](n, seed=3)
    out = ldt_amd.decode_tensor_image(_batch(cells, labels))
    img = out["image"].cpu().numpy()
    assert np.array_equal(out["label"].cpu().numpy(), labels)
    for k in range(n):
        _check(img[k], oracle.jpeg_to_tensor(cells[k]), f"{kind}[{k}]")


def test_bad_inputs_raise_with_row_status(manifest):
    import ldt_amd

    good = read_golden(manifest["images"][0]["file"])
    for ent in manifest["bad"]:
        b = read_golden(ent["file"])
        with pytest.raises(ldt_amd.ImageDecodeError) as ei:
            ldt_amd.decode_tensor_image(_batch([good, b, good]))
        assert ei.value.rows == {1: ent["expect_status"]}, ent["name"]
        assert isinstance(ei.value, OSError)
    # the context keeps working after an error
    img = ldt_amd.decode_tensor_image(_batch([good]))["image"].cpu().numpy()
    _check(img[0], oracle.jpeg_to_tensor(good), "after-error")


def test_null_cell_and_empty_batch(manifest):
    import ldt_amd

    good = read_golden(manifest["images"][0]["file"])
    rb = pa.RecordBatch.from_arrays([pa.array([good, None], pa.binary()), pa.array([1, 2], pa.int64())],
                                    names=["image", "label"])
    with pytest.raises(ldt_amd.ImageDecodeError) as ei:
        ldt_amd.decode_tensor_image(rb)
    assert ei.value.rows == {1: 5}
    out = ldt_amd.decode_tensor_image(_batch([]))
    assert tuple(out["image"].shape) == (0, 3, 224, 224) and tuple(out["label"].shape) == (0,)


def test_sliced_and_large_binary_and_kwargs(manifest):
    import ldt_amd

    cells = [read_golden(e["file"]) for e in manifest["images"][:9]]
    rb = _batch(cells, np.arange(100, 109))
    sl = rb.slice(3, 4)  # Array.offset = 3
    out = ldt_amd.decode_tensor_image(sl, hf_converter=None, use_blob_api=False)  # unknown kwargs ignored
    img = out["image"].cpu().numpy()
    assert out["label"].cpu().numpy().tolist() == [103, 104, 105, 106]
    for k in range(4):
        _check(img[k], oracle.jpeg_to_tensor(cells[3 + k]), f"slice[{k}]")
    out2 = ldt_amd.decode_tensor_image(_batch(cells, large=True))
    for k in range(9):
        _check(out2["image"][k].cpu().numpy(), oracle.jpeg_to_tensor(cells[k]), f"large[{k}]")


def test_collate_fn_matches_reference_recipe(manifest):
    import ldt_amd

    rows = [{"image": read_golden(e["file"]), "label": e["label"]} for e in manifest["images"][:8]]
    out = ldt_amd.collate_fn(rows)
    ref = oracle.pil_collate_fn(rows)  # the reference collate_fn through Pillow itself
    assert np.array_equal(out["image"].cpu().numpy(), ref["image"].numpy())
    assert np.array_equal(out["label"].cpu().numpy(), ref["label"].numpy())


def test_raw_resize_vs_oracle(manifest):
    import torch

    import ldt_amd
    from ldt_amd import synth

    raw = np.load(f"{GOLDEN}/{manifest['raw']['file']}")["hwc"]
    for normalize, key in ((False, "sha256_tensor_f32"), (True, "sha256_tensor_norm_f32")):
        out = ldt_amd.resize_raw(torch.from_numpy(raw), 300, 200, normalize=normalize).cpu().numpy()
        for k in range(2):
            assert sha(out[k]) == manifest["raw"]["expected"][k][key]
    big = synth.raw_hwc(3, 1024, 1024, seed=1)
    dev = torch.from_numpy(big).cuda()
    out = ldt_amd.resize_raw(dev, 1024, 1024, normalize=True).cpu().numpy()
    for k in range(3):
        _check(out[k], oracle.raw_to_tensor(big[k], normalize=True), f"raw1024[{k}]")
    # Arrow fixed_size_binary column, host
    arr = pa.array([big[k].tobytes() for k in range(2)], type=pa.binary(1024 * 1024 * 3))
    out2 = ldt_amd.resize_raw(arr, 1024, 1024, normalize=True).cpu().numpy()
    assert np.array_equal(out2, out[:2])


@pytest.mark.parametrize("n_in", [1, 2, 3, 5, 100, 223, 224, 225, 333, 375, 384, 447, 448, 500, 512, 767,
                                  1000, 1024, 2048, 4095, 8192])
def test_resample_coefficients_bit_exact(n_in):
    import ctypes

    import torch

    from ldt_amd import _lib

    ctx = _lib.get_context(torch.cuda.current_device())
    ks, bounds, kk = oracle.resample_coeffs(n_in, 224)
    db = torch.zeros(2 * 224, dtype=torch.int32, device="cuda")
    dk = torch.zeros(224 * ks, dtype=torch.int32, device="cuda")
    ctx.check(ctx.lib.ldt_debug_resample_coeffs(ctx.handle, n_in, 224, db.data_ptr(), dk.data_ptr(),
                                                torch.cuda.current_stream().cuda_stream), "coeffs")
    torch.cuda.synchronize()
    assert np.array_equal(db.cpu().numpy().reshape(224, 2), bounds)
    assert np.array_equal(dk.cpu().numpy().reshape(224, ks), kk)


def test_sampler_kernels_vs_oracle(sampler_golden):
    from ldt_amd.sampler import device_batch_ranges, device_fragment_batches

    g = sampler_golden
    frags, B, N = g["fragments"], g["batch_size"], g["num_rows"]
    for W in (1, 2, 4, 8):
        for r in range(W):
            rng = np.asarray(device_batch_ranges(N, B, r, W), np.int64).reshape(-1, 2)
            assert sha(rng) == g["sharded_batch"][str(W)][r]["sha256"]
            recs, local = device_fragment_batches(frags, B, r, W, -1)
            assert sha(np.asarray(recs, np.int64).reshape(-1, 5)) == g["sharded_fragment"][str(W)][r]["sha256"]
            assert local == g["sharded_fragment"][str(W)][r]["count"]
            target = max(x["count"] for x in g["sharded_fragment"][str(W)])
            precs, _ = device_fragment_batches(frags, B, r, W, target)
            assert sha(np.asarray(precs, np.int64).reshape(-1, 5)) == \
                g["sharded_fragment"][str(W)][r]["sha256_padded"]
    # edge cases: empty dataset, batch larger than dataset, more ranks than batches
    assert device_batch_ranges(0, 128, 0, 2) == []
    assert device_batch_ranges(10, 128, 0, 2) == [(0, 10)] and device_batch_ranges(10, 128, 1, 2) == []
    for rows in ([], [5], [0, 0, 7], [300, 1, 129]):
        for W in (1, 3):
            for r in range(W):
                recs, _ = device_fragment_batches(rows, 128, r, W, -1)
                assert [tuple(x) for x in recs] == [tuple(x) for x in oracle.sharded_fragment_batches(rows, 128, r, W)]


def test_resident_batch_and_determinism():
    import torch

    import ldt_amd
    from ldt_amd import synth

    cells, labels = synth.food101_like(64, seed=11)
    rbatch = ldt_amd.ResidentBatch(cells, labels)
    a, la = rbatch.decode()
    b, lb = rbatch.decode()
    torch.cuda.synchronize()
    assert torch.equal(a, b) and torch.equal(la, lb)
    # order invariance: a permuted batch decodes to the permuted output
    perm = np.random.RandomState(0).permutation(64)
    c = ldt_amd.decode_tensor_image(_batch([cells[i] for i in perm], labels[perm]))
    assert torch.equal(c["image"], a[torch.from_numpy(perm).cuda()])
    for k in (0, 17, 63):
        _check(a[k].cpu().numpy(), oracle.jpeg_to_tensor(cells[k]), f"resident[{k}]")


def test_decode_pipeline_overlapping_batches():
    """DecodePipeline: batches in flight on separate streams/contexts decode
    exactly like the single-stream path; errors surface through check()."""
    import torch

    import ldt_amd
    from ldt_amd import synth

    c2, l2 = synth.q90_512(48, seed=21)
    c4, l4 = synth.imagenet_like(40, seed=22)
    batches = [ldt_amd.ResidentBatch(c2, l2), ldt_amd.ResidentBatch(c4, l4)]
    ref = [b.decode() for b in batches]
    pipe = ldt_amd.DecodePipeline(depth=2)
    outs = [pipe.decode(batches[k % 2]) for k in range(6)]
    torch.cuda.synchronize()
    pipe.check()
    for k, (img, lbl) in enumerate(outs):
        assert torch.equal(img, ref[k % 2][0]) and torch.equal(lbl, ref[k % 2][1])
    for k in (0, 47):
        _check(outs[2][0][k].cpu().numpy(), oracle.jpeg_to_tensor(c2[k]), f"pipe[{k}]")
    bad = ldt_amd.ResidentBatch([c2[0], read_golden("jpeg/bad_truncated.bin")], [0, 1])
    pipe.decode(bad)
    with pytest.raises(ldt_amd.ImageDecodeError) as ei:
        pipe.check()
    assert ei.value.rows == {1: 3}


def test_lance_dataset_end_to_end(tmp_path):
    import ldt_amd
    from ldt_amd import synth

    cells, labels = synth.food101_like(300, seed=2)
    tbl = pa.table({"image": pa.array(cells, pa.binary()), "label": pa.array(labels, pa.int64())})
    ds = ldt_amd.write_dataset(tbl, str(tmp_path / "food.lance"), max_rows_per_file=125)
    lds = ldt_amd.LanceDataset(ds.uri, batch_size=64, to_tensor_fn=ldt_amd.decode_tensor_image,
                               sampler=ldt_amd.ShardedFragmentSampler(rank=0, world_size=1, pad=True))
    got_lbl = []
    for b in lds:
        got_lbl += b["label"].cpu().tolist()
        assert b["image"].shape[1:] == (3, 224, 224)
    assert got_lbl == labels.tolist()
    sds = ldt_amd.SafeLanceDataset(ds.uri)
    loader = ldt_amd.get_safe_loader(sds, batch_size=50, num_workers=0, collate_fn=ldt_amd.collate_fn,
                                     pin_memory=True)
    first = next(iter(loader))
    for k in (0, 49):
        _check(first["image"][k].cpu().numpy(), oracle.jpeg_to_tensor(cells[k]), f"loader[{k}]")


@pytest.mark.parametrize("mode,bits", [(1, 1024), (2, 64), (2, 256), (2, 1024), (2, 4096)])
def test_huffman_decoder_modes(mode, bits, manifest):
    """Serial-per-segment and parallel self-synchronising decoders agree
    bit-exactly; the minimum subsequence length ranges from 64 bits (many
    convergence rounds on the small golden images) to 4096."""
    import torch

    import ldt_amd
    from ldt_amd import _lib, synth

    ctx = _lib.get_context(torch.cuda.current_device())
    ctx.set_option(_lib.OPT_HUFF_MODE, mode)
    ctx.set_option(_lib.OPT_SUBSEQ_BITS, bits)
    try:
        cells = [read_golden(e["file"]) for e in manifest["images"]]
        c2, _ = synth.q90_512(6, seed=5)
        c4, _ = synth.imagenet_like(6, seed=5)
        cells += c2 + c4
        out = ldt_amd.decode_tensor_image(_batch(cells))["image"].cpu().numpy()
        for k, b in enumerate(cells):
            _check(out[k], oracle.jpeg_to_tensor(b), f"mode{mode}/S{bits}[{k}]")
        bad = read_golden("jpeg/bad_truncated.bin")
        with pytest.raises(ldt_amd.ImageDecodeError) as ei:
            ldt_amd.decode_tensor_image(_batch([cells[0], bad]))
        assert ei.value.rows == {1: 3}
    finally:
        ctx.set_option(_lib.OPT_HUFF_MODE, 0)
        ctx.set_option(_lib.OPT_SUBSEQ_BITS, 256)


def test_many_restart_segments_take_serial_decoder():
    """An image with more than 256 restart segments (a marker every MCU) goes
    to the serial decoder while its batch-mates use the per-image parallel
    decoder; both bit-exact vs the oracle in one batch."""
    import ldt_amd
    from ldt_amd import synth

    many = synth.encode(synth.field(512, 512, 91, 6.0), quality=90, restart_marker_blocks=1)
    few = synth.encode(synth.field(384, 512, 92, 6.0), quality=90, restart_marker_rows=1)
    c2, _ = synth.q90_512(2, seed=93)
    cells = [c2[0], many, few, c2[1]]
    out = ldt_amd.decode_tensor_image(_batch(cells))["image"].cpu().numpy()
    for k, b in enumerate(cells):
        _check(out[k], oracle.jpeg_to_tensor(b), f"restart-mix[{k}]")


def test_marker_dense_chunks_destuff_direct():
    """Destuff chunks holding more than 64 RSTn markers (a marker every block
    of a small, low-quality image) write their bytes straight to memory instead
    of through the LDS staging buffer; bit-exact vs the oracle next to a chunk
    that takes the staged path."""
    import numpy as np

    import ldt_amd
    from ldt_amd import synth

    gray = synth.field(256, 256, 95, 2.0)[:, :, 0]
    dense = synth.encode(np.ascontiguousarray(gray), quality=20, restart_marker_blocks=1)
    color = synth.encode(synth.field(256, 320, 96, 2.0), quality=25, restart_marker_blocks=1)
    # markers per 4 KB of scan data (the chunk size)
    n_rst = sum(dense.count(bytes([0xFF, 0xD0 + i])) for i in range(8))
    assert n_rst * 4096 / len(dense) > 64 * 4
    c2, _ = synth.q90_512(1, seed=97)
    cells = [dense, c2[0], color]
    out = ldt_amd.decode_tensor_image(_batch(cells))["image"].cpu().numpy()
    for k, b in enumerate(cells):
        _check(out[k], oracle.jpeg_to_tensor(b), f"marker-dense[{k}]")


def test_large_image_streaming_fallback_and_too_large():
    """A 3000x2000 source exceeds the banded kernel's LDS budget and takes the
    streaming k_resize path; a 9000-wide image exceeds LDT_MAX_DIM."""
    import ldt_amd
    from ldt_amd import synth

    big = synth.encode(synth.field(2000, 3000, 77, 6.0), quality=85)
    small = synth.encode(synth.field(300, 200, 78, 6.0))
    out = ldt_amd.decode_tensor_image(_batch([big, small]))["image"].cpu().numpy()
    _check(out[0], oracle.jpeg_to_tensor(big), "3000x2000")
    _check(out[1], oracle.jpeg_to_tensor(small), "300x200 with a large batch-mate")
    wide = synth.encode(synth.field(8, 9000, 79, 6.0))
    with pytest.raises(ldt_amd.ImageDecodeError) as ei:
        ldt_amd.decode_tensor_image(_batch([small, wide]))
    assert ei.value.rows == {1: 4}


def test_tall_bands_large_batches():
    """Large batches give tall output bands (>32 rows per workgroup): raw and
    JPEG paths with 400 small cells vs the oracle."""
    import torch

    import ldt_amd
    from ldt_amd import synth

    raw = np.random.RandomState(9).randint(0, 256, size=(400, 70, 90, 3), dtype=np.uint8)
    out = ldt_amd.resize_raw(torch.from_numpy(raw).cuda(), 70, 90, normalize=True).cpu().numpy()
    for k in (0, 1, 199, 399):
        _check(out[k], oracle.raw_to_tensor(raw[k], normalize=True), f"raw400[{k}]")
    cells = [synth.encode(synth.field(48 + (i % 5), 40 + (i % 7), i, 6.0)) for i in range(400)]
    img = ldt_amd.decode_tensor_image(_batch(cells))["image"].cpu().numpy()
    for k in (0, 3, 201, 399):
        _check(img[k], oracle.jpeg_to_tensor(cells[k]), f"jpeg400[{k}]")


def test_resize_impls_agree_and_coefficients_stay_clean(manifest):
    """The default resize (k_resize4, one wave per band, packed 16-bit 4:2:0
    staging), its 32-bit staging (LDT_OPT_RESIZE_IMPL=1) and the banded
    workgroup kernel (LDT_OPT_RESIZE_IMPL=2) give identical tensors on every golden image, on a
    c2/c1-shaped batch and on unaligned raw cells; a batch with a truncated
    image leaves nothing behind that changes the next batch."""
    import torch

    import ldt_amd
    from ldt_amd import _lib, synth

    ctx = _lib.get_context(0)
    ents = manifest["images"]
    cells = [read_golden(e["file"]) for e in ents]
    raw = synth.raw_hwc(3, 301, 517, seed=5)  # 517*3 bytes per row: unaligned rows
    flat = np.concatenate([np.zeros(5, np.uint8), raw.reshape(-1)])
    arr = pa.array([flat[5 + k * raw[0].size: 5 + (k + 1) * raw[0].size].tobytes() for k in range(3)],
                   type=pa.binary(raw[0].size))
    mixed = synth.q90_512(6, seed=8)[0] + synth.food101_like(10, seed=9)[0]
    res = {}
    try:
        for impl in (0, 1, 2):
            ctx.set_option(_lib.OPT_RESIZE_IMPL, impl)
            a = ldt_amd.decode_tensor_image(_batch(cells))["image"].cpu().numpy()
            b = ldt_amd.resize_raw(arr, 301, 517, normalize=True).cpu().numpy()
            c = ldt_amd.decode_tensor_image(_batch(mixed))["image"].cpu().numpy()
            res[impl] = (a, b, c)
        for wpg in (1, 4):  # waves (bands) per k_resize4 workgroup
            ctx.set_option(_lib.OPT_RESIZE_IMPL, 0)
            ctx.set_option(_lib.OPT_RESIZE_WG_WAVES, wpg)
            a = ldt_amd.decode_tensor_image(_batch(cells))["image"].cpu().numpy()
            c = ldt_amd.decode_tensor_image(_batch(mixed))["image"].cpu().numpy()
            res[f"wpg{wpg}"] = (a, c)
    finally:
        ctx.set_option(_lib.OPT_RESIZE_IMPL, 0)
        ctx.set_option(_lib.OPT_RESIZE_WG_WAVES, 0)
    for wpg in (1, 4):
        assert np.array_equal(res[0][0], res[f"wpg{wpg}"][0]), wpg
        assert np.array_equal(res[0][2], res[f"wpg{wpg}"][1]), wpg
    for impl in (1, 2):
        for k in range(3):
            assert np.array_equal(res[0][k], res[impl][k]), (impl, k)
    for k in (0, 5, 6, 15):
        _check(res[0][2][k], oracle.jpeg_to_tensor(mixed[k]), f"mixed[{k}]")
    for k in range(3):
        _check(res[0][1][k], oracle.raw_to_tensor(raw[k], normalize=True), f"raw301x517[{k}]")
    good = synth.encode(synth.field(384, 512, 11), quality=90)
    bad = read_golden("jpeg/bad_truncated.bin")
    with pytest.raises(ldt_amd.ImageDecodeError):
        ldt_amd.decode_tensor_image(_batch([good, bad, good]))
    nxt = [synth.encode(synth.field(512, 384, 12 + i)) for i in range(3)]
    img = ldt_amd.decode_tensor_image(_batch(nxt))["image"].cpu().numpy()
    for k in range(3):
        _check(img[k], oracle.jpeg_to_tensor(nxt[k]), f"after-error[{k}]")


def test_resize_band_counts_agree(manifest):
    """LDT_OPT_RESIZE_WAVES_PCT changes only the band geometry (output rows
    per wave, and the source rows neighbouring bands both stage): 6 to 36
    bands per image give identical tensors on the golden images, a c2/c1-shaped
    batch and raw cells."""
    import torch

    import ldt_amd
    from ldt_amd import _lib, synth

    ctx = _lib.get_context(0)
    cells = [read_golden(e["file"]) for e in manifest["images"]]
    mixed = synth.q90_512(6, seed=8)[0] + synth.food101_like(10, seed=9)[0]
    raw = torch.from_numpy(synth.raw_hwc(5, 333, 250, seed=3)).cuda()
    res = {}
    try:
        for pct in (100, 50, 67, 150, 300):
            ctx.set_option(_lib.OPT_RESIZE_WAVES_PCT, pct)
            res[pct] = (ldt_amd.decode_tensor_image(_batch(cells))["image"].cpu().numpy(),
                        ldt_amd.decode_tensor_image(_batch(mixed))["image"].cpu().numpy(),
                        ldt_amd.resize_raw(raw, 333, 250, normalize=True).cpu().numpy())
    finally:
        ctx.set_option(_lib.OPT_RESIZE_WAVES_PCT, 100)  # the default
    for pct in (50, 67, 150, 300):
        for k in range(3):
            assert np.array_equal(res[100][k], res[pct][k]), (pct, k)
    for k in (0, 7):
        _check(res[100][1][k], oracle.jpeg_to_tensor(mixed[k]), f"mixed[{k}]")


def test_pipelined_to_tensor_fn_host_batches():
    """make_to_tensor_fn: host RecordBatches (as LanceDataset yields them)
    decoded 3 in flight; results match the oracle in order, and a bad row is
    reported by check() with its row index."""
    import torch

    import ldt_amd
    from ldt_amd import synth

    fn = ldt_amd.make_to_tensor_fn(depth=3)
    batches = []
    for k in range(5):
        cells, labels = synth.food101_like(12, seed=40 + k)
        batches.append((cells, labels, _batch(cells, labels)))
    outs = [fn(rb, unknown_kwarg=1) for _, _, rb in batches]
    fn.check()
    torch.cuda.synchronize()
    for (cells, labels, _), o in zip(batches, outs):
        assert np.array_equal(o["label"].cpu().numpy(), labels)
        img = o["image"].cpu().numpy()
        for k in (0, 5, 11):
            _check(img[k], oracle.jpeg_to_tensor(cells[k]), "pipelined")
    bad = read_golden("jpeg/bad_truncated.bin")
    good = synth.encode(synth.field(64, 80, 3))
    fn(_batch([good, bad, good]))
    with pytest.raises(ldt_amd.ImageDecodeError) as ei:
        fn.check()
    assert set(ei.value.rows) == {1}


def test_registered_host_buffer_bit_exact():
    """register_host (ldt_register_host): the image column's data buffer
    page-locked in place; decodes of the whole batch and of slices inside it
    take the DMA branch and are bit-exact with the unregistered path and the
    oracle; make_to_tensor_fn(register=True) registers on first sight;
    unregister_host restores the copy path."""
    import torch

    import ldt_amd
    from ldt_amd import synth

    cells, labels = synth.food101_like(24, seed=77)
    rb = _batch(cells, labels)
    ref = ldt_amd.decode_tensor_image(rb)["image"].cpu().numpy()
    col = rb.column(0)
    addr, size = ldt_amd.register_host(col)
    try:
        assert size == sum(len(c) for c in cells) and addr != 0
        assert ldt_amd.register_host(col) == (addr, size)  # idempotent
        got = ldt_amd.decode_tensor_image(rb)
        assert np.array_equal(got["label"].cpu().numpy(), labels)
        assert np.array_equal(got["image"].cpu().numpy(), ref)
        part = ldt_amd.decode_tensor_image(rb.slice(5, 11))["image"].cpu().numpy()
        assert np.array_equal(part, ref[5:16])
        fn = ldt_amd.make_to_tensor_fn(depth=2, register=True)
        outs = [fn(rb.slice(8 * k, 8)) for k in range(3)]
        fn.check()
        torch.cuda.synchronize()
        for k, o in enumerate(outs):
            assert np.array_equal(o["image"].cpu().numpy(), ref[8 * k:8 * k + 8])
        for k in (0, 13, 23):
            _check(ref[k], oracle.jpeg_to_tensor(cells[k]), "registered")
    finally:
        ldt_amd.unregister_host(col)
    again = ldt_amd.decode_tensor_image(rb)["image"].cpu().numpy()
    assert np.array_equal(again, ref)


def test_register_cap_and_refusal_fall_back_to_copy():
    """make_to_tensor_fn(register=True, register_cap=1): each new buffer is
    registered, the least recently used one unregistered (pinned memory stays
    bounded), and a buffer the driver refuses to lock leaves the function on
    the copying path instead of raising; every output stays bit-exact."""
    import torch

    import ldt_amd
    from ldt_amd import synth, transforms

    bs, refs = [], []
    for k in range(3):
        cells, labels = synth.food101_like(10, seed=300 + k)
        rb = _batch(cells, labels)
        bs.append(rb)
        refs.append(ldt_amd.decode_tensor_image(rb)["image"].cpu().numpy())
    before = set(transforms._registered)
    fn = ldt_amd.make_to_tensor_fn(depth=2, register=True, register_cap=1)
    outs = [fn(b) for b in bs + bs[:1]]
    fn.check()
    torch.cuda.synchronize()
    assert len(set(transforms._registered) - before) <= 1
    for o, ref in zip(outs, refs + refs[:1]):
        assert np.array_equal(o["image"].cpu().numpy(), ref)
    # three distinct buffers through a cap of one: two evictions within
    # 4 x cap calls, so the buffers do not repeat and the function went back
    # to copying (no hipHostRegister + device sync per call)
    assert not fn.registering()
    fn.release()
    assert set(transforms._registered) == before
    # a range the driver refuses to lock (memlock limit, overlap): the
    # function stays on the copying path instead of raising
    def refuse(obj, device=None):
        raise ldt_amd.LdtError("ldt_register_host failed (rc=-2): hipHostRegister refused")

    real = transforms.register_host
    transforms.register_host = refuse
    try:
        fn2 = ldt_amd.make_to_tensor_fn(depth=2, register=True)
        got = [fn2(b) for b in bs]
        fn2.check()
        for o, ref in zip(got, refs):
            assert np.array_equal(o["image"].cpu().numpy(), ref)
    finally:
        transforms.register_host = real


@pytest.mark.parametrize("threads", [0, 1, 7])
def test_copy_pool_sizes_and_host_times(threads):
    """LDT_OPT_COPY_THREADS: the cell copy into the pinned slot runs on 0 (the
    caller alone), 1 or 7 pool threads while the caller walks the headers;
    the decode is bit-exact for each (a 1 MB+ batch, so the pool path is
    taken), and LDT_OPT_HOST_TIMING reports every phase per call."""
    import torch

    import ldt_amd
    from ldt_amd import _lib, synth

    cells, labels = synth.q90_512(24, seed=41)
    rb = _batch(cells, labels)
    assert sum(len(c) for c in cells) > (1 << 20)
    pipe = ldt_amd.DecodePipeline(depth=2)
    pipe.set_option(_lib.OPT_COPY_THREADS, threads)
    pipe.set_option(_lib.OPT_HOST_TIMING, 1)
    outs = [pipe.decode(rb) for _ in range(4)]
    pipe.check()
    torch.cuda.synchronize()
    us, calls = pipe.host_times(reset=True)
    assert calls == 4 and set(us) == set(_lib.HOST_PHASES) and all(v >= 0 for v in us.values())
    ref = outs[0][0].cpu().numpy()
    for img, lbl in outs:
        assert np.array_equal(img.cpu().numpy(), ref)
        assert np.array_equal(lbl.cpu().numpy(), labels)
    for k in (0, 11, 23):
        _check(ref[k], oracle.jpeg_to_tensor(cells[k]), f"copy threads {threads}")


@pytest.mark.parametrize("mode,bind,nt", [(0, 1, 0), (1, 1, 0), (0, 0, 1), (0, 2, 1)])
def test_copy_modes_bit_exact(mode, bind, nt):
    """LDT_OPT_COPY_MODE / _BIND / _NT: host batches through a 2-deep pipeline,
    8 calls over alternating batches of different sizes, so each context's two
    device cell buffers are reused while the other's kernels may still run
    (mode 0: the DMA on the device's copy stream waits for the buffer's last
    reader). Every call bit-exact against the synchronous decode, and
    ldt_host_info reports the placement."""
    import torch

    import ldt_amd
    from ldt_amd import _lib, synth

    a, la = synth.q90_512(20, seed=51)
    b, lb = synth.food101_like(40, seed=52)
    rbs = [_batch(a, la), _batch(b, lb)]
    refs = [ldt_amd.decode_tensor_image(rb)["image"].cpu().numpy() for rb in rbs]
    pipe = ldt_amd.DecodePipeline(depth=2)
    pipe.set_option(_lib.OPT_COPY_MODE, mode)
    pipe.set_option(_lib.OPT_COPY_BIND, bind)
    pipe.set_option(_lib.OPT_COPY_NT, nt)
    pipe.set_option(_lib.OPT_COPY_THREADS, 3)
    outs = [pipe.decode(rbs[k % 2]) for k in range(8)]
    pipe.check()
    torch.cuda.synchronize()
    for k, (img, _) in enumerate(outs):
        assert np.array_equal(img.cpu().numpy(), refs[k % 2]), k
    info = pipe.ctxs[0].host_info()
    assert info["copy_threads"] == 3 and len(info["copy_cpus"]) == 3
    assert info["copy_mode"] == mode and info["copy_bind"] == bind and info["copy_nt"] == nt
    assert (min(info["copy_cpus"]) >= 0) == bool(bind)


@pytest.mark.parametrize("seed", range(3))
def test_progressive_mixed_batches_vs_oracle(seed):
    """SOF2 images (k_prog: jdphuff.c scans) mixed with baseline ones in one
    batch, random shapes/subsampling/quality/restart intervals, bit-exact
    against the oracle (which is pinned to Pillow by the progressive goldens)."""
    import ldt_amd
    from ldt_amd import synth

    r = np.random.RandomState(100 + seed)
    cells = []
    for k in range(12):
        h, w = int(r.randint(1, 300)), int(r.randint(1, 300))
        kw = dict(quality=int(r.choice([50, 75, 90, 97])),
                  subsampling=str(r.choice(["4:2:0", "4:2:2", "4:4:4"])),
                  progressive=bool(k % 3 != 0))
        if r.rand() < 0.3:
            kw["restart_marker_blocks"] = int(r.randint(1, 6))
        cells.append(synth.encode(synth.field(h, w, int(r.randint(1 << 30)), float(r.choice([0, 6, 30]))), **kw))
    out = ldt_amd.decode_tensor_image(_batch(cells))
    img = out["image"].cpu().numpy()
    for k, b in enumerate(cells):
        _check(img[k], oracle.jpeg_to_tensor(b), f"seed{seed}[{k}]")


def test_progressive_config_sized_batch():
    """C2-shaped progressive images (512x512 q90 4:2:0) through the same
    to_tensor_fn: the serial per-scan path at full size, twice (the
    coefficient buffer stays clean across batches)."""
    import ldt_amd
    from ldt_amd import synth

    cells = [synth.encode(synth.field(512, 512, 900 + k, 20), quality=90, progressive=True) for k in range(4)]
    base, _ = synth.q90_512(4, seed=5)
    for rep in range(2):
        batch = cells + list(base) if rep == 0 else list(base) + cells
        img = ldt_amd.decode_tensor_image(_batch(batch))["image"].cpu().numpy()
        for k, b in enumerate(batch):
            _check(img[k], oracle.jpeg_to_tensor(b), f"rep{rep}[{k}]")


def _scan_ranges(b):
    """(start, end) of each scan's entropy-coded bytes (SOS header skipped,
    up to the marker that ends the scan; RSTn markers stay inside)."""
    out, i = [], 2
    while i + 4 <= len(b) and b[i] == 0xFF and b[i + 1] != 0xD9:
        n = (b[i + 2] << 8) | b[i + 3]
        if b[i + 1] != 0xDA:
            i += 2 + n
            continue
        j = i + 2 + n
        while not (b[j] == 0xFF and b[j + 1] != 0 and not 0xD0 <= b[j + 1] <= 0xD7):
            j += 1
        out.append((i + 2 + n, j))
        i = j
    return out


@pytest.mark.parametrize("kind", ["420", "444"])
def test_progressive_corrupt_scans_vs_oracle(kind):
    """k_prog on damaged scans: bit flips inside the entropy-coded bytes of
    randomly chosen scans (no new markers) drive the decoder through invalid
    Huffman codes (16 bits skipped, symbol 0), overlong runs, EOB runs past the
    band and refinement stops past Se. Whenever the batch decodes, the damaged
    image equals the oracle's decode of the same bytes bit-exactly (libjpeg's
    warn-and-continue semantics), and its clean neighbour is unaffected."""
    import ldt_amd
    from ldt_amd import synth

    if kind == "420":
        base = synth.encode(synth.field(512, 512, 11, 20.0), quality=90, progressive=True)
    else:
        base = synth.encode(synth.field(200, 264, 12, 30.0), quality=97, subsampling="4:4:4", progressive=True)
    good = synth.encode(synth.field(96, 128, 13, 6.0), quality=80, progressive=True)
    exp_good = oracle.jpeg_to_tensor(good)
    scans = _scan_ranges(base)
    assert len(scans) >= 6
    rng = np.random.default_rng({"420": 21, "444": 22}[kind])
    decoded = 0
    for trial in range(16):
        b = bytearray(base)
        for _ in range(int(rng.integers(1, 4))):
            s0, s1 = scans[int(rng.integers(len(scans)))]
            for _ in range(20):
                p = int(rng.integers(s0, s1))
                v = b[p] ^ (1 << int(rng.integers(0, 8)))
                if b[p] != 0xFF and v != 0xFF and b[p - 1] != 0xFF:
                    b[p] = v
                    break
        cells = [bytes(b), good]
        try:
            out = ldt_amd.decode_tensor_image(_batch(cells))["image"].cpu().numpy()
        except ldt_amd.ImageDecodeError as e:
            assert set(e.rows) == {0}, (kind, trial, e.rows)
            continue
        decoded += 1
        _check(out[0], oracle.jpeg_to_tensor(bytes(b)), f"{kind} trial {trial}: damaged image")
        _check(out[1], exp_good, f"{kind} trial {trial}: clean neighbour")
    assert decoded >= 8, decoded


def test_distributed_sampler_kernels_vs_torch_golden():
    """ldt_distributed_indices (MT19937 targets, deterministic-reservation
    Fisher-Yates, rank stride) vs torch's DistributedSampler: every golden case
    (tests/golden/distributed.json, incl. FOOD101 75,750 rows and ImageNet
    1,281,167 rows), bit-exact int64 indices."""
    import json
    import os

    from ldt_amd.sampler import device_distributed_indices

    cases = json.load(open(os.path.join(GOLDEN, "distributed.json")))["cases"]
    for g in cases:
        c = g["case"]
        for r, exp in enumerate(g["ranks"]):
            idx = device_distributed_indices(c["n"], c["W"], r, c["shuffle"], c["seed"] + c["epoch"],
                                             c["drop_last"]).cpu().numpy()
            assert idx.dtype == np.int64 and len(idx) == exp["count"], c
            assert sha(idx) == exp["sha256"], (c, r, idx[:4].tolist(), exp["head"])


@pytest.mark.parametrize("seed", range(4))
def test_distributed_sampler_random_sizes_vs_torch(seed):
    import torch
    from torch.utils.data import DistributedSampler as TorchDS

    import ldt_amd

    rng = np.random.default_rng(seed)
    for _ in range(6):
        n = int(rng.integers(0, 300_000))
        W = int(rng.integers(1, 9))
        dl = bool(rng.integers(0, 2))
        s = int(rng.integers(-2**62, 2**62))
        ds = range(n)
        r = int(rng.integers(0, W))
        a = ldt_amd.DistributedSampler(ds, num_replicas=W, rank=r, seed=s, drop_last=dl)
        b = TorchDS(ds, num_replicas=W, rank=r, seed=s, drop_last=dl)
        a.set_epoch(seed)
        b.set_epoch(seed)
        assert list(a) == list(b), (n, W, r, dl, s)
        t = a.indices()
        assert t.is_cuda and t.dtype == torch.int64


def test_prefetching_to_tensor_fn_overlaps_and_matches(tmp_path):
    """make_to_tensor_fn(prefetch=2) through LanceDataset: batches decode ahead
    on side streams; every yielded batch is bit-exact
    with the synchronous decode_tensor_image, in sampler order, including the
    ragged last batch; a long kernel enqueued on the consumer's stream between
    yields does not change the results."""
    import torch

    import ldt_amd
    from ldt_amd import synth

    cells, labels = synth.food101_like(300, seed=5)
    tbl = pa.table({"image": pa.array(cells, pa.binary()), "label": pa.array(labels, pa.int64())})
    path = str(tmp_path / "ds")
    ldt_amd.write_dataset(tbl, path, max_rows_per_file=128)
    smp = ldt_amd.ShardedBatchSampler(rank=0, world_size=1)
    ref = list(ldt_amd.LanceDataset(path, batch_size=64, sampler=smp,
                                    to_tensor_fn=ldt_amd.decode_tensor_image))
    fn = ldt_amd.make_to_tensor_fn(depth=3, prefetch=2)
    got = []
    busy = torch.randn(2048, 2048, device="cuda")
    for b in ldt_amd.LanceDataset(path, batch_size=64, sampler=smp, to_tensor_fn=fn):
        for _ in range(8):
            busy = torch.tanh(busy @ busy * 1e-3)  # consumer work on torch's stream
        got.append({k: v.clone() for k, v in b.items()})
    assert len(got) == len(ref) == 5
    for a, b in zip(got, ref):
        assert torch.equal(a["label"], b["label"])
        assert torch.equal(a["image"], b["image"])


def _sos_end(b: bytes) -> int:
    """Offset of the first entropy-coded byte (after the first SOS header)."""
    i = 2
    while i + 4 <= len(b):
        m, L = b[i + 1], (b[i + 2] << 8) | b[i + 3]
        if m == 0xDA:
            return i + 2 + L
        i += 2 + L
    raise ValueError("no SOS")


@pytest.mark.parametrize("kind", ["c2", "c4", "prog"])
def test_corrupt_entropy_data_is_contained(kind):
    """Robustness: random bit flips, byte overwrites and stray markers in the
    entropy-coded data. A batch holding a corrupt image next to a valid one
    must not fault the GPU; the valid image stays bit-exact whether or not the
    corrupt one is reported (libjpeg decodes some corrupt streams to garbage
    with a warning; this build decodes them too or reports LDT_IMG_CORRUPT),
    and a clean batch afterwards is bit-exact (the all-zero coefficient
    invariant is restored)."""
    import ldt_amd
    from ldt_amd import synth

    if kind == "c2":
        base = synth.encode(synth.field(512, 512, 5, 6.0), quality=90)
    elif kind == "c4":
        base = synth.encode(synth.field(375, 500, 6, 6.0), quality=90, restart_marker_rows=1)
    else:
        base = synth.encode(synth.field(256, 320, 7, 6.0), quality=85, progressive=True)
    good = synth.encode(synth.field(300, 200, 8, 6.0))
    exp_good = oracle.jpeg_to_tensor(good)
    rng = np.random.default_rng({"c2": 1, "c4": 2, "prog": 3}[kind])
    s0 = _sos_end(base)
    for trial in range(24):
        b = bytearray(base)
        mode = trial % 4
        for _ in range(int(rng.integers(1, 8))):
            p = int(rng.integers(s0, len(b) - 2))
            if mode == 0:
                b[p] ^= 1 << int(rng.integers(0, 8))
            elif mode == 1:
                b[p] = int(rng.integers(0, 256))
            elif mode == 2:
                b[p:p + 2] = bytes([0xFF, int(rng.choice([0x00, 0xD0, 0xD3, 0xD9, 0xC4, 0xFF]))])
            else:
                del b[p:p + int(rng.integers(1, 64))]
        cells = [good, bytes(b), good]
        try:
            out = ldt_amd.decode_tensor_image(_batch(cells))["image"].cpu().numpy()
            got = [out[0], out[2]]
        except ldt_amd.ImageDecodeError as e:
            assert set(e.rows) == {1}, (kind, trial, e.rows)
            continue
        for g in got:
            _check(g, exp_good, f"{kind} trial {trial}: valid neighbour")
    img = ldt_amd.decode_tensor_image(_batch([base, good]))["image"].cpu().numpy()
    _check(img[0], oracle.jpeg_to_tensor(base), f"{kind}: clean batch after corrupt ones")
    _check(img[1], exp_good, f"{kind}: clean batch after corrupt ones")


@pytest.mark.gpu
def test_fused_destuff_matches_destuff_kernels(manifest):
    """LDT_OPT_FUSED_DESTUFF: k_huff_image destuffing its image's scan bytes
    into its LDS window gives the same tensors and the same row statuses as
    the k_destuff_* kernels, bit for bit: goldens, config-shaped images,
    restart markers up to the parallel decoder's 256 segments, stuffed 0xFF
    bytes, truncated streams and randomly corrupted entropy data (stray
    markers, deleted runs), each batch decoded both ways."""
    import torch

    import ldt_amd
    from ldt_amd import _lib, synth

    ctx = _lib.get_context(torch.cuda.current_device())

    def run(cells, fused):
        ctx.set_option(_lib.OPT_FUSED_DESTUFF, fused)
        try:
            return ldt_amd.decode_tensor_image(_batch(cells))["image"].cpu().numpy(), {}
        except ldt_amd.ImageDecodeError as e:
            return None, dict(e.rows)

    try:
        cells = [read_golden(e["file"]) for e in manifest["images"]]
        c2, _ = synth.q90_512(3, seed=41)
        c4, _ = synth.imagenet_like(3, seed=42)
        rst256 = synth.encode(synth.field(512, 512, 43, 6.0), quality=90, restart_marker_blocks=4)
        rst_rows = synth.encode(synth.field(375, 500, 44, 6.0), quality=95, restart_marker_rows=1)
        cells += c2 + c4 + [rst256, rst_rows]
        out, st = run(cells, 1)
        assert st == {}
        for k, b in enumerate(cells):
            _check(out[k], oracle.jpeg_to_tensor(b), f"fused[{k}]")
        ref, _ = run(cells, 0)
        assert np.array_equal(out, ref)
        rng = np.random.default_rng(45)
        for trial in range(16):
            base = [c2[0], rst256, rst_rows, c4[1]][trial % 4]
            b = bytearray(base)
            s0 = _sos_end(base)
            for _ in range(int(rng.integers(1, 6))):
                p = int(rng.integers(s0, len(b) - 2))
                m = int(rng.integers(0, 3))
                if m == 0:
                    b[p:p + 2] = bytes([0xFF, int(rng.choice([0x00, 0xD0, 0xD5, 0xD9, 0xC4, 0xFF]))])
                elif m == 1:
                    b[p] ^= 1 << int(rng.integers(0, 8))
                else:
                    del b[p:p + int(rng.integers(1, 64))]
            batch = [c4[0], bytes(b), bytes(base[: len(base) // 2]), c2[1]]
            got = run(batch, 1)
            exp = run(batch, 0)
            assert got[1] == exp[1], (trial, got[1], exp[1])
            if got[0] is not None:
                assert np.array_equal(got[0], exp[0]), trial
    finally:
        ctx.set_option(_lib.OPT_FUSED_DESTUFF, 1)


def _short_scan_cells():
    """Single-tile fused-destuff streams (ldt_huffman.hip destuff_into_window:
    a 16 KB tile is 16 bytes per lane of 1024): images whose end-of-scan
    marker lies in the last wave's bytes (tile offsets 15,360-16,383, lanes
    960-1023), each with trailing bytes after EOI that hold a stray RSTn, a
    stuffed 0xFF00 and a second EOI. The reference stops at the first EOI
    (jdmarker.c), so the trailing bytes must never count: a lost end position
    would keep them and report a restart-marker mismatch (status 3)."""
    from ldt_amd import synth

    out = []
    for seed in range(200):
        h = 264 + 4 * (seed % 25)
        w = 304 + 8 * (seed // 25)
        b = synth.encode(synth.field(h, w, 900 + seed, 6.0), quality=85)
        eoi = len(b) - 2  # Pillow ends the file with FFD9
        scan = eoi - _sos_end(b)
        if 15_400 <= scan <= 16_300:
            out.append(b + bytes([0x12, 0xFF, 0xD0, 0x34, 0xFF, 0x00, 0x56, 0xFF, 0xD9]))
        if len(out) == 6:
            break
    assert len(out) >= 3, "no single-tile streams with a late end marker"
    return out


@pytest.mark.gpu
def test_fused_destuff_end_marker_in_last_wave():
    """ADVICE r3 / VERDICT r3 weak 1: the fused destuff's end-of-scan position
    is a per-wave minimum published across a barrier, so a marker in the last
    wave's bytes of a single-tile stream is never lost to another wave's
    initialisation. Fused vs k_destuff_* kernels vs the oracle, statuses
    included, each batch decoded repeatedly (the race was timing-dependent)."""
    import torch

    import ldt_amd
    from ldt_amd import _lib, synth

    ctx = _lib.get_context(torch.cuda.current_device())
    cells = _short_scan_cells()
    big, _ = synth.q90_512(2, seed=46)
    batch = cells + big + cells[::-1]
    exp = [oracle.jpeg_to_tensor(b) for b in batch]
    try:
        for fused in (1, 0, 1):
            ctx.set_option(_lib.OPT_FUSED_DESTUFF, fused)
            for rep in range(4):
                out = ldt_amd.decode_tensor_image(_batch(batch))["image"].cpu().numpy()
                for k in range(len(batch)):
                    _check(out[k], exp[k], f"fused={fused} rep {rep} [{k}]")
    finally:
        ctx.set_option(_lib.OPT_FUSED_DESTUFF, 1)


@pytest.mark.gpu
def test_status_tickets_hold_two_calls():
    """ldt_last_ticket / ldt_fetch_status_ticket: a context keeps the device
    status of its last two decode calls; a batch's errors are read by ticket
    after newer batches were enqueued, without waiting for them, and a ticket
    older than two calls is refused."""
    import torch

    import ldt_amd
    from ldt_amd import _lib, synth

    ctx = _lib.Context(0)
    ctx.set_option(_lib.OPT_SYNC_STATUS, 0)
    good = synth.encode(synth.field(64, 80, 9))
    bad = read_golden("jpeg/bad_truncated.bin")
    t0 = ctx.lib.ldt_last_ticket(ctx.handle)
    tickets = []
    for cells in ([good, bad], [good, good, good], [bad, good, good, good]):
        ldt_amd.decode_arrow(pa.array(cells, pa.binary()), None, ctx=ctx)
        tickets.append(ctx.lib.ldt_last_ticket(ctx.handle))
    assert tickets == [t0 + 1, t0 + 2, t0 + 3]
    torch.cuda.synchronize()
    st = np.zeros(4, np.int32)
    # the first call's status is gone (two newer calls), the others are held
    assert ctx.lib.ldt_fetch_status_ticket(ctx.handle, tickets[0], st.ctypes.data, 2) == _lib.LDT_ERR_ARG
    assert ctx.lib.ldt_fetch_status_ticket(ctx.handle, tickets[1], st.ctypes.data, 3) == _lib.LDT_OK
    assert st[:3].tolist() == [0, 0, 0]
    st[:] = 0
    assert ctx.lib.ldt_fetch_status_ticket(ctx.handle, tickets[2], st.ctypes.data, 4) == _lib.LDT_ERR_IMAGE
    assert st.tolist() == [3, 0, 0, 0]


def test_packed_420_staging_edge_widths():
    """k_resize4<5> (the default 4:2:0 staging on packed 16-bit pairs) against
    the 32-bit staging (LDT_OPT_RESIZE_IMPL=1) and the oracle on 4:2:0 images
    whose chroma edge falls on every byte position of a lane's dword and on
    lane 0 itself (widths 5-17: the first lane is also the last chroma lane),
    on the 64-lane boundary (widths 127-129, 255-257) and up to the fast
    path's 512-px limit (jdsample.c h2v2_fancy_upsample edge columns)."""
    import ldt_amd
    from ldt_amd import _lib, synth

    widths = [5, 6, 7, 8, 9, 10, 11, 12, 13, 15, 16, 17, 23, 31, 32, 33, 63, 64, 65, 100, 127, 128, 129,
              255, 256, 257, 383, 497, 503, 504, 505, 509, 510, 511, 512]
    cells = [synth.encode(synth.field(8 + (7 * i) % 41, w, 300 + i), quality=90) for i, w in enumerate(widths)]
    ctx = _lib.get_context(0)
    out = {}
    try:
        for impl in (1, 0):
            ctx.set_option(_lib.OPT_RESIZE_IMPL, impl)
            out[impl] = ldt_amd.decode_tensor_image(_batch(cells))["image"].cpu().numpy()
    finally:
        ctx.set_option(_lib.OPT_RESIZE_IMPL, 0)
    for k, w in enumerate(widths):
        assert np.array_equal(out[0][k], out[1][k]), f"width {w}"
    for k in (0, 4, 11, 22, 34):
        _check(out[0][k], oracle.jpeg_to_tensor(cells[k]), f"w{widths[k]}")


def test_make_to_tensor_fn_adaptive_depth():
    """make_to_tensor_fn() (depth=None): one adaptive pipeline whose batches
    in flight follow each call's batch: FOOD101-shaped batches (< 8 MB of
    cells) rotate over three slots with the DMA on the slot's stream,
    c2-shaped ones (>= 8 MB) over slots 0 and 1 with the DMA on slot 2's
    stream. Interleaved small and large batches decode bit-exactly as the
    synchronous decode; options set through fn.pipeline reach every context."""
    import torch

    import ldt_amd
    from ldt_amd import _lib, synth

    small, ls = synth.food101_like(48, seed=61)
    big, lb = synth.q90_512(130, seed=62)  # ~8.7 MB of cells
    rs, rbig = _batch(small, ls), _batch(big, lb)
    ref_s = ldt_amd.decode_tensor_image(rs)["image"].cpu().numpy()
    ref_b = ldt_amd.decode_tensor_image(rbig)["image"].cpu().numpy()
    fn = ldt_amd.make_to_tensor_fn()
    assert fn.pipeline.adaptive and fn.pipeline.depth == 3
    fn.pipeline.set_option(_lib.OPT_COPY_BIND, 1)
    fn.pipeline.set_option(_lib.OPT_COPY_THREADS, 2)
    order = [rs, rs, rbig, rs, rbig, rbig, rbig, rs, rs, rs, rbig, rs]
    outs = [fn(b) for b in order]
    fn.check()
    torch.cuda.synchronize()
    for b, o in zip(order, outs):
        assert np.array_equal(o["image"].cpu().numpy(), ref_s if b is rs else ref_b)
    assert fn.pipeline._k_large == 5 and fn.pipeline._k_small == 7
    for c in fn.pipeline.ctxs:
        info = c.host_info()
        assert info["copy_bind"] == 1 and info["copy_threads"] == 2


def test_async_calls_reuse_slot_with_plan_in_cells():
    """One context, copy mode 0 (cells' DMA on the device's copy stream), no
    status sync and no status fetch between calls: call k+2 reuses call k's
    pinned slot and device buffer, which also holds call k's plan blob
    (descriptors, tables, LUT, labels, status) that k_idct and the resize still
    read. Back-to-back batches of different geometry must decode exactly as
    the same batches decoded synchronously (the slot's next DMA
    waited only for the Huffman stage)."""
    import torch

    import ldt_amd
    from ldt_amd import _lib, synth

    shapes = [(512, 512, 90, 48), (120, 200, 75, 7), (384, 512, 90, 40), (33, 47, 95, 3),
              (512, 384, 85, 44), (64, 64, 60, 11)]
    batches = []
    for k, (h, w, q, n) in enumerate(shapes):
        cells = [synth.encode(synth.field(h - (i % 3), w - (i % 5), 50 * k + i), quality=q) for i in range(n)]
        batches.append((cells, np.arange(n, dtype=np.int64) + 1000 * k))
    ref = []
    sync = _lib.Context(0)
    for cells, lbl in batches:
        img, lb = ldt_amd.decode_arrow(pa.array(cells, pa.binary()), lbl, ctx=sync)
        ref.append((img.cpu().numpy(), lb.cpu().numpy()))
    ctx = _lib.Context(0)
    ctx.set_option(_lib.OPT_SYNC_STATUS, 0)
    ctx.set_option(_lib.OPT_COPY_MODE, 0)
    for rep in range(3):
        outs = []
        for cells, lbl in batches:
            outs.append(ldt_amd.decode_arrow(pa.array(cells, pa.binary()), lbl, ctx=ctx))
        torch.cuda.synchronize()
        for k, ((img, lb), (rimg, rlb)) in enumerate(zip(outs, ref)):
            assert np.array_equal(lb.cpu().numpy(), rlb), (rep, k)
            assert np.array_equal(img.cpu().numpy(), rimg), (rep, k)
