"""GPU tests of the decoder's study options and launch fallbacks:
the diagnostic counters (LDT_OPT_DEBUG_COUNTERS) and the LDS-window cap
(LDT_OPT_HUFF_WINDOW) leave the decoded tensors unchanged, and a batch with a
tall image keeps the band kernel (k_resize4) with fewer waves per workgroup
instead of falling back to the streaming kernel."""
import numpy as np
import pytest

from conftest import read_golden
from oracle import oracle

pytestmark = pytest.mark.gpu


def _decode(cells, labels=None):
    import ldt_amd
    from ldt_amd import synth

    labels = np.arange(len(cells)) if labels is None else labels
    out = ldt_amd.decode_tensor_image(synth.arrow_batch(cells, labels))
    return out["image"].cpu().numpy(), out["label"].cpu().numpy()


@pytest.fixture(scope="module")
def option_cells(manifest):
    from ldt_amd import synth

    golden = [read_golden(e["file"]) for e in manifest["images"]]
    c2, _ = synth.q90_512(24, seed=31)
    c1, _ = synth.food101_like(24, seed=32)
    c4, _ = synth.imagenet_like(16, seed=33)
    return golden + c2 + c1 + c4


@pytest.mark.parametrize("opt,value", [("DEBUG_COUNTERS", 1), ("HUFF_WINDOW", 0), ("HUFF_WINDOW", 16384),
                                       ("HUFF_WINDOW", 40000)])
def test_study_options_leave_tensors_unchanged(option_cells, opt, value):
    """Golden images + c2/c1/c4-shaped cells: the option's run equals the
    default run bit for bit (HUFF_WINDOW 0: every stream through k_destuff_* and
    global reads; 16 KB / 40 KB: the small streams keep the fused LDS path, the
    large ones read global memory)."""
    from ldt_amd import _lib

    ctx = _lib.get_context(0)
    base_img, base_lbl = _decode(option_cells)
    default = {"DEBUG_COUNTERS": 0, "HUFF_WINDOW": -1}[opt]
    ctx.set_option(getattr(_lib, "OPT_" + opt), value)
    try:
        img, lbl = _decode(option_cells)
    finally:
        ctx.set_option(getattr(_lib, "OPT_" + opt), default)
    assert np.array_equal(lbl, base_lbl)
    bad = [k for k in range(len(option_cells)) if not np.array_equal(img[k], base_img[k])]
    assert not bad, f"{opt}={value}: images {bad[:10]} differ from the default run"


def test_debug_counters_only_when_enabled(option_cells):
    """ldt_debug_counters refuses after a batch decoded without the option and
    reports one workgroup per parallel-decoded image with it."""
    from ldt_amd import _lib

    ctx = _lib.get_context(0)
    _decode(option_cells)
    with pytest.raises(_lib.LdtError):
        ctx.debug_counters()
    ctx.set_option(_lib.OPT_DEBUG_COUNTERS, 1)
    try:
        _decode(option_cells[-40:])  # c2/c1/c4-shaped: all on the parallel decoder
        cnt = ctx.debug_counters()
    finally:
        ctx.set_option(_lib.OPT_DEBUG_COUNTERS, 0)
    assert cnt[1] == 40, cnt           # workgroups = images
    assert cnt[2] >= cnt[1] and cnt[3] >= 1, cnt  # at least one round each
    assert cnt[5] > 0 and cnt[6] > 0, cnt  # write-pass symbols
    _decode(option_cells[:2])
    with pytest.raises(_lib.LdtError):
        ctx.debug_counters()


def test_tall_image_keeps_band_kernel():
    """A 512-wide, 5000-tall image (its vertical ring does not fit four waves'
    LDS in one workgroup) in a batch with ordinary cells: k_resize4 runs with
    fewer waves per workgroup (ldt_debug_last_resize) and every image is
    bit-exact against the oracle; an ordinary batch keeps 4 waves."""
    from ldt_amd import _lib, synth

    ctx = _lib.get_context(0)
    tall = synth.encode(synth.field(5000, 512, 77, 6.0), quality=90)
    cells = [tall] + synth.q90_512(3, seed=78)[0]
    img, _ = _decode(cells)
    wpg = ctx.lib.ldt_debug_last_resize(ctx.handle)
    assert wpg in (1, 2), f"tall batch took resize path {wpg} (0 = streaming kernel)"
    for k, c in enumerate(cells):
        assert np.array_equal(img[k], oracle.jpeg_to_tensor(c)), f"image {k}"
    _decode(cells[1:])
    assert ctx.lib.ldt_debug_last_resize(ctx.handle) == 4
