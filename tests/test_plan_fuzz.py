"""Fuzz of the host JPEG header planner under AddressSanitizer + UBSan (CPU).

The planner (lance-distributed-training_amd/csrc/ldt_plan.cpp: walk_markers,
build_huff, plan_progressive) parses untrusted cell bytes on the product path
before anything reaches the GPU. This test builds it alone for the CPU with
``-fsanitize=address,undefined`` (tests/fuzz/plan_fuzz.cpp feeds each cell in a
heap buffer of exactly its size) and drives it with:

* targeted header corruptions (SOF/DHT/DQT/DRI/SOS fields), each rejected
  with the expected LDT_IMG_* code — and rejected by Pillow 12.2 too, except
  the one documented divergence (a baseline SOS with Ss != 0, which libjpeg
  decodes with a warning and this build reports as UNSUPPORTED);
* every truncation inside the headers (baseline and progressive files);
* random byte overwrites inside the marker segments of every golden image.

Any sanitizer report fails the run (-fno-sanitize-recover=all, non-zero exit).
"""
import glob
import io
import os
import shutil
import struct
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, REPO

NOT_JPEG, UNSUPPORTED, CORRUPT = 1, 2, 3
SRC = [os.path.join(REPO, "tests", "fuzz", "plan_fuzz.cpp"),
       os.path.join(REPO, "lance-distributed-training_amd", "csrc", "ldt_plan.cpp")]


@pytest.fixture(scope="module")
def planner(tmp_path_factory):
    cxx = shutil.which("g++") or shutil.which("clang++")
    if cxx is None:
        pytest.skip("no host C++ compiler")
    exe = str(tmp_path_factory.mktemp("fuzz") / "plan_fuzz")
    subprocess.run([cxx, "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                    "-I/opt/rocm/include", "-D__HIP_PLATFORM_AMD__", *SRC, "-o", exe], check=True)

    def run(cells):
        inp = b"".join(struct.pack("<I", len(c)) + c for c in cells)
        r = subprocess.run([exe], input=inp, capture_output=True, timeout=300,
                           env=dict(os.environ, ASAN_OPTIONS="detect_leaks=0"))
        assert r.returncode == 0 and not r.stderr, r.stderr.decode(errors="replace")[-4000:]
        out = [int(x) for x in r.stdout.split()]
        assert len(out) == len(cells)
        return out
    run.exe = exe
    return run


def segments(b: bytes):
    """(marker, offset of 0xFF, length field) up to and including the first SOS."""
    i, out = 2, []
    while i + 4 <= len(b):
        m, L = b[i + 1], (b[i + 2] << 8) | b[i + 3]
        out.append((m, i, L))
        if m == 0xDA:
            break
        i += 2 + L
    return out


def _set(b: bytes, pos: int, val: int) -> bytes:
    x = bytearray(b)
    x[pos] = val
    return bytes(x)


def _pil_rejects(b: bytes) -> bool:
    from PIL import Image

    try:
        im = Image.open(io.BytesIO(b))
        im.load()
        return False
    except Exception:
        return True


def _golden(name):
    with open(os.path.join(GOLDEN, "jpeg", name), "rb") as f:
        return f.read()


def test_targeted_header_corruptions_rejected(planner):
    b = _golden("food_512x384_q75.jpg")
    seg = {m: (i, L) for m, i, L in reversed(segments(b))}  # first occurrence wins
    sof, sos, dht, dqt = seg[0xC0][0], seg[0xDA], seg[0xC4][0], seg[0xDB][0]
    x = bytearray(b)
    x[sof + 4 + 6 + 3 * 2] = x[sof + 4 + 6]  # component 3 reuses component 1's id
    dri = b[:sos[0]] + b"\xff\xdd\x00\x05\x00\x01\x00" + b[sos[0]:]  # DRI with length 5
    cases = {
        "sos_duplicate_selector": (_set(b, sos[0] + 4 + 1 + 2, b[sos[0] + 4 + 1]), {NOT_JPEG}),
        "sos_seglen_2": (b[:sos[0] + 2] + b"\x00\x02" + b[sos[0] + 4:], {NOT_JPEG}),
        "sos_ns_0": (_set(b, sos[0] + 4, 0), {NOT_JPEG}),
        "sof_precision_12": (_set(b, sof + 4, 12), {UNSUPPORTED}),
        "sof_ncomp_4": (_set(b, sof + 4 + 5, 4), {NOT_JPEG, UNSUPPORTED}),
        "sof_width_0": (_set(_set(b, sof + 7, 0), sof + 8, 0), {NOT_JPEG}),
        "sof_duplicate_id": (bytes(x), {NOT_JPEG}),
        "dht_class_2": (_set(b, dht + 4, 0x20), {NOT_JPEG}),
        "dht_counts_over_256": (_set(b, dht + 4 + 1 + 15, 200), {NOT_JPEG}),
        "dqt_table_5": (_set(b, dqt + 4, 0x05), {NOT_JPEG}),
        "dri_length_5": (dri, {NOT_JPEG}),
    }
    names = list(cases)
    got = planner([cases[k][0] for k in names])
    for k, st in zip(names, got):
        assert st in cases[k][1], (k, st)
        assert _pil_rejects(cases[k][0]), k  # Pillow/libjpeg-turbo rejects it as well
    # documented divergence: baseline SOS with Ss = 1 (libjpeg warns and decodes)
    assert planner([_set(b, sos[0] + 2 + sos[1] - 3, 1)]) == [UNSUPPORTED]


@pytest.mark.parametrize("name", ["food_512x384_q75.jpg", "c4_375x500_q90_rst.jpg", "gray_77x91.jpg",
                                  "prog_375x500_q90.jpg", "prog_rst_250x333_q90.jpg"])
def test_every_header_truncation(planner, name):
    b = _golden(name)
    segs = segments(b)
    m, i, L = segs[-1]
    end = i + 2 + L  # end of the first SOS header
    cuts = [b[:k] for k in range(0, end)]
    got = planner(cuts)
    for k, st in enumerate(got):
        assert st != 0, (name, k)
        if not name.startswith("prog"):
            assert st == NOT_JPEG, (name, k, st)


def test_random_header_overwrites(planner):
    rng = np.random.default_rng(1234)
    cells = []
    for path in sorted(glob.glob(os.path.join(GOLDEN, "jpeg", "*.jpg"))):
        with open(path, "rb") as f:
            b = f.read()
        segs = segments(b)
        if not segs:
            continue
        lo, hi = 2, segs[-1][1] + 2 + segs[-1][2]
        for _ in range(120):
            x = bytearray(b)
            for _ in range(int(rng.integers(1, 5))):
                x[int(rng.integers(lo, hi))] = int(rng.integers(0, 256))
            cells.append(bytes(x))
            # also a length field pushed past the cell
            y = bytearray(b)
            m, i, L = segs[int(rng.integers(0, len(segs)))]
            y[i + 2:i + 4] = struct.pack(">H", int(rng.integers(0, 65536)))
            cells.append(bytes(y))
    got = planner(cells)
    assert all(0 <= s <= 5 for s in got)
    assert sum(1 for s in got if s != 0) > len(got) // 4  # the mutations do reach the checks


def _all_marker_segments(b: bytes):
    """(offset, length) of every marker segment with a length field in the
    file, including the DHT/SOS headers between progressive scans."""
    out, i = [], 2
    while i + 4 <= len(b):
        if b[i] == 0xFF and b[i + 1] not in (0x00, 0xFF, 0xD8, 0xD9, 0x01) and not 0xD0 <= b[i + 1] <= 0xD7:
            L = (b[i + 2] << 8) | b[i + 3]
            out.append((i, L))
            i += 2 + L
        else:
            i += 1
    return out


def test_progressive_scan_header_overwrites(planner):
    """plan_progressive walks every scan header of a SOF2 file: mutate the
    DHT / SOS segments between scans, and cut the file inside each of them."""
    rng = np.random.default_rng(99)
    cells = []
    for path in sorted(glob.glob(os.path.join(GOLDEN, "jpeg", "prog_*.jpg"))):
        with open(path, "rb") as f:
            b = f.read()
        segs = [s for s in _all_marker_segments(b) if s[0] > segments(b)[-1][1]]  # after the first SOS
        assert segs, path
        for (i, L) in segs:
            cells.append(b[:i + 2 + int(rng.integers(0, L + 1))])
            for _ in range(8):
                x = bytearray(b)
                x[i + 2 + int(rng.integers(0, L))] = int(rng.integers(0, 256))
                cells.append(bytes(x))
    got = planner(cells)
    assert all(0 <= s <= 5 for s in got)


def test_progressive_scan_ranges(planner):
    """plan_progressive's scan byte ranges (the SSE2 end-of-scan search) against
    a byte-by-byte restatement: the first 0xFF followed by a byte that is not
    0x00, 0xFF or RSTn ends a scan. Progressive goldens, synthetic images with
    restart intervals, and copies whose scans were salted with 0xFF 0x00 /
    0xFF 0xFF / 0xFF RSTn pairs at random offsets (16-byte-boundary cases
    included)."""
    import subprocess as sp

    from ldt_amd import synth

    def ref_ranges(b):
        out, i = [], 2
        while i + 4 <= len(b):
            if b[i] != 0xFF:
                return None
            while i + 1 < len(b) and b[i + 1] == 0xFF:
                i += 1
            m = b[i + 1]
            if m == 0xD9:
                break
            if m == 0x01 or 0xD0 <= m <= 0xD7:
                i += 2
                continue
            n = (b[i + 2] << 8) | b[i + 3]
            if m != 0xDA:
                i += 2 + n
                continue
            s0 = i + 2 + n
            j = s0
            while j + 1 < len(b) and not (b[j] == 0xFF and b[j + 1] not in (0x00, 0xFF) and not 0xD0 <= b[j + 1] <= 0xD7):
                j += 1
            out.append((s0, j - s0))
            i = j
        return out

    cells = [open(e, "rb").read() for e in sorted(glob.glob(os.path.join(GOLDEN, "jpeg", "*.jpg")))
             if "prog" in os.path.basename(e)]
    assert len(cells) >= 5
    cells += [synth.encode(synth.field(96 + 17 * k, 80 + 9 * k, k, 12.0), quality=90, progressive=True,
                           **({"restart_marker_blocks": 2} if k % 2 else {})) for k in range(6)]
    rng = np.random.default_rng(7)
    salted = []
    for b in cells[:6]:
        rr = ref_ranges(b)
        bb = bytearray(b)
        for (s0, ln) in rr:
            for _ in range(6):
                if ln < 40:
                    break
                p = s0 + int(rng.integers(2, ln - 4))
                if bb[p - 1] == 0xFF:
                    continue
                bb[p:p + 2] = bytes([0xFF, int(rng.choice([0x00, 0xFF, 0xD3]))])
        salted.append(bytes(bb))
    cells += salted
    inp = b"".join(struct.pack("<I", len(c)) + c for c in cells)
    r = sp.run([planner.exe], input=inp, capture_output=True, timeout=300,
               env=dict(os.environ, ASAN_OPTIONS="detect_leaks=0", PLAN_SCANS="1"))
    assert r.returncode == 0 and not r.stderr, r.stderr.decode(errors="replace")[-2000:]
    lines = r.stdout.decode().splitlines()
    assert len(lines) == len(cells)
    checked = 0
    for b, line in zip(cells, lines):
        parts = line.split()
        if parts[-1] != "0":
            continue
        got = [tuple(int(x) for x in t.split(":")) for t in parts[:-1]]
        assert got == ref_ranges(b), (got[:3], ref_ranges(b)[:3])
        checked += 1
    assert checked >= len(cells) - len(salted)
