"""Host copy pool and placement (lance-distributed-training_amd/csrc/
ldt_hostcopy.cpp, HIP-free), built with g++ and ASan/UBSan here: byte-exact
copies through copy_bytes and the pool (non-temporal AVX2 stores and memcpy,
misaligned sources and destinations, 0-7 threads, repeated generations), and
the placement rules that size and bind each rank's pool (the
node's host budget shared by the local ranks)."""
import json
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = [os.path.join(REPO, "tools", "checks", "hostcopy_check.cpp"),
       os.path.join(REPO, "lance-distributed-training_amd", "csrc", "ldt_hostcopy.cpp")]


@pytest.fixture(scope="module")
def exe(tmp_path_factory):
    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    out = str(tmp_path_factory.mktemp("hostcopy") / "hostcopy_check")
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                    "-pthread", *SRC, "-o", out], check=True)
    return out


def _run(exe, *args, env=None):
    r = subprocess.run([exe, *map(str, args)], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, **(env or {})))
    assert r.returncode == 0, r.stderr[-2000:]
    return r.stdout


def test_copies_byte_exact(exe):
    assert "copy ok" in _run(exe, "copy")


def test_placement_distinct_cores_and_rank_blocks(exe):
    base = {k: v for k, v in os.environ.items() if k not in ("LOCAL_RANK", "LOCAL_WORLD_SIZE")}
    one = json.loads(_run(exe, "place", 3, 1, env=dict(base, LOCAL_RANK="0", LOCAL_WORLD_SIZE="1")))
    assert one["threads"] == 3 and len(set(one["cpus"])) == 3 and min(one["cpus"]) >= 0
    assert one["local_rank"] == 0 and one["local_world"] == 1
    if one["candidates"] >= 6:
        # the next local rank takes the next block of cores
        two = json.loads(_run(exe, "place", 3, 1, env=dict(base, LOCAL_RANK="1", LOCAL_WORLD_SIZE="2")))
        assert not set(one["cpus"]) & set(two["cpus"]), (one, two)
    unbound = json.loads(_run(exe, "place", 2, 0))
    assert unbound["cpus"] == [-1, -1]


def test_placement_thread_count_from_budget(exe):
    """-1: (quota or GPU-local cores) / LOCAL_WORLD_SIZE - 2, at most 6."""
    d = json.loads(_run(exe, "place", -1, 1, env={"LOCAL_WORLD_SIZE": "1", "LOCAL_RANK": "0"}))
    budget = d["quota"] if d["quota"] > 0 else d["candidates"]
    assert d["threads"] == max(0, min(6, int(budget) - 2))
    many = json.loads(_run(exe, "place", -1, 1, env={"LOCAL_WORLD_SIZE": "64", "LOCAL_RANK": "5"}))
    budget = many["quota"] if many["quota"] > 0 else many["candidates"]
    assert many["threads"] == max(0, min(6, int(budget / 64) - 2))
