"""bench.py keeps the driver's contract: one JSON line on stdout with the
required keys, roofline and measured-ceiling objects, for the headline (c2)
and the raw HBM-stress (c5) workloads. Small step counts; no CPU legs."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REQUIRED = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
            "scaling", "vs_baseline", "dtype", "data", "config", "roofline")


def _bench(*args):
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args], cwd=REPO, capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.gpu
@pytest.mark.parametrize("workload", ["c2", "c5"])
def test_bench_json_contract(workload):
    d = _bench("--workload", workload, "--steps", "3", "--warmup", "1", "--no-cpu-baseline")
    for k in REQUIRED:
        assert k in d, k
    with open(os.path.join(REPO, "BASELINE.json")) as f:
        assert d["metric"] == json.load(f)["metric"]
    assert d["unit"] == "img/s" and d["higher_is_better"] is True and d["scaling"] == "weak"
    assert d["n_gpus"] == 1 and d["steps"] == 3 and d["warmup"] == 1 and d["value"] > 0
    assert d["vs_baseline"] is None  # BASELINE.md publishes no number for this metric
    assert "workload" in d["config"] and d["config"]["workload"].startswith(workload)
    roof = d["roofline"]
    assert roof["bound"] == "hbm" and roof["unit"] == "GB/s" and roof["peak"] == 8000.0
    assert 0 < roof["frac"] < 1 and abs(roof["frac"] - roof["achieved"] / roof["peak"]) < 1e-3
    ceil = roof["measured_ceiling"]
    assert 1000 < ceil["stream_copy_gbs"] < 8000
    assert abs(d["value_per_gpu"] - d["value"] / d["n_gpus"]) <= 0.11
    if workload == "c2":
        assert d["dtype"] == "u8" and "standalone" in roof and "value_host_input" in d
        assert set(d["stages_ms_per_step"]) >= {"destuff", "huffman", "idct", "resize"}
        # BASELINE configs[2] / configs[3] legs beside the headline
        legs = d["config_legs"]
        assert legs["c3"]["dataset_leg"]["sampler"] == "ShardedBatchSampler"
        assert legs["c4"]["dataset_leg"]["sampler"] == "ShardedFragmentSampler(pad=True)"
        for leg in legs.values():
            assert leg["value"] > 0 and leg["per_gpu_batch"] == 128


def _free_port():
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.gpu
@pytest.mark.timeout(900)
@pytest.mark.parametrize("ranks", [2, 8])
def test_bench_multi_rank_rehearsal(ranks):
    """The N > 1 path of bench.py as the driver launches it (torchrun, one
    process per rank, barriers, max over ranks, rank 0 prints one line), with
    LDT_BENCH_BACKEND=gloo so that the ranks can share this box's one GPU. At
    8 ranks it rehearses the node's host budget: every rank sizes its copy
    pool from the cgroup quota / LOCAL_WORLD_SIZE and binds it to its own
    GPU-local cores, and the line reports each rank's placement and host
    phases (host_ranks)."""
    env = dict(os.environ, LDT_BENCH_BACKEND="gloo")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(ranks),
                        "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
                        os.path.join(REPO, "bench.py"), "--gpus", str(ranks), "--steps", "3", "--warmup", "1",
                        "--no-cpu-baseline", "--dataset-batches", "2", "--dataset-epochs", "1", "--host-reps", "1"],
                       cwd=REPO, capture_output=True, text=True, timeout=840, env=env)
    # the ranks' own tracebacks first (torchrun's summary follows them)
    assert r.returncode == 0, "\n".join(ln for ln in r.stderr.splitlines() if ln.startswith("[rank"))[-3000:] \
        + r.stderr[-1000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip().startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == ranks and d["config"]["global_batch"] == ranks * d["config"]["per_gpu_batch"]
    assert abs(d["value_per_gpu"] - d["value"] / ranks) <= 0.11
    for cw, per_rank in (("c3", 2), ("c4", None)):
        leg = d["config_legs"][cw]
        assert leg["value_per_gpu"] * ranks == pytest.approx(leg["value"], abs=0.06 * ranks)
        info = leg["dataset_leg"]
        assert info["images_all_ranks"] > 0 and info["epochs"] == 1
        if per_rank:
            # ShardedBatchSampler: every rank reads its `per_rank` batches of 128
            assert info["images_all_ranks"] == ranks * per_rank * 128
    hr = d["host_ranks"]
    assert [h["rank"] for h in hr] == list(range(ranks))
    for h in hr:
        assert h["local_world"] == ranks and set(h["host_us_per_call"]) >= {"parse", "copy_join"}
        assert h["copy_threads"] == len(h["copy_cpus"])
    # ranks that share a NUMA node never share a copy core
    used = [c for h in hr for c in h["copy_cpus"] if c >= 0]
    assert len(used) == len(set(used)) or len(used) > 64, used
