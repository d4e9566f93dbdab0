"""Benchmark of the MI355X batch-decode path (BASELINE.json metric).

One "step" = one batch of synthetic JPEG cells (already resident in HBM)
through the whole hot path: marker walk + plan upload, destuff, Huffman
decode, IDCT, fused upsample/colour/Resize(224,224)/ToTensor store, labels.
Default workload (N=1 and per rank for N>1, weak scaling): BASELINE.json
configs[1] — 512x512 baseline JPEG, 4:2:0, q90, batch 256 per GPU.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c2|c1|c4|c5|c2p]
    torchrun --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

Rank 0 prints ONE JSON line. The CPU baseline (rank 0, N=1 only) times the
reference's own CPU path on this host in this run: the map-style DataLoader
harness with the PIL collate_fn (lance_map_style.py:21-44, :54-69) at
num_workers 8 and at the box's CPU share, and the iterable to_tensor_fn in
one process (cpu_baseline below). value_host_input is the PCIe-inclusive rate
of the same steps (host RecordBatches).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
for _p in (os.path.join(REPO, "lance-distributed-training_amd"), REPO):
    if _p not in sys.path:
        sys.path.insert(0, _p)

METRIC = "decoded 224×224 fp32 images/sec per GPU and per node at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
OUT_BYTES = 3 * 224 * 224 * 4  # 602,112 B per image (float32 CHW)

WORKLOADS = {
    "c2": dict(desc="512x512 baseline JPEG 4:2:0 q90 (BASELINE configs[1]), to_tensor_fn", batch=256),
    "c1": dict(desc="FOOD101-shaped 512x384/384x512/512x512 JPEG, PIL defaults q75 4:2:0 (configs[0]/[2] data)",
               batch=128),
    "c4": dict(desc="ImageNet-shaped ~500x375 variable JPEG q90 with restart markers (configs[3] data)", batch=128),
    "c5": dict(desc="raw uint8 HWC 1024x1024 -> Resize 224 + Normalize (configs[4])", batch=1024),
    # not a BASELINE config: the c2 images encoded progressive (SOF2), to
    # measure the serial per-scan path
    "c2p": dict(desc="c2's 512x512 q90 4:2:0 images as progressive JPEG (SOF2)", batch=256),
}


def make_cells(workload: str, n: int, seed: int):
    from ldt_amd import synth

    if workload == "c2":
        return synth.q90_512(n, seed=seed)
    if workload == "c2p":
        return synth.q90_512(n, seed=seed, progressive=True)
    if workload == "c1":
        return synth.food101_like(n, seed=seed)
    if workload == "c4":
        return synth.imagenet_like(n, seed=seed)
    raise ValueError(workload)


CPU_SHARE = 16  # CPUs of the GPU box a run may use per GPU (os.cpu_count() shows the whole host)


def _rates(times, imgs):
    r = sorted(imgs / t for t in times)
    return {"best": round(r[-1], 1), "median": round(r[len(r) // 2], 1), "reps": [round(x, 1) for x in r]}


def cpu_baseline(cells, labels, batch: int = 128, reps: int = 5):
    """The reference's CPU path on this host, in this run.

    map-style legs: lance_map_style.py:54-69's harness, i.e. a stock torch
    DataLoader over the SafeLanceDataset shim with the reference PIL collate_fn
    (oracle.pil_collate_fn = lance_map_style.py:21-44: Pillow
    open/convert/Resize((224,224))/to_tensor, stack), batch 128 (config 1),
    pin_memory=True, persistent spawn workers; num_workers = 8 (the reference
    default, :137) and the box's CPU share. Each leg: one batch per worker
    (plus the prefetch queue) to warm up, then `reps` timed runs of
    2 x num_workers batches; best and median img/s.
    iterable leg: lance_iterable.py:38-50's decode_tensor_image on
    RecordBatches in the main process (num_workers=0, :75-77)."""
    import shutil
    import tempfile

    import numpy as np
    import pyarrow as pa
    import torch
    from PIL import __version__ as pil_version
    from PIL import features

    from oracle import oracle

    import ldt_amd as lds

    tmp = tempfile.mkdtemp(prefix="ldt_cpu_")
    try:
        n = len(cells)
        lds.write_dataset(pa.table({"image": pa.array(cells, pa.binary()),
                                    "label": pa.array(np.asarray(labels, np.int64))}), tmp)
        ds = lds.SafeLanceDataset(tmp)
        host = len(os.sched_getaffinity(0))
        legs = []
        for w in sorted({8, min(host, CPU_SHARE)}):
            need = batch * w * (4 + 2 * reps)  # warm-up + timed
            order = [i % n for i in range(need)]
            loader = lds.get_safe_loader(ds, batch_size=batch, sampler=order, num_workers=w,
                                         collate_fn=oracle.pil_collate_fn, pin_memory=True,
                                         persistent_workers=True)
            it = iter(loader)
            for _ in range(4 * w):  # every worker busy, prefetch queues full
                next(it)
            times = []
            for _ in range(reps):
                t0 = time.perf_counter()
                for _ in range(2 * w):
                    out = next(it)
                times.append(time.perf_counter() - t0)
            assert out["image"].shape == (batch, 3, 224, 224)
            del it, loader
            legs.append(dict(harness="map-style DataLoader(SafeLanceDataset, PIL collate_fn)",
                             num_workers=w, batch=batch, **_rates(times, 2 * batch * w)))
        rb = pa.RecordBatch.from_arrays([pa.array(cells[:batch], pa.binary()),
                                         pa.array(np.asarray(labels[:batch], np.int64))],
                                        names=["image", "label"])
        oracle.pil_decode_tensor_image(rb)
        times = []
        for _ in range(reps):
            t0 = time.perf_counter()
            oracle.pil_decode_tensor_image(rb)
            times.append(time.perf_counter() - t0)
        legs.append(dict(harness="iterable decode_tensor_image in the main process", num_workers=0,
                         batch=batch, **_rates(times, batch)))
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    ref = legs[0]
    return {
        "value": ref["median"], "unit": "img/s", "cores": ref["num_workers"], "kind": "reference",
        "sample": (f"the reference CPU path on this workload's cells: DataLoader(SafeLanceDataset shim, "
                   f"PIL collate_fn, batch {batch}, pin_memory, persistent spawn workers), "
                   f"{reps} x 2*num_workers timed batches per leg after warm-up; Pillow {pil_version} / "
                   f"libjpeg-turbo {features.version_feature('libjpeg_turbo')}; host affinity {host} CPUs "
                   f"(a one-GPU run may use {CPU_SHARE}); value = median of the "
                   f"num_workers={ref['num_workers']} leg (lance_map_style.py:137 default)"),
        "legs": legs,
        "torch_threads": torch.get_num_threads(),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--workload", default="c2", choices=sorted(WORKLOADS))
    ap.add_argument("--batch", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--input", choices=("resident", "host"), default="resident",
                    help="resident: cells already in HBM (value); host: Arrow RecordBatches in host "
                         "memory through the pipelined to_tensor_fn (PCIe-inclusive, DESIGN.md §7)")
    ap.add_argument("--no-stage-events", action="store_true",
                    help="time without the per-stage HIP events (no roofline)")
    ap.add_argument("--depth", type=int, default=3,
                    help="batches in flight (ldt_amd.DecodePipeline: one context + HIP stream each)")
    args = ap.parse_args()

    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    # LDT_BENCH_BACKEND=gloo: rehearsal of the multi-rank path on a 1-GPU box
    # (ranks then share the devices round-robin); the real runs use RCCL
    backend = os.environ.get("LDT_BENCH_BACKEND", "nccl")
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local % torch.cuda.device_count() if backend != "nccl" else local)
        dist.init_process_group(backend, rank=rank, world_size=world)
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    import ldt_amd
    from ldt_amd import _lib

    wl = WORKLOADS[args.workload]
    B = args.batch or wl["batch"]
    ctx = _lib.get_context(dev.index)
    ctx.set_option(_lib.OPT_SYNC_STATUS, 0)
    ctx.set_option(_lib.OPT_PROFILE, 0 if args.no_stage_events else 1)

    cells = None
    if args.workload == "c5":
        # synthetic uniform uint8 HWC 1024x1024 generated directly in HBM
        g = torch.Generator(device=dev)
        g.manual_seed(1234 + rank)
        raw = torch.randint(0, 256, (B, 1024, 1024, 3), dtype=torch.uint8, device=dev, generator=g)
        bytes_per_img = 1024 * 1024 * 3 + OUT_BYTES

        def step():
            return ldt_amd.resize_raw(raw, 1024, 1024, normalize=True)
    else:
        nb = 2  # two distinct batches, alternated
        batches, host_batches = [], []
        cells_all, labels_all = [], []
        import pyarrow as pa

        for k in range(nb):
            cells, labels = make_cells(args.workload, B, seed=1000 * rank + k)
            cells_all += cells
            labels_all += list(labels)
            host_batches.append(pa.RecordBatch.from_arrays(
                [pa.array(cells, pa.binary()), pa.array(np.asarray(labels, np.int64))],
                names=["image", "label"]))
            if args.input == "host":
                batches.append(host_batches[-1])
            else:
                batches.append(ldt_amd.ResidentBatch(cells, labels, device=dev))
        px = [ldt_amd_dims(c) for c in cells_all[:B]]
        bytes_per_img = float(np.mean([h * w * 3 for (h, w) in px])) + OUT_BYTES
        comp_bytes = float(np.mean([len(c) for c in cells_all]))
        it = [0]
        pipe = ldt_amd.DecodePipeline(depth=args.depth, device=dev, profile=not args.no_stage_events)
        for c in pipe.ctxs:  # tuning knobs (default minimum S = 256 bits, fitted per image)
            if os.environ.get("LDT_SUBSEQ_BITS"):
                c.set_option(_lib.OPT_SUBSEQ_BITS, int(os.environ["LDT_SUBSEQ_BITS"]))
            if os.environ.get("LDT_SYNC_WARM"):
                c.set_option(_lib.OPT_SYNC_WARM, int(os.environ["LDT_SYNC_WARM"]))

        def step():
            b = batches[it[0] % nb]
            it[0] += 1
            return pipe.decode(b)

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    for _ in range(args.warmup):
        step()
    prof = ctx if args.workload == "c5" else pipe
    barrier()
    prof.stage_times(reset=True)
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    barrier()
    elapsed = time.perf_counter() - t0
    stages = prof.stage_times(reset=True)
    if args.workload != "c5":
        pipe.check()  # every decoded image status OK
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed_max = float(t.item())
    total_imgs = B * args.steps * world
    value = total_imgs / elapsed_max

    # PCIe-inclusive rate in the same run: the same steps with
    # the cells in host Arrow RecordBatches through the pipelined to_tensor_fn
    def host_rate(bs):
        hp = ldt_amd.DecodePipeline(depth=args.depth, device=dev)
        for k in range(max(args.warmup, 2)):
            hp.decode(bs[k % nb])
        barrier()
        th0 = time.perf_counter()
        for k in range(args.steps):
            hp.decode(bs[k % nb])
        barrier()
        th = torch.tensor([time.perf_counter() - th0], dtype=torch.float64,
                          device=dev if backend == "nccl" else "cpu")
        if world > 1:
            dist.all_reduce(th, op=dist.ReduceOp.MAX)
        hp.check()
        return B * args.steps * world / float(th.item())

    value_host = value_registered = None
    if args.workload != "c5" and args.input == "resident":
        value_host = host_rate(host_batches)
        # the same host batches with their image buffers page-locked in place
        # (ldt_register_host): DMA from the caller's pages, no staging memcpy
        # (optional leg: a box whose memlock limit refuses the pinning reports null)
        try:
            for b in host_batches:
                ldt_amd.register_host(b.column(0), device=dev)
            value_registered = host_rate(host_batches)
        except ldt_amd.LdtError as e:
            print(f"bench: registered host leg skipped: {e}", file=sys.stderr)
        finally:
            for b in host_batches:
                ldt_amd.unregister_host(b.column(0))

    # standalone launch durations (one batch in flight, after the timed region)
    standalone = None
    if args.workload != "c5" and not args.no_stage_events:
        solo = ldt_amd.DecodePipeline(depth=1, device=dev, profile=True)
        for k in range(2):
            solo.decode(batches[k % nb])
        barrier()
        solo.stage_times(reset=True)
        for k in range(4):
            solo.decode(batches[k % nb])
        barrier()
        standalone = solo.stage_times(reset=True)
        solo.check()

    # measured HBM ceiling on this box, after the timed region
    ceiling = stream_copy_ceiling(dev)

    # roofline: the resize/normalise stage (north_star), from live HIP events
    rs_ms, rs_n = stages["resize"]
    rs_avg_s = rs_ms / max(rs_n, 1) / 1e3
    achieved = bytes_per_img * B / rs_avg_s / 1e9 if rs_avg_s > 0 else 0.0
    dominant = max((k for k in stages if k != "h2d"), key=lambda k: stages[k][0])
    res = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "img/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed_max / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": (f"synthetic (seeded PIL-encoded JPEG cells {'resident in HBM' if args.input == 'resident' else 'in host Arrow RecordBatches, copied over PCIe every step'}; FOOD101 offline-unavailable)"
                 if args.workload != "c5" else "synthetic (uniform uint8 HWC generated in HBM)"),
        "config": {"workload": f"{args.workload}: {wl['desc']}", "per_gpu_batch": B, "global_batch": B * world,
                   "parallelism": f"dp{world} (independent shards, no data-path collective)",
                   "pipeline_depth": 1 if args.workload == "c5" else args.depth,
                   "input": "resident" if args.workload == "c5" else args.input,
                   "output": "float32[N,3,224,224] + int64[N] on device"},
        "roofline": {
            "kernel": "k_resize (fused chroma upsample + YCbCr->RGB + BILINEAR 224 + ToTensor store)"
                      if args.workload != "c5" else "k_resize<raw> (BILINEAR 224 + Normalize store)",
            "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
            "bytes_per_unit": round(bytes_per_img, 1),
            "unit_basis": "SURVEY.md §8(d): H*W*3 (uint8 RGB in) + 602,112 (fp32 out) per image",
            "avg_launch_ms": round(rs_avg_s * 1e3, 4),
            "timing": ("HIP events on the kernel's stream over the timed region"
                       + (f"; {args.depth} batches in flight, so durations include the overlapping "
                          "batch's kernels" if args.workload != "c5" and args.depth > 1 else "")),
        },
        "stages_ms_per_step": {k: round(v[0] / max(v[1], 1), 4) for k, v in stages.items()},
        "dominant_stage": dominant,
    }
    if standalone is not None:
        sa_ms, sa_n = standalone["resize"]
        sa_s = sa_ms / max(sa_n, 1) / 1e3
        sa_ach = bytes_per_img * B / sa_s / 1e9 if sa_s > 0 else 0.0
        res["roofline"]["standalone"] = {
            "avg_launch_ms": round(sa_s * 1e3, 4), "achieved": round(sa_ach, 1),
            "frac": round(sa_ach / HBM_PEAK_GBS, 4),
            "timing": "HIP events, one batch in flight (4 batches after the timed region)"}
        res["stages_standalone_ms"] = {k: round(v[0] / max(v[1], 1), 4) for k, v in standalone.items()}
        res["roofline"]["standalone"]["frac_of_measured"] = round(sa_ach / ceiling, 4)
    res["roofline"]["measured_ceiling"] = {
        "stream_copy_gbs": round(ceiling, 1), "frac_of_measured": round(achieved / ceiling, 4),
        "method": "device-to-device copy of 1 GiB (read + write counted), torch's vectorised copy kernel, "
                  "best of 10, HIP events; measured after the timed region"}
    tr = load_profile(f"traffic_{args.workload}.json")
    if tr is not None and tr.get("batch", B) == B:
        res["roofline"]["traffic"] = tr["hbm_bytes_per_launch"]
        res["roofline"]["traffic_source"] = (f"profiles/{PROFILE_ROUND}/traffic_{args.workload}.json: rocprofv3 "
                                             "--pmc FETCH_SIZE and WRITE_SIZE passes (FETCH_SIZE x2, gfx950) "
                                             "over this bench at depth 1")
    dec = load_profile(f"pmc_{args.workload}_decode.json")
    if dec is not None:
        res["decode_efficiency"] = dec
    if args.workload != "c5":
        res["config"]["compressed_bytes_per_img"] = round(comp_bytes, 1)
    if value_host is not None:
        res["value_host_input"] = round(value_host, 1)
        res["value_host_input_note"] = ("same steps with the cells in host pa.RecordBatches (pinned copy + "
                                        "H2D every step, to_tensor_fn boundary); value keeps them in HBM")
    if value_registered is not None:
        res["value_host_registered"] = round(value_registered, 1)
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.workload != "c5":
        res["cpu_baseline"] = cpu_baseline(cells_all, labels_all)
        res["gpu_over_cpu"] = {f"num_workers={leg['num_workers']}": round(value / leg["median"], 1)
                               for leg in res["cpu_baseline"]["legs"]}
    elif rank == 0 and world == 1 and args.workload == "c5" and not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline_raw(raw[:8].cpu().numpy())
        res["gpu_over_cpu"] = round(value / res["cpu_baseline"]["value"], 2)
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


PROFILE_ROUND = "r2"


def stream_copy_ceiling(dev, nbytes: int = 1 << 30, reps: int = 10) -> float:
    """Measured HBM stream ceiling in GB/s: 2 * nbytes per device-to-device copy."""
    import torch

    a = torch.full((nbytes // 4,), 1.0, dtype=torch.float32, device=dev)
    b = torch.empty_like(a)
    b.copy_(a)
    torch.cuda.synchronize(dev)
    best = 0.0
    for _ in range(reps):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        b.copy_(a)
        e1.record()
        e1.synchronize()
        best = max(best, 2.0 * nbytes / (e0.elapsed_time(e1) / 1e3) / 1e9)
    del a, b
    torch.cuda.empty_cache()
    return best


def load_profile(name: str):
    """A committed PMC summary under profiles/<round>/ (None if absent)."""
    path = os.path.join(REPO, "profiles", PROFILE_ROUND, name)
    if not os.path.exists(path):
        return None
    with open(path) as f:
        return json.load(f)


def ldt_amd_dims(cell: bytes):
    """(H, W) from the SOF0/1/2 marker (host-side helper for byte accounting)."""
    i = 2
    while i + 4 <= len(cell):
        m = cell[i + 1]
        L = (cell[i + 2] << 8) | cell[i + 3]
        if m in (0xC0, 0xC1, 0xC2):
            return (cell[i + 5] << 8) | cell[i + 6], (cell[i + 7] << 8) | cell[i + 8]
        i += 2 + L
    raise ValueError("no SOF")


def cpu_baseline_raw(hwc):
    """Config 5 CPU leg: Pillow resize + to_tensor + Normalize, 1 process."""
    import numpy as np
    from PIL import Image

    MEAN = np.asarray((0.485, 0.456, 0.406), np.float32)[:, None, None]
    STD = np.asarray((0.229, 0.224, 0.225), np.float32)[:, None, None]
    t0 = time.perf_counter()
    reps = 0
    while time.perf_counter() - t0 < 5.0:
        for k in range(len(hwc)):
            rs = np.asarray(Image.fromarray(hwc[k]).resize((224, 224), Image.BILINEAR))
            t = rs.transpose(2, 0, 1).astype(np.float32) / np.float32(255)
            (t - MEAN) / STD
            reps += 1
    dt = time.perf_counter() - t0
    return {"value": round(reps / dt, 1), "unit": "img/s", "cores": 1, "kind": "reference",
            "sample": f"{reps} Pillow resize((224,224),BILINEAR)+to_tensor+Normalize of 1024x1024 uint8, 1 process"}


if __name__ == "__main__":
    main()
