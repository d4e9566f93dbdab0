"""Benchmark of the MI355X batch-decode path (BASELINE.json metric).

One "step" = one batch of synthetic JPEG cells through the whole hot path:
marker walk + plan upload, destuff, Huffman decode, IDCT, fused
upsample/colour/Resize(224,224)/ToTensor store, labels.
Default workload (N=1 and per rank for N>1, weak scaling): BASELINE.json
configs[1] — 512x512 baseline JPEG, 4:2:0, q90, batch 256 per GPU.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c2|c1|c3|c4|c5|c2p]
    torchrun --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

Three legs of the same workload, each timed between barriers (max over ranks):
  value             cells resident in HBM when the timed region starts (the
                    driver contract); everything else of the path is timed;
  value_host_input  the plug-in boundary: host pa.RecordBatches through the
                    pipelined to_tensor_fn (pinned copy + H2D every step);
  config_legs       BASELINE configs[2] and [3] as written, in a c2 run: the
                    dataset leg below over FOOD101-shaped cells with
                    ShardedBatchSampler (c3) and ImageNet-shaped cells with
                    ShardedFragmentSampler(pad=True) (c4), batch 128 per rank;
  value_dataset     the reference's iterable loop: an Arrow/Lance dataset of the
                    workload's cells read through LanceDataset + the sampler
                    (ShardedBatchSampler; ShardedFragmentSampler(pad=True) with
                    its RCCL all_reduce(MAX) for c4 = configs[3]) + the copying
                    to_tensor_fn (pylance yields fresh buffers per read), full
                    epochs (plan included) per rank; value_dataset_registered:
                    the same with the mapped fragments page-locked in place.
Each is whole-job (all ranks) with a *_per_gpu twin. Rank 0 prints ONE JSON
line. The CPU baseline (rank 0, N=1 only) times the reference's own CPU path
on this host in this run: the map-style DataLoader harness with the PIL
collate_fn (lance_map_style.py:21-44, :54-69) at num_workers 8 and at the
box's CPU share, and the iterable to_tensor_fn in one process.
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
    "c2": dict(desc="512x512 baseline JPEG 4:2:0 q90 (BASELINE configs[1]), to_tensor_fn", batch=256,
               sampler="batch"),
    "c1": dict(desc="FOOD101-shaped 512x384/384x512/512x512 JPEG, PIL defaults q75 4:2:0 (configs[0] data)",
               batch=128, sampler="batch"),
    "c3": dict(desc="FOOD101 LanceDataset iterable + ShardedBatchSampler, batch 128/rank (BASELINE configs[2]); "
                    "FOOD101-shaped PIL-default q75 cells", batch=128, sampler="batch"),
    "c4": dict(desc="ImageNet-shaped ~500x375 variable JPEG q90 with restart markers, ShardedFragmentSampler "
                    "pad=True over uneven fragments (BASELINE configs[3])", batch=128, sampler="fragment"),
    "c5": dict(desc="raw uint8 HWC 1024x1024 -> Resize 224 + Normalize (configs[4])", batch=1024),
    # not a BASELINE config: the c2 images encoded progressive (SOF2), to
    # measure the serial per-scan path
    "c2p": dict(desc="c2's 512x512 q90 4:2:0 images as progressive JPEG (SOF2)", batch=256, sampler="batch"),
}


def make_cells(workload: str, n: int, seed: int):
    from ldt_amd import synth

    if workload == "c2":
        return synth.q90_512(n, seed=seed)
    if workload == "c2p":
        return synth.q90_512(n, seed=seed, progressive=True)
    if workload in ("c1", "c3"):
        return synth.food101_like(n, seed=seed)
    if workload == "c4":
        return synth.imagenet_like(n, seed=seed)
    raise ValueError(workload)


# CPUs of the GPU box a one-GPU run may use (os.sched_getaffinity shows the
# whole host there); LDT_CPU_SHARE overrides it on hosts with another share
CPU_SHARE = int(os.environ.get("LDT_CPU_SHARE", "16"))
# the per-GPU share of a whole 8-GPU node (256 host CPUs / 8), the CPU budget a
# reference DataLoader per rank would have there
NODE_SHARE_PER_GPU = 32


def _cgroup_cpus():
    """CPUs granted by the cgroup quota (cpu.max), or None when unlimited/unknown."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        return None if q == "max" else round(float(q) / float(per), 2)
    except (OSError, ValueError):
        return None


def _rates(times, imgs):
    r = sorted(imgs / t for t in times)
    return {"best": round(r[-1], 1), "median": round(r[len(r) // 2], 1), "reps": [round(x, 1) for x in r]}


def cpu_baseline(cells, labels, batch: int = 128, reps: int = 7, workers=None):
    """The reference's CPU path on this host, in this run.

    map-style legs: lance_map_style.py:54-69's harness, i.e. a stock torch
    DataLoader over the SafeLanceDataset shim with the reference PIL collate_fn
    (oracle.pil_collate_fn = lance_map_style.py:21-44: Pillow
    open/convert/Resize((224,224))/to_tensor, stack), batch 128 (config 1),
    pin_memory=True, persistent spawn workers; num_workers = 8 (the reference
    default, :137) and the box's CPU share (or `workers`). Each leg: one batch
    per worker (plus the prefetch queue) to warm up, then `reps` timed runs of
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
    host = len(os.sched_getaffinity(0))
    if workers is None:
        workers = sorted({8, min(host, CPU_SHARE), min(host, NODE_SHARE_PER_GPU)})
    try:
        n = len(cells)
        lds.write_dataset(pa.table({"image": pa.array(cells, pa.binary()),
                                    "label": pa.array(np.asarray(labels, np.int64))}), tmp)
        ds = lds.SafeLanceDataset(tmp)
        legs = []
        for w in workers:
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
                   f"libjpeg-turbo {features.version_feature('libjpeg_turbo')}; legs: num_workers 8 (the "
                   f"reference default), {CPU_SHARE} (this box's CPU share for one GPU) and "
                   f"{NODE_SHARE_PER_GPU} (one GPU's share of a 256-CPU 8-GPU node); host affinity {host} "
                   f"CPUs (the whole-host leg, num_workers = len(os.sched_getaffinity(0)) per BASELINE.md "
                   f"section 3, is --cpu-workers all: it exceeds a one-GPU run's CPU share on the shared "
                   f"box); value = median of the num_workers={ref['num_workers']} leg "
                   f"(lance_map_style.py:137 default)"),
        "legs": legs,
        "host_cpus": host,
        "cgroup_cpus": _cgroup_cpus(),
        "cpu_share": CPU_SHARE,
        "torch_threads": torch.get_num_threads(),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--min-warm-s", type=float, default=0.25,
                    help="untimed warm-up of at least this many seconds beside the W steps")
    ap.add_argument("--workload", default="c2", choices=sorted(WORKLOADS))
    ap.add_argument("--batch", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-workers", default="",
                    help="comma-separated num_workers legs of the CPU baseline (default: 8, the CPU share and "
                         "the per-GPU share of an 8-GPU node; 'all' = len(os.sched_getaffinity(0)))")
    ap.add_argument("--no-stage-events", action="store_true",
                    help="time without the per-stage HIP events (no roofline)")
    ap.add_argument("--depth", type=int, default=None,
                    help="batches in flight (ldt_amd.DecodePipeline: one context + HIP stream each); default 3, "
                         "ldt_amd.PROGRESSIVE_DEPTH (5) for progressive workloads (a c2p batch takes ~13 ms on the device)")
    ap.add_argument("--dataset-batches", type=int, default=100,
                    help="batches per rank of one epoch of the dataset legs at N=1 (divided by the world size, at "
                         "least 12, so that the dataset rank 0 writes stays the same size; 0: skip the legs)")
    ap.add_argument("--dataset-epochs", type=int, default=4,
                    help="epochs in the dataset leg's timed region (each re-plans, as a training loop does; "
                         "4 x 100 c2 batches is ~0.17 s: with 2, single host hiccups moved the copying "
                         "leg by up to 10%% between runs)")
    ap.add_argument("--resize-impl", type=int, default=0,
                    help="LDT_OPT_RESIZE_IMPL of every context (0 auto: k_resize4; 1 its 32-bit 4:2:0 staging; 2 the streaming kernel)")
    ap.add_argument("--resize-waves-pct", type=int, default=0,
                    help="LDT_OPT_RESIZE_WAVES_PCT of every context (0: the library default, 100)")
    ap.add_argument("--resize-wg-waves", type=int, default=0,
                    help="LDT_OPT_RESIZE_WG_WAVES of every context (0: the library default, 2)")
    ap.add_argument("--copy-bind", type=int, default=-1,
                    help="LDT_OPT_COPY_BIND of the host legs (-1: the library default, 2)")
    ap.add_argument("--opt", action="append", default=[],
                    help="ID=VALUE: an extra ldt_set_option on every context of the resident leg (A/B runs)")
    ap.add_argument("--no-config-legs", action="store_true",
                    help="skip the configs[2]/configs[3] dataset legs (c3, c4) of a c2 run")
    ap.add_argument("--no-registered", action="store_true",
                    help="skip the host leg with the cell buffers page-locked in place (ldt_register_host)")
    ap.add_argument("--only-resident", action="store_true",
                    help="the resident leg alone (no host, dataset, config or standalone legs): the run a "
                         "rocprofv3 --stats summary of the line's timed launches is taken from")
    ap.add_argument("--host-depth", type=int, default=None,
                    help="batches in flight of the host-input legs (make_to_tensor_fn(depth)): default "
                         "make_to_tensor_fn's own choice (2 for batches of >= 8 MB of cells, with the cells' copy "
                         "stream: depth + 2 streams fit the process's 4 hardware queues; 3 below), 7 for "
                         "progressive workloads (high-priority slot streams, DecodePipeline)")
    ap.add_argument("--host-reps", type=int, default=3,
                    help="back-to-back runs of the copying host-input leg (value_host_input = their median)")
    ap.add_argument("--dataset-depth", type=int, default=None,
                    help="batches in flight of the dataset legs (default: --depth; 0: make_to_tensor_fn's own choice)")
    ap.add_argument("--dataset-register", action="store_true",
                    help="config legs (c3, c4) with the mapped fragments' image buffers page-locked in place "
                         "(register=True) instead of the copying to_tensor_fn (pylance hands to_tensor_fn a "
                         "fresh RecordBatch per read, lance_iterable.py:38-41, so copying is the realistic case)")
    ap.add_argument("--no-dataset-registered", action="store_true",
                    help="skip the registered-fragment dataset leg (value_dataset_registered)")
    ap.add_argument("--no-workload-legs", action="store_true",
                    help="skip the configs[4] (c5) and progressive (c2p) legs of a c2 run")
    args = ap.parse_args()
    progressive = args.workload.endswith("p")
    # progressive batches spend ~13 ms in k_prog: ldt_amd.PROGRESSIVE_DEPTH (5)
    # in flight, 4 slots on high-priority streams and 1 beside the consumer's
    # (the same rate in a DDP process: DESIGN.md §6)
    PROG_DEPTH = 5  # == ldt_amd.PROGRESSIVE_DEPTH (not imported before torch here)
    if args.depth is None:
        args.depth = PROG_DEPTH if progressive else 3
    if args.dataset_depth is None:
        args.dataset_depth = args.depth
    if args.host_depth is None:
        args.host_depth = PROG_DEPTH if progressive else 0  # 0: make_to_tensor_fn's own choice (depth=None)

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
    numa_cpus = None
    if os.environ.get("LDT_BENCH_NUMA", "1") != "0":
        # this rank on its GPU's NUMA node (numactl --cpunodebind per rank):
        # the host batches below are then allocated there, where the copy
        # pool reads them
        numa_cpus = len(ldt_amd.bind_numa(dev))
    ctx.set_option(_lib.OPT_SYNC_STATUS, 0)
    ctx.set_option(_lib.OPT_PROFILE, 0 if args.no_stage_events else 1)

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    def max_over_ranks(x: float) -> float:
        t = torch.tensor([x], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def timed(step, steps, warmup):
        for _ in range(warmup):
            step()
        barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        barrier()
        return max_over_ranks(time.perf_counter() - t0)

    cells = None
    if args.workload == "c5":
        # synthetic uniform uint8 HWC 1024x1024 generated directly in HBM
        g = torch.Generator(device=dev)
        g.manual_seed(1234 + rank)
        raw = torch.randint(0, 256, (B, 1024, 1024, 3), dtype=torch.uint8, device=dev, generator=g)
        bytes_per_img = 1024 * 1024 * 3 + OUT_BYTES

        def step():
            return ldt_amd.resize_raw(raw, 1024, 1024, device=dev, normalize=True)
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
            batches.append(ldt_amd.ResidentBatch(cells, labels, device=dev))
        px = [ldt_amd_dims(c) for c in cells_all[:B]]
        bytes_per_img = float(np.mean([h * w * 3 for (h, w) in px])) + OUT_BYTES
        comp_bytes = float(np.mean([len(c) for c in cells_all]))
        it = [0]
        pipe = ldt_amd.DecodePipeline(depth=args.depth, device=dev, profile=not args.no_stage_events)
        pipe.set_option(_lib.OPT_RESIZE_IMPL, args.resize_impl)
        if args.resize_waves_pct:
            pipe.set_option(_lib.OPT_RESIZE_WAVES_PCT, args.resize_waves_pct)
        if args.resize_wg_waves:
            pipe.set_option(_lib.OPT_RESIZE_WG_WAVES, args.resize_wg_waves)
        for o in args.opt:
            k, v = o.split("=")
            pipe.set_option(int(k), int(v))

        def step():
            b = batches[it[0] % nb]
            it[0] += 1
            return pipe.decode(b)

    # every slot context sees >= 2 calls (both pinned slots allocated) before timing
    warm = max(args.warmup, 2 * args.depth + 1) if args.workload != "c5" else args.warmup
    prof = ctx if args.workload == "c5" else pipe
    # at least W steps and --min-warm-s seconds untimed: the first ~10 ms of
    # decode after the setup run below the steady rate (K = 20 c2 steps timed
    # right after 7 warm-up steps measured 529k img/s against 570-580k for the
    # same box's later legs, profiles/r4/warm_ab_r4w.txt); the timed region is
    # still exactly K steps
    t_w = time.perf_counter()
    warm_run = 0
    while warm_run < warm or time.perf_counter() - t_w < args.min_warm_s:
        step()
        warm_run += 1
    torch.cuda.synchronize()
    barrier()
    prof.stage_times(reset=True)
    elapsed_max = timed(step, args.steps, 0)
    stages = prof.stage_times(reset=True)
    if args.workload != "c5":
        pipe.check()  # every decoded image status OK
    value = B * args.steps * world / elapsed_max

    # the plug-in boundary: the same steps with the cells in
    # host Arrow RecordBatches through the pipelined to_tensor_fn
    def host_rate(bs, register=False, fn=None):
        """One timed host leg; `fn` = the to_tensor_fn of an earlier leg to
        reuse (a training loop keeps one), else a new one with a full warm-up."""
        fresh = fn is None
        if fresh:
            fn = ldt_amd.make_to_tensor_fn(depth=args.host_depth or None, device=dev, register=register)
            fn.pipeline.set_option(_lib.OPT_HOST_TIMING, 1)
            if args.copy_bind >= 0:
                fn.pipeline.set_option(_lib.OPT_COPY_BIND, args.copy_bind)
            fn.pipeline.set_option(_lib.OPT_RESIZE_IMPL, args.resize_impl)
        k = [0]

        def hstep():
            fn(bs[k[0] % len(bs)])
            k[0] += 1

        # a fresh function's first steps allocate its pinned slots and start
        # its copy pool: at least 50 untimed steps and 0.25 s before the first
        # timed leg (a first leg right after the resident one ran up to 2x slower
        # after 50 steps alone: profiles/r4/spin_ab_r4.txt)
        t_w = time.perf_counter()
        nw = 0
        while nw < (max(warm, 50) if fresh else 2 * fn.pipeline.depth) or \
                (fresh and time.perf_counter() - t_w < 0.25):
            hstep()
            nw += 1
        torch.cuda.synchronize()
        barrier()
        fn.pipeline.host_times(reset=True)
        # each host leg times at least 100 steps (K = 20 batches of c2 are ~9 ms)
        host_steps = max(args.steps, 100)
        t = timed(hstep, host_steps, 0)
        fn.check()
        us, calls = fn.pipeline.host_times(reset=True)
        info = dict(fn.pipeline.ctxs[0].host_info(), host_depth=fn.pipeline.depth)
        if register:
            fn.release()
        return B * host_steps * world / t, {k_: round(v / max(calls, 1), 1) for k_, v in us.items()}, info, fn

    if args.only_resident:
        args.dataset_batches = 0
    value_host = value_registered = host_us = host_info = None
    host_reps = []
    if args.workload != "c5" and not args.only_resident:
        # the copying leg (the plug-in contract: fresh host batches every call)
        # `host_reps` times back to back; value_host_input = the median
        hfn = None
        for _ in range(max(1, args.host_reps)):
            v, host_us, host_info, hfn = host_rate(host_batches, fn=hfn)
            host_reps.append(v)
        value_host = sorted(host_reps)[len(host_reps) // 2]
        del hfn
        if not args.no_registered:
            try:
                value_registered, _, _, _ = host_rate(host_batches, register=True)
            except ldt_amd.LdtError as e:
                print(f"bench: registered host leg skipped: {e}", file=sys.stderr)
    # every rank's host copy placement and host phases (the node's host budget:
    # copy threads per rank from the cgroup quota / LOCAL_WORLD_SIZE, cores on
    # the rank's GPU-local NUMA node)
    host_ranks = None
    if host_info is not None:
        # the rank's host traffic (DESIGN.md §6 host budget): cells moved to
        # HBM per second by the copying leg (= its H2D rate), the copy pool's
        # DRAM rate while it copies (bytes per call / its span), and this
        # box's pinned H2D ceiling
        cell_bytes = comp_bytes * B
        host_gbs = {"h2d_gbs": round(cell_bytes * value_host / world / B / 1e9, 2),
                    "copy_pool_gbs": round(cell_bytes / max(host_us.get("copy_span", 0.0), 1e-3) / 1e3, 2),
                    "h2d_ceiling_gbs": round(h2d_ceiling(dev), 2)}
        mine = {"rank": rank, "local_rank": local, "device": dev.index, "host_us_per_call": host_us, **host_gbs,
                **{k_: host_info[k_] for k_ in ("copy_threads", "copy_cpus", "gpu_numa", "quota_cpus",
                                                 "local_world")}}
        if world > 1:
            host_ranks = [None] * world
            dist.all_gather_object(host_ranks, mine)
        else:
            host_ranks = [mine]

    value_dataset = value_dataset_reg = None
    dataset_info = dataset_reg_info = None
    if args.workload != "c5" and args.dataset_batches > 0:
        # pylance hands to_tensor_fn a fresh RecordBatch per read
        # (lance_iterable.py:38-41, :53-59): value_dataset is the copying
        # to_tensor_fn at its own depth; the registered-fragment variant
        # (register=True, mapped image buffers page-locked once) beside it
        value_dataset, dataset_info = dataset_rate(args, wl, B, world, rank, dev, cells_all, labels_all,
                                                   barrier, max_over_ranks, copy=True,
                                                   keep=not args.no_dataset_registered)
        if not args.no_dataset_registered:
            value_dataset_reg, dataset_reg_info = dataset_rate(args, wl, B, world, rank, dev, cells_all,
                                                               labels_all, barrier, max_over_ranks, copy=False)
    # BASELINE configs[2] (c3) and configs[3] (c4) as written — the reference's
    # iterable loop over FOOD101-shaped / ImageNet-shaped cells with its own
    # sampler — in the same run as the headline, so that every N of a scaling
    # sweep reports them beside it (the headline stays c2, whose per-N values
    # the sweep's efficiency is computed from)
    config_legs = {}
    if args.workload == "c2" and args.dataset_batches > 0 and not args.no_config_legs:
        for cw in ("c3", "c4"):
            cwl = WORKLOADS[cw]
            cb = cwl["batch"]
            cc, cl = [], []
            for k in range(2):
                c_, l_ = make_cells(cw, cb, seed=7000 + 1000 * rank + k)
                cc += c_
                cl += list(l_)
            v, info = dataset_rate(args, cwl, cb, world, rank, dev, cc, cl, barrier, max_over_ranks, tag=cw)
            config_legs[cw] = {"workload": f"{cw}: {cwl['desc']}", "value": round(v, 1),
                               "value_per_gpu": round(v / world, 1), "per_gpu_batch": cb,
                               "compressed_bytes_per_img": round(float(np.mean([len(c) for c in cc])), 1),
                               "dataset_leg": info}

    # standalone launch durations (one batch in flight, after the timed region)
    standalone = None
    if args.workload != "c5" and not args.no_stage_events and not args.only_resident:
        solo = ldt_amd.DecodePipeline(depth=1, device=dev, profile=True)
        solo.set_option(_lib.OPT_RESIZE_IMPL, args.resize_impl)
        for k in range(3):
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

    # configs[4] (c5: raw 1024^2 -> 224 + Normalize, the HBM-roofline stress)
    # and the progressive path (c2p) in the same run as the headline, each
    # with its own roofline / host-input / CPU figures (the driver runs only
    # the default command)
    workload_legs = {}
    if args.workload == "c2" and not args.only_resident and not args.no_workload_legs:
        cpu_ok = rank == 0 and world == 1 and not args.no_cpu_baseline
        # c2p first: after the c5 leg's 3.2 GB host transfers (and its pinned
        # staging) the c2p host-input leg measured 41k img/s against 51.5k
        # in its own line
        workload_legs["c2p"] = leg_c2p(args, dev, world, rank, barrier, max_over_ranks, cpu_ok)
        workload_legs["c5"] = leg_c5(args, dev, world, rank, barrier, max_over_ranks, cpu_ok)


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
        "warmup_run": {"steps": warm_run, "min_s": args.min_warm_s},
        "ms_per_step": round(elapsed_max / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": ("synthetic (seeded PIL-encoded JPEG cells; value: resident in HBM when the timed region starts; "
                 "value_host_input: host Arrow RecordBatches through to_tensor_fn; FOOD101 offline-unavailable)"
                 if args.workload != "c5" else "synthetic (uniform uint8 HWC generated in HBM)"),
        "config": {"workload": f"{args.workload}: {wl['desc']}", "per_gpu_batch": B, "global_batch": B * world,
                   "parallelism": f"dp{world} (independent shards, no data-path collective)",
                   "pipeline_depth": 1 if args.workload == "c5" else args.depth,
                   "input": "resident",
                   "output": "float32[N,3,224,224] + int64[N] on device"},
        "value_per_gpu": round(value / world, 1),
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
    if value_host is not None:
        res["value_host_input"] = round(value_host, 1)
        res["value_host_input_per_gpu"] = round(value_host / world, 1)
        res["value_host_input_note"] = ("the same workload (max(steps, 100) timed steps per leg, after >= 50 "
                                        "steps and 0.25 s of warm-up) with the cells in host pa.RecordBatches "
                                        "through the pipelined to_tensor_fn (make_to_tensor_fn(depth)): pinned copy "
                                        "overlapped with the header walk, one H2D DMA per step on the "
                                        "device's copy stream; median of value_host_input_reps; "
                                        "value_host_registered: the same with the two batches' image buffers "
                                        "page-locked in place (register=True), DMA without the host copy")
        res["host_us_per_call"] = host_us
        res["value_host_input_reps"] = [round(v, 1) for v in host_reps]
        res["host_placement"] = dict(host_info, numa_bound_cpus=numa_cpus)
        res["host_ranks"] = host_ranks
    if value_registered is not None:
        res["value_host_registered"] = round(value_registered, 1)
    if config_legs:
        res["config_legs"] = config_legs
    if value_dataset is not None:
        res["value_dataset"] = round(value_dataset, 1)
        res["value_dataset_per_gpu"] = round(value_dataset / world, 1)
        res["dataset_leg"] = dataset_info
    if value_dataset_reg is not None:
        res["value_dataset_registered"] = round(value_dataset_reg, 1)
        res["value_dataset_registered_per_gpu"] = round(value_dataset_reg / world, 1)
        res["dataset_registered_leg"] = dataset_reg_info
    if workload_legs:
        res["workload_legs"] = workload_legs
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
        res["roofline"]["traffic_source"] = (f"{tr['source']}: rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE "
                                             "passes (FETCH_SIZE x2, gfx950) over this bench at depth 1")
    dec = load_profile(f"pmc_{args.workload}_decode.json")
    if dec is not None:
        res["decode_efficiency"] = dec
    if args.workload != "c5":
        res["config"]["compressed_bytes_per_img"] = round(comp_bytes, 1)
    res["profiles_build"] = {"csrc_sha16": csrc_digest(), "refused_stale": STALE}
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.workload != "c5":
        host_cpus = len(os.sched_getaffinity(0))
        workers = sorted({host_cpus if x == "all" else int(x) for x in args.cpu_workers.split(",") if x}) or None
        res["cpu_baseline"] = cpu_baseline(cells_all, labels_all, workers=workers)
        res["gpu_over_cpu"] = {f"num_workers={leg['num_workers']}": round(value / leg["median"], 1)
                               for leg in res["cpu_baseline"]["legs"]}
        if value_host is not None:
            res["gpu_over_cpu_host_input"] = {f"num_workers={leg['num_workers']}": round(value_host / leg["median"], 1)
                                              for leg in res["cpu_baseline"]["legs"]}
    elif rank == 0 and world == 1 and args.workload == "c5" and not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline_raw(raw[:8].cpu().numpy())
        res["gpu_over_cpu"] = round(value / res["cpu_baseline"]["value"], 2)
    # the headline figures once more at the end of the line, after the long
    # cpu_baseline / workload_legs blobs, so that a tail of the output keeps them
    summary = {k: res[k] for k in ("value", "value_host_input", "value_host_registered", "value_dataset",
                                   "value_dataset_registered") if k in res}
    if config_legs:
        summary.update({f"config_legs.{k}": v["value"] for k, v in config_legs.items()})
    for k, v in workload_legs.items():
        summary[f"workload_legs.{k}"] = v["value"]
        if "value_host_input" in v:
            summary[f"workload_legs.{k}.host_input"] = v["value_host_input"]
    if "gpu_over_cpu" in res:
        summary["gpu_over_cpu"] = res["gpu_over_cpu"]
    summary["roofline.frac"] = res["roofline"]["frac"]
    if "standalone" in res["roofline"]:
        summary["roofline.standalone.frac"] = res["roofline"]["standalone"]["frac"]
    res["summary"] = summary
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


def dataset_rate(args, wl, B, world, rank, dev, cells, labels, barrier, max_over_ranks, tag=None, copy=None,
                 keep=False):
    """The reference's iterable loop (lance_iterable.py:53-72, :86-116) over an
    Arrow/Lance dataset of this workload's cells: LanceDataset + the sampler +
    the pipelined to_tensor_fn, `dataset_epochs` full epochs per rank in the
    timed region (each epoch's plan — device shard kernel, and for pad=True
    the all_reduce(MAX) over the process group — included). Rank 0 writes the
    dataset (the workload's cells repeated to `dataset_batches` batches per
    rank) into fragments of the config's shape; every rank then runs one
    untimed epoch and the timed ones. Padding batches (pad=True) are decoded
    and counted. `copy` (default: not --dataset-register): the copying
    to_tensor_fn at make_to_tensor_fn's own depth, else registered fragments at
    --dataset-depth. `keep`: leave the dataset for the next leg over the same
    cells (it is then not written again; an exception removes it). Returns
    (whole-job img/s, info)."""
    import shutil

    import numpy as np
    import pyarrow as pa

    import ldt_amd
    from ldt_amd import _lib

    copy = not args.dataset_register if copy is None else copy
    # the dataset rank 0 writes holds every rank's rows: per-rank batches
    # shrink with the world size (at least 12, or the whole request when that
    # is smaller) so that it stays ~1.7 GB at c2
    nbatch = max(min(12, args.dataset_batches), args.dataset_batches // world)
    # FOOD101's fragments [12500 x 6, 750] (create_datasets/classification.py:16,60)
    # scaled so that a rank reads about `nbatch` batches
    if wl["sampler"] == "fragment":
        # ShardedFragmentSampler: rank r owns fragments r, r+W, ...; at W = 8
        # ranks 0-5 own a full fragment, rank 6 the short one, rank 7 none
        F = max(1, round(nbatch / -(-6 // world))) * B
    else:
        # ShardedBatchSampler: global row ranges, nbatch per rank
        F = -(-(nbatch * B * world * 12500 // 75750) // B) * B
    sizes = [F] * 6 + [max(1, F * 750 // 12500)]
    if wl["sampler"] != "fragment":
        sizes = [F] * (nbatch * B * world // F) + ([nbatch * B * world % F] if nbatch * B * world % F else [])
    rows = sum(sizes)
    import tempfile

    # the path names every size the dataset depends on; a directory left by an
    # interrupted run is reused only when its row count matches
    path = os.path.join(tempfile.gettempdir(),
                        f"ldt_bench_ds_{os.environ.get('MASTER_PORT', '0')}_{tag or args.workload}_{world}"
                        f"_n{len(cells)}_b{B}_f{F}_r{rows}")
    if rank == 0:
        if os.path.isdir(path):
            try:
                ok = ldt_amd.dataset(path).count_rows() == rows
            except Exception:
                ok = False
            if not ok:
                shutil.rmtree(path, ignore_errors=True)
        if not os.path.isdir(path):
            n = len(cells)
            idx = np.arange(rows) % n
            tbl = pa.table({"image": pa.array([cells[i] for i in idx], pa.binary()),
                            "label": pa.array(np.asarray(labels, np.int64)[idx])})
            ldt_amd.write_dataset(tbl, path, max_rows_per_file=F)
            del tbl
    barrier()
    try:
        return _dataset_epochs(args, wl, B, world, rank, dev, path, rows, sizes, nbatch, copy, barrier,
                               max_over_ranks)
    finally:
        if rank == 0 and not keep:
            shutil.rmtree(path, ignore_errors=True)


def _dataset_epochs(args, wl, B, world, rank, dev, path, rows, sizes, nbatch, copy, barrier, max_over_ranks):
    """dataset_rate's timed part over the dataset at `path`."""
    import ldt_amd
    from ldt_amd import _lib

    if wl["sampler"] == "fragment":
        sampler = ldt_amd.ShardedFragmentSampler(rank=rank, world_size=world, pad=True)
    else:
        sampler = ldt_amd.ShardedBatchSampler(rank=rank, world_size=world)
    # the fragments are memory-mapped Arrow IPC files whose image buffers live
    # as long as the dataset: page-locked once per fragment (register=True),
    # every batch sliced from them is DMAed without a host copy
    # 3 in flight as the resident leg: the configs' batches of 128 need the
    # concurrency more than the copy stream (DMA on the slot streams here,
    # DecodePipeline's choice at depth 3)
    fn = ldt_amd.make_to_tensor_fn(depth=None if copy else (args.dataset_depth or None), device=dev,
                                   register=not copy)
    fn.pipeline.set_option(_lib.OPT_RESIZE_IMPL, args.resize_impl)
    ds = ldt_amd.LanceDataset(path, batch_size=B, sampler=sampler, to_tensor_fn=fn)

    def epoch():
        imgs = 0
        for b in ds:  # lance_iterable.py:107-109: batch["image"].to(device) is a no-op here
            imgs += b["image"].shape[0]
        return imgs

    epoch()
    fn.check()
    barrier()
    t0 = time.perf_counter()
    imgs = sum(epoch() for _ in range(args.dataset_epochs))
    barrier()
    t = max_over_ranks(time.perf_counter() - t0)
    fn.check()
    tot_imgs = imgs
    if world > 1:
        import torch
        import torch.distributed as dist

        tt = torch.tensor([imgs], dtype=torch.int64, device=dev if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(tt)
        tot_imgs = int(tt.item())
    barrier()
    info = {"sampler": type(sampler).__name__ + ("(pad=True)" if wl["sampler"] == "fragment" else ""),
            "rows": rows, "fragments": sizes if len(sizes) <= 16 else f"{len(sizes)} fragments",
            "target_batches_per_rank": nbatch, "epochs": args.dataset_epochs,
            "images_all_ranks": tot_imgs, "elapsed_ms_max": round(t * 1e3, 3),
            "timing": "full epochs per rank (plan + every batch, padding included) between barriers, "
                      "max over ranks",
            "harness": (f"LanceDataset(path, batch_size, sampler, to_tensor_fn=make_to_tensor_fn(depth={fn.pipeline.depth}, "
                        f"register={not copy}))")}
    return tot_imgs / t, info


def _warm_then_time(step, steps, warm, min_s, barrier, max_over_ranks):
    """At least `warm` untimed steps and `min_s` seconds, then exactly `steps`
    timed between barriers (max over ranks)."""
    t_w = time.perf_counter()
    n = 0
    while n < warm or time.perf_counter() - t_w < min_s:
        step()
        n += 1
    barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    barrier()
    return max_over_ranks(time.perf_counter() - t0)


def leg_c5(args, dev, world, rank, barrier, max_over_ranks, cpu_ok):
    """BASELINE configs[4]: raw uint8 HWC 1024x1024 -> Resize(224,224) +
    Normalize (lance_iterable.py:29-31), batch 1024 per GPU, the HBM-roofline
    stress of the resize/normalise stage. `value`: the cells in HBM (generated
    there); roofline from the resize launches' HIP events over the timed
    region; `value_host_input` (N=1): the same batch from pageable host memory
    through ldt_resize_raw (pinned copy + one H2D per step: PCIe/host bound,
    SURVEY.md §8(d)); CPU leg: Pillow resize + to_tensor + Normalize."""
    import torch

    import ldt_amd
    from ldt_amd import _lib

    B, H, W = WORKLOADS["c5"]["batch"], 1024, 1024
    g = torch.Generator(device=dev)
    g.manual_seed(1234 + rank)
    raw = torch.randint(0, 256, (B, H, W, 3), dtype=torch.uint8, device=dev, generator=g)
    ctx = _lib.get_context(dev.index)
    ctx.set_option(_lib.OPT_PROFILE, 1)
    K = max(args.steps, 20)
    ctx.stage_times(reset=True)
    t = _warm_then_time(lambda: ldt_amd.resize_raw(raw, H, W, device=dev, normalize=True), K, 3, 0.25, barrier, max_over_ranks)
    st = ctx.stage_times(reset=True)
    bpi = H * W * 3 + OUT_BYTES
    ms, n = st["resize"]
    avg_s = ms / max(n, 1) / 1e3
    ach = bpi * B / avg_s / 1e9 if avg_s > 0 else 0.0
    leg = {"workload": f"c5: {WORKLOADS['c5']['desc']}", "per_gpu_batch": B,
           "value": round(B * K * world / t, 1), "value_per_gpu": round(B * K / t, 1),
           "input": "resident (generated in HBM)", "steps": K, "ms_per_step": round(t / K * 1e3, 3),
           "roofline": {"kernel": "k_resize4<raw> (BILINEAR 224 + Normalize store)", "bound": "hbm",
                        "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(ach / HBM_PEAK_GBS, 4), "bytes_per_unit": bpi,
                        "unit_basis": "SURVEY.md §8(d): 1024*1024*3 + 602,112 B per image",
                        "avg_launch_ms": round(avg_s * 1e3, 4),
                        "timing": "HIP events around every resize launch over the timed region (one batch in "
                                  "flight, so per-launch durations)"}}
    tr = load_profile("traffic_c5.json")
    if tr is not None and tr.get("batch", B) == B:
        leg["roofline"]["traffic"] = tr["hbm_bytes_per_launch"]
        leg["roofline"]["traffic_source"] = tr.get("source")
    if world == 1:
        host = raw.cpu()
        th = _warm_then_time(lambda: ldt_amd.resize_raw(host, H, W, device=dev, normalize=True), 3, 1, 0.0, barrier,
                             max_over_ranks)
        leg["value_host_input"] = round(B * 3 / th, 1)
        leg["value_host_input_note"] = ("pageable host uint8 [1024,1024,1024,3] -> ldt_resize_raw: pinned "
                                        "copy + one 3.2 GB H2D per step, then the kernel (3 timed steps); "
                                        "bound by the host copy and PCIe, not the GPU")
        del host
    if cpu_ok:
        leg["cpu_baseline"] = cpu_baseline_raw(raw[:8].cpu().numpy(), budget_s=3.0)
        leg["gpu_over_cpu"] = round(leg["value"] / leg["cpu_baseline"]["value"], 1)
    del raw
    torch.cuda.empty_cache()
    return leg


def leg_c2p(args, dev, world, rank, barrier, max_over_ranks, cpu_ok):
    """The c2 images encoded progressive (SOF2), batch
    256, 5 in flight (DecodePipeline: 4 slots on high-priority streams):
    `value` with the cells resident (DecodePipeline(depth=PROGRESSIVE_DEPTH)),
    `value_host_input` from a host RecordBatch (make_to_tensor_fn(depth=PROGRESSIVE_DEPTH)); CPU leg: the
    reference map-style DataLoader at this box's CPU share of workers."""
    import numpy as np
    import pyarrow as pa
    import torch

    import ldt_amd
    from ldt_amd import _lib

    B = WORKLOADS["c2p"]["batch"]
    cells, labels = make_cells("c2p", B, seed=1000 * rank)
    rb = ldt_amd.ResidentBatch(cells, labels, device=dev)
    # the resident leg on its own 7-deep pipeline, the host leg on the
    # to_tensor_fn's (both on the device's shared slot streams)
    pipe = ldt_amd.DecodePipeline(depth=ldt_amd.PROGRESSIVE_DEPTH, device=dev)
    for c in pipe.ctxs:
        c.set_option(_lib.OPT_PROFILE, 1)
    # ~4 ms per batch 5 deep: at least 60 steps, so that fill and drain stay small
    K = max(args.steps, 60)
    pipe.stage_times(reset=True)
    t = _warm_then_time(lambda: pipe.decode(rb), K, 15, 0.25, barrier, max_over_ranks)
    st = pipe.stage_times(reset=True)
    pipe.check()
    for c in pipe.ctxs:
        c.set_option(_lib.OPT_PROFILE, 0)
    leg = {"workload": f"c2p: {WORKLOADS['c2p']['desc']}", "per_gpu_batch": B, "pipeline_depth": ldt_amd.PROGRESSIVE_DEPTH,
           "value": round(B * K * world / t, 1), "value_per_gpu": round(B * K / t, 1), "steps": K,
           "compressed_bytes_per_img": round(float(np.mean([len(c) for c in cells])), 1),
           "stages_ms_per_launch": {k: round(v[0] / max(v[1], 1), 4) for k, v in st.items()}}
    del pipe
    host = pa.RecordBatch.from_arrays([pa.array(cells, pa.binary()), pa.array(np.asarray(labels, np.int64))],
                                      names=["image", "label"])
    fn = ldt_amd.make_to_tensor_fn(depth=ldt_amd.PROGRESSIVE_DEPTH, device=dev)
    th = _warm_then_time(lambda: fn(host), K, 15, 0.25, barrier, max_over_ranks)
    fn.check()
    leg["value_host_input"] = round(B * K * world / th, 1)
    leg["value_host_input_per_gpu"] = round(B * K / th, 1)
    del fn
    torch.cuda.synchronize(dev)
    if cpu_ok:
        share = min(len(os.sched_getaffinity(0)), CPU_SHARE)
        cb = cpu_baseline(cells, labels, reps=3, workers=[share])
        leg["cpu_baseline"] = cb
        leg["gpu_over_cpu_host_input"] = round(leg["value_host_input"] / cb["value"], 1)
    return leg


PROFILE_ROUND = "r6"  # committed PMC summaries: this round's, else the newest earlier one


def h2d_ceiling(dev, nbytes: int = 256 << 20, reps: int = 5) -> float:
    """Pinned host -> HBM copy rate in GB/s (best of `reps` 256 MB DMAs)."""
    import torch

    src = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    dst = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    dst.copy_(src, non_blocking=True)
    torch.cuda.synchronize(dev)
    best = 0.0
    for _ in range(reps):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        dst.copy_(src, non_blocking=True)
        e1.record()
        e1.synchronize()
        best = max(best, nbytes / (e0.elapsed_time(e1) / 1e3) / 1e9)
    del src, dst
    return best


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


def csrc_digest() -> str:
    """sha256 (16 hex digits) over the kernel and ABI sources (csrc/*.hip,
    *.cpp, *.hpp and include/ldt.h): the build a PMC summary was measured on.
    The tools that write profiles/ summaries record it (tools/traffic_summary.py,
    tools/decode_eff.py)."""
    import hashlib

    h = hashlib.sha256()
    d = os.path.join(REPO, "lance-distributed-training_amd", "csrc")
    for name in sorted(os.listdir(d)):
        if name.endswith((".hip", ".cpp", ".hpp")):
            h.update(name.encode())
            with open(os.path.join(d, name), "rb") as f:
                h.update(f.read())
    with open(os.path.join(REPO, "include", "ldt.h"), "rb") as f:
        h.update(f.read())
    return h.hexdigest()[:16]


STALE = []  # committed summaries refused by load_profile (reported in the line)


def load_profile(name: str):
    """A committed PMC summary under profiles/<round>/ — this round's, else the
    newest earlier round's — measured on the current kernels: its recorded
    csrc_sha16 must equal csrc_digest(), so a summary of older kernels (or one
    without the digest) is refused and listed in STALE. None if absent or
    stale; the dict gains its source path."""
    rnd = int(PROFILE_ROUND[1:])
    cur = csrc_digest()
    for r in range(rnd, 0, -1):
        path = os.path.join(REPO, "profiles", f"r{r}", name)
        if os.path.exists(path):
            with open(path) as f:
                d = json.load(f)
            rel = os.path.relpath(path, REPO)
            if not isinstance(d, dict) or d.get("csrc_sha16") != cur:
                STALE.append({"file": rel, "csrc_sha16": d.get("csrc_sha16") if isinstance(d, dict) else None,
                              "current": cur})
                return None
            d.setdefault("source", rel)
            return d
    return None


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


def cpu_baseline_raw(hwc, budget_s: float = 5.0):
    """Config 5 CPU leg: Pillow resize + to_tensor + Normalize, 1 process."""
    import numpy as np
    from PIL import Image

    MEAN = np.asarray((0.485, 0.456, 0.406), np.float32)[:, None, None]
    STD = np.asarray((0.229, 0.224, 0.225), np.float32)[:, None, None]
    t0 = time.perf_counter()
    reps = 0
    while time.perf_counter() - t0 < budget_s:
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
