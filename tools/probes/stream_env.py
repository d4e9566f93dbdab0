"""Does the pipeline's rate survive a DDP-like process?

One process per run (stream-to-queue binding is per process): creates the
streams a DDP training process would (lance_iterable.py:80,95: the process
group and DDP before the loop) BEFORE or AFTER building the to_tensor_fn, then
times the host-input legs of c2 (make_to_tensor_fn(), adaptive) and c2p
(make_to_tensor_fn(depth=ldt_amd.PROGRESSIVE_DEPTH)) with a comm-like stream the consumer waits on at
every step (DDP's gradient all-reduce). usage:
    python tools/probes/stream_env.py clean|before|ref|after [c2|c2p] [steps]
(ref: the reference's order, lance_iterable.py:78-95: pipeline built, then
the process group / DDP streams, then the pipeline's first batch)
Prints one JSON line."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "lance-distributed-training_amd"))
sys.path.insert(0, REPO)


def ddp_env(dev):
    """Process group (RCCL, world 1, one all_reduce so that its communicator
    and streams exist), four torch side streams used once, and the comm-like
    stream returned for the per-step wait. LDT_ENV_PG=0 / LDT_ENV_SIDE=0 /
    LDT_ENV_COMM=0 leave out the process group, the side streams, or the
    comm stream's per-step wait (isolating which part costs the pipeline)."""
    import torch
    import torch.distributed as dist

    t = torch.ones(1 << 20, device=dev)
    if os.environ.get("LDT_ENV_PG", "1") == "1":
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(29500 + os.getpid() % 1000))
        dist.init_process_group("nccl", rank=0, world_size=1)
        dist.all_reduce(t)
    side = [torch.cuda.Stream(dev) for _ in range(int(os.environ.get("LDT_ENV_SIDE", "4")))]
    for s in side:
        with torch.cuda.stream(s):
            t.add_(1)
    comm = torch.cuda.Stream(dev)
    torch.cuda.synchronize(dev)
    return comm, side, t


def main():
    mode = sys.argv[1]
    wl = sys.argv[2] if len(sys.argv) > 2 else "c2"
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 100
    import numpy as np
    import pyarrow as pa
    import torch

    import ldt_amd
    from bench import make_cells

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    comm = side = buf = None
    if mode == "before":
        comm, side, buf = ddp_env(dev)
    depth = int(os.environ.get("LDT_PROBE_DEPTH", "0")) or (ldt_amd.PROGRESSIVE_DEPTH if wl == "c2p" else None)
    if os.environ.get("LDT_PROBE_PREV") == "1":
        # an earlier pipeline of the process (a c2 to_tensor_fn), used, then dropped
        import pyarrow as pa0
        from bench import make_cells as mc0

        prev = ldt_amd.make_to_tensor_fn(device=dev)
        cp, lp = mc0("c2", 64, seed=13)
        rb0 = pa0.RecordBatch.from_arrays([pa0.array(cp, pa0.binary()), pa0.array(np.asarray(lp, np.int64))],
                                          names=["image", "label"])
        for _ in range(4):
            prev(rb0)
        torch.cuda.synchronize(dev)
        del prev
    fn = ldt_amd.make_to_tensor_fn(depth=depth, device=dev)
    if mode == "ref":
        # lance_iterable.py:78-95's order: the to_tensor_fn (and its streams)
        # built with the dataset, then DDP's collectives and streams, then the
        # loop's first batch
        comm, side, buf = ddp_env(dev)
    resident = os.environ.get("LDT_PROBE_RESIDENT") == "1"
    B = 256
    cells, labels = make_cells(wl, B, seed=11)
    host = [pa.RecordBatch.from_arrays([pa.array(cells, pa.binary()), pa.array(np.asarray(labels, np.int64))],
                                       names=["image", "label"])]
    cells2, labels2 = make_cells(wl, B, seed=12)
    host.append(pa.RecordBatch.from_arrays([pa.array(cells2, pa.binary()),
                                            pa.array(np.asarray(labels2, np.int64))], names=["image", "label"]))
    fn(host[0])  # first use of the pipeline's streams
    torch.cuda.synchronize(dev)
    if mode == "after":
        comm, side, buf = ddp_env(dev)
    k = [0]

    rbs = [ldt_amd.ResidentBatch(cells, labels, device=dev), ldt_amd.ResidentBatch(cells2, labels2, device=dev)]

    def step():
        out = fn.pipeline.decode(rbs[k[0] % 2]) if resident else fn(host[k[0] % 2])
        k[0] += 1
        if comm is not None and os.environ.get("LDT_ENV_COMM", "1") == "1":
            # DDP-like: the consumer's stream waits for a comm-stream op
            comm.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(comm):
                buf.mul_(1.0)
            torch.cuda.current_stream(dev).wait_stream(comm)
        return out

    t0 = time.perf_counter()
    n = 0
    while n < 60 or time.perf_counter() - t0 < 0.5:
        step()
        n += 1
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    fn.check()
    print(json.dumps({"mode": mode, "workload": wl, "img_s": round(B * steps / dt, 1), "steps": steps,
                      "slot_priority_env": os.environ.get("LDT_SLOT_PRIORITY"),
                      "depth": fn.pipeline.depth, "high_priority": fn.pipeline.high_priority,
                      "resident": resident}), flush=True)
    import torch.distributed as dist

    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
