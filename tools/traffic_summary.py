"""Per-launch HBM traffic of the resize kernel from tools/traffic.sh output.

FETCH_SIZE / WRITE_SIZE are rocprofv3's derived counters in KiB per dispatch
(TCC memory-side requests). MI355X_MICROARCH.md (HBM section): on gfx950
FETCH_SIZE reports exactly half the bytes of wide streaming reads (128-B
requests tallied at 64 B), so it is doubled; WRITE_SIZE is exact for 16-B
stores. Printed as JSON; bench.py embeds it as roofline.traffic."""
import csv, glob, json, os, sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import csrc_digest  # noqa: E402

d, workload = sys.argv[1], sys.argv[2]
vals = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    per = []
    for f in glob.glob(f"{d}/{c}/*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if "k_resize" in r["Kernel_Name"] and r["Counter_Name"] == c:
                per.append(float(r["Counter_Value"]))
    vals[c] = per
bench = {}
try:  # the bench line of the FETCH_SIZE pass: batch and algorithmic bytes
    for line in open(f"{d}/FETCH_SIZE.log"):
        if line.startswith("{"):
            bench = json.loads(line)
except OSError:
    pass
fetch = sum(vals["FETCH_SIZE"]) / max(len(vals["FETCH_SIZE"]), 1) * 1024
write = sum(vals["WRITE_SIZE"]) / max(len(vals["WRITE_SIZE"]), 1) * 1024
print(json.dumps({
    "csrc_sha16": csrc_digest(),
    "workload": workload, "kernel": "k_resize4", "dispatches": [len(vals["FETCH_SIZE"]), len(vals["WRITE_SIZE"])],
    "fetch_size_raw_bytes": round(fetch), "write_size_bytes": round(write),
    "hbm_bytes_per_launch": round(2 * fetch + write),
    "correction": "FETCH_SIZE x2 (gfx950 128-B read requests tallied at 64 B, MI355X_MICROARCH.md HBM)",
    "batch": bench.get("config", {}).get("per_gpu_batch"),
    "algorithmic_bytes_per_launch": round(bench["roofline"]["bytes_per_unit"] * bench["config"]["per_gpu_batch"])
    if bench else None,
    "note": "JPEG: the kernel reads Y/Cb/Cr planes (1.5 B/px at 4:2:0), not RGB; traffic below the algorithmic "
            "H*W*3 basis is expected" if workload != "c5" else "raw HWC uint8 in, float32 CHW out",
}))
