"""Per-kernel efficiency from tools/pmc.sh passes (SQ + GRBM counters).

  valu_util   = SQ_INSTS_VALU * 2 / (cycles * 1024): a wave64 VALU instruction
                holds a SIMD-32 for 2 cycles (MI355X_MICROARCH.md), 1024 SIMDs;
                cycles = GRBM_GUI_ACTIVE / 8 (summed over the 8 XCDs)
  valu_active = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES (share of wave lifetime
                issuing VALU)
  lds_bank_conflict = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
usage: python tools/decode_eff.py <pmc dir> <workload> > summary.json"""
import collections, csv, glob, json, os, sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import csrc_digest  # noqa: E402

d, wl = sys.argv[1], sys.argv[2]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{d}/p*/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("ldt::", "")
        acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {"csrc_sha16": csrc_digest(), "workload": wl, "source": "rocprofv3 --pmc passes (tools/pmc.sh) over one batch at a time", "kernels": {}}
for k, c in sorted(acc.items()):
    m = {n: sum(v) / len(v) for n, v in c.items()}
    if "SQ_INSTS_VALU" not in m or "GRBM_GUI_ACTIVE" not in m:
        continue
    cyc = m["GRBM_GUI_ACTIVE"] / 8.0
    e = {"cycles": round(cyc), "valu_util": round(m["SQ_INSTS_VALU"] * 2 / (cyc * 1024), 4)}
    if m.get("SQ_WAVE_CYCLES"):
        e["valu_active"] = round(m.get("SQ_ACTIVE_INST_VALU", 0) / m["SQ_WAVE_CYCLES"], 4)
        e["wait_any"] = round(m.get("SQ_WAIT_ANY", 0) / m["SQ_WAVE_CYCLES"], 4)
    if m.get("SQ_LDS_IDX_ACTIVE"):
        e["lds_bank_conflict"] = round(m.get("SQ_LDS_BANK_CONFLICT", 0) / m["SQ_LDS_IDX_ACTIVE"], 4)
    e["valu_insts"] = round(m["SQ_INSTS_VALU"])
    e["waves"] = round(m.get("SQ_WAVES", 0))
    out["kernels"][k] = e
print(json.dumps(out, indent=1))
