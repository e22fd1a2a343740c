"""MFMA utilisation per kernel from a rocprofv3 --pmc pass holding SQ_VALU_MFMA_BUSY_CYCLES
and GRBM_GUI_ACTIVE: the MFMA-busy cycles summed over the SIMDs / (the kernel's GPU-busy cycles x
1024 SIMDs), where the kernel's cycles are GRBM_GUI_ACTIVE / 8 (rocprofv3 reports GRBM_GUI_ACTIVE
summed over the 8 XCDs: MI355X_MICROARCH.md, DVFS give-back).

  python tools/mfma_util.py <pmc dir> [kernel-name substring ...]
"""
import collections
import csv
import glob
import json
import os
import re
import sys

SIMDS = 1024  # 256 CUs x 4 SIMDs (MI355X)


def main():
    d = sys.argv[1]
    keys = sys.argv[2:] or ["fd_main_kernel", "attn_", "wgrad_v2"]
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    names, grids = {}, {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            did = r["Dispatch_Id"]
            names[did], grids[did] = r["Kernel_Name"], r.get("Grid_Size", "")
            per[did][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = collections.defaultdict(list)
    raw = collections.defaultdict(lambda: collections.defaultdict(list))
    for did, c in per.items():
        n = names[did]
        k = next((k for k in keys if k in n), None)
        if k is None or "SQ_VALU_MFMA_BUSY_CYCLES" not in c or "GRBM_GUI_ACTIVE" not in c:
            continue
        busy, gui = sum(c["SQ_VALU_MFMA_BUSY_CYCLES"]), sum(c["GRBM_GUI_ACTIVE"]) / 8.0
        short = re.split(r"[(<]", n.replace("(anonymous namespace)::", "").replace("void ", ""))[0][-60:]
        out[(short, grids[did])].append(busy / (gui * SIMDS))
        for cn, vals in c.items():  # every counter of the pass, summed over its instances
            raw[(short, grids[did])][cn].append(sum(vals))
    res = {}
    for (n, g), v in out.items():
        r = {"mfma_util": round(sum(v) / len(v), 4), "dispatches": len(v)}
        cs = {cn: sum(x) / len(x) for cn, x in raw[(n, g)].items()}
        r["counters_per_dispatch"] = {cn: float(f"{x:.4g}") for cn, x in sorted(cs.items())}
        if cs.get("SQ_INSTS_MFMA"):
            r["valu_per_mfma"] = round(cs.get("SQ_INSTS_VALU", 0.0) / cs["SQ_INSTS_MFMA"], 3)
            r["mfma_busy_per_mfma"] = round(cs["SQ_VALU_MFMA_BUSY_CYCLES"] / cs["SQ_INSTS_MFMA"], 2)
        res[f"{n} grid={g}"] = r
    # whole calls: a main pass with the prep dispatch right before it (busy and active cycles summed)
    order = sorted(per, key=lambda x: int(x))
    calls = collections.defaultdict(list)
    for prev, did in zip(order, order[1:]):
        n, pn = names[did], names[prev]
        c, pc = per[did], per[prev]
        if "prep" in pn and "prep" not in n and all(k in x for x in (c, pc)
                                                    for k in ("SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE")):
            busy = sum(c["SQ_VALU_MFMA_BUSY_CYCLES"]) + sum(pc["SQ_VALU_MFMA_BUSY_CYCLES"])
            gui = (sum(c["GRBM_GUI_ACTIVE"]) + sum(pc["GRBM_GUI_ACTIVE"])) / 8.0
            short = re.split(r"[(<]", n.replace("(anonymous namespace)::", "").replace("void ", ""))[0][-60:]
            calls[short].append(busy / (gui * SIMDS))
    for n, v in calls.items():
        res[f"whole call: prep + {n}"] = {"mfma_util": round(sum(v) / len(v), 4), "calls": len(v)}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
