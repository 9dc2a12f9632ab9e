"""Per-variant effective clock and MFMA busy from scripts/clock_ab.sh (rocprofv3 --kernel-trace + --pmc
GRBM_GUI_ACTIVE / SQ_* of the fused kernels).  Diagnostic.

effective clock = GRBM_GUI_ACTIVE / 8 XCDs / kernel duration (MI355X_MICROARCH.md, DVFS give-back)
"""
import csv
import glob
import os
import sys

for d in sys.argv[1:]:
    ctr = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if "rdn::" not in r["Kernel_Name"] or "generate" in r["Kernel_Name"]:
                    continue
                k = int(r["Dispatch_Id"])
                ctr.setdefault(k, {}).setdefault(r["Counter_Name"], 0.0)
                ctr[k][r["Counter_Name"]] += float(r["Counter_Value"])
    dur = {}
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                dur[int(r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    rows = [(k, c, dur[k]) for k, c in sorted(ctr.items()) if k in dur and dur[k] > 2e-3]
    if not rows:
        print(d, "no dispatches")
        continue
    clk = [c["GRBM_GUI_ACTIVE"] / 8 / t / 1e9 for _, c, t in rows]
    busy = [c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / max(c.get("SQ_BUSY_CU_CYCLES", 1), 1) / 4 for _, c, t in rows]
    ms = [t * 1e3 for _, _, t in rows]
    print(f"{os.path.basename(d.rstrip('/')):10s} dispatches {len(rows):3d}  kernel ms {sorted(ms)[len(ms) // 2]:8.3f}  "
          f"clock GHz {sorted(clk)[len(clk) // 2]:.3f}  mfma_busy/(4 x busy_cu) {sorted(busy)[len(busy) // 2]:.3f}")
