"""Side-by-side per-dispatch PMC averages of the fused RRCDNet kernel from scripts/gpu_pmc.sh runs.

    python tools/pmc_compare.py gpurun_out/pmc_f16f8 gpurun_out/pmc_bf16x3 ...
"""
import csv
import glob
import os
import sys


def collect(d):
    vals = {}
    for f in glob.glob(os.path.join(d, "p*", "*counter_collection.csv")):
        per = {}
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if "rrcdnet" not in r["Kernel_Name"]:
                    continue
                k = (r["Counter_Name"], r["Dispatch_Id"])
                per[k] = per.get(k, 0.0) + float(r["Counter_Value"])
        agg = {}
        for (n, _), v in per.items():
            agg.setdefault(n, []).append(v)
        for n, v in agg.items():
            vals[n] = sum(v) / len(v)
    return vals


dirs = sys.argv[1:]
data = [collect(d) for d in dirs]
names = sorted(set().union(*data))
print(f"{'counter':28s}" + "".join(f"{os.path.basename(d):>18s}" for d in dirs))
for n in names:
    print(f"{n:28s}" + "".join(f"{x.get(n, float('nan')):18.4g}" for x in data))
for x, d in zip(data, dirs):
    g = x.get("GRBM_GUI_ACTIVE", 1)
    se = 32  # SQ_* PMC values are summed over the XCDs' SEs; ratios below are per-CU-cycle proxies
    print(os.path.basename(d),
          "mfma_busy/busy_cu %.3f" % (x.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / max(x.get("SQ_BUSY_CU_CYCLES", 1), 1)),
          "lds_active/busy_cu %.3f" % (x.get("SQ_LDS_IDX_ACTIVE", 0) / max(x.get("SQ_BUSY_CU_CYCLES", 1), 1)),
          "bank_conf/lds_active %.3f" % (x.get("SQ_LDS_BANK_CONFLICT", 0) / max(x.get("SQ_LDS_IDX_ACTIVE", 1), 1)),
          "wait_lds/wave_cyc %.3f" % (x.get("SQ_WAIT_INST_LDS", 0) / max(x.get("SQ_WAVE_CYCLES", 1), 1)),
          "wait_any/wave_cyc %.3f" % (x.get("SQ_WAIT_ANY", 0) / max(x.get("SQ_WAVE_CYCLES", 1), 1)),
          "wait_inst/wave_cyc %.3f" % (x.get("SQ_WAIT_INST_ANY", 0) / max(x.get("SQ_WAVE_CYCLES", 1), 1)))
