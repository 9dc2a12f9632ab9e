"""Per-variant PMC averages of an A/B run of tools/ablate.py under rocprofv3 --pmc (diagnostic).

tools/ablate.py run interleaves its libraries: per round, each library gets one warm-up and three timed
launches of the same kernel, in ABLATE_ONLY order.  This script assigns the kernel's dispatches to the
variants by that order and reports, per variant, the mean of every counter and the ratios DESIGN cites
(MFMA busy of SIMD cycles, VALU-MFMA co-execution share of the MFMA-busy cycles).

    python tools/coexec_ab.py gpurun_out/final6 rdn::h16fw::rrcdnet_walk base,prio > profiles/r06/rocprof/coexec_ab.json
"""
import csv
import glob
import json
import os
import sys


def main():
    src, kernel, names = sys.argv[1], sys.argv[2], sys.argv[3].split(",")
    per = {n: {} for n in names}
    for d in sorted(glob.glob(os.path.join(src, "coexec_*"))):
        if not os.path.isdir(d):
            continue
        rows = {}
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    if kernel in r["Kernel_Name"]:
                        key = int(r.get("Dispatch_Id") or r.get("Correlation_Id") or 0)
                        rows.setdefault(key, {}).setdefault(r["Counter_Name"], 0.0)
                        rows[key][r["Counter_Name"]] += float(r["Counter_Value"])
        for i, key in enumerate(sorted(rows)):
            v = names[(i // 4) % len(names)]
            for c, x in rows[key].items():
                per[v].setdefault(c, []).append(x)
    out = {}
    for v, cs in per.items():
        m = {c: sum(x) / len(x) for c, x in cs.items()}
        rec = {"dispatches": max((len(x) for x in cs.values()), default=0), "per_dispatch": m}
        if m.get("SQ_BUSY_CU_CYCLES") and "SQ_VALU_MFMA_BUSY_CYCLES" in m:
            rec["mfma_busy_frac_of_simd_cycles"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (4 * m["SQ_BUSY_CU_CYCLES"])
        if m.get("SQ_VALU_MFMA_BUSY_CYCLES") and "SQ_VALU_MFMA_COEXEC_CYCLES" in m:
            rec["coexec_frac_of_mfma_busy"] = m["SQ_VALU_MFMA_COEXEC_CYCLES"] / m["SQ_VALU_MFMA_BUSY_CYCLES"]
        if m.get("SQ_WAVE_CYCLES"):
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if c in m:
                    rec[c.lower() + "_frac_of_wave_cycles"] = m[c] / m["SQ_WAVE_CYCLES"]
        out[v] = rec
    print(json.dumps({"kernel": kernel, "source": src, "variants": out}, indent=1))


if __name__ == "__main__":
    main()
