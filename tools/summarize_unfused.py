"""Summarise the unfused-baseline runs of scripts/gpu_round.sh into profiles/<round>/unfused_baseline.json.

    python tools/summarize_unfused.py gpurun_out/unf profiles/r01

HBM bytes per spectrum of the PyTorch-ROCm eager RRCDNet forward = sum over every dispatch of the
PMC pass (rocprofv3 --pmc FETCH_SIZE, --pmc WRITE_SIZE, separate passes) that belong to the last
of 4 forwards of 64 spectra (tools/unfused_baseline.py --warmup 2 --steps 2) / 64.  FETCH_SIZE is reported raw and doubled
(the gfx950 correction of MI355X_MICROARCH.md §HBM holds for 16-B/lane streaming reads; MIOpen's
access widths are uncalibrated, so the true figure lies between the two).
"""
import csv
import glob
import json
import os
import sys

BATCH = 64
MIN_K = 120


def total_kib(d, counter):
    """KiB of `counter` summed over the dispatches of ONE steady-state forward: the run's last
    forwards are identical, so the forward is the shortest period K >= MIN_K of the dispatch-name
    sequence ending at e (names[e-K:e] == names[e-2K:e-K]), e scanned back over the trailing
    non-forward dispatches (earlier dispatches include MIOpen's find-mode benchmarking)."""
    per = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if r["Counter_Name"] == counter and "rocclr" not in r["Kernel_Name"]:
                    i = int(r["Dispatch_Id"])
                    name, v = per.get(i, (r["Kernel_Name"], 0.0))
                    per[i] = (name, v + float(r["Counter_Value"]))
    seq = [per[i] for i in sorted(per)]
    names = [n for n, _ in seq]
    # the run ends with a few non-forward dispatches (isfinite check); a forward is > MIN_K
    # dispatches, longer than the 7-dispatch-per-layer period inside one conv stack
    for e in range(len(seq), len(seq) - 40, -1):
        for k in range(MIN_K, e // 2 + 1):
            if names[e - k:e] == names[e - 2 * k:e - k]:
                return sum(v for _, v in seq[e - k:e]), k
    raise RuntimeError(f"{d}: no repeated forward at the end of the dispatch sequence")


def main():
    src, dst = sys.argv[1], sys.argv[2]
    out = {}
    for dt in ("fp32", "bf16"):
        try:
            with open(os.path.join(src, f"unfused_{dt}.json")) as fh:
                rec = json.load(fh)
        except OSError:
            continue
        fk, nd = total_kib(os.path.join(src, f"pmc_{dt}_FETCH_SIZE"), "FETCH_SIZE")
        wk, _ = total_kib(os.path.join(src, f"pmc_{dt}_WRITE_SIZE"), "WRITE_SIZE")
        lo = (fk + wk) * 1024 / BATCH
        hi = (2 * fk + wk) * 1024 / BATCH
        rec.update({"pmc_dispatches_per_forward": nd,
                    "hbm_bytes_per_spectrum_raw": lo, "hbm_bytes_per_spectrum_fetch_x2": hi,
                    "hbm_gbps_raw": lo * rec["spectra_per_s"] / 1e9,
                    "hbm_gbps_fetch_x2": hi * rec["spectra_per_s"] / 1e9,
                    "pmc_source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE over all dispatches of "
                                  f"tools/unfused_baseline.py --dtype {dt} --steps 2 --warmup 2 --batch 64 (last forward)"})
        out[dt] = rec
    os.makedirs(dst, exist_ok=True)
    with open(os.path.join(dst, "unfused_baseline.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    for dt, r in out.items():
        print(f"{dt}: {r['spectra_per_s']:.0f} spectra/s, {r['pmc_dispatches_per_forward']:.0f} dispatches/forward, "
              f"{r['hbm_bytes_per_spectrum_raw']/1e6:.1f}-{r['hbm_bytes_per_spectrum_fetch_x2']/1e6:.1f} MB/spectrum, "
              f"{r['hbm_gbps_raw']:.0f}-{r['hbm_gbps_fetch_x2']:.0f} GB/s")


if __name__ == "__main__":
    main()
