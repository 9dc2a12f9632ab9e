"""Forward throughput of every network x engine dtype on one GPU.

    python tools/throughput_table.py [--out profiles/r01/throughput.md] [--archs ...] [--dtypes ...]

Inputs come from the on-device simulator (resident in HBM before timing); weights are the
architecture's random init; one timed launch = one forward over the batch.  Algorithmic TFLOP/s
counts only the Conv1d FLOPs, against the dense MFMA peak of the dtype.
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "data-simulation-and-noise-reduction-of-distributed-fiber-raman-intensity_amd"))
sys.path.insert(0, ROOT)

from bench import PEAK_TFLOPS, flops_per_spectrum  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--archs", nargs="*", default=["DenoiseCNN", "RRCDNet", "DSDN", "ADSDN", "PIDN", "APIDN"])
    ap.add_argument("--dtypes", nargs="*", default=["f16", "f16-plain", "f16f8", "bf16x3", "bf16-unsafe", "fp32"])
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import raman_mi355x as R
    from raman_mi355x import engine
    dev = torch.device("cuda")
    rows = ["| network | L | dtype | batch | ms / launch | spectra/s | algorithmic TFLOP/s | frac of dense peak |",
            "|---|---|---|---|---|---|---|---|"]
    for arch in args.archs:
        for L in ([10000, 16384] if arch in ("PIDN", "APIDN") else [10000]):
            for dt in args.dtypes:
                B = {"f16": 4096, "f16-plain": 4096, "bf16-unsafe": 4096, "bf16x3": 2048, "f16f8": 2048, "fp32": 1024}[dt]
                if arch in ("ADSDN", "APIDN"):
                    B //= 2
                B = max(64, B * 10000 // L)
                torch.manual_seed(0)
                m = R.MODELS[arch]().to(dev).eval().set_engine_dtype(dt)
                _, noisy, _, _ = engine.generate(B, 7, signal_length=L, device=dev)
                x = noisy.view(B, 1, L)
                packed = m.packed_weights(dev)
                y = torch.empty_like(x)
                engine.forward(arch, m.engine_code, packed, x, out=y, check=False)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.reps):
                    engine.forward(arch, m.engine_code, packed, x, out=y, check=False)
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / args.reps
                sps = B / (ms * 1e-3)
                tf = flops_per_spectrum(arch, L) * sps / 1e12
                rows.append(f"| {arch} | {L} | {dt} | {B} | {ms:.2f} | {sps:,.0f} | {tf:.0f} | {tf / PEAK_TFLOPS[dt]:.3f} |")
                print(rows[-1], flush=True)
                del x, y, noisy
    text = "\n".join(rows) + "\n"
    if args.out:
        with open(args.out, "w") as fh:
            fh.write(text)


if __name__ == "__main__":
    main()
