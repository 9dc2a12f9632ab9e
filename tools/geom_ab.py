"""A/B of the RDN_F16 CBAM team kernel's two geometries in ONE process (diagnostic, not the product):
RDN_T16_GEOM=640 (640-row tiles, 8 waves, one workgroup per CU) against the default 320-row tiles of
4 waves (two workgroups per CU).  Interleaved rounds, on-device simulator inputs, random-init weights;
prints spectra/s per geometry and the max-abs difference of the two outputs.

    python tools/geom_ab.py [--archs ADSDN APIDN] [--rounds 4] [--reps 3]
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
    ap.add_argument("--archs", nargs="*", default=["ADSDN", "APIDN", "APIDN:16384"])
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--batch", type=int, default=2048)
    args = ap.parse_args()
    import raman_mi355x as R
    from raman_mi355x import engine
    dev = torch.device("cuda")
    for spec in args.archs:
        arch, L = (spec.split(":") + ["10000"])[:2]
        L = int(L)
        B = max(64, args.batch * 10000 // L)
        torch.manual_seed(0)
        m = R.MODELS[arch]().to(dev).eval().set_engine_dtype("f16")
        _, noisy, _, _ = engine.generate(B, 7, signal_length=L, device=dev)
        x = noisy.view(B, 1, L)
        packed = m.packed_weights(dev)
        outs, times = {}, {"640": [], "320": []}
        for r in range(args.rounds):
            for g in ("640", "320") if r % 2 == 0 else ("320", "640"):
                os.environ["RDN_T16_GEOM"] = g
                y = torch.empty_like(x)
                engine.forward(arch, m.engine_code, packed, x, out=y, check=True)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.reps):
                    engine.forward(arch, m.engine_code, packed, x, out=y, check=False)
                e1.record()
                torch.cuda.synchronize()
                times[g].append(e0.elapsed_time(e1) / args.reps)
                outs[g] = y
        os.environ.pop("RDN_T16_GEOM", None)
        d = (outs["640"] - outs["320"]).abs().max().item()
        fin = bool(torch.isfinite(outs["320"]).all())
        line = [f"{arch} L={L} B={B}"]
        for g in ("640", "320"):
            ms = min(times[g])
            sps = B / (ms * 1e-3)
            frac = flops_per_spectrum(arch, L) * sps / 1e12 / PEAK_TFLOPS["f16"]
            line.append(f"geom {g}: {ms:.2f} ms {sps:,.0f} spectra/s frac {frac:.3f} (all ms {[round(t, 2) for t in times[g]]})")
        line.append(f"max|y640 - y320| {d:.2e} finite {fin}")
        print(" | ".join(line), flush=True)


if __name__ == "__main__":
    main()
