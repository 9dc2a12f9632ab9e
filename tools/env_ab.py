"""A/B of a host-side environment knob of the engine in ONE process (diagnostic, not the product):
the forward timed with VAR unset against VAR=VALUE, interleaved rounds, on-device simulator inputs,
random-init weights; prints spectra/s per arm and the max-abs difference of the two outputs.

    python tools/env_ab.py --var RDN_T16_FULL_T --value 1 [--archs ADSDN APIDN APIDN:16384] [--dtype f16]
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
    ap.add_argument("--var", required=True)
    ap.add_argument("--value", default="1")
    ap.add_argument("--dtype", default="f16")
    args = ap.parse_args()
    import raman_mi355x as R
    from raman_mi355x import engine
    dev = torch.device("cuda")
    for spec in args.archs:
        arch, L = (spec.split(":") + ["10000"])[:2]
        L = int(L)
        B = max(64, args.batch * 10000 // L)
        torch.manual_seed(0)
        m = R.MODELS[arch]().to(dev).eval().set_engine_dtype(args.dtype)
        _, noisy, _, _ = engine.generate(B, 7, signal_length=L, device=dev)
        x = noisy.view(B, 1, L)
        packed = m.packed_weights(dev)
        arms = ("default", f"{args.var}={args.value}")
        outs, times = {}, {a: [] for a in arms}
        for r in range(args.rounds):
            for g in arms if r % 2 == 0 else arms[::-1]:
                if g == "default":
                    os.environ.pop(args.var, None)
                else:
                    os.environ[args.var] = args.value
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
        os.environ.pop(args.var, None)
        d = (outs[arms[0]] - outs[arms[1]]).abs().max().item()
        fin = bool(torch.isfinite(outs[arms[0]]).all() and torch.isfinite(outs[arms[1]]).all())
        line = [f"{arch} L={L} B={B}"]
        for g in arms:
            ms = min(times[g])
            sps = B / (ms * 1e-3)
            frac = flops_per_spectrum(arch, L) * sps / 1e12 / PEAK_TFLOPS["f16"]
            line.append(f"{g}: {ms:.2f} ms {sps:,.0f} spectra/s frac {frac:.3f} (all ms {[round(t, 2) for t in times[g]]})")
        line.append(f"max|y_a - y_b| {d:.2e} finite {fin}")
        print(" | ".join(line), flush=True)


if __name__ == "__main__":
    main()
