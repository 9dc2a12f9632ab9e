"""Calibrate RDN_F16MIX: which big layers keep the e4m3 correction (GPU, golden fixtures only).

    python tools/f16mix_select.py [--arch RRCDNet] [--steps 12]

Greedy on the GPU: start from plain f16 on every layer; at each step add the layer whose correction
lowers the worst error most, where the error is the max over the trained and synthetic weight sets
and all six golden input sets of max|y - ref| / max(1, max|ref|) (the north-star 2e-2 bf16 bar,
normalised like tests/test_forward_gpu.py).  Each step's mask is also timed (RRCDNet, L = 10,000).
The chosen default goes into csrc/pack.cpp f16mix_default_mask.
"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "data-simulation-and-noise-reduction-of-distributed-fiber-raman-intensity_amd"))
sys.path.insert(0, ROOT)

from conftest import INPUT_SETS, golden_inputs, golden_state_dict, input_array, load_golden  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="RRCDNet")
    ap.add_argument("--steps", type=int, default=12)
    ap.add_argument("--batch", type=int, default=2048)
    args = ap.parse_args()
    from raman_mi355x import engine
    dev = torch.device("cuda")
    g = load_golden(args.arch)
    inp = golden_inputs()
    whichs = ["synth"] + (["trained"] if any(k.startswith("w::") for k in g.files) else [])
    sds = {w: golden_state_dict(args.arch, w) for w in whichs}
    xs = {n: torch.from_numpy(np.ascontiguousarray(input_array(inp, n))).unsqueeze(1).to(dev) for n in INPUT_SETS}
    n_layers = {"DenoiseCNN": 18, "RRCDNet": 29, "DSDN": 32, "PIDN": 30}[args.arch]

    def error(layers):
        worst = {}
        for w in whichs:
            blob = engine.pack(args.arch, sds[w], "f16mix", dev, corrected_layers=layers)
            e = 0.0
            for n, x in xs.items():
                y = engine.forward(args.arch, "f16mix", blob, x).squeeze(1).cpu().numpy()
                ref = g[f"{w}_{n}"]
                e = max(e, float(np.abs(y - ref).max()) / max(1.0, float(np.abs(ref).max())))
            worst[w] = e
        return max(worst.values()), worst

    _, noisy, _, _ = engine.generate(args.batch, 1, signal_length=10000, device=dev)
    xb = noisy.view(args.batch, 1, 10000)
    yb = torch.empty_like(xb)

    def timing(layers):
        blob = engine.pack(args.arch, sds[whichs[-1]], "f16mix", dev, corrected_layers=layers)
        for _ in range(2):
            engine.forward(args.arch, "f16mix", blob, xb, out=yb, check=False)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            engine.forward(args.arch, "f16mix", blob, xb, out=yb, check=False)
        e1.record()
        torch.cuda.synchronize()
        return args.batch / (e0.elapsed_time(e1) / 3 * 1e-3)

    chosen = []
    e, per = error(chosen)
    print(f"step 0: mask {chosen} worst {e:.3e} {per} {timing(chosen):.0f} spectra/s", flush=True)
    for step in range(1, args.steps + 1):
        best = None
        for k in range(n_layers):
            if k in chosen:
                continue
            ek, _ = error(chosen + [k])
            if best is None or ek < best[1]:
                best = (k, ek)
        chosen.append(best[0])
        e, per = error(chosen)
        mask = sum(1 << k for k in chosen)
        print(f"step {step}: add {best[0]:2d} -> {sorted(chosen)} mask 0x{mask:x} worst {e:.3e} "
              f"{ {k: f'{v:.2e}' for k, v in per.items()} } {timing(chosen):.0f} spectra/s", flush=True)
    full = list(range(n_layers))
    e, per = error(full)
    print(f"all corrected (= f16f8): worst {e:.3e} {timing(full):.0f} spectra/s", flush=True)


if __name__ == "__main__":
    main()
