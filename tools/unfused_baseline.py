"""Unfused baseline: the reference RRCDNet forward as PyTorch-ROCm eager executes it on MI355X.

SURVEY.md §8(d) / BASELINE.json north_star: the fused engine's choices are evidenced against the
unfused per-layer path (one MIOpen Conv1d kernel per layer, separate BatchNorm and ReLU kernels,
every 64 x L activation written to and re-read from HBM).  This runs exactly the reference module
structure (RRCDNet/train.py:77-98: ``x - (right_net(x) + left_net(x)) / 2``) through the engine's
drop-in class, whose submodules are plain ``nn.Conv1d``/``nn.BatchNorm1d``/``nn.ReLU`` with the
reference state_dict layout, bypassing the engine's ``forward``.

    python tools/unfused_baseline.py [--batch 256] [--steps 5] [--dtype fp32|bf16] [--out f.json]

Prints one JSON line: spectra/s, kernel launches per forward, the minimum per-layer HBM bytes of
an unfused path ((Cin+Cout)*L*s per conv layer) and the achieved GB/s at that
minimum.  Run it under ``rocprofv3 --pmc FETCH_SIZE`` / ``--pmc WRITE_SIZE`` (separate passes) for
the measured bytes (tools/summarize_profiles.py --unfused).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "data-simulation-and-noise-reduction-of-distributed-fiber-raman-intensity_amd"))

import torch  # noqa: E402

import raman_mi355x as R  # noqa: E402

L = 10000
BIG, STEMS, HEADS = 29, 2, 2          # RRCDNet conv layers
FLOPS = (BIG * 2 * 64 * 64 * 3 + (STEMS + HEADS) * 2 * 64 * 3) * L


def min_unfused_bytes(s):
    """(Cin+Cout)*L*s per conv layer, BN and ReLU fused into it (the best an unfused path can do)."""
    return (BIG * 128 + STEMS * 65 + HEADS * 65) * L * s


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    assert torch.cuda.is_available(), "needs a HIP device"
    dt = torch.float32 if a.dtype == "fp32" else torch.bfloat16
    torch.manual_seed(0)
    m = R.RRCDNet()
    for mod in m.modules():          # non-trivial BN statistics (eval mode uses them)
        if isinstance(mod, torch.nn.BatchNorm1d):
            mod.running_mean.uniform_(-0.5, 0.5)
            mod.running_var.uniform_(0.5, 2.0)
    m = m.to("cuda", dt).eval()
    x = torch.rand(a.batch, 1, L, device="cuda", dtype=dt)

    def fwd(v):                      # RRCDNet/train.py:92-98, eager
        return v - (m.right_net(v) + m.left_net(v)) / 2

    with torch.no_grad():
        for _ in range(a.warmup):
            fwd(x)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            y = fwd(x)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
    s = 4 if a.dtype == "fp32" else 2
    sps = a.batch * a.steps / el
    rec = {"what": "unfused PyTorch-ROCm eager RRCDNet (MIOpen conv + BN + ReLU kernels per layer)",
           "dtype": a.dtype, "batch": a.batch, "steps": a.steps, "signal_length": L,
           "spectra_per_s": sps, "ms_per_forward": el / a.steps * 1e3,
           "algorithmic_tflops": sps * FLOPS / 1e12,
           "min_unfused_bytes_per_spectrum": min_unfused_bytes(s),
           "gbps_at_min_bytes": sps * min_unfused_bytes(s) / 1e9,
           "out_finite": bool(torch.isfinite(y).all().item()),
           "torch": torch.__version__}
    line = json.dumps(rec)
    print(line)
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(line + "\n")


if __name__ == "__main__":
    main()
