"""A/B of the walk geometry (fused16_walk.hip) against the 640-row tiles, in one process on one GPU.

Times engine.forward with RDN_WALK=0 / 1 interleaved (the knob is read per call, abi.cpp walk_tiles)
on on-device simulator spectra, and checks the two outputs are bitwise equal.

    python tools/walk_ab.py [--batch 8192] [--L 10000] [net:dtype ...]    (default DenoiseCNN:f16 RRCDNet:f16-plain)
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "data-simulation-and-noise-reduction-of-distributed-fiber-raman-intensity_amd"))


def main():
    import torch
    import raman_mi355x as R
    from raman_mi355x import engine
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--L", type=int, default=10000)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("specs", nargs="*", default=["DenoiseCNN:f16", "RRCDNet:f16-plain"])
    a = ap.parse_args()
    dev = torch.device("cuda")
    os.environ["RDN_SHORT_TILES"] = "0"
    _, noisy, _, _ = engine.generate(a.batch, 1, signal_length=a.L, device=dev)
    x = noisy.view(a.batch, 1, a.L)
    torch.manual_seed(0)
    for spec in a.specs:
        arch, dtype = spec.split(":")
        model = R.MODELS[arch]()
        packed = engine.pack(arch, model.state_dict(), dtype, dev)
        outs, times = {}, {"0": [], "1": []}
        for rnd in range(a.rounds):
            for knob in ("0", "1"):
                os.environ["RDN_WALK"] = knob
                y = engine.forward(arch, dtype, packed, x)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(3):
                    engine.forward(arch, dtype, packed, x, out=y)
                e1.record()
                torch.cuda.synchronize()
                times[knob].append(e0.elapsed_time(e1) / 3)
                if rnd == 0:
                    outs[knob] = y.clone()
        same = bool(torch.equal(outs["0"], outs["1"]))
        t0, t1 = min(times["0"]), min(times["1"])
        print(f"{arch:10s} {dtype:9s} B={a.batch} L={a.L}: tiles {t0:8.3f} ms ({a.batch / t0 * 1e3:9.0f}/s)  "
              f"walk {t1:8.3f} ms ({a.batch / t1 * 1e3:9.0f}/s)  walk/tiles {t1 / t0:.4f}  bitwise-equal {same}",
              flush=True)


if __name__ == "__main__":
    main()
