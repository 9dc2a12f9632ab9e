"""Where the 'f16' (RDN_F16MIX) error of config 1's data comes from, and what a per-tile fallback
to f16f8 would leave (diagnostic, not part of the product).

    python tools/f16mix_spike_eval.py            # GPU box

Runs RRCDNet 'f16' (640-row hybrid tiles) and 'f16f8' over the 1000 spectra of data/test.npz
(oracle.refgen, seed 20250410) with the trained fixture weights and the held-out weights, and
composes per 640-row tile (T = 582 outputs, 29-row halo): the f16f8 output where the tile's input
window leaves [lo, hi], the hybrid output elsewhere.  Prints the max-abs error against the fp32 CPU
reference for several windows, and the fraction of tiles that would take the f16f8 path.
"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "data-simulation-and-noise-reduction-of-distributed-fiber-raman-intensity_amd"))
sys.path.insert(0, ROOT)

T, H = 582, 29


def main():
    import raman_mi355x as R
    from conftest import GOLDEN, golden_state_dict
    from oracle.models import forward as oracle_forward
    from oracle.refgen import generate_signals
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    np.random.seed(20250410)
    clean, noisy, _, _ = generate_signals(1000)
    X = torch.tensor(noisy, dtype=torch.float32)
    x = X.numpy()
    L = x.shape[1]
    tiles = (L + T - 1) // T
    h = np.load(os.path.join(GOLDEN, "heldout_RRCDNet.npz"))
    weights = {"fixture": golden_state_dict("RRCDNet", "trained"),
               "heldout": {k[3:]: torch.from_numpy(np.array(h[k])) for k in h.files if k.startswith("w::")}}
    os.environ["RDN_SHORT_TILES"] = "0"
    # per tile window extremes of the input
    wmax = np.zeros((1000, tiles))
    wmin = np.zeros((1000, tiles))
    for t in range(tiles):
        a, b = max(0, t * T - H), min(L, t * T - H + 640)
        wmax[:, t] = x[:, a:b].max(axis=1)
        wmin[:, t] = x[:, a:b].min(axis=1)
    for wn, sd in weights.items():
        t0 = time.time()
        ref = torch.cat([oracle_forward("RRCDNet", sd, X[i:i + 50].unsqueeze(1)) for i in range(0, 1000, 50)]).squeeze(1).numpy()
        outs = {}
        for dt in ("f16", "f16f8"):
            m = R.RRCDNet()
            m.load_state_dict(sd)
            m = m.cuda().eval().set_engine_dtype(dt)
            with torch.no_grad():
                outs[dt] = torch.cat([m(X[i:i + 250].unsqueeze(1).cuda()).cpu() for i in range(0, 1000, 250)]).squeeze(1).numpy()
        e16 = np.abs(outs["f16"] - ref)
        e8 = np.abs(outs["f16f8"] - ref)
        print(f"{wn}: oracle {time.time() - t0:.0f} s; f16 max {e16.max():.4e}, f16f8 max {e8.max():.4e}", flush=True)
        for hi, lo in ((9e9, -9e9), (1.6, -0.6), (1.5, -0.5), (1.4, -0.4), (1.35, -0.35), (1.3, -0.3), (1.25, -0.25)):
            fall = (wmax > hi) | (wmin < lo)
            comp = e16.copy()
            for t in range(tiles):
                a, b = t * T, min(L, (t + 1) * T)
                sel = fall[:, t]
                comp[sel, a:b] = e8[sel, a:b]
            per = comp.max(axis=1)
            i = int(per.argmax())
            print(f"  window [{lo:+.2f}, {hi:.2f}]: fallback tiles {fall.mean() * 100:.2f} %, max-abs {per.max():.4e} "
                  f"(spectrum {i}), p99 {np.quantile(per, 0.99):.3e}, >1.8e-2 {int((per > 1.8e-2).sum())}", flush=True)


if __name__ == "__main__":
    main()
