"""Error of RDN_F16MIX on RRCDNet for a list of candidate correction sets (GPU, golden fixtures):
max-abs against the reference on every input set, trained and synthetic weights (2e-2 bar)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "data-simulation-and-noise-reduction-of-distributed-fiber-raman-intensity_amd"))
from conftest import INPUT_SETS, golden_inputs, golden_state_dict, input_array, load_golden  # noqa: E402

CANDIDATES = [[], [14], [13, 14], [12, 13, 14], [11, 12, 13, 14], [13, 14, 28], [13, 14, 27, 28],
              [12, 13, 14, 26, 27, 28], [11, 12, 13, 14, 25, 26, 27, 28], [10, 11, 12, 13, 14],
              [0, 13, 14], [0, 13, 14, 15], [0, 10, 13, 14], list(range(29))]


def main():
    from raman_mi355x import engine
    dev = torch.device("cuda")
    g = load_golden("RRCDNet")
    inp = golden_inputs()
    xs = {n: torch.from_numpy(np.ascontiguousarray(input_array(inp, n))).unsqueeze(1).to(dev) for n in INPUT_SETS}
    for layers in CANDIDATES:
        out = {}
        for w in ("trained", "synth"):
            blob = engine.pack("RRCDNet", golden_state_dict("RRCDNet", w), "f16mix", dev, corrected_layers=layers)
            e = 0.0
            for n, x in xs.items():
                y = engine.forward("RRCDNet", "f16mix", blob, x).squeeze(1).cpu().numpy()
                e = max(e, float(np.abs(y - g[f"{w}_{n}"]).max()))
            out[w] = e
        print(f"{str(layers):40s} trained max-abs {out['trained']:.3e}  synth max-abs {out['synth']:.3e}", flush=True)


if __name__ == "__main__":
    main()
