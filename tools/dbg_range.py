"""Diagnostic (not part of the product): after a saturating RRCDNet 'f16' launch (inputs x1000), run
normal spectra of ragged lengths on the 256-row hybrid (RDN_SHORT_TILES=1) and report which tiles
voted saturated (their outputs are NaN) when the range word comes up."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "data-simulation-and-noise-reduction-of-distributed-fiber-raman-intensity_amd"))
os.environ.setdefault("RDN_SHORT_TILES", "1")
from conftest import golden_inputs, golden_state_dict  # noqa: E402
import raman_mi355x as R  # noqa: E402
from raman_mi355x import _lib, engine  # noqa: E402

T, H = 256 - 58, 29
sd = golden_state_dict("RRCDNet", "trained")
m = R.RRCDNet()
m.load_state_dict(sd, strict=True)
m = m.cuda().eval().set_engine_dtype(sys.argv[1] if len(sys.argv) > 1 else "f16")
code = m.engine_code
packed = m.packed_weights(torch.device("cuda"))
base = golden_inputs()["main_noisy"][:2]
big = torch.from_numpy((base * 1000.0).astype(np.float32)).unsqueeze(1).cuda()
hits = 0
for rep in range(3):
    for L in (1200, 2049, 1000, 5000, 333, 4099):
        wsb = engine.Workspace("RRCDNet", code, 2, big.shape[-1], big.device)
        engine.forward("RRCDNet", code, packed, big, check=False, workspace=wsb)
        try:
            wsb.check()
        except _lib.RangeError:
            pass
        for B in (2, 16):
            x = torch.from_numpy(np.ascontiguousarray(np.tile(base[:, :L], (B // 2, 1)))).unsqueeze(1).cuda()
            ws = engine.Workspace("RRCDNet", code, B, L, x.device)
            y = engine.forward("RRCDNet", code, packed, x, check=False, workspace=ws)
            try:
                ws.check()
            except _lib.RangeError:
                hits += 1
                yy = y.squeeze(1).cpu().numpy()
                tiles = (L + T - 1) // T
                bad = sorted({(n, int(p) // T) for n, p in zip(*np.nonzero(np.isnan(yy)))})
                print(f"rep {rep} L {L} B {B}: RDN_ERANGE; tiles/spectrum {tiles}; NaN (spectrum, tile): {bad[:12]}"
                      f"{' ...' if len(bad) > 12 else ''} ({len(bad)})", flush=True)
print("false range errors:", hits)
