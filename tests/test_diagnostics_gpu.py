"""Diagnostics, NOT parity tests: the measured error envelope of the 'bf16-unsafe' mode.

Single-rounding bf16 (one bf16 rounding of every weight and activation, RDN_BF16) carries no
tolerance claim: it misses the north-star 2e-2 bar on trained RRCDNet (0.24), 1DCNN / DSDN / RRCDNet
synthetic weights (0.12 / 0.19 / 0.024).  The engine refuses plain 'bf16' and exposes
this mode only as 'bf16-unsafe'.  These tests pin the envelope so that a regression in the kernel
(not the format) is still caught; they say nothing about the 2e-2 contract.
"""
import numpy as np
import pytest
import torch

from conftest import INPUT_SETS, golden_state_dict, input_array, load_golden

pytestmark = pytest.mark.gpu

ARCHS = ["DenoiseCNN", "RRCDNet", "DSDN", "ADSDN", "PIDN", "APIDN"]
ENVELOPE = 0.3          # max-abs / max(1, max|ref|), measured worst 0.24 (trained RRCDNet)


def _cases():
    out = []
    for a in ARCHS:
        out.append((a, "synth"))
        if any(k.startswith("w::") for k in load_golden(a).files):
            out.append((a, "trained"))
    return out


@pytest.mark.parametrize("arch,which", _cases())
def test_bf16_unsafe_error_envelope(arch, which, inputs):
    import raman_mi355x as R
    g = load_golden(arch)
    m = R.MODELS[arch]()
    m.load_state_dict(golden_state_dict(arch, which), strict=True)
    m = m.cuda().eval().set_engine_dtype("bf16-unsafe")
    for name in INPUT_SETS:
        ref = g[f"{which}_{name}"]
        x = torch.from_numpy(np.ascontiguousarray(input_array(inputs, name))).unsqueeze(1).cuda()
        with torch.no_grad():
            y = m(x).squeeze(1).cpu().numpy()
        err = np.abs(y - ref).max()
        scale = max(1.0, float(np.abs(ref).max()))
        print(f"{arch}/{which}/{name}: bf16-unsafe max-abs {err:.3e} (2e-2 bar {'met' if err <= 2e-2 * scale else 'NOT met'})")
        assert np.isfinite(y).all()
        assert err <= ENVELOPE * scale, f"{arch}/{which}/{name}: {err:.3e}"
