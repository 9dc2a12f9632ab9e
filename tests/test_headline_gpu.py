"""The headline mode ('f16' = RDN_F16MIX on RRCDNet, the hybrid kernel bench.py times) pinned on its
own workload and on data its tuning never saw.

* Held-out set (tests/golden/heldout_RRCDNet.npz, make_golden.py --heldout): RRCDNet trained 2500
  Adam steps at the reference's LR from another seed and training pool than the fixtures
  tools/f16mix_select.py chose the correction mask on; inputs drawn by the reference generator with
  a fresh seed, half of them spiked (extreme_noise_prob = 1).  Bars as in test_forward_gpu.py:
  16-bit max-abs <= 2e-2 (trained weights), fp32 max-rel <= 1e-5.  The mask is NOT re-selected here.
* Many-workgroup batch independence: a spectrum computed alone equals the same spectrum inside a
  300-spectrum batch (5400 workgroups, every CU busy several times over), bitwise, and the batch is
  bitwise reproducible (the hybrid parks right-head rows in y and re-reads them, rrcdnet_hybrid.hpp).
* The bench workload itself: on-device simulator inputs at L = 10,000, batch 8192, random-init
  weights seeded as bench.py seeds them; a sample of spectra (first, middle, last workgroups)
  against the CPU oracle.
"""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

BF16_ABS = 2e-2
F32_REL = 1e-5
SEED = 20250410


def _heldout():
    g = np.load(os.path.join(GOLDEN, "heldout_RRCDNet.npz"))
    sd = {k[3:]: torch.from_numpy(np.array(g[k])) for k in g.files if k.startswith("w::")}
    return g, sd


def _model(sd, dtype):
    import raman_mi355x as R
    m = R.RRCDNet()
    m.load_state_dict(sd, strict=True)
    return m.cuda().eval().set_engine_dtype(dtype)


def _run(m, x_np):
    x = torch.from_numpy(np.ascontiguousarray(x_np)).unsqueeze(1).cuda()
    with torch.no_grad():
        y = m(x)
    torch.cuda.synchronize()
    return y.squeeze(1).cpu().numpy()


@pytest.mark.parametrize("tiles", ["0", "1"])
@pytest.mark.parametrize("dtype", ["f16", "f16f8", "bf16x3"])
def test_heldout_16bit_within_tolerance(dtype, tiles, monkeypatch):
    """'f16' (RDN_F16MIX, the shipped correction mask) on held-out trained weights and inputs, on the
    640-row hybrid (RDN_SHORT_TILES=0) and the 256-row latency tiles (=1)."""
    monkeypatch.setenv("RDN_SHORT_TILES", tiles)
    g, sd = _heldout()
    m = _model(sd, dtype)
    assert dtype != "f16" or m.engine_code == 5
    for name in ("main", "odd"):
        y = _run(m, g[f"in_{name}"])
        err = float(np.abs(y - g[f"ref_{name}"]).max())
        print(f"heldout/{name}: {dtype} (short tiles {tiles}) max-abs {err:.3e}")
        assert np.isfinite(y).all()
        assert err <= BF16_ABS, f"heldout/{name}: {dtype} max-abs {err:.3e} > {BF16_ABS}"


def test_heldout_plain_f16_is_outside_the_bar_the_mix_fixes():
    """Why the correction exists, on data the mask never saw: plain f16 (RDN_F16) is strictly worse
    than 'f16' (RDN_F16MIX) on the held-out set (reported, the bar is only asserted for 'f16')."""
    g, sd = _heldout()
    e_mix = float(np.abs(_run(_model(sd, "f16"), g["in_main"]) - g["ref_main"]).max())
    e_plain = float(np.abs(_run(_model(sd, "f16-plain"), g["in_main"]) - g["ref_main"]).max())
    print(f"heldout: f16 (mix) {e_mix:.3e}, f16-plain {e_plain:.3e}")
    assert e_mix < e_plain


def test_heldout_fp32_matches_reference():
    g, sd = _heldout()
    m = _model(sd, "fp32")
    for name in ("main", "odd"):
        ref = g[f"ref_{name}"]
        y = _run(m, g[f"in_{name}"])
        rel = float(np.abs(y - ref).max() / np.abs(ref).max())
        print(f"heldout/{name}: fp32 max-rel {rel:.2e}")
        assert rel <= F32_REL


def _sim(n, L, first=0):
    from raman_mi355x import engine
    c, x, _, _ = engine.generate(n, SEED, first_index=first, signal_length=L, device="cuda")
    return c, x.view(n, 1, L)


def test_hybrid_batch_independence_many_workgroups(monkeypatch):
    """300 simulator spectra at L = 10,000 (18 tiles each: 5400 workgroups): in-batch outputs equal
    the same spectra computed alone, bitwise, and a second run of the batch is bitwise identical."""
    from raman_mi355x import engine
    monkeypatch.setenv("RDN_SHORT_TILES", "0")      # a lone spectrum would otherwise take the 256-row tiles
    g, sd = _heldout()
    m = _model(sd, "f16")
    packed = m.packed_weights(torch.device("cuda"))
    _, x = _sim(300, 10000, first=777)
    y1 = engine.forward("RRCDNet", m.engine_code, packed, x)
    y2 = engine.forward("RRCDNet", m.engine_code, packed, x)
    torch.cuda.synchronize()
    assert torch.equal(y1, y2)
    for i in (0, 1, 149, 150, 298, 299):
        yi = engine.forward("RRCDNet", m.engine_code, packed, x[i:i + 1].clone())
        assert torch.equal(yi[0], y1[i]), i
    # the latency geometry (one spectrum, 256-row tiles) stays within the bar of the 640-row result
    monkeypatch.setenv("RDN_SHORT_TILES", "1")
    ys = engine.forward("RRCDNet", m.engine_code, packed, x[5:6].clone())
    assert float((ys[0] - y1[5]).abs().max()) <= BF16_ABS


@pytest.mark.parametrize("weights", ["random", "heldout"])
def test_bench_workload_sample_matches_oracle(weights):
    """bench.py's step: 8192 on-device simulator spectra (seed 20250410, indices 0..8191) through the
    'f16' hybrid; spectra in the first, middle and last workgroups against the CPU oracle."""
    import raman_mi355x as R
    from oracle.models import forward as oracle_forward
    from raman_mi355x import engine
    if weights == "random":
        torch.manual_seed(1234)                       # bench.py's random-init weights
        m = R.RRCDNet()
        sd = {k: v.clone() for k, v in m.state_dict().items()}
        m = m.cuda().eval().set_engine_dtype("f16")
    else:
        _, sd = _heldout()
        m = _model(sd, "f16")
    B, L = 8192, 10000
    _, x = _sim(B, L)
    y = engine.forward("RRCDNet", m.engine_code, m.packed_weights(torch.device("cuda")), x)
    torch.cuda.synchronize()
    assert bool(torch.isfinite(y).all())
    idx = [0, 1, 4095, 4096, 8190, 8191]
    xs = x[idx].cpu()
    ref = oracle_forward("RRCDNet", sd, xs).squeeze(1).numpy()
    got = y[idx].squeeze(1).cpu().numpy()
    err = float(np.abs(got - ref).max())
    tol = BF16_ABS if weights == "heldout" else BF16_ABS * max(1.0, float(np.abs(ref).max()))
    print(f"bench workload ({weights} weights): max-abs {err:.3e} over spectra {idx} (tol {tol:.2e})")
    assert err <= tol
