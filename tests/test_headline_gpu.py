"""The headline mode ('f16' = RDN_F16MIX on RRCDNet, the hybrid kernel bench.py times) pinned on its
own workload and on data its tuning never saw.

* Tuning set (tests/golden/heldout_RRCDNet.npz, make_golden.py --heldout): RRCDNet trained 2,500 CPU
  Adam steps at L = 1,000; round 3 chose the corrected tail length and the spiked-tile window after
  evaluating on it (tools/f16mix_tail_eval.py), so it is a tuning set, not a held-out one.
* Held-out set (tests/golden/heldout2_RRCDNet.npz, tests/golden/train_heldout_gpu.py + make_golden.py
  --heldout2): RRCDNet trained at the reference's own recipe -- Adam 3e-4, batch 32, MSE, 200 epochs
  (28,200 steps) over 4,500 spectra at L = 10,000, best-validation checkpoint -- on a pool and with
  seeds nothing else used, created after the RDN_F16MIX design was frozen; inputs drawn by the
  reference generator with a fresh seed, half of them spiked.  Plus config 1's own 1,000 spectra
  (np.random.seed(20250410), 数据集产生.py:84) through it.
  Bars as in test_forward_gpu.py: 16-bit max-abs <= 2e-2 (trained weights), fp32 max-rel <= 1e-5.
* Many-workgroup batch independence: a spectrum computed alone equals the same spectrum inside a
  300-spectrum batch (5400 workgroups, every CU busy several times over), bitwise, and the batch is
  bitwise reproducible (the hybrid keeps each tile's right-head rows in VGPRs over the left branch,
  rrcdnet_hybrid.hpp; no tile reads another tile's outputs).
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


SETS = {"tuning": "heldout_RRCDNet.npz", "heldout2": "heldout2_RRCDNet.npz"}


def _heldout(which="tuning"):
    g = np.load(os.path.join(GOLDEN, SETS[which]))
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


@pytest.mark.parametrize("which", list(SETS))
@pytest.mark.parametrize("tiles", ["0", "1"])
@pytest.mark.parametrize("dtype", ["f16", "f16f8", "bf16x3"])
def test_heldout_16bit_within_tolerance(dtype, tiles, which, monkeypatch):
    """'f16' (RDN_F16MIX, the shipped correction mask) on held-out trained weights and inputs, on the
    640-row hybrid (RDN_SHORT_TILES=0) and the 256-row latency tiles (=1)."""
    monkeypatch.setenv("RDN_SHORT_TILES", tiles)
    g, sd = _heldout(which)
    m = _model(sd, dtype)
    assert dtype != "f16" or m.engine_code == 5
    for name in ("main", "odd"):
        y = _run(m, g[f"in_{name}"])
        err = float(np.abs(y - g[f"ref_{name}"]).max())
        print(f"{which}/{name}: {dtype} (short tiles {tiles}) max-abs {err:.3e}")
        assert np.isfinite(y).all()
        assert err <= BF16_ABS, f"{which}/{name}: {dtype} max-abs {err:.3e} > {BF16_ABS}"


@pytest.mark.parametrize("which", list(SETS))
def test_heldout_plain_f16_is_outside_the_bar_the_mix_fixes(which):
    """Why the correction exists, on data the mask never saw: plain f16 (RDN_F16) is strictly worse
    than 'f16' (RDN_F16MIX) on the held-out set (reported, the bar is only asserted for 'f16')."""
    g, sd = _heldout(which)
    e_mix = float(np.abs(_run(_model(sd, "f16"), g["in_main"]) - g["ref_main"]).max())
    e_plain = float(np.abs(_run(_model(sd, "f16-plain"), g["in_main"]) - g["ref_main"]).max())
    print(f"heldout: f16 (mix) {e_mix:.3e}, f16-plain {e_plain:.3e}")
    assert e_mix < e_plain


@pytest.mark.parametrize("which", list(SETS))
def test_heldout_fp32_matches_reference(which):
    """fp32 within 1e-5 max-relative of the exact (float64) reference forward, and of the fp32 reference
    to 1e-5 plus the fp32 reference's own distance from exact: on the 200-epoch RRCDNet (heldout2) the
    reference's fp32 CPU forward is itself 1.5e-5 from exact, so 1e-5 of IT is not a property any
    other fp32 summation order can have."""
    g, sd = _heldout(which)
    m = _model(sd, "fp32")
    for name in ("main", "odd"):
        ref, ex = g[f"ref_{name}"], g[f"f64_{name}"]
        y = _run(m, g[f"in_{name}"])
        sc = float(np.abs(ex).max())
        rel64 = float(np.abs(y - ex).max()) / sc
        rel = float(np.abs(y - ref).max()) / sc
        ref_own = float(np.abs(ref - ex).max()) / sc
        print(f"{which}/{name}: fp32 max-rel {rel:.2e} vs the fp32 reference, {rel64:.2e} vs exact "
              f"(the reference itself {ref_own:.2e} from exact)")
        assert rel64 <= F32_REL
        assert rel <= F32_REL + ref_own


@pytest.mark.xfail(reason="known miss (DESIGN.md §4): on the 200-epoch RRCDNet the reference's own fp32 CPU forward "
                          "is 1.49e-5 from exact, the engine's 8.4e-6; they differ by 1.44e-5 > 1e-5", strict=True)
def test_heldout2_fp32_plain_bar_against_fp32_reference():
    """The north-star fp32 bar exactly as written -- max-rel <= 1e-5 against the reference's fp32
    forward -- on the held-out RRCDNet.  It is NOT met there (the engine is within 1e-5 of the exact
    float64 forward, test_heldout_fp32_matches_reference, and closer to it than the reference is);
    kept as an expected failure so the measured miss stays visible in every run."""
    g, sd = _heldout("heldout2")
    m = _model(sd, "fp32")
    worst = 0.0
    for name in ("main", "odd"):
        ref = g[f"ref_{name}"]
        y = _run(m, g[f"in_{name}"])
        worst = max(worst, float(np.abs(y - ref).max()) / float(np.abs(ref).max()))
    print(f"heldout2: fp32 max-rel {worst:.2e} vs the fp32 reference (bar {F32_REL})")
    assert worst <= F32_REL


def test_heldout2_config1_thousand_spectra():
    """Config 1's own data (1,000 spectra of np.random.seed(20250410), the reference's test.npz,
    regenerated bit-exact by oracle.refgen) through the realistically trained held-out RRCDNet: 'f16'
    against the engine's fp32 path, which is within 1e-5 x max|ref| of the reference (pinned by the
    fp32 tests), so |f16 - ref| <= |f16 - fp32| + 1e-5 max|ref| <= 2e-2; the worst spectrum is also
    checked against the CPU oracle directly.  The margin is printed."""
    from oracle.models import forward as oracle_forward
    from oracle.refgen import generate_signals
    g, sd = _heldout("heldout2")
    np.random.seed(SEED)
    _, noisy, _, _ = generate_signals(1000, signal_length=10000)
    m16, m32 = _model(sd, "f16"), _model(sd, "fp32")
    worst, wi, top = 0.0, -1, 0.0
    for b0 in range(0, 1000, 250):
        xb = noisy[b0:b0 + 250].astype(np.float32)
        y16, y32 = _run(m16, xb), _run(m32, xb)
        e = np.abs(y16 - y32).max(axis=1)
        top = max(top, float(np.abs(y32).max()))
        if e.max() > worst:
            worst, wi = float(e.max()), b0 + int(e.argmax())
    slack = F32_REL * top
    print(f"heldout2 x config 1 (1000 spectra): 'f16' vs fp32 max-abs {worst:.3e} (spectrum {wi}), "
          f"bar {BF16_ABS} - {slack:.1e}: margin {BF16_ABS / (worst + slack):.2f}x")
    assert worst + slack <= BF16_ABS
    xw = noisy[wi:wi + 1].astype(np.float32)
    ref = oracle_forward("RRCDNet", sd, torch.from_numpy(xw).unsqueeze(1)).squeeze(1).numpy()
    assert float(np.abs(_run(m16, xw) - ref).max()) <= BF16_ABS


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
