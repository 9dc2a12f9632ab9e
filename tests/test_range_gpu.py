"""Inputs far outside normalised intensity (VERDICT r03 "safe-range contract"): the golden inputs scaled
by 10, 100 and 1000 through every arithmetic mode.  The reference takes any float32 input
(RRCDNet/train.py:95-98), so every mode must either match or say so:

* the drop-in module always matches: the 16-bit modes are defined on normalised intensity (|x| <= 4,
  models.INPUT_GATE; every simulated spectrum lies in [-1, 2]), and a batch beyond it -- or one whose
  activations leave the e4m3 planes' range -- is re-run in fp32;
* the engine API raises RangeError for RDN_F16F8 / RDN_F16MIX once an activation leaves the e4m3
  planes' range (|v| > 1792: the trained networks reach 9-28 at scale 1, ~300 at 10, ~3,000 at 100),
  and the saturated tiles are NaN.

Judging fp32 at these scales: the networks become ill-conditioned (sigmoid heads, CBAM gating, deep
residual sums), and the reference's own fp32 forward drifts from the exact (float64) one -- APIDN at 10x
by 4e-3, ADSDN at 1000x by 39-50 of outputs ~2,500 (profiles/r05/ablate/fp32_rescomp.log).  At 1000x the
CBAM networks are chaotic: the fp32 result's distance from float64 is a draw whose size depends on the
summation order -- the same reference forward gives 39 on one host CPU and 50 on another, and fp32
forwards whose weights differ by one rounding (1 ulp) give 10-52.  So the fp32 noise floor is taken as
the largest distance from float64 of four fp32 oracle forwards: the reference weights and three 1-ulp
perturbations of them; each result is held to the exact forward with the bar
max(1e-5 x max|y64|, 2 x floor).  On the well-conditioned cases the floor is the reference's own
distance within a factor ~2.  Every forward here comes from the oracle (oracle/models.py, the functional
restatement pinned against the reference's fixtures), the float64 one on float64 weights and inputs.
"""
import warnings

import numpy as np
import pytest
import torch

from conftest import golden_state_dict

pytestmark = pytest.mark.gpu

NETS = ["DenoiseCNN", "RRCDNet", "DSDN", "PIDN", "ADSDN", "APIDN"]
SCALES = [10.0, 100.0, 1000.0]
_REFS = {}


def _perturbed(sd, seed):
    """the weights with every element moved by -1, 0 or +1 ulp of fp32 (seeded)"""
    g = torch.Generator().manual_seed(seed)
    return {k: (v * (1 + torch.randint(-1, 2, v.shape, generator=g).float() * 2.0 ** -24)).float()
            if v.is_floating_point() and v.numel() > 1 else v for k, v in sd.items()}


def _refs(arch, x):
    """(fp32 noise floor, float64 exact forward) of the trained network on x (CPU oracle; cached): the
    floor is the largest distance from float64 of the fp32 forward and of three 1-ulp perturbations."""
    from oracle import models as om
    key = (arch, x.shape, float(np.abs(x).max()), float(x.ravel()[0]))
    if key not in _REFS:
        sd = golden_state_dict(arch, "trained")
        sd64 = {k: v.double() if v.is_floating_point() else v for k, v in sd.items()}
        xt = torch.from_numpy(x).unsqueeze(1)
        with torch.no_grad():
            y64 = om.FORWARD[arch](sd64, xt.double()).squeeze(1).numpy()
            floor = max(float(np.abs(om.forward(arch, w, xt).squeeze(1).numpy() - y64).max())
                        for w in [sd] + [_perturbed(sd, s) for s in range(3)])
        _REFS[key] = (floor, y64)
    return _REFS[key]


FACTOR = 2.0      # x the fp32 noise floor (was 8 x the reference's own distance)


def _bar(floor, y64):
    return max(1e-5 * float(np.abs(y64).max()), FACTOR * floor)


def _x(inputs):
    # two spectra at L = 10,000 plus two short ones: several tiles, both edge geometries
    return inputs["main_noisy"][:2], inputs["edge1000_noisy"]


@pytest.mark.parametrize("scale", SCALES)
@pytest.mark.parametrize("dtype", ["fp32", "f16", "f16f8", "bf16x3"])
@pytest.mark.parametrize("arch", NETS)
def test_module_matches_exact_forward_on_scaled_inputs(arch, dtype, scale, inputs):
    import raman_mi355x as R
    sd = golden_state_dict(arch, "trained")
    m = R.MODELS[arch]()
    m.load_state_dict(sd, strict=True)
    m = m.cuda().eval().set_engine_dtype(dtype)
    for x in _x(inputs):
        xs = (x * scale).astype(np.float32)
        floor, y64 = _refs(arch, xs)
        m._range_warned = False                # the module warns once; re-arm it per input
        with torch.no_grad(), warnings.catch_warnings(record=True) as w:
            warnings.simplefilter("always", RuntimeWarning)
            y = m(torch.from_numpy(xs).unsqueeze(1).cuda()).squeeze(1).cpu().numpy()
        assert np.isfinite(y).all(), (arch, dtype, scale)
        if dtype != "fp32":                   # beyond the 16-bit domain: the module ran fp32
            assert any("ran in fp32" in str(r.message) for r in w), (arch, dtype, scale)
        err = float(np.abs(y - y64).max())
        assert err <= _bar(floor, y64), (arch, dtype, scale, err, _bar(floor, y64))


@pytest.mark.parametrize("dtype", ["f16f8", "f16"])
@pytest.mark.parametrize("arch", NETS)
def test_engine_reports_saturation(arch, dtype, inputs):
    """engine.forward on a range-checked mode (f16f8; 'f16' on RRCDNet = RDN_F16MIX): at every scale
    either the launch stayed in range (no error, every output finite) or rdn_forward_status reports
    RDN_ERANGE and some outputs are NaN; scale 1000 saturates every network; the sticky word clears."""
    import raman_mi355x as R
    from raman_mi355x import _lib, engine
    sd = golden_state_dict(arch, "trained")
    m = R.MODELS[arch]()
    m.load_state_dict(sd, strict=True)
    m = m.cuda().eval().set_engine_dtype(dtype)
    code = m.engine_code
    if code not in engine.RANGE_CODES:
        pytest.skip(f"{arch} '{dtype}' is RDN_F16 (f16 range, no e4m3 planes)")
    x = inputs["main_noisy"][:2]
    for scale in [1.0] + SCALES:
        xs = torch.from_numpy((x * scale).astype(np.float32)).unsqueeze(1).cuda()
        ws = engine.Workspace(arch, code, xs.shape[0], xs.shape[-1], xs.device)
        y = engine.forward(arch, code, m.packed_weights(xs.device), xs, check=False, workspace=ws)
        yy = y.squeeze(1).cpu().numpy()
        try:
            ws.check()
            saturated = False
        except _lib.RangeError as e:
            assert "1792" in str(e)
            saturated = True
        print(f"{arch} {dtype} x{scale:g}: saturated {saturated}")
        assert saturated == (not np.isfinite(yy).all()), (arch, scale)
        assert not (scale == 1.0 and saturated), arch
        assert saturated or scale < 1000, (arch, scale)
        ws.check()                                                # the sticky word was cleared


def test_module_reruns_saturated_batch_in_fp32(inputs):
    """The drop-in module never returns NaN tiles: a saturated 'f16' RRCDNet batch is re-run in fp32
    (one RuntimeWarning per module) and matches the fp32 path exactly; back in range it runs 'f16'."""
    import raman_mi355x as R
    sd = golden_state_dict("RRCDNet", "trained")
    m = R.RRCDNet()
    m.load_state_dict(sd, strict=True)
    m = m.cuda().eval().set_engine_dtype("f16")
    x = torch.from_numpy((inputs["main_noisy"][:2] * 100.0).astype(np.float32)).unsqueeze(1).cuda()
    with pytest.warns(RuntimeWarning, match="ran in fp32"):
        y = m(x)
    y32 = R.RRCDNet()
    y32.load_state_dict(sd, strict=True)
    y32 = y32.cuda().eval()(x)
    assert torch.equal(y, y32)
    y1 = m(torch.from_numpy(inputs["main_noisy"][:2]).unsqueeze(1).cuda())      # back in range: 'f16'
    assert torch.isfinite(y1).all()


@pytest.mark.parametrize("short", ["1", "0"])
@pytest.mark.parametrize("dtype", ["f16", "f16f8"])
def test_no_false_range_error_after_saturated_launch(dtype, short, inputs, monkeypatch):
    """The range guard sees only rows inside [0, L).  On an edge tile of the 256-row hybrid the rows
    beyond L + 1 are computed from LDS rows no wave keeps current (idle waves skip them), i.e. from
    whatever an earlier workgroup left there: a saturating launch (inputs x1000) first fills the LDS
    with large values, then normal spectra of ragged lengths -- edge tiles with idle waves -- must run
    without RDN_ERANGE and without NaN, in both tile geometries (RDN_SHORT_TILES)."""
    import raman_mi355x as R
    from raman_mi355x import _lib, engine
    monkeypatch.setenv("RDN_SHORT_TILES", short)
    sd = golden_state_dict("RRCDNet", "trained")
    m = R.RRCDNet()
    m.load_state_dict(sd, strict=True)
    m = m.cuda().eval().set_engine_dtype(dtype)
    code = m.engine_code
    packed = m.packed_weights(torch.device("cuda"))
    base = inputs["main_noisy"][:2]
    big = torch.from_numpy((base * 1000.0).astype(np.float32)).unsqueeze(1).cuda()
    for L in (1200, 2049, 1000, 5000, 333, 4099):
        ws_big = engine.Workspace("RRCDNet", code, big.shape[0], big.shape[-1], big.device)
        engine.forward("RRCDNet", code, packed, big, check=False, workspace=ws_big)
        with pytest.raises(_lib.RangeError):
            ws_big.check()                                       # x1000 saturates (test above)
        for B in (2, 16):
            x = torch.from_numpy(np.ascontiguousarray(np.tile(base[:, :L], (B // 2, 1)))).unsqueeze(1).cuda()
            ws = engine.Workspace("RRCDNet", code, B, L, x.device)
            y = engine.forward("RRCDNet", code, packed, x, check=False, workspace=ws)
            ws.check()                                           # no RangeError
            assert torch.isfinite(y).all(), (dtype, short, L, B)


@pytest.mark.parametrize("arch,dtype,scale", [("RRCDNet", "f16", 100.0), ("DSDN", "f16f8", 1000.0),
                                              ("ADSDN", "f16f8", 1000.0)])
def test_range_signal_survives_flush_denormal(arch, dtype, scale, inputs):
    """the module reads the status word as an integer (the kernels set bit 0 = 1u, a float
    denormal), so the host's denormals-are-zero mode (torch.set_flush_denormal(True)) cannot hide the
    range signal: a saturating batch is still re-run in fp32 and returned without NaN."""
    import raman_mi355x as R
    sd = golden_state_dict(arch, "trained")
    m = R.MODELS[arch]()
    m.load_state_dict(sd, strict=True)
    m = m.cuda().eval().set_engine_dtype(dtype)
    ref = R.MODELS[arch]()
    ref.load_state_dict(sd, strict=True)
    ref = ref.cuda().eval()
    x = torch.from_numpy((inputs["main_noisy"][:2] * scale).astype(np.float32)).unsqueeze(1).cuda()
    if not torch.set_flush_denormal(True):
        pytest.skip("this host CPU has no denormals-are-zero mode")
    try:
        with torch.no_grad(), pytest.warns(RuntimeWarning, match="ran in fp32"):
            y = m(x)
    finally:
        torch.set_flush_denormal(False)
    with torch.no_grad():
        assert torch.equal(y, ref(x))
    assert torch.isfinite(y).all()


@pytest.mark.parametrize("arch", ["ADSDN", "APIDN"])
def test_cbam_saturation_taints_whole_spectrum(arch, inputs):
    """in the CBAM team kernel (f16f8) a saturated tile's clamped statistics reach every tile
    of its spectrum through the hand-offs, so a saturated spectrum is NaN at every position -- never
    finite-but-wrong tiles beside NaN ones -- while spectra without a saturated tile stay finite and
    equal to the same launch without the saturated spectrum."""
    import raman_mi355x as R
    from raman_mi355x import _lib, engine
    sd = golden_state_dict(arch, "trained")
    m = R.MODELS[arch]()
    m.load_state_dict(sd, strict=True)
    m = m.cuda().eval().set_engine_dtype("f16f8")
    code = m.engine_code
    base = inputs["main_noisy"][:2]
    packed = m.packed_weights(torch.device("cuda"))
    for scale in (10.0, 100.0, 1000.0):
        # spectrum 0 scaled, spectrum 1 normal: one launch, separate teams
        xs = np.stack([base[0] * scale, base[1]]).astype(np.float32)
        x = torch.from_numpy(xs).unsqueeze(1).cuda()
        ws = engine.Workspace(arch, code, 2, x.shape[-1], x.device)
        y = engine.forward(arch, code, packed, x, check=False, workspace=ws).squeeze(1).cpu().numpy()
        try:
            ws.check()
            saturated = False
        except _lib.RangeError:
            saturated = True
        fin = np.isfinite(y)
        print(f"{arch} x{scale:g}: saturated {saturated}, finite fraction {fin[0].mean():.3f} / {fin[1].mean():.3f}")
        assert fin[0].all() or not fin[0].any(), (arch, scale, fin[0].mean())
        assert fin[1].all(), (arch, scale)
        assert saturated == (not fin[0].all()), (arch, scale)
    assert saturated, arch                                        # x1000 saturates (test above)
    x1 = torch.from_numpy(base[1:2].astype(np.float32)).unsqueeze(1).cuda()
    y1 = engine.forward(arch, code, packed, x1, check=True).squeeze(1).cpu().numpy()
    assert np.array_equal(y1[0], y[1]), arch


@pytest.mark.parametrize("arch,dtype", [("RRCDNet", "f16"), ("DSDN", "f16"), ("ADSDN", "f16"), ("APIDN", "f16"),
                                        ("ADSDN", "f16f8"), ("APIDN", "bf16x3")])
def test_status_ex_reports_input_gate(arch, dtype, inputs):
    """rdn_forward_status_ex (ABI v6) reports the input gate of every network -- the fused networks' status
    word and the CBAM team workspaces alike (their stems raise it): set for an input beyond [-4, 4], not
    for normalised intensity, cleared by the read; rdn_forward_status fails on neither."""
    import raman_mi355x as R
    from raman_mi355x import engine
    m = R.MODELS[arch]()
    m.load_state_dict(golden_state_dict(arch, "trained"), strict=True)
    m = m.cuda().eval().set_engine_dtype(dtype)
    code = m.engine_code
    x = inputs["main_noisy"][:2]
    for scale, want in ((1.0, 0), (5.0, engine.STATUS_GATE), (1.0, 0)):
        xs = torch.from_numpy((x * scale).astype(np.float32)).unsqueeze(1).cuda()
        ws = engine.Workspace(arch, code, xs.shape[0], xs.shape[-1], xs.device)
        engine.forward(arch, code, m.packed_weights(xs.device), xs, check=False, workspace=ws)
        flags = ws.check()
        assert flags & engine.STATUS_GATE == want, (arch, dtype, scale, flags)
        assert not flags & engine.STATUS_TIMEOUT
        assert ws.check() == 0                                   # read and cleared


@pytest.mark.parametrize("arch", ["ADSDN", "APIDN"])
def test_cbam_module_gate_without_host_pass(arch, inputs, monkeypatch):
    """The CBAM networks' batch-1 module path takes the input gate from the team workspace's status words
    (no aminmax pass over x): a spectrum beyond the gate re-runs in fp32 with one warning, one inside it
    stays 'f16' and equals the engine's 'f16' forward bit for bit."""
    import raman_mi355x as R
    from raman_mi355x import engine

    def no_aminmax(*a, **k):
        raise AssertionError("the module must not scan x on the host side")
    monkeypatch.setattr(torch, "aminmax", no_aminmax)
    m = R.MODELS[arch]()
    m.load_state_dict(golden_state_dict(arch, "trained"), strict=True)
    m = m.cuda().eval().set_engine_dtype("f16")
    x = torch.from_numpy(inputs["main_noisy"][:1].astype(np.float32)).unsqueeze(1).cuda()
    with torch.no_grad(), warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always", RuntimeWarning)
        y = m(x)
        assert not w
        ref = engine.forward(arch, m.engine_code, m.packed_weights(x.device), x)
        assert torch.equal(y, ref)
        y5 = m(x * 5.0)
        assert any("ran in fp32" in str(r.message) for r in w)
        ref5 = engine.forward(arch, 0, m._fp32_weights(x.device), x * 5.0)
        assert torch.equal(y5, ref5)


def test_walk_saturation_nans_rest_of_spectrum(monkeypatch):
    """The RDN_F16MIX walk (one workgroup per spectrum, carries across tiles): a tile whose activations
    leave the e4m3 planes' range NaNs its outputs AND every later tile of the spectrum -- the clamped
    values travel on in the carry rows, so no later tile of that spectrum may report finite outputs.
    Spectra that stay in range are untouched, the status word reports RDN_ERANGE, and the module re-runs
    the batch in fp32.  Inputs stay inside the spike window [-0.3, 1.3] (so the walk, not the tiled
    fallback, runs); the right branch's convs are scaled up so the activations grow along the spectrum."""
    import raman_mi355x as R
    from raman_mi355x import _lib, engine
    monkeypatch.setenv("RDN_WALK", "1")
    monkeypatch.setenv("RDN_SHORT_TILES", "0")
    sd = {k: v.clone() for k, v in golden_state_dict("RRCDNet", "synth").items()}
    for k in sd:
        if k.startswith("right_net.") and k.endswith(".0.weight") and sd[k].shape[1] == 64:
            sd[k] *= 1.55          # CPU fp32: spectrum 1 first exceeds 1792 at position 3113, 2 at 0
    m = R.RRCDNet()
    m.load_state_dict(sd, strict=True)
    m = m.cuda().eval().set_engine_dtype("f16")
    n, L = 4, 6000
    p = np.arange(L, dtype=np.float32) / L
    x = np.zeros((n, L), np.float32)
    x[0] = 0.05 * np.sin(p * 40)                      # small: stays in range (max |v| 548)
    x[1] = 1.25 * p                                   # ramp: saturates part-way along
    x[2] = 1.25 * p[::-1]                             # ramp down: saturates from the first tiles
    x[3] = 0.5 + 0.0 * p                              # stays in range (max |v| 1532)
    xs = torch.from_numpy(x).unsqueeze(1).cuda()
    ws = engine.Workspace("RRCDNet", m.engine_code, n, L, xs.device)
    y = engine.forward("RRCDNet", m.engine_code, m.packed_weights(xs.device), xs, check=False,
                       workspace=ws).squeeze(1).cpu().numpy()
    with pytest.raises(_lib.RangeError):
        ws.check()
    bad = np.isnan(y)
    assert bad.any(), "the scaled weights must saturate some tile"
    for i in range(n):
        if bad[i].any():
            first = int(np.argmax(bad[i]))
            assert bad[i, first:].all(), f"spectrum {i}: finite outputs after a saturated tile"
        print(f"spectrum {i}: NaN from {int(np.argmax(bad[i])) if bad[i].any() else None}")
    assert not bad[0].any() and not bad[3].any()
    first1 = int(np.argmax(bad[1]))
    assert bad[1].any() and 0 < first1 < L, first1          # a finite prefix, then NaN to the end
    assert bad[2].any()
    with torch.no_grad(), warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always", RuntimeWarning)
        ym = m(xs)
    assert torch.isfinite(ym).all() and any("ran in fp32" in str(r.message) for r in w)
