"""The on-device evaluation pipeline bench.py times beside the headline:
simulate -> fused forward -> fp64 metric sums, chunk by chunk into reused buffers, no host sync.

Checks that chunking is invisible: the chunked run's spectra, outputs and exact metric accumulators
equal one whole-batch run bit for bit (simulator keyed on the global spectrum index, forward
independent of batch neighbours, integer accumulation), and that the pipeline's outputs and metrics
match the CPU oracle on the same simulated inputs (oracle forward fp32 1e-5 relative; 'f16' -- the
headline RDN_F16MIX -- and f16f8 2e-2 abs; metrics oracle 1e-10).
"""
import numpy as np
import pytest
import torch

from conftest import golden_state_dict

pytestmark = pytest.mark.gpu

SEED = 20250410


def _pipeline(model, arch, dtype, n, chunk, L, first=0):
    from raman_mi355x import engine
    dev = torch.device("cuda")
    packed = model.packed_weights(dev)
    clean = torch.empty((chunk, L), dtype=torch.float32, device=dev)
    noisy = torch.empty((chunk, L), dtype=torch.float32, device=dev)
    y = torch.empty((chunk, 1, L), dtype=torch.float32, device=dev)
    sums = torch.zeros(5, dtype=torch.float64, device=dev)
    acc = engine.new_acc(dev)
    xs, ys = [], []
    for i0 in range(0, n, chunk):
        engine.generate(chunk, SEED, first_index=first + i0, signal_length=L, device=dev, out=(clean, noisy))
        engine.forward(arch, model.engine_code, packed, noisy.view(chunk, 1, L), out=y)
        engine.metrics(y.view(chunk, L), clean, sums=sums, per_spectrum=False, acc=acc)
        xs.append(noisy.cpu().numpy().copy())
        ys.append(y.view(chunk, L).cpu().numpy().copy())
    torch.cuda.synchronize()
    return np.concatenate(xs), np.concatenate(ys), sums.cpu().numpy(), acc.cpu().numpy()


def _model(arch, dtype):
    import raman_mi355x as R
    m = R.MODELS[arch]()
    m.load_state_dict(golden_state_dict(arch, "trained" if arch == "RRCDNet" else "synth"), strict=True)
    return m.cuda().eval().set_engine_dtype(dtype)


@pytest.mark.parametrize("dtype", ["fp32", "f16", "f16f8"])
@pytest.mark.parametrize("arch", ["RRCDNet", "ADSDN"])
def test_chunked_pipeline_equals_whole_batch(arch, dtype, monkeypatch):
    monkeypatch.setenv("RDN_SHORT_TILES", "0")        # the same tile geometry at both chunk sizes
    m = _model(arch, dtype)
    xc, yc, sc, ac = _pipeline(m, arch, dtype, n=6, chunk=2, L=1500)
    xw, yw, sw, aw = _pipeline(m, arch, dtype, n=6, chunk=6, L=1500)
    assert np.array_equal(xc, xw)
    assert np.array_equal(yc, yw)
    assert sc[4] == sw[4] == 6
    np.testing.assert_allclose(sc[:4], sw[:4], rtol=1e-12)
    assert np.array_equal(ac, aw)                      # exact accumulators: the same bits


@pytest.mark.parametrize("dtype", ["fp32", "f16", "f16f8"])
def test_pipeline_matches_oracle(dtype):
    from oracle.metrics import per_spectrum
    from oracle.models import forward as oracle_forward
    from raman_mi355x import engine
    arch, L = "RRCDNet", 2000
    m = _model(arch, dtype)
    x, y, sums, acc = _pipeline(m, arch, dtype, n=4, chunk=2, L=L, first=1000)
    ref = oracle_forward(arch, golden_state_dict(arch, "trained"), torch.from_numpy(x).unsqueeze(1)).squeeze(1).numpy()
    scale = max(np.abs(ref).max(), 1e-30)
    err = np.abs(y - ref).max()
    tol = 1e-5 * scale if dtype == "fp32" else 2e-2          # trained weights: the plain 2e-2 max-abs bar
    assert err <= tol, f"{dtype}: {err:.3e} > {tol:.3e}"
    # metric sums of the pipeline vs the oracle's metrics on the pipeline's own outputs
    clean, _, _, _ = engine.generate(4, SEED, first_index=1000, signal_length=L, device="cuda")
    ref_sums = per_spectrum(y, clean.cpu().numpy()).sum(axis=0)
    np.testing.assert_allclose(sums[:4], ref_sums, rtol=1e-10, atol=1e-12)
    assert sums[4] == 4
    exact = engine.acc_value(torch.from_numpy(acc)).numpy()
    np.testing.assert_allclose(exact[:4], ref_sums, rtol=1e-10, atol=1e-12)
    assert exact[4] == 4


def test_metrics_clean_f64_and_exact_sums():
    """rdn_metrics_ex reads a float64 clean reference as the reference's metrics do (evaulate.py:34-35)
    and its exact accumulator equals the exactly summed per-spectrum values rounded once."""
    from fractions import Fraction
    from oracle.metrics import per_spectrum
    from raman_mi355x import engine
    rng = np.random.default_rng(3)
    c64 = rng.uniform(0, 1, (9, 777))
    y = (c64 + rng.normal(0, 0.05, c64.shape)).astype(np.float32)
    yd = torch.from_numpy(y).cuda()
    acc = engine.new_acc("cuda")
    per, _ = engine.metrics(yd, torch.from_numpy(c64).cuda(), acc=acc)
    ref = per_spectrum(y, c64)
    np.testing.assert_allclose(per.cpu().numpy(), ref, rtol=1e-10, atol=1e-13)
    per32, _ = engine.metrics(yd, torch.from_numpy(c64.astype(np.float32)).cuda())
    assert not np.array_equal(per.cpu().numpy(), per32.cpu().numpy())        # the fp64 clean was used
    got = engine.acc_value(acc).numpy()
    p = per.cpu().numpy()
    for k in range(4):
        exact = sum((abs(Fraction(float(v))) * 2 ** 128).__floor__() * (1 if v >= 0 else -1) for v in p[:, k])
        assert got[k] == float(Fraction(exact, 2 ** 128)), k
    assert got[4] == 9


@pytest.mark.parametrize("walk", ["1", "0"])
@pytest.mark.parametrize("arch,dtype", [("RRCDNet", "f16"), ("RRCDNet", "f16-plain"), ("DenoiseCNN", "f16"),
                                        ("PIDN", "f16"), ("DSDN", "f16"), ("ADSDN", "f16"), ("RRCDNet", "fp32")])
def test_forward_metrics_equals_forward_then_metrics(arch, dtype, walk, monkeypatch):
    """rdn_forward_metrics (the metric epilogue, */evaulate.py:25-39): on the walk geometry (RDN_WALK=1,
    the f16 modes of the walk networks) the forward kernel meters each spectrum itself; elsewhere the
    metrics kernel follows the forward.  Either way y and every spectrum's four values are the bits of
    rdn_forward followed by rdn_metrics_ex (one shared fp64 routine), for fp32 and fp64 clean, and the
    exact accumulators are equal."""
    from raman_mi355x import engine
    monkeypatch.setenv("RDN_WALK", walk)
    monkeypatch.setenv("RDN_SHORT_TILES", "0")
    m = _model(arch, dtype)
    dev = torch.device("cuda")
    packed = m.packed_weights(dev)
    n, L = 5, 2345
    clean, noisy, _, _ = engine.generate(n, SEED, first_index=777, signal_length=L, device=dev)
    x = noisy.view(n, 1, L)
    walks = walk == "1" and arch in ("RRCDNet", "DenoiseCNN", "PIDN", "DSDN") and dtype != "fp32"
    for c in (clean, clean.double()):
        y0 = engine.forward(arch, m.engine_code, packed, x)
        acc0 = engine.new_acc(dev)
        per0, sums0 = engine.metrics(y0.view(n, L), c, acc=acc0)
        acc1 = engine.new_acc(dev)
        y1, per1, sums1, fused = engine.forward_metrics(arch, m.engine_code, packed, x, c, per_spectrum=True, acc=acc1)
        assert fused == walks
        assert torch.equal(y0, y1)
        assert torch.equal(per0, per1)
        assert torch.equal(acc0, acc1)
        np.testing.assert_allclose(sums1.cpu().numpy(), sums0.cpu().numpy(), rtol=1e-14)
        assert sums1[4].item() == n


def test_forward_metrics_spiked_spectra_take_the_epilogue(monkeypatch):
    """The RDN_F16MIX walk's spiked spectra (the tiled hybrid, tile by tile, inside the walk kernel) are
    metered by the same epilogue: a batch of spiked and clean spectra meters all of them, and the values
    equal the standalone metrics kernel's."""
    from raman_mi355x import engine
    monkeypatch.setenv("RDN_WALK", "1")
    monkeypatch.setenv("RDN_SHORT_TILES", "0")
    m = _model("RRCDNet", "f16")
    dev = torch.device("cuda")
    n, L = 6, 3000
    clean, noisy, _, _ = engine.generate(n, SEED, first_index=4242, signal_length=L, device=dev)
    noisy[1, 100:140] += 1.0                     # spikes: outside [-0.3, 1.3]
    noisy[4, 2900:2950] -= 0.9
    x = noisy.view(n, 1, L)
    y0 = engine.forward("RRCDNet", m.engine_code, m.packed_weights(dev), x)
    per0, _ = engine.metrics(y0.view(n, L), clean)
    y1, per1, sums1, fused = engine.forward_metrics("RRCDNet", m.engine_code, m.packed_weights(dev), x, clean,
                                                    per_spectrum=True)
    assert fused
    assert torch.equal(y0, y1)
    assert torch.equal(per0, per1)
    assert sums1[4].item() == n


@pytest.mark.parametrize("arch", ["RRCDNet", "DSDN", "ADSDN"])
def test_evaluate_synthetic_fused_metering_same_bits(arch, monkeypatch):
    """Config 4's driver (evaluate_synthetic) metering through the walk kernels' epilogue
    (rdn_forward_metrics) and through forward + the metrics kernel: the same exact accumulators (the
    per-spectrum values are the same bits, metrics.hpp), on ragged chunks (20 spectra in chunks of 8);
    RDN_WALK=1 forces the walk geometry where it exists (ADSDN: the team kernel, never fused)."""
    from raman_mi355x.evaluate import evaluate_synthetic
    monkeypatch.setenv("RDN_WALK", "1")
    m = _model(arch, "f16")
    kw = dict(seed=SEED, signal_length=1500, batch_size=8, first_index=123)
    fused = evaluate_synthetic({arch: m}, 20, fused_metrics=True, **kw)[arch]
    plain = evaluate_synthetic({arch: m}, 20, fused_metrics=False, **kw)[arch]
    assert fused["acc"] == plain["acc"] and fused["acc"][-1] == 20
    assert fused["means"] == plain["means"]
