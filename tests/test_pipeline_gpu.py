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
