"""The reference evaluation flow (*/evaulate.py:25-39, :60-80) end to end on the engine: a reference-format
``test.npz`` (regenerated bit-exact by oracle.refgen, written by raman_mi355x.dataset), the batched
device ``evaluate`` and the reference's batch-1 loop through the drop-in module, against the CPU
oracle (the reference's ops) and the skimage 0.18.3 goldens; ``write_metrics`` in %.6f."""
import os
import re

import numpy as np
import pytest
import torch

from conftest import GOLDEN, golden_state_dict, load_golden

pytestmark = pytest.mark.gpu


def _dataset(tmp_path, n, L):
    from oracle.refgen import generate_signals
    from raman_mi355x.dataset import load_dataset, save_dataset
    np.random.seed(20250410)                        # SURVEY.md §8d config 1 seed
    c, x, s, sd = generate_signals(n, signal_length=L)
    path = tmp_path / "test.npz"
    save_dataset(path, c, x, s, sd)
    return load_dataset(path)


def _module(arch, which, dtype, tmp_path):
    import raman_mi355x as R
    path = tmp_path / f"{arch}_best.pth"
    torch.save(golden_state_dict(arch, which), path)           # what */train.py:200 writes
    m = R.MODELS[arch]().cuda()
    m.load_state_dict(torch.load(path, map_location="cuda", weights_only=True))   # */evaulate.py:65-66
    return m.eval().set_engine_dtype(dtype)


@pytest.mark.parametrize("arch,dtype", [("DenoiseCNN", "fp32"), ("RRCDNet", "fp32"), ("RRCDNet", "f16")])
def test_evaluate_flow_matches_reference_cpu_path(arch, dtype, tmp_path, monkeypatch):
    from oracle.metrics import per_spectrum
    from oracle.models import forward as oracle_forward
    from raman_mi355x.evaluate import evaluate, write_metrics
    d = _dataset(tmp_path, 24, 10000)
    noisy, clean = d["noisy_signals"], d["clean_signals"]
    assert noisy.dtype == np.float64 and d["snrs"].shape == (24, 1)
    m = _module(arch, "trained", dtype, tmp_path)

    # the reference's loop shape (evaulate.py:29-37): one spectrum per forward through the module
    def batch1_loop():
        out = []
        with torch.no_grad():
            for xs in noisy:
                t = torch.tensor(xs, dtype=torch.float32).unsqueeze(0).unsqueeze(0).cuda()
                out.append(m(t).cpu().squeeze().numpy())
        return np.stack(out)
    # the reference CPU path: fp32 forward of the reference ops + the reference metric functions
    sd = golden_state_dict(arch, "trained")
    y_ref = oracle_forward(arch, sd, torch.tensor(noisy, dtype=torch.float32).unsqueeze(1)).squeeze(1).numpy()
    scale = np.abs(y_ref).max()
    tol = 1e-5 * scale if dtype == "fp32" else 2e-2
    # batch 1 picks the 256-row latency tiles for RDN_F16 / RDN_F16MIX (abi.cpp short_tiles), whose
    # RDN_F16MIX rounds differently from the 640-row hybrid: within the bar, not bitwise equal
    assert np.abs(batch1_loop() - y_ref).max() <= tol
    # one geometry for the bitwise comparison of the batched device metrics below
    monkeypatch.setenv("RDN_SHORT_TILES", "0")
    got = evaluate(m, noisy, clean, batch_size=10)              # batched, ragged last batch
    y1 = batch1_loop()
    assert np.abs(y1 - y_ref).max() <= tol
    ref = per_spectrum(y_ref, clean).mean(axis=0)
    mine = per_spectrum(y1, clean).mean(axis=0)
    keys = ("MSE", "SSIM", "Smoothness", "Peak2Peak")
    rtol = 1e-4 if dtype == "fp32" else 5e-2
    for i, k in enumerate(keys):
        # batched device metrics vs host metrics of the batch-1 outputs: same outputs, fp64 both
        assert abs(got[k] - mine[i]) <= 1e-11 * max(1.0, abs(mine[i])), (k, got[k], mine[i])
        assert abs(got[k] - ref[i]) <= rtol * abs(ref[i]), (k, got[k], ref[i])
    out = write_metrics(got, root=str(tmp_path / "eval_results"))
    text = open(os.path.join(out, "metrics.txt")).read().splitlines()
    assert [ln.split(":")[0] for ln in text] == list(keys)
    for ln, k in zip(text, keys):
        assert re.fullmatch(rf"{k}: -?\d+\.\d{{6}}", ln) and ln == f"{k}: {got[k]:.6f}"


def test_evaluate_matches_skimage_golden(tmp_path, inputs):
    """Trained RRCDNet (fp32 engine) on the golden main inputs: the evaluate means equal the means of
    the reference metric functions + skimage 0.18.3 on the reference's own outputs (metrics.npz rows
    0-2), to the fp32 forward's difference."""
    from raman_mi355x.evaluate import evaluate
    g = np.load(os.path.join(GOLDEN, "metrics.npz"))
    m = _module("RRCDNet", "trained", "fp32", tmp_path)
    got = evaluate(m, inputs["main_noisy"], inputs["main_clean64"])
    ref = g["per_spectrum"][:3].mean(axis=0)
    for i, k in enumerate(("MSE", "SSIM", "Smoothness", "Peak2Peak")):
        assert abs(got[k] - ref[i]) <= 1e-5 * abs(ref[i]), (k, got[k], ref[i])


def test_evaluate_accepts_any_module(tmp_path, inputs):
    """evaluate() takes any nn.Module as evaulate.py:25-39 does: a plain PyTorch module (here the engine
    module's eager forward wrapped in another module) runs model(x) per batch; the device metrics then
    agree with the engine module's own evaluation to the fp32 forward's difference."""
    from raman_mi355x.evaluate import evaluate
    m = _module("RRCDNet", "trained", "fp32", tmp_path)

    class Plain(torch.nn.Module):
        def __init__(self, inner):
            super().__init__()
            self.inner = inner

        def forward(self, x):
            return self.inner.eager_forward(x)

    a = evaluate(Plain(m), inputs["main_noisy"], inputs["main_clean64"], batch_size=2)
    b = evaluate(m, inputs["main_noisy"], inputs["main_clean64"], batch_size=2)
    for k in a:
        assert abs(a[k] - b[k]) <= 1e-5 * abs(b[k]), (k, a[k], b[k])


def test_workspace_is_bound_to_its_stream():
    """A CBAM Workspace made on one stream is refused on another (its check() waits for its own stream)."""
    import raman_mi355x as R
    from raman_mi355x import engine
    m = R.ADSDN().cuda().eval().set_engine_dtype("f16")
    x = torch.rand(2, 1, 700, device="cuda")
    ws = engine.Workspace("ADSDN", m.engine_code, 2, 700, x.device)
    engine.forward("ADSDN", m.engine_code, m.packed_weights(x.device), x, workspace=ws)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        with pytest.raises(ValueError, match="stream"):
            engine.forward("ADSDN", m.engine_code, m.packed_weights(x.device), x, workspace=ws)
    torch.cuda.synchronize()
