"""Empty batches through every entry point, every network and engine dtype: the reference modules
accept an (0, 1, L) input (nn.Conv1d on an empty batch, */train.py forward) and return an empty
(0, 1, L) output; so must the drop-in modules, engine.forward / forward_metrics (no launch, zero
metric sums, status words untouched), the metrics pass and the simulator.  A following non-empty call
on the same cached workspace is unaffected (bitwise equal to a fresh module)."""
import numpy as np
import pytest
import torch

from conftest import golden_state_dict

pytestmark = pytest.mark.gpu

ARCHS = ["DenoiseCNN", "RRCDNet", "DSDN", "ADSDN", "PIDN", "APIDN"]


def _model(arch, dtype):
    import raman_mi355x as R
    m = R.MODELS[arch]()
    m.load_state_dict(golden_state_dict(arch, "synth"), strict=True)
    return m.cuda().eval().set_engine_dtype(dtype)


@pytest.mark.parametrize("dtype", ["fp32", "f16", "f16f8"])
@pytest.mark.parametrize("arch", ARCHS)
def test_empty_batch_module_and_engine(arch, dtype):
    from raman_mi355x import engine
    m = _model(arch, dtype)
    L = 700
    x0 = torch.empty((0, 1, L), dtype=torch.float32, device="cuda")
    with torch.no_grad():
        y0 = m(x0)
        assert tuple(y0.shape) == (0, 1, L) and y0.dtype == torch.float32 and y0.is_cuda
        # a non-empty batch on the same module (its workspace cached by the empty call) is unaffected
        x = torch.from_numpy(np.random.default_rng(9).uniform(0, 1, (3, 1, L)).astype(np.float32)).cuda()
        y = m(x)
        fresh = _model(arch, dtype)(x)
    torch.cuda.synchronize()
    assert torch.equal(y, fresh)
    packed = m.packed_weights(x0.device)
    ye = engine.forward(arch, m.engine_code, packed, x0)
    assert tuple(ye.shape) == (0, 1, L)
    clean0 = torch.empty((0, L), dtype=torch.float32, device="cuda")
    y1, per, sums, fused = engine.forward_metrics(arch, m.engine_code, packed, x0, clean0, per_spectrum=True,
                                                  acc=engine.new_acc(x0.device))
    assert tuple(y1.shape) == (0, 1, L) and tuple(per.shape) == (0, 4)
    assert not fused
    assert torch.count_nonzero(sums).item() == 0


def test_empty_metrics_and_simulator():
    from raman_mi355x import engine
    dev = torch.device("cuda")
    clean, noisy, snr, std = engine.generate(0, 1, signal_length=500, device=dev)
    assert tuple(clean.shape) == tuple(noisy.shape) == (0, 500) and snr.numel() == std.numel() == 0
    acc = engine.new_acc(dev)
    sums = torch.zeros(5, dtype=torch.float64, device=dev)
    out = engine.metrics(noisy, clean, sums=sums, per_spectrum=True, acc=acc)
    torch.cuda.synchronize()
    assert torch.count_nonzero(sums).item() == 0 and torch.count_nonzero(acc).item() == 0
    assert out is not None


@pytest.mark.parametrize("arch", ["RRCDNet", "ADSDN"])
def test_workspace_made_for_empty_batch_still_reports_status(arch):
    """A Workspace created for n = 0 and reused for a larger batch (its geometry does not depend on n):
    check() still reads the sticky status words -- here the input gate of an input beyond |x| = 4."""
    from raman_mi355x import engine
    m = _model(arch, "f16")
    L = 700
    x0 = torch.empty((0, 1, L), dtype=torch.float32, device="cuda")
    ws = engine.Workspace(arch, m.engine_code, 0, L, x0.device)
    packed = m.packed_weights(x0.device)
    engine.forward(arch, m.engine_code, packed, x0, check=False, workspace=ws)
    assert ws.check() == 0
    x = torch.from_numpy(np.random.default_rng(4).uniform(0, 1, (3, 1, L)).astype(np.float32)).cuda()
    x[1, 0, 100] = 9.0
    if not ws.fits(arch, m.engine_code, 3, L, x.device):
        pytest.skip("this geometry sizes the workspace by n")
    engine.forward(arch, m.engine_code, packed, x, check=False, workspace=ws, _ws_checked=True)
    assert ws.check() & engine.STATUS_GATE
    assert ws.check() == 0                             # read and cleared
