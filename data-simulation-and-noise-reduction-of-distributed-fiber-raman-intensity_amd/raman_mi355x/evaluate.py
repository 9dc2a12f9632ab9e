"""Batched, on-device replacements of the reference evaluation harness (*/evaulate.py).

``evaluate(model, noisy_data, clean_data)`` returns the same dict as evaulate.py:25-39
({MSE, SSIM, Smoothness, Peak2Peak} averaged over spectra) but runs the forward in batches and the
metrics in the fp64 device kernel instead of a batch-1 loop with a host sync per spectrum.  The
clean reference stays float64 (evaulate.py:34-35 compares against the float64 test.npz arrays).

``evaluate_synthetic(models, total, ...)`` is the config-4 driver: a fixed total of
N simulator spectra, rank r of W owning indices [r·N/W, (r+1)·N/W), chunked generate -> forward ->
metric sums per network, one all-reduce at the end.  The simulator is counter-based and the sums
are exact integer accumulators (rdn_metrics_ex), so the four means are the same bits for any W,
batch size or atomics order.

Under torch.distributed each rank evaluates its contiguous shard and the metric accumulators are
all-reduced (RCCL over xGMI for CUDA tensors).  The CBAM networks' hand-off status is checked once
per network at the end (engine.Workspace), not per batch.  ``write_metrics`` produces
evaulate.py:78-80's ``metrics.txt`` format.
"""
import os
import sys
import time
from datetime import datetime

import numpy as np
import torch
import torch.distributed as dist

from . import _lib, engine
from .distributed import shard, world

KEYS = ("MSE", "SSIM", "Smoothness", "Peak2Peak")


def _as_rows(a):
    if torch.is_tensor(a):
        return a.reshape(a.shape[0], -1)
    a = np.asarray(a)
    return a.reshape(a.shape[0], -1)


def _all_reduce_acc(acc):
    """SUM all-reduce of an exact accumulator (int64, exact under any reduction order)."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        if dist.get_backend() == "gloo" and acc.is_cuda:        # gloo reduces host tensors
            h = acc.cpu()
            dist.all_reduce(h, op=dist.ReduceOp.SUM)
            acc.copy_(h)
        else:
            dist.all_reduce(acc, op=dist.ReduceOp.SUM)
    return acc


def means_from_acc(acc):
    """{MSE, SSIM, Smoothness, Peak2Peak} means of an exact accumulator (evaulate.py:39)."""
    s = engine.acc_value(acc).tolist()
    if s[4] <= 0:
        raise ValueError("no spectra were evaluated")
    return {k: s[i] / s[4] for i, k in enumerate(KEYS)}


def _engine_module(model):
    """A raman_mi355x network whose own forward is the engine (not a subclass overriding forward)."""
    from .models import _EngineNet
    return isinstance(model, _EngineNet) and type(model).forward is _EngineNet.forward


def _finish(model, ws):
    """One status read after all of a network's batches (rdn_forward_status_ex: the sticky words of every
    forward since): raises on a timed-out CBAM hand-off or a saturated tile, and RangeError when a 16-bit
    forward saw an input beyond the gate (the kernels' stems raise it, fused and CBAM networks alike)."""
    from .models import INPUT_GATE
    flags = ws.check() if ws is not None else 0
    if flags & engine.STATUS_GATE and model.engine_code != 0:
        raise _lib.RangeError(f"evaluate: |input| beyond the 16-bit modes' domain ({INPUT_GATE}, normalised "
                              f"intensity); evaluate this data in 'fp32'")


def _workspace(model, n, L, device):
    if (not _engine_module(model) or not engine.needs_workspace(model.ARCH, model.engine_code)
            or torch.device(device).type != "cuda"):
        return None
    return engine.Workspace(model.ARCH, model.engine_code, n, L, device)


def evaluate(model, noisy_data, clean_data, batch_size=1024, device=None):
    """evaulate.py:25-39 batched on the device.  Inputs beyond the 16-bit modes' domain (|x| > 4) or
    activations beyond the e4m3 planes' range raise RangeError after the run (one check at the end,
    no per-batch wait) -- unlike the module's own forward, which re-runs such a batch in fp32: evaluate
    such data with the module in 'fp32'."""
    model.eval()
    if device is None:
        device = next(model.parameters()).device
    device = torch.device(device)
    noisy = _as_rows(noisy_data)
    clean = _as_rows(clean_data)
    if noisy.shape != clean.shape:
        raise ValueError(f"noisy {tuple(noisy.shape)} vs clean {tuple(clean.shape)}")
    lo, hi = shard(noisy.shape[0])
    L = noisy.shape[1]
    if device.type != "cuda":
        raise RuntimeError("raman_mi355x.evaluate runs its metrics on the GPU; on a CPU device use the module "
                           "itself in the reference's evaulate.py loop (its forward falls back to eager PyTorch)")
    acc = engine.new_acc(device)
    ws = _workspace(model, min(batch_size, max(hi - lo, 1)), L, device)
    # fp64 clean stays fp64 (the metrics compare against the same float64 values as evaulate.py)
    cdt = torch.float64 if (clean.dtype == torch.float64 if torch.is_tensor(clean) else clean.dtype == np.float64) \
        else torch.float32
    with torch.no_grad():
        for b0 in range(lo, hi, batch_size):
            b1 = min(hi, b0 + batch_size)
            x = torch.as_tensor(noisy[b0:b1], dtype=torch.float32).to(device).unsqueeze(1)
            c = torch.as_tensor(clean[b0:b1], dtype=cdt).to(device)
            if _engine_module(model) and model.uses_engine(x):
                # the engine's forward + metric sums (fused into the forward kernel on the walk geometry)
                engine.forward_metrics(model.ARCH, model.engine_code, model.packed_weights(x.device), x, c, acc=acc,
                                       check=False, workspace=ws)
            else:
                y = model(x)
                engine.metrics(y.squeeze(1), c, per_spectrum=False, acc=acc)
    _finish(model, ws)
    _all_reduce_acc(acc)
    return means_from_acc(acc)


def evaluate_synthetic(models, total, seed=20250410, signal_length=10000, batch_size=8192, device=None,
                       first_index=0, gen_kwargs=None, log_every_s=0.0, fused_metrics=True):
    """Config 4: ``total`` simulator spectra [first_index, first_index + total),
    sharded over the ranks as [r·N/W, (r+1)·N/W), each chunk generated on the device, denoised by
    every model in ``models`` (name -> module) and metered into that model's exact accumulator.
    Returns {name: {"means", "spectra", "seconds", "spectra_per_s"}} with the all-reduced means
    (identical for any world size) and the max-over-ranks wall time of the loop.  ``log_every_s`` > 0
    prints progress to stderr about that often (the loop then waits for the device every 64 chunks,
    so the printed count is what the GPU has finished).  ``fused_metrics=False`` meters with the separate
    metrics kernel after each forward (the A/B of the metric epilogue; the same bits)."""
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device())
    device = torch.device(device)
    gen_kwargs = gen_kwargs or {}
    rank, W = world()
    lo, hi = shard(total, rank, W)
    L = int(signal_length)
    B = max(1, min(batch_size, hi - lo)) if hi > lo else 1
    clean = torch.empty((B, L), dtype=torch.float32, device=device)
    noisy = torch.empty((B, L), dtype=torch.float32, device=device)
    y = torch.empty((B, 1, L), dtype=torch.float32, device=device)
    out = {}
    with torch.no_grad():
        for name, model in models.items():
            model.eval()
            acc = engine.new_acc(device)
            ws = _workspace(model, B, L, device)
            packed = model.packed_weights(device)
            if dist.is_available() and dist.is_initialized():
                dist.barrier()
            torch.cuda.synchronize(device)
            t0 = time.perf_counter()
            t_log = t0
            for i, b0 in enumerate(range(lo, hi, B)):
                if log_every_s > 0 and i % 64 == 63:
                    torch.cuda.synchronize(device)
                    if time.perf_counter() - t_log >= log_every_s:
                        t_log = time.perf_counter()
                        print(f"[evaluate_synthetic rank {rank}] {name}: {b0 - lo} / {hi - lo} spectra, "
                              f"{t_log - t0:.1f} s", file=sys.stderr, flush=True)
                nb = min(B, hi - b0)
                engine.generate(nb, seed, first_index=first_index + b0, signal_length=L, device=device,
                                out=(clean[:nb], noisy[:nb]), **gen_kwargs)
                # forward + metric sums in one call: on the walk geometry the forward kernel meters each
                # spectrum itself (no second pass over y); otherwise the metrics kernel follows it
                if fused_metrics:
                    engine.forward_metrics(model.ARCH, model.engine_code, packed, noisy[:nb].view(nb, 1, L),
                                           clean[:nb], out=y[:nb], acc=acc, check=False, workspace=ws)
                else:
                    engine.forward(model.ARCH, model.engine_code, packed, noisy[:nb].view(nb, 1, L), out=y[:nb],
                                   check=False, workspace=ws)
                    engine.metrics(y[:nb].view(nb, L), clean[:nb], per_spectrum=False, acc=acc)
            _finish(model, ws)              # waits for the stream; raises on a timed-out hand-off / range / gate
            torch.cuda.synchronize(device)
            el = time.perf_counter() - t0
            t = torch.tensor([el], dtype=torch.float64)
            if dist.is_available() and dist.is_initialized() and W > 1:
                tt = t.to(device) if dist.get_backend() != "gloo" else t
                dist.all_reduce(tt, op=dist.ReduceOp.MAX)
                t = tt.cpu()
            _all_reduce_acc(acc)
            el = float(t.item())
            out[name] = {"means": means_from_acc(acc), "acc": acc.cpu().tolist(), "spectra": int(total),
                         "seconds": el, "spectra_per_s": total / el if el > 0 else None}
    return out


def write_metrics(metrics, root="eval_results"):
    save_dir = os.path.join(root, datetime.now().strftime("%Y%m%d_%H%M%S"))
    os.makedirs(save_dir, exist_ok=True)
    with open(os.path.join(save_dir, "metrics.txt"), "w") as f:
        for k, v in metrics.items():
            f.write(f"{k}: {v:.6f}\n")
    return save_dir
