"""Batched, on-device replacement of the reference evaluation harness (*/evaulate.py).

``evaluate(model, noisy_data, clean_data)`` returns the same dict as evaulate.py:25-39
({MSE, SSIM, Smoothness, Peak2Peak} averaged over spectra) but runs the forward in batches and the
metrics in the fp64 device kernel instead of a batch-1 loop with a host sync per spectrum.  Under
torch.distributed each rank evaluates its contiguous shard and the metric sums are all-reduced.
``write_metrics`` produces evaulate.py:78-80's ``metrics.txt`` format.
"""
import os
from datetime import datetime

import numpy as np
import torch

from . import engine
from .distributed import all_reduce_sums, means, shard


def _as_rows(a):
    if torch.is_tensor(a):
        return a.reshape(a.shape[0], -1)
    a = np.asarray(a)
    return a.reshape(a.shape[0], -1)


def evaluate(model, noisy_data, clean_data, batch_size=1024, device=None):
    model.eval()
    if device is None:
        device = next(model.parameters()).device
    device = torch.device(device)
    noisy = _as_rows(noisy_data)
    clean = _as_rows(clean_data)
    if noisy.shape != clean.shape:
        raise ValueError(f"noisy {tuple(noisy.shape)} vs clean {tuple(clean.shape)}")
    lo, hi = shard(noisy.shape[0])
    sums = torch.zeros(5, dtype=torch.float64, device=device)
    with torch.no_grad():
        for b0 in range(lo, hi, batch_size):
            b1 = min(hi, b0 + batch_size)
            x = torch.as_tensor(noisy[b0:b1], dtype=torch.float32).to(device).unsqueeze(1)
            c = torch.as_tensor(clean[b0:b1], dtype=torch.float32).to(device)
            y = model(x)
            engine.metrics(y.squeeze(1), c, sums=sums, per_spectrum=False)
    all_reduce_sums(sums)
    return means(sums)


def write_metrics(metrics, root="eval_results"):
    save_dir = os.path.join(root, datetime.now().strftime("%Y%m%d_%H%M%S"))
    os.makedirs(save_dir, exist_ok=True)
    with open(os.path.join(save_dir, "metrics.txt"), "w") as f:
        for k, v in metrics.items():
            f.write(f"{k}: {v:.6f}\n")
    return save_dir
