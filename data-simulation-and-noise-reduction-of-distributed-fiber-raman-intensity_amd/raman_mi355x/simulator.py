"""Drop-in for ``generate_signals`` (数据集产生.py:5-64), generated on the GPU.

``generate_signals`` keeps the reference signature and return convention (float64 numpy arrays:
clean (N, L), noisy (N, L), snrs (N, 1), noise_std (N, 1)); ``generate`` returns device tensors
for pipelines that feed the engine directly.  Spectrum i of stream ``seed`` is a pure function of
(seed, i) — see csrc/generator.hip — so ``first_index`` selects any slice of an endless data set.
"""
import numpy as np
import torch

from . import engine


def generate(num_samples, seed=20250410, first_index=0, signal_length=10000, snr_range=(20, 37),
             extreme_noise_prob=0.05, max_repeat=40, device="cuda"):
    clean, noisy, snr, nstd = engine.generate(int(num_samples), seed, first_index, signal_length, snr_range,
                                              extreme_noise_prob, max_repeat, device)
    return clean, noisy, snr.view(-1, 1), nstd.view(-1, 1)


def generate_signals(num_samples, signal_length=10000, snr_range=(20, 37), extreme_noise_prob=0.05,
                     max_repeat=40, seed=None, first_index=0, device="cuda"):
    if seed is None:
        seed = int(np.random.randint(0, 2**63 - 1, dtype=np.int64))
    out = generate(num_samples, seed, first_index, signal_length, snr_range, extreme_noise_prob, max_repeat, device)
    return tuple(t.double().cpu().numpy() for t in out)
