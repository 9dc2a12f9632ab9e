"""Deterministic synthetic reference-format state_dicts (TEST INFRASTRUCTURE — see oracle/__init__).

The reference ships no checkpoints, so fixtures are built from seeded weights.
Every tensor gets its own PCG64 stream keyed by (seed, crc32(key)), so the result does not depend
on key order.  BatchNorm running statistics are randomised away from (0, 1) so that the engine's
load-time BN folding is actually exercised; convolution weights use a fan-in Kaiming scale so that
activations neither vanish nor explode through 30+ layers.
"""
import zlib

import numpy as np
import torch


def _rng(seed, key):
    return np.random.default_rng([int(seed), zlib.crc32(key.encode())])


def synth_tensor(seed, key, shape, dtype=torch.float32):
    if dtype == torch.int64:                      # BatchNorm num_batches_tracked
        return torch.tensor(1000, dtype=torch.int64)
    r = _rng(seed, key)
    leaf = key.rsplit(".", 1)[-1]
    shape = tuple(shape)
    if leaf == "running_mean":
        a = r.uniform(-0.15, 0.15, shape)
    elif leaf == "running_var":
        a = r.uniform(0.5, 1.6, shape)
    elif leaf == "weight" and len(shape) == 3:    # Conv1d (Cout, Cin, K)
        fan_in = shape[1] * shape[2]
        a = r.standard_normal(shape) * np.sqrt(2.0 / fan_in)
    elif leaf == "weight" and len(shape) == 2:    # Linear (out, in)
        a = r.standard_normal(shape) * np.sqrt(1.0 / shape[1])
    elif leaf == "bias":
        a = r.uniform(-0.05, 0.05, shape)
    else:
        raise KeyError(f"no synthesis rule for {key} {shape}")
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32))


def synth_state_dict(template, seed, conv_gain=1.0):
    """``template``: ordered {key: (shape, dtype)}.  BN is recognised by its running stats.

    ``conv_gain`` scales the 64->64 convolution weights (deep residual stacks need < 1 to stay finite).
    """
    bn_prefixes = {k.rsplit(".", 1)[0] for k in template if k.endswith("running_mean")}
    out = {}
    for key, (shape, dtype) in template.items():
        prefix = key.rsplit(".", 1)[0]
        if prefix in bn_prefixes and key.endswith((".weight", ".bias")):
            r = _rng(seed, key)
            lo, hi = (0.7, 1.3) if key.endswith(".weight") else (-0.1, 0.1)
            out[key] = torch.from_numpy(r.uniform(lo, hi, tuple(shape)).astype(np.float32))
        else:
            t = synth_tensor(seed, key, shape, dtype)
            if conv_gain != 1.0 and t.dim() == 3 and t.shape[0] == t.shape[1] == 64:
                t = t * np.float32(conv_gain)
            out[key] = t
    return out
