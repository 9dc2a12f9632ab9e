"""CPU emulation of the engine's reduced-precision conv arithmetic (tolerance sweep).

Emulates, per Conv1d(64,64,3): operands rounded to the chosen format (optionally split into a
hi + lo pair), products accumulated in fp64 (upper bound of the fp32 MFMA accumulate), bias +
activation in fp32, and the stored activation rounded to the activation format.  Compares against
the reference-faithful fp32 CPU oracle on the golden inputs.

    python tools/precision_sweep.py [arch] [weights: trained|synth]
"""
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def q(t, fmt):
    if fmt == "f32":
        return t.float().double()
    if fmt == "bf16":
        return t.float().bfloat16().double()
    if fmt == "f16":
        return t.float().half().double()
    raise ValueError(fmt)


def split(t, fmt, terms):
    hi = q(t, fmt)
    if terms == 1:
        return [hi]
    lo = q(t - hi, fmt)
    return [hi, lo]


def conv_emul(x, w, b, dil, wfmt, xfmt, wterms, xterms):
    ws = split(w, wfmt, wterms)
    xs = split(x, xfmt, xterms)
    y = 0
    for i, wi in enumerate(ws):
        for j, xj in enumerate(xs):
            if i + j >= max(wterms, xterms):      # drop lo*lo
                continue
            y = y + F.conv1d(xj, wi, None, padding=dil * (w.shape[-1] // 2), dilation=dil)
    return y + b.double()[None, :, None]


def fold(sd, conv, bn):
    w = sd[conv + ".weight"].double()
    b = sd[conv + ".bias"].double()
    if bn:
        s = sd[bn + ".weight"].double() / torch.sqrt(sd[bn + ".running_var"].double() + 1e-5)
        w = w * s[:, None, None]
        b = (b - sd[bn + ".running_mean"].double()) * s + sd[bn + ".bias"].double()
    return w.float().double(), b.float().double()


def rrcdnet(sd, x, mode):
    wfmt, xfmt, wt, xt = mode if mode else (None,)*4
    x = x.double()

    def big(h, conv, bn, dil, relu=True):
        w, b = fold(sd, conv, bn)
        y = conv_emul(h, w, b, dil, wfmt, xfmt, wt, xt)
        y = torch.relu(y) if relu else y
        return y.float().double()

    def stem(conv, bn):
        w, b = fold(sd, conv, bn)
        return torch.relu(F.conv1d(x, w, b, padding=1)).float().double()

    def head(h, conv):
        w, b = fold(sd, conv, None)
        return conv_emul(h, w, b, 1, wfmt, xfmt, wt, xt)

    r = stem("right_net.0", "right_net.1")
    for i in range(3, 18):
        r = big(r, f"right_net.{i}.0", f"right_net.{i}.1", 1)
    r = head(r, "right_net.18")
    h = stem("left_net.0", "left_net.1")
    for i in range(3, 10):
        h = big(h, f"left_net.{i}.0", None, 2)
    h = big(h, "left_net.10", "left_net.11", 1)
    for i in range(13, 19):
        h = big(h, f"left_net.{i}.0", None, 2)
    left = head(h, "left_net.19")
    return (x - (r + left) / 2).float()


def main():
    from conftest import golden_inputs, golden_state_dict, load_golden
    which = sys.argv[2] if len(sys.argv) > 2 else "trained"
    sd = golden_state_dict("RRCDNet", which)
    g = load_golden("RRCDNet")
    x = torch.from_numpy(golden_inputs()["main_noisy"][:1]).unsqueeze(1)
    ref = torch.from_numpy(g[f"{which}_main"][:1]).unsqueeze(1)
    modes = [("f32", "f32", 1, 1), ("bf16", "bf16", 1, 1), ("bf16", "bf16", 1, 2), ("bf16", "bf16", 2, 1),
             ("bf16", "bf16", 2, 2), ("f16", "f16", 1, 1), ("f16", "bf16", 1, 1), ("bf16", "f16", 1, 1),
             ("f16", "f16", 1, 2)]
    for mode in modes:
        y = rrcdnet(sd, x, mode)
        print(f"W {mode[0]}x{mode[2]}  X {mode[1]}x{mode[3]}: max-abs {float((y - ref).abs().max()):.3e}")


if __name__ == "__main__":
    main()
