"""CPU emulation of RRCDNet's 16-bit modes: which layers need the e4m3 correction when the heads read
the last layer's fp32 accumulators (head fused into that layer's epilogue) instead of its stored
f16 (+ e4m3 residue) activations.  Diagnostic, not part of the product.

Model per Conv1d(64, 64, 3): plain layer = f16(W) x (stored activation), fp64 accumulation (upper
bound of the fp32 MFMA chain), bias + ReLU, output stored as f16 unless the consumer is corrected
(then the producer also writes the e4m3 planes: modelled as the fp32 value); corrected layer =
W x activation in fp32.  Head: 'f16' (f16 activations, exact weights: fused16), 'split' (f16 + e4m3
residue ~ fp32: the in-place head), 'fused' (the fp32 accumulators of the last layer).  Error as
tests/test_forward_gpu.py test_16bit_within_tolerance measures it (bar 2e-2).

    python tools/head_fusion_emul.py
"""
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from conftest import INPUT_SETS, golden_inputs, golden_state_dict, input_array, load_golden  # noqa: E402

from precision_sweep import fold  # noqa: E402


def f16(t):
    return t.float().half().double()


def f32(t):
    return t.float().double()


def e4m3_split(t):
    """f16 hi + e4m3 residue (the in-place tile's split planes), fp64"""
    hi = f16(t)
    lo = (t - hi).float()
    # e4m3 with a per-value scale is ~4 significant bits of the residue
    m, e = torch.frexp(lo)
    lo4 = torch.ldexp(torch.round(m * 16) / 16, e).double()
    return hi + lo4


def rrcdnet(sd, x, corrected, head, term="both"):
    """corrected: set of big-layer indices (0-14 right, 15-28 left) computed from fp32 operands
    (term 'both'), from fp32 activations and f16 weights ('x': only the activation residue
    corrected) or from f16 activations and fp32 weights ('w')."""
    x = x.double()
    layers = []       # (conv, bn, dil) per big layer, blob order
    for i in range(3, 18):
        layers.append((f"right_net.{i}.0", f"right_net.{i}.1", 1))
    for i in range(3, 10):
        layers.append((f"left_net.{i}.0", None, 2))
    layers.append(("left_net.10", "left_net.11", 1))
    for i in range(13, 19):
        layers.append((f"left_net.{i}.0", None, 2))

    def store(y, k):
        """activation as the consumer of layer k's output sees it"""
        last = k in (14, 28)
        if last:     # head: one mode for both heads, or "right/left"
            hm = head.split("/")
            return {"f16": f16, "split": e4m3_split, "fused": f32}[hm[0] if k == 14 or len(hm) == 1 else hm[1]](y)
        return f32(y) if (k + 1) in corrected and term != "w" else f16(y)

    def branch(stem_conv, stem_bn, ks, head_conv):
        w, b = fold(sd, stem_conv, stem_bn)
        h = torch.relu(F.conv1d(x, w, b, padding=1))
        h = f32(h) if ks[0] in corrected and term != "w" else f16(h)
        for k in ks:
            conv, bn, dil = layers[k]
            w, b = fold(sd, conv, bn)
            wq = w if k in corrected and term != "x" else f16(w)
            y = torch.relu(F.conv1d(h, wq, b, padding=dil, dilation=dil))
            h = store(y, k)
        w, b = fold(sd, head_conv, None)
        return F.conv1d(h, w, b, padding=1)

    r = branch("right_net.0", "right_net.1", list(range(0, 15)), "right_net.18")
    l = branch("left_net.0", "left_net.1", list(range(15, 29)), "left_net.19")
    return (x - (r + l) / 2).float()


def worst(corrected, head, data, term="both"):
    """per weight set: the test's error / tolerance ratio x 2e-2 (trained: max-abs; synth: max-abs /
    max(1, max|ref|))"""
    out = {}
    for which, sd, xs, refs in data:
        e = 0.0
        for x, ref in zip(xs, refs):
            y = rrcdnet(sd, x, corrected, head, term).squeeze(1).numpy()
            scale = 1.0 if which == "trained" else max(1.0, float(np.abs(ref).max()))
            e = max(e, float(np.abs(y - ref).max()) / scale)
        out[which] = e
    return out


def main():
    torch.set_num_threads(8)
    g = load_golden("RRCDNet")
    inp = golden_inputs()
    data = []
    for which in ["synth", "trained"]:
        sd = golden_state_dict("RRCDNet", which)
        xs = [torch.from_numpy(np.ascontiguousarray(input_array(inp, s))).unsqueeze(1) for s in INPUT_SETS]
        refs = [g[f"{which}_{s}"] for s in INPUT_SETS]
        data.append((which, sd, xs, refs))
    configs = [(set(), "f16", "both"), (set(), "split", "both"), (set(), "fused", "both"),
               ({12, 13, 14}, "split", "both"), ({12, 13, 14}, "fused", "both"), ({13, 14}, "fused", "both"),
               ({14}, "fused", "both"), ({13, 14, 28}, "fused", "both"),
               ({12, 13, 14}, "split", "x"), ({12, 13, 14}, "split", "w"), ({11, 12, 13, 14}, "split", "x"),
               ({10, 11, 12, 13, 14}, "split", "x")]
    if len(sys.argv) > 1 and sys.argv[1] == "heads":
        configs = [({12, 13, 14}, "split/f16", "both"), ({12, 13, 14}, "f16/split", "both"), ({12, 13, 14}, "f16", "both"),
                   ({11, 12, 13, 14}, "f16", "both"), ({12, 13, 14, 28}, "split/f16", "both")]
    elif len(sys.argv) > 1:
        configs = [c for c in configs if c[2] != "both"]
    for corrected, head, term in configs:
        w = worst(corrected, head, data, term)
        print(f"corrected {sorted(corrected)!s:20s} ({term:4s}) head {head:9s}: " +
              "  ".join(f"{k} {v:.3e}" for k, v in w.items()), flush=True)


if __name__ == "__main__":
    main()
