"""CPU emulation of RDN_F16MIX with the correction MFMA's operands in e2m3 (fp6, block-scaled) instead of
e4m3: does the corrected tail keep its precision?  Diagnostic, not part of the product.

Corrected layer (right big layers 10-14), per tap and 64 input channels:
    y = f16(W) . f16(X)                                 (the f16 MFMAs, fp64 accumulation here)
      + Q(W_lo) . Q(X_hi) + Q(W_hi) . Q(X_lo)          (the block-scaled correction MFMA)
with W_lo = W - f16(W), X_lo = X - f16(X).  Q:
  e4m3  (shipped)   per-value 3-bit mantissa; activations at fixed scales (hi / 4, lo * 2^9, subnormals
                    below 2^-6), weights with one E8M0 scale per 32-value block
  e2m3  (candidate) one E8M0 scale per block of 16 channels -- hi and lo parts of the same 16 channels
                    sharing it (lo pre-scaled by 2^11 on both sides), chosen from the block max; e2m3
                    values (subnormal step 1/8, max 7.5)
  e2m3s (optimistic) as e2m3 with separate scales for the hi and lo parts
Plain layers: f16 weights and activations.  Heads: right split (f16 + e4m3 residue), left f16 (the
shipped hybrid).  Data: config 1's 1000 spectra (oracle.refgen), the worst SEL of each weight set.

    python tools/f6_emul.py [--sel 32]
"""
import argparse
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

from conftest import GOLDEN, golden_state_dict  # noqa: E402
from head_fusion_emul import e4m3_split, f16  # noqa: E402
from precision_sweep import fold  # noqa: E402

TAIL = set(range(10, 15))


def q_e4m3_value(t, min_exp=-6):
    """per-value e4m3 rounding (3-bit mantissa), subnormal step 2^(min_exp - 3)"""
    m, e = torch.frexp(t)                     # t = m 2^e, |m| in [0.5, 1)
    e = torch.clamp(e, min=min_exp + 1)
    step = torch.ldexp(torch.ones_like(t), e - 4)
    return torch.round(t / step) * step


def q_e2m3_block(t, dim, scale_from=None):
    """e2m3 with one power-of-two scale per block along `dim` (block max -> [4, 8))"""
    amax = (scale_from if scale_from is not None else t).abs().amax(dim=dim, keepdim=True)
    _, e = torch.frexp(amax)                  # amax in [2^(e-1), 2^e)
    s = torch.ldexp(torch.ones_like(amax), e - 3)     # amax / s in [4, 8)
    v = t / s
    a = v.abs()
    step = torch.where(a < 2, 0.125, torch.where(a < 4, 0.25, 0.5))
    q = torch.clamp(torch.round(a / step) * step, max=7.5)
    return torch.sign(v) * q * s


def blocks_x(t):
    """[B, 64, L] -> [B, 4, 16, L] (16-channel blocks)"""
    return t.reshape(t.shape[0], 4, 16, t.shape[-1])


def blocks_w(t):
    """[64, 64, 3] -> [64, 4, 16, 3]"""
    return t.reshape(64, 4, 16, 3)


def correction(w, x, dil, fmt):
    """Q(W_lo) . Q(X_hi) + Q(W_hi) . Q(X_lo) for one conv"""
    wh, xh = f16(w), f16(x)
    wl, xl = w - wh, x - xh
    if fmt == "exact":
        a1, b1, a2, b2 = wl, xh, wh, xl
    elif fmt == "e4m3":
        b1 = q_e4m3_value(xh / 4) * 4
        b2 = q_e4m3_value(xl * 2 ** 9) / 2 ** 9
        # weights: 32-value blocks, scale to the block max (e4m3 max 448 -> the block max at ~2^8)
        a1 = q_e4m3_value(wl * 2 ** 11) / 2 ** 11
        a2 = q_e4m3_value(wh)
    else:
        xs, ws = blocks_x, blocks_w
        if fmt == "e2m3":        # hi and lo parts share the block's scale (lo pre-scaled by 2^11)
            xsc = torch.maximum(xs(xh).abs(), xs(xl).abs() * 2 ** 11)
            wsc = torch.maximum(ws(wh).abs(), ws(wl).abs() * 2 ** 11)
            b1 = q_e2m3_block(xs(xh), 2, xsc).reshape(x.shape)
            b2 = (q_e2m3_block(xs(xl) * 2 ** 11, 2, xsc) / 2 ** 11).reshape(x.shape)
            a1 = (q_e2m3_block(ws(wl) * 2 ** 11, 2, wsc) / 2 ** 11).reshape(w.shape)
            a2 = q_e2m3_block(ws(wh), 2, wsc).reshape(w.shape)
        else:                    # e2m3s: separate scales
            b1 = q_e2m3_block(xs(xh), 2).reshape(x.shape)
            b2 = q_e2m3_block(xs(xl), 2).reshape(x.shape)
            a1 = q_e2m3_block(ws(wl), 2).reshape(w.shape)
            a2 = q_e2m3_block(ws(wh), 2).reshape(w.shape)
    return F.conv1d(b1, a1, padding=dil, dilation=dil) + F.conv1d(b2, a2, padding=dil, dilation=dil)


def rrcdnet(sd, x, fmt):
    x = x.double()
    layers = []
    for i in range(3, 18):
        layers.append((f"right_net.{i}.0", f"right_net.{i}.1", 1))
    for i in range(3, 10):
        layers.append((f"left_net.{i}.0", None, 2))
    layers.append(("left_net.10", "left_net.11", 1))
    for i in range(13, 19):
        layers.append((f"left_net.{i}.0", None, 2))

    def branch(stem_conv, stem_bn, ks, head_conv, split_head):
        w, b = fold(sd, stem_conv, stem_bn)
        h = torch.relu(F.conv1d(x, w, b, padding=1))
        h = f16(h)
        for k in ks:
            conv, bn, dil = layers[k]
            w, b = fold(sd, conv, bn)
            # the f16 product; a corrected layer's input keeps its fp32 value for the residue
            y = F.conv1d(f16(h), f16(w), b, padding=dil, dilation=dil)
            if k in TAIL:
                y = y + correction(w, h, dil, fmt)
            y = torch.relu(y)
            last = k in (14, 28)
            if last:
                h = e4m3_split(y) if split_head else f16(y)
            else:
                h = y.float().double() if (k + 1) in TAIL else f16(y)
        w, b = fold(sd, head_conv, None)
        return F.conv1d(h, w, b, padding=1)

    r = branch("right_net.0", "right_net.1", list(range(0, 15)), "right_net.18", True)
    l = branch("left_net.0", "left_net.1", list(range(15, 29)), "left_net.19", False)
    return (x - (r + l) / 2).float()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sel", type=int, default=32)
    ap.add_argument("--fmts", nargs="*", default=["exact", "e4m3", "e2m3", "e2m3s"])
    args = ap.parse_args()
    from oracle.models import forward as oracle_forward
    from oracle.refgen import generate_signals
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    np.random.seed(20250410)
    _, noisy, _, _ = generate_signals(1000)
    X = torch.tensor(noisy, dtype=torch.float32)
    h2 = np.load(os.path.join(GOLDEN, "heldout2_RRCDNet.npz"))
    h1 = np.load(os.path.join(GOLDEN, "heldout_RRCDNet.npz"))
    weights = {"fixture": golden_state_dict("RRCDNet", "trained"),
               "tuning": {k[3:]: torch.from_numpy(np.array(h1[k])) for k in h1.files if k.startswith("w::")},
               "heldout2": {k[3:]: torch.from_numpy(np.array(h2[k])) for k in h2.files if k.startswith("w::")}}
    for wn, sd in weights.items():
        cache = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"f6_emul_{wn}.npz")
        if os.path.exists(cache):
            c = np.load(cache)
            ref, per = c["ref"], c["per"]
        else:
            ref = torch.cat([oracle_forward("RRCDNet", sd, X[i:i + 50].unsqueeze(1)) for i in range(0, 1000, 50)]).squeeze(1).numpy()
            per = np.concatenate([np.abs(rrcdnet(sd, X[i:i + 25].unsqueeze(1), "e4m3").squeeze(1).numpy() - ref[i:i + 25]).max(axis=1)
                                  for i in range(0, 1000, 25)])
            np.savez(cache, ref=ref, per=per)
        sel = np.argsort(per)[::-1][:args.sel].copy()
        xs = X[sel].unsqueeze(1)
        line = []
        for fmt in args.fmts:
            y = torch.cat([rrcdnet(sd, xs[i:i + 16], fmt) for i in range(0, len(sel), 16)]).squeeze(1).numpy()
            line.append(f"{fmt} {np.abs(y - ref[sel]).max():.4e}")
        print(f"{wn:9s} worst {args.sel} of 1000 (e4m3 max {per.max():.4e}): " + "  ".join(line), flush=True)


if __name__ == "__main__":
    main()
