"""Train the realistically-trained held-out RRCDNet for the headline parity pin (run on a GPU box).

    python tests/golden/train_heldout_gpu.py --out scratch/heldout2 [--steps 12000] [--max-seconds 1000]

Fixture generation (test infrastructure), not product code.  The reference trains RRCDNet for 200
epochs over 4,500 training spectra at L = 10,000 with Adam (LR 3e-4), batch 32, MSE loss, shuffled
batches, keeping the checkpoint of the best validation loss (RRCDNet/train.py:117-121, :150-200;
data from 数据集产生.py:67-84: 5,000 train/val spectra, 90 % train).  This script does the same on
the GPU for ``--steps`` Adam steps (default 12,000 = 85 epochs of 141 steps) on a pool drawn by
``oracle.refgen`` (the bit-exact restatement of the reference generator) with seeds no other
fixture, tuning run or test uses, and validates on the remaining 10 % every ``--val-every`` steps.
The module trained is ``raman_mi355x.RRCDNet`` in training mode, i.e. its eager path: the reference
forward on the reference submodule tree (models.py), so its state_dict IS a reference checkpoint.

It is resumable (``--out``/ckpt.pt holds model, optimizer, RNG and pool seed), prints a progress line
at least every minute, and writes ``--out``/best.npz (state_dict of the best validation loss as
float32 arrays, plus train_steps / val_loss / train_loss).  make_golden.py --heldout2 then computes
the reference's own outputs for it on the build host.
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
for p in (ROOT, os.path.join(ROOT, "data-simulation-and-noise-reduction-of-distributed-fiber-raman-intensity_amd")):
    sys.path.insert(0, p)

POOL_SEED = 61_803          # training/validation pool: 5,000 spectra, as the reference's train_val.npz
TORCH_SEED = 2_718


def make_pool(n, L):
    from oracle.refgen import generate_signals
    rng = np.random.RandomState(POOL_SEED)
    clean, noisy, _, _ = generate_signals(n, signal_length=L, rng=rng)
    return clean.astype(np.float32), noisy.astype(np.float32)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--steps", type=int, default=12000)
    ap.add_argument("--max-seconds", type=float, default=1000.0)
    ap.add_argument("--val-every", type=int, default=1000)
    ap.add_argument("--pool", type=int, default=5000)
    ap.add_argument("--L", type=int, default=10000)
    ap.add_argument("--device", default="cuda")
    args = ap.parse_args()
    os.makedirs(args.out, exist_ok=True)
    import raman_mi355x as R

    t0 = time.time()
    clean, noisy = make_pool(args.pool, args.L)
    ntr = int(args.pool * 0.9)
    print(f"pool {args.pool} x {args.L} in {time.time() - t0:.0f}s", flush=True)
    dev = torch.device(args.device)
    xc = torch.from_numpy(clean).unsqueeze(1).to(dev)
    xn = torch.from_numpy(noisy).unsqueeze(1).to(dev)

    torch.manual_seed(TORCH_SEED)
    model = R.RRCDNet().to(dev)
    opt = torch.optim.Adam(model.parameters(), lr=3e-4)
    step, best, best_sd, losses = 0, float("inf"), None, []
    gen = torch.Generator().manual_seed(TORCH_SEED)
    perm, pos = torch.randperm(ntr, generator=gen), 0
    ck = os.path.join(args.out, "ckpt.pt")
    if os.path.exists(ck):
        st = torch.load(ck, map_location=dev, weights_only=True)
        model.load_state_dict(st["model"])
        opt.load_state_dict(st["opt"])
        step, best, losses, pos = st["step"], st["best"], st["losses"], st["pos"]
        perm = st["perm"]
        gen.set_state(st["gen"].cpu())
        perm = perm.cpu()
        best_sd = {k: v.cpu() for k, v in st["best_sd"].items()} if st["best_sd"] is not None else None
        print(f"resumed at step {step}, best val {best:.6f}", flush=True)

    def validate():
        model.eval()
        tot, cnt = 0.0, 0
        with torch.no_grad():
            for i in range(ntr, args.pool, 64):
                y = model.eager_forward(xn[i:i + 64])
                tot += torch.nn.functional.mse_loss(y, xc[i:i + 64], reduction="sum").item()
                cnt += y.numel()
        model.train()
        return tot / cnt

    def save():
        torch.save({"model": model.state_dict(), "opt": opt.state_dict(), "step": step, "best": best,
                    "losses": losses, "pos": pos, "perm": perm, "gen": gen.get_state(), "best_sd": best_sd}, ck)

    model.train()
    t_start, t_print, step0 = time.time(), time.time(), step
    while step < args.steps and time.time() - t0 < args.max_seconds:
        if pos + 32 > ntr:                                 # a new shuffled epoch (DataLoader shuffle=True)
            perm, pos = torch.randperm(ntr, generator=gen), 0
        idx = perm[pos:pos + 32].to(dev)
        pos += 32
        opt.zero_grad()
        loss = torch.nn.functional.mse_loss(model(xn[idx]), xc[idx])
        loss.backward()
        opt.step()
        step += 1
        if step % 50 == 0:
            losses.append(loss.item())
        if step % args.val_every == 0 or step == args.steps:
            v = validate()
            if v < best:
                best = v
                best_sd = {k: t.detach().cpu().clone() for k, t in model.state_dict().items()}
            save()
            print(f"step {step}: val {v:.3e} (best {best:.3e})", flush=True)
        if time.time() - t_print > 30:
            rate = (time.time() - t_start) / max(1, step - step0)
            print(f"step {step}: loss {np.mean(losses[-10:]) if losses else float('nan'):.3e} "
                  f"({rate * 1e3:.1f} ms/step, {time.time() - t0:.0f}s)", flush=True)
            t_print = time.time()
    save()
    if best_sd is not None:
        rec = {f"w::{k}": v.numpy() for k, v in best_sd.items()}
        rec.update(train_steps=np.array(step), val_loss=np.array(best),
                   train_loss=np.array(float(np.mean(losses[-20:])) if losses else np.nan),
                   pool_seed=np.array(POOL_SEED), torch_seed=np.array(TORCH_SEED))
        np.savez(os.path.join(args.out, "best.npz"), **rec)
    print(f"done: {step} steps, best val {best:.4e}, {time.time() - t0:.0f}s", flush=True)


if __name__ == "__main__":
    main()
