"""BASELINE.json config 1 end to end: 1DCNN evaluate.py on data/test.npz (GPU box).

    python tools/config1_eval.py [--n 1000] [--arch DenoiseCNN] [--dtype fp32] [--out profiles/r02/config1.json]

1. Regenerates the reference's ``data/test.npz`` (np.random.seed(20250410), generate_signals(1000):
   oracle.refgen, bit-exact with the reference generator) in its on-disk format
   (raman_mi355x.dataset, 数据集产生.py:67-79).
2. Saves the trained golden state_dict as a checkpoint and loads it the way */evaulate.py:65-66 does
   (strict, torch.load weights_only).  The reference ships no checkpoint; these are the fixture's
   briefly trained weights (tests/golden/make_golden.py).
3. Evaluates it three ways and compares the four means:
   * reference CPU path: the reference's ops on the CPU (oracle.models, fp32) in evaulate.py's batch-1
     loop + the reference metric functions and skimage-0.18.3 SSIM (oracle.metrics);
   * engine, the reference's batch-1 loop through the drop-in module (host round trip per spectrum);
   * engine, batched device evaluate (raman_mi355x.evaluate, fp64 device metrics) + metrics.txt.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "data-simulation-and-noise-reduction-of-distributed-fiber-raman-intensity_amd"))
sys.path.insert(0, ROOT)

from conftest import golden_state_dict  # noqa: E402

KEYS = ("MSE", "SSIM", "Smoothness", "Peak2Peak")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1000)
    ap.add_argument("--arch", default="DenoiseCNN")
    ap.add_argument("--dtype", default="fp32")
    ap.add_argument("--cpu-n", type=int, default=None, help="spectra for the CPU path (default: all)")
    ap.add_argument("--workdir", default=os.path.join(os.environ.get("TMPDIR", "/tmp"), "rdn_config1"))
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    import raman_mi355x as R
    from oracle.metrics import per_spectrum
    from oracle.models import forward as oracle_forward
    from oracle.refgen import generate_signals
    from raman_mi355x.dataset import load_dataset, save_dataset
    from raman_mi355x.evaluate import evaluate, write_metrics

    os.makedirs(os.path.join(args.workdir, "data"), exist_ok=True)
    t0 = time.perf_counter()
    np.random.seed(20250410)
    c, x, s, sd = generate_signals(args.n)
    path = os.path.join(args.workdir, "data", "test.npz")
    save_dataset(path, c, x, s, sd)
    t_gen = time.perf_counter() - t0
    d = load_dataset(path)
    noisy, clean = d["noisy_signals"], d["clean_signals"]

    ckpt = os.path.join(args.workdir, f"{args.arch}_best.pth")
    torch.save(golden_state_dict(args.arch, "trained"), ckpt)
    m = R.MODELS[args.arch]().cuda()
    m.load_state_dict(torch.load(ckpt, map_location="cuda", weights_only=True))
    m = m.eval().set_engine_dtype(args.dtype)

    rec = {"config": "BASELINE.json configs[0]: 1DCNN evaluate.py on data/test.npz", "n": args.n,
           "arch": args.arch, "engine_dtype": args.dtype, "dataset_seconds": t_gen}

    # engine, batched device evaluate
    evaluate(m, noisy[:8], clean[:8])                       # warm-up (pack, first launch)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    got = evaluate(m, noisy, clean)
    torch.cuda.synchronize()
    t_b = time.perf_counter() - t0
    mdir = write_metrics(got, root=os.path.join(args.workdir, "eval_results"))
    rec["engine_batched"] = {"means": got, "seconds": t_b, "spectra_per_s": args.n / t_b,
                             "metrics_txt": open(os.path.join(mdir, "metrics.txt")).read()}

    # engine, the reference's batch-1 loop (evaulate.py:29-37): host round trip + host metrics
    t0 = time.perf_counter()
    y1 = []
    with torch.no_grad():
        for xs in noisy:
            inp = torch.tensor(xs, dtype=torch.float32).unsqueeze(0).unsqueeze(0).cuda()
            y1.append(m(inp).cpu().squeeze().numpy())
    t_fwd = time.perf_counter() - t0
    y1 = np.stack(y1)
    p1 = per_spectrum(y1, clean)
    t_1 = time.perf_counter() - t0
    rec["engine_batch1_loop"] = {"means": dict(zip(KEYS, p1.mean(axis=0).tolist())), "seconds": t_1,
                                 "forward_only_seconds": t_fwd, "spectra_per_s": args.n / t_1,
                                 "forward_spectra_per_s": args.n / t_fwd}

    # reference CPU path
    ncpu = args.cpu_n or args.n
    sdict = golden_state_dict(args.arch, "trained")
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    t0 = time.perf_counter()
    yr = []
    for xs in noisy[:ncpu]:
        yr.append(oracle_forward(args.arch, sdict, torch.tensor(xs, dtype=torch.float32).view(1, 1, -1)).view(-1).numpy())
    t_cf = time.perf_counter() - t0
    yr = np.stack(yr)
    pr = per_spectrum(yr, clean[:ncpu])
    t_c = time.perf_counter() - t0
    rec["reference_cpu_path"] = {"means": dict(zip(KEYS, pr.mean(axis=0).tolist())), "n": ncpu, "seconds": t_c,
                                 "spectra_per_s": ncpu / t_c, "forward_spectra_per_s": ncpu / t_cf,
                                 "threads": torch.get_num_threads(), "torch": torch.__version__}
    scale = float(np.abs(yr).max())
    rec["max_rel_output_diff_engine_vs_cpu"] = float(np.abs(y1[:ncpu] - yr).max()) / scale
    rec["max_abs_output_diff_engine_vs_cpu"] = float(np.abs(y1[:ncpu] - yr).max())
    rec["output_max_abs"] = scale
    pe = per_spectrum(y1[:ncpu], clean[:ncpu]).mean(axis=0)
    rec["max_rel_mean_diff_engine_vs_cpu"] = float(np.max(np.abs(pe - pr.mean(axis=0)) / np.abs(pr.mean(axis=0))))
    rec["max_rel_mean_diff_batched_vs_batch1"] = max(abs(got[k] - rec["engine_batch1_loop"]["means"][k]) /
                                                    abs(rec["engine_batch1_loop"]["means"][k]) for k in KEYS)
    text = json.dumps(rec, indent=1)
    print(text)
    if args.out:
        os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
        with open(args.out, "w") as fh:
            fh.write(text + "\n")


if __name__ == "__main__":
    main()
