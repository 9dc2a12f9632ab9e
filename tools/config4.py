"""BASELINE.json config 4: RRCDNet + DSDN/ADSDN data-parallel evaluation of a fixed total of N
simulator spectra, one process per GPU.

    python tools/config4.py --total 100000000                       # one GPU, all N
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 tools/config4.py --total 100000000

Rank r of W generates spectrum indices [r·N/W, (r+1)·N/W) on its GPU (counter-based simulator:
spectrum i is the same on any rank), denoises each chunk with every network and meters it into an
exact integer accumulator (rdn_metrics_ex); the accumulators are all-reduced once (RCCL over xGMI,
int64 SUM), so the printed means are the same bits for any W.  Prints one JSON line (rank 0):
spectra/s per network (max-over-ranks wall time of its loop) and the four evaulate.py means.
Reference loop replaced: RRCDNet/evaulate.py:25-39; networks DSDN/train.py:101-126,
ADSDN/train.py:150-167, RRCDNet/train.py:72-98.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "data-simulation-and-noise-reduction-of-distributed-fiber-raman-intensity_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--total", type=int, default=1_000_000, help="N: spectra over all ranks")
    ap.add_argument("--archs", default="RRCDNet,DSDN,ADSDN")
    ap.add_argument("--dtype", default="f16")
    ap.add_argument("--batch", type=int, default=8192, help="spectra per chunk per rank")
    ap.add_argument("--L", type=int, default=10000)
    ap.add_argument("--seed", type=int, default=20250410)
    ap.add_argument("--weights", default="trained", choices=["trained", "random"])
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"])
    ap.add_argument("--out", default=None)
    ap.add_argument("--no-fused-metrics", action="store_true",
                    help="meter with the separate metrics kernel (A/B of rdn_forward_metrics' epilogue)")
    args = ap.parse_args()

    distributed = "WORLD_SIZE" in os.environ
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if distributed and args.dist_backend == "gloo":
        local %= torch.cuda.device_count()
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    if distributed:
        if args.dist_backend == "gloo":
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)

    import raman_mi355x as R
    from raman_mi355x.distributed import world
    from raman_mi355x.evaluate import evaluate_synthetic
    rank, W = world()
    models = {}
    for a in args.archs.split(","):
        torch.manual_seed(1234)
        m = R.MODELS[a]()
        if args.weights == "trained":
            from conftest import golden_state_dict
            m.load_state_dict(golden_state_dict(a, "trained"), strict=True)
        models[a] = m.to(dev).eval().set_engine_dtype(args.dtype)
    evaluate_synthetic(models, 2 * W, seed=args.seed, signal_length=args.L, batch_size=2, device=dev)   # warm-up
    res = evaluate_synthetic(models, args.total, seed=args.seed, signal_length=args.L, batch_size=args.batch,
                             device=dev, log_every_s=30.0, fused_metrics=not args.no_fused_metrics)
    if rank == 0:
        rec = {"config": "BASELINE.json configs[3]", "total_spectra": args.total, "n_gpus": W,
               "dist_backend": args.dist_backend if distributed else None, "dtype": args.dtype, "L": args.L,
               "batch_per_rank": args.batch, "weights": args.weights, "fused_metrics": not args.no_fused_metrics,
               "networks": {a: {k: v for k, v in r.items()} for a, r in res.items()}}
        line = json.dumps(rec)
        print(line, flush=True)
        if args.out:
            os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
            with open(args.out, "w") as fh:
                fh.write(line + "\n")
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
