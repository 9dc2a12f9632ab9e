"""Headline benchmark: denoised spectra/s of the fused RRCDNet forward on MI355X (BASELINE.json).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--arch RRCDNet] [--dtype f16] [--batch B]

The headline dtype is 'f16', the engine's fastest mode within the north-star 16-bit tolerance
(2e-2 max-abs): on RRCDNet that is RDN_F16MIX -- one v_mfma_f32_16x16x32_f16 per product (the bf16
MFMA rate) on f16 weights and activations with fp32 accumulation on 24 of the 29 64-channel layers,
the last five right-branch layers with the block-scaled e4m3 correction (parity in
profiles/r04/parity_table.md).
The f16 + e4m3-correction mode (f16f8, ~15 significant bits), split bf16 (bf16x3), single-rounding
bf16 ('bf16-unsafe', NOT within 2e-2 on trained RRCDNet) and fp32 (compensated, within 1e-5) are
timed as "variants" in the same line.

One step = one forward of the fused network over a batch of B synthetic spectra per GPU (L = 10000),
generated on-device by the engine's simulator BEFORE the timed region (inputs resident in HBM).
Data-parallel over N GPUs, one process per GPU (torch.distributed.run; `python bench.py --gpus N`
without a launcher starts it itself, before any GPU call): every rank simulates its own
spectrum-index range (index_blocks: headline, pipeline and config-4 blocks disjoint across ranks and
legs), so per-GPU work is fixed as N grows ("weak" scaling); the only collective is the end-of-run
metric all-reduce (outside the timed region), plus the timing barrier/max.  Rank 0 prints ONE JSON
line.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "data-simulation-and-noise-reduction-of-distributed-fiber-raman-intensity_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "denoised spectra/sec (node) RRCDNet bf16/fp32 at 1/2/4/8 GPU; % MFMA peak"
# Dense MFMA peaks, MI355X_MICROARCH.md §Chip-level parameters (spec values)
PEAK_TFLOPS = {"f16": 2500.0, "f16-plain": 2500.0, "bf16-unsafe": 2500.0, "bf16x3": 2500.0, "f16f8": 2500.0, "fp32": 157.3}
# conv layer counts per network: (64->64 convs, stems, heads) — SURVEY.md §2 table
LAYERS = {"DenoiseCNN": (18, 1, 1), "RRCDNet": (29, 2, 2), "DSDN": (32, 1, 1), "PIDN": (30, 1, 1),
          "ADSDN": (32, 1, 1), "APIDN": (30, 1, 1)}
SA_CONVS = {"ADSDN": 17, "APIDN": 15}
# MFMA cycles per product relative to one bf16 MFMA (v_mfma_f32_16x16x32_bf16 = 16 cycles per K=32)
# ('f16' on RRCDNet = RDN_F16MIX: 24 plain layers + 5 corrected at 2 units, bench.mfma_cost)
MFMA_COST = {"f16": 1, "f16-plain": 1, "bf16-unsafe": 1, "bf16x3": 3, "f16f8": 2}


# BASELINE.json configs[i] each network's throughput is quoted on
CONFIG_OF = {"DenoiseCNN": 1, "RRCDNet": 2, "DSDN": 3, "ADSDN": 3, "PIDN": 4, "APIDN": 4}


def mfma_cost(arch, dtype):
    """bf16-MFMA units executed per algorithmic product: RDN_F16MIX (Python 'f16' on RRCDNet) runs the
    layers of its correction mask with the e4m3 correction (2 units) and the rest plain (1)."""
    if dtype == "f16" and arch == "RRCDNet":
        from raman_mi355x import engine
        k = bin(engine.default_correction_mask(arch)).count("1")
        big = LAYERS[arch][0]
        return (big - k + 2 * k) / big
    return MFMA_COST.get(dtype)


def flops_per_spectrum(arch, L):
    """Algorithmic FLOPs: sum over Conv1d layers of 2*Cin*Cout*K*L."""
    big, stems, heads = LAYERS[arch]
    per_pos = big * 2 * 64 * 64 * 3 + stems * 2 * 64 * 3 + heads * 2 * 64 * 3 + SA_CONVS.get(arch, 0) * 2 * 2 * 7
    return per_pos * L


PIPELINE_STEPS = 8          # timed steps per pipeline leg (each leg ~0.5 s at the default batch)


def index_blocks(world, rank, B, steps_pipeline=PIPELINE_STEPS, B4=8192, chunks4=4):
    """Simulator spectrum indices each leg of rank `rank` generates (half-open ranges): the headline
    batch, the pipeline's steps + 1 batches, and the config-4 driver's total (evaluate_synthetic
    shards [first, first + total) over the ranks itself).  Disjoint across legs and ranks."""
    head = (rank * B, (rank + 1) * B)
    p0 = world * B + rank * (steps_pipeline + 1) * B
    pipe = (p0, p0 + (steps_pipeline + 1) * B)
    c4first = world * B + world * (steps_pipeline + 1) * B
    c4total = world * chunks4 * B4
    # the sustained (config 3) window: a block of 2^32 indices per rank far beyond the others
    return {"headline": head, "pipeline": pipe, "config4_first": c4first, "config4_total": c4total,
            "config4_warmup_first": c4first + c4total, "sustained_first": (1 << 40) + rank * (1 << 32)}


def launch_ranks(n, argv):
    """`python bench.py --gpus N` without a launcher: start N ranks under torch.distributed.run
    (127.0.0.1 rendezvous) as a child process and return its exit code.  Called before anything
    touches the GPU (torch.cuda.device_count() does not initialise it on this image)."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + argv
    progress(f"launching {n} ranks: {' '.join(cmd[1:])}")
    return subprocess.call(cmd)


def progress(msg):
    """One line per bench stage on stderr (the JSON line stays alone on stdout)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def _cpu_model_name():
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _reference_inputs(n, L):
    """Spectra of the reference's own generator (oracle.refgen, bit-exact with 数据集产生.py:5-64),
    seeded like config 1's data/test.npz."""
    from oracle.refgen import generate_signals
    state = np.random.get_state()
    np.random.seed(20250410)
    clean, noisy, _, _ = generate_signals(n, signal_length=L)
    np.random.set_state(state)
    return clean, noisy


def _weights(arch):
    """The trained golden state_dict (tests/golden; the reference ships no checkpoint), else random init."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    try:
        from conftest import golden_state_dict, load_golden
        if any(k.startswith("w::") for k in load_golden(arch).files):
            return golden_state_dict(arch, "trained"), "trained golden fixture (tests/golden)"
    except (ImportError, OSError):
        pass
    import raman_mi355x as R
    torch.manual_seed(0)
    return R.MODELS[arch]().state_dict(), "random init"


def _cpu_quota():
    """CPUs of this process's cgroup CPU quota (cgroup v2 cpu.max / v1 cfs), None if unlimited."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, p = fh.read().split()[:2]
        return None if q == "max" else max(1, int(int(q) // int(p)))
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as fh:
            q = int(fh.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as fh:
            p = int(fh.read())
        return None if q <= 0 else max(1, q // p)
    except (OSError, ValueError):
        return None


def cpu_baseline(arch, L, seconds):
    """The reference CPU path, restated (oracle.models: the reference's fp32 PyTorch-CPU ops, pinned to
    the reference by the golden fixtures), in the evaulate.py:29-37 loop shape on the box's host cores:
    batch-1 forwards without metrics (`value`), batch-1 with the per-spectrum metrics of
    evaulate.py:34-37 (oracle.metrics: MSE, skimage-0.18.3 SSIM, Smoothness, Peak2Peak), and a
    batched-16 forward loop (BASELINE.md CPU-baseline plan), at torch.set_num_threads(os.cpu_count())
    as BASELINE.md prescribes; the batch-1 loop also at 16 threads (the GPU box's CPU share: its
    os.cpu_count() reports the whole host).  Bounded: ~`seconds` per variant."""
    from oracle.metrics import per_spectrum
    from oracle.models import forward as oracle_forward
    ncpu = os.cpu_count() or 1
    quota = _cpu_quota()
    # torch.set_num_threads(os.cpu_count()) as BASELINE.md prescribes, capped at the CPUs this process
    # may actually run on: the GPU box reports the whole host (256) but grants a 16-CPU quota, and 256
    # threads on 16 CPUs ran one batch-1 RRCDNet forward in 22 s (round 3)
    threads = min(ncpu, quota) if quota else ncpu
    sd, wsrc = _weights(arch)
    clean, noisy = _reference_inputs(64, L)
    xs = [torch.tensor(v, dtype=torch.float32).view(1, 1, -1) for v in noisy]

    def loop(body):
        body(0)                                              # warm-up
        n, t0 = 0, time.perf_counter()
        while True:
            body(n)
            n += 1
            el = time.perf_counter() - t0
            if el >= seconds and n >= 3:
                return n, el

    torch.set_num_threads(threads)
    progress(f"cpu baseline: batch-1 loop at {threads} threads")
    n1, e1 = loop(lambda i: oracle_forward(arch, sd, xs[i % len(xs)]))
    n2, e2 = loop(lambda i: per_spectrum(oracle_forward(arch, sd, xs[i % len(xs)]).view(1, -1).numpy(),
                                         clean[i % len(xs)][None]))
    progress("cpu baseline: batched-16 loop")
    xb = torch.tensor(noisy[:16], dtype=torch.float32).unsqueeze(1)
    n3, e3 = loop(lambda i: oracle_forward(arch, sd, xb))
    try:
        avail = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        avail = None
    return {"value": n1 / e1, "unit": "spectra/s", "cores": threads, "kind": "port",
            "sample": f"{n1} batch-1 fp32 {arch} forwards at L={L} ({e1:.1f} s), evaulate.py:29-32 loop shape, "
                      f"oracle.models (the reference's ops) at torch.set_num_threads({threads}) = min(os.cpu_count() "
                      f"= {ncpu}, cgroup CPU quota = {quota}); weights: {wsrc}; inputs: the reference generator "
                      "(oracle.refgen, seed 20250410)",
            "with_metrics_spectra_per_s": n2 / e2,
            "batched16_spectra_per_s": 16 * n3 / e3,
            "note": "batched-16 runs the oracle's functional forward on a (16,1,L) tensor: PyTorch-CPU's (oneDNN) "
                    "batch-16 Conv1d is slower per spectrum than batch 1 at L = 10,000 on these hosts (3.5x on the "
                    "build container at 8 threads); it is the reference's own batched path (RRCDNet/train.py:166)",
            "host": {"cpu_model": _cpu_model_name(), "os_cpu_count": ncpu, "cgroup_cpu_quota": quota,
                     "sched_affinity_cpus": avail, "torch": torch.__version__}}


def batch1_latency(model, code, arch, L, dev, n=200):
    """The reference's evaluate loop shape through the drop-in module (evaulate.py:29-32): one spectrum
    per forward.  `host_loop`: host array -> tensor -> device -> forward -> .cpu() per spectrum;
    `device_resident`: input already on the GPU, forward + sync per spectrum."""
    _, noisy = _reference_inputs(8, L)
    with torch.no_grad():
        for _ in range(3):
            model(torch.tensor(noisy[0], dtype=torch.float32).view(1, 1, -1).to(dev)).cpu()
        t0 = time.perf_counter()
        for i in range(n):
            model(torch.tensor(noisy[i % 8], dtype=torch.float32).unsqueeze(0).unsqueeze(0).to(dev)).cpu().squeeze().numpy()
        host = (time.perf_counter() - t0) / n
        xd = torch.tensor(noisy[0], dtype=torch.float32).view(1, 1, -1).to(dev)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(n):
            model(xd)
            torch.cuda.synchronize()
        dres = (time.perf_counter() - t0) / n
    return {"host_loop_ms_per_spectrum": host * 1e3, "host_loop_spectra_per_s": 1.0 / host,
            "device_resident_ms_per_spectrum": dres * 1e3, "spectra": n, "L": L, "engine_dtype_code": code,
            "note": "module forward at batch 1 (evaulate.py:29-32); per call: pack-cache key check, one fused launch"}


def traffic_per_spectrum(arch, dtype):
    """HBM bytes per spectrum of the dominant kernel from the committed rocprofv3 PMC summary
    (FETCH_SIZE x 2 + WRITE_SIZE, the gfx950 correction of MI355X_MICROARCH.md §HBM), or None."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        with open(path) as fh:
            rec = json.load(fh).get(f"{arch}/{dtype}")
        return (rec["bytes_per_spectrum"], rec["source"]) if rec else (None, None)
    except (OSError, ValueError, KeyError):
        return None, None


def time_forward(engine, arch, dtype, packed, x, y, steps, warmup, stream):
    for _ in range(warmup):
        engine.forward(arch, dtype, packed, x, out=y, check=False)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(steps):
        engine.forward(arch, dtype, packed, x, out=y, check=False)
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / steps


def time_pipeline(engine, arch, dtype, packed, seed, first, B, L, steps, stream, dev):
    """SURVEY.md §8d configs 3-4 end to end, reported beside `value` (never as it): per step the
    device simulator writes B fresh spectra (indices first + i*B, i = 0..steps: the caller gives each
    rank a disjoint block of (steps + 1) * B indices), the fused forward denoises them and meters them
    into the evaluate sums (evaulate.py:29-39) — no host sync, nothing leaves HBM.  The step is
    simulate -> rdn_forward_metrics (on the walk geometry the forward kernel computes each spectrum's
    metrics after its walk: no second pass over y); also timed: each stage alone and the unfused step
    (simulate -> forward -> metrics kernel) on the same buffers."""
    clean = torch.empty((B, L), dtype=torch.float32, device=dev)
    noisy = torch.empty((B, L), dtype=torch.float32, device=dev)
    y = torch.empty((B, 1, L), dtype=torch.float32, device=dev)
    sums = torch.zeros(5, dtype=torch.float64, device=dev)

    def gen(i):
        engine.generate(B, seed, first_index=first + i * B, signal_length=L, device=dev, out=(clean, noisy))

    def fwd():
        engine.forward(arch, dtype, packed, noisy.view(B, 1, L), out=y, check=False)

    def met():
        engine.metrics(y.view(B, L), clean, sums=sums, per_spectrum=False)

    fused = []

    def fwdmet():
        fused.append(engine.forward_metrics(arch, dtype, packed, noisy.view(B, 1, L), clean, out=y, sums=sums,
                                            check=False)[3])

    def timed(fn):
        fn(0)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for i in range(steps):
            fn(i + 1)
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / steps

    ms_gen = timed(gen)
    ms_fwd = timed(lambda i: fwd())
    ms_met = timed(lambda i: met())
    ms_fm = timed(lambda i: fwdmet())
    ms_unfused = timed(lambda i: (gen(i), fwd(), met()))
    sums.zero_()
    ms_all = timed(lambda i: (gen(i), fwdmet()))
    return {"spectra_per_s_per_gpu": B / (ms_all * 1e-3), "ms_per_step": ms_all, "batch": B, "steps": steps,
            "stage_ms": {"simulate": ms_gen, "forward": ms_fwd, "metrics": ms_met, "forward_metrics": ms_fm},
            "metric_epilogue_fused": all(fused), "unfused_ms_per_step": ms_unfused,
            "spectra_metered": int(sums[4].item()),
            "note": "simulate -> forward with the metric epilogue (rdn_forward_metrics) per step, all on device "
                    "(configs 3-4); unfused_ms_per_step: simulate -> forward -> separate metrics kernel"}


class ClockSampler:
    """Background sampler of the GPU's graphics clock (torch.cuda.clock_rate: amdsmi, MHz) and board
    power (torch.cuda.power_draw) while a leg runs; empty if the query is unavailable on the box."""

    def __init__(self, dev, period=0.25):
        import threading
        self.dev, self.period, self.clk, self.pw = dev, period, [], []
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, daemon=True)

    def _run(self):
        while not self._stop.is_set():
            try:
                self.clk.append(float(torch.cuda.clock_rate(self.dev)))
            except Exception:            # noqa: BLE001 - no amdsmi / no permission: report nothing
                return
            try:
                self.pw.append(float(torch.cuda.power_draw(self.dev)))
            except Exception:            # noqa: BLE001
                pass
            self._stop.wait(self.period)

    def __enter__(self):
        self._t.start()
        return self

    def __exit__(self, *exc):
        self._stop.set()
        self._t.join(timeout=5)

    def summary(self):
        def st(v):
            v = [a for a in v if a > 0]
            return {"mean": sum(v) / len(v), "min": min(v), "max": max(v), "samples": len(v)} if v else None
        return {"gfx_clock_mhz": st(self.clk), "power_draw": st(self.pw)}


def time_sustained(engine, arch, dtype, packed, seed, first, B, L, seconds, min_spectra, stream, dev, fl_per_spectrum,
                   peak):
    """the on-device simulator feeding the fused forward for >= `seconds` and
    >= `min_spectra` distinct spectra (indices first + i*B), reported beside the short headline window:
    spectra/s over the whole window (simulate + forward), the forward kernels' own time and roofline
    fraction (HIP events around every forward), per-window rates (drift), and the graphics clock."""
    clean = torch.empty((B, L), dtype=torch.float32, device=dev)
    noisy = torch.empty((B, L), dtype=torch.float32, device=dev)
    y = torch.empty((B, 1, L), dtype=torch.float32, device=dev)
    steps = max(1, -(-min_spectra // B))
    ev = lambda: torch.cuda.Event(enable_timing=True)   # noqa: E731
    # every step's outputs count only if finite: the workspace's status word (a saturated e4m3 tile) is
    # checked once after the window, and a device flag ANDs in each step's finiteness (no host sync)
    ws = engine.Workspace(arch, dtype, B, L, dev) if engine.needs_workspace(arch, engine.resolve_dtype(arch, dtype)) \
        else None
    finite = torch.ones((), dtype=torch.bool, device=dev)
    # one untimed step (pack / launch caches), then the window
    engine.generate(B, seed, first_index=first, signal_length=L, device=dev, out=(clean, noisy))
    engine.forward(arch, dtype, packed, noisy.view(B, 1, L), out=y, check=False)
    torch.cuda.synchronize()
    marks, fwd = [], []
    t0 = time.perf_counter()
    with ClockSampler(dev) as clk:
        i = 0
        while True:
            engine.generate(B, seed, first_index=first + (i + 1) * B, signal_length=L, device=dev, out=(clean, noisy))
            a, b = ev(), ev()
            a.record(stream)
            engine.forward(arch, dtype, packed, noisy.view(B, 1, L), out=y, check=False, workspace=ws)
            b.record(stream)
            fwd.append((a, b))
            torch.logical_and(finite, torch.isfinite(y).all(), out=finite)
            i += 1
            if i % 16 == 0:
                torch.cuda.synchronize()
                marks.append((i, time.perf_counter()))
                if i >= steps and marks[-1][1] - t0 >= seconds:
                    break
        torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if ws is not None:
        ws.check()                               # raises on a saturated tile in any step of the window
    if not bool(finite):
        raise RuntimeError("non-finite outputs in the sustained window")
    ms_fwd = [a.elapsed_time(b) for a, b in fwd]
    kms = sum(ms_fwd) / len(ms_fwd)
    n_win = 4
    q = max(1, len(ms_fwd) // n_win)
    win = [sum(ms_fwd[k * q:(k + 1) * q]) / q for k in range(n_win)]
    return {"spectra": i * B, "seconds": el, "spectra_per_s": i * B / el, "steps": i, "batch": B,
            "forward_kernel_ms": kms, "forward_spectra_per_s": B / (kms * 1e-3),
            "roofline_frac": fl_per_spectrum * B / (kms * 1e-3) / 1e12 / peak,
            "forward_kernel_ms_by_quarter": win, "first_index": first,
            **clk.summary(),
            "note": "config 3 steady state: per step the device simulator writes B fresh spectra and the fused forward "
                    "denoises them; forward_kernel_ms from HIP events around each forward on the launch stream"}


def _model(R, arch, dtype, dev, trained=True):
    """Module of `arch` on `dev` with the trained golden fixture weights (or random init)."""
    torch.manual_seed(1234)
    m = R.MODELS[arch]()
    src = "random init"
    if trained:
        sd, src = _weights(arch)
        m.load_state_dict(sd, strict=True)
    return m.to(dev).eval().set_engine_dtype(dtype), src


def config_keys(R, engine, args, dev, stream, world, rank, blocks):
    """BASELINE.json configs 2, 4 and 5 as extra keys of the bench line (each labelled with its own
    configs[i]), on the trained golden fixture weights.  Config 4 runs at every world size (the
    data-parallel driver: rank r owns [r*N/W, (r+1)*N/W), exact metric sums all-reduced, so its means
    are identical for any W); configs 2 and 5 are single-GPU configurations (rank 0 of a 1-GPU run)."""
    from raman_mi355x.evaluate import evaluate_synthetic
    out = {}
    L = args.L
    # config 4: RRCDNet + DSDN/ADSDN data-parallel, fixed total N (evaluate_synthetic)
    B4 = args.config4_batch
    total = world * args.config4_chunks * B4
    models = {a: _model(R, a, args.dtype, dev)[0] for a in args.config4_archs.split(",")}
    assert total == blocks["config4_total"]
    evaluate_synthetic({a: m for a, m in models.items()}, world * 2, seed=args.seed, signal_length=L,
                       batch_size=2, device=dev, first_index=blocks["config4_warmup_first"])  # warm-up (pack, launch)
    progress(f"config 4: {total} spectra x {len(models)} networks")
    res = evaluate_synthetic(models, total, seed=args.seed, signal_length=L, batch_size=B4, device=dev,
                             first_index=blocks["config4_first"])
    cfg4 = {"config": "BASELINE.json configs[3]", "total_spectra": total, "batch_per_gpu": B4,
            "first_index": blocks["config4_first"],
            "dtype": args.dtype, "signal_length": L, "n_gpus": world,
            "note": "evaluate_synthetic: per chunk on-device simulate -> fused forward -> exact metric sums; rank r "
                    "owns spectrum indices [r*N/W, (r+1)*N/W); the accumulators are all-reduced once (means "
                    "identical for any W); CBAM hand-off status checked once per network"}
    for a, r in res.items():
        sps = r["spectra_per_s"]
        cfg4[a] = {"spectra_per_s": sps, "seconds": r["seconds"], "means": r["means"], "engine_dtype_code": models[a].engine_code,
                   "roofline_frac_per_gpu": flops_per_spectrum(a, L) * sps / world / 1e12 / PEAK_TFLOPS[args.dtype]}
    out["config4"] = cfg4
    if world > 1 or rank != 0:
        return out
    # config 2: 1DCNN fp32 on config2_n on-device spectra
    progress(f"config 2: DenoiseCNN fp32, {args.config2_n} spectra")
    m2, src = _model(R, "DenoiseCNN", "fp32", dev)
    evaluate_synthetic({"DenoiseCNN": m2}, 4, seed=args.seed, signal_length=L, batch_size=4, device=dev)
    r2 = evaluate_synthetic({"DenoiseCNN": m2}, args.config2_n, seed=args.seed, signal_length=L,
                            batch_size=args.config2_batch, device=dev)["DenoiseCNN"]
    x2 = engine.generate(args.config2_batch, args.seed, signal_length=L, device=dev)[1].view(-1, 1, L)
    ms2 = time_forward(engine, "DenoiseCNN", m2.engine_code, m2.packed_weights(dev), x2, torch.empty_like(x2), 3, 1, stream)
    del x2
    out["config2"] = {"config": "BASELINE.json configs[1]", "arch": "DenoiseCNN", "dtype": "fp32",
                      "spectra": args.config2_n, "signal_length": L, "weights": src,
                      "spectra_per_s": r2["spectra_per_s"], "seconds": r2["seconds"], "means": r2["means"],
                      "forward_kernel_ms": ms2, "forward_batch": args.config2_batch,
                      "roofline_frac": flops_per_spectrum("DenoiseCNN", L) * args.config2_batch / (ms2 * 1e-3) / 1e12
                      / PEAK_TFLOPS["fp32"],
                      "note": "end to end (simulate -> forward -> metrics) over all spectra; roofline_frac from the "
                              "forward kernel alone (HIP events)"}
    # config 5: PIDN / APIDN at L = 16384, 'f16' and fp32, plus the f16-vs-fp32 gap on the same inputs
    progress("config 5: PIDN / APIDN at L = 16384")
    L5 = 16384
    cfg5 = {"config": "BASELINE.json configs[4]", "signal_length": L5}
    for a in ("PIDN", "APIDN"):
        nb = {"PIDN": 2500, "APIDN": 1250}[a]
        x5 = engine.generate(nb, args.seed, first_index=10 ** 9, signal_length=L5, device=dev)[1].view(nb, 1, L5)
        y5 = torch.empty_like(x5)
        rec = {}
        outs = {}
        for dt, n in (("f16", nb), ("fp32", nb // 4)):
            m5, src = _model(R, a, dt, dev)
            pk = m5.packed_weights(dev)
            ms = time_forward(engine, a, m5.engine_code, pk, x5[:n], y5[:n], 3, 1, stream)
            ws = engine.Workspace(a, m5.engine_code, 64, L5, dev) if a in engine.CBAM_ARCHS else None
            outs[dt] = engine.forward(a, m5.engine_code, pk, x5[:64], check=True, workspace=ws).cpu()
            rec[dt] = {"spectra_per_s": n / (ms * 1e-3), "kernel_ms": ms, "batch": n,
                       "roofline_frac": flops_per_spectrum(a, L5) * n / (ms * 1e-3) / 1e12 / PEAK_TFLOPS[dt]}
        rec["f16_vs_fp32_max_abs_64_spectra"] = float((outs["f16"] - outs["fp32"]).abs().max())
        rec["weights"] = src
        cfg5[a] = rec
        del x5, y5
    out["config5"] = cfg5
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--arch", default="RRCDNet")
    ap.add_argument("--dtype", default="f16", choices=["f16", "f16-plain", "bf16-unsafe", "bf16x3", "f16f8", "fp32"])
    ap.add_argument("--batch", type=int, default=8192, help="spectra per GPU per step")
    ap.add_argument("--L", type=int, default=10000)
    ap.add_argument("--seed", type=int, default=20250410)
    ap.add_argument("--cpu-seconds", type=float, default=6.0, help="per CPU-baseline variant (3 variants)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-variants", action="store_true", help="skip timing the other engine dtypes")
    ap.add_argument("--no-batch1", action="store_true", help="skip the batch-1 evaluate-loop latency")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="skip timing the simulate -> forward -> metrics pipeline (SURVEY.md §8d configs 3-4)")
    ap.add_argument("--no-configs", action="store_true", help="skip the configs 2/4/5 keys")
    ap.add_argument("--sustained-seconds", type=float, default=10.0,
                    help="config 3 steady-state window (also >= --sustained-spectra); 0 skips it")
    ap.add_argument("--sustained-spectra", type=int, default=2_000_000)
    ap.add_argument("--config2-n", type=int, default=1_000_000, help="config 2 spectra (1DCNN fp32)")
    ap.add_argument("--config2-batch", type=int, default=65536)
    ap.add_argument("--config4-batch", type=int, default=8192)
    ap.add_argument("--config4-chunks", type=int, default=4, help="config 4 chunks per rank")
    ap.add_argument("--config4-archs", default="RRCDNet,DSDN,ADSDN",
                    help="(ranks sharing one GPU under gloo must leave out the CBAM networks: their team "
                         "kernel assumes the whole device)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (RCCL over xGMI, one rank per GPU); gloo rehearses the N>1 path with ranks "
                         "sharing the visible GPUs (collectives staged through host memory)")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        if args.dist_backend == "nccl" and args.gpus > torch.cuda.device_count():
            raise SystemExit(f"--gpus {args.gpus}: only {torch.cuda.device_count()} GPU(s) visible; one RCCL rank "
                             "per GPU (rehearse more ranks with --dist-backend gloo)")
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # launched by torch.distributed.run (WORLD_SIZE set, even at 1): a process group over RCCL ("nccl")
    # or gloo; a plain `python bench.py` runs without one
    distributed = "WORLD_SIZE" in os.environ
    gloo = distributed and args.dist_backend == "gloo"
    if gloo:
        local = local % torch.cuda.device_count()
    if distributed:
        torch.cuda.set_device(local)
        if gloo:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    def all_reduce(t, op=dist.ReduceOp.SUM):
        if gloo:                                  # gloo reduces host tensors
            h = t.cpu()
            dist.all_reduce(h, op=op)
            t.copy_(h)
        else:
            dist.all_reduce(t, op=op)

    import raman_mi355x as R
    from raman_mi355x import engine

    torch.manual_seed(1234)                       # random-init weights of the architecture
    model = R.MODELS[args.arch]().to(dev).eval().set_engine_dtype(args.dtype)
    B, L = args.batch, args.L
    blocks = index_blocks(world, rank, B, PIPELINE_STEPS, args.config4_batch, args.config4_chunks)
    clean, noisy, _, _ = engine.generate(B, args.seed, first_index=blocks["headline"][0], signal_length=L, device=dev)
    x = noisy.view(B, 1, L)
    y = torch.empty_like(x)
    packed = model.packed_weights(dev)
    code = model.engine_code                      # the ABI dtype the module resolved args.dtype to
    stream = torch.cuda.current_stream(dev)

    def step():
        engine.forward(args.arch, code, packed, x, out=y, check=False)

    progress(f"headline: {args.arch} {args.dtype} batch {B}, {args.warmup} + {args.steps} steps")
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kernel_ms = ev0.elapsed_time(ev1) / args.steps      # one fused kernel launch per step
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if distributed:
        all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())

    # the timed launches ran unchecked (check=False); a failed CBAM hand-off would show as NaN here
    if not bool(torch.isfinite(y).all()):
        raise RuntimeError("non-finite outputs in the timed forward")
    # evaluation metrics of the last step, all-reduced across ranks (RCCL over xGMI) — untimed
    _, sums = engine.metrics(y.view(B, L), clean)
    if distributed:
        all_reduce(sums)
    sums = sums.cpu().tolist()

    variants = {}
    if not args.no_variants:
        progress("variants")
        for dt in ("f16", "f16-plain", "f16f8", "bf16x3", "bf16-unsafe", "fp32"):
            if dt == args.dtype:
                continue
            nb = B if dt != "fp32" else max(1, B // 4)
            pk = model.set_engine_dtype(dt).packed_weights(dev)
            ms = time_forward(engine, args.arch, model.engine_code, pk, x[:nb], y[:nb], 3, 1, stream)
            variants[dt] = {"spectra_per_s_per_gpu": nb / (ms * 1e-3), "kernel_ms": ms, "batch": nb,
                            "roofline_frac": flops_per_spectrum(args.arch, L) * nb / (ms * 1e-3) / 1e12 / PEAK_TFLOPS[dt]}
        model.set_engine_dtype(args.dtype)

    # the headline kernel on the trained golden fixture weights (the clock the chip holds depends on
    # the operands: MI355X_MICROARCH.md DVFS give-back), beside the random-init `value`
    trained = None
    if not args.no_variants:
        mt, tsrc = _model(R, args.arch, args.dtype, dev)
        ms = time_forward(engine, args.arch, mt.engine_code, mt.packed_weights(dev), x, y, max(3, args.steps // 4), 1, stream)
        trained = {"spectra_per_s_per_gpu": B / (ms * 1e-3), "kernel_ms": ms, "batch": B, "weights": tsrc,
                   "roofline_frac": flops_per_spectrum(args.arch, L) * B / (ms * 1e-3) / 1e12 / PEAK_TFLOPS[args.dtype]}
        del mt

    batch1 = None
    if not args.no_batch1 and rank == 0:
        progress("batch-1 latency")
        batch1 = batch1_latency(model, code, args.arch, L, dev)

    pipeline = None
    if not args.no_pipeline:
        progress("pipeline")
        # each rank's pipeline block of (PIPELINE_STEPS + 1)*B indices after every rank's headline batch
        pipeline = time_pipeline(engine, args.arch, code, packed, args.seed, blocks["pipeline"][0], B, L,
                                 PIPELINE_STEPS, stream, dev)

    sustained = None
    if args.sustained_seconds > 0:
        progress(f"sustained: >= {args.sustained_seconds:g} s and >= {args.sustained_spectra} spectra")
        sustained = time_sustained(engine, args.arch, code, packed, args.seed, blocks["sustained_first"], B, L,
                                   args.sustained_seconds, args.sustained_spectra, stream, dev,
                                   flops_per_spectrum(args.arch, L), PEAK_TFLOPS[args.dtype])

    configs = None
    if not args.no_configs:
        configs = config_keys(R, engine, args, dev, stream, world, rank, blocks)

    if rank == 0:
        total = world * B * args.steps
        fl = flops_per_spectrum(args.arch, L) * B              # per launch
        achieved = fl / (kernel_ms * 1e-3) / 1e12
        peak = PEAK_TFLOPS[args.dtype]
        tps, tsrc = traffic_per_spectrum(args.arch, args.dtype)
        rec = {
            "metric": METRIC, "value": total / elapsed, "unit": "spectra/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
            "data": "synthetic (on-device simulator, 数据集产生.py contract; random-init weights)",
            "config": {"workload": f"{args.arch} {args.dtype} fused forward, on-device simulator inputs "
                                   f"(BASELINE.json configs[{CONFIG_OF[args.arch]}])", "engine_dtype_code": code,
                       "arch": args.arch, "signal_length": L, "batch_per_gpu": B, "global_batch": B * world,
                       "parallelism": f"dp{world}", **({"dist_backend": "gloo (rehearsal)"} if gloo else {})},
            "roofline": {"bound": "mfma", "achieved": achieved, "peak": peak, "unit": "TFLOP/s",
                         "frac": achieved / peak, "traffic": tps * B if tps else None,
                         "traffic_source": tsrc, "algorithmic_bytes": 8 * L * B,
                         "kernel_ms": kernel_ms, "flops_per_launch": fl,
                         "mfma_cost_per_product_bf16_units": mfma_cost(args.arch, args.dtype),
                         "executed_bf16_equiv_tflops": (achieved * mfma_cost(args.arch, args.dtype)
                                                        if mfma_cost(args.arch, args.dtype) else None)},
            "variants": variants,
            "trained_weights": trained,
            "pipeline": pipeline,
            "sustained": sustained,
            "configs": configs,
            "batch1": batch1,
            "metrics_mean": {k: sums[i] / sums[4] for i, k in enumerate(["MSE", "SSIM", "Smoothness", "Peak2Peak"])},
        }
        if world == 1 and not args.no_cpu_baseline:
            rec["cpu_baseline"] = cpu_baseline(args.arch, L, args.cpu_seconds)
        print(json.dumps(rec), flush=True)
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
