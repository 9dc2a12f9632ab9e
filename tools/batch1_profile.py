"""Where the batch-1 call's time goes (the reference's evaulate.py:29-32 loop shape; diagnostic).

Device-resident RRCDNet 'f16' at L = 10,000, one spectrum per call:
  module   model(x) + torch.cuda.synchronize()          (what bench.py batch1 times)
  engine   engine.forward(..., check=False) + synchronize (no status read, no pack-cache check)
  raw      the ctypes rdn_forward call + synchronize     (no Python argument handling)
  kernel   HIP events around 200 back-to-back launches
and a cProfile of the module path (top entries by own time).

    python tools/batch1_profile.py
"""
import cProfile
import ctypes
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "data-simulation-and-noise-reduction-of-distributed-fiber-raman-intensity_amd"))
sys.path.insert(0, ROOT)


def main():
    import torch
    import raman_mi355x as R
    from raman_mi355x import _lib, engine
    from bench import _reference_inputs
    dev = torch.device("cuda")
    arch, n = os.environ.get("B1_ARCH", "RRCDNet"), 400
    m = R.MODELS[arch]().to(dev).eval().set_engine_dtype(os.environ.get("B1_DTYPE", "f16"))
    _, noisy = _reference_inputs(2, 10000)
    x = torch.tensor(noisy[0], dtype=torch.float32).view(1, 1, -1).to(dev)
    packed, code = m.packed_weights(dev), m.engine_code
    ws = m._workspace(x)
    y = torch.empty_like(x)
    lib = _lib.lib()
    sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    args = (engine.ARCH_ID[arch], code, ctypes.c_void_p(packed.data_ptr()), ctypes.c_void_p(x.data_ptr()),
            ctypes.c_void_p(y.data_ptr()), 1, 10000, ws.ptr if ws is not None else None, ws.bytes if ws is not None else 0, sp)

    def per_call(fn):
        with torch.no_grad():
            for _ in range(20):
                fn()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(n):
                fn()
            return (time.perf_counter() - t0) / n * 1e3

    def module():
        m(x)
        torch.cuda.synchronize()

    def eng():
        engine.forward(arch, code, packed, x, out=y, check=False, workspace=ws)
        torch.cuda.synchronize()

    def raw():
        lib.rdn_forward(*args)
        torch.cuda.synchronize()

    res = {"module": per_call(module), "engine": per_call(eng), "raw": per_call(raw)}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        lib.rdn_forward(*args)
    e1.record()
    torch.cuda.synchronize()
    res["kernel_back_to_back"] = e0.elapsed_time(e1) / n
    print(" ".join(f"{k} {v:.4f} ms" for k, v in res.items()), flush=True)
    pr = cProfile.Profile()
    with torch.no_grad():
        pr.enable()
        for _ in range(n):
            m(x)
            torch.cuda.synchronize()
        pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(18)


if __name__ == "__main__":
    main()
