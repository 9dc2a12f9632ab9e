"""RDN_F16MIX correction-tail sweep on config 1's data (diagnostic, not part of the product).

    python tools/ablate.py build tail3 tail4 tail5      # build container
    python tools/f16mix_tail_eval.py tail3 tail4 tail5  # GPU box

For each tools/ablate.py variant (RDN_F16MIX_TAIL = number of corrected right-branch layers), the
'f16' RRCDNet forward of the 1000 spectra of config 1's data/test.npz (oracle.refgen, seed
20250410, bit-exact with 数据集产生.py) on both tile geometries, with the trained golden fixture
weights and the held-out weights, against the fp32 CPU reference (oracle.models): max-abs error,
the worst spectrum, its output scale, and how many spectra exceed 1.5e-2 / 2e-2.
"""
import ctypes
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "data-simulation-and-noise-reduction-of-distributed-fiber-raman-intensity_amd"))
sys.path.insert(0, ROOT)


def main():
    from conftest import GOLDEN, golden_state_dict
    from oracle.models import forward as oracle_forward
    from oracle.refgen import generate_signals
    from raman_mi355x import _lib, engine
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    np.random.seed(20250410)
    _, noisy, _, _ = generate_signals(1000)
    X = torch.tensor(noisy, dtype=torch.float32)
    h = np.load(os.path.join(GOLDEN, "heldout_RRCDNet.npz"))
    weights = {"fixture": golden_state_dict("RRCDNet", "trained"),
               "heldout": {k[3:]: torch.from_numpy(np.array(h[k])) for k in h.files if k.startswith("w::")}}
    refs = {}
    for wn, sd in weights.items():
        t0 = time.time()
        refs[wn] = torch.cat([oracle_forward("RRCDNet", sd, X[i:i + 50].unsqueeze(1)) for i in range(0, 1000, 50)]).squeeze(1).numpy()
        print(f"oracle {wn}: {time.time() - t0:.1f} s, max|ref| {np.abs(refs[wn]).max():.3f}", flush=True)
    dev = torch.device("cuda")
    xd = X.to(dev)
    names = engine.param_names("RRCDNet")
    for var in sys.argv[1:]:
        lib = ctypes.CDLL(os.path.join(ROOT, "tools", "ablate_build", f"lib_{var}.so"))
        for fn, (args, res) in _lib._SIGNATURES.items():
            if hasattr(lib, fn):
                getattr(lib, fn).argtypes = args
                getattr(lib, fn).restype = res
        for wn, sd in weights.items():
            host = [sd[k].detach().float().contiguous() for k in names]
            ptrs = (ctypes.c_void_p * len(host))(*[t.data_ptr() for t in host])
            numels = (ctypes.c_int64 * len(host))(*[t.numel() for t in host])
            size = ctypes.c_size_t()
            assert lib.rdn_packed_size(1, 5, ctypes.byref(size)) == 0
            blob = torch.empty(size.value, dtype=torch.uint8)
            assert lib.rdn_pack(1, 5, ptrs, numels, len(host), ctypes.c_void_p(blob.data_ptr()), size.value) == 0
            mask = ctypes.c_uint64()
            lib.rdn_get_correction_mask(1, 5, ctypes.c_void_p(blob.data_ptr()), size.value, ctypes.byref(mask))
            packed = blob.to(dev)
            for tiles in ("0", "1"):
                os.environ["RDN_SHORT_TILES"] = tiles
                y = torch.empty_like(xd)
                for i in range(0, 1000, 250):
                    rc = lib.rdn_forward(1, 5, ctypes.c_void_p(packed.data_ptr()), ctypes.c_void_p(xd[i:i + 250].data_ptr()),
                                         ctypes.c_void_p(y[i:i + 250].data_ptr()), 250, 10000, None, 0,
                                         ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
                    assert rc == 0, lib.rdn_last_error()
                torch.cuda.synchronize()
                e = np.abs(y.cpu().numpy() - refs[wn]).max(axis=1)
                i = int(e.argmax())
                print(f"{var} mask {mask.value:#x} {wn:8s} short_tiles={tiles}: max-abs {e.max():.4e} (spectrum {i}, "
                      f"max|ref| {np.abs(refs[wn][i]).max():.2f}), p99 {np.quantile(e, 0.99):.3e}, "
                      f">1.5e-2: {int((e > 1.5e-2).sum())}, >2e-2: {int((e > 2e-2).sum())}", flush=True)


if __name__ == "__main__":
    main()
