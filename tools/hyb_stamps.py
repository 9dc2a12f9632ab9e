"""Phase costs of the RDN_F16MIX hybrid (diagnostic, not part of the product): the `hybstamps` build of
tools/ablate.py (-DRDN_HYB_STAMPS=1, rrcdnet_hybrid.hpp HybStamps) sums s_memtime deltas per phase over
the full tiles' workgroups into the range workspace.

    python tools/ablate.py build hybstamps     # build container
    python tools/hyb_stamps.py                 # GPU box: 2048 simulator spectra, random-init RRCDNet
"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "data-simulation-and-noise-reduction-of-distributed-fiber-raman-intensity_amd"))
PHASES = ["right stem", "window vote", "right ping-pong layers 0-7", "layers 8, 9 (staged) + tail operands",
          "in-place corrected tail (5)", "right head (MFMA)", "left layer-0 operands + barrier", "left stem",
          "left layers 15-28 (14)", "left head + vote + combine + store"]
PER_LAYER = {2: 8, 4: 5, 8: 14}
# RDN_WALK=1: the RDN_F16MIX walk kernel (rrcdnet_hybrid_walk.hpp), stamps summed over a spectrum's tiles
WALK_PHASES = ["right stem + barrier", "right ping-pong layers 0-8 (9)", "layer 9 staged + planes + tail operands",
               "in-place corrected tail (5)", "right head (MFMA)", "left operands + stem + barriers",
               "left layers 15-28 (14)", "left head", "vote + combine + store + barrier", "-"]
WALK_PER_LAYER = {1: 9, 3: 5, 6: 14}
if os.environ.get("RDN_WALK") == "1":
    PHASES, PER_LAYER = WALK_PHASES, WALK_PER_LAYER


def main():
    import raman_mi355x as R
    from raman_mi355x import _lib, engine
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "ablate_build", f"lib_{sys.argv[1] if len(sys.argv) > 1 else 'hybstamps'}.so"))
    for fn, (args, res) in _lib._SIGNATURES.items():
        if hasattr(lib, fn):
            getattr(lib, fn).argtypes, getattr(lib, fn).restype = args, res
    dev = torch.device("cuda")
    B, L = 2048, 10000
    # no spikes: every spectrum takes the walk (a spiked one would stamp the tiled phases into the sums)
    _, noisy, _, _ = engine.generate(B, 1, signal_length=L, device=dev,
                                     extreme_noise_prob=0.0 if os.environ.get("RDN_WALK") == "1" else 0.05)
    torch.manual_seed(0)
    model = R.RRCDNet()
    names = engine.param_names("RRCDNet")
    sd = model.state_dict()
    host = [sd[k].detach().float().contiguous() for k in names]
    ptrs = (ctypes.c_void_p * len(host))(*[t.data_ptr() for t in host])
    numels = (ctypes.c_int64 * len(host))(*[t.numel() for t in host])
    size = ctypes.c_size_t()
    assert lib.rdn_packed_size(1, 5, ctypes.byref(size)) == 0
    blob = torch.empty(size.value, dtype=torch.uint8)
    assert lib.rdn_pack(1, 5, ptrs, numels, len(host), ctypes.c_void_p(blob.data_ptr()), size.value) == 0
    blob = blob.to(dev)
    y = torch.empty_like(noisy)
    ws = torch.zeros(1024, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream().cuda_stream
    for _ in range(3):                                  # warm-up
        lib.rdn_forward(1, 5, blob.data_ptr(), noisy.data_ptr(), y.data_ptr(), B, L, ws.data_ptr(), 1024, stream)
    torch.cuda.synchronize()
    ws.zero_()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        assert lib.rdn_forward(1, 5, blob.data_ptr(), noisy.data_ptr(), y.data_ptr(), B, L, ws.data_ptr(), 1024, stream) == 0
    e1.record()
    torch.cuda.synchronize()
    w = ws.view(torch.int64).cpu().tolist()
    n = w[1 + len(PHASES)]
    tot = sum(w[1:1 + len(PHASES)])
    wt = int(os.environ.get("RDN_WALK_ROWS_MIX", "576"))     # the walk tile of the build (common.hpp)
    tiles = -(-(L + 28) // wt) if os.environ.get("RDN_WALK") == "1" else 1
    print(f"{e0.elapsed_time(e1) / 5:.2f} ms per forward of {B} spectra; {n} hybrid workgroups stamped; "
          f"{tot / n:.0f} cycles per workgroup ({tiles} tiles each; per tile below)")
    n *= tiles
    for k, name in enumerate(PHASES):
        c = w[1 + k] / n
        extra = f"  ({c / PER_LAYER[k]:.0f} per layer)" if k in PER_LAYER else ""
        print(f"  {name:42s} {c:9.0f} cycles  {100 * w[1 + k] / tot:5.1f} %{extra}")
    if os.environ.get("RDN_WALK") == "1" and len(w) > 72 and w[36]:
        # every wave's view of the ping-pong ReLU layers (fused16.hpp layer, RDN_HYB_STAMPS)
        print("  ping-pong ReLU layer per wave (cycles per layer): fill (entry -> first MFMA issue) / MFMA "
              "stream (first -> last issue) / drain (-> last store) / barrier wait")
        for wv in range(8):
            q = w[32 + 5 * wv: 37 + 5 * wv]
            nl = q[4]
            print(f"    wave {wv}: " + " / ".join(f"{v / nl:.0f}" for v in q[:4]) + f"  = {sum(q[:4]) / nl:.0f}")
    if os.environ.get("RDN_WALK") == "1" and len(w) > 95 and w[80]:
        # every wave's cycles working / waiting at the corrected walk layers' block barriers
        print("  corrected layer per wave (cycles per layer): working / waiting at block barriers")
        for wv in range(8):
            print(f"    wave {wv}: {w[80 + 2 * wv] / (n * 5):.0f} / {w[81 + 2 * wv] / (n * 5):.0f}")
    if os.environ.get("RDN_WALK") == "1" and any(w[16:22]):
        # wave 0's view of each corrected layer, per block (inplace.hpp conv, RDN_HYB_STAMPS)
        blocks = w[16:22]
        per = n * 5
        print("  corrected layer, wave 0, per block (cycles per layer): " +
              "  ".join(f"{'stores' if k == 5 else 'block ' + str(k)} {v / per:.0f}" for k, v in enumerate(blocks)) +
              f"  = {sum(blocks) / per:.0f}")


if __name__ == "__main__":
    main()
