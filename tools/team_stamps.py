"""Per-phase cycle breakdown of the team-persistent CBAM kernel (diagnostic, not part of the product).

Uses the `stamps` variant of tools/ablate.py (cbam.hip built with -DRDN_TEAM_STAMPS=1): wave 0 of every
workgroup sums s_memtime deltas per phase into the last 16 KiB of the forward workspace.

    python tools/ablate.py build stamps      # build container
    python tools/team_stamps.py [ARCH] [DTYPE] [L]   # GPU box
"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "data-simulation-and-noise-reduction-of-distributed-fiber-raman-intensity_amd"))

PHASES = ["save_identity", "conv1", "conv2", "publish:atomic", "wait", "apply:pointwise", "stem/head/store",
          "loop-other", "publish:rows", "publish:barrier", "apply:slots", "apply:mlp", "apply:spatial-stats",
          "apply:sa-conv", "publish16:reduce", "publish16:barrier"]
NSTAMP = 16


def main():
    import raman_mi355x as R
    from raman_mi355x import _lib, engine
    arch = sys.argv[1] if len(sys.argv) > 1 else "APIDN"
    dtype = sys.argv[2] if len(sys.argv) > 2 else "bf16x3"
    L = int(sys.argv[3]) if len(sys.argv) > 3 else 10000
    variant = sys.argv[4] if len(sys.argv) > 4 else "stamps"
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "ablate_build", f"lib_{variant}.so"))
    for fn, (args, res) in _lib._SIGNATURES.items():
        getattr(lib, fn).argtypes = args
        getattr(lib, fn).restype = res
    dev = torch.device("cuda")
    B = 1024
    _, noisy, _, _ = engine.generate(B, 3, signal_length=L, device=dev)
    x = noisy.view(B, 1, L)
    y = torch.empty_like(x)
    torch.manual_seed(0)
    model = R.MODELS[arch]()
    names = engine.param_names(arch)
    sd = model.state_dict()
    host = [sd[k].detach().float().contiguous() for k in names]
    ptrs = (ctypes.c_void_p * len(host))(*[t.data_ptr() for t in host])
    numels = (ctypes.c_int64 * len(host))(*[t.numel() for t in host])
    a, code = engine.ARCH_ID[arch], engine.resolve_dtype(arch, dtype)
    size = ctypes.c_size_t()
    assert lib.rdn_packed_size(a, code, ctypes.byref(size)) == 0
    blob = torch.empty(size.value, dtype=torch.uint8)
    assert lib.rdn_pack(a, code, ptrs, numels, len(host), ctypes.c_void_p(blob.data_ptr()), size.value) == 0
    packed = blob.to(dev)
    assert lib.rdn_workspace_size(a, code, B, L, ctypes.byref(size), None) == 0
    ws = torch.zeros(size.value, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream().cuda_stream
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for it in range(2):
        e0.record()
        rc = lib.rdn_forward(a, code, packed.data_ptr(), x.data_ptr(), y.data_ptr(), B, L,
                             ctypes.c_void_p(ws.data_ptr()), size.value, stream)
        e1.record()
        assert rc == 0, lib.rdn_last_error()
        torch.cuda.synchronize()
    ms = e0.elapsed_time(e1)
    st = ws[-256 * NSTAMP * 8:].view(torch.int64).view(256, NSTAMP).cpu().double()
    used = st.sum(1) > 0
    # per tile index (workgroup id % TT): the conv phase and the poll phase, to see which tiles of a
    # team the others wait for (TT from L: 640-row tiles with 6-row halos)
    tt = -(-L // 628)
    wg = torch.arange(256)[used]
    # team16_forward's XCD-aware placement: workgroups 8r + x, r < R0, are tile r % TT of a team on XCD x
    teams = int(used.sum()) // tt
    r0 = ((teams * tt // 8) // tt) * tt
    byt = {}
    for i, g in zip(wg.tolist(), st[used]):
        t = (i >> 3) % tt if i < 8 * r0 else (i - 8 * r0) % tt
        byt.setdefault(t, []).append(g)
    print("per tile: conv cycles / poll cycles (mean over teams)")
    for t in sorted(byt):
        g = torch.stack(byt[t])
        print(f"  tile {t:2d}: conv {g[:, 1].mean():.4e}  poll {g[:, 10].mean() + g[:, 4].mean():.4e}")
    # per team: total cycles (mean / max over its tiles); teams >= 8 * (r0 // tt) are the ones not
    # confined to one XCD
    byteam = {}
    for i, g in zip(wg.tolist(), st[used]):
        team = ((i >> 3) // tt) * 8 + (i & 7) if i < 8 * r0 else 8 * (r0 // tt) + (i - 8 * r0) // tt
        byteam.setdefault(team, []).append(g.sum().item())
    print("per team: total cycles mean / max over its tiles (spectra per team: %d)" % -(-1024 // teams))
    for tm in sorted(byteam):
        v = byteam[tm]
        print(f"  team {tm:2d}{' (spread)' if tm >= 8 * (r0 // tt) else ''}: {sum(v) / len(v):.4e} / {max(v):.4e}")
    print("per phase: edge tiles 0 / TT-1 against interior tile 1 (mean over teams)")
    for k, p in enumerate(PHASES):
        m = [torch.stack(byt[t])[:, k].mean().item() for t in (0, 1, tt - 1)]
        if max(m) > 0:
            print(f"  {p:18s} tile0 {m[0]:.4e}  tile1 {m[1]:.4e}  tile{tt - 1} {m[2]:.4e}  (edge - interior: {m[0] - m[1]:+.3e} / {m[2] - m[1]:+.3e})")
    st = st[used]
    tot = st.sum(1)
    print(f"[{variant}] {arch} {dtype} L={L} B={B}: {ms:.2f} ms, {B / ms * 1e3:,.0f} spectra/s, {int(used.sum())} workgroups")
    print(f"total cycles per WG: mean {tot.mean():.3e} min {tot.min():.3e} max {tot.max():.3e} "
          f"(=> {tot.mean() / (ms * 1e-3) / 1e9:.3f} G s_memtime ticks/s)")
    for k, p in enumerate(PHASES):
        c = st[:, k]
        print(f"  {p:18s} mean {c.mean():.3e} ({100 * c.mean() / tot.mean():5.1f}%)  min {c.min():.3e} max {c.max():.3e}")


if __name__ == "__main__":
    main()
