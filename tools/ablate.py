"""Diagnostic ablation of the in-place kernels (not part of the product).

Builds libraman_mi355x variants with RDN_ABLATE_* / RDN_IP_NB macros into /tmp and times the RRCDNet
forward of each in ONE process (interleaved rounds), so the deltas say which resource bounds the
kernel: MFMA issue (NOLDS), LDS traffic (NOMFMA), the write-back (NOSTORE).

    python tools/ablate.py build      # in the build container (hipcc)
    python tools/ablate.py run        # on the GPU box
"""
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "data-simulation-and-noise-reduction-of-distributed-fiber-raman-intensity_amd", "csrc")
OUT = os.path.join(ROOT, "tools", "ablate_build")
VARIANTS = {"base": "", "prev": "", "cur": "", "cur2": "", "nolds": "-DRDN_ABLATE_NOLDS",
            "nomfma": "-DRDN_ABLATE_NOMFMA", "nostore": "-DRDN_ABLATE_NOSTORE", "noaload": "-DRDN_ABLATE_NOALOAD",
            "pf3": "-DRDN_H16_PF=3", "ieee": "", "stamps": "-DRDN_TEAM_STAMPS=1", "nobar": "-DRDN_ABLATE_NOBARRIER", "dsdn3": "-DRDN_DSDN_NBK=3", "comp0": "-DRDN_F32_COMP=0",
            "chunk1": "-DRDN_F32_CHUNK=1", "chunk3": "-DRDN_F32_CHUNK=3", "chunk4": "-DRDN_F32_CHUNK=4",
            "h16f16": "-DRDN_H16_F16=1", "ld2": "-DRDN_H16_LDSTEP=2", "ld3": "-DRDN_H16_LDSTEP=3", "ld4": "-DRDN_H16_LDSTEP=4", "pf2": "-DRDN_H16_PF=2", "pf4": "-DRDN_H16_PF=4", "alledge": "-DRDN_ABLATE_ALLEDGE -DRDN_TEAM_STAMPS=1",
            "tail3": "-DRDN_F16MIX_TAIL=3", "tail4": "-DRDN_F16MIX_TAIL=4", "tail5": "-DRDN_F16MIX_TAIL=5", "nowin": "-DRDN_F16MIX_WIN=0", "nostem": "-DRDN_ABLATE_NOSTEM",
            "tail0": "-DRDN_F16MIX_TAIL=0", "tail2": "-DRDN_F16MIX_TAIL=2", "hybstamps": "-DRDN_HYB_STAMPS=1",
            "w512": "-DRDN_WALK_ROWS=512", "w448": "-DRDN_WALK_ROWS=448", "mix512": "-DRDN_WALK_ROWS_MIX=512", "mhead": "", "lbar": "", "stg": "", "vote": "", "comb": "", "track": "", "trk2": "", "sdpp": "", "cur": "", "resplain": "", "rescomp0": "-DRDN_F32_COMP_RES=0", "reschunk6": "-DRDN_F32_COMP_RES=1 -DRDN_F32_CHUNK_RES=6", "reschunk3": "-DRDN_F32_COMP_RES=1 -DRDN_F32_CHUNK_RES=3", "reschunk4": "-DRDN_F32_COMP_RES=1 -DRDN_F32_CHUNK_RES=4", "reschunk2": "-DRDN_F32_COMP_RES=1 -DRDN_F32_CHUNK_RES=2", "nozero": "-DRDN_ABLATE_NOZERO", "nozst": "-DRDN_ABLATE_NOZERO -DRDN_TEAM_STAMPS=1", "estag": "-DRDN_H16_ESTAG=1",
            "prio": "-DRDN_SETPRIO=1", "prio2": "-DRDN_SETPRIO=2", "es3": "-DRDN_H16_ESPLIT=3", "es5": "-DRDN_H16_ESPLIT=5",
            "sgb2": "-DRDN_H16_SGB=2", "sgb4": "-DRDN_H16_SGB=4", "remap": "-DRDN_HALF_REMAP=1",
            "prioremap": "-DRDN_SETPRIO=1 -DRDN_HALF_REMAP=1", "tstag": "-DRDN_TAIL_STAG=1",
            "tsgb1": "-DRDN_TAIL_SGB=1", "tsgb2": "-DRDN_TAIL_SGB=2", "tsgb4": "-DRDN_TAIL_SGB=4", "tsgb8": "-DRDN_TAIL_SGB=8",
            "stgfirst": "-DRDN_STAGE_FIRST=1",
            "tearly": "-DRDN_TAIL_EARLY=1", "tearlyhs": "-DRDN_TAIL_EARLY=1 -DRDN_HYB_STAMPS=1",
            "psw2": "-DRDN_PRIO_SWITCH=2", "psw3": "-DRDN_PRIO_SWITCH=3", "psw4": "-DRDN_PRIO_SWITCH=4",
            "psw5": "-DRDN_PRIO_SWITCH=5", "psw6": "-DRDN_PRIO_SWITCH=6", "psw4hs": "-DRDN_PRIO_SWITCH=4 -DRDN_HYB_STAMPS=1",
            "tnoaload": "-DRDN_ABLATE_NOALOAD_TAIL", "tnoaloadhs": "-DRDN_ABLATE_NOALOAD_TAIL -DRDN_HYB_STAMPS=1",
            "tswap": "-DRDN_TAIL_SWAP=1", "tswapearly": "-DRDN_TAIL_SWAP=1 -DRDN_TAIL_EARLY=1",
            "tswapearlyhs": "-DRDN_TAIL_SWAP=1 -DRDN_TAIL_EARLY=1 -DRDN_HYB_STAMPS=1",
            "tswape2": "-DRDN_TAIL_SWAP=1 -DRDN_TAIL_EARLY=2", "tswape3": "-DRDN_TAIL_SWAP=1 -DRDN_TAIL_EARLY=3"}


def build():
    """Compile every requested variant (all objects in parallel, 8 jobs), then link each."""
    import torch
    from concurrent.futures import ThreadPoolExecutor
    tlib = os.path.join(os.path.dirname(torch.__file__), "lib")
    os.makedirs(OUT, exist_ok=True)
    srcs = ["fused16.hip", "fused16_f16.hip", "fused16_small.hip", "fused16_walk.hip", "fused_inplace.hip", "cbam.hip", "generator.hip", "metrics.hip", "abi.cpp",
            "pack.cpp"]
    only = sys.argv[2:]
    names = [n for n in VARIANTS if not only or n in only]
    jobs = []
    for name in names:
        flag = VARIANTS[name]
        # "prev": the sources of another tree (ABLATE_PREV_SRC = its csrc directory, e.g. a git archive of
        # the last commit) for an A/B against the working tree in one process
        src_dir = os.environ.get("ABLATE_PREV_SRC", CSRC) if name == "prev" else CSRC
        for s in srcs:
            if not os.path.exists(os.path.join(src_dir, s)):
                continue
            o = os.path.join(OUT, f"{name}_{s}.o")
            cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-mcode-object-version=5",
                   "-fno-gpu-rdc", "-c", os.path.join(src_dir, s), "-o", o] + flag.split()
            if s in ("fused16.hip", "fused16_f16.hip", "fused16_small.hip", "fused16_walk.hip", "fused_inplace.hip", "cbam.hip") and name != "ieee":
                cmd += ["-fno-honor-nans", "-mno-amdgpu-ieee"]
            if s == "generator.hip":
                cmd += ["-ffp-contract=off"]
            jobs.append(cmd)
    with ThreadPoolExecutor(int(os.environ.get("ABLATE_JOBS", "8"))) as ex:
        for r in ex.map(lambda c: subprocess.run(c, cwd=os.path.dirname(c[c.index("-c") + 1]), capture_output=True,
                                                 text=True), jobs):
            if r.returncode:
                print(r.stderr[-3000:])
                raise SystemExit("compile failed")
    for name in names:
        objs = [os.path.join(OUT, f"{name}_{s}.o") for s in srcs if os.path.exists(os.path.join(OUT, f"{name}_{s}.o"))]
        subprocess.run(["g++", "-shared", "-o", os.path.join(OUT, f"lib_{name}.so")] + objs +
                       [f"-L{tlib}", "-l:libamdhip64.so", f"-Wl,-rpath,{tlib}"], check=True)
        print("built", name, flush=True)


def run():
    import torch
    sys.path.insert(0, os.path.join(ROOT, "data-simulation-and-noise-reduction-of-distributed-fiber-raman-intensity_amd"))
    import raman_mi355x as R
    from raman_mi355x import _lib, engine
    dev = torch.device("cuda")
    L = int(os.environ.get("RDN_ABLATE_L", "10000"))          # spectrum length (default 10,000)
    B = max(64, 2048 * 10000 // L)
    clean, noisy, _, _ = engine.generate(B, 1, signal_length=L, device=dev)
    x = noisy.view(B, 1, L)
    y = torch.empty_like(x)
    torch.manual_seed(0)
    arch = os.environ.get("RDN_ABLATE_ARCH", "RRCDNet")     # network to time (default RRCDNet)
    aid = engine._arch(arch)
    model = R.MODELS[arch]()
    libs = {}
    only = os.environ.get("ABLATE_ONLY", "").split(",") if os.environ.get("ABLATE_ONLY") else None
    for name in VARIANTS:
        if not os.path.exists(os.path.join(OUT, f"lib_{name}.so")) or (only and name not in only):
            continue
        lib = ctypes.CDLL(os.path.join(OUT, f"lib_{name}.so"))
        for fn, (args, res) in _lib._SIGNATURES.items():
            if not hasattr(lib, fn):
                continue
            getattr(lib, fn).argtypes = args
            getattr(lib, fn).restype = res
        libs[name] = lib
    results = {}
    names = engine.param_names(arch)
    sd = model.state_dict()
    host = [sd[k].detach().float().contiguous() for k in names]
    ptrs = (ctypes.c_void_p * len(host))(*[t.data_ptr() for t in host])
    numels = (ctypes.c_int64 * len(host))(*[t.numel() for t in host])

    def pack_with(lib, code):
        size = ctypes.c_size_t()
        assert lib.rdn_packed_size(aid, code, ctypes.byref(size)) == 0
        blob = torch.empty(size.value, dtype=torch.uint8)
        rc = lib.rdn_pack(aid, code, ptrs, numels, len(host), ctypes.c_void_p(blob.data_ptr()), size.value)
        assert rc == 0, lib.rdn_last_error()
        return blob.to(dev)

    for dtype in sys.argv[2:] or ["bf16x3", "fp32"]:
        code = engine.resolve_dtype(aid, dtype)
        packed = {name: pack_with(lib, code) for name, lib in libs.items()}
        times = {k: [] for k in libs}
        outs = {}
        wss = {}
        for name, lib in libs.items():          # CBAM networks: the team kernel's workspace
            wsz = ctypes.c_size_t()
            assert lib.rdn_workspace_size(aid, code, B, L, ctypes.byref(wsz), None) == 0
            wss[name] = (torch.zeros(max(1, wsz.value), dtype=torch.uint8, device=dev), wsz.value)
        for rnd in range(4):
            for name, lib in libs.items():
                stream = torch.cuda.current_stream().cuda_stream
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                wsp, wsn = wss[name][0].data_ptr(), wss[name][1]
                lib.rdn_forward(aid, code, packed[name].data_ptr(), x.data_ptr(), y.data_ptr(), B, L, wsp, wsn, stream)
                e0.record()
                for _ in range(3):
                    rc = lib.rdn_forward(aid, code, packed[name].data_ptr(), x.data_ptr(), y.data_ptr(), B, L, wsp, wsn, stream)
                    assert rc == 0, lib.rdn_last_error()
                e1.record()
                torch.cuda.synchronize()
                times[name].append(e0.elapsed_time(e1) / 3)
                if rnd == 0:
                    outs[name] = y[:64].clone()
        ref = outs.get("base")
        for name, t in times.items():
            results[(dtype, name)] = min(t)
            diff = float((outs[name] - ref).abs().max()) if ref is not None else float("nan")
            print(f"{dtype:7s} {name:9s} {min(t):8.2f} ms  ({B / min(t) * 1e3:9.0f} spectra/s)  max|y-base| {diff:.3e}",
                  flush=True)


def parity():
    """Max error of every built variant against the golden fixtures (reference fp32 outputs and the
    float64 forward), per network and weight set:  python tools/ablate.py parity fp32 [archs...]"""
    import numpy as np
    import torch
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    sys.path.insert(0, os.path.join(ROOT, "data-simulation-and-noise-reduction-of-distributed-fiber-raman-intensity_amd"))
    from conftest import INPUT_SETS, golden_inputs, golden_state_dict, input_array, load_golden
    from raman_mi355x import _lib, engine
    dev = torch.device("cuda")
    dtype = sys.argv[2] if len(sys.argv) > 2 else "fp32"
    archs = sys.argv[3:] or ["RRCDNet", "DenoiseCNN", "PIDN", "DSDN", "ADSDN", "APIDN"]
    inp = golden_inputs()
    for name in VARIANTS:
        path = os.path.join(OUT, f"lib_{name}.so")
        if not os.path.exists(path):
            continue
        lib = ctypes.CDLL(path)
        for fn, (args, res) in _lib._SIGNATURES.items():
            if not hasattr(lib, fn):
                continue
            getattr(lib, fn).argtypes = args
            getattr(lib, fn).restype = res
        for arch in archs:
            aid = engine._arch(arch)
            code = engine.resolve_dtype(arch, dtype)
            g = load_golden(arch)
            for which in ["synth", "trained"]:
                if which == "trained" and not any(k.startswith("w::") for k in g.files):
                    continue
                sd = golden_state_dict(arch, which)
                names = engine.param_names(arch)
                host = [sd[k].detach().float().contiguous() for k in names]
                ptrs = (ctypes.c_void_p * len(host))(*[t.data_ptr() for t in host])
                numels = (ctypes.c_int64 * len(host))(*[t.numel() for t in host])
                size = ctypes.c_size_t()
                assert lib.rdn_packed_size(aid, code, ctypes.byref(size)) == 0
                blob = torch.empty(size.value, dtype=torch.uint8)
                assert lib.rdn_pack(aid, code, ptrs, numels, len(host), ctypes.c_void_p(blob.data_ptr()), size.value) == 0
                blob = blob.to(dev)
                worst = [0.0, 0.0, 0.0]
                for s_ in INPUT_SETS:
                    xn = torch.from_numpy(np.ascontiguousarray(input_array(inp, s_))).to(dev)
                    y = torch.empty_like(xn)
                    wsz = ctypes.c_size_t()
                    lib.rdn_workspace_size(aid, code, xn.shape[0], xn.shape[1], ctypes.byref(wsz), None)
                    ws = torch.empty(max(1, wsz.value), dtype=torch.uint8, device=dev)
                    rc = lib.rdn_forward(aid, code, blob.data_ptr(), xn.data_ptr(), y.data_ptr(), xn.shape[0], xn.shape[1],
                                         ws.data_ptr(), wsz.value, torch.cuda.current_stream().cuda_stream)
                    assert rc == 0, lib.rdn_last_error()
                    yh = y.cpu().numpy()
                    ref, ex = g[f"{which}_{s_}"], g[f"f64_{which}_{s_}"]
                    sc = max(np.abs(ref).max(), 1e-30)
                    worst = [max(worst[0], np.abs(yh - ref).max() / sc), max(worst[1], np.abs(yh - ex).max() / sc),
                             max(worst[2], np.abs(ref - ex).max() / sc)]
                print(f"{name:8s} {arch:10s} {which:7s} {dtype}: vs ref {worst[0]:.2e}  vs f64 {worst[1]:.2e}  "
                      f"(ref vs f64 {worst[2]:.2e})", flush=True)


def _perturbed(sd, seed):
    """the weights with every element moved by -1, 0 or +1 ulp of fp32 (tests/test_range_gpu.py)"""
    import torch
    g = torch.Generator().manual_seed(seed)
    return {k: (v * (1 + torch.randint(-1, 2, v.shape, generator=g).float() * 2.0 ** -24)).float()
            if v.is_floating_point() and v.numel() > 1 else v for k, v in sd.items()}


def scaled():
    """fp32 on scaled inputs (tests/test_range_gpu.py's cases): per built variant, network and scale, the
    engine's max distance from the float64 forward over the reference fp32's own distance (the test's
    factor):  python tools/ablate.py scaled [archs...]"""
    import numpy as np
    import torch
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    sys.path.insert(0, os.path.join(ROOT, "data-simulation-and-noise-reduction-of-distributed-fiber-raman-intensity_amd"))
    from conftest import golden_inputs, golden_state_dict
    import raman_mi355x as R
    from raman_mi355x import _lib, engine
    dev = torch.device("cuda")
    archs = sys.argv[2:] or ["DenoiseCNN", "RRCDNet", "DSDN", "PIDN", "ADSDN", "APIDN"]
    inp = golden_inputs()
    xs = [inp["main_noisy"][:2], inp["edge1000_noisy"]]
    libs = {}
    for name in VARIANTS:
        path = os.path.join(OUT, f"lib_{name}.so")
        if os.path.exists(path):
            lib = ctypes.CDLL(path)
            for fn, (args, res) in _lib._SIGNATURES.items():
                if hasattr(lib, fn):
                    getattr(lib, fn).argtypes = args
                    getattr(lib, fn).restype = res
            libs[name] = lib
    for arch in archs:
        sd = golden_state_dict(arch, "trained")
        m32, m64 = R.MODELS[arch](), R.MODELS[arch]()
        m32.load_state_dict(sd, strict=True)
        m64.load_state_dict(sd, strict=True)
        m32, m64 = m32.eval(), m64.double().eval()
        aid, code = engine._arch(arch), engine.resolve_dtype(arch, "fp32")
        names = engine.param_names(arch)
        host = [sd[k].detach().float().contiguous() for k in names]
        ptrs = (ctypes.c_void_p * len(host))(*[t.data_ptr() for t in host])
        numels = (ctypes.c_int64 * len(host))(*[t.numel() for t in host])
        for scale in [1.0, 10.0, 100.0, 1000.0]:
            refs = []
            for x in xs:
                xt = torch.from_numpy((x * scale).astype(np.float32)).unsqueeze(1)
                with torch.no_grad():
                    y64 = m64(xt.double()).squeeze(1).numpy()
                    # fp32 noise floor as tests/test_range_gpu.py: the reference weights and three 1-ulp
                    # perturbations, the largest distance from float64
                    floor = float(np.abs(m32(xt).squeeze(1).numpy() - y64).max())
                    for seed in range(3):
                        mp = R.MODELS[arch]()
                        mp.load_state_dict(_perturbed(sd, seed), strict=True)
                        floor = max(floor, float(np.abs(mp.eval()(xt).squeeze(1).numpy() - y64).max()))
                    refs.append((xt, m32(xt).squeeze(1).numpy(), y64, floor))
            line = []
            for name, lib in libs.items():
                size = ctypes.c_size_t()
                assert lib.rdn_packed_size(aid, code, ctypes.byref(size)) == 0
                blob = torch.empty(size.value, dtype=torch.uint8)
                assert lib.rdn_pack(aid, code, ptrs, numels, len(host), ctypes.c_void_p(blob.data_ptr()), size.value) == 0
                blob = blob.to(dev)
                worst_e, worst_r, worst_q, worst_f = 0.0, 0.0, 0.0, 0.0
                for xt, r32, y64, floor in refs:
                    xd = xt.to(dev)
                    y = torch.empty_like(xd)
                    wsz = ctypes.c_size_t()
                    lib.rdn_workspace_size(aid, code, xd.shape[0], xd.shape[-1], ctypes.byref(wsz), None)
                    ws = torch.empty(max(1, wsz.value), dtype=torch.uint8, device=dev)
                    rc = lib.rdn_forward(aid, code, blob.data_ptr(), xd.data_ptr(), y.data_ptr(), xd.shape[0], xd.shape[-1],
                                         ws.data_ptr(), wsz.value, torch.cuda.current_stream().cuda_stream)
                    assert rc == 0, lib.rdn_last_error()
                    yh = y.squeeze(1).cpu().numpy()
                    e_, r_ = float(np.abs(yh - y64).max()), float(np.abs(r32 - y64).max())
                    bar = max(1e-5 * float(np.abs(y64).max()), r_)       # test_range_gpu's bar at factor 1
                    fbar = max(1e-5 * float(np.abs(y64).max()), floor)
                    worst_e, worst_r, worst_q = max(worst_e, e_), max(worst_r, r_), max(worst_q, e_ / bar)
                    worst_f = max(worst_f, e_ / fbar)
                # worst over the inputs of (engine distance) / max(1e-5 max|y64|, reference distance), and
                # of (engine distance) / max(1e-5 max|y64|, fp32 noise floor)
                line.append(f"{name} {worst_e:.2e} ({worst_q:.2f}x ref, {worst_f:.2f}x floor)")
            print(f"{arch:10s} x{scale:<6g} ref32-vs-f64 {worst_r:.2e} | " + " | ".join(line), flush=True)


if __name__ == "__main__":
    {"build": build, "run": run, "parity": parity, "scaled": scaled}[sys.argv[1]]()
