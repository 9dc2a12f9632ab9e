import ctypes, os, sys
import numpy as np, torch
ROOT = "/root/repo"
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "data-simulation-and-noise-reduction-of-distributed-fiber-raman-intensity_amd"))
import raman_mi355x as R
from raman_mi355x import _lib, engine
from oracle.weights import synth_state_dict
model = R.RRCDNet()
tmpl = {k: (tuple(v.shape), v.dtype) for k, v in model.state_dict().items()}
sd = synth_state_dict(tmpl, 1234)
names = engine.param_names("RRCDNet")
host = [sd[k].detach().float().contiguous() for k in names]
ptrs = (ctypes.c_void_p * len(host))(*[t.data_ptr() for t in host])
numels = (ctypes.c_int64 * len(host))(*[t.numel() for t in host])
dev = torch.device("cuda")
for B in (2, 64):
    x = torch.from_numpy(np.random.default_rng(0 if B == 2 else 1).uniform(0, 1, (B, 1, 1200)).astype(np.float32)).to(dev)
    for name in sys.argv[1:]:
        lib = ctypes.CDLL(os.path.join(ROOT, "tools", "ablate_build", f"lib_{name}.so"))
        for fn, (args, res) in _lib._SIGNATURES.items():
            if hasattr(lib, fn):
                getattr(lib, fn).argtypes, getattr(lib, fn).restype = args, res
        size = ctypes.c_size_t()
        assert lib.rdn_packed_size(1, 5, ctypes.byref(size)) == 0
        blob = torch.empty(size.value, dtype=torch.uint8)
        assert lib.rdn_pack(1, 5, ptrs, numels, len(host), ctypes.c_void_p(blob.data_ptr()), size.value) == 0
        blob = blob.to(dev)
        y = torch.empty_like(x)
        ws = torch.zeros(256, dtype=torch.uint8, device=dev)
        rc = lib.rdn_forward(1, 5, blob.data_ptr(), x.data_ptr(), y.data_ptr(), B, 1200, ws.data_ptr(), 256, torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        w = ws.view(torch.int32).cpu().numpy()
        yy = y.cpu().numpy()
        print(name, B, "rc", rc, "status words", w[:4], "nan rows", int(np.isnan(yy).sum()), "absmax", float(np.nanmax(np.abs(yy))), flush=True)
