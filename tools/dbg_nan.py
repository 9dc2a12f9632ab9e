import sys, torch
sys.path.insert(0,'/root/repo'); sys.path.insert(0,'/root/repo/data-simulation-and-noise-reduction-of-distributed-fiber-raman-intensity_amd')
import raman_mi355x as R
from raman_mi355x import engine
dev=torch.device("cuda")
torch.manual_seed(1234)
for dt in ["f16","bf16-unsafe","f16f8"]:
    m=R.RRCDNet().to(dev).eval().set_engine_dtype(dt)
    for B in [3, 64, 8192]:
        clean,noisy,_,_=engine.generate(B,20250410,signal_length=10000,device=dev)
        with torch.no_grad(): y=m(noisy.view(B,1,10000))
        bad=~torch.isfinite(y)
        print(dt, m.engine_code, B, "nonfinite:", int(bad.sum()), "rows:", torch.nonzero(bad.view(B,-1).any(1)).flatten()[:8].tolist(), "maxabs", float(y[torch.isfinite(y)].abs().max()), flush=True)
        if bad.any():
            i=int(torch.nonzero(bad.view(B,-1).any(1)).flatten()[0]); pos=torch.nonzero(bad.view(B,-1)[i]).flatten()
            print("  spectrum", i, "positions", pos[:10].tolist(), "count", len(pos), "x range", float(noisy[i].min()), float(noisy[i].max()))
