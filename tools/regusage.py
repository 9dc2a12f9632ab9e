"""Per-kernel VGPR / spill / scratch table of one HIP source (hipcc -Rpass-analysis=kernel-resource-usage).

    python tools/regusage.py csrc/fused_inplace.hip [extra hipcc flags]
"""
import re
import subprocess
import sys

src = sys.argv[1]
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-fno-gpu-rdc", "-fno-honor-nans",
       "-mno-amdgpu-ieee", "--cuda-device-only", "-c", src, "-o", "/dev/null",
       "-Rpass-analysis=kernel-resource-usage"] + sys.argv[2:]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark: +(Function Name|VGPRs|AGPRs|ScratchSize \[bytes/lane\]|SGPRs Spill|VGPRs Spill|Occupancy \[waves/SIMD\]): (\S+)", line)
    if not m:
        continue
    k, v = m.groups()
    if k == "Function Name":
        cur = {"name": subprocess.run(["c++filt", v], capture_output=True, text=True).stdout.strip()}
        rows.append(cur)
    else:
        cur[k.split(" [")[0]] = v
for r in rows:
    print(f"{r['name'][:70]:70s} VGPR {r.get('VGPRs','?'):>4} AGPR {r.get('AGPRs','?'):>4} vspill {r.get('VGPRs Spill','?'):>4} "
          f"scratch {r.get('ScratchSize','?'):>4} occ {r.get('Occupancy','?')}")
