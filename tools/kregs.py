#!/usr/bin/env python3
"""Per-kernel register / spill / occupancy table of a HIP source (hipcc -Rpass-analysis).

    python tools/kregs.py csrc/src/kernels/bitpar_pull.hip [name-regex]
"""
import re
import subprocess
import sys

src = sys.argv[1]
pat = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-Icsrc/include", "-D__HIP_PLATFORM_AMD__",
       "--offload-arch=gfx950", "-x", "hip", "-c", src, "-o", "/tmp/kregs.o",
       "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur = None
rows = []
for line in out.splitlines():
    m = re.search(r"remark: +([^\[]+?) ?\[", line)
    if not m:
        if "error" in line:
            print(line)
        continue
    t = m.group(1).strip()
    if t.startswith("Function Name:"):
        name = t.split(":", 1)[1].strip()
        dm = subprocess.run(["c++filt", name], capture_output=True,
                            text=True).stdout.strip()
        dm = re.sub(r"\(.*", "", dm).replace("msbfs::bp::", "")
        cur = {"name": dm}
        rows.append(cur)
    elif cur is not None and ":" in t:
        k, v = t.split(":", 1)
        cur[k.strip()] = v.strip()
for r in rows:
    if pat and not pat.search(r["name"]):
        continue
    print(f'{r["name"][:70]:70s} vgpr={r.get("VGPRs","?"):>4} spill={r.get("VGPRs Spill","?"):>3} '
          f'occ={r.get("Occupancy [waves/SIMD]","?")} lds={r.get("LDS Size [bytes/block]","?")}')
