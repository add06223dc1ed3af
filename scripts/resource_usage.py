#!/usr/bin/env python3
"""Print VGPR / SGPR / LDS / occupancy per kernel (hipcc -Rpass-analysis=kernel-resource-usage)."""
import re
import subprocess
import sys

srcs = sys.argv[1:] or ["kernels.hip", "wide.hip"]
for src in srcs:
    out = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-x", "hip", "-c", src,
                          "-o", "/dev/null", "-Rpass-analysis=kernel-resource-usage"], capture_output=True,
                         text=True).stderr
    cur = None
    rows = {}
    for line in out.splitlines():
        m = re.search(r"remark: (.*?)(?: \[-Rpass)", line)
        if not m:
            continue
        t = m.group(1).strip()
        if t.startswith("Function Name:"):
            cur = t.split(":", 1)[1].strip()
            rows[cur] = {}
        elif cur and ":" in t:
            k, v = t.split(":", 1)
            rows[cur][k.strip()] = v.strip()
    for name, r in rows.items():
        dm = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
        dm = re.sub(r"\(.*", "", dm)
        print(f"{dm[:60]:60s} VGPR={r.get('VGPRs','?'):>4} AGPR={r.get('AGPRs','?'):>3} SGPR={r.get('SGPRs','?'):>3} "
              f"spill={r.get('VGPRs Spill','?')}/{r.get('SGPRs Spill','?')} LDS={r.get('LDS Size [bytes/block]','?'):>6} "
              f"occ={r.get('Occupancy [waves/SIMD]','?')}")
