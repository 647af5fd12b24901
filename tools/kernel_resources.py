#!/usr/bin/env python
"""Summarise hipcc -Rpass-analysis=kernel-resource-usage remarks per kernel.

usage: python tools/kernel_resources.py [csrc/file.hip ...]   (default: every irl-maxent_amd/csrc/*.hip)
"""
import re
import subprocess
import sys

def main(files):
    for f in files:
        out = subprocess.run(["hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off", "-c", "-o", "/dev/null", f,
                              "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True).stderr
        cur = None
        rows = {}
        for line in out.splitlines():
            m = re.search(r"remark:\s+(.+?): (.+?) \[-Rpass", line)
            if not m:
                continue
            k, v = m.group(1), m.group(2)
            if k == "Function Name":
                cur = v
                rows[cur] = {}
            elif cur:
                rows[cur][k] = v
        demangled = subprocess.run(["c++filt"], input="\n".join(rows), capture_output=True, text=True).stdout.split("\n")
        for name, dm in zip(rows, demangled):
            r = rows[name]
            print(f"{dm[:60]:60s} vgpr={r.get('VGPRs','?'):>4} agpr={r.get('AGPRs','?'):>3} sgpr={r.get('TotalSGPRs','?'):>3} "
                  f"vspill={r.get('VGPRs Spill','?'):>3} sspill={r.get('SGPRs Spill','?'):>3} occ={r.get('Occupancy [waves/SIMD]','?')} "
                  f"lds={r.get('LDS Size [bytes/block]','?')}")

if __name__ == "__main__":
    import glob
    import os
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    main(sys.argv[1:] or sorted(glob.glob(os.path.join(here, "irl-maxent_amd", "csrc", "*.hip"))))
