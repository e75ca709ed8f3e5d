#!/usr/bin/env python3
"""Register / spill / occupancy table of the engine's gfx950 kernels (compiler remarks).

  python3 tools/kernel_resources.py [extra hipcc flags...]   (CPU only; hipcc cross-compiles)
"""
import re
import subprocess
import sys
import os

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SRC = os.path.join(REPO, "neptune-mip_amd", "csrc", "nep_kernels.hip")


def main():
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-c", SRC, "-o",
           "/tmp/_nep_res.o", "-Rpass-analysis=kernel-resource-usage"] + sys.argv[1:]
    out = subprocess.run(cmd, capture_output=True, text=True).stderr
    rows, cur = [], None
    for line in out.splitlines():
        m = re.search(r"remark: (?:\S+: )?\s*([A-Za-z /\[\]]+?): (.+?) \[-Rpass", line)
        if not m:
            continue
        k, v = m.group(1).strip(), m.group(2).strip()
        if k == "Function Name":
            cur = {"name": subprocess.run(["c++filt", v], capture_output=True, text=True).stdout.strip()}
            rows.append(cur)
        elif cur is not None:
            cur[k] = v
    print(f"{'kernel':70s} {'VGPR':>5s} {'AGPR':>5s} {'vspill':>6s} {'sspill':>6s} {'occ':>4s} {'LDS':>6s}")
    for r in rows:
        n = r["name"].replace("nep::", "").split("(")[0]
        print(f"{n:70s} {r.get('VGPRs', '?'):>5s} {r.get('AGPRs', '?'):>5s} {r.get('VGPRs Spill', '?'):>6s} "
              f"{r.get('SGPRs Spill', '?'):>6s} {r.get('Occupancy [waves/SIMD]', '?'):>4s} "
              f"{r.get('LDS Size [bytes/block]', '?'):>6s}")


if __name__ == "__main__":
    main()
