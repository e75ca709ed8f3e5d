"""Register budget of the hot kernels (CPU: hipcc cross-compiles gfx950 with the compiler's resource remarks):
the plain x passes of rows wider than 512 destinations (CPL 4 / 8) that the launchers use — workgroups of 4 or 8
waves, and 16 at CPL 4 — and the facility model's at CPL 4 keep every VGPR in registers.  Held to 6 waves per SIMD
they spilled 60 (CPL 4) to 280 (CPL 8) VGPRs per lane to scratch and the 1024x512 lone root ran its x pass at
370 us a launch instead of 128 (DESIGN.md §6 "N > 512")."""
import os
import re
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "neptune-mip_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"


def _compile(src):
    return subprocess.Popen([HIPCC, "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-c",
                             os.path.join(CSRC, src), "-o", os.devnull, "-Rpass-analysis=kernel-resource-usage"],
                            stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True)


def _resources(proc):
    out = proc.communicate(timeout=900)[1]
    rows, cur = {}, None
    for line in out.splitlines():
        m = re.search(r"remark: (?:\S+: )?\s*([A-Za-z /\[\]]+?): (.+?) \[-Rpass", line)
        if not m:
            continue
        k, v = m.group(1).strip(), m.group(2).strip()
        if k == "Function Name":
            cur = rows.setdefault(v, {})
        elif cur is not None:
            cur[k] = v
    return rows


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_wide_row_passes_do_not_spill():
    # mangled: x_pass<CPL, CHECK=false, INIT=false, FIRST=false, TW>
    pk, pf = _compile("nep_kernels.hip"), _compile("nep_fac.hip")   # (both at once)
    k = _resources(pk)
    want = {f"_ZN3nep6x_passILi{cpl}ELb0ELb0ELb0ELi{tw}EEEvNS_10DeviceViewEPKiiiii": (cpl, tw)
            for cpl, tw in ((4, 4), (4, 8), (4, 16), (8, 4), (8, 8))}
    f = _resources(pf)
    want_f = {f"_ZN3nep10fac_x_passILi4ELb0ELb0ELb0ELi{tw}EEEvNS_10DeviceViewEPKiiiii": (4, tw) for tw in (4, 8)}
    for rows, names in ((k, want), (f, want_f)):
        for name, (cpl, tw) in names.items():
            assert name in rows, name
            assert int(rows[name].get("VGPRs Spill", "0")) == 0, (name, rows[name])
