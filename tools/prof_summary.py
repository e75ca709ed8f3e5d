#!/usr/bin/env python3
"""Kernel statistics from a rocprofv3 `--kernel-trace --stats` run's rocpd database.

  python3 tools/prof_summary.py gpurun_out/prof [--functions F] > profiles/r02/kernel_stats_by_slots.csv

rocprofv3 7.x writes its results as one SQLite (rocpd) file; this prints the per-kernel summary its
`--stats` CSV holds (calls, total / average / min / max ns, share of GPU time), split additionally by
the number of LP slots a launch carries, so a kernel's 1-LP root-solve launches and its 32-LP
streaming launches are not averaged together:
  * x_pass: its grid is one workgroup per (function, slot), padded to a multiple of 8 for the
    XCD-aware order (csrc/nep_kernels.hip launch_x_tw), so slots = ceil(workgroups / F) with F =
    --functions (the bench's 256);
  * node_pass / scalar_pass / init kernels: slots = grid_y (resp. grid_x / block for scalar_pass).
"""
import argparse
import glob
import math
import os
import sqlite3
import sys


def slots_of(name, gx, gy, wx, F):
    wgs = gx // max(1, wx)
    if "x_pass" in name:
        return int(math.ceil(wgs / F - 1e-9)) if F else wgs
    if "scalar_pass" in name:
        return wgs
    return gy


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir", nargs="?", default="gpurun_out/prof")
    ap.add_argument("--functions", type=int, default=256)
    a = ap.parse_args()
    dbs = sorted(glob.glob(os.path.join(a.dir, "**", "*.db"), recursive=True))
    if not dbs:
        sys.exit(f"no rocpd database under {a.dir}")
    agg = {}
    for db in dbs:
        c = sqlite3.connect(db)
        for name, gx, gy, wx, dur, vg, sg, lds, scr in c.execute(
                "select name, grid_x, grid_y, workgroup_x, duration, vgpr_count, sgpr_count, lds_size, "
                "scratch_size from kernels"):
            key = (name, slots_of(name, gx, gy, wx, a.functions))
            e = agg.setdefault(key, [0, 0, math.inf, 0, vg, sg, lds, scr])
            e[0] += 1
            e[1] += dur
            e[2] = min(e[2], dur)
            e[3] = max(e[3], dur)
    total = sum(e[1] for e in agg.values()) or 1
    print('"Name","Slots","Calls","TotalDurationNs","AverageNs","MinNs","MaxNs","Percentage","VGPR","SGPR","LDS",'
          '"Scratch"')
    for (name, sl), e in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print('"%s",%d,%d,%d,%.1f,%d,%d,%.3f,%d,%d,%d,%d' % (name, sl, e[0], e[1], e[1] / e[0], e[2], e[3],
                                                             100.0 * e[1] / total, e[4], e[5], e[6], e[7]))


if __name__ == "__main__":
    main()
