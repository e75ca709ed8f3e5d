#!/usr/bin/env python3
"""Kernel statistics from a rocprofv3 `--kernel-trace --stats` run's rocpd database.

  python3 tools/prof_summary.py gpurun_out/prof7 > profiles/r01/kernel_stats.csv

rocprofv3 7.x writes its results as one SQLite (rocpd) file; this prints the same per-kernel
summary its `--stats` CSV holds (calls, total / average / min / max ns, share of GPU time), split
additionally by grid_y (= LP slots in the launch), so a kernel's 1-LP root-solve launches and its
16-LP streaming launches are not averaged together.
"""
import glob
import os
import sqlite3
import sys


def main(d):
    dbs = sorted(glob.glob(os.path.join(d, "**", "*.db"), recursive=True))
    if not dbs:
        sys.exit(f"no rocpd database under {d}")
    rows = []
    for db in dbs:
        c = sqlite3.connect(db)
        rows += list(c.execute(
            "select name, grid_y, count(*), sum(duration), avg(duration), min(duration), max(duration), "
            "max(vgpr_count), max(sgpr_count), max(lds_size), max(scratch_size) from kernels group by name, grid_y"))
    total = sum(r[3] for r in rows) or 1
    print('"Name","GridY","Calls","TotalDurationNs","AverageNs","MinNs","MaxNs","Percentage",'
          '"VGPR","SGPR","LDS","Scratch"')
    for r in sorted(rows, key=lambda r: -r[3]):
        print('"%s",%d,%d,%d,%.1f,%d,%d,%.3f,%d,%d,%d,%d' % (r[0], r[1], r[2], r[3], r[4], r[5], r[6],
                                                             100.0 * r[3] / total, r[7], r[8], r[9], r[10]))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof")
