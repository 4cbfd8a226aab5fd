"""Kernel statistics from a rocprofv3 database (ROCm 7 writes rocpd SQLite by
default): per-kernel calls, total / mean / min / max us and share of GPU time,
plus the launch geometry and register / LDS footprint of each kernel.

    python tools/rocpd_stats.py gpurun_out/r03p/prof/w4_results.db > profiles/r03_v6/kernel_stats.csv
"""
from __future__ import annotations

import csv
import sqlite3
import sys


def main(path: str):
    db = sqlite3.connect(path)
    rows = db.execute(
        "select name, count(*), sum(duration), avg(duration), min(duration), max(duration), max(grid_x), "
        "max(workgroup_x), max(lds_size), max(vgpr_count), max(accum_vgpr_count), max(scratch_size) "
        "from kernels group by name order by sum(duration) desc").fetchall()
    total = sum(r[2] for r in rows) or 1.0
    w = csv.writer(sys.stdout)
    w.writerow(["kernel", "calls", "total_us", "mean_us", "min_us", "max_us", "pct", "grid_x", "wg_x", "lds_bytes",
                "vgpr", "agpr", "scratch"])
    for r in rows:  # durations are ns
        w.writerow([r[0][:120], r[1], round(r[2] / 1e3, 2), round(r[3] / 1e3, 3), round(r[4] / 1e3, 3),
                    round(r[5] / 1e3, 3), round(100.0 * r[2] / total, 2)] + list(r[6:]))


if __name__ == "__main__":
    main(sys.argv[1])
