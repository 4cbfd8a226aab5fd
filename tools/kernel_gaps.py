"""Back-to-back timing of one kernel from a rocprofv3 kernel trace (CSV): per
dispatch its duration, the period to the next dispatch's start and the gap from
its end to the next start (negative: the launches overlap).  Medians over the
steady part of the run (the last `--last` dispatches).

    python tools/kernel_gaps.py gpurun_out/x/prof/run_kernel_trace.csv --kernel lanes_round_kernel
"""
from __future__ import annotations

import argparse
import csv
import json
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--kernel", default="lanes_round_kernel")
    ap.add_argument("--last", type=int, default=1000)
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            if a.kernel in r["Kernel_Name"]:
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    rows.sort()
    rows = rows[-a.last:]
    dur = [(e - s) / 1e3 for s, e in rows]
    per = [(rows[i + 1][0] - rows[i][0]) / 1e3 for i in range(len(rows) - 1)]
    gap = [(rows[i + 1][0] - rows[i][1]) / 1e3 for i in range(len(rows) - 1)]
    med = lambda v: round(statistics.median(v), 2) if v else None
    print(json.dumps({"kernel": a.kernel, "dispatches": len(rows), "duration_us": med(dur), "period_us": med(per),
                      "end_to_next_start_us": med(gap), "p10_gap": round(sorted(gap)[len(gap) // 10], 2) if gap else None,
                      "p90_gap": round(sorted(gap)[9 * len(gap) // 10], 2) if gap else None}))


if __name__ == "__main__":
    main()
