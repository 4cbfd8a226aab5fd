"""Per-round kernel timeline from a rocprofv3 kernel trace (csv): the median
duration and the median gap before each kernel position of a steady-state round.
Usage: python tools/trace_rounds.py <run_kernel_trace.csv> [first_kernel_substring]"""
import csv
import statistics
import sys


def main():
    path = sys.argv[1]
    head = sys.argv[2] if len(sys.argv) > 2 else "stats_prep_kernel"
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ks = [(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
    starts = [i for i, k in enumerate(ks) if head in k[0]]
    rounds = [ks[a:b] for a, b in zip(starts, starts[1:])]
    if not rounds:
        print("no rounds found")
        return
    n = statistics.mode(len(r) for r in rounds)
    rounds = [r for r in rounds if len(r) == n][len(rounds) // 4:]  # steady state
    print(f"{len(rounds)} rounds of {n} kernels; round period median "
          f"{statistics.median(r[-1][2] - r[0][1] for r in rounds) / 1000:.2f} us (first start -> last end)")
    period = [b[0][1] - a[0][1] for a, b in zip(rounds, rounds[1:])]
    print(f"start-to-start period median {statistics.median(period) / 1000:.2f} us")
    for j in range(n):
        name = rounds[0][j][0].split("(")[0][:60]
        dur = statistics.median(r[j][2] - r[j][1] for r in rounds) / 1000
        gap = statistics.median(r[j][1] - r[j - 1][2] for r in rounds) / 1000 if j else 0.0
        print(f"{j:2d} {name:60s} gap {gap:6.2f}  dur {dur:6.2f}")


if __name__ == "__main__":
    main()
