"""Per-kernel summary of rocprofv3 PMC passes (tools/pmc_profile.sh).

Averages every counter per dispatch for each kernel and derives:
  mfma_busy_frac   SQ_VALU_MFMA_BUSY_CYCLES / (SQ_BUSY_CYCLES * 4 SIMDs)  (rough)
  lds_conflict     SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  wait_frac        SQ_WAIT_ANY / SQ_WAVE_CYCLES  (waves parked on s_waitcnt / barriers)
  hbm_read_KB      2 * FETCH_SIZE  (gfx950 reports half of wide streaming reads,
                   MI355X_MICROARCH.md §HBM) ; hbm_write_KB = WRITE_SIZE
  l2_hit           TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum)
Usage: python tools/pmc_summary.py gpurun_out/pmc [--markdown]
"""
import collections
import csv
import glob
import os
import sys


def short_name(name: str) -> str:
    """Kernel name without namespaces and parameter list.  (Round 4's version cut at the
    first '(' BEFORE removing '(anonymous namespace)', so every kernel of psx's anonymous
    namespaces collapsed into one row with an empty name: lanes_round_kernel averaged
    with the 1-KB publish launch and the rest -- the inconsistent SQ_WAVES / MFMA rows.)"""
    n = name.replace("(anonymous namespace)::", "").replace("void ", "").replace("psx::", "")
    return n.split("(")[0].strip() or name


def load(root):
    """{kernel: {counter: [value per dispatch]}}, the rows of one dispatch (several
    dimension instances, if the profiler splits them) summed first."""
    per = collections.defaultdict(float)
    grids = {}
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for i, r in enumerate(csv.DictReader(open(f))):
            k = short_name(r.get("Kernel_Name", "?"))
            disp = (f, r.get("Dispatch_Id") or r.get("Correlation_Id") or str(i))
            per[(k, disp, r["Counter_Name"])] += float(r["Counter_Value"])
            if r.get("Grid_Size"):
                grids[k] = r["Grid_Size"]
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for (k, disp, c), v in per.items():
        acc[k][c].append(v)
    return acc, grids


def main(argv):
    root = argv[0] if argv else "gpurun_out/pmc"
    acc, grids = load(root)
    rows = []
    for k, cs in acc.items():
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        calls = max(len(v) for v in cs.values())
        d = {"kernel": k, "dispatches": calls, "grid": grids.get(k, "")}
        if "SQ_VALU_MFMA_BUSY_CYCLES" in avg and avg.get("SQ_BUSY_CYCLES"):
            d["mfma_busy_frac"] = avg["SQ_VALU_MFMA_BUSY_CYCLES"] / (4 * avg["SQ_BUSY_CYCLES"])
        if avg.get("SQ_LDS_IDX_ACTIVE"):
            d["lds_conflict"] = avg.get("SQ_LDS_BANK_CONFLICT", 0.0) / avg["SQ_LDS_IDX_ACTIVE"]
        if avg.get("SQ_WAVE_CYCLES") and "SQ_WAIT_ANY" in avg:
            d["wait_frac"] = avg["SQ_WAIT_ANY"] / avg["SQ_WAVE_CYCLES"]
        if "FETCH_SIZE" in avg:
            d["hbm_read_KB"] = 2 * avg["FETCH_SIZE"]
        if "WRITE_SIZE" in avg:
            d["hbm_write_KB"] = avg["WRITE_SIZE"]
        if avg.get("TCC_HIT_sum", 0) + avg.get("TCC_MISS_sum", 0) > 0:
            d["l2_hit"] = avg["TCC_HIT_sum"] / (avg["TCC_HIT_sum"] + avg["TCC_MISS_sum"])
        for c in ("SQ_INSTS_VALU_MFMA_MOPS_BF16", "SQ_INSTS_MFMA", "SQ_WAVES", "SQ_INSTS_VMEM_RD",
                  "SQ_INSTS_VMEM_WR", "SQ_INSTS_LDS", "SQ_LDS_UNALIGNED_STALL"):
            if c in avg:
                d[c] = avg[c]
        rows.append(d)
    rows.sort(key=lambda d: -d["dispatches"])
    cols = ["kernel", "dispatches", "grid", "mfma_busy_frac", "lds_conflict", "wait_frac", "hbm_read_KB", "hbm_write_KB",
            "l2_hit", "SQ_INSTS_MFMA", "SQ_INSTS_VALU_MFMA_MOPS_BF16", "SQ_WAVES", "SQ_INSTS_VMEM_RD",
            "SQ_INSTS_VMEM_WR", "SQ_INSTS_LDS", "SQ_LDS_UNALIGNED_STALL"]
    print("| " + " | ".join(cols) + " |")
    print("|" + "---|" * len(cols))
    for d in rows:
        print("| " + " | ".join((f"{d[c]:.4g}" if isinstance(d.get(c), float) else str(d.get(c, ""))) for c in cols)
              + " |")


if __name__ == "__main__":
    main(sys.argv[1:])
