"""Micro-benchmark of the worker local solve on one GPU (device time per solve).

Variants isolate the cost of: the stats/prep kernel, one active slot (eval +
tail), empty slots, and the buffer size.  Usage: python tools/bench_solver.py
"""
import sys
import time

import torch

sys.path.insert(0, ".")
from psx.models.logreg import ModelSpec  # noqa: E402
from psx.ops.lr import LocalSolveOp, SolverOptions  # noqa: E402
from psx.runtime.buffer import DeviceRing  # noqa: E402
from psx.utils.data import synth_finefood  # noqa: E402


def time_solve(op, ring, B, w, reps=200):
    for _ in range(10):
        op.run(ring, B, 0, w)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        op.run(ring, B, 0, w)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000.0 / reps


def stamps(B=1024, opts=None):
    """Phase timeline of one solve (needs PSX_SOLVER_STAMPS=1)."""
    import os

    os.environ["PSX_SOLVER_STAMPS"] = "1"
    dev = "cuda:0"
    spec = ModelSpec(1024, 6)
    ds = synth_finefood(1024, seed=0)
    ring = DeviceRing(1024, spec.Fp, dev)
    ring.place(ds.X, ds.y)
    w = spec.init("random", seed=1).to(dev)
    op = LocalSolveOp(spec, 1024, dev, opts or SolverOptions())
    for _ in range(5):
        op.run(ring, B, 0, w)
    torch.cuda.synchronize()
    h = torch.cuda.current_stream().cuda_stream
    st = op._native.read_stamps(h)
    # fwd_kernel (workgroup 0): start, staged, fwd, softmax/R written, partials written;
    # bwd_update_kernel (workgroup 0): start, backward done, G reduced, controller
    # start / done (after the all-gather), controller written back, end
    names = ["fwd0", "fwd_end", "bwd0", "bwd_mfma", "g_red", "ctrl", "ctrl_done", "ctrl_wb", "bwd_end", "staged",
             "fwd", "softmax", "-"]
    order = [0, 9, 10, 11, 1, 2, 3, 4, 5, 6, 7, 8]
    print(f"--- stamps B={B} (us, relative to slot 0 start; 100 MHz) ---")
    base = st[0]
    sv = st[30 * 16: 30 * 16 + 5]
    extra = ""
    if sv[3] >= base - 10 ** 6 and sv[3] > 0 and sv[4] > 0:  # persistent solve: its start / tile staged
        extra = f" (persistent: start={(sv[3] - base) / 100.0:.2f} staged={(sv[4] - base) / 100.0:.2f})"
    print(f"stats_prep start={(sv[0] - base) / 100.0:.2f} end={(sv[1] - base) / 100.0:.2f}  "
          f"finalize start={(sv[2] - base) / 100.0:.2f}{extra}")
    ph = ["start", "mfma", "publish", "gathered"]
    rows = []
    for p_ in range(4):
        v = [st[(16 + p_ * 2 + (wg >> 4)) * 16 + (wg & 15)] for wg in range(32)]
        v = [(x - base) / 100.0 for x in v if x >= base]
        if v:
            rows.append(f"{ph[p_]} min={min(v):.2f} max={max(v):.2f}")
    if rows:
        print("slot 1 per-workgroup bwd phases: " + "; ".join(rows))
    for slot in range(op.opts.nslots):
        row = st[slot * 16: slot * 16 + 13]
        if row[0] == 0 or row[0] < base:
            continue
        print(f"slot {slot}: " + " ".join(f"{names[k]}={(row[k] - base) / 100.0:.2f}" for k in order
                                          if row[k] >= base))


def ingest_variants():
    """Solve + fused ingest of n new rows per solve (the window's newest n rows come
    from a device-resident data set, as in the engines): device time per solve and
    the stats_prep kernel's span from the device stamps."""
    import os

    os.environ["PSX_SOLVER_STAMPS"] = "1"
    dev = "cuda:0"
    spec = ModelSpec(1024, 6)
    ds = synth_finefood(8192, seed=0)
    sX, sy = ds.X.to(dev), ds.y.to(dev)
    ring = DeviceRing(1024, spec.Fp, dev)
    ring.place(ds.X[:1024], ds.y[:1024])
    w = spec.init("random", seed=1).to(dev)
    h = torch.cuda.current_stream().cuda_stream
    for n in (0, 64, 256, 1024):
        op = LocalSolveOp(spec, 1024, dev, SolverOptions())
        op.run(ring, 1024, 0, w)
        k = [0]

        def one():
            if n == 0:
                op.run(ring, 1024, 0, w)
            else:
                first = (k[0] * n) % (8192 - n)
                op._native.run_ingest(1024, 0, h, sX.data_ptr(), sy.data_ptr(), first, 1, n, 1024 - n)
            k[0] += 1

        for _ in range(10):
            one()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(200):
            one()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1000.0 / 200
        st = op._native.read_stamps(h)
        sv = st[30 * 16: 30 * 16 + 7]
        ph = "" if n == 0 else f" (loads in {(sv[5] - sv[0]) / 100.0:.2f}, copies+sums {(sv[6] - sv[0]) / 100.0:.2f})"
        print(f"ingest {n:5d} rows: {us:8.2f} us/solve  stats_prep span {(sv[1] - sv[0]) / 100.0:.2f} us{ph} "
              f"evals={op.stats.cpu().tolist()[0]}", flush=True)


def main():
    if "--ingest" in sys.argv:
        ingest_variants()
        return
    if "--stamps" in sys.argv:
        stamps(1024)
        stamps(32)
        return
    if "--stamps-persist" in sys.argv:
        stamps(1024, SolverOptions(persist=True))
        stamps(32, SolverOptions(persist=True))
        return
    dev = "cuda:0"
    spec = ModelSpec(1024, 6)
    ds = synth_finefood(1024, seed=0)
    ring = DeviceRing(1024, spec.Fp, dev)
    ring.place(ds.X, ds.y)
    w = spec.init("random", seed=1).to(dev)
    rows = []
    for name, opts, B in [
        ("default lbfgs x2 (9 slots)", SolverOptions(), 1024),
        ("lbfgs x2, ls_max=2 (5 slots)", SolverOptions(ls_max=2), 1024),
        ("init only (1 slot)", SolverOptions(iters=1, ls_max=0), 1024),
        ("gd x1 (2 slots)", SolverOptions(mode="gd", iters=1), 1024),
        ("gd x4 (5 slots)", SolverOptions(mode="gd", iters=4), 1024),
        ("default, B=32 (1 tile)", SolverOptions(), 32),
        ("init only, B=32", SolverOptions(iters=1, ls_max=0), 32),
        ("default, hipGraph replay", SolverOptions(use_graph=True), 1024),
        ("persistent (one launch)", SolverOptions(persist=True), 1024),
        ("persistent, B=32", SolverOptions(persist=True), 32),
        ("persistent, ls_max=2", SolverOptions(persist=True, ls_max=2), 1024),
    ]:
        op = LocalSolveOp(spec, 1024, dev, opts)
        us = time_solve(op, ring, B, w)
        st = op.stats.cpu().tolist()
        rows.append((name, us, st))
        print(f"{name:32s} {us:9.2f} us/solve  stats(evals,acc,lsfail,reset)={st}", flush=True)
    # host-side cost of one graph launch (no sync)
    op = LocalSolveOp(spec, 1024, dev, SolverOptions())
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(200):
        op.run(ring, 1024, 0, w)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    print(f"host enqueue per solve: {(t1 - t0) / 200 * 1e6:.1f} us")
    op = LocalSolveOp(spec, 1024, dev, SolverOptions(persist=True))
    op.run(ring, 1024, 0, w)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(200):
        op.run(ring, 1024, 0, w)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    print(f"host enqueue per solve (persistent): {(t1 - t0) / 200 * 1e6:.1f} us")


if __name__ == "__main__":
    main()
