"""Device time of one wide/sparse local solve (csrc/solver/wide_solver.hip).

Fills a worker ring with a window of sparse rows (bench config sparse1m by
default), times N back-to-back solves with HIP events, and with --stamps
prints the dots-kernel phase timeline (PSX_WIDE_STAMPS).
Usage: python tools/bench_wide.py [--features F] [--classes K] [--rows B] [--stamps]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--features", type=int, default=1 << 20)
    ap.add_argument("--labels", default="finefood", choices=["finefood", "binary"])
    ap.add_argument("--rows", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--stamps", action="store_true")
    ap.add_argument("--no-graph", action="store_true")
    a = ap.parse_args()
    if a.stamps:
        os.environ["PSX_WIDE_STAMPS"] = "1"
    import torch

    from psx.models.wide import WideSpec
    from psx.ops.lr import SolverOptions, stream_handle
    from psx.ops.sparse import SparseRing, WideSolveOp, nz_capacity
    from psx.utils.data import synth_sparse

    dev = "cuda:0"
    ds = synth_sparse(a.rows * 4, num_features=a.features, labels=a.labels, device=dev)
    K = 1 if a.labels == "binary" else 6
    spec = WideSpec(a.features, K)
    NZ = nz_capacity(ds.max_nnz)
    ring = SparseRing(a.rows, NZ, dev)
    ring.ingest_from(ds, 0, 1, a.rows, 0)
    op = WideSolveOp(spec, a.rows, NZ, dev, SolverOptions(zero_const=False, use_graph=not a.no_graph))
    w = spec.init("random", seed=0, device=dev)
    for _ in range(5):
        op.run(ring, a.rows, 0, w)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.reps):
        op.run(ring, a.rows, 0, w)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1000.0 / a.reps
    U = op.host_count()
    print(f"wide solve: F={a.features} K={K} B={a.rows} NZ={NZ} U={U} stats={op.stats.tolist()} "
          f"graph={not a.no_graph}: {us:.1f} us/solve")
    if a.stamps:
        st = op._native.read_stamps(stream_handle(dev))
        names = ["entry", "last_in", "reduced", "ctrl_loaded", "ctrl_done", "stored"]
        for s in range(len(st) // 8):
            row = st[s * 8: s * 8 + 6]
            if row[0] == 0:
                continue
            print(f"slot {s}: " + " ".join(f"{n}=+{(v - row[0]) / 100.0:.2f}us" for n, v in zip(names[1:], row[1:])))


if __name__ == "__main__":
    main()
