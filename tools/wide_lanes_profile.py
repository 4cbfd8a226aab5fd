"""Phase timeline of the wide model's lanes launch (csrc/solver/wide_solver.h WideLanes)
from the device's s_memrealtime stamps (PSX_WIDE_STAMPS=1, 100 MHz): per lane, the
last solve's prefix (begin .. prep), every slot's forward+backward, dot products and
controller, and the finalisation.  One JSON line per lane on stdout.

    PSX_WIDE_STAMPS=1 python tools/wide_lanes_profile.py --workers 8 --iters 20
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workers", type=int, default=8)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--train-rows", type=int, default=400_000)
    ap.add_argument("--features", type=int, default=1 << 20)
    a = ap.parse_args()
    os.environ.setdefault("PSX_WIDE_STAMPS", "1")
    import torch

    from psx.ops.lr import SolverOptions, stream_handle
    from psx.runtime.config import PSConfig
    from psx.runtime.engine import LocalEngine
    from psx.utils.data import synth_sparse

    kw = dict(num_features=a.features, labels="finefood", nnz_mean=48, max_nnz=128, device="cuda:0")
    train, test = synth_sparse(a.train_rows, seed=0, **kw), synth_sparse(20000, seed=1, **kw)
    cfg = PSConfig(num_workers=a.workers, consistency_model=-1, producer_time_per_event=0, stream_mode="per_iter",
                   rows_per_iter=64, epochs=1000, max_iters=a.iters, min_buffer_size=128, max_buffer_size=1024,
                   init="random", model="wide", solver=SolverOptions(iters=2, zero_const=False))
    eng = LocalEngine(cfg, "cuda:0", train=train, test=test)
    out = eng.run()
    torch.cuda.synchronize()
    s = stream_handle("cuda:0")
    for w in eng.workers:
        st = w.solver._native.read_stamps(s)
        t0 = st[7]
        us = lambda t: round((t - t0) / 100.0, 2) if t else None  # noqa: E731
        slots = []
        for k in range(len(st) // 8):
            row = st[8 * k: 8 * k + 8]
            if not row[6] or row[6] < t0:
                break
            slots.append({"fwd": us(row[6]), "dots": us(row[0]), "last_in": us(row[1]), "ctrl_done": us(row[5])})
        prefix = {"planned": us(st[23]), "assigned": us(st[31]), "stats": us(st[39]), "prepared": us(st[47])}
        print(json.dumps({"worker": w.k, "U": w.solver.host_count(), "prefix": prefix, "slots": slots,
                          "finalize": us(st[15]),
                          "wide_lanes": out.get("wide_lanes")}))


if __name__ == "__main__":
    main()
