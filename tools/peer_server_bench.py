"""Ceiling of the peer data plane's asynchronous server (PeerServer + server_persist_kernel)
on one MI355X: N stand-in workers whose inbox slots are pre-armed (every slice tag far
ahead), so every delta is ready when its command arrives; the host runs the real C++
tracker (ASP: each delta releases its own worker), writes the commands -- one per delta,
or batches of B (kSrvBatch) -- and the kernel applies them slice-parallel, in order, and
writes every release's receive slot.  No reply queues.  Reports applied deltas/s, us per
delta and the host's share, per batch size; --rows adds the server rows (worker 0's
deltas, the MFMA test-set pass on the server kernel's workgroups).

Reference: ServerProcessor.java:143-183 (one GRADIENTS_TOPIC partition: deltas applied
serially in arrival order, the released workers answered right after each update).

    python tools/peer_server_bench.py --workers 56 --deltas 20000 --batch 1 8 16 32 [--rows]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(N: int, deltas: int, batch: int, rows: bool, nwg: int):
    import torch

    from psx import _native
    from psx.models.logreg import ModelSpec
    from psx.ops.lr import EvalSet
    from psx.utils.data import synth_finefood
    from psx.utils.logsink import LogSink

    h, host = _native.hip(), _native.host
    dev = torch.device("cuda:0")
    spec = ModelSpec(1024, 6)
    NS = spec.Fp // 32
    inbox = h.PeerRegion(spec.P, NS, N, 0)
    inbox.fill_tags(0x7FFFFFFF)  # every delta of every worker "arrived"
    rx = h.PeerRegion(spec.P, NS, N, 0)
    tracker = host.VectorClockTracker(N, -1)
    w = torch.zeros(spec.P, dtype=torch.float32, device=dev)
    d = dict(nworkers=N, lr=1.0 / N, K=spec.K, F=spec.F, FP=spec.Fp, P=int(spec.P), w=w.data_ptr(), inbox=inbox.base,
             rx=[rx.data(j) for j in range(N)], rx_tag=[rx.tags(j) for j in range(N)], api=host.capi(),
             tracker=tracker.handle, standin=1, batch=batch, nwg=nwg, worker_timeout_s=60.0)
    keep = []
    if rows:
        test = synth_finefood(4877, seed=1)
        ev = EvalSet(spec, test.X, test.y, dev)
        log = LogSink(spec.eval_classes, dev)
        keep += [ev, log]
        d.update(sink=log.native.handle, Xt=ev.X.data_ptr(), yt=ev.y.data_ptr(), T=int(ev.T))
    ps = h.PeerServer(d)
    ps.warm_up()
    ps.bench_async(min(deltas, 2000))  # warm-up (the code object, the queues)
    t, th = ps.bench_async(deltas)
    torch.cuda.synchronize()
    out = {"workers": N, "deltas": deltas, "batch": batch, "nwg": nwg, "server_rows": rows,
           "deltas_per_s": round(deltas / t, 1), "us_per_delta": round(t * 1e6 / deltas, 3),
           "host_us_per_delta": round(th * 1e6 / deltas, 3),
           "deltas_per_command": round(ps.deltas_per_command, 2)}
    if rows:
        keep[1].close()
    del ps
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--workers", type=int, default=56)
    ap.add_argument("--deltas", type=int, default=20000)
    ap.add_argument("--batch", type=int, nargs="+", default=[1, 4, 8, 16, 32])
    ap.add_argument("--nwg", type=int, default=32)
    ap.add_argument("--rows", action="store_true")
    a = ap.parse_args(argv)
    for b in a.batch:
        print(json.dumps(run(a.workers, a.deltas, b, a.rows, a.nwg)), flush=True)


if __name__ == "__main__":
    main()
