"""Host enqueue cost of one local solve (no device sync inside the burst), by
variant: plain, with a riding evaluation pass, with the fused server update,
both.  Usage: python tools/launch_probe.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from psx.models.logreg import ModelSpec  # noqa: E402
from psx.ops.lr import EvalScratch, EvalSet, Fragments, LocalSolveOp, SolverOptions  # noqa: E402
from psx.runtime.buffer import DeviceRing  # noqa: E402
from psx.utils.data import synth_finefood  # noqa: E402
from psx.utils.logsink import LogSink  # noqa: E402


def main():
    dev = "cuda:0"
    spec = ModelSpec(1024, 6)
    ds = synth_finefood(1024, seed=0)
    te = synth_finefood(4877, seed=1)
    ring = DeviceRing(1024, spec.Fp, dev)
    ring.place(ds.X, ds.y)
    w = spec.init("random", seed=1).to(dev)
    op = LocalSolveOp(spec, 1024, dev, SolverOptions(use_graph=False))
    ev = EvalSet(spec, te.X, te.y, dev)
    sc = EvalScratch(dev)
    srv_frag = Fragments(spec, dev, coff=16 - spec.K)
    srv_frag.refresh(w)
    log = LogSink(spec.K, dev, pool=4096)
    wsrv = w.clone()
    n = int(os.environ.get("N", "50"))

    def ride():
        _, seq_w, addr_w = log.native.acquire()
        _, seq_s, addr_s = log.native.acquire()
        return ev.ride_args(op.frag, srv_frag, sc, addr_w, seq_w, op.loss, addr_s, seq_s)

    cases = {
        "plain": lambda: op.run(ring, 1024, 0, w),
        "ride": lambda: op.run(ring, 1024, 0, w, ride=ride()),
        "apply": lambda: op.run(ring, 1024, 0, w, apply=(wsrv, 1.0, srv_frag)),
        "ride+apply": lambda: op.run(ring, 1024, 0, w, ride=ride(), apply=(wsrv, 1.0, srv_frag)),
    }
    for name, fn in cases.items():
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"{name:12s} host {1e6 * (t1 - t0) / n:7.1f} us/solve  wall {1e6 * (t2 - t0) / n:7.1f} us/solve",
              flush=True)
    os._exit(0)  # the records were never submitted: skip the sink's flush


if __name__ == "__main__":
    main()
