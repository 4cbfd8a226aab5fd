"""Device time of the evaluation kernel variants (one MI355X): single model,
paired (shared buffer), paired from two buffers, paired + fused server update."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from psx.models.logreg import ModelSpec  # noqa: E402
from psx.ops.lr import EvalScratch, EvalSet, Fragments  # noqa: E402
from psx.utils.data import synth_finefood  # noqa: E402
from psx.utils.logsink import LogSink  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    spec = ModelSpec(1024, 6)
    te = synth_finefood(4877, seed=1)
    ev = EvalSet(spec, te.X, te.y, dev)
    g = torch.Generator().manual_seed(0)
    w = (torch.randn(spec.P, generator=g) * 0.1).to(dev)
    fa = Fragments(spec, dev)
    fa.refresh(w)
    sb = Fragments(spec, dev, coff=16 - spec.K)
    sa = Fragments(spec, dev, coff=0, share=sb)
    sb.refresh(w)
    sa.refresh(w)
    cur, nxt = Fragments(spec, dev, coff=16 - spec.K), Fragments(spec, dev, coff=16 - spec.K)
    cur.refresh(w)
    d = torch.zeros(spec.P, device=dev)
    log = LogSink(spec.K, dev)
    sc = EvalScratch(dev)
    loss = torch.zeros(1, device=dev)
    n = int(os.environ.get("N", "500"))
    cases = {
        "single": lambda: log.worker_eval(ev, fa, w, sc, loss, 0, 0, 0),
        "paired shared buffer": lambda: log.pair_eval(ev, sa, w, loss, 0, 0, 0, sb, w, 0, 0, sc),
        "paired two buffers": lambda: log.pair_eval(ev, fa, w, loss, 0, 0, 0, cur, w, 0, 0, sc),
        "paired + fused update": lambda: log.pair_eval(ev, fa, w, loss, 0, 0, 0, cur, w, 0, 0, sc,
                                                       apply=(w, [d], 1.0, nxt)),
        "paired, fresh fragments": lambda: (fa.refresh(w), cur.refresh(w),
                                            log.pair_eval(ev, fa, w, loss, 0, 0, 0, cur, w, 0, 0, sc)),
    }
    for name, fn in cases.items():
        for _ in range(20):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n):
            fn()
        e1.record()
        torch.cuda.synchronize()
        print(f"{name:28s} {1000 * e0.elapsed_time(e1) / n:8.2f} us/launch (back to back)", flush=True)
    log.close()


if __name__ == "__main__":
    main()
