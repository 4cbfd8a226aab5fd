"""Determinism check of the in-process BSP engine on one GPU: the same fixed-window
run repeated, with / without the riding evaluation (PSX_EVAL_RIDE).  Prints the
max |w_a - w_b| of the final server weights per pair of runs."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from psx.runtime.config import PSConfig  # noqa: E402
from psx.runtime.engine import LocalEngine  # noqa: E402
from psx.utils.data import synth_finefood  # noqa: E402


def run(ride: str, iters: int, N: int = 1):
    os.environ["PSX_EVAL_RIDE"] = ride
    train, test = synth_finefood(8000, seed=0), synth_finefood(1000, seed=1)
    cfg = PSConfig(num_workers=N, consistency_model=0, producer_time_per_event=0, stream_mode="per_iter",
                   rows_per_iter=128, epochs=1000, max_iters=iters, init="random", min_buffer_size=512,
                   max_buffer_size=512)
    eng = LocalEngine(cfg, "cuda:0", train=train, test=test)
    eng.run()
    torch.cuda.synchronize()
    return eng.server.w.cpu().clone(), [tuple(r[1:4]) for r in eng.log.book.server]


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    for it in (1, 2, 3, iters):
        a0, s0 = run("0", it)
        a1, s1 = run("0", it)
        b0, t0 = run("1", it)
        b1, t1 = run("1", it)
        d = lambda x, y: (x - y).abs().max().item()  # noqa: E731
        print(f"iters={it}: ride0 vs ride0 {d(a0, a1):.3e}  ride1 vs ride1 {d(b0, b1):.3e}  "
              f"ride1 vs ride0 {d(a0, b0):.3e}  rows equal: {s0 == s1} {t0 == t1} {s0 == t0}", flush=True)


if __name__ == "__main__":
    main()
