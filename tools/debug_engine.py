"""Debug helper: run the bench configuration on CPU and GPU side by side and
report where the server weights diverge (max |w_gpu - w_cpu| per round), then
a longer GPU run with periodic metrics.  Usage: python tools/debug_engine.py"""
import sys

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
from psx.runtime.engine import LocalEngine  # noqa: E402
from psx.utils.data import synth_finefood  # noqa: E402


def make(device, rounds, a):
    train = synth_finefood(20000, seed=0)
    test = synth_finefood(1000, seed=1)
    cfg = bench.build_cfg(a, 1)
    cfg.max_iters = rounds
    return LocalEngine(cfg, device, train=train, test=test)


def main():
    a = bench.parse([])
    cpu = make("cpu", 1, a)
    gpu = make("cuda:0", 1, a)
    for r in range(int(sys.argv[1]) if len(sys.argv) > 1 else 12):
        for e in (cpu, gpu):
            e.log = bench._fresh_log(e)
            e.run()
        wg, wc = gpu.server.w.cpu(), cpu.server.w
        st = gpu.workers[0].solver.stats.cpu().tolist()
        stc = cpu.workers[0].solver.stats.tolist()
        print(f"round {r}: max|dw|={float((wg - wc).abs().max()):.3e} max|w|={float(wc.abs().max()):.3e} "
              f"nan={bool(torch.isnan(wg).any())} loss g/c={gpu.workers[0].solver.loss.item():.5f}/"
              f"{cpu.workers[0].solver.loss.item():.5f} stats g={st} c={stc} "
              f"acc g/c={gpu.log.book.server[-1][3]:.3f}/{cpu.log.book.server[-1][3]:.3f}", flush=True)
    g2 = make("cuda:0", 300, a)
    g2.run()
    for row in g2.log.book.server[::30]:
        print("gpu server", row)
    print("nan in w:", bool(torch.isnan(g2.server.w).any()), "max|w|", float(g2.server.w.abs().max()))


if __name__ == "__main__":
    main()
