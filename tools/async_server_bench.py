"""Host cost and throughput of the native SSP/ASP server loop on one MI355X
(LocalP2P transport + stand-in workers: the server side of configs 3/4 in
isolation).  Prints one JSON line per configuration.

    python tools/async_server_bench.py [--iters 3000] [--out profiles/.../async_server.json]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=3000)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from psx.parallel.async_local import LocalAsyncHarness
    from psx.utils.data import synth_finefood

    test = synth_finefood(4877, seed=1)
    rows = []
    for n, c in ((1, -1), (4, -1), (7, -1), (7, 3), (7, 0)):
        hs = LocalAsyncHarness(n, c, test=test)
        try:
            hs.run(50)  # warm-up (kernels, queues)
            r = hs.run(a.iters)
        finally:
            hs.close()
        r.update(workers=n, consistency=c, iters_per_worker=a.iters)
        rows.append(r)
        print(json.dumps(r), flush=True)
    if a.out:
        os.makedirs(os.path.dirname(a.out), exist_ok=True)
        with open(a.out, "w") as fh:
            json.dump(rows, fh, indent=1)


if __name__ == "__main__":
    main()
