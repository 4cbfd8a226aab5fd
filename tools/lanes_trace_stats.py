"""Per-round statistics of the BSP lanes loop's device phase stamps (PSX_LANES_TRACE_OUT=path:
the engines append one JSON line per call with LanesLoop.trace_take's rows; multi-rank runs
write path.rank<r>).  Each BSP row is {0, round, lane, worker, stage, solve, solved, updated}
in s_memrealtime ticks (10 ns).  Per round: the first lane's stage (round start), the slowest
lane's ingest (stage -> solve), solve (solve -> solved) and update (solved -> updated), and the
hand-off gap from the round's last update to the next round's first stage -- the push /
update / pull path (in process: the last lane's slice apply; peer_sum: the push into the
server GPU's inbox, the server kernel's update, the pull from the receive slot).

    python tools/lanes_trace_stats.py gpurun_out/x/trace.rank1 [--skip 20]
"""
from __future__ import annotations

import argparse
import json
import statistics


def load(path):
    rows = []
    with open(path) as fh:
        for line in fh:
            line = line.strip()
            if line:
                rows.extend(r for r in json.loads(line)["rows"] if r[0] == 0 and min(r[4:8]) > 0)
    return rows


def stats(rows, skip=0):
    rounds = {}
    for r in rows:
        d = rounds.setdefault(int(r[1]), [])
        d.append([int(x) for x in r[4:8]])
    keys = sorted(rounds)[skip:]
    out = {"rounds": len(keys)}
    if len(keys) < 2:
        return out
    us = lambda t: t / 100.0
    start = {k: min(x[0] for x in rounds[k]) for k in keys}
    last_upd = {k: max(x[3] for x in rounds[k]) for k in keys}
    per = {
        "interval": [us(start[b] - start[a]) for a, b in zip(keys, keys[1:]) if b == a + 1],
        "ingest": [us(max(x[1] - x[0] for x in rounds[k])) for k in keys],
        "solve": [us(max(x[2] - x[1] for x in rounds[k])) for k in keys],
        "update": [us(max(x[3] - x[2] for x in rounds[k])) for k in keys],
        "handoff": [us(start[b] - last_upd[a]) for a, b in zip(keys, keys[1:]) if b == a + 1],
        "first_to_last_updated": [us(last_upd[k] - start[k]) for k in keys],
    }
    for name, v in per.items():
        if v:
            v = sorted(v)
            out[name] = {"median": round(statistics.median(v), 2), "p10": round(v[len(v) // 10], 2),
                         "p90": round(v[(9 * len(v)) // 10], 2)}
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("paths", nargs="+")
    ap.add_argument("--skip", type=int, default=10, help="rounds skipped at the start of the file (warm-up)")
    a = ap.parse_args(argv)
    for p in a.paths:
        print(json.dumps({"file": p, **stats(load(p), a.skip)}))


if __name__ == "__main__":
    main()
