"""The peer_sum hand-off, split at the server kernel's stamps: PSX_LANES_TRACE_OUT=path runs
write the lanes kernels' per-round device stamps and (rank 0) the server kernel's per-command
stamps {command, read, applied, evaluated} into path.rank0 / path.rank<r>; all are
s_memrealtime ticks (10 ns) of one GPU when the server and the lanes share it (the colocated
rank 0, or the one-GPU rehearsals).  Per round k: the interval between the rounds' first
stages, the hand-off (last lane's push of round k -> round k + 1's first stage), and its parts
-- push -> the server's apply of round k, apply -> the next stage, and the server row's
evaluation after the apply.

    python tools/psum_handoff.py gpurun_out/x/trace.rank0 [--skip 10]
"""
from __future__ import annotations

import argparse
import bisect
import json


def load(path):
    rows, srv = [], []
    with open(path) as fh:
        for line in fh:
            if not line.strip():
                continue
            d = json.loads(line)
            rows += [r for r in d.get("rows", []) if r[0] == 0 and min(r[4:8]) > 0]
            srv += d.get("server", [])
    return rows, sorted(srv)


def split(rows, srv, skip=10):
    rounds = {}
    for r in rows:
        rounds.setdefault(int(r[1]), []).append(r)
    keys = sorted(rounds)[skip:]
    push = {k: max(x[7] for x in rounds[k]) for k in keys}
    stage = {k: min(x[4] for x in rounds[k]) for k in keys}
    app = [s[2] for s in srv]
    ev = [s[3] for s in srv]
    cols = {"interval": [], "handoff": [], "push->applied": [], "applied->next_stage": [], "applied->evaluated": []}
    for k in keys:
        if k + 1 not in stage:
            continue
        cols["interval"].append((stage[k + 1] - stage[k]) / 100.0)
        cols["handoff"].append((stage[k + 1] - push[k]) / 100.0)
        i = bisect.bisect_left(app, push[k])  # the first server apply after the round's last push
        if i < len(app):
            cols["push->applied"].append((app[i] - push[k]) / 100.0)
            cols["applied->next_stage"].append((stage[k + 1] - app[i]) / 100.0)
            cols["applied->evaluated"].append((ev[i] - app[i]) / 100.0)
    out = {"rounds": len(cols["interval"])}
    for name, v in cols.items():
        if v:
            v = sorted(v)
            out[name] = {"median": round(v[len(v) // 2], 2), "p10": round(v[len(v) // 10], 2),
                         "p90": round(v[(9 * len(v)) // 10], 2)}
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("paths", nargs="+")
    ap.add_argument("--skip", type=int, default=10)
    a = ap.parse_args(argv)
    for p in a.paths:
        rows, srv = load(p)
        print(json.dumps({"file": p, **split(rows, srv, a.skip)}))


if __name__ == "__main__":
    main()
