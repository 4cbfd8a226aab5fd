"""Server + worker checkpoint / resume (new capability: the
reference loses its weights on restart, ServerProcessor.java:35,57,188-191,
and only Kafka offsets survive).

``server.ckpt`` holds the fp32 master weights (device layout; for the dense
model also the reference's flat column-major layout), the model shape, the
tracker's vector clocks / "sent" / "live" flags and the update count.
``worker<k>.ckpt`` holds worker k's stream cursor (the producer offset the run
replays from), its sliding-window state and the buffered rows themselves, so a
resumed run continues exactly where the checkpoint was taken.

Off the hot path: the weights (up to 10^8 x KP floats for the wide model) are
copied device->pinned host on a side stream ordered after the update that
produced them, and a background thread waits for that copy and writes the
file (temp file + atomic rename: a crash never leaves a torn checkpoint).
Files are plain tensors/ints read back with ``torch.load(weights_only=True)``.
"""
from __future__ import annotations

import os
import threading

import torch

from ..models.logreg import ModelSpec, to_reference_layout

CKPT_NAME = "server.ckpt"
FORMAT = 2


def worker_ckpt_name(k: int) -> str:
    return f"worker{int(k)}.ckpt"


def _spec_meta(spec) -> dict:
    wide = not isinstance(spec, ModelSpec)
    return {"model": "wide" if wide else "dense", "num_features": int(spec.F), "num_classes": int(spec.K)}


def _atomic_save(state: dict, final: str) -> str:
    tmp = final + ".tmp"
    torch.save(state, tmp)
    os.replace(tmp, final)
    return final


class _HostCopy:
    """D2H snapshot of a device tensor, off the hot path.

    The tensor is first cloned on the PRODUCING stream (an HBM-speed device copy
    ordered right after the update that produced it), and the pinned-host copy
    then reads that clone on a side stream.  The next update on the producing
    stream can therefore rewrite the tensor at once without tearing the snapshot
    (the clone is only reused after the previous write finished: Checkpointer.submit
    waits for it)."""

    def __init__(self):
        self.buf = None
        self.dev = None
        self.event = None

    def start(self, t: torch.Tensor) -> torch.Tensor:
        if t.device.type != "cuda":
            self.event = None
            return t.detach().clone()
        flat = t.detach().view(-1)
        if self.buf is None or self.buf.numel() != t.numel() or self.buf.dtype != t.dtype:
            self.buf = torch.empty(t.numel(), dtype=t.dtype, pin_memory=True)
            self.dev = torch.empty_like(flat)
        main = torch.cuda.current_stream(t.device)
        self.dev.copy_(flat)  # snapshot in stream order: before the next update of t
        side = _side_stream(t.device)
        ready = torch.cuda.Event()
        ready.record(main)
        side.wait_event(ready)
        with torch.cuda.stream(side):
            self.buf.copy_(self.dev, non_blocking=True)
            self.event = torch.cuda.Event()
            self.event.record(side)
        return self.buf

    def wait(self):
        if self.event is not None:
            self.event.synchronize()


_SIDE = {}


def _side_stream(device):
    key = torch.device(device).index or 0
    if key not in _SIDE:
        _SIDE[key] = torch.cuda.Stream(device)
    return _SIDE[key]


class Checkpointer:
    """One checkpoint in flight at a time; ``wait()`` drains it."""

    def __init__(self):
        self._thread = None
        self._copy = _HostCopy()
        self.written = []

    def wait(self):
        if self._thread is not None:
            self._thread.join()
            self._thread = None

    def submit(self, path_dir: str, server=None, workers=(), extra: dict | None = None, sync: bool = False):
        self.wait()  # the pinned buffer is reused: the previous write must be done
        os.makedirs(path_dir, exist_ok=True)
        jobs = []
        if server is not None:
            spec = server.spec
            w_host = self._copy.start(server.w)
            tr = server.tracker
            meta = {
                "format": FORMAT,
                **_spec_meta(spec),
                "clocks": torch.tensor(tr.clocks(), dtype=torch.int64),
                "sent": torch.tensor(tr.sent_flags(), dtype=torch.uint8),
                "live": torch.tensor([1 if tr.is_live(k) else 0 for k in range(tr.num_workers)], dtype=torch.uint8),
                "updates": int(server.updates),
                "consistency_model": int(tr.consistency_model),
            }
            if extra:
                meta["extra"] = {k: v for k, v in extra.items() if isinstance(v, (int, float, str))}
            jobs.append(("server", meta, w_host, spec))
        for wk in workers:  # small: cursor, window, ring rows (synchronous device copies)
            jobs.append(("worker", wk.k, worker_state(wk), None))

        def write():
            self._copy.wait()
            for kind, a, b, spec in jobs:
                if kind == "server":
                    state = dict(a)
                    state["w"] = b.clone()
                    if isinstance(spec, ModelSpec):
                        state["w_reference_layout"] = to_reference_layout(spec, state["w"])
                    self.written.append(_atomic_save(state, os.path.join(path_dir, CKPT_NAME)))
                else:
                    self.written.append(_atomic_save(b, os.path.join(path_dir, worker_ckpt_name(a))))

        if sync:
            write()
        else:
            self._thread = threading.Thread(target=write, daemon=True)
            self._thread.start()


def worker_state(wk) -> dict:
    ring = wk.ring
    if hasattr(ring, "flush"):
        ring.flush()  # a deferred ingest belongs to the saved rows
    tensors = {}
    for name in ("X", "y", "idx", "val", "nnz"):
        t = getattr(ring, name, None)
        if isinstance(t, torch.Tensor):
            tensors["ring_" + name] = t.detach().cpu().clone()
    return {
        "format": FORMAT,
        "worker": int(wk.k),
        "vc": int(wk.vc),
        "iters": int(wk.iters),
        "next_local": int(wk.source.next_local),
        "window_head": int(wk.window.head),
        "window_size": int(wk.window.size),
        "tuples_seen": int(wk.window.tuples_seen),
        "seen_at_solve": int(getattr(wk, "_seen_at_solve", 0)),  # the tuple cadence's origin
        **tensors,
    }


def restore_worker(wk, state: dict) -> None:
    ring = wk.ring
    if hasattr(ring, "pending"):
        ring.pending = None  # superseded by the restored rows
    for name in ("X", "y", "idx", "val", "nnz"):
        key = "ring_" + name
        if key in state:
            getattr(ring, name).copy_(state[key].to(getattr(ring, name).device))
    if hasattr(ring, "sync_transposed"):
        ring.sync_transposed()
    wk.window.restore(int(state["window_head"]), int(state["window_size"]), int(state["tuples_seen"]))
    wk.source.next_local = int(state["next_local"])
    wk.vc = int(state["vc"])
    wk.iters = int(state["iters"])
    wk._seen_at_solve = int(state.get("seen_at_solve", 0))


# ---- compatibility helpers (synchronous) -------------------------------------
def save_server(path_dir: str, server, extra: dict | None = None) -> str:
    ck = Checkpointer()
    ck.submit(path_dir, server, (), extra, sync=True)
    return os.path.join(path_dir, CKPT_NAME)


def load_server(path_dir: str) -> dict:
    return torch.load(os.path.join(path_dir, CKPT_NAME), map_location="cpu", weights_only=True)


def restore_server(server, state: dict) -> None:
    spec = server.spec
    if state["num_features"] != spec.F or state["num_classes"] != spec.K:
        raise ValueError("checkpoint model shape does not match the data")
    if state.get("model", "dense") != _spec_meta(spec)["model"]:
        raise ValueError("checkpoint was written by the other model kind (dense vs wide)")
    server.w.copy_(state["w"].to(server.w.device))
    if server.frag is not None:
        server.frag.refresh(server.w)
    server.tracker.restore(state["clocks"].tolist(), state["sent"].tolist())
    live = state.get("live")
    if live is not None:
        for k, flag in enumerate(live.tolist()):
            if not flag:
                server.tracker.retire(k)
    server.updates = int(state["updates"])


_CKPTS: dict = {}


def _checkpointer(cfg) -> Checkpointer:
    key = id(cfg)
    if key not in _CKPTS:
        _CKPTS[key] = Checkpointer()
    return _CKPTS[key]


def maybe_checkpoint(cfg, server, step: int, workers=()) -> None:
    """Every ``checkpoint_every`` steps: asynchronous server (+ worker) checkpoint."""
    if cfg.checkpoint_dir and cfg.checkpoint_every and step % cfg.checkpoint_every == 0:
        _checkpointer(cfg).submit(cfg.checkpoint_dir, server, workers, {"step": step})


def flush_checkpoints(cfg) -> None:
    ck = _CKPTS.get(id(cfg))
    if ck is not None:
        ck.wait()


def maybe_resume(cfg, server, workers=()) -> bool:
    """Restore the server (if given) and every worker that has a checkpoint file."""
    if not (cfg.resume and cfg.checkpoint_dir):
        return False
    found = False
    if server is not None and os.path.exists(os.path.join(cfg.checkpoint_dir, CKPT_NAME)):
        restore_server(server, load_server(cfg.checkpoint_dir))
        found = True
    for wk in workers:
        p = os.path.join(cfg.checkpoint_dir, worker_ckpt_name(wk.k))
        if os.path.exists(p):
            restore_worker(wk, torch.load(p, map_location="cpu", weights_only=True))
            found = True
    return found
