"""Server checkpoint / resume (new capability; the reference loses its weights
on restart: ServerProcessor.java:35,57,188-191).

A checkpoint holds the fp32 master weights (device layout, plus a copy in the
reference's flat column-major layout), the model shape, the vector clocks and
"sent" flags of the tracker and the update count.  It is written with
``torch.save`` of plain tensors/ints and read back with ``weights_only=True``.
Writes go to a temp file + atomic rename so a crash never leaves a torn file.
"""
from __future__ import annotations

import os

import torch

from ..models.logreg import to_reference_layout

CKPT_NAME = "server.ckpt"


def save_server(path_dir: str, server, extra: dict | None = None) -> str:
    os.makedirs(path_dir, exist_ok=True)
    spec = server.spec
    w = server.w.detach().float().cpu()
    state = {
        "format": 1,
        "num_features": spec.F,
        "num_classes": spec.K,
        "w": w,
        "w_reference_layout": to_reference_layout(spec, w),
        "clocks": torch.tensor(server.tracker.clocks(), dtype=torch.int64),
        "sent": torch.tensor(server.tracker.sent_flags(), dtype=torch.uint8),
        "updates": int(server.updates),
        "consistency_model": int(server.tracker.consistency_model),
    }
    if extra:
        state["extra"] = {k: v for k, v in extra.items() if isinstance(v, (int, float, str))}
    final = os.path.join(path_dir, CKPT_NAME)
    tmp = final + ".tmp"
    torch.save(state, tmp)
    os.replace(tmp, final)
    return final


def load_server(path_dir: str) -> dict:
    return torch.load(os.path.join(path_dir, CKPT_NAME), map_location="cpu", weights_only=True)


def restore_server(server, state: dict) -> None:
    spec = server.spec
    if state["num_features"] != spec.F or state["num_classes"] != spec.K:
        raise ValueError("checkpoint model shape does not match the data")
    server.w.copy_(state["w"].to(server.w.device))
    if server.frag is not None:
        server.frag.refresh(server.w)
    server.tracker.restore(state["clocks"].tolist(), state["sent"].tolist())
    server.updates = int(state["updates"])


def maybe_checkpoint(cfg, server, step: int) -> None:
    if cfg.checkpoint_dir and cfg.checkpoint_every and step % cfg.checkpoint_every == 0:
        save_server(cfg.checkpoint_dir, server, {"step": step})


def maybe_resume(cfg, server) -> bool:
    if cfg.resume and cfg.checkpoint_dir and os.path.exists(os.path.join(cfg.checkpoint_dir, CKPT_NAME)):
        restore_server(server, load_server(cfg.checkpoint_dir))
        return True
    return False
