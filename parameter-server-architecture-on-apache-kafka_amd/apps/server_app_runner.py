"""ServerAppRunner -- rank 0 of the parameter server (reference:
src/main/java/de/hpi/datastreams/apps/ServerAppRunner.java:14-102).

Modes:
* distributed (default): this process is the server rank 0 of a world of
  1 + num_workers ranks; ``WorkerAppRunner`` starts the worker ranks (one per
  GPU).  The reference's 20 s / 10 s startup sleeps are replaced by the
  torch.distributed rendezvous; the server broadcasts its run configuration
  (training data, producer rate, consistency model, solver) to the workers.
* ``--inprocess``: server + all workers in this process on one device
  (single MI355X or CPU).

Usage: python -m psx.apps.server_app_runner [-training F] [-test F] [-c C] [-p P] [-v] [-l] ...
"""
from __future__ import annotations

import json
import os
import sys

import torch

from .cli import parse_or_exit, print_params, server_config, server_parser


def _device(a):
    if a.device:
        return a.device
    return "cuda:0" if torch.cuda.is_available() else "cpu"


def main(argv=None) -> int:
    a = parse_or_exit(server_parser(), sys.argv[1:] if argv is None else argv)
    cfg = server_config(a)
    remote_host = os.environ.get("PSX_REMOTE_HOST", "kafka") if a.remote else "127.0.0.1"
    if a.verbose:
        print_params("server", {
            "training_data_file_path": cfg.train_path,
            "test_data_file_path": cfg.test_path,
            "consistency_model": cfg.consistency_model,
            "producer_time_per_event": cfg.producer_time_per_event,
            "rendezvous address": f"{remote_host}:{a.master_port or os.environ.get('MASTER_PORT', 29500)}",
            "num_workers": cfg.num_workers,
            "mode": "in-process" if a.inprocess else "distributed",
        })
    device = _device(a)
    if a.inprocess:
        from ..runtime.engine import LocalEngine

        out = LocalEngine(cfg, device).run()
    else:
        import torch.distributed as dist

        from ..parallel.dist import DistEngine, init_from_env, rccl_trace_env

        if a.rccl_trace:
            os.environ.update(rccl_trace_env(a.log_dir))
        os.environ["RANK"] = "0"
        os.environ["LOCAL_RANK"] = str(torch.device(device).index or 0) if device.startswith("cuda") else "0"
        os.environ["WORLD_SIZE"] = str(cfg.num_workers + 1)
        os.environ["MASTER_ADDR"] = remote_host
        if a.master_port:
            os.environ["MASTER_PORT"] = str(a.master_port)
        rank, world, dev = init_from_env(cpu=device == "cpu")
        payload = [cfg.to_dict()]
        dist.broadcast_object_list(payload, src=0)
        eng = None
        try:
            eng = DistEngine(cfg, rank, world, dev)
            out = eng.run()
        finally:
            if eng is not None:  # the control / data planes (IPC maps, shm queues, server launch) even on failure
                eng.close()
            dist.destroy_process_group()
    if a.verbose or not a.logging:
        print(json.dumps({k: (float(v) if hasattr(v, "item") else v) for k, v in out.items()}), file=sys.stderr)
    return 0


if __name__ == "__main__":
    sys.exit(main())
