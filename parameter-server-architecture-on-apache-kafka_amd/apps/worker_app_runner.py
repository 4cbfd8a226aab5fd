"""WorkerAppRunner -- starts the worker ranks (reference:
src/main/java/de/hpi/datastreams/apps/WorkerAppRunner.java:13-94).

The reference hosts all logical workers as Kafka-Streams tasks of ONE JVM
(4 stream threads, BaseKafkaApp.java:70).  Here every worker is its own
process bound to its own GPU (worker i -> GPU first_gpu + i), joined to the
server's world as rank 1 + i.  Buffer flags (-min/-max/-bc) and the test set
are per-worker settings; everything else comes from the server's broadcast.

Usage: python -m psx.apps.worker_app_runner [-test F] [-min N] [-max N] [-bc X] [-v] [-l] [--num_workers N]
"""
from __future__ import annotations

import os
import sys

from .cli import parse_or_exit, print_params, worker_parser


def _worker_main(i: int, a_dict: dict, env: dict):
    os.environ.update(env)
    import torch
    import torch.distributed as dist

    from ..ops.lr import SolverOptions
    from ..parallel.dist import DistEngine, init_from_env
    from ..runtime.config import PSConfig

    n = a_dict["num_workers"]
    os.environ["RANK"] = str(1 + i)
    os.environ["WORLD_SIZE"] = str(1 + n)
    cpu = a_dict["device"] == "cpu" or not torch.cuda.is_available()
    if not cpu:
        ng = torch.cuda.device_count()
        os.environ["LOCAL_RANK"] = str((a_dict["first_gpu"] + i) % ng)
    rank, world, dev = init_from_env(cpu=cpu)
    payload = [None]
    dist.broadcast_object_list(payload, src=0)
    d = dict(payload[0])
    d["solver"] = SolverOptions(**d["solver"])
    cfg = PSConfig(**d)
    cfg.test_path = a_dict["test_data_file_path"]
    cfg.min_buffer_size = a_dict["min_buffer_size"]
    cfg.max_buffer_size = a_dict["max_buffer_size"]
    cfg.buffer_size_coefficient = a_dict["buffer_size_coefficient"]
    cfg.logging = cfg.logging or a_dict["logging"]
    eng = None
    try:
        eng = DistEngine(cfg, rank, world, dev)
        eng.run()
    finally:
        if eng is not None:  # the control / data planes (IPC maps, shm queues) even on failure
            eng.close()
        dist.destroy_process_group()


def main(argv=None) -> int:
    a = parse_or_exit(worker_parser(), sys.argv[1:] if argv is None else argv)
    if a.verbose:
        print_params("worker", {
            "test_data_file_path": a.test_data_file_path,
            "min_buffer_size": a.min_buffer_size,
            "max_buffer_size": a.max_buffer_size,
            "buffer_size_coefficient": a.buffer_size_coefficient,
            "num_workers": a.num_workers,
        })
    import torch.multiprocessing as mp

    env = {"MASTER_ADDR": os.environ.get("PSX_REMOTE_HOST", "kafka") if a.remote else "127.0.0.1"}
    if a.master_port:
        env["MASTER_PORT"] = str(a.master_port)
    elif "MASTER_PORT" in os.environ:
        env["MASTER_PORT"] = os.environ["MASTER_PORT"]
    if a.rccl_trace:
        from ..parallel.dist import rccl_trace_env

        env.update(rccl_trace_env(a.log_dir))
    a_dict = vars(a).copy()
    if a_dict["device"] is None:
        a_dict["device"] = "auto"
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_worker_main, args=(i, a_dict, env)) for i in range(a.num_workers)]
    for p in procs:
        p.start()
    rc = 0
    for p in procs:
        p.join()
        rc = max(rc, p.exitcode or 0)
    return rc


if __name__ == "__main__":
    sys.exit(main())
