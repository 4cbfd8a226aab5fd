"""One rank of the shared-GPU multi-rank rehearsal (tests/test_gpu_ipc_lanes.py):
DistEngine's BSP lanes loop with a dedicated server rank and worker ranks of 4
lanes each, every rank on GPU 0 (PSX_GPU_OVERSUBSCRIBE=1: gloo control plane,
the IPC transport of csrc/comm/ipc_comm.h for the round's reduce + broadcast).

usage: python tests/_ipc_rank.py <out_dir> <bounded|vote>   (torchrun-style env)"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def cfg_for(world: int, mode: str):
    from psx.runtime.config import PSConfig

    if mode == "peer_sum_colo2":
        # (one-off rehearsal, PSX_PSUM_REHEARSE_MULTI=1) the colocated form across two ranks:
        # rank 0 = the server kernel + 3 lanes, rank 1 = 3 lanes pushing into inbox slot 1
        return PSConfig(num_workers=6, consistency_model=0, producer_time_per_event=0,
                        stream_mode="per_iter", rows_per_iter=1024, epochs=1000, max_iters=6,
                        min_buffer_size=128, max_buffer_size=1024, init="random", seed=0, server_colocated=True,
                        workers_per_rank=3, bsp_schedule="peer_sum", worker_timeout_s=20.0, idle_wait_s=20.0)
    if mode in ("peer_sum_colo", "peer_sum_colo_vote"):
        # peer_sum with the server colocated, world 1: rank 0's server kernel (XCD 7) + its own
        # 7 lanes (XCDs 0-6) in ONE process -- the server's command thread beside the lanes loop
        vote = mode.endswith("_vote")
        return PSConfig(num_workers=7, consistency_model=0, producer_time_per_event=0,
                        stream_mode="per_iter", rows_per_iter=1024, epochs=1000, max_iters=0 if vote else 6,
                        max_wallclock_s=1.5 if vote else 0.0, min_buffer_size=128, max_buffer_size=1024,
                        init="random", seed=0, server_colocated=True, workers_per_rank=7, bsp_schedule="peer_sum",
                        worker_timeout_s=20.0, idle_wait_s=20.0)
    if mode in ("peer_sum", "peer_sum_vote"):
        # BSP with rank-level sums over the peer data plane (--bsp_schedule peer_sum): 1 GPU server
        # rank + one worker rank x 6 lanes, no collective per round; _vote: an unbounded run (1.5 s)
        vote = mode == "peer_sum_vote"
        return PSConfig(num_workers=(world - 1) * 6, consistency_model=0, producer_time_per_event=0,
                        stream_mode="per_iter", rows_per_iter=1024, epochs=1000, max_iters=0 if vote else 6,
                        max_wallclock_s=1.5 if vote else 0.0, min_buffer_size=128, max_buffer_size=1024,
                        init="random", seed=0, server_colocated=False, workers_per_rank=6, bsp_schedule="peer_sum",
                        worker_timeout_s=20.0, idle_wait_s=20.0)
    if mode == "peer_bsp":  # sequential consistency over the peer data plane: 1 GPU server + ranks x 3 lanes
        return PSConfig(num_workers=(world - 1) * 3, consistency_model=0, producer_time_per_event=0,
                        stream_mode="per_iter", rows_per_iter=1024, epochs=1000, max_iters=6, min_buffer_size=128,
                        max_buffer_size=1024, init="random", seed=0, server_colocated=False, workers_per_rank=3,
                        bsp_schedule="peer", worker_timeout_s=20.0)
    if mode.startswith("async") or mode.startswith("peer"):
        # SSP(2) / ASP: 1 server rank + worker ranks x 3 lanes -- async_*: a CPU server and
        # the host shared-memory data plane; peer_*: a GPU server rank and the peer data
        # plane (csrc/comm/peer_bus.h), worker 1 a straggler (+2 ms per iteration)
        c = -1 if mode.endswith("_asp") else 2
        peer = mode.startswith("peer")
        return PSConfig(num_workers=(world - 1) * 3, consistency_model=c, producer_time_per_event=0,
                        stream_mode="per_iter", rows_per_iter=1024, epochs=1000, max_iters=8, min_buffer_size=128,
                        max_buffer_size=1024, init="random", seed=0, server_colocated=False, workers_per_rank=3,
                        async_plane="peer" if peer else "host", inject_worker_delay_ms={1: 2.0} if peer else {},
                        worker_timeout_s=25.0)  # (a stuck transport raises with its reason, inside the test's limit)
    return PSConfig(num_workers=(world - 1) * 4, consistency_model=0, producer_time_per_event=0,
                    stream_mode="per_iter", rows_per_iter=1024, epochs=1000,
                    max_iters=6 if mode == "bounded" else 0, max_wallclock_s=0.0 if mode == "bounded" else 1.5,
                    min_buffer_size=128, max_buffer_size=1024, init="random", seed=0, server_colocated=False,
                    bsp_schedule="reduce_bcast", workers_per_rank=4)


def main():
    out_dir, mode = sys.argv[1], sys.argv[2]
    import faulthandler

    # a hang names its frames (before the test's limit; the peer modes' native timeouts first)
    faulthandler.dump_traceback_later(100 if mode.startswith("peer") else 80, exit=True)
    import torch
    import torch.distributed as dist

    from psx.parallel.dist import DistEngine, init_from_env
    from psx.utils.data import synth_finefood

    os.environ.setdefault("PSX_PSUM_DIAG", "1")
    rank, world, device = init_from_env()
    if mode.startswith("async") and rank == 0:  # (see test_async_lanes_worker_ranks; peer_*: a GPU server)
        device = torch.device("cpu")
    train, test = synth_finefood(20000, seed=0), synth_finefood(4877, seed=1)
    eng = DistEngine(cfg_for(world, mode), rank, world, device, train=train, test=test)
    kind = None
    out = eng.run()
    res = {"rank": rank, "rounds": int(eng.rounds),
           "lanes": getattr(eng, "_lanes", None) is not None or bool(out.get("lanes")), "updates": out.get("updates")}
    for key in ("data_plane", "host_us_per_update", "elapsed_s"):
        if key in out:
            res[key] = out[key]
    if rank == 0:
        torch.save(eng.server.w.detach().cpu(), os.path.join(out_dir, f"w_{mode}.pt"))
        res["server_rows"] = [[float(r[1]), float(r[2]), float(r[3])] for r in eng.log.book.server]
        res["max_vc_gap"] = out.get("max_vc_gap")
        ps = getattr(eng, "_pserver", None)
        if ps is not None:
            res["arrivals"] = [list(a) for a in ps.arrivals]
    else:
        res["async_lanes"] = bool(out.get("async_lanes"))
    if rank > 0 and mode.startswith("peer_sum"):  # (diagnostics) receive / push slice tags after the run
        res["psum_tags"] = getattr(eng, "_psum_tags", None)
    with open(os.path.join(out_dir, f"{mode}_rank{rank}.json"), "w") as fh:
        json.dump(res, fh)
    print("result:", json.dumps({k: v for k, v in res.items() if k != "server_rows"}), flush=True)
    dist.barrier()
    dist.destroy_process_group()
    del kind


if __name__ == "__main__":
    main()
