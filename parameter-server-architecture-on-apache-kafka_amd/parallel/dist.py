"""Multi-process parameter server over torch.distributed (RCCL on MI355X, gloo on CPU).

One process per GPU.  The reference's Kafka bus (BaseKafkaApp.java:27-33:
INPUT_DATA / WEIGHTS_TOPIC / GRADIENTS_TOPIC) becomes:

* data        -> every rank holds the dataset in its own HBM and takes its
                 round-robin shard (no cross-GPU traffic at all);
* push / pull -> RCCL collectives (BSP) or point-to-point send/recv plus a
                 shared-memory token queue (SSP/ASP), see below.

Sequential (BSP, c = 0) schedules, chosen with ``--bsp_schedule``:
  allreduce     every rank is a worker and holds a replica of the server
                state: ncclAllReduce(delta) then every replica applies the same
                w += lr * sum(delta) (deterministic, bitwise identical), rank 0
                evaluates and logs.  ONE collective per round -- the cheapest
                schedule on point-to-point xGMI (ring, per-link bound).
  reduce_bcast  the textbook PS: ncclReduce(delta -> server) then
                ncclBroadcast(w <- server).  Works with a dedicated server rank
                (contributes zeros) or a colocated one.
  sharded       key-range sharded server (new capability): every
                rank owns P/world of the master weights; ncclReduceScatter(delta)
                -> shard update -> ncclAllGather(w).

Bounded-delay (SSP, c = D > 0) and eventual (ASP, c = -1) need a dedicated
server rank 0 (workers are ranks 1..N).  A worker pushes a (worker, vc) token
into the shm control queue and ncclSend's its delta; the server pops tokens in
arrival order (= the single GRADIENTS_TOPIC partition), ncclRecv's from that
worker, applies, and ncclSend's the new weights to every worker the tracker
releases.  A worker always posts its recv right after its send and the server
only receives from workers whose token it has seen, so the send/recv graph is
acyclic (deadlock free).
"""
from __future__ import annotations

import json
import os
import time

import torch
import torch.distributed as dist

from .. import _native
from ..models.logreg import ModelSpec
from ..ops.lr import EvalSet, is_gpu
from ..runtime.config import PSConfig
from ..runtime.engine import load_datasets
from ..runtime.roles import ServerRole, WorkerRole
from ..utils.checkpoint import maybe_checkpoint, maybe_resume
from ..utils.logsink import LogSink, summarize
from ..utils.trace import Tracer

KIND_DELTA, KIND_FINAL = 0, 1


def init_from_env(cpu: bool = False):
    """Initialise torch.distributed from torchrun's env (RANK/WORLD_SIZE/LOCAL_RANK)."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29500")
    if cpu or not torch.cuda.is_available():
        device = torch.device("cpu")
        backend = "gloo"
    else:
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
        backend = "nccl"
    if not dist.is_initialized():
        kw = {"device_id": device} if backend == "nccl" else {}
        dist.init_process_group(backend=backend, rank=rank, world_size=world, **kw)
    return rank, world, device


def ctrl_queue_name() -> str:
    return f"/psx_ctrl_{os.environ.get('MASTER_PORT', '29500')}_{os.environ.get('TORCHELASTIC_RUN_ID', 'x')}"[:250]


class DistEngine:
    def __init__(self, cfg: PSConfig, rank: int, world: int, device, train=None, test=None):
        self.cfg, self.rank, self.world, self.device = cfg, rank, world, torch.device(device)
        self.async_mode = cfg.consistency_model != 0
        self.dedicated = self.async_mode or not cfg.server_colocated
        n_workers = world - 1 if self.dedicated else world
        if n_workers < 1:
            raise ValueError("need at least one worker rank (world size >= 2 with a dedicated server)")
        if cfg.num_workers != n_workers:
            cfg.num_workers = n_workers
        self.spec, train, test = load_datasets(cfg, train, test)
        self.is_server = rank == 0
        self.worker_id = (rank - 1) if self.dedicated else rank
        self.is_worker = self.worker_id >= 0
        self.evalset = EvalSet(self.spec, test.X, test.y, self.device) if test is not None else None
        wp = sp = None
        append = False
        if cfg.logging:
            # rank 0 creates both files (with the reference headers); worker ranks
            # then append whole lines to the shared logs-worker.csv
            wpath = f"{cfg.log_dir}/logs-worker.csv"
            if rank == 0:
                sp = f"{cfg.log_dir}/logs-server.csv"
                if self.is_worker:
                    wp = wpath
                else:
                    with open(wpath, "w") as fh:
                        fh.write("timestamp;partition;vectorClock;loss;fMeasure;accuracy;numTuplesSeen\n")
            elif self.is_worker:
                wp, append = wpath, True
            dist.barrier()
        # every rank evaluates (workers log their local model each iteration, as the
        # reference does); only files requested with -l are written
        self.log = LogSink(self.spec.K, self.device, wp, sp, keep_records=(rank == 0), worker_append=append)
        self.tracer = Tracer(cfg.trace_path.replace(".json", f".rank{rank}.json") if cfg.trace_path else None, rank)
        w0 = self.spec.init(cfg.init, seed=cfg.seed)
        # every rank keeps a server replica in the allreduce schedule; otherwise only rank 0
        replicated = (not self.async_mode) and cfg.bsp_schedule in ("allreduce", "sharded")
        self.server = ServerRole(self.spec, cfg, self.device, self.evalset, w0) if (self.is_server or replicated) else None
        if self.server is not None and self.is_server:
            maybe_resume(cfg, self.server)
        self.t0 = time.time()
        self.worker = None
        if self.is_worker:
            self.worker = WorkerRole(self.worker_id, self.spec, cfg, self.device, train.to(self.device), self.evalset,
                                     t0=self.t0)
        self.rounds = 0
        self._ctrl = None

    # ------------------------------------------------------------------
    def run(self) -> dict:
        if self.async_mode:
            out = self._run_async()
        else:
            out = self._run_bsp()
        if self.log is not None:
            self.log.close()
            if self.log.book is not None:
                out.update(summarize(self.log.book))
        self.tracer.close()
        return out

    def _all_ready(self) -> bool:
        flag = torch.tensor([1 if (self.worker is None or self.worker.ready()) else 0], dtype=torch.int32,
                            device=self.device)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        return bool(flag.item())

    def _agree_stop(self, rounds_done: int, t_start: float) -> bool:
        c = self.cfg
        if c.max_iters:
            return rounds_done >= c.max_iters
        local = 1 if (c.max_wallclock_s and time.time() - t_start >= c.max_wallclock_s) else 0
        if not c.max_wallclock_s and self.worker is not None and self.worker.source.exhausted:
            local = 1
        flag = torch.tensor([local], dtype=torch.int32, device=self.device)
        dist.all_reduce(flag, op=dist.ReduceOp.MAX)
        return bool(flag.item())

    # ------------------------------------------------------------------
    def _run_bsp(self) -> dict:
        cfg, spec = self.cfg, self.spec
        sched = cfg.bsp_schedule
        srv, wk = self.server, self.worker
        P = spec.P
        zeros = torch.zeros(P, dtype=torch.float32, device=self.device)
        if wk is not None:
            wk.w.copy_(srv.w if srv is not None else zeros)
        # bootstrap pull (vc 0): everybody starts from rank 0's weights
        boot = srv.w if srv is not None else (wk.w if wk is not None else zeros)
        dist.broadcast(boot, src=0)
        if srv is not None and srv.frag is not None:
            srv.frag.refresh(srv.w)
        if wk is not None:
            wk.w.copy_(boot)
        # wait until every worker has data
        while True:
            if wk is not None:
                wk.ingest()
            if self._all_ready():
                break
            time.sleep(0.001)
        shard = (P + self.world - 1) // self.world
        if sched == "sharded":
            pad = torch.zeros(shard * self.world, dtype=torch.float32, device=self.device)
            wfull = torch.zeros(shard * self.world, dtype=torch.float32, device=self.device)
            wfull[:P].copy_(srv.w)
            myd = torch.zeros(shard, dtype=torch.float32, device=self.device)
        N = cfg.num_workers
        lr = cfg.lr
        t_start = time.time()
        r = self.rounds
        check_every = 1 if not cfg.max_iters else 0
        while True:
            if cfg.max_iters and r - self.rounds >= cfg.max_iters:
                break
            if check_every and self._agree_stop(r - self.rounds, t_start):
                break
            with self.tracer.span("ingest"):
                if wk is not None:
                    wk.ingest()
            with self.tracer.span("solve"):
                delta = wk.compute(self.log) if wk is not None else zeros
            logged = False
            with self.tracer.span("comm", schedule=sched):
                if sched == "allreduce":
                    dist.all_reduce(delta, op=dist.ReduceOp.SUM)
                    if self.rank == 0:  # update + server eval row in one kernel
                        srv.apply_and_log(delta, r, self.log, lr)
                        logged = True
                    else:
                        srv.apply(delta, lr)
                    new_w = srv.w
                elif sched == "reduce_bcast":
                    dist.reduce(delta, dst=0, op=dist.ReduceOp.SUM)
                    if srv is not None:
                        srv.apply_and_log(delta, r, self.log, lr)
                        logged = True
                        new_w = srv.w
                    else:
                        new_w = wk.w
                    dist.broadcast(new_w, src=0)
                else:  # sharded
                    pad[:P].copy_(delta)
                    dist.reduce_scatter_tensor(myd, pad, op=dist.ReduceOp.SUM)
                    lo = self.rank * shard
                    wfull[lo:lo + shard].add_(myd, alpha=lr)
                    dist.all_gather_into_tensor(wfull, wfull[lo:lo + shard].clone())
                    srv.w.copy_(wfull[:P])
                    if srv.frag is not None:
                        srv.frag.refresh(srv.w)
                    new_w = srv.w
            if srv is not None:
                if self.rank == 0:
                    for k in range(N):
                        srv.tracker.received(k, r)
                    if not logged:
                        srv.log_eval(r, self.log)
                    for k in range(N):
                        srv.tracker.sent(k, r + 1)
                    maybe_checkpoint(cfg, srv, r + 1)
                srv.updates += N
            if wk is not None:
                if new_w is not wk.w:
                    wk.w.copy_(new_w)
                wk.vc = r + 1
            r += 1
            if self.log is not None:
                self.log.drain()
        if is_gpu(self.device):
            torch.cuda.synchronize(self.device)
        elapsed = time.time() - t_start
        self.rounds = r
        return {"rounds": r, "updates": r * N, "elapsed_s": elapsed,
                "updates_per_s": r * N / elapsed if elapsed > 0 else 0.0,
                "max_vc_gap": int(srv.tracker.max_gap) if (srv is not None and self.rank == 0) else 0}

    # ------------------------------------------------------------------
    def _open_ctrl(self):
        name = ctrl_queue_name()
        if self.rank == 0:
            self._ctrl = _native.host.CtrlQueue(name, 1024, True)
        dist.barrier()
        if self.rank != 0:
            self._ctrl = _native.host.CtrlQueue(name, 1024, False)
        dist.barrier()

    def _run_async(self) -> dict:
        self._open_ctrl()
        try:
            if self.is_server:
                return self._server_loop()
            return self._worker_loop()
        finally:
            dist.barrier()
            if self.rank == 0 and self._ctrl is not None:
                self._ctrl.unlink()

    def _server_loop(self) -> dict:
        cfg, srv = self.cfg, self.server
        N = cfg.num_workers
        buf = torch.zeros(self.spec.P, dtype=torch.float32, device=self.device)
        for j in range(N):  # bootstrap: vc 0 to every worker (tracker untouched)
            dist.send(srv.w, dst=j + 1)
        finished = set()
        t_start = time.time()
        while len(finished) < N:
            tok = self._ctrl.pop(600.0)
            if tok is None:
                raise TimeoutError("server: no worker token for 600 s (worker died?)")
            k, v = int(tok.worker), int(tok.vc)
            with self.tracer.span("recv", worker=k, vc=v):
                dist.recv(buf, src=k + 1)
            if k == 0:  # server eval rows follow worker-0 deltas (ServerProcessor.java:154-165)
                srv.apply_and_log(buf, v, self.log)
            else:
                srv.apply(buf)
            srv.updates += 1
            if tok.kind == KIND_FINAL:
                finished.add(k)
            for j, u in srv.tracker.on_delta(k, v):
                if j in finished:
                    continue
                dist.send(srv.w, dst=j + 1)
            maybe_checkpoint(cfg, srv, srv.updates)
            if self.log is not None:
                self.log.drain()
        if is_gpu(self.device):
            torch.cuda.synchronize(self.device)
        elapsed = time.time() - t_start
        return {"rounds": int(srv.tracker.min_clock()), "updates": srv.updates, "elapsed_s": elapsed,
                "updates_per_s": srv.updates / elapsed if elapsed > 0 else 0.0, "max_vc_gap": int(srv.tracker.max_gap)}

    def _worker_loop(self) -> dict:
        cfg, wk = self.cfg, self.worker
        tok = _native.host.CtrlToken()
        tok.worker = wk.k
        dist.recv(wk.w, src=0)
        wk.vc = 0
        max_iters = cfg.max_iters or 1 << 62
        t_start = time.time()
        it = 0
        while True:
            wk.ingest()
            while not wk.ready():
                time.sleep(0.001)
                wk.ingest()
            delta = wk.compute(self.log)
            it += 1
            final = it >= max_iters or (cfg.max_wallclock_s and time.time() - t_start >= cfg.max_wallclock_s) or (
                not cfg.max_iters and not cfg.max_wallclock_s and wk.source.exhausted)
            tok.vc = wk.vc
            tok.kind = KIND_FINAL if final else KIND_DELTA
            tok.aux = wk.tuples_seen
            if is_gpu(self.device):
                torch.cuda.current_stream(self.device).synchronize()  # delta ready before the token is visible
            if not self._ctrl.push(tok, 600.0):
                raise TimeoutError("worker: control queue full for 600 s")
            dist.send(delta, dst=0)
            if final:
                break
            dist.recv(wk.w, src=0)
            wk.vc += 1
            if self.log is not None:
                self.log.drain()
        if is_gpu(self.device):
            torch.cuda.synchronize(self.device)
        elapsed = time.time() - t_start
        return {"rounds": it, "updates": it, "elapsed_s": elapsed}


def run_distributed(cfg: PSConfig, cpu: bool = False, train=None, test=None) -> dict:
    rank, world, device = init_from_env(cpu)
    try:
        eng = DistEngine(cfg, rank, world, device, train=train, test=test)
        return eng.run()
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def bench_distributed(a, build_cfg) -> dict:
    """bench.py body for N > 1 GPUs (one rank per GPU, launched by torchrun)."""
    import bench as bench_mod  # noqa: F401  (constants)

    from ..utils.data import synth_finefood

    rank, world, device = init_from_env(cpu=a.cpu)
    cfg = build_cfg(a, world)
    train = synth_finefood(a.train_rows, num_features=a.features, seed=0)
    test = synth_finefood(a.test_rows, num_features=a.features, seed=1)
    cfg.max_iters = a.warmup
    eng = DistEngine(cfg, rank, world, device, train=train, test=test)
    if a.warmup:
        eng._run_bsp() if not eng.async_mode else None
    if eng.log is not None:
        eng.log.close()
        eng.log = LogSink(eng.spec.K, eng.device, keep_records=(rank == 0))
    cfg.max_iters = a.steps
    dist.barrier()
    if is_gpu(device):
        torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    out = eng._run_bsp()
    dist.barrier()
    if is_gpu(device):
        torch.cuda.synchronize(device)
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    res = None
    if rank == 0:
        eng.log.close()
        summ = summarize(eng.log.book)
        ups = a.steps * world / dt
        res = {
            "metric": "server_updates_per_s (PS push/pull rounds, multinomial LR; test accuracy reported alongside)",
            "value": round(ups, 2),
            "unit": "updates/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(dt * 1000.0 / a.steps, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(ups / bench_mod.REF_UPDATES_PER_S_4W, 1),
            "dtype": "bf16",
            "data": "synthetic (fine-food-reviews-shaped, 90k train / 4877 test, random-init weights)",
            "config": {
                "model": "multinomial-logreg F=1024 K=6 (P=6150), local solver L-BFGS x2 + strong-Wolfe",
                "global_batch": a.buffer * world,
                "seq_len": a.features,
                "parallelism": f"ps-bsp dp{world} ({cfg.bsp_schedule}, RCCL)",
                "consistency": a.consistency,
                "rows_per_step_per_worker": a.rows_per_step,
            },
            "test_accuracy": summ.get("final_server_acc"),
            "test_f1": summ.get("final_server_f1"),
            "best_test_f1": summ.get("best_server_f1"),
        }
        print(json.dumps(res), flush=True)
    dist.barrier()
    dist.destroy_process_group()
    return res
