import os, sys, faulthandler
faulthandler.dump_traceback_later(60, exit=True)
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import torch, torch.distributed as dist
from psx.parallel.dist import DistEngine, init_from_env
from psx.runtime.config import PSConfig
from psx.utils.data import synth_sparse
rank, world, dev = init_from_env()
sp = os.environ.get("SP", "1") == "1"
cfg = PSConfig(num_workers=world - 1, consistency_model=-1, producer_time_per_event=0, stream_mode="per_iter",
               rows_per_iter=64, epochs=100, max_iters=int(os.environ.get("IT", "20")), min_buffer_size=64, max_buffer_size=256,
               init="random", model="wide", sparse_push=sp)
kw = dict(num_features=int(os.environ.get("F", "100000")), nnz_mean=48, max_nnz=128, device=dev)
tr, te = synth_sparse(20000, seed=0, **kw), synth_sparse(500, seed=1, **kw)
eng = DistEngine(cfg, rank, world, dev, train=tr, test=te)
out = eng._run_async()
print("rank", rank, "done", out.get("updates"), flush=True)
out = eng._run_async()
print("rank", rank, "done2", out.get("updates"), flush=True)
dist.barrier(); dist.destroy_process_group()
