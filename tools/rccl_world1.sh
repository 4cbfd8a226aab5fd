#!/bin/bash
# RCCL code path on a 1-GPU box: the multi-rank bench body (DistEngine, nccl backend,
# native RCCL communicator) with world size 1 (PSX_BENCH_DIST=1).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PSX_BENCH_DIST=1
while IFS= read -r args; do
  [ -z "$args" ] && continue
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29555 bench.py --gpus 1 $args > gpurun_out/rccl_w1.log 2>&1
  rc=$?
  echo "== $args rc=$rc"; grep -v amdgpu.ids gpurun_out/rccl_w1.log | tail -1 | cut -c1-330
  grep -v amdgpu.ids gpurun_out/rccl_w1.log | tail -1 >> gpurun_out/rccl_w1.jsonl
  [ $rc -eq 0 ] || exit $rc
done <<'ARGS'
--steps 2000 --warmup 200
--steps 2000 --warmup 200 --chain
--steps 20 --warmup 5
--steps 300 --warmup 30 --schedule sharded
--steps 300 --warmup 30 --schedule reduce_bcast
ARGS
