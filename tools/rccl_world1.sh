#!/bin/bash
# RCCL code path on a 1-GPU box: the multi-rank bench body (DistEngine, nccl backend) with world size 1.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for args in "--steps 300 --warmup 30" "--steps 300 --warmup 30 --schedule sharded" "--steps 300 --warmup 30 --schedule reduce_bcast" "--model sharded100m --steps 100 --warmup 10"; do
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29555 bench.py --gpus 2 $args > gpurun_out/rccl_w1.log 2>&1
  rc=$?
  echo "== $args rc=$rc"; grep -v amdgpu.ids gpurun_out/rccl_w1.log | tail -2 | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
done
