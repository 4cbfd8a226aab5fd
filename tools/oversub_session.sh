#!/bin/bash
# Multi-rank GPU schedules on a ONE-GPU box: 2..4 ranks share GPU 0 over gloo
# (PSX_GPU_OVERSUBSCRIBE=1; RCCL itself needs one GPU per rank).  Exercises the
# DistEngine GPU paths (replica aliasing, paired eval on rank 0, in-place
# sharded all-gather, sparse p2p pushes, watchdog tokens) before an 8-GPU run.
# Limitation of THIS harness only: gloo p2p of CUDA tensors of tens of MB in
# both directions at once stalls (ASP with 2^20 x 8 weights), so the wide runs
# use smaller feature spaces; RCCL p2p has no such issue and CPU gloo passes.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/oversub
export PSX_GPU_OVERSUBSCRIBE=1
i=0
while read -r n args; do
  i=$((i+1))
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29600+i)) bench.py --gpus $n $args > gpurun_out/oversub/run$i.log 2>&1
  rc=$?
  echo "== n=$n $args rc=$rc"
  grep -v amdgpu.ids gpurun_out/oversub/run$i.log | grep '"metric"' | cut -c1-20 >/dev/null && \
    python -c "import json,sys; d=[json.loads(l) for l in open('gpurun_out/oversub/run$i.log') if l.startswith('{')][-1]; print(d['value'], d['ms_per_step'], d['config']['parallelism'], d['test_accuracy'])"
  [ $rc -eq 0 ] || { tail -20 gpurun_out/oversub/run$i.log; exit $rc; }
done <<'LIST'
2 --steps 200 --warmup 20
4 --steps 200 --warmup 20
3 --steps 200 --warmup 20 --schedule sharded
3 --steps 200 --warmup 20 --schedule reduce_bcast
3 --steps 100 --warmup 10 --consistency -1
3 --steps 100 --warmup 10 --consistency 2
3 --model sparse1m --features 100000 --train-rows 200000 --steps 100 --warmup 10
2 --model sharded100m --features 10000000 --train-rows 200000 --steps 50 --warmup 5
LIST
echo oversub done
