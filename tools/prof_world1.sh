#!/bin/bash
# rocprofv3 kernel trace of the RCCL (DistEngine) bench body with world size 1,
# bench.py started directly (no launcher under the profiler).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1 MASTER_PORT=29561 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_w1 -o run -- python3 bench.py --gpus 2 --steps 300 --warmup 30 ${BENCH_ARGS:-} > gpurun_out/prof_w1.log 2>&1
rc=$?; echo "prof rc=$rc"; grep metric gpurun_out/prof_w1.log | cut -c1-300
exit $rc
