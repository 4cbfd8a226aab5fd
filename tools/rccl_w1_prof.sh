#!/bin/bash
# The multi-rank BSP body (DistEngine, nccl backend, native RCCL communicator) at world size 1:
# bench + rocprofv3 kernel trace.  No launcher: the rank's env is set here, so the profiled
# program is python itself.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29561
OUT=gpurun_out/w1
mkdir -p $OUT
timeout -k 10 240 python bench.py --gpus 2 --steps 2000 --warmup 200 > $OUT/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep '^{' $OUT/bench.log | cut -c1-330; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python bench.py --gpus 2 --steps 2000 --warmup 200 ${EXTRA:-} > $OUT/bench2.log 2>&1
rc=$?; echo "bench2 rc=$rc"; grep '^{' $OUT/bench2.log | cut -c1-330; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --gpus 2 --steps 300 --warmup 50 > $OUT/prof.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
echo w1 done
