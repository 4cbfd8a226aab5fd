#!/bin/bash
# cProfile of the host loop of the RCCL (DistEngine) bench body, world size 1.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29562 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1
mkdir -p gpurun_out
timeout -k 10 300 python -m cProfile -o gpurun_out/w1.pstats bench.py --gpus 2 --steps ${STEPS:-3000} --warmup 100 ${BENCH_ARGS:-} > gpurun_out/pyprof_w1.log 2>&1
rc=$?; echo "rc=$rc"; grep metric gpurun_out/pyprof_w1.log | cut -c1-200
[ $rc -eq 0 ] || exit $rc
python - <<'PY'
import pstats
p = pstats.Stats("gpurun_out/w1.pstats")
p.sort_stats("tottime").print_stats(45)
PY
