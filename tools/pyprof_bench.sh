#!/bin/bash
# cProfile of the host loop of bench.py (in-process engine, one GPU).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -m cProfile -o gpurun_out/bench.pstats bench.py --steps ${STEPS:-3000} --warmup 100 ${BENCH_ARGS:-} > gpurun_out/pyprof_bench.log 2>&1
rc=$?; echo "rc=$rc"; grep -o '"ms_per_step": [0-9.]*' gpurun_out/pyprof_bench.log
[ $rc -eq 0 ] || exit $rc
python - <<'PY'
import pstats
p = pstats.Stats("gpurun_out/bench.pstats")
p.sort_stats("tottime").print_stats(30)
PY
