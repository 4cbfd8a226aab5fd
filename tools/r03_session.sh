#!/bin/bash
# Round-3 GPU session A: the multi-lane round kernel (tests, headline bench forms).
set -o pipefail
OUT=gpurun_out/r03a
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 420 python -u -m pytest tests/test_gpu_lanes.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest_lanes.log 2>&1 \
&& timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $OUT/bench_short.json 2> $OUT/bench_short.err \
&& timeout -k 10 120 python bench.py --steps 2000 --warmup 200 > $OUT/bench_long.json 2> $OUT/bench_long.err \
&& timeout -k 10 120 python bench.py --workers 4 --steps 2000 --warmup 200 > $OUT/bench_w4.json 2> $OUT/bench_w4.err \
&& timeout -k 10 120 python bench.py --workers 8 --steps 2000 --warmup 200 > $OUT/bench_w8.json 2> $OUT/bench_w8.err
echo "session rc=$?"
