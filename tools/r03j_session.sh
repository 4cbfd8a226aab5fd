#!/bin/bash
# Round-3 GPU session J: lanes (side-stream evaluation) + key-range (maintained
# margins) tests, 8-worker and sharded100m benches, kernel trace of both.
set -o pipefail
OUT=gpurun_out/r03j
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gpu_lanes.py tests/test_gpu_keyrange.py -m gpu -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 1
timeout -k 10 120 python bench.py --workers 8 > $OUT/bench_w8.json 2> $OUT/bench_w8.err || exit 1
timeout -k 10 120 python bench.py > $OUT/bench_w4.json 2> $OUT/bench_w4.err || exit 1
timeout -k 10 400 python bench.py --model sharded100m > $OUT/bench_sharded100m.json 2> $OUT/bench_sharded100m.err || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o w8 -- python3 bench.py --workers 8 --steps 200 --warmup 20 --no-accuracy-run > $OUT/bench_w8_prof.json 2> $OUT/prof_w8.err || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o kr -- python3 bench.py --model sharded100m --steps 300 --warmup 30 > $OUT/bench_kr_prof.json 2> $OUT/prof_kr.err || exit 1
echo "session done"
