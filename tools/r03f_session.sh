#!/bin/bash
# Round-3 GPU session F: lanes tests (epoch-wrap ring rows), default bench.
set -o pipefail
OUT=gpurun_out/r03f
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_lanes.py -v --timeout 120 --timeout-method thread > $OUT/pytest_lanes.log 2>&1 || exit 1
timeout -k 10 120 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
echo "session done"
