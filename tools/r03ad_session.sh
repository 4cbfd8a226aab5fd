#!/bin/bash
# Round-3 GPU session AD: lanes tests (incl. the inline evaluation variant) on the final tree.
set -o pipefail
OUT=gpurun_out/r03ad
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_lanes.py tests/test_gpu_comm.py -m gpu -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
echo "pytest rc=$?" >> $OUT/pytest.log
echo "session done"
