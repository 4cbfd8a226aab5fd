#!/bin/bash
# Round-3 GPU session H: key-range + comm tests, kernel trace of the sharded100m
# key-range bench.
set -o pipefail
OUT=gpurun_out/r03h
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gpu_keyrange.py tests/test_gpu_comm.py -m gpu -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
echo "pytest rc=$?" >> $OUT/pytest.log
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o kr -- python3 bench.py --model sharded100m --steps 300 --warmup 30 > $OUT/bench_prof.json 2> $OUT/prof.err || exit 1
echo "session done"
