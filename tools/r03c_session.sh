#!/bin/bash
# Round-3 GPU session C: the full GPU suite after the lanes / native-server changes,
# then the lanes phase timeline.
set -o pipefail
OUT=gpurun_out/r03c
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
echo "pytest rc=$?" >> $OUT/pytest_gpu.log
export PSX_LANES_STAMPS=1
for L in 1 4 8; do
  timeout -k 10 120 python tools/lanes_profile.py --lanes $L --rounds 400 >> $OUT/lanes_profile.jsonl || exit 1
  timeout -k 10 120 python tools/lanes_profile.py --lanes $L --rounds 400 --no-eval >> $OUT/lanes_profile.jsonl || exit 1
done
echo "session done"
