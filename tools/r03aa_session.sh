#!/bin/bash
# Round-3 GPU session AA: the riders' timeline (PSX_LANES_STAMPS, rider stamps) at 4
# and 8 lanes; lanes tests after the stamp plumbing.
set -o pipefail
OUT=gpurun_out/r03aa
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 200 python -u -m pytest tests/test_gpu_lanes.py -m gpu -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
echo "pytest rc=$?" >> $OUT/pytest.log
grep -q "Fatal\|core dumped\|HSA_STATUS" $OUT/pytest.log && exit 1
for L in 4 8; do
  PSX_LANES_STAMPS=1 timeout -k 10 120 python tools/lanes_profile.py --lanes $L --rounds 400 >> $OUT/lanes_profile.jsonl 2> $OUT/lanes_profile.err || exit 1
done
echo "session done"
