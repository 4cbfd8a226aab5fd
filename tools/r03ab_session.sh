#!/bin/bash
# Round-3 GPU session AB (final validation of the committed tree): full GPU suite,
# smoke, the driver's bench form, the riders' timeline at 4 / 8 lanes.
set -o pipefail
OUT=gpurun_out/r03ab
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
echo "pytest rc=$?" >> $OUT/pytest_gpu.log
grep -q "Fatal\|core dumped\|HSA_STATUS" $OUT/pytest_gpu.log && exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_short.json 2> $OUT/bench_short.err || exit 1
timeout -k 10 120 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
for L in 4 8; do
  PSX_LANES_STAMPS=1 timeout -k 10 120 python tools/lanes_profile.py --lanes $L --rounds 400 >> $OUT/lanes_profile.jsonl 2> $OUT/lanes_profile.err || exit 1
done
echo "session done"
