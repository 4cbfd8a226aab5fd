#!/bin/bash
# Round-3 GPU session W (final): full GPU suite, smoke, the driver's bench forms at the
# new default (8 workers per GPU, one per XCD) and at 4 workers, kernel trace.
set -o pipefail
OUT=gpurun_out/r03w
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
echo "pytest rc=$?" >> $OUT/pytest_gpu.log
grep -q "Fatal\|core dumped\|HSA_STATUS" $OUT/pytest_gpu.log && exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_short.json 2> $OUT/bench_short.err || exit 1
timeout -k 10 120 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
timeout -k 10 120 python bench.py --workers 4 > $OUT/bench_w4.json 2> $OUT/bench_w4.err || exit 1
timeout -k 10 120 python bench.py --workers 4 --steps 20 --warmup 5 > $OUT/bench_w4_short.json 2> $OUT/bench_w4_short.err || exit 1
PSX_BENCH_DIST=1 timeout -k 10 200 python bench.py --colocated-server --steps 200 --warmup 20 > $OUT/bench_dist_world1.json 2> $OUT/bench_dist_world1.err || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o w8 -- python3 bench.py --steps 200 --warmup 20 --no-accuracy-run > $OUT/bench_prof.json 2> $OUT/prof.err || exit 1
echo "session done"
