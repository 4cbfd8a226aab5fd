#!/bin/bash
# Large-window solver on one MI355X: bench at 1M and 16M rows per worker,
# kernel stats, and FETCH_SIZE (HBM bytes) of the row-parallel passes.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/bigwin
mkdir -p $OUT
B1="--buffer 1048576 --rows-per-step 65536 --warmup 20 --steps 20"
B16="--buffer 16777216 --rows-per-step 1048576 --warmup 18 --steps 6"
timeout -k 10 300 python -u bench.py $B1 > $OUT/bench_1m.log 2>&1 || exit $?
tail -1 $OUT/bench_1m.log
timeout -k 10 400 python -u bench.py $B16 > $OUT/bench_16m.log 2>&1 || exit $?
tail -1 $OUT/bench_16m.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof1m -o run -- python3 bench.py $B1 > $OUT/prof1m.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/pmc1m -o run -- python3 bench.py --buffer 1048576 --rows-per-step 65536 --warmup 20 --steps 4 > $OUT/pmc1m.log 2>&1 || exit $?
echo bigwindow done
