#!/bin/bash
# r02_v3 evidence: headline bench, rocprofv3 kernel stats + per-round timeline,
# solver variants (chain / gpf / persistent) with phase stamps, host cost.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r02v3
mkdir -p $OUT
timeout -k 10 200 python bench.py > $OUT/bench.json.log 2>&1 || exit $?
grep '^{' $OUT/bench.json.log | tail -1 > $OUT/bench.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 400 --warmup 50 > $OUT/prof.log 2>&1 || exit $?
python tools/trace_rounds.py $OUT/prof/run_kernel_trace.csv > $OUT/round_timeline.txt 2>&1
cp $OUT/prof/run_kernel_stats.csv $OUT/kernel_stats.csv
timeout -k 10 120 python tools/bench_solver.py > $OUT/bench_solver.txt 2>&1 || exit $?
PSX_SOLVER_GPF=1 timeout -k 10 120 python tools/bench_solver.py > $OUT/bench_solver_gpf.txt 2>&1 || exit $?
timeout -k 10 120 python tools/bench_solver.py --stamps > $OUT/stamps_chain.txt 2>&1 || exit $?
PSX_SOLVER_GPF=1 timeout -k 10 120 python tools/bench_solver.py --stamps > $OUT/stamps_gpf.txt 2>&1 || exit $?
timeout -k 10 120 python tools/bench_solver.py --stamps-persist > $OUT/stamps_persist.txt 2>&1 || exit $?
timeout -k 10 120 python tools/launch_probe.py > $OUT/launch_probe.txt 2>&1 || exit $?
echo r02v3 done
