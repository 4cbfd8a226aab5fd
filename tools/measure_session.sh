#!/bin/bash
# Measurement session: dense bench x2, wide benches, accuracy vs wall-clock, rocprofv3 kernel stats.
# Every GPU step has its own limit; the first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/measure
mkdir -p $O
run() { local name=$1; shift; timeout -k 10 "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; grep -v amdgpu.ids $O/$name.log | tail -${TAIL:-1} | cut -c1-400; [ $rc -eq 0 ] || exit $rc; }
run bench_dense_a 300 python bench.py
run bench_dense_b 300 python bench.py
run bench_sparse1m 300 python bench.py --model sparse1m
run bench_sharded100m 300 python bench.py --model sharded100m
TAIL=6 run acc_bsp 300 python tools/accuracy_wallclock.py --workers 1 2 4 8 --consistency 0 --json $O/acc_bsp.json
TAIL=6 run acc_asp 300 python tools/accuracy_wallclock.py --workers 1 2 4 8 --consistency -1 --json $O/acc_asp.json
TAIL=6 run acc_ssp 300 python tools/accuracy_wallclock.py --workers 4 8 --consistency 3 --json $O/acc_ssp.json
run prof_dense 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_dense -o run -- python3 bench.py --steps 300 --warmup 50
echo measure done
