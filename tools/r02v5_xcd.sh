#!/bin/bash
# One-XCD persistent solve: correctness, solver microbench (one XCD vs spread vs chain), engine bench.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02v5_xcd}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/bench_solver.py > $OUT/bench_solver_xcd.txt 2>&1
rc=$?; echo "bench_solver rc=$rc"; grep -E "default lbfgs|persistent|B=32" $OUT/bench_solver_xcd.txt; [ $rc -eq 0 ] || exit $rc
PSX_PERSIST_XCD=0 timeout -k 10 200 python tools/bench_solver.py > $OUT/bench_solver_spread.txt 2>&1
rc=$?; echo "bench_solver spread rc=$rc"; grep -E "persistent" $OUT/bench_solver_spread.txt; [ $rc -eq 0 ] || exit $rc
PSX_SOLVER_STAMPS=1 timeout -k 10 120 python tools/bench_solver.py --stamps-persist > $OUT/stamps_persist_xcd.txt 2>&1 && PSX_SOLVER_STAMPS=1 timeout -k 10 120 python tools/bench_solver.py --stamps > $OUT/stamps_chain.txt 2>&1
rc=$?; echo "stamps rc=$rc"; [ $rc -eq 0 ] || exit $rc
for v in ${VARIANTS:-"--chain" "" "--workers 4"}; do
  timeout -k 10 300 python bench.py $v >> $OUT/bench_variants.jsonl 2>> $OUT/bench_err.log
  rc=$?; echo "bench [$v] rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python - <<'PY'
import json
for l in open("gpurun_out/" + __import__("os").environ.get("TAG", "r02v5_xcd") + "/bench_variants.jsonl"):
    d = json.loads(l)
    print(d["value"], d["ms_per_step"], d["best_test_f1"])
PY
echo "session done"
