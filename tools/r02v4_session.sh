#!/bin/bash
# GPU session: GPU tests, smoke, headline bench (fresh windows) and accuracy variants.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r02v4
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
IFS=';' read -ra VS <<< "${VARIANTS:-;--rows-per-step 64 --server-lr 1.0;--server-lr 1.0}"
for v in "${VS[@]}"; do
  timeout -k 10 300 python bench.py $v >> $OUT/bench_variants.jsonl 2> $OUT/bench_err.log
  rc=$?; echo "bench [$v] rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python - <<'PY'
import json
for l in open("gpurun_out/r02v4/bench_variants.jsonl"):
    d = json.loads(l)
    print(d["value"], d["config"]["rows_per_step_per_worker"], d["config"]["server_lr"], d["steps"], d["best_test_f1"], d["test_accuracy"], d["time_to_f1_0.40_s"])
PY
if [ -n "${PROF:-}" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 300 --warmup 50 > $OUT/prof.log 2>&1
  rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
echo "session done"
