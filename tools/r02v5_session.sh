#!/bin/bash
# GPU session: GPU suite, smoke, headline bench (default + the driver's short form), kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02v5}
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench_err.log
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_short.json 2>> $OUT/bench_err.log
rc=$?; echo "bench short rc=$rc"; [ $rc -eq 0 ] || exit $rc
python - <<'PY'
import json
for f in ("bench.json", "bench_short.json"):
    d = json.loads(open("gpurun_out/" + __import__("os").environ.get("TAG", "r02v5") + "/" + f).read().strip().splitlines()[-1])
    print(f, d["value"], d["ms_per_step"], d["best_test_f1"], d.get("accuracy_run", {}).get("best_test_f1"))
PY
if [ -n "${PROF:-}" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 300 --warmup 50 --no-accuracy-run > $OUT/prof.log 2>&1
  rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
echo "session done"
