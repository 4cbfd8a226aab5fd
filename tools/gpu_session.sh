#!/bin/bash
# One gpurun session: GPU tests, smoke, short bench, rocprofv3 kernel stats.
# Every GPU step has its own time limit; a crash/timeout/fault ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
STEPS="${STEPS:-tests smoke bench prof}"
ok_rc() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }   # 1 = test failures (not a crash)
for s in $STEPS; do
  case $s in
    tests)
      timeout -k 10 ${TEST_TIMEOUT:-420} python -m pytest tests -m gpu -x -q ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1
      rc=$?; echo "pytest rc=$rc"; tail -5 $OUT/pytest_gpu.log
      ok_rc $rc || exit $rc ;;
    smoke)
      timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
      rc=$?; echo "smoke rc=$rc"; tail -3 $OUT/smoke.log
      [ $rc -eq 0 ] || exit $rc ;;
    bench)
      timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > $OUT/bench.log 2>&1 && timeout -k 10 300 python bench.py ${BENCH_ARGS:-} >> $OUT/bench.log 2>&1
      rc=$?; echo "bench rc=$rc"; tail -2 $OUT/bench.log
      [ $rc -eq 0 ] || exit $rc ;;
    solver)
      timeout -k 10 240 python tools/bench_solver.py > $OUT/bench_solver.log 2>&1
      rc=$?; echo "bench_solver rc=$rc"; tail -12 $OUT/bench_solver.log
      [ $rc -eq 0 ] || exit $rc
      timeout -k 10 120 python tools/bench_solver.py --stamps > $OUT/stamps.log 2>&1
      rc=$?; echo "stamps rc=$rc"; cat $OUT/stamps.log
      [ $rc -eq 0 ] || exit $rc ;;
    prof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps ${PROF_STEPS:-300} --warmup 50 > $OUT/prof.log 2>&1
      rc=$?; echo "prof rc=$rc"; tail -2 $OUT/prof.log
      [ $rc -eq 0 ] || exit $rc ;;
  esac
done
echo "session done"
