#!/bin/bash
# One parameterised gpurun session (replaces the per-session one-off scripts).
#   OUT=gpurun_out/<name>  STEPS="tests smoke bench ssp asp lanes async ipc ab prof timeline probe fault" bash tools/gpu_session.sh
# Every GPU step has its own time limit; a crash / timeout / fault ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/session}
mkdir -p "$OUT"
STEPS="${STEPS:-tests smoke bench prof}"
PYT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
ok_rc() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }   # 1 = test failures (not a crash)
for s in $STEPS; do
  case $s in
    async)   # the asynchronous lanes loop's GPU tests
      timeout -k 10 ${ASYNC_TIMEOUT:-400} $PYT tests/test_gpu_async_lanes.py ${PYTEST_ARGS:-} > $OUT/pytest_async.log 2>&1
      rc=$?; echo "async tests rc=$rc"; grep -E "PASS|FAIL|ERROR|assert" $OUT/pytest_async.log | tail -20
      ok_rc $rc || exit $rc ;;
    lanes)   # the lanes loops (BSP riders / lane evaluation, IPC ranks on one GPU)
      timeout -k 10 ${LANES_TIMEOUT:-500} $PYT tests/test_gpu_lanes.py tests/test_gpu_ipc_lanes.py ${PYTEST_ARGS:-} > $OUT/pytest_lanes.log 2>&1
      rc=$?; echo "lanes tests rc=$rc"; grep -E "PASS|FAIL|ERROR" $OUT/pytest_lanes.log | tail -30
      ok_rc $rc || exit $rc ;;
    tests)
      timeout -k 10 ${TEST_TIMEOUT:-600} $PYT tests -m gpu ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1
      rc=$?; echo "pytest rc=$rc"; tail -5 $OUT/pytest_gpu.log
      ok_rc $rc || exit $rc ;;
    smoke)
      timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
      rc=$?; echo "smoke rc=$rc"; tail -3 $OUT/smoke.log
      [ $rc -eq 0 ] || exit $rc ;;
    bench)   # the driver's form, then the default
      timeout -k 10 300 python bench.py --steps 20 --warmup 5 ${BENCH_ARGS:-} > $OUT/bench_short.json 2> $OUT/bench_short.err &&
        timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err
      rc=$?; echo "bench rc=$rc"; cat $OUT/bench_short.json | head -c 600; echo
      [ $rc -eq 0 ] || exit $rc ;;
    ab)      # same-box A/B of the BSP round variants (driver form, 3 repeats each)
      # AB_VARIANTS: space-separated env assignments, "-" = the defaults
      for v in ${AB_VARIANTS:-- PSX_LANES_LANE_EVAL=1 - PSX_LANES_LANE_EVAL=1}; do
        [ "$v" = "-" ] && v=""
        timeout -k 10 200 env $v python bench.py --steps ${AB_STEPS:-200} --warmup 20 ${BENCH_ARGS:-} > $OUT/ab.tmp 2>> $OUT/ab.err
        rc=$?; [ $rc -eq 0 ] || { echo "ab [$v] rc=$rc"; exit $rc; }
        echo "[$v] $(python -c "import json;d=json.load(open('$OUT/ab.tmp'));print(d['value'],d['ms_per_step'])")" | tee -a $OUT/ab.txt
      done ;;
    probe)   # the standalone evaluation probe (tools/eval_probe.hip, built beforehand)
      timeout -k 10 60 ./tools/eval_probe 200 > $OUT/eval_probe.json 2> $OUT/eval_probe.err; rc=$?
      echo "probe rc=$rc"; cat $OUT/eval_probe.json
      [ $rc -eq 0 ] || [ $rc -eq 3 ] || exit $rc ;;
    ipc)     # the multi-process ranks sharing the GPU (IPC transport)
      timeout -k 10 300 $PYT tests/test_gpu_ipc_lanes.py > $OUT/pytest_ipc.log 2>&1; rc=$?
      echo "ipc rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed" $OUT/pytest_ipc.log | tail -8
      ok_rc $rc || exit $rc ;;
    timeline)  # the lanes kernel's phase stamps (tools/lanes_profile.py)
      PSX_LANES_STAMPS=1 timeout -k 10 120 python tools/lanes_profile.py --lanes 8 --rounds 400 >> $OUT/lanes_profile.jsonl 2>> $OUT/lanes_profile.err || exit 1 ;;
    fault)   # the round-3 matrix fault's configuration on the Python concurrent-stream path
      # (4 workers, producer clock -p 500, BSP, PSX_NATIVE_LANES=0 keeps it off the lanes
      # loop); FAULT_ENV adds e.g. AMD_SERIALIZE_KERNEL=3.  Runs LAST: nothing follows it.
      python -c "import sys; sys.path[:0] = ['tools', '.']; import experiment_matrix as m; m.ensure_data('data')" > $OUT/fault_data.log 2>&1 || exit 1
      timeout -k 10 ${FAULT_TIMEOUT:-90} env PSX_NATIVE_LANES=0 ${FAULT_ENV:-} python -X faulthandler -m psx.apps.server_app_runner --inprocess --device cuda -training data/train.bin -test data/test.bin -p ${FAULT_P:-500} -c 0 --num_workers 4 -l --log_dir $OUT/fault_run --max_wallclock_s ${FAULT_S:-45} --async_scheduler threads > $OUT/fault_run.out 2>&1
      rc=$?; echo "fault run rc=$rc"; tail -5 $OUT/fault_run.out
      exit $rc ;;
    ssp|asp)
      c=10; [ $s = asp ] && c=-1
      timeout -k 10 300 python bench.py --consistency $c --steps ${ASYNC_STEPS:-300} --warmup 30 ${BENCH_ARGS:-} > $OUT/bench_$s.json 2> $OUT/bench_$s.err
      rc=$?; echo "bench $s rc=$rc"; head -c 700 $OUT/bench_$s.json; echo
      [ $rc -eq 0 ] || exit $rc ;;
    prof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps ${PROF_STEPS:-300} --warmup 50 ${BENCH_ARGS:-} > $OUT/prof.log 2>&1
      rc=$?; echo "prof rc=$rc"; tail -2 $OUT/prof.log
      [ $rc -eq 0 ] || exit $rc ;;
  esac
done
echo "session done"
