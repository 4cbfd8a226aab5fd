#!/bin/bash
# One parameterised gpurun session (replaces every per-session one-off script).
#   OUT=gpurun_out/<name>  STEPS="tests smoke bench ..." bash tools/gpu_session.sh
# Steps (each GPU step has its own time limit; a crash / timeout / fault ends the script):
#   tests smoke bench ssp asp lanes async ipc ab prof rocprof timeline asyncprof probe pmc
#   secondary multirank world1 world1ps sparse fault
# Knobs: BENCH_ARGS (extra bench.py arguments), PYTEST_ARGS, AB_VARIANTS / AB_STEPS,
#   MR_RUNS (multirank: lines "name n args..."), SEC_RUNS (secondary: lines "name args...").
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/session}
mkdir -p "$OUT"
STEPS="${STEPS:-tests smoke bench prof}"
PYT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
ok_rc() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }   # 1 = test failures (not a crash)
fatal_rc() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
# value / ms per step / parallelism of a bench JSON line in file $1 (the last JSON line)
val() { python - "$1" <<'PY'
import json, sys
try:
    ls = [l for l in open(sys.argv[1]) if l.startswith('{"metric"')]
    d = json.loads(ls[-1])
    print(d.get("value"), d.get("ms_per_step"), d["config"].get("parallelism"), d.get("best_test_f1"))
except Exception as e:
    print("n/a", e)
PY
}
# one bench.py run: name, timeout, args...
bench_run() {
  local n=$1 t=$2; shift 2
  timeout -k 10 $t python bench.py "$@" > $OUT/$n.json 2> $OUT/$n.err; local rc=$?
  echo "$n rc=$rc $(val $OUT/$n.json)"
  [ $rc -eq 0 ] || tail -3 $OUT/$n.err | cut -c1-300
  return $rc
}
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
      timeout -k 10 ${TEST_TIMEOUT:-900} $PYT tests -m gpu ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1
      rc=$?; echo "pytest rc=$rc"; tail -5 $OUT/pytest_gpu.log; grep -E "FAILED|ERROR" $OUT/pytest_gpu.log | head -20
      ok_rc $rc || exit $rc ;;
    smoke)
      timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
      rc=$?; echo "smoke rc=$rc"; tail -3 $OUT/smoke.log
      [ $rc -eq 0 ] || exit $rc ;;
    bench)   # the driver's form, then the default
      bench_run bench_short 300 --steps 20 --warmup 5 ${BENCH_ARGS:-} && bench_run bench 300 ${BENCH_ARGS:-} || exit 1 ;;
    ab)      # same-box A/B of round variants (3 repeats each by default)
      # AB_VARIANTS: space-separated env assignments, "-" = the defaults
      for v in ${AB_VARIANTS:-- PSX_LANES_LANE_EVAL=1 - PSX_LANES_LANE_EVAL=1}; do
        [ "$v" = "-" ] && v=""
        timeout -k 10 200 env $v python bench.py --steps ${AB_STEPS:-200} --warmup 20 ${BENCH_ARGS:-} > $OUT/ab.tmp 2>> $OUT/ab.err
        rc=$?; [ $rc -eq 0 ] || { echo "ab [$v] rc=$rc"; exit $rc; }
        echo "[$v] $(val $OUT/ab.tmp)" | tee -a $OUT/ab.txt
      done ;;
    probe)   # the standalone evaluation probe (tools/eval_probe.hip, built beforehand)
      timeout -k 10 60 ./tools/eval_probe 200 > $OUT/eval_probe.json 2> $OUT/eval_probe.err; rc=$?
      echo "probe rc=$rc"; cat $OUT/eval_probe.json
      [ $rc -eq 0 ] || [ $rc -eq 3 ] || exit $rc ;;
    ipc)     # the multi-process ranks sharing the GPU (IPC transport, peer data plane)
      timeout -k 10 400 $PYT tests/test_gpu_ipc_lanes.py ${PYTEST_ARGS:-} > $OUT/pytest_ipc.log 2>&1; rc=$?
      echo "ipc rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed" $OUT/pytest_ipc.log | tail -12
      ok_rc $rc || exit $rc ;;
    timeline)  # the lanes kernel's phase stamps (tools/lanes_profile.py)
      PSX_LANES_STAMPS=1 timeout -k 10 120 python tools/lanes_profile.py --lanes 8 --rounds 400 >> $OUT/lanes_profile.jsonl 2>> $OUT/lanes_profile.err || exit 1 ;;
    asyncprof)  # the asynchronous lanes' per-ticket phases (tools/async_profile.py)
      PSX_LANES_STAMPS=1 timeout -k 10 120 python tools/async_profile.py --consistency -1 --iters 300 > $OUT/async_profile.json 2> $OUT/async_profile.err
      rc=$?; echo "async profile rc=$rc"; [ $rc -eq 0 ] || exit $rc ;;
    pmc)     # PMC passes of the BSP bench (tools/pmc_profile.sh), summarised
      bash tools/pmc_profile.sh > $OUT/pmc.log 2>&1; rc=$?; echo "pmc rc=$rc"; tail -3 $OUT/pmc.log
      [ $rc -eq 0 ] || exit $rc
      mv gpurun_out/pmc $OUT/pmc 2>/dev/null; python tools/pmc_summary.py $OUT/pmc > $OUT/pmc_summary.md; head -5 $OUT/pmc_summary.md ;;
    fault)   # the round-3 matrix fault's configuration on the Python concurrent-stream path
      # (4 workers, producer clock -p 500, BSP, PSX_NATIVE_LANES=0 keeps it off the lanes
      # loop); FAULT_ENV adds e.g. AMD_SERIALIZE_KERNEL=3.  Runs LAST: nothing follows it.
      python -c "import sys; sys.path[:0] = ['tools', '.']; import experiment_matrix as m; m.ensure_data('data')" > $OUT/fault_data.log 2>&1 || exit 1
      timeout -k 10 ${FAULT_TIMEOUT:-90} env PSX_NATIVE_LANES=0 ${FAULT_ENV:-} python -X faulthandler -m psx.apps.server_app_runner --inprocess --device cuda -training data/train.bin -test data/test.bin -p ${FAULT_P:-500} -c 0 --num_workers 4 -l --log_dir $OUT/fault_run --max_wallclock_s ${FAULT_S:-45} --async_scheduler threads > $OUT/fault_run.out 2>&1
      rc=$?; echo "fault run rc=$rc"; tail -5 $OUT/fault_run.out
      exit $rc ;;
    ssp|asp)
      c=10; [ $s = asp ] && c=-1
      bench_run bench_$s 300 --consistency $c --steps ${ASYNC_STEPS:-300} --warmup 30 ${BENCH_ARGS:-} || exit 1 ;;
    secondary)  # the secondary bench rows (4 / 1 workers, longer windows, a long run)
      while read -r n args; do
        [ -z "$n" ] && continue
        bench_run $n 300 $args; rc=$?; fatal_rc $rc && exit $rc
      done <<< "${SEC_RUNS:-w4 --workers 4 --steps 300 --warmup 30
w4_short --workers 4 --steps 20 --warmup 5
w1 --workers 1 --steps 300 --warmup 30
buf4096 --buffer 4096 --steps 100 --warmup 10
long --steps 3000 --warmup 30}" ;;
    multirank)  # bench.py's multi-rank paths with every rank on GPU 0 (disjoint XCDs, gloo control plane;
      # peer_sum with a dedicated server rank: the colocated default needs a GPU per rank, world1ps)
      while read -r n g args; do
        [ -z "$n" ] && continue
        PSX_GPU_OVERSUBSCRIBE=1 PSX_PG_TIMEOUT_S=120 bench_run $n 240 --gpus $g $args; rc=$?; fatal_rc $rc && exit $rc
      done <<< "${MR_RUNS:-peer_sum_2x7 2 --workers 7 --schedule peer_sum --dedicated-server --steps 300 --warmup 30
peer_sum_2x6 2 --workers 6 --schedule peer_sum --dedicated-server --steps 300 --warmup 30
reduce_bcast_3x3 3 --workers 3 --schedule reduce_bcast --steps 20 --warmup 5
peer_bsp_3x3 3 --workers 3 --schedule peer --steps 20 --warmup 5
ssp3_3x3 3 --workers 3 --consistency 3 --steps 20 --warmup 5
asp_3x3 3 --workers 3 --consistency -1 --steps 20 --warmup 5}" ;;
    world1)  # the multi-rank bench body with one rank (PSX_BENCH_DIST=1: RCCL communicator, DistEngine)
      PSX_BENCH_DIST=1 bench_run world1 300 --colocated-server --steps 300 --warmup 30 --no-accuracy-run || exit 1 ;;
    world1ps)  # the multi-GPU default (peer_sum, server kernel colocated on rank 0) with one rank:
      # the server kernel on XCD 7 beside rank 0's 7 lanes, one process; then in process, 7 workers
      PSX_BENCH_DIST=1 bench_run world1_psum 300 --steps ${W1_STEPS:-300} --warmup 30 --no-accuracy-run || exit 1
      bench_run inproc_w7 300 --workers 7 --steps ${W1_STEPS:-300} --warmup 30 --no-accuracy-run || exit 1 ;;
    sparse)  # BASELINE configs 4 / 5
      for w in 1 4 8; do bench_run sparse1m_w$w 300 --model sparse1m --workers $w --steps 40 --warmup 10; rc=$?; fatal_rc $rc && exit $rc; done
      bench_run sharded100m 300 --model sharded100m --steps 40 --warmup 10; rc=$?; fatal_rc $rc && exit $rc ;;
    prof|rocprof)  # rocprofv3 kernel statistics of the BSP bench (+ the ASP bench for rocprof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bsp -- python3 bench.py --steps ${PROF_STEPS:-300} --warmup 50 --no-accuracy-run ${BENCH_ARGS:-} > $OUT/prof.log 2>&1
      rc=$?; echo "prof bsp rc=$rc"; tail -1 $OUT/prof.log | cut -c1-200
      [ $rc -eq 0 ] || exit $rc
      if [ $s = rocprof ]; then
        timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o asp -- python3 bench.py --consistency -1 --steps 300 --warmup 30 --no-accuracy-run > $OUT/prof_asp.log 2>&1
        rc=$?; echo "prof asp rc=$rc"; [ $rc -eq 0 ] || exit $rc
      fi ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "session done"
