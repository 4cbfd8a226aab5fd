#!/bin/bash
# Round-4 GPU session (one script, steps chosen by STEPS): the evaluation probe,
# the IPC multi-rank tests, the lanes phase timeline.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r04_s6}; mkdir -p $OUT
PYT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
for s in ${STEPS:-probe ipc}; do
  case $s in
    probe)
      timeout -k 10 60 ./tools/eval_probe 200 > $OUT/eval_probe.json 2> $OUT/eval_probe.err; rc=$?
      echo "probe rc=$rc"; cat $OUT/eval_probe.json
      [ $rc -eq 0 ] || [ $rc -eq 3 ] || exit $rc ;;
    ipc)
      timeout -k 10 300 $PYT tests/test_gpu_ipc_lanes.py > $OUT/pytest_ipc.log 2>&1; rc=$?
      echo "ipc rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed" $OUT/pytest_ipc.log | tail -8
      [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc ;;
    lanes)
      timeout -k 10 400 $PYT tests/test_gpu_lanes.py > $OUT/pytest_lanes.log 2>&1; rc=$?
      echo "lanes rc=$rc"; grep -E "FAIL|ERROR|passed|failed" $OUT/pytest_lanes.log | tail -8
      [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc ;;
    ab)   # AB_VARIANTS: env assignments, "-" = the defaults
      for v in ${AB_VARIANTS:-- PSX_RIDERS_TILE=1 - PSX_RIDERS_TILE=1}; do
        [ "$v" = "-" ] && v=""
        v=${v//,/ }  # (a,b: two assignments)
        timeout -k 10 200 env $v python bench.py --steps 200 --warmup 20 > $OUT/ab.tmp 2>> $OUT/ab.err || exit 1
        echo "[$v] $(python -c "import json;d=json.load(open('$OUT/ab.tmp'));print(d['value'],d['ms_per_step'])")" | tee -a $OUT/ab.txt
      done ;;
    fault)   # the round-3 matrix fault's configuration on the Python concurrent-stream path
      # (4 workers, producer clock -p 500, BSP, PSX_NATIVE_LANES=0 keeps it off the lanes
      # loop); FAULT_ENV adds e.g. AMD_SERIALIZE_KERNEL=3.  Runs LAST: nothing follows it.
      python -c "import sys; sys.path[:0] = ['tools', '.']; import experiment_matrix as m; m.ensure_data('data')" > $OUT/fault_data.log 2>&1 || exit 1
      timeout -k 10 ${FAULT_TIMEOUT:-90} env PSX_NATIVE_LANES=0 ${FAULT_ENV:-} python -X faulthandler -m psx.apps.server_app_runner --inprocess --device cuda -training data/train.bin -test data/test.bin -p ${FAULT_P:-500} -c 0 --num_workers 4 -l --log_dir $OUT/fault_run --max_wallclock_s ${FAULT_S:-45} --async_scheduler threads > $OUT/fault_run.out 2>&1
      rc=$?; echo "fault run rc=$rc"; tail -5 $OUT/fault_run.out; wc -l $OUT/fault_run/*.csv
      exit $rc ;;
    timeline)
      for v in 0 1; do
        PSX_RIDERS_TILE=$((v * 2)) PSX_LANES_STAMPS=1 timeout -k 10 120 python tools/lanes_profile.py --lanes 8 --rounds 400 >> $OUT/lanes_profile.jsonl 2>> $OUT/lanes_profile.err || exit 1
      done ;;
  esac
done
echo "session done"
