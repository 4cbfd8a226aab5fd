set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/s3; mkdir -p $O
PYT="python -u -m pytest -v -s --timeout 200 --timeout-method thread"
timeout -k 10 400 $PYT -x tests/test_gpu_ipc_lanes.py -k peer > $O/pytest_peer.log 2>&1; rc=$?
echo "peer rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed|Error" $O/pytest_peer.log | tail -8
[ $rc -le 1 ] || exit $rc
PSX_LANES_STAMPS=1 timeout -k 10 120 python tools/lanes_profile.py --lanes 8 --rounds 400 > $O/lanes_profile.jsonl 2> $O/lanes_profile.err; echo "timeline rc=$?"
export PSX_LANES_OVERLAP=0 PMC_STEPS=150
bash tools/pmc_profile.sh > $O/pmc.log 2>&1; rc=$?; echo "pmc rc=$rc"; cat $O/pmc.log
mv gpurun_out/pmc $O/pmc_serial 2>/dev/null
python tools/pmc_summary.py $O/pmc_serial > $O/pmc_summary.md; head -5 $O/pmc_summary.md
PSX_LANES_STAMPS=1 timeout -k 10 120 python tools/async_profile.py --consistency -1 --iters 300 > $O/async_profile.json 2> $O/async_profile.err; echo "async profile rc=$?"
