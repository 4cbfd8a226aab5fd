set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${SESS:-full}; mkdir -p $O
timeout -k 10 900 python -u -m pytest -v --timeout 200 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; grep -E "FAILED|ERROR" $O/pytest_gpu.log | head -20
[ $rc -le 1 ] || exit $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; echo "smoke rc=$?"; tail -1 $O/smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_short.json 2> $O/bench_short.err; echo "bench short rc=$? $(python -c "import json;d=json.load(open('$O/bench_short.json'));print(d['value'], d['ms_per_step'])")"
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err; echo "bench rc=$? $(python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'], d['ms_per_step'])")"
SESS=${SESS:-full} bash tools/r05_s4.sh
