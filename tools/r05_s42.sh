# One-wave acquire fences (async iteration top, BSP overlapped-launch entry): tests + benches.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${SESS:-s42}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_lanes.py tests/test_gpu_async_lanes.py tests/test_gpu_engine.py > $O/pytest_lanes.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $O/pytest_lanes.log
[ $rc -eq 0 ] || exit $rc
PSX_LANES_STAMPS=1 timeout -k 10 120 python tools/async_profile.py --consistency -1 --iters 300 > $O/async_profile.json 2> $O/async_profile.err || exit 1
for i in 1 2; do
  timeout -k 10 300 python bench.py > $O/bench_$i.json 2> $O/bench_$i.err || exit 1
  echo "bench $i $(python -c "import json;d=json.load(open('$O/bench_$i.json'));print(d['value'], d['ms_per_step'])")"
done
for c in -1 10; do
  timeout -k 10 300 python bench.py --consistency $c --steps 300 --warmup 30 > $O/bench_c$c.json 2> $O/bench_c$c.err || exit 1
  echo "bench c=$c $(python -c "import json;d=json.load(open('$O/bench_c$c.json'));print(d['value'], d['ms_per_step'])")"
done
