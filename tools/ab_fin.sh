set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/ab
for f in 1 0 1 0; do
  PSX_FIN_INPLACE=$f timeout -k 10 200 python bench.py > gpurun_out/ab/b$f.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/ab/b$f.json')); print('fin=$f', d['value'], d['best_test_f1'])"
done
for f in 1 0; do
  PSX_FIN_INPLACE=$f timeout -k 10 200 python tools/bench_solver.py --ingest > gpurun_out/ab/s$f.log 2>&1 || exit 1
  echo "fin=$f"; grep ingest gpurun_out/ab/s$f.log
done
