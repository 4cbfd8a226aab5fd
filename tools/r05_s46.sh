# Round 5 closing refresh of the secondary bench rows (README performance table).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${SESS:-s46}; mkdir -p $O
run() {  # name, bench.py arguments
  local n=$1; shift
  timeout -k 10 300 python bench.py "$@" > $O/$n.json 2> $O/$n.err || { echo "$n failed"; exit 1; }
  echo "$n $(python -c "import json;d=json.load(open('$O/$n.json'));print(d['value'], d['ms_per_step'], d.get('best_test_f1'))")"
}
run w4 --workers 4 --steps 300 --warmup 30
run w4_short --workers 4 --steps 20 --warmup 5
run w1 --workers 1 --steps 300 --warmup 30
run buf4096 --buffer 4096 --steps 100 --warmup 10
run long --steps 3000 --warmup 30
