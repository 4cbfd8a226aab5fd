# Round 5: bench.py's multi-rank code paths rehearsed on ONE GPU (PSX_GPU_OVERSUBSCRIBE=1:
# gloo control plane, every rank on GPU 0, disjoint XCDs per rank).  Numbers are not
# scaling numbers (the ranks share one GPU); this checks the paths run end to end.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp PSX_GPU_OVERSUBSCRIBE=1 PSX_PG_TIMEOUT_S=120
O=gpurun_out/${SESS:-multirank}; mkdir -p $O
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 240 python bench.py "$@" > $O/$n.json 2> $O/$n.err; local rc=$?
  echo "$n rc=$rc $(python -c "import json;d=json.load(open('$O/$n.json'));print(d['value'], d['ms_per_step'], d['config']['parallelism'])" 2>/dev/null)"
  tail -2 $O/$n.err | cut -c1-300
  case $rc in 124|137|134|139) exit $rc;; esac
}
run allreduce_2x4 --gpus 2 --workers 4 --steps 20 --warmup 5
run reduce_bcast_3x3 --gpus 3 --workers 3 --dedicated-server --steps 20 --warmup 5
run peer_bsp_3x3 --gpus 3 --workers 3 --schedule peer --steps 20 --warmup 5
run ssp3_3x3 --gpus 3 --workers 3 --consistency 3 --steps 20 --warmup 5
run asp_3x3 --gpus 3 --workers 3 --consistency -1 --steps 20 --warmup 5
