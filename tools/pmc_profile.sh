#!/bin/bash
# PMC counter passes over a short bench.py run (rocprofv3 --pmc, csv).
# Each pass is its own profiler run with counters only (no runtime/sys trace),
# sized to the gfx950 slot limits (SQ 8, TCC 4: FETCH_SIZE costs 3, WRITE_SIZE 2).
# PMC_BENCH_ARGS: extra bench.py arguments (e.g. --model sparse1m --workers 8); PMC_OUT: output dir.
# Output: gpurun_out/pmc/passN/..._counter_collection.csv; summary via
#   python tools/pmc_summary.py gpurun_out/pmc
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${PMC_OUT:-gpurun_out/pmc}
mkdir -p $OUT
STEPS="${PMC_STEPS:-150}"
run_pass() {
  local name=$1; shift
  timeout -k 10 240 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o $name -- \
    python3 bench.py --steps $STEPS --warmup 20 --no-accuracy-run ${PMC_BENCH_ARGS:-} > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  return $rc
}
run_pass p1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE &&
run_pass p2 SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_LDS_UNALIGNED_STALL GRBM_GUI_ACTIVE &&
run_pass p3 FETCH_SIZE &&
run_pass p4 WRITE_SIZE TCC_HIT_sum TCC_MISS_sum
