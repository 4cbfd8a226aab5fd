// Native driver of one worker's local solve.
//
// The reference runs, per worker iteration, a Spark job: build a DataFrame from
// the buffer, fit(), evaluate on the test set, diff the coefficients
// (reference: LogisticRegressionTaskSpark.java:142-221).  Here the whole chain
//   stats_prep -> (fwd, bwd_update) x (1 + iters) -> tail -> finalize
// (each slot = one function evaluation + one controller step, see
// csrc/kernels/solve_kernels.hip) is captured ONCE into a hipGraph and
// replayed per iteration: the host pays one graph launch and the device runs
// the chain back to back with no host synchronisation; line-search control
// flow is resolved on device and slots after convergence exit immediately.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

#include "../kernels/lr_kernels.h"
#include "../kernels/solve_kernels.h"

namespace psx {

struct SolverBuffers {
  // caller-owned (torch tensors)
  const uint16_t* X = nullptr;  // ring [cap][Fp] bf16
  const float* Xf = nullptr;    // ring [cap][Fp] fp32 (cfg.xf32)
  const uint16_t* XT = nullptr; // ring feature-major [Fp][cap] bf16
  const int32_t* y = nullptr;   // ring labels [cap]
  const float* w_old = nullptr; // [P] current model (worker copy)
  float* delta = nullptr;       // [P] out: w_new - w_old
  float* w_new = nullptr;       // [P] out (optional)
  uint16_t* wf_hi = nullptr;    // [16*Fp] out: fragments of w_new (for test eval)
  uint16_t* wf_lo = nullptr;
  float* b_fin = nullptr;       // [16] out
  float* loss = nullptr;        // [1] out
  int* stats = nullptr;         // [4] out: evals, accepted steps, ls failures, direction resets
};

class LocalSolver {
 public:
  LocalSolver(const SolverCfg& cfg, const SolverBuffers& buf, int max_eval_wg, bool use_graph);
  ~LocalSolver();
  LocalSolver(const LocalSolver&) = delete;
  LocalSolver& operator=(const LocalSolver&) = delete;

  // Enqueue one local solve over window [start, start+B) of the ring on `stream`;
  // `ing` (n > 0): first ingest those new rows, the newest of the window, into
  // the ring inside the solve's first kernel.
  // `ride` (optional): an evaluation pass (of models this solve does not write
  // before its last slot) executed by extra workgroups of the slots' bwd_update
  // launches.  `ap` (optional): a server update fused into the finalisation
  // (SolveDev::ap_w).  Both: eager solver only; small windows only for `ride`.
  void run(int B, int start, hipStream_t stream, const RingIngest& ing = RingIngest{}, const EvalRide* ride = nullptr,
           const FusedApply* ap = nullptr);
  const SolverCfg& cfg() const { return cfg_; }
  int eval_wg() const { return nwg_eval_; }
  int kernels_per_solve() const {  // stats_prep + slots + (tail with finalize | finalize); rows: 3 per slot
    if (persist_) return 1;
    return rows_mode_ ? 3 + (dv_.gred ? 3 : 2) * cfg_.nslots : 2 + 2 * nfast_;
  }
  bool rows_mode() const { return rows_mode_; }
  bool eager() const { return !use_graph_; }
  bool persistent() const { return persist_; }
  // Debug access to the device controller (synchronous copy).
  void read_ctrl(Ctrl* out, hipStream_t stream);
  // Phase timeline of the last solve (PSX_SOLVER_STAMPS=1 at construction):
  // [slot][k] s_memrealtime ticks (100 MHz); empty when disabled.
  std::vector<long long> read_stamps(hipStream_t stream);

 private:
  void enqueue_body(hipStream_t s, int B, int start, const RingIngest& ing, bool capturing, const EvalRide* ride);
  int ride_split_ = 2;       // riding evaluation tiles over the first 2 bwd_update launches
  bool fin_inplace_ = true;  // the last bwd_update launch finalises (PSX_FIN_INPLACE=0: the tail does)
  SolverCfg cfg_;
  SolveDev dv_{};
  int nwg_eval_;
  int nfast_;
  bool rows_mode_ = false;  // large window: row-parallel fused passes (solve_kernels.h)
  bool persist_ = false;    // small window: the whole solve in one persistent launch
  bool gpf_ = false;        // small window: backward from the forward's feature-major partials
  SolveDev dvp_{};          // the persistent launch's view (tile / statistics partials)
  bool use_graph_;
  void* ws_ = nullptr;
  size_t ws_bytes_ = 0;
  SolveParams* prm_ = nullptr;
  // the graph's first node (stats_prep) takes the window as kernel arguments,
  // rewritten per run with hipGraphExecKernelNodeSetParams
  hipGraphNode_t stats_node_ = nullptr;
  struct StatsArgs {
    SolverCfg cfg;
    SolveParams* prm;
    SolveDev dv;
    Ctrl* ctrl;
    int B, start;
    RingIngest ing;
  } stats_args_{};
  void* stats_kp_[7] = {};
  hipKernelNodeParams stats_params_{};
  Ctrl* ctrl_ = nullptr;
  hipStream_t cap_stream_ = nullptr;
  hipGraph_t graph_ = nullptr;
  hipGraphExec_t exec_ = nullptr;
};

void hip_check(hipError_t e, const char* what);

}  // namespace psx
