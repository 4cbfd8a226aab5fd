// Native driver of one worker's local solve on the wide / sparse model.
//
// Same role as LocalSolver (solver.h) for rows that are sparse and models too
// wide for the dense MFMA tiles (BASELINE.json configs 4 and 5):
//   begin -> plan [-> owner order] | assign -> lid/stats -> prep -> (fwdbwd, dots+ctrl, apply) x nslots
//         -> [memset dense delta] -> finalize
// is captured once into a hipGraph; per run only the first node's kernel
// arguments (the window) change.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <vector>

#include "../kernels/wide_kernels.h"

namespace psx {

struct WideBuffers {
  const int32_t* ridx = nullptr;  // ring [cap][NZ]
  const uint16_t* rval = nullptr; // ring [cap][NZ] bf16
  const int32_t* rnnz = nullptr;  // [cap]
  const int32_t* ry = nullptr;    // [cap]
  const float* w_old = nullptr;   // [F*KP + KP]
  float* dloc = nullptr;          // [PLmax] out
  float* wloc = nullptr;          // [PLmax] out
  float* loss = nullptr;          // [1] out
  int* stats = nullptr;           // [4] out
  float* delta_dense = nullptr;   // [F*KP + KP] out (cfg.dense_delta)
  int32_t* uniq = nullptr;        // [min(F, cap*NZ)] out: local id -> feature
  // pull mode (cfg.pulled): the caller fills w_pull [umax][KP] (old weights of
  // local id i) and w_pull_b [KP] between plan() and finish(); w_old is unused.
  // Without pull mode a given w_pull_b holds the intercepts (w_old's are not read).
  const float* w_pull = nullptr;
  const float* w_pull_b = nullptr;
};

class WideSolver {
 public:
  WideSolver(const WideCfg& cfg, const WideBuffers& buf, bool use_graph);
  ~WideSolver();
  WideSolver(const WideSolver&) = delete;
  WideSolver& operator=(const WideSolver&) = delete;

  void run(int B, int start, hipStream_t stream);
  // pull mode: phase 1 (window features -> local ids, grouped by owner when
  // cfg.own_W > 1), then -- once w_pull holds the old weights of uniq[0..U) --
  // phase 2 (the solve).  Each phase is one hipGraph replay.
  void plan(int B, int start, hipStream_t stream);
  void finish(hipStream_t stream);
  // [kMaxOwners] per-owner feature counts of the last plan (pull mode, own_W > 1)
  const unsigned* owner_counts_dev() const { return dv_.own; }
  const WideCfg& cfg() const { return cfg_; }
  int64_t plmax() const { return dv_.PLmax; }
  // Device arrays valid after a run (until the next run's first kernel):
  const int2* table() const { return dv_.htab; }
  unsigned table_mask() const { return dv_.hmask; }
  const int32_t* uniq() const { return dv_.uniq; }
  const unsigned* ucount_dev() const { return dv_.cnt; }
  // U of the last finished run (pinned host mirror; valid after the stream synced).
  unsigned ucount_host() const { return host_u_ ? __atomic_load_n(host_u_, __ATOMIC_ACQUIRE) : 0u; }
  void read_ctrl(Ctrl* out, hipStream_t stream);
  // dots-kernel phase stamps of the last solve (PSX_WIDE_STAMPS=1 at construction): [slot][8]
  // s_memrealtime ticks (100 MHz): entry, last block in, dots reduced, ctrl loaded, ctrl stepped, ctrl stored
  std::vector<long long> read_stamps(hipStream_t stream);
  size_t workspace_bytes() const { return ws_bytes_; }
  const WideDev& dev() const { return dv_; }
  int kernels_per_solve() const {
    if (cfg_.persist) return 1;
    const int nf = cfg_.sc.mode == 1 ? cfg_.sc.nslots : std::min(cfg_.sc.nslots, 1 + cfg_.sc.iters);
    return 5 + 3 * nf + (cfg_.sc.nslots > nf ? 1 : 0) + 1;
  }

 private:
  void enqueue_plan(hipStream_t s, int B, int start);
  void enqueue_rest(hipStream_t s);
  void check_window(int B, int start) const;
  WideCfg cfg_;
  WideDev dv_{};
  bool use_graph_;
  int nblk_dots_ = 1;
  void* ws_ = nullptr;
  size_t ws_bytes_ = 0;
  unsigned* host_u_ = nullptr;
  hipGraphNode_t begin_node_ = nullptr;
  struct BeginArgs {
    WideDev d;
    int B, start;
  } begin_args_{};
  void* begin_kp_[3] = {};
  hipKernelNodeParams begin_params_{};
  hipStream_t cap_stream_ = nullptr;
  hipGraph_t graph_ = nullptr;  // whole solve, or phase 1 in pull mode
  hipGraphExec_t exec_ = nullptr;
  hipGraph_t graph2_ = nullptr;  // pull mode: phase 2
  hipGraphExec_t exec2_ = nullptr;
};

const void* wide_begin_symbol();

// Several in-process workers' solves in ONE launch (wide_lanes_kernel): lane l runs
// solvers[l]'s persistent solve on XCD xcd0 + l.  The solvers keep their own
// workspaces and outputs (delta, local model, table, loss, stats), so everything that
// reads a WideSolver after run() reads it after a lanes launch too.  Every solver
// must be bound to the same w_old (the server weights) and share one configuration.
// Also the lanes' evaluation pass (launch_wide_eval_multi): the worker rows of the
// last launch + optionally one server row of w.
class WideLanes {
 public:
  WideLanes(const std::vector<WideSolver*>& solvers, int xcd0);
  ~WideLanes();
  WideLanes(const WideLanes&) = delete;
  WideLanes& operator=(const WideLanes&) = delete;
  int lanes() const { return (int)solvers_.size(); }
  void run(const std::vector<int>& B, const std::vector<int>& start, hipStream_t stream);
  // worker rows of lanes [0, nov) (slot / seq per lane, their losses) and with
  // server_slot != 0 the row of the plain weights w (the model every lane pulled)
  void eval(const int64_t* indptr, const int32_t* idx, const uint16_t* val, const int32_t* y, int T, const float* w,
            int nov, const std::vector<uintptr_t>& slots, const std::vector<unsigned long long>& seqs,
            uintptr_t server_slot, unsigned long long server_seq, hipStream_t stream);
  // the server update of the lanes' sparse pushes, one after the other in `order`:
  // w[uniq[i] * KP + c] += lr * dloc[KP + i * KP + c] (ServerProcessor.java:148-151)
  void apply(float* w, float lr, const std::vector<int>& order, hipStream_t stream);
  int64_t launches() const { return launches_; }

 private:
  std::vector<WideSolver*> solvers_;
  WideCfg cfg_;
  int xcd0_;
  size_t lds_ = 0;
  WideDev* devs_ = nullptr;   // [L] device table
  unsigned* claim_ = nullptr; // [2][16]
  int* acc_ = nullptr;        // [kWideEvalCopies][kWideMaxEval][256] cells at stride kAccStride
  unsigned* ticket_ = nullptr;
  unsigned* pres_ = nullptr;  // [F] overlay presence words of the evaluation pass (null: table probes)
  float* ov_ = nullptr;       // [F][kWideMaxLanes][KP] the lanes' local coefficients
  int* lidt_ = nullptr;       // [F][kWideMaxLanes] their local ids
  bool ov_live_ = false;      // the table holds the last eval's lanes (apply consumes it)
  unsigned* bm_ = nullptr;    // [L][nw_] window-feature bitmaps of the evaluation pass (null: off)
  int64_t nw_ = 0;
  int gpx_ = 32;              // lane workgroups per XCD (32 x co-resident lane workgroups per CU)
  int64_t launches_ = 0;
};

}  // namespace psx
