// Native BSP round loop of the key-range sharded parameter server (BASELINE.json
// config 5: a 10^8-feature model whose weights are partitioned across the ranks).
//
// Reference: messages carry the KeyRange of their weights (BaseMessage.java:
// 24-27, KeyRange.java:11-49) and the README sketches servers that own ranges
// of the key space (README.md:117-119, 333); the running system has one server
// holding everything.  Here every rank hosts one worker AND the server shard of
// its key range [lo, hi) = [rank*S, min(F, (rank+1)*S)), S = ceil(F / world):
// the coefficients of other ranges never exist on it.  Per round, with one host
// synchronisation (the pull sizes) and no P-sized buffer anywhere:
//
//   ingest   the worker's due rows -> its HBM ring (sparse CSR gather)
//   plan     the window's distinct features -> local ids, grouped by owner
//            (the wide solver's first phase, one hipGraph)
//   pull     counts all-to-all; ids to their owners; the owners gather their
//            coefficients and send them back (RCCL send/recv, grouped)
//   solve    the local L-BFGS solve in the window subspace (second phase)
//   push     the deltas of those same features to their owners (the ids are
//            already there from the pull); every owner applies w += lr * delta
//            sender by sender in rank order (deterministic); the intercepts are
//            replicated and all-reduced
//   rows     the test margins of the global model are maintained: each worker
//            adds the window overlay of its delta to them (its worker row, one
//            pass over the test rows), the per-row sums are all-reduced (T KP
//            floats) into z += lr * sum, and the server row (rank 0) is z + the
//            intercepts; every margin_refresh rounds z is recomputed from the
//            shards (partial margins of each key range, all-reduced)
//
// Bytes on the wire per round: 4 W + 8 U + 8 U KP (+ KP intercepts + T KP
// margins for the rows) with U the window's distinct features -- proportional
// to the window, independent of F.  At world 1 every exchange is local, the
// solve reads the shard in place (one hipGraph, no pull phase) and the round
// needs no host synchronisation at all.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <memory>
#include <vector>

#include "../comm/rccl_comm.h"
#include "../host/capi.h"
#include "../kernels/wide_kernels.h"
#include "../solver/wide_solver.h"

namespace psx {

struct KeyRangeLoopCfg {
  WideCfg wcfg;  // model / ring / solver options (pulled, own_W, own_S are set by the loop)
  bool use_graph = true;
  // producer: worker k of N reads CSR rows k, k + N, ... (`epochs` passes)
  const int64_t* indptr = nullptr;
  const int32_t* idx = nullptr;
  const uint16_t* val = nullptr;
  const int32_t* y = nullptr;
  int64_t ds_rows = 0;
  int k = 0, N = 1;
  int per_iter_rows = 0;  // > 0: rows per round; 0: the producer clock p_ms
  double p_ms = 0.0;
  int64_t epochs = 1;
  double t0_ms = 0.0;
  // the worker's ring [cap][NZ] + window (SlidingWindow*)
  int32_t* ridx = nullptr;
  uint16_t* rval = nullptr;
  int32_t* rnnz = nullptr;
  int32_t* ry = nullptr;
  int* trunc = nullptr;
  uintptr_t window = 0;
  // this rank's server shard: coefficients of [lo, hi) then KP zeros, and the
  // replicated intercepts b [KP]
  float* shard = nullptr;
  float* b = nullptr;
  float lr = 1.f;
  // solver outputs (caller-owned)
  float* dloc = nullptr;
  float* wloc = nullptr;
  float* loss = nullptr;
  int* stats = nullptr;
  int32_t* uniq = nullptr;
  // evaluation: the whole test CSR (worker rows) and its entries in [lo, hi)
  // with local ids (partial margins)
  const int64_t* t_indptr = nullptr;
  const int32_t* t_idx = nullptr;
  const uint16_t* t_val = nullptr;
  const int32_t* t_y = nullptr;
  int T = 0;
  const int64_t* s_indptr = nullptr;
  const int32_t* s_idx = nullptr;
  const uint16_t* s_val = nullptr;
  uintptr_t sink = 0;  // MetricsSink* (0: no rows)
  bool log_server = true;
  bool log_workers = true;
  uintptr_t tracker = 0;  // VectorClockTracker* (rank 0)
  uintptr_t api = 0;      // HostApi*
  // the rows' margins are updated incrementally (z += lr * X_test * sum of the
  // round's deltas) and recomputed from the shards every `margin_refresh` rounds
  int margin_refresh = 256;
};

class KeyRangeLoop {
 public:
  // comm: RCCL communicator of the job (nullptr: world 1)
  KeyRangeLoop(const KeyRangeLoopCfg& cfg, RcclComm* comm);
  ~KeyRangeLoop();
  KeyRangeLoop(const KeyRangeLoop&) = delete;
  KeyRangeLoop& operator=(const KeyRangeLoop&) = delete;

  // Run `rounds` rounds from round r0 (collective: every rank calls it with the
  // same arguments); returns the rounds run (fewer when the stream is exhausted).
  int64_t run(int64_t rounds, int64_t r0, hipStream_t stream, double max_wait_s = 600.0);
  int64_t lo() const { return lo_; }
  int64_t hi() const { return hi_; }
  int64_t shard_size() const { return S_; }
  // bytes this rank sent to other ranks: model traffic (counts, ids, pulled
  // values, pushed deltas, intercepts) and evaluation traffic (margins)
  int64_t model_bytes() const { return model_bytes_; }
  int64_t eval_bytes() const { return eval_bytes_; }
  int64_t last_round_bytes() const { return last_round_bytes_; }
  // distinct features of the last window (after a synchronisation at world 1)
  int64_t last_u() const;
  int64_t next_local() const { return next_local_; }
  void set_next_local(int64_t v) { next_local_ = v; }
  bool exhausted() const { return next_local_ >= local_total_ * cfg_.epochs; }
  double host_us_per_round() const { return rounds_run_ ? host_ns_ / 1000.0 / (double)rounds_run_ : 0.0; }
  int64_t rounds_run() const { return rounds_run_; }
  size_t device_bytes() const { return ws_bytes_ + solver_->workspace_bytes(); }
  const WideSolver& solver() const { return *solver_; }

 private:
  const HostApi& api() const { return *api_; }
  void check(int64_t rc, const char* what) const;
  int64_t poll(double now_ms, hipStream_t stream);
  void margins(float* z, hipStream_t stream);
  void exchange(const void* send, const int64_t* soff, const int64_t* scnt, void* recv, const int64_t* roff,
                const int64_t* rcnt, int elem, int dtype, hipStream_t stream);

  KeyRangeLoopCfg cfg_;
  RcclComm* comm_;
  const HostApi* api_;
  int W_ = 1, rank_ = 0, KP_ = 1;
  int64_t S_ = 0, lo_ = 0, hi_ = 0;
  int umax_ = 0;
  std::unique_ptr<WideSolver> solver_;
  void* ws_ = nullptr;
  size_t ws_bytes_ = 0;
  float* w_pull_ = nullptr;    // [umax][KP]
  int32_t* req_ids_ = nullptr; // [W * umax] ids requested from this owner
  float* req_vals_ = nullptr;  // [W * umax][KP] pulled answers, then pushed deltas
  float* db_ = nullptr;        // [KP] intercept deltas (all-reduced)
  float* z_ = nullptr;   // [T][KP] test margins of the global model (coefficients only)
  float* dz_ = nullptr;  // [T][KP] this round's margin update (all-reduced over the ranks)
  int* acc_ = nullptr;
  unsigned* ticket_ = nullptr;
  unsigned* cnt_dev_ = nullptr;  // [2W]: recv counts
  unsigned* cnt_host_ = nullptr; // pinned [2W]: send counts, recv counts
  int64_t local_total_ = 0, next_local_ = 0;
  std::vector<double> times_;
  bool margins_ready_ = false;
  int64_t model_bytes_ = 0, eval_bytes_ = 0, last_round_bytes_ = 0;
  int64_t rounds_run_ = 0;
  double host_ns_ = 0.0;
};

}  // namespace psx
