// Native round loop of the sequential-consistency (BSP) parameter server for
// one worker per process: the in-process engine with one worker, and every rank
// of the multi-GPU allreduce schedule (worker + colocated server replica).
//
// Reference round (the sequential model, ServerProcessor.java:143-183 +
// WorkerTrainingProcessor.java:63-98 + WorkerSamplingProcessor.java:50-135):
// the producer delivers tuples into the worker's buffer, the worker fits its
// buffer from the current weights (LogisticRegressionTaskSpark.java:142-221),
// evaluates its local model, pushes the delta; the server applies the sum of
// the round's deltas (lr = 1/N), evaluates the global model, and the worker
// pulls the new weights.
//
// Here one call runs many rounds with no Python in between, every round
// enqueued on ONE stream with no host synchronisation:
//   * producer + window: the arrival schedule (per-iteration rows, or the
//     reference producer clock via due_rows) and the adaptive window
//     (SlidingWindow) of the host runtime, through its C ABI (capi.h);
//   * the new rows are copied into the HBM ring by the solve's first kernel
//     (fused ingest) -- or by ring-ingest launches when a delivery wraps an epoch;
//   * the local solve (LocalSolver) carries, in spare workgroups of its
//     bwd_update launches, the evaluation pass of the previous round's rows
//     (worker row = the local model, server row = the global model; EvalRide);
//   * world 1: the server update is fused into the solve's finalisation;
//     world > 1: RCCL all-reduce of the delta over xGMI, then the update launch;
//   * the rows' records go to the metrics sink (pinned slots the evaluation
//     writes, published by sequence number), the tracker advances one round.
// The last round's rows are evaluated by flush() (one standalone launch).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#include "../comm/rccl_comm.h"
#include "../host/capi.h"
#include "../solver/solver.h"

namespace psx {

struct BspLoopCfg {
  // producer (worker k of N reads dataset rows k, k + N, ...; `epochs` passes)
  const uint16_t* dsX = nullptr;  // dataset rows [rows][Fp] bf16 (device)
  const int32_t* dsy = nullptr;
  int64_t ds_rows = 0;
  int k = 0, N = 1;
  int per_iter_rows = 0;  // > 0: this many rows per round (throughput runs); 0: producer clock p_ms
  double p_ms = 0.0;
  int64_t epochs = 1;
  double t0_ms = 0.0;  // producer start, epoch milliseconds (arrival clocks are relative to it)
  // ring + window
  uint16_t* X = nullptr;
  uint16_t* XT = nullptr;
  int32_t* y = nullptr;
  int64_t cap = 0;
  int Fp = 0, K = 0, F = 0;
  uintptr_t window = 0;  // SlidingWindow* (host runtime)
  // solver outputs read by the evaluation (the worker's local model)
  const uint16_t* whi = nullptr;
  const uint16_t* wlo = nullptr;
  const float* wb = nullptr;
  const float* loss = nullptr;
  float* delta = nullptr;  // [P]
  // server replica (colocated): w, its fragments at columns scoff
  float* w = nullptr;
  uint16_t* shi = nullptr;
  uint16_t* slo = nullptr;
  float* sb = nullptr;
  int scoff = 0;
  float lr = 1.f;
  uintptr_t tracker = 0;  // VectorClockTracker* (0: none on this rank)
  // evaluation
  const uint16_t* Xt = nullptr;
  const int32_t* yt = nullptr;
  int T = 0;
  int* acc = nullptr;
  unsigned* ticket = nullptr;
  uintptr_t sink = 0;      // MetricsSink* (0: no rows)
  bool log_server = true;  // server rows on this rank
  uintptr_t api = 0;       // HostApi*
};

struct BspRow {  // a deferred evaluation row
  int64_t vc = -1, nseen = 0, ts = 0;
};

class BspLoop {
 public:
  // comm: RCCL communicator of the allreduce schedule (nullptr: world 1, the
  // update fused into the solve)
  BspLoop(LocalSolver* solver, RcclComm* comm, const BspLoopCfg& cfg);
  // Run `rounds` rounds starting at round r0 with the producer cursor at
  // `next_local`; returns the rounds run (fewer when the stream is exhausted
  // and the window is empty).
  int64_t run(int64_t rounds, int64_t r0, hipStream_t stream);
  // Evaluate the deferred rows of the last round (standalone launch).
  void flush(hipStream_t stream);
  int64_t next_local() const { return next_local_; }
  void set_next_local(int64_t v) { next_local_ = v; }
  bool exhausted() const { return next_local_ >= local_total_ * cfg_.epochs; }
  int64_t updates() const { return updates_; }
  double host_us_per_round() const { return rounds_run_ ? host_ns_ / 1000.0 / (double)rounds_run_ : 0.0; }

 private:
  const HostApi& api() const { return *api_; }
  void check(int64_t rc, const char* what) const;
  int64_t poll(double now_ms, RingIngest* fused, hipStream_t stream);
  void acquire(uint64_t* seq, uintptr_t* addr, int* slot);
  LocalSolver* solver_;
  RcclComm* comm_;
  BspLoopCfg cfg_;
  const HostApi* api_;
  int64_t local_total_ = 0, next_local_ = 0;
  std::vector<double> times_;
  BspRow pend_w_, pend_s_;
  int64_t updates_ = 0, rounds_run_ = 0;
  double host_ns_ = 0.0;
};

}  // namespace psx
