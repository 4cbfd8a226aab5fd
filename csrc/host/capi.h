// C ABI of the host runtime (_psx_host) for the GPU runtime (_psx_hip).
//
// The two extensions are separate shared objects (the host one builds with g++
// and needs no GPU).  The native asynchronous server loop in _psx_hip drives
// objects the host runtime owns -- the vector-clock tracker (MessageTracker),
// the shared-memory token queue (the GRADIENTS_TOPIC control plane) and the
// metrics sink (the server CSV log) -- through this table of plain function
// pointers: no C++ object crosses the library boundary, only opaque handles.
#pragma once
#include <cstdint>

#include "ctrl.h"
#include "sink_record.h"

namespace psx {

constexpr int kHostApiVersion = 4;

struct HostApi {
  int version;
  // VectorClockTracker (tracker.h).  The release lists are written to
  // (ks[i], vs[i]), at most `cap` entries; the return value is the count.
  int (*tracker_on_delta)(void* tracker, int k, int64_t v, int* ks, int64_t* vs, int cap);
  int (*tracker_retire)(void* tracker, int k, int* ks, int64_t* vs, int cap);
  int (*tracker_is_live)(void* tracker, int k);
  int (*tracker_revive)(void* tracker, int k);
  int64_t (*tracker_clock)(void* tracker, int k);
  void (*tracker_sent)(void* tracker, int k, int64_t v);
  // CtrlQueue (ctrl.h): 1 = token popped / pushed, 0 = timeout
  int (*ctrl_pop)(void* queue, CtrlToken* out, double timeout_s);
  int (*ctrl_push)(void* queue, const CtrlToken* tok, double timeout_s);
  // MetricsSink (metrics_sink.h): reserve an EvalSlot (its host address is
  // written to *addr) and hand the finished record to the logger thread
  int (*sink_acquire)(void* sink, uint64_t* seq, uintptr_t* addr);
  void (*sink_submit)(void* sink, int slot, uint64_t seq, int kind, int64_t ts, int64_t partition, int64_t vc,
                      int64_t nseen);
  // Exceptions thrown by the functions above are caught at this boundary: the
  // message of the last failure on this thread (empty: none).
  const char* (*last_error)();
  // ---- version 2: the native BSP round loop (csrc/runtime/bsp_loop.h) ----
  // SlidingWindow (sampling.h): n arrivals -> slot of the first (the n slots are
  // consecutive modulo the ring), -1 on error; the window after it.
  int64_t (*window_insert_many)(void* window, const double* times_ms, int64_t n);
  int (*window_state)(void* window, int64_t* size, int64_t* start, int64_t* seen);
  // producer schedule (dataset.h due_rows): rows of worker k due by now_ms
  int64_t (*due_rows)(int k, int num_workers, double p_ms, int64_t total_rows, int64_t next_local, double now_ms,
                      int64_t max_rows, double* times_out);
  // VectorClockTracker::bsp_round: every live worker's delta of round v received,
  // the weights of v + 1 sent
  int (*tracker_bsp_round)(void* tracker, int64_t v);
  // ---- version 3: batched metrics-sink hand-over (the lanes loop: a round's rows
  // under one lock and one wake-up).  addrs[i]: host address of slots[i]; 0 / -1 ----
  int (*sink_acquire_many)(void* sink, int n, int* slots, uint64_t* seqs, uintptr_t* addrs);
  int (*sink_submit_many)(void* sink, int n, const SinkRecord* recs);
  // ---- version 4: the asynchronous lanes loop (SSP / ASP, csrc/runtime/lanes_loop.h)
  // carries releases over launches: 1 = the weights of worker k's clock were
  // dispatched (k is busy or about to start), 0 = idle, -1 = error ----
  int (*tracker_is_sent)(void* tracker, int k);
};

const HostApi* host_api();

}  // namespace psx
