// Host loop of the peer data plane's server rank (SSP / ASP across GPUs).
//
// Reference: ServerProcessor.process (ServerProcessor.java:143-183) -- apply
// every gradient on arrival in the single partition's order, log a server row
// on worker-0 gradients, answer the workers MessageTracker releases
// (MessageTracker.java:69-87) with the weights after that update.
//
// Division of labour (csrc/comm/peer_bus.h, csrc/kernels/server_persist.h):
//   * device: ONE persistent launch on this GPU applies the deltas (already in
//     this GPU's inbox: the workers' lanes wrote them over xGMI), writes the new
//     weights into the released workers' receive slots on their GPUs and
//     evaluates the server rows;
//   * host (this class): pops the worker ranks' tokens from the shared-memory
//     queue in arrival order, runs the C++ vector-clock tracker, writes one
//     64-B command per token into a pinned ring, and answers each release on
//     the worker's rank reply queue with its pull tag.  It never waits for the
//     device and never synchronises a stream per delta (host_us_per_update).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <exception>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "../comm/peer_bus.h"
#include "../host/capi.h"
#include "../kernels/server_persist.h"
#include "async_server.h"

namespace psx {

struct PeerServerCfg {
  int nworkers = 0;
  float lr = 1.f;
  int K = 0, F = 0, FP = 0;
  int64_t P = 0;
  float* w = nullptr;            // fp32 master weights [P] on this GPU
  const uint16_t* Xt = nullptr;  // test set (server rows)
  const int32_t* yt = nullptr;
  int T = 0;
  uintptr_t inbox = 0;           // this rank's PeerRegion (one slot per worker)
  PeerLayout lay;                // its layout (P, NS, slots = nworkers)
  std::vector<uintptr_t> rx, rx_tag;  // per worker: its receive slot / slice tags on its GPU (IPC mappings)
  uintptr_t api = 0, tracker = 0, ctrl = 0, sink = 0;
  std::vector<uintptr_t> replies;     // per worker: its rank's reply queue
  double worker_timeout_s = 600.0;
  int sxcd = 0;                  // the XCD of the persistent launch
  // peer_sum BSP (run_bsp): the "workers" are the worker RANKS -- inbox slot j / receive
  // slot j = worker rank j's lane sum / weights; no token queues, no reply queues (the
  // rounds are the protocol); tag_wait_s bounds a round's wait for the ranks' sums (a
  // paced stream can hold a round for as long as its rows take)
  bool bsp = false;
  double tag_wait_s = 600.0;
  // workgroups of the server launch on its XCD (<= 32, each owns every nwg-th slice): a
  // GPU shared with other ranks' launches gets fewer, leaving CUs of the XCD to them
  int nwg = kSrvWg;
  // asynchronous plane: deltas per server command (1..64) -- the tokens already popped when
  // a command is written go as ONE batch command, applied in token order slice-parallel
  // (1: one command per delta)
  int batch = 64;
  // stand-in workers (tools/peer_server_bench.py): no token / reply queues needed
  bool standin = false;
  // commands written ahead of the kernel's reads at most (0: the ring, 256).  Each BSP
  // round's command holds a metrics-sink slot for its server row from the moment it is
  // written: the colocated peer_sum rank 0 shares its sink with its own lanes, whose worker
  // rows must still find slots
  int ahead = 0;
};

class PeerServer {
 public:
  PeerServer(const PeerServerCfg& cfg, hipStream_t stream);
  ~PeerServer();
  PeerServer(const PeerServer&) = delete;
  PeerServer& operator=(const PeerServer&) = delete;
  // New run (AsyncServer::begin semantics): launches the persistent kernel if it is
  // not running and sends every live worker the weights of its clock.
  void begin();
  // Serve tokens until every worker finished (the launch then drains: w is final),
  // a checkpoint is due (drained as well) or a worker needs the caller's decision.
  AsyncStatus run(int64_t checkpoint_every);
  void fail(int k);
  // peer_sum BSP: `rounds` rounds from round r0 -- one command per round (the ranks' sums
  // summed, applied, the weights written into every rank's receive slot; the server row of
  // the global model into the metrics sink, vc = the round), the tracker advanced per
  // round; returns once the launch has drained (w final).  The ranks' lanes loops run the
  // same rounds (LanesLoop::set_peer_sum).
  int64_t run_bsp(int64_t rounds, int64_t r0);
  // run_bsp on a host thread of its own (returns at once): the server rank that also hosts
  // lanes (rank 0 of the colocated peer_sum form) runs its own lanes loop meanwhile, then
  // run_bsp_join (the rounds' result; rethrows the thread's error)
  void run_bsp_async(int64_t rounds, int64_t r0);
  int64_t run_bsp_join();
  // peer_sum BSP bring-up: the current weights into every rank's receive slot (tag 0: the
  // pull of round 0)
  void seed_rx();
  int64_t bsp_rounds() const { return (int64_t)bsp_n_; }
  // deltas per command of the asynchronous plane so far (batching)
  double deltas_per_command() const { return batches_ ? (double)batched_deltas_ / (double)batches_ : 0.0; }
  // Microbenchmark (stand-in workers, inbox tags pre-armed): `deltas` asynchronous deltas
  // (ASP: worker i % N, each releasing itself) through the tracker, the commands (batches of
  // cfg.batch) and the server kernel, no reply queues; worker 0's deltas produce server rows
  // when a sink is bound; returns {seconds to drain, host seconds}
  std::vector<double> bench_async(int64_t deltas, int log_every);
  std::string bsp_tags() const;  // (failure reports) every rank's push / pull slice tags
  // (tools) per-command device stamps of the next launches: a ring of cap commands;
  // trace_take (the launch drained) -> {command, read, applied, evaluated} s_memrealtime ticks
  void set_trace(int cap);
  std::vector<std::vector<long long>> trace_take();
  double host_us_per_round() const { return bsp_run_ ? bsp_ns_ / 1000.0 / (double)bsp_run_ : 0.0; }
  // Stop the persistent launch and wait for it (idempotent).
  void stop();
  // One launch that stops at once, drained here: the first launch's one-time device work
  // (code object load, copy paths) done before other ranks' persistent launches hold CUs
  // of a shared GPU.
  void warm_up() {
    launch();
    stop();
  }
  int64_t updates() const { return updates_; }
  void set_updates(int64_t u) { updates_ = u; }
  int64_t tokens() const { return tokens_; }
  int64_t commands() const { return (int64_t)cmds_; }
  double host_us_per_update() const { return updates_run_ ? host_ns_ / 1000.0 / (double)updates_run_ : 0.0; }
  std::vector<int> failed() const;
  bool running() const { return running_; }
  // (worker, vc) of every delta in arrival order (the single partition's order; tests
  // replay it through a fresh tracker), the first kMaxArrivals
  static constexpr size_t kMaxArrivals = 1 << 20;
  const std::vector<std::pair<int, int64_t>>& arrivals() const { return arrivals_; }

 private:
  const HostApi& api() const { return *api_; }
  void check_api(int rc, const char* what) const;
  void check_device() const;
  void launch();
  void wait_ring();  // until the next command's ring slot is free
  void write_cmd(const SrvCmd& c);
  // command k (-1: none) + releases (ks, vs) + replies; returns after the host part.
  // A delta (k >= 0) joins the open batch (flushed by flush_batch, at a logging delta or
  // when full); a release-only command flushes the batch first
  void issue(int k, int64_t vc, const int* ks, const int64_t* vs, int n);
  void flush_batch();
  int log_worker() const;

  PeerServerCfg cfg_;
  hipStream_t stream_;
  const HostApi* api_;
  int NS_ = 0;
  // device workspace
  void* ws_ = nullptr;
  SrvArgs args_{};
  // pinned
  TagChunk* cmd_ring_ = nullptr;
  unsigned long long* err_host_ = nullptr;
  unsigned long long* consumed_host_ = nullptr;
  int ring_ = 256;
  uint64_t cmds_ = 0;          // commands written (the kernel's numbering: 1..cmds_)
  uint64_t cmds_launch_ = 0;   // commands written before the current launch
  int64_t launches_ = 0;
  bool running_ = false;
  std::vector<uint32_t> ptag_;  // pulls sent per worker (the device counters' mirror)
  std::vector<uint8_t> finished_, failed_, dead_;
  std::vector<double> busy_since_;
  std::vector<int> rel_k_;
  std::vector<int64_t> rel_v_;
  std::vector<std::pair<int, int64_t>> arrivals_;
  // the open batch: entries, its server-row slot (the last entry's), the replies owed
  TagChunk* ent_ring_ = nullptr;  // pinned [ent_cap_][kEntChunks]
  int ent_cap_ = 0;
  uint64_t ents_ = 0;             // entries written (the kernel's numbering: 1..ents_)
  std::vector<SrvEnt> bat_;
  int bat_slot_ = -1;
  uint64_t bat_seq_ = 0;
  uintptr_t bat_addr_ = 0;
  int64_t bat_vc_ = 0;
  std::vector<CtrlToken> bat_rep_;
  int64_t batches_ = 0, batched_deltas_ = 0;
  int64_t updates_ = 0, tokens_ = 0, updates_run_ = 0;
  double host_ns_ = 0.0;
  uint64_t bsp_n_ = 0;  // BSP rounds commanded so far (the tag of the last one)
  long long* tr_ = nullptr;
  int tr_cap_ = 0;
  uint64_t tr_taken_ = 0;
  int64_t bsp_run_ = 0;
  double bsp_ns_ = 0.0;
  std::thread bsp_thr_;  // run_bsp_async
  std::exception_ptr bsp_err_;
  int64_t bsp_ret_ = 0;
};

}  // namespace psx
