// Native server loop of the asynchronous consistency models (SSP, ASP).
//
// Reference: ServerProcessor.process (ServerProcessor.java:143-183) consumes
// GRADIENTS_TOPIC -- ONE Kafka partition, so deltas are applied strictly one
// after another in arrival order -- applies w += lr * delta, logs a server row
// on worker-0 deltas, and answers every worker the MessageTracker releases
// (MessageTracker.java:69-87).  Here:
//   * arrival order = the shared-memory token queue (csrc/host/ctrl.h): a worker
//     pushes (worker, vc) once its delta is complete on its GPU;
//   * data plane = RCCL point-to-point over xGMI: for each token the loop enqueues
//     ncclRecv(delta <- worker), the update kernel, the evaluation kernel (server
//     rows) and one grouped ncclSend(w -> j) per released worker, all on ONE
//     server stream, so updates, evaluations and snapshots are ordered exactly
//     like the single partition (no torn reads: a send of w is enqueued after the
//     update that produced it and before the next one);
//   * no host synchronisation: the loop never waits for the device, only for
//     tokens; the device runs the enqueued schedule behind it.
// The tracker, token queue and metrics sink belong to the host runtime
// (_psx_host) and are driven through its C ABI (csrc/host/capi.h).
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "../comm/rccl_comm.h"
#include "../host/capi.h"

namespace psx {

enum AsyncModel : int { kAsyncDense = 0, kAsyncWideSparse = 1, kAsyncWideDense = 2 };

// Point-to-point data plane of the server loop.  Peer 0 is the server, worker
// k is peer k + 1.  Every operation is stream-ordered on the server's stream.
class P2P {
 public:
  virtual ~P2P() = default;
  virtual int size() const = 0;  // server + workers
  virtual void send(const void* buf, size_t count, int dtype, int peer, hipStream_t s) = 0;
  virtual void recv(void* buf, size_t count, int dtype, int peer, hipStream_t s) = 0;
  virtual void group_start() {}
  virtual void group_end() {}
};

// RCCL over xGMI: one process per GPU (the production transport).
class RcclP2P : public P2P {
 public:
  explicit RcclP2P(RcclComm* c);
  int size() const override { return c_->size(); }
  void send(const void* buf, size_t count, int dtype, int peer, hipStream_t s) override {
    c_->send(buf, count, dtype, peer, s);
  }
  void recv(void* buf, size_t count, int dtype, int peer, hipStream_t s) override {
    c_->recv(buf, count, dtype, peer, s);
  }
  void group_start() override { c_->group_start(); }
  void group_end() override { c_->group_end(); }

 private:
  RcclComm* c_;
};

// Same-process transport (server and workers on ONE GPU -- RCCL refuses two
// ranks per device): worker k's pushed payloads sit in its outboxes (one per
// dtype: feature ids int32, values fp32), its pulled weights land in its inbox;
// a recv / send is a stream-ordered device copy, and every send to k bumps k's
// release counter, which in-process workers poll.  Exercises the identical
// server loop on a one-GPU box (tests, the host-cost microbench).
class LocalP2P : public P2P {
 public:
  LocalP2P(int nworkers, const std::vector<uintptr_t>& out_f32, const std::vector<uintptr_t>& out_i32,
           const std::vector<uintptr_t>& inbox);
  int size() const override { return n_ + 1; }
  void send(const void* buf, size_t count, int dtype, int peer, hipStream_t s) override;
  void recv(void* buf, size_t count, int dtype, int peer, hipStream_t s) override;
  void group_start() override;
  void group_end() override;  // one release per peer that got sends in the group
  int64_t released(int k) const;

 private:
  int n_;
  bool in_group_ = false;
  std::vector<int> group_peers_;
  std::vector<uintptr_t> out_f32_, out_i32_, inbox_;
  std::unique_ptr<std::atomic<int64_t>[]> released_;
};

// Host shared-memory transport between processes (one host, no GPU transport):
// a byte FIFO per direction per worker in one POSIX shm segment, messages in the
// order they are sent (RCCL's per-peer send / recv order).  It carries the same
// server loop across processes on the CPU (tests, the plumbing config) and on a
// GPU whose ranks cannot open an RCCL communicator (several ranks per device):
// device buffers are staged through the host after a stream synchronisation.
// rank 0 = the server (creates the segment), rank k + 1 = worker k.
class HostP2P : public P2P {
 public:
  HostP2P(const std::string& name, int nworkers, int rank, bool create, bool device, size_t cap_bytes,
          double timeout_s);
  ~HostP2P() override;
  int size() const override { return n_ + 1; }
  void send(const void* buf, size_t count, int dtype, int peer, hipStream_t s) override;
  void recv(void* buf, size_t count, int dtype, int peer, hipStream_t s) override;
  void unlink();

 private:
  struct Chan;
  Chan* chan(int idx) const;
  int out_chan(int peer) const;
  int in_chan(int peer) const;
  void write(Chan* c, const char* src, size_t n);
  void read(Chan* c, char* dst, size_t n);
  std::string name_;
  int n_, rank_;
  bool owner_, device_;
  size_t cap_, map_bytes_ = 0;
  double timeout_s_;
  char* base_ = nullptr;
  // pinned staging (device ranks): the copies run on the DMA engines, so a rank whose
  // CUs are held by a persistent launch still moves its messages
  char* bounce_ = nullptr;
  size_t bounce_bytes_ = 0;
  char* staging(size_t bytes);
};

struct AsyncServerCfg {
  int nworkers = 0;
  int model = kAsyncDense;
  float lr = 1.f;
  int64_t P = 0;         // weight entries (dense pushes carry P floats)
  float* w = nullptr;    // fp32 master weights [P]
  float* buf = nullptr;  // receive buffer [P] (dense pushes)
  // dense model: evaluation fragments of w + the device-resident test set
  int K = 0, F = 0, FP = 0, coff = 0;
  uint16_t* fhi = nullptr;
  uint16_t* flo = nullptr;
  float* fb = nullptr;
  const uint16_t* Xt = nullptr;
  const int32_t* yt = nullptr;
  int T = 0;
  // wide model: sparse pushes (feature ids, values) + CSR test set
  int KP = 0;
  int64_t Fw = 0;
  int umax = 0;
  int32_t* ubuf = nullptr;  // [umax]
  float* dbuf = nullptr;    // [KP + umax * KP]
  const int64_t* t_indptr = nullptr;
  const int32_t* t_idx = nullptr;
  const uint16_t* t_val = nullptr;
  const int32_t* t_y = nullptr;
  // evaluation scratch (accumulators + ticket of the server's evaluations)
  int* acc = nullptr;
  unsigned* ticket = nullptr;
  // host runtime handles (capi.h); sink 0: no server rows
  uintptr_t api = 0, tracker = 0, ctrl = 0, sink = 0;
  double worker_timeout_s = 600.0;
  // sparse pull (kAsyncWideSparse): the applied pushes go into a ring log
  // (lids[logcap] ids, lvals[logcap * KP] values); a released worker receives
  // the entries since its previous pull (sizes on its reply queue) unless the
  // dense vector is cheaper, it fell behind the log, or dense_every sparse pulls
  // passed (a dense refresh bounds the atomics' rounding drift)
  int sparse_pull = 0;
  int32_t* lids = nullptr;
  float* lvals = nullptr;
  int64_t logcap = 0;
  std::vector<uintptr_t> replies;  // per-worker reply CtrlQueue handles
  int dense_every = 64;
  // worker k's p2p peer (empty: k + 1, one worker per rank).  Several workers per
  // rank (the asynchronous lanes loop on worker GPUs) share their rank's peer and
  // reply queue: a dense pull then also carries a reply token, so the rank knows
  // which of its workers the next weights are for (per-peer send order)
  std::vector<int> peer;
  // host memory server (CPU ranks): the update / log / evaluation run on the host
  // (same arithmetic as the kernels; no evaluation fragments)
  int cpu = 0;
};

enum AsyncCode : int {
  kAsyncDone = 0,        // every worker sent its final delta (or failed)
  kAsyncErrorToken = 1,  // `worker` reported an error: caller decides (retire via fail(), or abort)
  kAsyncWatchdog = 2,    // `worker` busy and silent longer than the timeout
  kAsyncCheckpoint = 3,  // `updates` reached a multiple of checkpoint_every
};

struct AsyncStatus {
  int code = kAsyncDone;
  int worker = -1;
  int64_t updates = 0;
};

class AsyncServer {
 public:
  AsyncServer(P2P* p2p, const AsyncServerCfg& cfg, hipStream_t stream);
  // New run: workers that finished the previous run rejoin (failed ones stay
  // retired), every live worker gets the weights of its current clock (the
  // bootstrap: vc 0 on a fresh tracker).
  void begin();
  // Serve tokens until every worker finished (or a code that needs the caller).
  AsyncStatus run(int64_t checkpoint_every);
  // Retire worker k (failed): the tracker stops waiting for it; the workers it
  // held back are answered.
  void fail(int k);
  int64_t updates() const { return updates_; }
  void set_updates(int64_t u) { updates_ = u; }
  int64_t tokens() const { return tokens_; }
  double host_us_per_update() const { return updates_run_ ? host_ns_ / 1000.0 / (double)updates_run_ : 0.0; }
  std::vector<int> failed() const;
  void set_stream(hipStream_t s) { stream_ = s; }

 private:
  const HostApi& api() const { return *api_; }
  void check_api(int rc, const char* what) const;
  void send_weights(const int* ks, const int64_t* vs, int n);
  void apply_and_log(const CtrlToken& t);
  void apply_cpu(const CtrlToken& t);
  void eval_cpu(char* slot, uint64_t seq);
  int log_worker() const;
  int peer_of(int k) const { return cfg_.peer.empty() ? k + 1 : cfg_.peer[k]; }

  P2P* comm_;
  AsyncServerCfg cfg_;
  hipStream_t stream_;
  const HostApi* api_;
  std::vector<uint8_t> finished_, failed_;  // this run
  std::vector<uint8_t> dead_;               // failed in any run: never revived
  std::vector<double> busy_since_;  // < 0: not busy (weights not sent / delta back)
  std::vector<int> rel_k_;
  std::vector<int64_t> rel_v_;
  int64_t log_pos_ = 0;                 // ids appended to the log so far
  std::vector<int64_t> last_pos_;       // log position of each worker's last pull (-1: dense next)
  std::vector<int> since_dense_;        // sparse pulls since the worker's last dense pull
  int64_t sparse_pulls_ = 0, dense_pulls_ = 0, pull_floats_ = 0;

 public:
  int64_t sparse_pulls() const { return sparse_pulls_; }
  int64_t dense_pulls() const { return dense_pulls_; }
  int64_t pull_floats() const { return pull_floats_; }  // values + ids moved by pulls
  int64_t updates_ = 0, tokens_ = 0, updates_run_ = 0;
  double host_ns_ = 0.0;
};

// In-process stand-ins for the worker ranks of a LocalP2P server: thread k
// waits until the server has released it for its next clock (LocalP2P's
// release counter), then pushes the token of a delta already in its outbox
// (vc = its clock, the last one FINAL).  Workers that do no training: the
// protocol, the tracker decisions and the server's host cost in isolation.
class LocalFeeder {
 public:
  // vc0[k]: worker k's clock at the start (the tracker's); the release counter's
  // value at construction is the baseline (construct before the server's begin())
  LocalFeeder(uintptr_t api, uintptr_t ctrl, LocalP2P* p2p, int nworkers, int64_t iters, int64_t token_n,
              double timeout_s, const std::vector<int64_t>& vc0, const std::vector<uintptr_t>& replies = {});
  int64_t sparse_pulls() const { return sparse_.load(); }
  ~LocalFeeder();
  void start();
  // true: every thread pushed all its tokens; false: a thread timed out waiting
  bool join();

 private:
  void run(int k);
  const HostApi* api_;
  uintptr_t ctrl_;
  LocalP2P* p2p_;
  int n_;
  int64_t iters_, token_n_;
  double timeout_s_;
  std::vector<int64_t> vc0_, base_;
  std::vector<uintptr_t> replies_;  // sparse pull: each release comes with a reply token
  std::atomic<int64_t> sparse_{0};
  std::vector<std::thread> th_;
  std::atomic<int> failed_{0};
};

}  // namespace psx
