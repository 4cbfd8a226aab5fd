// Native BSP round loop of up to 8 in-process workers sharing one MI355X
// ("lanes", csrc/kernels/lanes_kernels.h): ONE launch per round.
//
// Reference: the worker JVM hosts every logical worker (BaseKafkaApp.java:25,70,
// WorkerApp.java:31-43); under sequential consistency the server answers once
// every worker's gradient of the round arrived (ServerProcessor.java:111-120)
// with w += (1/N) delta_k applied per gradient (ServerProcessor.java:148-151).
//
// Per round, from C++ with no host synchronisation:
//   * every lane's producer delivers its due rows (per-round rows or the
//     reference producer clock) into its adaptive window (SlidingWindow, host
//     runtime C ABI); the rows themselves are copied into the lane's HBM ring by
//     the round kernel (a delivery that wraps its shard's epoch: the first part
//     by a ring-ingest launch);
//   * one lanes_round launch: every lane's solve on its own XCD, the cross-lane
//     update (the last lane to finish a slice applies the lane sum), and rider
//     workgroups evaluating the previous round's local + global models into the
//     metrics sink's pinned slots (worker rows, server row);
//   * multi-rank (comm != nullptr): the kernel writes the lane sum instead; the
//     rank reduces it to the server rank over RCCL and receives the new weights
//     by broadcast (BASELINE config 2/3 topology); on the server rank the update
//     and its fragments follow the reduce;
//   * multi-rank peer_sum (set_peer_sum, no communicator): the kernel stores the
//     lane sum into the rank's inbox slot on the server GPU itself and the next
//     round's launch -- already dispatched -- pulls the server kernel's update from
//     this rank's receive slot: no collective, host or kernel boundary in between;
//   * the vector-clock tracker advances one round; the device error word (pinned)
//     is polled: a timed-out cross-workgroup wait surfaces as an exception naming
//     the round.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

#include "../comm/comm.h"
#include "async_server.h"
#include "../host/capi.h"
#include "../kernels/lanes_kernels.h"

namespace psx {

struct LanesLoopCfg {
  SolverCfg scfg;  // K, F, Fp, P, cap, iters, hist, ls_max, mode, center, zero_const, nslots, gd_lr, tol
  // producer: worker k of N reads dataset rows k, k + N, ... (`epochs` passes)
  const uint16_t* dsX = nullptr;
  const int32_t* dsy = nullptr;
  int64_t ds_rows = 0;
  int N = 1;              // logical workers in the whole job
  int per_iter_rows = 0;  // > 0: rows per round; 0: the producer clock p_ms
  double p_ms = 0.0;
  int64_t epochs = 1;
  double t0_ms = 0.0;
  // lanes of this process
  int L = 0;
  std::vector<int> k;             // worker ids
  std::vector<uintptr_t> X, XT, y;  // rings [cap][Fp] bf16 (+ optional feature-major copy, kept in step), labels
  std::vector<uintptr_t> window;  // SlidingWindow*
  // server state (replica): w [P], its evaluation fragments (two buffers, columns scoff..)
  float* w = nullptr;
  float lr = 1.f;
  // (a third buffer enables overlapped launches, LanesArgs::ovl)
  uint16_t* shi[kLaneBufs] = {nullptr, nullptr, nullptr};
  uint16_t* slo[kLaneBufs] = {nullptr, nullptr, nullptr};
  float* sb[kLaneBufs] = {nullptr, nullptr, nullptr};
  int scoff = 0;
  // evaluation
  const uint16_t* Xt = nullptr;
  const int32_t* yt = nullptr;
  int T = 0;
  // the test set in ELL form (psx/ops/lr.py EvalSet.ell), used by the asynchronous lanes'
  // evaluation; tnz == 0: the dense pass
  const uint16_t* Ti = nullptr;
  const uint16_t* Tv = nullptr;
  int tnz = 0;
  uintptr_t sink = 0;       // MetricsSink* (0: no rows)
  bool log_server = true;   // server rows on this rank
  bool log_workers = true;  // worker rows on this rank
  uintptr_t tracker = 0;    // VectorClockTracker* (0: none)
  uintptr_t api = 0;        // HostApi*
  int server_rank = 0;      // multi-rank: the rank that applies the update
  // multi-rank schedule: false = reduce to the server rank, update there, broadcast
  // the weights (the PS push / pull); true = all-reduce of the lane sums, every rank
  // applies the same update to its replica (one collective per round)
  bool allreduce = false;
  // stream-driven cadence (the CLI's --iter_new_rows / --iter_new_frac / --iter_new_cap,
  // psx/runtime/config.py:new_tuples_needed): a round starts once every lane saw at
  // least max(new_rows, min(ceil(new_frac * window), new_cap)) new tuples since its
  // last solve (or its stream ended); 0 / 0.0: every round solves at once
  int new_rows = 0;
  double new_frac = 0.0;
  int new_cap = 0;
  // ... capped at new_ramp << (the lane's completed solves) for its first solves (0: off)
  int new_ramp = 0;
  // asynchronous consistency (run_async): the worker whose deltas produce the
  // server rows (ServerProcessor.java:154: worker 0, or the lowest live one;
  // -1: none) and injected straggler delays per lane (us, tests / fault injection)
  int log_worker = 0;
  std::vector<int> delay_us;
  // first XCD of this process's lanes (lane l on XCD xcd0 + l): processes that
  // share one GPU (IpcComm) take disjoint XCDs
  int xcd0 = 0;
};

class LanesLoop {
 public:
  // comm: the multi-rank job's transport (RcclComm: one rank per GPU; IpcComm:
  // ranks sharing one GPU) -- nullptr: one rank.  A rank with L == 0 is a
  // dedicated server rank.
  LanesLoop(const LanesLoopCfg& cfg, Comm* comm);
  ~LanesLoop();
  LanesLoop(const LanesLoop&) = delete;
  LanesLoop& operator=(const LanesLoop&) = delete;
  // Run `rounds` rounds from round r0; returns the rounds run (fewer when every
  // lane's stream is exhausted and its window empty).  max_wait_s: how long a
  // round may wait for a lane's first rows.  deadline_ms > 0 (epoch ms): a round
  // still waiting for rows or for the cadence at that time is not run (the call
  // returns the rounds run so far) -- the wall-clock stop of a producer-clock run.
  int64_t run(int64_t rounds, int64_t r0, hipStream_t stream, double max_wait_s = 600.0, double deadline_ms = 0.0);
  // Asynchronous consistency (SSP / ASP, the tracker's model): ONE persistent
  // launch (lanes_async.hip) serves `updates` solves.  The lanes the tracker has
  // dispatched start at once; every token (ticket, lane, vc) a lane pushes is
  // consumed here in ticket order -- its rows to the metrics sink,
  // tracker.on_delta, a release record (window, new rows, snapshot, slots) for
  // every released lane -- until `updates` solves ran (or the streams ended /
  // the deadline passed); then every lane gets a stop record and the launch
  // drains.  Releases not yet started carry over to the next call.  Returns the
  // updates applied.  per_lane > 0: no lane starts more than per_lane solves in this
  // call (max_iters = iterations per worker, also under ASP where fast workers would
  // otherwise take the slow ones' share of `updates`).
  int64_t run_async(int64_t updates, hipStream_t stream, double max_wait_s = 600.0, double deadline_ms = 0.0,
                    int64_t per_lane = 0);
  // lane_budget[l]: the most solves lane l starts in this call (empty: no per-lane bound) --
  // a chunked run (checkpoints) passes each worker's remaining share of max_iters
  int64_t run_async(int64_t updates, hipStream_t stream, double max_wait_s, double deadline_ms,
                    const std::vector<int64_t>& lane_budget);
  // Multi-rank SSP / ASP on a worker GPU: the server is rank 0 (AsyncServer,
  // async_server.h).  Same persistent launch in remote mode: a lane's push only
  // publishes its token; this loop sends the delta to peer 0 (`p2p`, on
  // `comm_stream`) with a control token (queue `ctrl`: worker, vc, FINAL on the
  // lane's last of `iters` solves), and answers the server's reply tokens (this
  // rank's queue `reply`: which worker the next weights are for) by receiving the
  // weights into that lane's slot and releasing the lane once they landed.
  // Returns the solves run (every lane's FINAL token sent).
  // p2p == nullptr: the peer data plane (set_peer) -- no host transfer at all.
  int64_t run_async_remote(P2P* p2p, uintptr_t ctrl, uintptr_t reply, int64_t iters, hipStream_t stream,
                           hipStream_t comm_stream, double max_wait_s = 600.0, double deadline_ms = 0.0);
  // Peer data plane (csrc/comm/peer_bus.h) for run_async_remote: this rank's receive
  // region (slot l = lane l's weights, written by the server GPU) and, per lane, its
  // worker's slot in the server's inbox (an IPC mapping).  Then run_async_remote takes
  // no transport: the lanes push their deltas into the inbox themselves and wait for
  // their slots' tags; the host only forwards tokens and answers reply tokens.
  void set_peer(uintptr_t rx_data, uintptr_t rx_tags, int64_t rx_stride, const std::vector<uintptr_t>& inbox,
                const std::vector<uintptr_t>& inbox_tag);
  bool peer() const { return peer_rx_ != nullptr; }
  // peer_sum BSP (multi-rank sequential consistency over the peer data plane; needs the
  // overlapped launches and no communicator): this rank's lane sums go to its inbox slot on
  // the server GPU (push / push_tag, an IPC mapping), the next round's weights come from
  // its receive slot (rx / rx_tag, fine-grained memory the server kernel writes, tag =
  // round + 1 after round `round`'s update) -- LanesArgs::push.  wait_s bounds a round's
  // pull wait (the slowest rank's round).  After a run() the rank's w holds the last update.
  void set_peer_sum(uintptr_t rx, uintptr_t rx_tag, uintptr_t push, uintptr_t push_tag, double wait_s);
  bool peer_sum() const { return psum_rx_ != nullptr; }
  // (diagnostics) this rank's receive-slot tags then its push tags, [2][FP/32] (synchronous)
  std::vector<unsigned> peer_sum_tags() const;
  // Ranks sharing one GPU: workgroups of this loop's launches on the XCDs of `mask` leave
  // at once (LanesArgs::xcd_skip) -- none of this loop's lanes may sit there
  void set_xcd_skip(unsigned mask);
  // Fault injection for the NEXT run_async (the Python schedulers'
  // --inject_worker_crash / --inject_worker_stop): crash[l] >= 0 -- lane l fails when
  // released after crash[l] more solves (no delta; `drop`: the tracker retires its
  // worker and the run goes on, else the run stops at once); stop[l] >= 0 -- lane l
  // leaves cleanly after stop[l] more solves (its last delta applied, then retired).
  // Empty vectors: none.  The workers concerned: crashed() / left() after the run.
  void set_injection(const std::vector<int64_t>& crash, const std::vector<int64_t>& stop, bool drop);
  // --trace / --perf_log: record every lane's phase times on the device (ring of cap
  // rounds / tickets; 0: off).  trace_take synchronises `s` and returns the entries
  // since the last take: BSP {0, round, lane, worker, stage, solve, solved, updated},
  // asynchronous {1, ticket, lane, worker, released, solved, pushed, 0} in s_memrealtime
  // ticks (100 MHz); clock_ref = {host CLOCK_MONOTONIC ns before, device ticks, ns after}.
  void set_trace(int cap);
  std::vector<std::vector<int64_t>> trace_take(hipStream_t s);
  std::vector<int64_t> clock_ref(hipStream_t s);
  const std::vector<int>& crashed() const { return crashed_; }
  const std::vector<int>& left() const { return left_; }
  // Debug (tests): every applied ticket's delta into buf [cap][P] (device, slot (t - 1) %
  // cap) and a host log per ticket of what the release that solved it carried:
  // {ticket, lane, worker, vc, snapshot ticket, B, start, first, step, n, first2, n2}
  void set_async_debug(uintptr_t buf, int cap) {
    dbg_delta_ = reinterpret_cast<float*>(buf);
    dbg_cap_ = cap;
  }
  const std::vector<std::vector<int64_t>>& async_log() const { return alog_; }
  // Allocate (and zero) the asynchronous workspace now: ranks sharing one GPU do this
  // before any rank's persistent launch holds CUs a fill kernel would wait for.  With
  // the peer data plane also one empty launch (every lane stopped at once) that drains
  // here: the first launch's one-time device work (the code object's load, the
  // runtime's copy paths) must not wait behind another rank's persistent launch.
  void prepare_async();
  int64_t tickets() const { return (int64_t)aticket_; }  // deltas applied by the asynchronous loop so far
  double host_us_per_update() const { return async_updates_ ? async_ns_ / 1000.0 / (double)async_updates_ : 0.0; }
  // host time spent per consumed token (token seen -> its rows handed over, tracker, the
  // releases it triggers written): the host loop's share of an asynchronous update
  double host_busy_us_per_token() const { return tok_n_ ? tok_ns_ / 1000.0 / (double)tok_n_ : 0.0; }
  // Evaluate the last round's rows (one launch of riders only).
  void flush(hipStream_t stream);
  void set_sink(uintptr_t sink) { cfg_.sink = sink; }
  // Idle waits of run_async / run_async_remote (a row-starved stream, a lane waiting for
  // its release): this bound, never below the in-flight watchdog max_wait_s (the CLI's
  // --idle_wait; default 600 s).  A short --worker_timeout then only bounds busy workers.
  void set_idle_wait(double s) { idle_wait_s_ = s > 0.0 ? s : 600.0; }
  void set_lr(float lr) { cfg_.lr = lr; }
  int64_t next_local(int lane) const { return next_local_.at(lane); }
  void set_next_local(int lane, int64_t v) { next_local_.at(lane) = v; }
  // tuples seen by lane `lane` when its last solve started (the cadence's origin)
  int64_t seen_at_solve(int lane) const { return seen_at_solve_.at(lane); }
  void set_seen_at_solve(int lane, int64_t v) { seen_at_solve_.at(lane) = v; }
  // new tuples lane windows of `size` rows wait for (0: no cadence)
  int64_t new_tuples_needed(int64_t size, int64_t updates = -1) const;  // updates < 0: no ramp
  bool exhausted(int lane) const { return next_local_[lane] >= local_total_[lane] * cfg_.epochs; }
  bool all_exhausted() const;
  int hand_off_scope() const { return S_; }  // 2: one-XCD hand-offs, 1: sc1 (placement check failed)
  // true: a round's rows are evaluated by a launch of their own on a side stream
  // that co-runs with the next round (8 lanes: no XCD left for riders)
  bool side_eval() const { return side_eval_; }
  // true (PSX_LANES_LANE_EVAL=1): each lane evaluates its own local model inside the
  // round kernel; false (default): the rider workgroups evaluate the previous round
  bool lane_eval() const { return lane_eval_; }
  // true (PSX_LANES_OVERLAP=1, one rank, rider evaluation, three fragment buffers):
  // consecutive rounds overlap (LanesArgs::ovl)
  bool overlap() const { return ovl_; }
  double host_us_per_round() const { return rounds_run_ ? host_ns_ / 1000.0 / (double)rounds_run_ : 0.0; }
  // the host loop's time per round by phase (us): [0] deliveries + window wait, [1]
  // evaluation slots (sink), [2] the launches (+ the stream operations of overlap),
  // [3] rows handed over, tracker, error words
  std::vector<double> host_phases_us() const {
    std::vector<double> v(4, 0.0);
    for (int i = 0; i < 4; ++i) v[i] = rounds_run_ ? host_ph_ns_[i] / 1000.0 / (double)rounds_run_ : 0.0;
    return v;
  }
  int64_t rounds_run() const { return rounds_run_; }
  int lanes() const { return cfg_.L; }
  // device stats of lane l's last solve: evals, accepted, ls failures, resets, error
  std::vector<int> stats(int lane, hipStream_t stream) const;
  float loss(int lane, hipStream_t stream) const;
  // the lane's last delta [P] (device pointer)
  uintptr_t delta_ptr(int lane) const;
  // stream-ordered copies of lane `lane`'s last loss (1 float) and delta (P floats);
  // a null destination is skipped
  void copy_out(int lane, uintptr_t loss_dst, uintptr_t delta_dst, hipStream_t stream) const;
  // every lane's at once (one launch): loss_dst / delta_dst per lane, 0 = skip
  void copy_out_all(const std::vector<uintptr_t>& loss_dst, const std::vector<uintptr_t>& delta_dst,
                    hipStream_t stream) const;
  // fault injection (tests): the rounds from r on run with a wait budget of `spin` polls
  void inject_spin_timeout(int64_t round, int spin) {
    inject_round_ = round;
    inject_spin_ = spin;
  }
  // Raise if a lane's solve reported a timed-out cross-workgroup wait (the pinned
  // error words; no synchronisation: call after one to cover every enqueued round).
  void poll_errors() { check_errors(-1); }
  // phase timeline of lane `lane`'s last solve (PSX_LANES_STAMPS=1 at construction):
  // [slot][k] s_memrealtime ticks (100 MHz), row 30 = the round's own phases
  std::vector<long long> read_stamps(int lane, hipStream_t stream) const;
  // the riders' timeline of the last launch that evaluated (PSX_LANES_STAMPS=1;
  // EvalMulti::dbg layout)
  std::vector<long long> read_rider_stamps(hipStream_t stream) const;
  // placement probe: blockIdx % 8 == XCC_ID for every workgroup of a large launch
  static bool probe_placement(hipStream_t stream);

 private:
  struct Pending {  // deferred evaluation rows of the previous round
    bool valid = false;
    bool workers = true;  // worker rows pending too (rider evaluation); false: the server row only
    int64_t vc = 0;
    int par = 0;
    std::vector<int64_t> nseen;
  };
  const HostApi& api() const { return *api_; }
  void check(int64_t rc, const char* what) const;
  int64_t poll(int lane, double now_ms, LaneRound* r, hipStream_t stream);
  // the rows staged for the round kernel in `r`: into the lane's ring by ring-ingest launches
  void flush_ingest(int lane, LaneRound* r, hipStream_t stream);
  void fill_eval(EvalMulti* ev, const Pending& p, std::vector<int>* slots, std::vector<uint64_t>* seqs,
                 std::vector<int>* kinds);
  void submit_rows(const Pending& p, const std::vector<int>& slots, const std::vector<uint64_t>& seqs,
                   const std::vector<int>& kinds);
  // lane evaluation (LanesArgs::lane_eval): this round's worker rows + the previous
  // round's server row in the round kernel; returns the rows to submit after the launch
  int fill_lane_eval(LanesArgs* a, int64_t r, int par, const std::vector<int64_t>& seen, SinkRecord* recs);
  void check_errors(int64_t round);
  int rider_count(int nmodels, int L) const;
  // ---- asynchronous loop ----
  void ensure_async();
  int64_t poll_async(int lane, double now_ms);  // due rows -> window + the lane's pending runs
  bool try_release(int lane, int64_t vc, double now_ms, int64_t snap = -1);
  void launch_async(hipStream_t stream, bool remote);
  void write_release(int lane, const RelRec& q);
  void stop_all(hipStream_t stream);
  void stop_lane(int l);  // lane l's stop record (once per launch)
  std::string launch_report();  // (failure reports) the persistent launch's progress

  LanesLoopCfg cfg_;
  Comm* comm_;
  const HostApi* api_;
  int S_ = 2;
  int P_ = 0;
  std::vector<int64_t> local_total_, next_local_, seen_at_solve_;
  std::vector<double> times_;
  void* ws_ = nullptr;  // device workspace of every lane + shared buffers
  LaneDev* lanes_dev_ = nullptr;
  std::vector<LaneDev> lanes_;
  unsigned* arrive_ = nullptr;
  int* acc_ = nullptr;
  unsigned* ticket_ = nullptr;
  unsigned* claim_ = nullptr;
  int64_t launches_ = 0;
  float* dsum_ = nullptr;
  uint16_t *upd_hi_ = nullptr, *upd_lo_ = nullptr;  // fragments of an update nobody evaluates
  float* upd_b_ = nullptr;
  unsigned long long* err_host_ = nullptr;  // pinned [kMaxLanes]
  // side-stream evaluation: events by round parity (round done -> evaluation;
  // evaluation done -> the round that rewrites that parity's fragments)
  bool side_eval_ = false;
  bool lane_eval_ = true;
  bool xcd_riders_ = false;
  bool tile_riders_ = false;
  bool lane_riders_ = false;
  int riders_ppi_ = 0;
  bool riders_gq_ = false;
  int* lacc_ = nullptr;
  unsigned* lticket_ = nullptr;
  hipStream_t side_ = nullptr;
  hipEvent_t ev_round_[2] = {nullptr, nullptr}, ev_eval_[2] = {nullptr, nullptr};
  bool eval_pending_[2] = {false, false};
  int* acc2_ = nullptr;
  unsigned* ticket2_ = nullptr;
  // cross-stream ordering: 0 = HIP events, 1 = stream memory ops on device flags
  // (PSX_SIDE_SYNC=value), 2 = none on the main stream (measurement only)
  int side_sync_ = 0;
  unsigned* sflags_ = nullptr;  // [0] last round done (main), [1] last evaluation done (side)
  long long* rider_dbg_ = nullptr;  // PSX_LANES_STAMPS: the riders' stamps
  // overlapped launches (PSX_LANES_OVERLAP=1, LanesArgs::ovl): rounds alternate between
  // the caller's stream and ostream_
  bool ovl_ = false;
  hipStream_t ostream_ = nullptr;
  hipEvent_t ovl_in_ = nullptr, ovl_out_ = nullptr, ovl_last_ = nullptr;
  unsigned* applied_ = nullptr;  // [32] LanesArgs::applied
  unsigned* evdone_ = nullptr;   // LanesArgs::evdone
  unsigned* ovlq_ = nullptr;     // the riders' tile queue (EvalMulti::xq) of overlapped launches
  int* slab_ = nullptr;          // EvalMulti::slab (overlapped launches, tile-resident riders)
  bool slab_on_ = false;         // PSX_RIDERS_SLAB (default 1): the slab form with overlap
  uint64_t ovl_n_ = 0;           // overlapped launches so far (LanesArgs::round)
  bool ovl_chain_ = false;       // a launch of this run() call precedes (wait for its dispatch)
  int ovl_prev_grid_ = 0, ovl_prev_cpar_ = 0;
  void ovl_wait_last(hipStream_t stream);  // a separate ring-ingest launch: after the last round
  int64_t eval_round_[2] = {-1, -1};
  Pending pend_;
  int last_par_ = 0;  // parity of the last round run
  int64_t inject_round_ = -1;
  int inject_spin_ = 0;
  int64_t rounds_run_ = 0;
  double host_ns_ = 0.0;
  double host_ph_ns_[4] = {0.0, 0.0, 0.0, 0.0};
  // asynchronous loop state (allocated by the first run_async)
  void* aws_ = nullptr;                 // device workspace
  AsyncLaneDev* al_dev_ = nullptr;      // device table
  std::vector<AsyncLaneDev> al_;
  AsyncRelease* rel_host_ = nullptr;    // pinned [L]
  AsyncToken* tok_host_ = nullptr;      // pinned [ring]
  AsyncArgs aargs_{};
  int R_ = 64, ring_ = 64;
  uint64_t aticket_ = 0;                // last ticket applied (device counter mirror)
  std::vector<uint64_t> relc_;          // release records written per lane
  std::vector<LaneRound> pend_r_;       // new stream rows not yet in the lane's ring
  enum { kIdle = 0, kWant = 1, kRunning = 2, kGone = 6 };
  std::vector<int> state_;
  std::vector<int64_t> inj_crash_, inj_stop_;  // set_injection (consumed by the next run_async)
  bool inj_drop_ = true;
  std::vector<int> crashed_, left_;             // workers that crashed / left in the last run
  long long* tr_ = nullptr;                     // set_trace ring (device)
  int tr_cap_ = 0;
  int64_t tr_n_ = 0, tr_taken_ = 0;             // BSP rounds recorded / taken
  std::vector<int64_t> tr_round_;               // round of each BSP ring slot
  uint64_t tr_tick_ = 0;                        // asynchronous: last ticket taken
  std::vector<uint8_t> lane_stopped_;           // lanes already sent their stop record (this launch)
  std::vector<int64_t> want_vc_;
  struct RunRec {
    int64_t vc = 0, nseen = 0;
    int slot_w = -1, slot_s = -1;
    uint64_t seq_w = 0, seq_s = 0;
    int64_t snap = 0;  // the pulled snapshot's ticket
    LaneRound r{};     // the window + new rows of the release
  };
  float* dbg_delta_ = nullptr;
  int dbg_cap_ = 0;
  std::vector<std::vector<int64_t>> alog_;
  std::vector<RunRec> runrec_;
  std::vector<int> lane_of_;            // worker id -> lane (-1: not on this loop)
  int log_lane_ = -1;
  int64_t launch_no_ = 0;
  double rel_wait_s_ = 60.0;  // the lanes' release / pull wait budget of the current run (device)
  double idle_wait_s_ = 600.0;  // set_idle_wait
  std::vector<hipEvent_t> pull_ev_;     // remote mode: a lane's weights received
  // peer data plane (set_peer): receive region, per-lane inbox slots, the pull tag of
  // each lane's pending release
  float* peer_rx_ = nullptr;
  unsigned* peer_rx_tag_ = nullptr;
  int64_t peer_stride_ = 0;
  std::vector<uintptr_t> peer_inbox_, peer_inbox_tag_;
  std::vector<unsigned> pull_tag_;
  // peer_sum BSP (set_peer_sum)
  const float* psum_rx_ = nullptr;
  const unsigned* psum_rx_tag_ = nullptr;
  float* psum_push_ = nullptr;
  unsigned* psum_push_tag_ = nullptr;
  long long psum_ticks_ = 0;
  unsigned xcd_skip_ = 0;  // set_xcd_skip
  // the persistent launch runs on a stream of its own (non-blocking: no implicit
  // synchronisation of the null stream, e.g. a host-staged transfer, waits for it),
  // ordered after / before the caller's stream by events
  hipStream_t astream_ = nullptr;
  hipEvent_t aev_in_ = nullptr, aev_out_ = nullptr;
  int64_t async_updates_ = 0;
  double async_ns_ = 0.0;
  int64_t tok_n_ = 0;
  double tok_ns_ = 0.0;
};

}  // namespace psx
