// Native BSP round loop (see bsp_loop.h).
#include "bsp_loop.h"

#include <chrono>
#include <stdexcept>
#include <string>
#include <thread>

#include "../kernels/lr_kernels.h"

namespace psx {

namespace {
double epoch_ms() {
  using namespace std::chrono;
  return (double)duration_cast<microseconds>(system_clock::now().time_since_epoch()).count() / 1000.0;
}
int64_t steady_ns() {
  using namespace std::chrono;
  return duration_cast<nanoseconds>(steady_clock::now().time_since_epoch()).count();
}
}  // namespace

BspLoop::BspLoop(LocalSolver* solver, RcclComm* comm, const BspLoopCfg& cfg)
    : solver_(solver), comm_(comm), cfg_(cfg), api_(reinterpret_cast<const HostApi*>(cfg.api)) {
  if (!solver_) throw std::invalid_argument("BspLoop: no solver");
  if (!api_ || api_->version != kHostApiVersion) throw std::invalid_argument("BspLoop: host runtime API mismatch");
  if (!cfg_.dsX || !cfg_.dsy || cfg_.ds_rows <= 0 || cfg_.N < 1 || cfg_.k < 0 || cfg_.k >= cfg_.N)
    throw std::invalid_argument("BspLoop: bad dataset / worker id");
  if (!cfg_.X || !cfg_.XT || !cfg_.y || cfg_.cap <= 0 || cfg_.cap != solver_->cfg().cap || !cfg_.window)
    throw std::invalid_argument("BspLoop: bad ring");
  if (cfg_.Fp != solver_->cfg().Fp || cfg_.K != solver_->cfg().K || cfg_.F != solver_->cfg().F)
    throw std::invalid_argument("BspLoop: model shape differs from the solver's");
  if (cfg_.per_iter_rows <= 0 && !(cfg_.p_ms > 0.0))
    throw std::invalid_argument("BspLoop: need rows per round or a producer period");
  if (!cfg_.w || !cfg_.shi || !cfg_.slo || !cfg_.sb || !cfg_.delta || cfg_.scoff < 0 || cfg_.scoff + cfg_.K > 16)
    throw std::invalid_argument("BspLoop: bad server replica");
  if (cfg_.sink && (!cfg_.Xt || !cfg_.yt || cfg_.T <= 0 || !cfg_.acc || !cfg_.ticket || !cfg_.whi || !cfg_.wlo ||
                    !cfg_.wb || cfg_.K > cfg_.scoff))
    throw std::invalid_argument("BspLoop: bad evaluation set / worker fragments");
  if (solver_->rows_mode() || !solver_->eager())
    throw std::invalid_argument("BspLoop: needs the eager small-window solver");
  local_total_ = cfg_.ds_rows > cfg_.k ? (cfg_.ds_rows - cfg_.k + cfg_.N - 1) / cfg_.N : 0;
  if (local_total_ == 0) throw std::invalid_argument("BspLoop: worker has no rows");
}

void BspLoop::check(int64_t rc, const char* what) const {
  if (rc < 0) throw std::runtime_error(std::string("BspLoop: ") + what + ": " + api().last_error());
}

void BspLoop::acquire(uint64_t* seq, uintptr_t* addr, int* slot) {
  *slot = api().sink_acquire(reinterpret_cast<void*>(cfg_.sink), seq, addr);
  check(*slot, "metrics sink acquire");
}

// Deliver the due rows (WorkerSamplingProcessor.java:50-113 through the window
// of the host runtime): every contiguous run but the last is copied into the
// ring by a ring-ingest launch; the last run is handed to the solve's first
// kernel (*fused) when it fits.  Returns the number of rows delivered.
int64_t BspLoop::poll(double now_ms, RingIngest* fused, hipStream_t stream) {
  if (exhausted()) return 0;
  const int64_t limit = local_total_ * cfg_.epochs - next_local_;
  int64_t n;
  if (cfg_.per_iter_rows > 0) {
    n = cfg_.per_iter_rows < limit ? cfg_.per_iter_rows : limit;
    times_.assign((size_t)n, now_ms);
  } else {
    const int64_t epoch = next_local_ / local_total_;
    const int64_t cur = next_local_ - epoch * local_total_;
    int64_t mx = limit < local_total_ - cur ? limit : local_total_ - cur;
    if (mx > (int64_t(1) << 22)) mx = int64_t(1) << 22;
    times_.resize(mx > 0 ? (size_t)mx : 1);
    n = api().due_rows(cfg_.k, cfg_.N, cfg_.p_ms, cfg_.ds_rows, cur, now_ms, mx, times_.data());
    check(n, "due_rows");
  }
  if (n <= 0) return 0;
  const int64_t first = api().window_insert_many(reinterpret_cast<void*>(cfg_.window), times_.data(), n);
  check(first, "window insert");
  const int64_t cap = cfg_.cap;
  const int64_t keep = n < cap ? n : cap;  // only the last cap rows can survive in the window
  const int64_t skip = n - keep;
  int64_t slot = (first + skip) % cap, pos = next_local_ + skip, remaining = keep;
  while (remaining > 0) {  // split at the shard's epoch boundaries
    const int64_t cur = pos % local_total_;
    const int64_t run = remaining < local_total_ - cur ? remaining : local_total_ - cur;
    const int64_t src_first = cfg_.k + cur * cfg_.N;
    if (run == remaining && run <= kMaxFusedIngest) {
      *fused = RingIngest{cfg_.dsX, cfg_.dsy, (long long)src_first, (long long)cfg_.N, (int)run, (int)slot};
    } else {
      launch_ring_ingest(cfg_.dsX, cfg_.dsy, src_first, cfg_.N, run, cfg_.X, cfg_.XT, cfg_.y, slot, cap, cfg_.Fp,
                         stream);
    }
    slot = (slot + run) % cap;
    pos += run;
    remaining -= run;
  }
  next_local_ += n;
  return n;
}

int64_t BspLoop::run(int64_t rounds, int64_t r0, hipStream_t stream) {
  const int64_t t_begin = steady_ns();
  const int64_t KF = (int64_t)cfg_.K * cfg_.Fp;
  const int64_t P = KF + cfg_.K;
  void* win = reinterpret_cast<void*>(cfg_.window);
  void* sink = reinterpret_cast<void*>(cfg_.sink);
  int64_t done = 0;
  for (; done < rounds; ++done) {
    const int64_t r = r0 + done;
    const double now = epoch_ms();
    RingIngest ing{};
    poll(now - cfg_.t0_ms, &ing, stream);
    int64_t size = 0, start = 0, seen = 0;
    check(api().window_state(win, &size, &start, &seen), "window state");
    // no rows yet: wait for the producer as the Python loop does (a poll that
    // delivers anything makes the window non-empty, so no staged run is lost);
    // an exhausted stream with an empty window ends the run
    const double wait0 = epoch_ms();
    while (size <= 0 && !exhausted()) {
      if (epoch_ms() - wait0 > 600e3) throw std::runtime_error("BspLoop: no rows for 600 s");
      std::this_thread::sleep_for(std::chrono::microseconds(500));
      poll(epoch_ms() - cfg_.t0_ms, &ing, stream);
      check(api().window_state(win, &size, &start, &seen), "window state");
    }
    if (size <= 0) break;
    // ---- the previous round's rows ride in this solve ----
    EvalRide ride{};
    bool riding = false;
    int slot_w = -1, slot_s = -1;
    uint64_t seq_w = 0, seq_s = 0;
    if (sink && (pend_w_.vc >= 0 || pend_s_.vc >= 0)) {
      uintptr_t addr_w = 0, addr_s = 0;
      ride.Xt = cfg_.Xt;
      ride.yt = cfg_.yt;
      ride.T = cfg_.T;
      ride.K = cfg_.K;
      ride.acc = cfg_.acc;
      ride.ticket = cfg_.ticket;
      ride.nticket = (unsigned)ride.ntiles();
      if (pend_w_.vc >= 0) {
        acquire(&seq_w, &addr_w, &slot_w);
        ride.whi = cfg_.whi;
        ride.wlo = cfg_.wlo;
        ride.wb = cfg_.wb;
        ride.coff1 = 0;
        ride.loss = cfg_.loss;
        ride.slot = reinterpret_cast<char*>(addr_w);
        ride.seq = seq_w;
        if (pend_s_.vc >= 0) {
          acquire(&seq_s, &addr_s, &slot_s);
          ride.shi = cfg_.shi;
          ride.slo = cfg_.slo;
          ride.sb = cfg_.sb;
          ride.coff2 = cfg_.scoff;
          ride.slot2 = reinterpret_cast<char*>(addr_s);
          ride.seq2 = seq_s;
        }
      } else {  // a server row alone: the global model is the pass's only model
        acquire(&seq_s, &addr_s, &slot_s);
        ride.whi = cfg_.shi;
        ride.wlo = cfg_.slo;
        ride.wb = cfg_.sb;
        ride.coff1 = cfg_.scoff;
        ride.slot = reinterpret_cast<char*>(addr_s);
        ride.seq = seq_s;
      }
      riding = true;
    }
    FusedApply ap{};
    if (!comm_) {  // world 1: w = w_old + lr * delta inside the solve's finalisation
      ap.w = cfg_.w;
      ap.lr = cfg_.lr;
      ap.hi = cfg_.shi;
      ap.lo = cfg_.slo;
      ap.b = cfg_.sb;
      ap.coff = cfg_.scoff;
    }
    solver_->run((int)size, (int)start, stream, ing, riding ? &ride : nullptr, comm_ ? nullptr : &ap);
    if (riding) {  // records in the reference's order: the server row, then the worker row
      if (slot_s >= 0)
        api().sink_submit(sink, slot_s, seq_s, 1, pend_s_.ts, -1, pend_s_.vc, 0);
      if (slot_w >= 0)
        api().sink_submit(sink, slot_w, seq_w, 0, pend_w_.ts, cfg_.k, pend_w_.vc, pend_w_.nseen);
      pend_w_ = BspRow{};
      pend_s_ = BspRow{};
    }
    const int64_t ts_w = -1;  // the sink stamps the row when its evaluation lands
    if (comm_) {  // the round's deltas summed over the ranks (xGMI), then the update
      comm_->all_reduce(cfg_.delta, cfg_.delta, (size_t)P, RcclComm::kF32, stream);
      launch_server_apply(cfg_.K, cfg_.F, cfg_.Fp, cfg_.w, cfg_.delta, cfg_.lr, cfg_.shi, cfg_.slo, cfg_.sb, stream,
                          cfg_.scoff);
      hip_check(hipGetLastError(), "server update launch");
    }
    if (sink) {
      pend_w_ = BspRow{r, seen, ts_w};
      if (cfg_.log_server) pend_s_ = BspRow{r, 0, -1};
    }
    if (cfg_.tracker) check(api().tracker_bsp_round(reinterpret_cast<void*>(cfg_.tracker), r), "tracker");
  }
  rounds_run_ += done;
  updates_ += done;
  host_ns_ += (double)(steady_ns() - t_begin);
  return done;
}

void BspLoop::flush(hipStream_t stream) {
  if (!cfg_.sink || (pend_w_.vc < 0 && pend_s_.vc < 0)) return;
  void* sink = reinterpret_cast<void*>(cfg_.sink);
  int slot_w = -1, slot_s = -1;
  uint64_t seq_w = 0, seq_s = 0;
  uintptr_t addr_w = 0, addr_s = 0;
  EvalApply ea{};
  if (pend_w_.vc >= 0) {
    acquire(&seq_w, &addr_w, &slot_w);
    if (pend_s_.vc >= 0) {
      acquire(&seq_s, &addr_s, &slot_s);
      ea.shi = cfg_.shi;
      ea.slo = cfg_.slo;
      ea.sb = cfg_.sb;
    }
    launch_eval_apply(cfg_.Fp, cfg_.K, cfg_.Xt, cfg_.yt, cfg_.T, cfg_.whi, cfg_.wlo, cfg_.wb, cfg_.acc, stream,
                      cfg_.ticket, reinterpret_cast<void*>(addr_w), cfg_.loss, seq_w, 0, cfg_.scoff,
                      slot_s >= 0 ? reinterpret_cast<void*>(addr_s) : nullptr, seq_s, ea);
  } else {
    acquire(&seq_s, &addr_s, &slot_s);
    launch_eval_apply(cfg_.Fp, cfg_.K, cfg_.Xt, cfg_.yt, cfg_.T, cfg_.shi, cfg_.slo, cfg_.sb, cfg_.acc, stream,
                      cfg_.ticket, reinterpret_cast<void*>(addr_s), nullptr, seq_s, cfg_.scoff, 0, nullptr, 0, ea);
  }
  hip_check(hipGetLastError(), "evaluation launch");
  if (slot_s >= 0) api().sink_submit(sink, slot_s, seq_s, 1, pend_s_.ts, -1, pend_s_.vc, 0);
  if (slot_w >= 0) api().sink_submit(sink, slot_w, seq_w, 0, pend_w_.ts, cfg_.k, pend_w_.vc, pend_w_.nseen);
  pend_w_ = BspRow{};
  pend_s_ = BspRow{};
}

}  // namespace psx
