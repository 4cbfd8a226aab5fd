// Native key-range sharded BSP loop (see keyrange_loop.h).
#include "keyrange_loop.h"

#include <chrono>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>

#include "../kernels/common.h"
#include "../kernels/keyrange_kernels.h"
#include "../solver/solver.h"  // hip_check

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
size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }
}  // namespace

KeyRangeLoop::KeyRangeLoop(const KeyRangeLoopCfg& cfg, RcclComm* comm)
    : cfg_(cfg), comm_(comm), api_(reinterpret_cast<const HostApi*>(cfg.api)) {
  if (!api_ || api_->version != kHostApiVersion) throw std::invalid_argument("KeyRangeLoop: host runtime API mismatch");
  W_ = comm_ ? comm_->size() : 1;
  rank_ = comm_ ? comm_->rank() : 0;
  if (W_ > kMaxOwners) throw std::invalid_argument("KeyRangeLoop: at most 64 ranks");
  WideCfg& c = cfg_.wcfg;
  KP_ = c.KP;
  S_ = (c.F + W_ - 1) / W_;
  lo_ = (int64_t)rank_ * S_;
  hi_ = lo_ + S_ < c.F ? lo_ + S_ : c.F;
  if (lo_ >= hi_) throw std::invalid_argument("KeyRangeLoop: more ranks than features");
  if (!cfg_.indptr || !cfg_.idx || !cfg_.val || !cfg_.y || cfg_.ds_rows <= 0 || cfg_.k < 0 || cfg_.k >= cfg_.N)
    throw std::invalid_argument("KeyRangeLoop: bad dataset / worker id");
  if (cfg_.per_iter_rows <= 0 && !(cfg_.p_ms > 0.0))
    throw std::invalid_argument("KeyRangeLoop: need rows per round or a producer period");
  if (!cfg_.ridx || !cfg_.rval || !cfg_.rnnz || !cfg_.ry || !cfg_.trunc || !cfg_.window)
    throw std::invalid_argument("KeyRangeLoop: bad ring / window");
  if (!cfg_.shard || !cfg_.b) throw std::invalid_argument("KeyRangeLoop: no shard");
  const bool evaluates = cfg_.sink && (cfg_.log_server || cfg_.log_workers);
  if (evaluates && (!cfg_.t_indptr || !cfg_.t_idx || !cfg_.t_val || !cfg_.t_y || cfg_.T <= 0 || !cfg_.s_indptr ||
                    !cfg_.s_idx || !cfg_.s_val))
    throw std::invalid_argument("KeyRangeLoop: no test set");
  local_total_ = cfg_.ds_rows > cfg_.k ? (cfg_.ds_rows - cfg_.k + cfg_.N - 1) / cfg_.N : 0;
  if (local_total_ == 0) throw std::invalid_argument("KeyRangeLoop: the worker has no rows");
  c.pulled = W_ > 1 ? 1 : 0;  // world 1: the solve reads the (whole) shard in place
  c.own_W = W_;
  c.own_S = S_;
  c.dense_delta = 0;
  // the launch chain (graph replay) by default; PSX_WIDE_PERSIST=1: the whole solve
  // (pull mode: its second phase) in one persistent launch.  Measured on MI355X
  // (profiles/r03_v5): sharded100m 0.163 ms per round with the chain, 0.365 ms with
  // the persistent launch -- its 256 workgroups x 512 threads pay a grid barrier per
  // phase (~9 per solve + 3 per slot) where the chain's small launches overlap
  const char* wp = std::getenv("PSX_WIDE_PERSIST");
  c.persist = wp ? (wp[0] == '1' ? 1 : 0) : 0;
  const int64_t E = (int64_t)c.cap * c.NZ;
  umax_ = (int)(c.F < E ? c.F : E);

  size_t off = 0;
  auto take = [&](size_t bytes) {
    const size_t o = off;
    off = align_up(off + bytes, 256);
    return o;
  };
  const size_t o_pull = take((size_t)umax_ * KP_ * 4 + 64);
  const size_t o_rid = W_ > 1 ? take((size_t)W_ * umax_ * 4) : 0;
  const size_t o_rval = W_ > 1 ? take((size_t)W_ * umax_ * KP_ * 4) : 0;
  const size_t o_db = take(16 * 4);
  const size_t o_z0 = evaluates ? take((size_t)cfg_.T * KP_ * 4) : 0;
  const size_t o_z1 = evaluates ? take((size_t)cfg_.T * KP_ * 4) : 0;
  if (cfg_.margin_refresh < 1) cfg_.margin_refresh = 1;
  const size_t o_acc = take((size_t)512 * kAccStride * 4);
  const size_t o_tic = take(64);
  const size_t o_cnt = take((size_t)2 * kMaxOwners * 4);
  ws_bytes_ = off;
  hip_check(hipMalloc(&ws_, ws_bytes_), "hipMalloc(keyrange workspace)");
  hip_check(hipMemset(ws_, 0, ws_bytes_), "hipMemset(keyrange workspace)");
  char* bp = static_cast<char*>(ws_);
  w_pull_ = reinterpret_cast<float*>(bp + o_pull);
  req_ids_ = W_ > 1 ? reinterpret_cast<int32_t*>(bp + o_rid) : nullptr;
  req_vals_ = W_ > 1 ? reinterpret_cast<float*>(bp + o_rval) : nullptr;
  db_ = reinterpret_cast<float*>(bp + o_db);
  if (evaluates) {
    z_ = reinterpret_cast<float*>(bp + o_z0);
    dz_ = reinterpret_cast<float*>(bp + o_z1);
  }
  acc_ = reinterpret_cast<int*>(bp + o_acc);
  ticket_ = reinterpret_cast<unsigned*>(bp + o_tic);
  cnt_dev_ = reinterpret_cast<unsigned*>(bp + o_cnt);
  hip_check(hipHostMalloc((void**)&cnt_host_, 2 * kMaxOwners * 4, hipHostMallocCoherent | hipHostMallocMapped),
            "hipHostMalloc(counts)");
  std::memset(cnt_host_, 0, 2 * kMaxOwners * 4);

  WideBuffers wb;
  wb.ridx = cfg_.ridx;
  wb.rval = cfg_.rval;
  wb.rnnz = cfg_.rnnz;
  wb.ry = cfg_.ry;
  wb.w_pull = W_ > 1 ? w_pull_ : nullptr;
  wb.w_old = W_ > 1 ? nullptr : cfg_.shard;
  wb.w_pull_b = cfg_.b;  // the replicated intercepts are read in place
  wb.dloc = cfg_.dloc;
  wb.wloc = cfg_.wloc;
  wb.loss = cfg_.loss;
  wb.stats = cfg_.stats;
  wb.uniq = cfg_.uniq;
  solver_ = std::make_unique<WideSolver>(c, wb, cfg_.use_graph);
}

KeyRangeLoop::~KeyRangeLoop() {
  solver_.reset();
  if (ws_) (void)hipFree(ws_);
  if (cnt_host_) (void)hipHostFree(cnt_host_);
}

void KeyRangeLoop::check(int64_t rc, const char* what) const {
  if (rc < 0) throw std::runtime_error(std::string("KeyRangeLoop: ") + what + ": " + api().last_error());
}

int64_t KeyRangeLoop::last_u() const { return (int64_t)solver_->ucount_host(); }

// The worker's due rows -> its window and ring (WorkerSamplingProcessor.java:
// 50-113 through the host runtime's SlidingWindow; the rows are gathered from
// the resident CSR dataset, split at the shard's epoch boundaries).
int64_t KeyRangeLoop::poll(double now_ms, hipStream_t stream) {
  if (exhausted()) return 0;
  const int64_t lt = local_total_;
  const int64_t limit = lt * cfg_.epochs - next_local_;
  int64_t n;
  if (cfg_.per_iter_rows > 0) {
    n = cfg_.per_iter_rows < limit ? cfg_.per_iter_rows : limit;
    times_.assign((size_t)n, now_ms);
  } else {
    const int64_t epoch = next_local_ / lt, cur = next_local_ - epoch * lt;
    int64_t mx = limit < lt - cur ? limit : lt - cur;
    if (mx > (int64_t(1) << 22)) mx = int64_t(1) << 22;
    times_.resize(mx > 0 ? (size_t)mx : 1);
    n = api().due_rows(cfg_.k, cfg_.N, cfg_.p_ms, cfg_.ds_rows, cur, now_ms, mx, times_.data());
    check(n, "due_rows");
  }
  if (n <= 0) return 0;
  const int64_t first = api().window_insert_many(reinterpret_cast<void*>(cfg_.window), times_.data(), n);
  check(first, "window insert");
  const int64_t cap = cfg_.wcfg.cap;
  const int64_t keep = n < cap ? n : cap, skip = n - keep;
  int64_t slot = (first + skip) % cap, pos = next_local_ + skip, remaining = keep;
  while (remaining > 0) {
    const int64_t cur = pos % lt;
    const int64_t run = remaining < lt - cur ? remaining : lt - cur;
    launch_sparse_ring_ingest(cfg_.indptr, cfg_.idx, cfg_.val, cfg_.y, cfg_.k + cur * (int64_t)cfg_.N, cfg_.N, run,
                              cfg_.ridx, cfg_.rval, cfg_.rnnz, cfg_.ry, slot, (int)cap, cfg_.wcfg.NZ, cfg_.trunc,
                              stream);
    slot = (slot + run) % cap;
    pos += run;
    remaining -= run;
  }
  hip_check(hipGetLastError(), "sparse ring ingest");
  next_local_ += n;
  return n;
}

// Reduced partial margins of the sharded global model (coefficients only).
void KeyRangeLoop::margins(float* z, hipStream_t stream) {
  const WideCfg& c = cfg_.wcfg;
  launch_wide_logits(c.K, KP_, hi_ - lo_, cfg_.s_indptr, cfg_.s_idx, cfg_.s_val, cfg_.T, cfg_.shard, z, stream);
  hip_check(hipGetLastError(), "partial margins");
  if (W_ > 1) {
    comm_->all_reduce(z, z, (size_t)cfg_.T * KP_, RcclComm::kF32, stream);
    eval_bytes_ += (int64_t)cfg_.T * KP_ * 4;
  }
}

// Segment j of `send` (elements [soff[j], soff[j] + scnt[j])) -> rank j, segment
// j of `recv` <- rank j; the rank's own segment is a device copy.
void KeyRangeLoop::exchange(const void* send, const int64_t* soff, const int64_t* scnt, void* recv,
                            const int64_t* roff, const int64_t* rcnt, int elem, int dtype, hipStream_t stream) {
  const char* sp = static_cast<const char*>(send);
  char* rp = static_cast<char*>(recv);
  const size_t es = 4;
  if (scnt[rank_] > 0)
    hip_check(hipMemcpyAsync(rp + (size_t)roff[rank_] * elem * es, sp + (size_t)soff[rank_] * elem * es,
                             (size_t)scnt[rank_] * elem * es, hipMemcpyDeviceToDevice, stream),
              "keyrange self copy");
  comm_->group_start();
  for (int j = 0; j < W_; ++j) {
    if (j == rank_) continue;
    if (scnt[j] > 0) {
      comm_->send(sp + (size_t)soff[j] * elem * es, (size_t)scnt[j] * elem, dtype, j, stream);
      last_round_bytes_ += scnt[j] * elem * (int64_t)es;
    }
    if (rcnt[j] > 0) comm_->recv(rp + (size_t)roff[j] * elem * es, (size_t)rcnt[j] * elem, dtype, j, stream);
  }
  comm_->group_end();
}

int64_t KeyRangeLoop::run(int64_t rounds, int64_t r0, hipStream_t stream, double max_wait_s) {
  const int64_t t_begin = steady_ns();
  const WideCfg& c = cfg_.wcfg;
  const bool evaluates = cfg_.sink && (cfg_.log_server || cfg_.log_workers);
  void* sink = reinterpret_cast<void*>(cfg_.sink);
  if (evaluates && !margins_ready_) {  // the margins the first worker row builds on
    margins(z_, stream);
    margins_ready_ = true;
  }
  std::vector<int64_t> scnt(W_), rcnt(W_), soff(W_), roff(W_);
  int64_t done = 0;
  for (; done < rounds; ++done) {
    const int64_t r = r0 + done;
    const int par = (int)(r & 1);
    last_round_bytes_ = 0;
    // ---- deliveries, then the window (BSP: every worker has rows) ----
    int64_t size = 0, start = 0, seen = 0;
    const double wait0 = epoch_ms();
    for (;;) {
      poll(epoch_ms() - cfg_.t0_ms, stream);
      check(api().window_state(reinterpret_cast<void*>(cfg_.window), &size, &start, &seen), "window state");
      if (size > 0) break;
      if (exhausted()) {
        rounds_run_ += done;
        host_ns_ += (double)(steady_ns() - t_begin);
        return done;
      }
      if (epoch_ms() - wait0 > max_wait_s * 1000.0) throw std::runtime_error("KeyRangeLoop: no rows");
      std::this_thread::sleep_for(std::chrono::microseconds(500));
    }
    const int32_t* ids = cfg_.uniq;
    if (W_ > 1) {
      // ---- plan: the window's features, grouped by owner ----
      solver_->plan((int)size, (int)start, stream);
      // ---- pull: counts, ids to the owners, coefficients back ----
      const unsigned* own = solver_->owner_counts_dev();
      {
        hip_check(hipMemcpyAsync(cnt_host_, own, (size_t)W_ * 4, hipMemcpyDeviceToHost, stream), "send counts");
        hip_check(hipMemcpyAsync(cnt_dev_ + rank_, own + rank_, 4, hipMemcpyDeviceToDevice, stream), "self count");
        comm_->group_start();
        for (int j = 0; j < W_; ++j) {
          if (j == rank_) continue;
          comm_->send(own + j, 1, RcclComm::kI32, j, stream);
          comm_->recv(cnt_dev_ + j, 1, RcclComm::kI32, j, stream);
        }
        comm_->group_end();
        hip_check(hipMemcpyAsync(cnt_host_ + W_, cnt_dev_, (size_t)W_ * 4, hipMemcpyDeviceToHost, stream),
                  "recv counts");
        hip_check(hipStreamSynchronize(stream), "pull sizes");
        last_round_bytes_ += (int64_t)(W_ - 1) * 4;
      }
      int64_t so = 0, ro = 0;
      for (int j = 0; j < W_; ++j) {
        scnt[j] = cnt_host_[j];
        rcnt[j] = cnt_host_[W_ + j];
        soff[j] = so;
        roff[j] = ro;
        so += scnt[j];
        ro += rcnt[j];
      }
      if (so > umax_ || ro > (int64_t)W_ * umax_) throw std::runtime_error("KeyRangeLoop: pull sizes out of range");
      exchange(ids, soff.data(), scnt.data(), req_ids_, roff.data(), rcnt.data(), 1, RcclComm::kI32, stream);
      launch_kr_gather(cfg_.shard, lo_, KP_, req_ids_, nullptr, (int)ro, req_vals_, 0, stream);
      hip_check(hipGetLastError(), "keyrange gather");
      exchange(req_vals_, roff.data(), rcnt.data(), w_pull_, soff.data(), scnt.data(), KP_, RcclComm::kF32, stream);
      // ---- the local solve in the window subspace ----
      solver_->finish(stream);
      // ---- push: deltas of the pulled features to their owners; intercepts all-reduced ----
      exchange(cfg_.dloc + KP_, soff.data(), scnt.data(), req_vals_, roff.data(), rcnt.data(), KP_, RcclComm::kF32,
               stream);
      hip_check(hipMemcpyAsync(db_, cfg_.dloc, (size_t)KP_ * 4, hipMemcpyDeviceToDevice, stream), "intercept delta");
      comm_->all_reduce(db_, db_, (size_t)KP_, RcclComm::kF32, stream);
      last_round_bytes_ += (int64_t)KP_ * 4;
      for (int j = 0; j < W_; ++j)  // sender by sender, in rank order
        launch_kr_apply(cfg_.shard, lo_, KP_, req_ids_ + roff[j], nullptr, (int)rcnt[j], req_vals_ + roff[j] * KP_,
                        cfg_.lr, cfg_.b, j == 0 ? db_ : nullptr, 0, stream);
    } else {  // the whole key space is local: solve from the shard in place, apply
      solver_->run((int)size, (int)start, stream);
      launch_kr_apply(cfg_.shard, lo_, KP_, ids, solver_->ucount_dev(), 0, cfg_.dloc + KP_, cfg_.lr, cfg_.b,
                      cfg_.dloc, umax_, stream);
    }
    hip_check(hipGetLastError(), "keyrange update");
    model_bytes_ += last_round_bytes_;
    // ---- rows: worker k's local model (the margins + its window delta), then the
    // global model of round r (the margins + every worker's delta, all-reduced) ----
    if (evaluates) {
      uint64_t seq = 0;
      uintptr_t addr = 0;
      int slot = -1;
      if (cfg_.log_workers) {
        slot = api().sink_acquire(sink, &seq, &addr);
        check(slot, "metrics sink acquire");
      }
      launch_kr_worker_rows(c.K, KP_, cfg_.t_indptr, cfg_.t_idx, cfg_.t_val, cfg_.t_y, cfg_.T, z_, solver_->table(),
                            solver_->table_mask(), cfg_.dloc, cfg_.wloc, dz_, acc_, ticket_,
                            reinterpret_cast<void*>(addr), cfg_.loss, seq, stream);
      hip_check(hipGetLastError(), "worker row");
      if (slot >= 0) api().sink_submit(sink, slot, seq, 0, -1, cfg_.k, r, seen);
      if (W_ > 1) {
        comm_->all_reduce(dz_, dz_, (size_t)cfg_.T * KP_, RcclComm::kF32, stream);
        eval_bytes_ += (int64_t)cfg_.T * KP_ * 4;
      }
      const bool srow = cfg_.log_server && rank_ == 0;
      const bool refresh = (r + 1) % cfg_.margin_refresh == 0;
      seq = 0;
      addr = 0;
      slot = -1;
      if (srow) {
        slot = api().sink_acquire(sink, &seq, &addr);
        check(slot, "metrics sink acquire");
      }
      if (refresh) {  // exact margins from the shards (bounds the drift of the updates)
        margins(z_, stream);
        hip_check(hipMemsetAsync(dz_, 0, (size_t)cfg_.T * KP_ * 4, stream), "zero margin update");
      }
      launch_kr_server_rows(c.K, KP_, cfg_.t_y, cfg_.T, z_, dz_, cfg_.lr, cfg_.b, acc_, ticket_,
                            reinterpret_cast<void*>(addr), seq, stream);
      hip_check(hipGetLastError(), "server row");
      if (slot >= 0) api().sink_submit(sink, slot, seq, 1, -1, -1, r, 0);
    }
    if (cfg_.tracker && rank_ == 0) check(api().tracker_bsp_round(reinterpret_cast<void*>(cfg_.tracker), r), "tracker");
  }
  rounds_run_ += done;
  host_ns_ += (double)(steady_ns() - t_begin);
  return done;
}

}  // namespace psx
