#include "metrics_sink.h"

#include <sys/prctl.h>

#include <chrono>
#include <cstring>
#include <stdexcept>

namespace psx {

void weighted_f1_accuracy(const int32_t* conf16, int K, double* f1, double* acc) {
  // Spark MulticlassMetrics: weightedFMeasure = sum over labels present in the
  // data of (label count / total) * F1(label); precision/recall are 0 when
  // their denominator is 0 (reference Metrics.java:15-24).
  double total = 0.0, tp_sum = 0.0, wf1 = 0.0;
  double tc[16] = {0}, pc[16] = {0};
  for (int t = 0; t < K; ++t)
    for (int p = 0; p < K; ++p) {
      const double v = conf16[t * 16 + p];
      tc[t] += v;
      pc[p] += v;
      total += v;
    }
  if (total <= 0.0) {
    *f1 = 0.0;
    *acc = 0.0;
    return;
  }
  for (int c = 0; c < K; ++c) {
    const double tp = conf16[c * 16 + c];
    tp_sum += tp;
    const double prec = pc[c] > 0.0 ? tp / pc[c] : 0.0;
    const double rec = tc[c] > 0.0 ? tp / tc[c] : 0.0;
    const double f = prec + rec > 0.0 ? 2.0 * prec * rec / (prec + rec) : 0.0;
    wf1 += tc[c] / total * f;
  }
  *f1 = wf1;
  *acc = tp_sum / total;
}

bool MetricsSink::read_tagged(const EvalSlot& s, uint64_t seq, int32_t* conf16, float* loss) const {
  // chunk i = 4 words at byte 16 i: {tag, payload x 3}; each chunk is one 16-B
  // device store, so a chunk whose tag matches carries its own payload
  const uint32_t tag = (uint32_t)seq | 0x80000000u;  // eval_tag (lanes_kernels.h)
  const volatile uint32_t* w = reinterpret_cast<const volatile uint32_t*>(&s);
  const int K = K_, cells = K * K, nch = 1 + (cells + 2) / 3;
  for (int i = 0; i < nch; ++i)
    if (w[4 * i] != tag) return false;
  __atomic_thread_fence(__ATOMIC_ACQUIRE);
  for (int i = 0; i < 256; ++i) conf16[i] = 0;
  uint32_t lb = w[1];
  std::memcpy(loss, &lb, 4);
  for (int c = 0; c < cells; ++c) conf16[(c / K) * 16 + c % K] = (int32_t)w[4 * (1 + c / 3) + 1 + c % 3];
  // re-check: a chunk rewritten meanwhile would be a protocol error, not a torn read
  for (int i = 0; i < nch; ++i)
    if (w[4 * i] != tag) return false;
  return true;
}

MetricsSink::MetricsSink(uintptr_t slots, int nslots, int K, CsvLogger* wlog, CsvLogger* slog, bool keep_records)
    : slots_(reinterpret_cast<EvalSlot*>(slots)), nslots_(nslots), K_(K), wlog_(wlog), slog_(slog),
      keep_(keep_records) {
  if (!slots_ || nslots_ < 1) throw std::invalid_argument("MetricsSink needs at least one slot");
  if (K_ < 1 || K_ > 16) throw std::invalid_argument("MetricsSink: K must be in [1,16]");
  for (int i = nslots_ - 1; i >= 0; --i) {
    __atomic_store_n(&slots_[i].seq, 0ull, __ATOMIC_RELAXED);
    free_.push_back(i);
  }
  th_ = std::thread([this] { run(); });
}

MetricsSink::~MetricsSink() { close(); }

int MetricsSink::acquire(uint64_t* seq) {
  std::unique_lock<std::mutex> lk(mu_);
  cv_free_.wait(lk, [&] { return !free_.empty() || stop_; });
  if (stop_) throw std::runtime_error("MetricsSink is closed");
  const int s = free_.back();
  free_.pop_back();
  *seq = next_seq_++;
  return s;
}

void MetricsSink::acquire_many(int n, int* slots, uint64_t* seqs) {
  if (n < 0 || n > nslots_) throw std::invalid_argument("MetricsSink: acquire_many beyond the slot pool");
  std::unique_lock<std::mutex> lk(mu_);
  cv_free_.wait(lk, [&] { return (int)free_.size() >= n || stop_; });
  if (stop_) throw std::runtime_error("MetricsSink is closed");
  for (int i = 0; i < n; ++i) {
    slots[i] = free_.back();
    free_.pop_back();
    seqs[i] = next_seq_++;
  }
}

uintptr_t MetricsSink::slot_address(int slot) const {
  if (slot < 0 || slot >= nslots_) throw std::out_of_range("slot");
  return reinterpret_cast<uintptr_t>(&slots_[slot]);
}

void MetricsSink::submit(int slot, uint64_t seq, int kind, int64_t ts, int64_t partition, int64_t vc,
                         int64_t nseen) {
  if (slot < 0 || slot >= nslots_) throw std::out_of_range("slot");
  {
    std::lock_guard<std::mutex> lk(mu_);
    pending_.push_back(Pending{slot, seq, kind, ts, partition, vc, nseen});
    ++submitted_;
  }
  cv_work_.notify_one();
}

void MetricsSink::submit_many(int n, const SinkRecord* recs) {
  for (int i = 0; i < n; ++i)
    if (recs[i].slot < 0 || recs[i].slot >= nslots_) throw std::out_of_range("slot");
  {
    std::lock_guard<std::mutex> lk(mu_);
    for (int i = 0; i < n; ++i) {
      const SinkRecord& r = recs[i];
      pending_.push_back(Pending{r.slot, r.seq, r.kind, r.ts, r.partition, r.vc, r.nseen});
    }
    submitted_ += n;
  }
  if (n > 0) cv_work_.notify_one();
}

void MetricsSink::run() {
  // the waits below are 5 us sleeps: with the default 50 us timer slack a row that
  // lands while this thread sleeps was seen ~60 us late (every run's last rows)
  (void)prctl(PR_SET_TIMERSLACK, 2000UL, 0, 0, 0);
  for (;;) {
    Pending p;
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_work_.wait(lk, [&] { return stop_ || !pending_.empty(); });
      if (pending_.empty()) return;  // stop requested and nothing left
      p = pending_.front();
    }
    // the producer (a kernel or the CPU path) publishes seq after the payload, or
    // (kSinkTagged) tags every 16-B chunk of it with the sequence number
    EvalSlot& s = slots_[p.slot];
    const bool tagged = (p.kind & kSinkTagged) != 0;
    int32_t conf[256];
    float tloss = 0.f;
    int spins = 0;
    while (tagged ? !read_tagged(s, p.seq, conf, &tloss) : __atomic_load_n(&s.seq, __ATOMIC_ACQUIRE) != p.seq) {
      if (++spins < 64) continue;
      std::this_thread::sleep_for(std::chrono::microseconds(spins < 4096 ? 5 : 200));
      std::lock_guard<std::mutex> lk(mu_);
      if (stop_ && spins > 100000) break;  // closing with a producer that never ran: give up
    }
    double ts = (double)p.ts;
    if (p.ts < 0)  // stamped now: the evaluation just completed
      ts = (double)std::chrono::duration_cast<std::chrono::microseconds>(
               std::chrono::system_clock::now().time_since_epoch())
               .count() /
           1000.0;
    double f1 = 0.0, acc = 0.0;
    weighted_f1_accuracy(tagged ? conf : s.conf, K_, &f1, &acc);
    const double loss = tagged ? tloss : s.loss;
    if ((p.kind & 1) == 0) {
      if (wlog_) wlog_->log_worker((int64_t)ts, p.partition, p.vc, loss, f1, acc, p.nseen);
    } else {
      if (slog_) slog_->log_server((int64_t)ts, p.vc, f1, acc);
    }
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (keep_) {
        if ((p.kind & 1) == 0)
          wrows_.push_back(WorkerRow{ts, p.partition, p.vc, loss, f1, acc, p.nseen});
        else
          srows_.push_back(ServerRow{ts, p.vc, f1, acc});
      }
      pending_.pop_front();
      free_.push_back(p.slot);
      processed_.fetch_add(1);
    }
    cv_free_.notify_one();
    cv_done_.notify_all();
  }
}

bool MetricsSink::flush(double timeout_s) {
  std::unique_lock<std::mutex> lk(mu_);
  auto done = [&] { return processed_.load() >= submitted_; };
  if (timeout_s <= 0.0) {
    cv_done_.wait(lk, done);
    return true;
  }
  const auto deadline = std::chrono::system_clock::now() +
                        std::chrono::duration_cast<std::chrono::system_clock::duration>(
                            std::chrono::duration<double>(timeout_s));
  return cv_done_.wait_until(lk, deadline, done);
}

void MetricsSink::close() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (stop_ && !th_.joinable()) return;
    stop_ = true;
  }
  cv_work_.notify_all();
  cv_free_.notify_all();
  if (th_.joinable()) th_.join();
}

std::vector<WorkerRow> MetricsSink::worker_rows() {
  std::lock_guard<std::mutex> lk(mu_);
  return wrows_;
}

std::vector<ServerRow> MetricsSink::server_rows() {
  std::lock_guard<std::mutex> lk(mu_);
  return srows_;
}

}  // namespace psx
