// Host-runtime self-test, built with -fsanitize=address,undefined by
// tests/test_host_sanitizers.py (sanitizer builds of the host
// C++; GPU sanitizers are not available on this pool).  Exercises every host
// component with real threads and shared memory:
//   VectorClockTracker (BSP / SSP / ASP golden cases),
//   SlidingWindow + RateEstimator (cases I/II/III, ring wrap),
//   CtrlQueue (POSIX-shm MPSC: 4 producer threads, 1 consumer),
//   csv_probe / csv_load (header detection, multithreaded parse, bf16),
//   CsvLogger + MetricsSink (producer thread publishing EvalSlots),
//   tracker fault handling (retire / bsp_round),
//   libsvm_save / libsvm_load round trip (multithreaded mmap parser).
// Exit status 0 = all checks passed.
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <unistd.h>
#include <vector>

#include "../host/ctrl.h"
#include "../host/dataset.h"
#include "../host/libsvm.h"
#include "../host/logger.h"
#include "../host/metrics_sink.h"
#include "../host/sampling.h"
#include "../host/tracker.h"

using namespace psx;

static int g_fail = 0;
#define CHECK(cond)                                                   \
  do {                                                                \
    if (!(cond)) {                                                    \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #cond); \
      ++g_fail;                                                       \
    }                                                                 \
  } while (0)

static void test_tracker() {
  // BSP: nobody is released until every worker's delta for round v arrived.
  VectorClockTracker bsp(3, 0);
  CHECK(bsp.on_delta(0, 0).empty());
  CHECK(bsp.on_delta(1, 0).empty());
  auto rel = bsp.on_delta(2, 0);
  CHECK(rel.size() == 3);
  for (auto& p : rel) CHECK(p.second == 1);
  // ASP: the sender alone is answered, immediately.
  VectorClockTracker asp(2, -1);
  auto r1 = asp.on_delta(1, 0);
  CHECK(r1.size() == 1 && r1[0].first == 1 && r1[0].second == 1);
  // SSP(1): a worker may run ahead of the slowest by the bound only.
  VectorClockTracker ssp(2, 1);
  int64_t v0 = 0;
  int released = 0;
  for (int it = 0; it < 6; ++it) {
    auto r = ssp.on_delta(0, v0);
    released += (int)r.size();
    bool again = false;
    for (auto& p : r)
      if (p.first == 0) again = true, v0 = p.second;
    if (!again) break;
  }
  CHECK(ssp.max_gap() <= 2);
  CHECK(released >= 1);
  // invariant violations are hard errors
  bool threw = false;
  try {
    VectorClockTracker t(2, 0);
    t.received(0, 5);
  } catch (const std::exception&) {
    threw = true;
  }
  CHECK(threw);
}

static void test_tracker_faults() {
  // BSP with 3 workers: 0 and 1 wait for worker 2, which then fails; retiring
  // it releases the two waiting workers with the next version.
  VectorClockTracker bsp(3, 0);
  CHECK(bsp.on_delta(0, 0).empty());
  CHECK(bsp.on_delta(1, 0).empty());
  auto rel = bsp.retire(2);
  CHECK(rel.size() == 2);
  for (auto& p : rel) CHECK(p.first != 2 && p.second == 1);
  CHECK(!bsp.is_live(2) && bsp.num_live() == 2);
  CHECK(bsp.min_clock() == 1);  // the dead worker's clock no longer counts
  // later rounds involve the live workers only
  CHECK(bsp.on_delta(0, 1).empty());
  CHECK(bsp.on_delta(1, 1).size() == 2);
  // SSP(0 slack = 1): a retired straggler stops holding the fast worker back
  VectorClockTracker ssp(2, 1);
  auto r = ssp.on_delta(0, 0);
  CHECK(r.size() == 1 && r[0].second == 1);
  CHECK(ssp.on_delta(0, 1).empty());  // 2 ahead of worker 1 -> held
  auto r2 = ssp.retire(1);
  CHECK(r2.size() == 1 && r2[0].first == 0 && r2[0].second == 2);
  // whole BSP rounds in one call (the collective schedules)
  VectorClockTracker b2(4, 0);
  for (int64_t v = 0; v < 5; ++v) b2.bsp_round(v);
  for (int k = 0; k < 4; ++k) CHECK(b2.clock(k) == 5 && b2.is_sent(k));
  CHECK(b2.max_gap() <= 1);  // same as applying the deltas one by one
}

static void test_libsvm() {
  char path[] = "/tmp/psx_selftest_svm_XXXXXX";
  int fd = mkstemp(path);
  CHECK(fd >= 0);
  close(fd);
  const int64_t rows = 5000;
  std::vector<int64_t> indptr(1, 0);
  std::vector<int32_t> idx;
  std::vector<uint16_t> val;
  std::vector<int32_t> y(rows);
  for (int64_t r = 0; r < rows; ++r) {
    const int n = (int)(r % 7);
    for (int j = 0; j < n; ++j) {
      idx.push_back((int32_t)((r * 131 + j * 977) % 100000 + j));
      val.push_back(f32_to_bf16(0.25f * (float)(j + 1) * ((r & 1) ? -1.f : 1.f)));
    }
    indptr.push_back((int64_t)idx.size());
    y[r] = (int32_t)(r % 5 + 1);
  }
  for (int zb = 0; zb < 2; ++zb) {
    libsvm_save(path, indptr.data(), idx.data(), val.data(), y.data(), rows, zb != 0);
    SparseRows s = libsvm_load(path, zb != 0, 4);
    CHECK((int64_t)s.y.size() == rows && s.indptr == indptr && s.idx == idx && s.val == val && s.y == y);
    int32_t mx = -1;
    for (auto i : idx) mx = i > mx ? i : mx;
    CHECK(s.max_feature == mx);
  }
  unlink(path);
}

static void test_window() {
  SlidingWindow w(2, 8, 100.0, 500, 16);
  std::vector<double> t(40);
  for (int i = 0; i < 40; ++i) t[i] = i;  // 1 ms apart -> target clamps to max
  std::vector<int64_t> slots(40);
  w.insert_many(t.data(), 40, slots.data());
  CHECK(w.size() == 8);
  CHECK(w.head() == 39 % 16);
  CHECK(w.start() == ((39 - 8 + 1) % 16));
  for (int i = 1; i < 40; ++i) CHECK(slots[i] == (slots[i - 1] + 1) % 16);
  CHECK(w.tuples_seen() == 40);
  // slow arrivals shrink the target (case III) down to min
  SlidingWindow s(2, 8, 0.3, 500);
  for (int i = 0; i < 20; ++i) s.insert(i * 60000.0);
  CHECK(s.size() == 2);
  RateEstimator r(4);
  CHECK(std::fabs(r.mean_interarrival_ms() - 1000.0) < 1e-12);
  for (int i = 0; i < 10; ++i) r.arrival(i * 10.0);
  CHECK(std::fabs(r.mean_interarrival_ms() - 10.0) < 1e-12);
}

static void test_ctrl_queue() {
  const std::string name = "/psx_selftest_" + std::to_string(getpid());
  CtrlQueue q(name, 64, true);
  constexpr int kProducers = 4, kPer = 500;
  std::vector<std::thread> th;
  for (int p = 0; p < kProducers; ++p)
    th.emplace_back([&, p] {
      CtrlQueue qp(name, 64, false);
      for (int i = 0; i < kPer; ++i) {
        CtrlToken t{p, 0, i, 0, 0};
        if (!qp.push(t, 10.0)) std::abort();
      }
    });
  std::vector<int64_t> last(kProducers, -1);
  int got = 0;
  while (got < kProducers * kPer) {
    CtrlToken t;
    if (!q.pop(&t, 10.0)) break;
    CHECK(t.worker >= 0 && t.worker < kProducers);
    CHECK(t.vc == last[t.worker] + 1);  // per-producer FIFO
    last[t.worker] = t.vc;
    ++got;
  }
  for (auto& x : th) x.join();
  CHECK(got == kProducers * kPer);
  q.unlink();
}

static void test_csv() {
  char path[] = "/tmp/psx_selftest_XXXXXX";
  int fd = mkstemp(path);
  CHECK(fd >= 0);
  std::string body = "a,b,c,Score\n";
  for (int r = 0; r < 1000; ++r) body += std::to_string(r * 0.5) + ",0," + std::to_string(-r) + "," +
                                         std::to_string(r % 5 + 1) + "\n";
  CHECK(write(fd, body.data(), body.size()) == (ssize_t)body.size());
  close(fd);
  CsvInfo info = csv_probe(path, 0);
  CHECK(info.header && info.rows == 1000 && info.cols == 4);
  const int64_t stride = 8;
  std::vector<float> xf(info.rows * stride, -7.f);
  std::vector<uint16_t> xb(info.rows * stride);
  std::vector<int32_t> y(info.rows);
  csv_load(path, info, -1, stride, xf.data(), xb.data(), y.data(), 4);
  for (int r = 0; r < 1000; ++r) {
    CHECK(xf[r * stride + 0] == (float)(r * 0.5));
    CHECK(xf[r * stride + 2] == (float)(-r));
    CHECK(xf[r * stride + 3] == 0.f);  // padding zeroed
    CHECK(y[r] == r % 5 + 1);
    CHECK(xb[r * stride + 0] == f32_to_bf16(xf[r * stride + 0]));
  }
  unlink(path);
}

static void test_metrics_sink() {
  char path[] = "/tmp/psx_selftest_log_XXXXXX";
  int fd = mkstemp(path);
  close(fd);
  CsvLogger wlog(path, true, true);
  constexpr int kSlots = 3, kRecs = 200;
  std::vector<EvalSlot> slots(kSlots);
  std::memset(slots.data(), 0, sizeof(EvalSlot) * kSlots);
  MetricsSink sink(reinterpret_cast<uintptr_t>(slots.data()), kSlots, 2, &wlog, nullptr, true);
  // the "device": fills slots asynchronously, publishing seq last
  std::atomic<int> produced{0};
  for (int i = 0; i < kRecs; ++i) {
    uint64_t seq = 0;
    const int s = sink.acquire(&seq);
    std::thread([&, s, seq, i] {
      EvalSlot& e = slots[s];
      std::memset(e.conf, 0, sizeof(e.conf));
      e.conf[0] = 3 + (i % 2);  // true 0 -> pred 0
      e.conf[1] = 1;            // true 0 -> pred 1
      e.conf[17] = 4;           // true 1 -> pred 1
      e.loss = 0.5f;
      __atomic_store_n(&e.seq, seq, __ATOMIC_RELEASE);
      produced.fetch_add(1);
    }).detach();
    sink.submit(s, seq, 0, 1000 + i, 0, i, 10 * i);
  }
  CHECK(sink.flush(30.0));
  auto rows = sink.worker_rows();
  CHECK((int)rows.size() == kRecs);
  for (int i = 0; i < kRecs && i < (int)rows.size(); ++i) {
    const double tp0 = 3 + (i % 2), tot = tp0 + 5;
    CHECK(rows[i].vc == i);
    CHECK(std::fabs(rows[i].acc - (tp0 + 4) / tot) < 1e-12);
  }
  while (produced.load() < kRecs) std::this_thread::yield();
  sink.close();
  wlog.close();
  FILE* f = std::fopen(path, "r");
  int lines = 0;
  char buf[512];
  while (f && std::fgets(buf, sizeof buf, f)) ++lines;
  if (f) std::fclose(f);
  CHECK(lines == kRecs + 1);
  unlink(path);
}

int main() {
  test_tracker();
  test_tracker_faults();
  test_libsvm();
  test_window();
  test_ctrl_queue();
  test_csv();
  test_metrics_sink();
  if (g_fail) {
    std::fprintf(stderr, "%d check(s) failed\n", g_fail);
    return 1;
  }
  std::printf("host selftest: all checks passed\n");
  return 0;
}
