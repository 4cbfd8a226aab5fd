// Host-runtime self-test, built with -fsanitize=address,undefined by
// tests/test_host_sanitizers.py (sanitizer builds of the host
// C++; GPU sanitizers are not available on this pool).  Exercises every host
// component with real threads and shared memory:
//   VectorClockTracker (BSP / SSP / ASP golden cases),
//   SlidingWindow + RateEstimator (cases I/II/III, ring wrap),
//   CtrlQueue (POSIX-shm MPSC: 4 producer threads, 1 consumer),
//   csv_probe / csv_load (header detection, multithreaded parse, bf16),
//   CsvLogger + MetricsSink (producer thread publishing EvalSlots).
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
