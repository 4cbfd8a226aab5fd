// C ABI table of the host runtime (see capi.h).
#include "capi.h"

#include <exception>
#include <string>

#include "dataset.h"
#include "metrics_sink.h"
#include "sampling.h"
#include "tracker.h"

namespace psx {
namespace {

thread_local std::string g_err;

template <class F>
int guarded(F&& f, int on_error) {
  try {
    g_err.clear();
    return f();
  } catch (const std::exception& e) {
    g_err = e.what();
  } catch (...) {
    g_err = "unknown exception";
  }
  return on_error;
}

int copy_out(const std::vector<std::pair<int, int64_t>>& rel, int* ks, int64_t* vs, int cap) {
  if ((int)rel.size() > cap) throw std::length_error("release list larger than the caller's buffer");
  for (size_t i = 0; i < rel.size(); ++i) {
    ks[i] = rel[i].first;
    vs[i] = rel[i].second;
  }
  return (int)rel.size();
}

int c_on_delta(void* t, int k, int64_t v, int* ks, int64_t* vs, int cap) {
  return guarded([&] { return copy_out(static_cast<VectorClockTracker*>(t)->on_delta(k, v), ks, vs, cap); }, -1);
}
int c_retire(void* t, int k, int* ks, int64_t* vs, int cap) {
  return guarded([&] { return copy_out(static_cast<VectorClockTracker*>(t)->retire(k), ks, vs, cap); }, -1);
}
int c_is_live(void* t, int k) {
  return guarded([&] { return static_cast<VectorClockTracker*>(t)->is_live(k) ? 1 : 0; }, -1);
}
int c_revive(void* t, int k) {
  return guarded(
      [&] {
        static_cast<VectorClockTracker*>(t)->revive(k);
        return 0;
      },
      -1);
}
int64_t c_clock(void* t, int k) {
  try {
    g_err.clear();
    return static_cast<VectorClockTracker*>(t)->clock(k);
  } catch (const std::exception& e) {
    g_err = e.what();
  }
  return -1;
}
void c_sent(void* t, int k, int64_t v) {
  guarded(
      [&] {
        static_cast<VectorClockTracker*>(t)->sent(k, v);
        return 0;
      },
      -1);
}
int c_pop(void* q, CtrlToken* out, double timeout_s) {
  return guarded([&] { return static_cast<CtrlQueue*>(q)->pop(out, timeout_s) ? 1 : 0; }, -1);
}
int c_push(void* q, const CtrlToken* t, double timeout_s) {
  return guarded([&] { return static_cast<CtrlQueue*>(q)->push(*t, timeout_s) ? 1 : 0; }, -1);
}
int c_acquire(void* s, uint64_t* seq, uintptr_t* addr) {
  return guarded(
      [&] {
        auto* sink = static_cast<MetricsSink*>(s);
        const int slot = sink->acquire(seq);
        *addr = sink->slot_address(slot);
        return slot;
      },
      -1);
}
void c_submit(void* s, int slot, uint64_t seq, int kind, int64_t ts, int64_t partition, int64_t vc, int64_t nseen) {
  guarded(
      [&] {
        static_cast<MetricsSink*>(s)->submit(slot, seq, kind, ts, partition, vc, nseen);
        return 0;
      },
      -1);
}
const char* c_last_error() { return g_err.c_str(); }

int64_t c_window_insert_many(void* w, const double* t, int64_t n) {
  try {
    g_err.clear();
    return static_cast<SlidingWindow*>(w)->insert_many(t, n, nullptr);
  } catch (const std::exception& e) {
    g_err = e.what();
  }
  return -1;
}
int c_window_state(void* w, int64_t* size, int64_t* start, int64_t* seen) {
  return guarded(
      [&] {
        auto* win = static_cast<SlidingWindow*>(w);
        *size = win->size();
        *start = win->size() > 0 ? win->start() : 0;
        *seen = win->tuples_seen();
        return 0;
      },
      -1);
}
int64_t c_due_rows(int k, int n, double p_ms, int64_t total, int64_t next_local, double now_ms, int64_t max_rows,
                   double* times) {
  try {
    g_err.clear();
    return due_rows(k, n, p_ms, total, next_local, now_ms, max_rows, times);
  } catch (const std::exception& e) {
    g_err = e.what();
  }
  return -1;
}
int c_bsp_round(void* t, int64_t v) {
  return guarded(
      [&] {
        static_cast<VectorClockTracker*>(t)->bsp_round(v);
        return 0;
      },
      -1);
}

int c_acquire_many(void* s, int n, int* slots, uint64_t* seqs, uintptr_t* addrs) {
  return guarded(
      [&] {
        auto* sink = static_cast<MetricsSink*>(s);
        sink->acquire_many(n, slots, seqs);
        for (int i = 0; i < n; ++i) addrs[i] = sink->slot_address(slots[i]);
        return 0;
      },
      -1);
}
int c_submit_many(void* s, int n, const SinkRecord* recs) {
  return guarded(
      [&] {
        static_cast<MetricsSink*>(s)->submit_many(n, recs);
        return 0;
      },
      -1);
}

int c_is_sent(void* t, int k) {
  return guarded([&] { return static_cast<VectorClockTracker*>(t)->is_sent(k) ? 1 : 0; }, -1);
}

const HostApi kApi{kHostApiVersion, c_on_delta,   c_retire,         c_is_live,       c_revive,
                   c_clock,         c_sent,       c_pop,            c_push,          c_acquire,
                   c_submit,        c_last_error, c_window_insert_many, c_window_state, c_due_rows,
                   c_bsp_round,     c_acquire_many, c_submit_many, c_is_sent};

}  // namespace

const HostApi* host_api() { return &kApi; }

}  // namespace psx
