// Adaptive sliding-window buffer bookkeeping (host side).
//
// The reference keeps, per logical worker, a Kafka key-value store slice of
// `max` slots and scans it on every tuple (reference:
// src/main/java/de/hpi/datastreams/processors/WorkerSamplingProcessor.java:50-135).
// Its observable semantics are:
//   * a window of the <=500 most recent inter-arrival times gives the mean Δt;
//     with no samples the mean defaults to 1000 ms;
//   * target = clamp(round(bc * 60000 / mean_ms), min, max);
//   * the buffer always holds the s most recent tuples, with
//       s <- min(s + 1, target)  if s < target   (case I: fill an empty slot)
//       s <- target              otherwise       (cases II/III: overwrite / shrink)
// Here that becomes O(1) ring arithmetic: the device ring has capacity >= `max`,
// the newest tuple lands at `head`, and the trainable window is the `size`
// slots ending at head.  No per-tuple scan.
#pragma once
#include <cstdint>
#include <deque>

namespace psx {

class RateEstimator {
 public:
  explicit RateEstimator(int window = 500) : window_(window) {}
  // Record an arrival at wall-clock `now_ms`.
  void arrival(double now_ms);
  // Mean inter-arrival time in ms (1000 when fewer than two arrivals).
  double mean_interarrival_ms() const;
  int samples() const { return static_cast<int>(deltas_.size()); }

 private:
  int window_;
  bool have_last_ = false;
  double last_ms_ = 0.0;
  double sum_ = 0.0;
  std::deque<double> deltas_;
};

// Result of ingesting one tuple.
struct SlotAssignment {
  int64_t slot;          // ring slot the tuple must be written to
  int64_t insertion_id;  // 1-based id of the tuple (== number of tuples seen)
  int64_t size;          // window size after the insert
  int64_t target;        // target size used for this insert
};

class SlidingWindow {
 public:
  // ring_capacity (>= max_size; 0 = max_size): modulus of the slot ring, which
  // the device side rounds up to whole 32-row tiles.
  SlidingWindow(int64_t min_size, int64_t max_size, double buffer_coefficient, int rate_window = 500,
                int64_t ring_capacity = 0);

  // Target size for the current arrival rate.
  int64_t target_size() const;
  // Register a tuple arriving at `now_ms`; returns where it goes.
  SlotAssignment insert(double now_ms);
  // Bulk form used by the streaming path: `n` tuples with arrival stamps.
  // Returns the slot of the first tuple; slots are consecutive modulo capacity.
  int64_t insert_many(const double* now_ms, int64_t n, int64_t* slots_out);

  int64_t size() const { return size_; }
  int64_t capacity() const { return cap_; }  // ring modulus
  int64_t max_size() const { return max_; }
  int64_t head() const { return head_; }  // slot of the newest tuple (-1 when empty)
  // First slot of the window: the window is [start, start+size) modulo capacity.
  int64_t start() const;
  int64_t tuples_seen() const { return seen_; }
  double mean_interarrival_ms() const { return rate_.mean_interarrival_ms(); }

  void restore(int64_t head, int64_t size, int64_t seen);

 private:
  int64_t min_, max_, cap_;
  double bc_;
  RateEstimator rate_;
  int64_t head_ = -1;
  int64_t size_ = 0;
  int64_t seen_ = 0;
};

}  // namespace psx
