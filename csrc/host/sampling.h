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
#include <vector>

namespace psx {

// The last `window` inter-arrival times in a fixed ring (no allocation per
// arrival: a window of 1,024 new rows per round is 1,024 arrivals, on the round
// loop's critical host path for every lane).  The running sum is updated in the
// same order as a FIFO would (+ newest, then - evicted), so the estimate is the
// same to the last bit.
class RateEstimator {
 public:
  explicit RateEstimator(int window = 500) : window_(window > 0 ? window : 0), buf_(window_ + 1, 0.0) {}
  // Record an arrival at wall-clock `now_ms`.
  void arrival(double now_ms) {
    if (have_last_) {
      const double d = now_ms - last_ms_;
      buf_[tail_] = d;
      tail_ = tail_ + 1 == (int)buf_.size() ? 0 : tail_ + 1;
      sum_ += d;
      if (++n_ > window_) {
        sum_ -= buf_[head_];
        head_ = head_ + 1 == (int)buf_.size() ? 0 : head_ + 1;
        --n_;
      }
    }
    have_last_ = true;
    last_ms_ = now_ms;
  }
  // k arrivals at the last stamp (k zero deltas): the same state as k arrival()
  // calls -- adding 0.0 leaves the sum unchanged (it is never -0.0), the evictions of
  // the entries present before the call are subtracted in order (an entry is evicted
  // before its slot is rewritten: the buffer holds window + 1), and the evictions of
  // this call's own zeros change nothing.  O(window), not O(k): a round's 1,024-row
  // delivery to 8 workers cost ~42 us of the host loop one zero at a time.
  void zeros(int64_t k) {
    if (!have_last_) {  // the first of them only sets the stamp
      if (k <= 0) return;
      have_last_ = true;
      --k;
    }
    if (k <= 0) return;
    const int64_t B = (int64_t)buf_.size();
    const int64_t e = n_ + k > window_ ? n_ + k - window_ : 0;  // evictions
    const int64_t eo = e < n_ ? e : n_;                          // ... of entries present before
    int h = head_;
    for (int64_t i = 0; i < eo; ++i) {
      const double v = buf_[h];
      if (v != 0.0) sum_ -= v;  // (x - 0.0 == x: only the nonzero deltas form the chain)
      h = h + 1 == (int)B ? 0 : h + 1;
    }
    const int64_t kw = k < B ? k : B;  // the slots this call's zeros end in
    int64_t t = (tail_ + (k - kw)) % B;
    for (int64_t i = 0; i < kw; ++i) {
      buf_[t] = 0.0;
      t = t + 1 == B ? 0 : t + 1;
    }
    tail_ = (int)((tail_ + k) % B);
    head_ = (int)((head_ + e) % B);
    n_ = (int)(n_ + k - e);
  }
  // Mean inter-arrival time in ms (1000 when fewer than two arrivals).
  double mean_interarrival_ms() const { return n_ == 0 ? 1000.0 : sum_ / static_cast<double>(n_); }
  int samples() const { return n_; }
  bool has_last() const { return have_last_; }
  double last_ms() const { return last_ms_; }

 private:
  int window_;
  bool have_last_ = false;
  double last_ms_ = 0.0;
  double sum_ = 0.0;
  std::vector<double> buf_;  // ring of window_ + 1 slots: [head_, tail_) holds n_ deltas
  int head_ = 0, tail_ = 0, n_ = 0;
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
  int64_t last_target_ = -1;  // target of the previous insert (-1: none)
};

}  // namespace psx
