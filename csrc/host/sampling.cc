#include "sampling.h"

#include <algorithm>
#include <cmath>
#include <stdexcept>

namespace psx {

SlidingWindow::SlidingWindow(int64_t min_size, int64_t max_size, double bc, int rate_window, int64_t ring_capacity)
    : min_(min_size), max_(max_size), cap_(ring_capacity > max_size ? ring_capacity : max_size), bc_(bc),
      rate_(rate_window) {
  if (min_size <= 0 || max_size <= 0 || min_size > max_size)
    throw std::invalid_argument("need 0 < min_buffer_size <= max_buffer_size");
  if (!(bc > 0.0)) throw std::invalid_argument("buffer_size_coefficient must be > 0");
}

int64_t SlidingWindow::target_size() const {
  double mean = rate_.mean_interarrival_ms();
  // events per minute.  Deliberate deviation: a zero mean inter-arrival time (a
  // burst; every row of a per-iteration poll shares one timestamp) means "as fast
  // as possible" -> the max window.  The reference computes (int) Math.round(
  // bc * 60000 / 0.0) = (int) Long.MAX_VALUE = -1 there and so clamps to the MIN
  // window (WorkerSamplingProcessor.java:115-122) -- an overflow artefact, not a
  // policy.  Pinned by tests/test_sampling.py::test_zero_mean_interarrival_policy.
  double per_min = mean > 0.0 ? 60000.0 / mean : static_cast<double>(max_) / bc_ + 1.0;
  double t = std::floor(bc_ * per_min + 0.5);  // java.lang.Math.round
  if (!(t == t)) t = static_cast<double>(max_);
  int64_t ti = t > static_cast<double>(max_) ? max_ : static_cast<int64_t>(t);
  return std::min(max_, std::max(min_, ti));
}

SlotAssignment SlidingWindow::insert(double now_ms) {
  // A zero inter-arrival time cannot raise the mean (the estimator gains a 0 and
  // at most loses a non-negative delta), so a target already at max stays there:
  // the rows of one delivery (equal stamps) skip the two fp64 divisions of
  // target_size() -- 1,024 of them per lane and round in the lanes loop.
  const bool zero_dt = rate_.has_last() && now_ms == rate_.last_ms();
  rate_.arrival(now_ms);
  const int64_t target = (zero_dt && last_target_ == max_) ? max_ : target_size();
  last_target_ = target;
  if (size_ < target)
    size_ += 1;
  else
    size_ = target;
  head_ = head_ + 1 == cap_ ? 0 : head_ + 1;  // (no 64-bit modulo on the per-row path)
  seen_ += 1;
  return SlotAssignment{head_, seen_, size_, target};
}

int64_t SlidingWindow::insert_many(const double* now_ms, int64_t n, int64_t* slots_out) {
  int64_t first = -1;
  for (int64_t i = 0; i < n;) {
    if (!slots_out && i > 0 && last_target_ == max_ && now_ms[i] == now_ms[i - 1]) {
      // a run of equal stamps with the target at max (see insert()): k rows at
      // once -- k zero deltas into the estimator, the size grows by one per row
      int64_t j = i + 1;
      while (j < n && now_ms[j] == now_ms[i]) ++j;
      const int64_t k = j - i;
      rate_.zeros(k);
      size_ = size_ + k < max_ ? size_ + k : max_;
      head_ = (head_ + k) % cap_;
      seen_ += k;
      i = j;
      continue;
    }
    SlotAssignment a = insert(now_ms[i]);
    if (i == 0) first = a.slot;
    if (slots_out) slots_out[i] = a.slot;
    ++i;
  }
  return first;
}

int64_t SlidingWindow::start() const {
  if (size_ == 0) return 0;
  return ((head_ - size_ + 1) % cap_ + cap_) % cap_;
}

void SlidingWindow::restore(int64_t head, int64_t size, int64_t seen) {
  if (size < 0 || size > max_ || head < -1 || head >= cap_) throw std::invalid_argument("bad window state");
  head_ = head;
  size_ = size;
  seen_ = seen;
  last_target_ = -1;
}

}  // namespace psx
