#include "sampling.h"

#include <algorithm>
#include <cmath>
#include <stdexcept>

namespace psx {

void RateEstimator::arrival(double now_ms) {
  if (have_last_) {
    double d = now_ms - last_ms_;
    deltas_.push_back(d);
    sum_ += d;
    if (static_cast<int>(deltas_.size()) > window_) {
      sum_ -= deltas_.front();
      deltas_.pop_front();
    }
  }
  have_last_ = true;
  last_ms_ = now_ms;
}

double RateEstimator::mean_interarrival_ms() const {
  if (deltas_.empty()) return 1000.0;
  return sum_ / static_cast<double>(deltas_.size());
}

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
  rate_.arrival(now_ms);
  int64_t target = target_size();
  if (size_ < target)
    size_ += 1;
  else
    size_ = target;
  head_ = (head_ + 1) % cap_;
  seen_ += 1;
  return SlotAssignment{head_, seen_, size_, target};
}

int64_t SlidingWindow::insert_many(const double* now_ms, int64_t n, int64_t* slots_out) {
  int64_t first = -1;
  for (int64_t i = 0; i < n; ++i) {
    SlotAssignment a = insert(now_ms[i]);
    if (i == 0) first = a.slot;
    if (slots_out) slots_out[i] = a.slot;
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
}

}  // namespace psx
