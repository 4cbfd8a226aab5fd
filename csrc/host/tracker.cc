#include "tracker.h"

#include <algorithm>
#include <climits>
#include <stdexcept>
#include <string>

namespace psx {

VectorClockTracker::VectorClockTracker(int num_workers, int consistency_model)
    : c_(consistency_model), vc_(num_workers, 0), sent_(num_workers, 1), live_(num_workers, 1) {
  if (num_workers <= 0) throw std::invalid_argument("num_workers must be > 0");
  if (consistency_model < -1)
    throw std::invalid_argument("consistency_model must be -1 (eventual), 0 (sequential) or D>0 (bounded delay)");
}

void VectorClockTracker::received(int k, int64_t v) {
  if (k < 0 || k >= num_workers()) throw std::out_of_range("worker id " + std::to_string(k));
  if (!live_[k]) throw std::logic_error("delta from retired worker " + std::to_string(k));
  if (vc_[k] != v)
    throw std::logic_error("worker " + std::to_string(k) + " pushed vc " + std::to_string(v) +
                           " but tracker expected " + std::to_string(vc_[k]));
  vc_[k] += 1;
  sent_[k] = 0;
  max_gap_ = std::max(max_gap_, max_clock() - min_clock());
}

void VectorClockTracker::sent(int k, int64_t v) {
  if (k < 0 || k >= num_workers()) throw std::out_of_range("worker id " + std::to_string(k));
  if (vc_[k] != v)
    throw std::logic_error("dispatching vc " + std::to_string(v) + " to worker " + std::to_string(k) +
                           " whose clock is " + std::to_string(vc_[k]));
  sent_[k] = 1;
}

// Clocks of live workers only: a retired worker no longer holds the others back.
int64_t VectorClockTracker::min_clock() const {
  int64_t m = INT64_MAX;
  for (size_t j = 0; j < vc_.size(); ++j)
    if (live_[j]) m = std::min(m, vc_[j]);
  return m == INT64_MAX ? 0 : m;
}
int64_t VectorClockTracker::max_clock() const {
  int64_t m = INT64_MIN;
  for (size_t j = 0; j < vc_.size(); ++j)
    if (live_[j]) m = std::max(m, vc_[j]);
  return m == INT64_MIN ? 0 : m;
}

std::vector<std::pair<int, int64_t>> VectorClockTracker::retire(int k) {
  if (k < 0 || k >= num_workers()) throw std::out_of_range("worker id " + std::to_string(k));
  std::vector<std::pair<int, int64_t>> out;
  if (!live_[k]) return out;
  live_[k] = 0;
  if (num_live() == 0) return out;
  // the failed worker may have been the slowest: release whoever it held back
  const int64_t lo = min_clock();
  for (int j = 0; j < num_workers(); ++j) {
    if (!live_[j] || sent_[j]) continue;
    if ((c_ == 0 && lo >= vc_[j]) || (c_ > 0 && lo >= vc_[j] - c_)) {
      sent(j, vc_[j]);
      out.emplace_back(j, vc_[j]);
    }
  }
  return out;
}

void VectorClockTracker::revive(int k) {
  if (k < 0 || k >= num_workers()) throw std::out_of_range("worker id " + std::to_string(k));
  live_[k] = 1;
}

int VectorClockTracker::num_live() const {
  int n = 0;
  for (auto l : live_) n += l ? 1 : 0;
  return n;
}

std::vector<std::pair<int, int64_t>> VectorClockTracker::releasable(int k, int64_t v) const {
  std::vector<std::pair<int, int64_t>> out;
  const int n = num_workers();
  if (c_ == -1) {  // eventual: answer the sender only
    out.emplace_back(k, v + 1);
    return out;
  }
  const int64_t lo = min_clock();
  if (c_ == 0) {  // sequential: the whole round completes together
    if (lo >= v + 1)
      for (int j = 0; j < n; ++j)
        if (live_[j]) out.emplace_back(j, v + 1);
    return out;
  }
  // bounded delay: every idle worker that is at most c ahead of the slowest
  for (int j = 0; j < n; ++j)
    if (live_[j] && !sent_[j] && lo >= vc_[j] - c_) out.emplace_back(j, vc_[j]);
  return out;
}

std::vector<std::pair<int, int64_t>> VectorClockTracker::on_delta(int k, int64_t v) {
  received(k, v);
  auto rel = releasable(k, v);
  for (auto& kv : rel) sent(kv.first, kv.second);
  return rel;
}

void VectorClockTracker::bsp_round(int64_t v) {
  for (int k = 0; k < num_workers(); ++k)
    if (live_[k]) received(k, v);
  for (int k = 0; k < num_workers(); ++k)
    if (live_[k]) sent(k, v + 1);
}

void VectorClockTracker::restore(const std::vector<int64_t>& vc, const std::vector<uint8_t>& sent) {
  if (vc.size() != vc_.size() || sent.size() != sent_.size())
    throw std::invalid_argument("tracker restore: worker count mismatch");
  vc_ = vc;
  sent_ = sent;
  max_gap_ = max_clock() - min_clock();
}

}  // namespace psx
