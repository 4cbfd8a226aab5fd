// Vector-clock tracker for the parameter server's consistency models.
//
// Semantics follow the reference's MessageTracker/ServerProcessor pair
// (reference: src/main/java/de/hpi/datastreams/processors/MessageTracker.java:10-88,
//  ServerProcessor.java:95-134), re-expressed as a flat struct-of-arrays that the
// server scheduler thread queries once per arriving delta:
//   * per worker k: vc[k] = number of deltas received, sent[k] = weights for vc[k]
//     already dispatched (i.e. the worker is busy).
//   * init vc = 0, sent = true (the bootstrap broadcast is not tracked).
//   * c == 0  : sequential / BSP        -> release everybody once min(vc) >= v+1
//   * c  > 0  : bounded delay / SSP(c)  -> release every idle k with min(vc) >= vc[k]-c
//   * c == -1 : eventual / ASP          -> release only the sender
//   * c <= -2 : rejected at construction (reference quirk Q4 stalls forever).
// Protocol violations (unexpected vector clocks) raise std::logic_error, which is
// the hard-error analogue of the reference's IllegalArgumentException.
#pragma once
#include <cstdint>
#include <utility>
#include <vector>

namespace psx {

class VectorClockTracker {
 public:
  VectorClockTracker(int num_workers, int consistency_model);

  // A delta from worker `k` computed against weights version `v` has arrived.
  void received(int k, int64_t v);
  // Weights version `v` has been dispatched to worker `k`.
  void sent(int k, int64_t v);

  // Which (worker, version) pairs must receive the current weights after the
  // delta (k, v) has been applied.  Does not mutate; call sent() per pair.
  std::vector<std::pair<int, int64_t>> releasable(int k, int64_t v) const;

  // A whole BSP round in one call: every live worker's delta of version v has
  // been applied and every live worker receives version v + 1.
  void bsp_round(int64_t v);

  // received() + releasable() + sent() for every released pair.
  std::vector<std::pair<int, int64_t>> on_delta(int k, int64_t v);

  // Fault tolerance: drop a failed worker.  Its clock stops counting towards
  // min/max, and workers it was holding back under BSP/SSP are released
  // (returned, already marked sent).
  std::vector<std::pair<int, int64_t>> retire(int k);
  // A worker retired because it FINISHED a run rejoins the next run at its clock
  // (failed workers stay retired).
  void revive(int k);
  bool is_live(int k) const { return live_.at(k) != 0; }
  int num_live() const;

  int64_t min_clock() const;
  int64_t max_clock() const;
  int64_t clock(int k) const { return vc_.at(k); }
  bool is_sent(int k) const { return sent_.at(k) != 0; }
  int num_workers() const { return static_cast<int>(vc_.size()); }
  int consistency_model() const { return c_; }
  // Largest (max vc - min vc) observed so far: the staleness actually realised.
  int64_t max_gap() const { return max_gap_; }

  // Checkpoint support.
  std::vector<int64_t> clocks() const { return vc_; }
  std::vector<uint8_t> sent_flags() const { return sent_; }
  void restore(const std::vector<int64_t>& vc, const std::vector<uint8_t>& sent);

 private:
  int c_;
  std::vector<int64_t> vc_;
  std::vector<uint8_t> sent_;
  std::vector<uint8_t> live_;
  int64_t max_gap_ = 0;
};

}  // namespace psx
