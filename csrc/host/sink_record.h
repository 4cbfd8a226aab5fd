// A finished evaluation record handed to the metrics sink in a batch
// (MetricsSink::submit_many, HostApi::sink_submit_many): kind 0 = worker row,
// 1 = server row; ts < 0: stamped by the sink when the evaluation lands.
#pragma once
#include <cstdint>

namespace psx {

struct SinkRecord {
  int slot, kind;
  uint64_t seq;
  int64_t ts, partition, vc, nseen;
};

}  // namespace psx
