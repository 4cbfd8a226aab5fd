// A finished evaluation record handed to the metrics sink in a batch
// (MetricsSink::submit_many, HostApi::sink_submit_many): kind 0 = worker row,
// 1 = server row, | kSinkTagged: the slot's payload is tagged 16-B chunks
// (chunk 0 = {tag, loss bits, K, 0}, chunk 1 + i = {tag, cells 3i .. 3i + 2} of
// the K x K confusion counts [true][pred], tag = eval_tag(seq)) instead of
// conf[256] / loss / seq; ts < 0: stamped by the sink when the evaluation lands.
#pragma once
#include <cstdint>

namespace psx {

constexpr int kSinkTagged = 2;

struct SinkRecord {
  int slot, kind;
  uint64_t seq;
  int64_t ts, partition, vc, nseen;
};

}  // namespace psx
