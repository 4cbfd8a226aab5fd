// Peer data plane of the asynchronous consistency models across GPUs.
//
// Reference: the push (WorkerTrainingProcessor.java:95-97: a GradientMessage on
// GRADIENTS_TOPIC) and the selective reply (ServerProcessor.java:172-182: a
// WeightsMessage to the workers the MessageTracker releases) ride the Kafka
// topic bus (BaseKafkaApp.java:25-33).
//
// MI355X: the server rank and every worker rank export one region of
// FINE-GRAINED device memory (coherent for other agents' system-scope accesses)
// through HIP IPC (dma-buf); every other rank maps it.  The kernels then move the
// data themselves over xGMI -- no RCCL kernel beside the persistent launches, no
// host staging, no stream synchronisation:
//   * server region = the inbox: per worker k, [P] delta floats + [FP/32] slice
//     tags; worker k's lane stores its delta slices there and then each slice's
//     tag (vc + 1) (lanes_async.hip peer_push_slice);
//   * worker-rank region = the receive slots: per lane, [P] weights + [FP/32]
//     slice tags; the server kernel stores the weights after an update into every
//     released worker's slot and then the slice tags (the pull count)
//     (server_persist.hip);
//   * the host control plane stays the token queues (ctrl.h): a worker rank's
//     host forwards each lane token to the server's queue; the server's host
//     answers the releases on the worker ranks' reply queues (with the pull tag).
// On one GPU the same code runs between processes on disjoint XCDs (the IPC
// mappings then alias the same HBM), which is how the tests rehearse it.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <string>

namespace psx {

// Layout of a region of `slots` message slots of P floats + NS slice tags.
struct PeerLayout {
  int64_t P = 0;     // floats per message
  int NS = 0;        // slice tags per message (FP / 32)
  int slots = 0;
  int64_t stride() const { return (P + 63) / 64 * 64; }                    // floats between slots
  size_t data_bytes() const { return (size_t)slots * (size_t)stride() * 4; }
  size_t tag_off() const { return (data_bytes() + 255) / 256 * 256; }      // bytes: [slots][NS] u32 tags
  size_t bytes() const { return tag_off() + ((size_t)slots * (size_t)NS * 4 + 255) / 256 * 256; }
};

// One exported region (fine-grained device memory, zeroed).
class PeerRegion {
 public:
  PeerRegion(const PeerLayout& lay, int device);
  ~PeerRegion();
  PeerRegion(const PeerRegion&) = delete;
  PeerRegion& operator=(const PeerRegion&) = delete;
  std::string handle() const;  // 64-byte hipIpcMemHandle_t for the other ranks
  void fill_tags(unsigned value);  // (tools) every slice tag of every slot = value
  uintptr_t base() const { return reinterpret_cast<uintptr_t>(p_); }
  const PeerLayout& layout() const { return lay_; }
  float* data(int slot) const { return reinterpret_cast<float*>(p_) + (size_t)slot * (size_t)lay_.stride(); }
  unsigned* tags(int slot) const {
    return reinterpret_cast<unsigned*>(static_cast<char*>(p_) + lay_.tag_off()) + (size_t)slot * lay_.NS;
  }

 private:
  PeerLayout lay_;
  void* p_ = nullptr;
};

// Another rank's region, mapped into this process.
class PeerMapping {
 public:
  PeerMapping(const std::string& handle, const PeerLayout& lay);
  ~PeerMapping();
  PeerMapping(const PeerMapping&) = delete;
  PeerMapping& operator=(const PeerMapping&) = delete;
  uintptr_t base() const { return reinterpret_cast<uintptr_t>(p_); }
  float* data(int slot) const { return reinterpret_cast<float*>(p_) + (size_t)slot * (size_t)lay_.stride(); }
  unsigned* tags(int slot) const {
    return reinterpret_cast<unsigned*>(static_cast<char*>(p_) + lay_.tag_off()) + (size_t)slot * lay_.NS;
  }
  void close();

 private:
  PeerLayout lay_;
  void* p_ = nullptr;
};

}  // namespace psx
