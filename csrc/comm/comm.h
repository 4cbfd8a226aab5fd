// Device-buffer collectives of the parameter-server schedules, by transport.
//
// The reference's bus is three Kafka topics (BaseKafkaApp.java:25-33,
// ServerApp.java:31-42): workers push deltas into one GRADIENTS_TOPIC
// partition, the server publishes weights to WEIGHTS_TOPIC.  In psx the BSP
// round's push / pull are stream-ordered collectives on device buffers:
//   * RcclComm (rccl_comm.h) -- RCCL over xGMI, one process per GPU: production;
//   * IpcComm  (ipc_comm.h)  -- several processes sharing ONE GPU (RCCL refuses
//     two ranks per device): HIP IPC-mapped staging buffers + stream memory
//     operations on flags, so the multi-rank code of the loops can be rehearsed
//     on a one-GPU machine with the same enqueue-only, no-host-sync schedule.
// Every call is enqueued on stream `s` and returns at once; sums are in rank
// order.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>

namespace psx {

class Comm {
 public:
  enum Dtype { kF32 = 0, kI32 = 1, kU8 = 2 };
  virtual ~Comm() = default;
  virtual int rank() const = 0;
  virtual int size() const = 0;
  // sums (float / int32); in-place capable (send == recv)
  virtual void all_reduce(const void* send, void* recv, size_t count, int dtype, hipStream_t s) = 0;
  virtual void reduce(const void* send, void* recv, size_t count, int dtype, int root, hipStream_t s) = 0;
  virtual void broadcast(const void* send, void* recv, size_t count, int dtype, int root, hipStream_t s) = 0;
};

}  // namespace psx
