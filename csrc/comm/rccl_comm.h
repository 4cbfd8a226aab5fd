// Native RCCL communicator for the parameter-server collectives.
//
// The reference moves every gradient push / weight pull through Kafka topics
// (reference: src/main/java/de/hpi/datastreams/apps/WorkerApp.java:60-80,
// ServerApp.java:46-70).  Here the BSP schedules are RCCL collectives over
// xGMI; issuing them through torch.distributed costs ~30 us of host time per
// call (Python + c10d bookkeeping), which at a ~100 us round makes the loop
// host-bound.  This communicator calls RCCL directly (a few us per call) on
// caller-chosen HIP streams with raw device pointers.
//
// The RCCL entry points are resolved at run time from the RCCL library already
// mapped into the process by PyTorch (dlsym), so exactly one RCCL instance is
// used; librccl.so.1 is dlopen'ed only when none is loaded.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

#include "comm.h"

namespace psx {

class RcclComm : public Comm {
 public:
  // 128-byte unique id (rank 0 creates it; every rank passes the same bytes)
  static std::string unique_id();
  static bool available();
  RcclComm(const std::string& id, int nranks, int rank, int device);
  ~RcclComm();
  RcclComm(const RcclComm&) = delete;
  RcclComm& operator=(const RcclComm&) = delete;

  int rank() const override { return rank_; }
  int size() const override { return nranks_; }
  // all collectives sum (float / int32) and are in-place capable
  void all_reduce(const void* send, void* recv, size_t count, int dtype, hipStream_t s) override;
  void reduce(const void* send, void* recv, size_t count, int dtype, int root, hipStream_t s) override;
  void broadcast(const void* send, void* recv, size_t count, int dtype, int root, hipStream_t s) override;
  void reduce_scatter(const void* send, void* recv, size_t recvcount, int dtype, hipStream_t s);
  void all_gather(const void* send, void* recv, size_t sendcount, int dtype, hipStream_t s);
  void send(const void* buf, size_t count, int dtype, int peer, hipStream_t s);
  void recv(void* buf, size_t count, int dtype, int peer, hipStream_t s);
  void group_start();
  void group_end();
  // Overlap: fork() makes the communicator's own side stream wait for the work
  // enqueued so far on `compute`; collectives issued on side_stream() then run
  // beside later compute work; join() makes `compute` wait for them.
  hipStream_t side_stream() const { return side_; }
  void fork(hipStream_t compute);
  void join(hipStream_t compute);
  // collective teardown (every rank); abort() for error paths
  void close();
  void abort();

 private:
  void release_stream();
  void* comm_ = nullptr;
  int nranks_, rank_;
  hipStream_t side_ = nullptr;
  hipEvent_t ev_fork_ = nullptr, ev_join_ = nullptr;
};

}  // namespace psx
