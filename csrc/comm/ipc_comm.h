// Same-device multi-process transport (see comm.h): ranks that share ONE GPU
// exchange device buffers through HIP IPC (dma-buf) mappings.
//
// Every rank exports one area: two staging boxes (by collective parity) and a
// flag line {posted seq, consumed seq}.  A collective of sequence number q:
//   post:    wait until every peer consumed q - 2 (the box of this parity is free),
//            copy the contribution into the own box, write posted = q;
//   collect: wait until the needed peers posted q, sum their boxes in rank order
//            (a small kernel reading the IPC mappings) or copy the root's box;
//   finish:  write consumed = q.
// Waits are hipStreamWaitValue64 packets and flags hipStreamWriteValue64, all on
// the caller's stream: like RCCL the host only enqueues, the device orders.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

#include "comm.h"

namespace psx {

class IpcComm : public Comm {
 public:
  // max_bytes: the largest contribution of one collective
  IpcComm(int nranks, int rank, int device, size_t max_bytes);
  ~IpcComm() override;
  IpcComm(const IpcComm&) = delete;
  IpcComm& operator=(const IpcComm&) = delete;
  // the exported area's IPC handle (64 bytes) to hand to every rank
  std::string handle() const;
  // every rank's handle in rank order: map the peers' areas
  void connect(const std::vector<std::string>& handles);
  int rank() const override { return rank_; }
  int size() const override { return nranks_; }
  void all_reduce(const void* send, void* recv, size_t count, int dtype, hipStream_t s) override;
  void reduce(const void* send, void* recv, size_t count, int dtype, int root, hipStream_t s) override;
  void broadcast(const void* send, void* recv, size_t count, int dtype, int root, hipStream_t s) override;
  // unmap the peers (every rank; after the last collective completed)
  void close();
  int64_t collectives() const { return (int64_t)seq_; }

 private:
  static constexpr size_t kFlagBytes = 256;  // posted @ 0, consumed @ 128
  char* box(int r, uint64_t q) const { return base_[r] + kFlagBytes + (q & 1) * max_; }
  uint64_t* posted(int r) const { return reinterpret_cast<uint64_t*>(base_[r]); }
  uint64_t* consumed(int r) const { return reinterpret_cast<uint64_t*>(base_[r] + 128); }
  void live() const;
  void post(const void* src, size_t bytes, uint64_t q, hipStream_t s);
  void wait_posted(int r, uint64_t q, hipStream_t s);
  void finish(uint64_t q, hipStream_t s);
  void sum(void* dst, size_t count, int dtype, uint64_t q, hipStream_t s);

  int nranks_, rank_;
  size_t max_;
  char* own_ = nullptr;
  std::vector<char*> base_;      // every rank's area (own + IPC mappings)
  void* srcs_dev_ = nullptr;     // [2 parities][nranks] box pointers for the sum kernel
  uint64_t seq_ = 0;
  bool connected_ = false;
};

}  // namespace psx
