// Host control plane for the asynchronous consistency models.
//
// In the reference every gradient travels through GRADIENTS_TOPIC, a single
// Kafka partition that serialises the server (reference:
// src/main/java/de/hpi/datastreams/apps/ServerApp.java:36-38,
// WorkerTrainingProcessor.java:95-97).  RCCL has no "receive from any rank",
// so the MI355X design splits that topic in two:
//   * data plane: the delta itself moves GPU->GPU with ncclSend/ncclRecv;
//   * control plane (this file): a (worker, vector clock) token tells the
//     server which ncclRecv to post next.  Tokens live in a bounded lock-free
//     MPSC ring in POSIX shared memory, so a push/pop is a few atomics (~100 ns)
//     instead of a broker round trip.
// The ring is a Vyukov bounded queue: each slot carries a sequence number, so
// producers never overwrite unread tokens and the consumer never reads torn ones.
#pragma once
#include <atomic>
#include <cstdint>
#include <string>

namespace psx {

struct CtrlToken {
  int32_t worker;
  int32_t kind;  // 0 = delta pushed, 1 = worker finished, 2 = worker error
  int64_t vc;
  int64_t aux;   // free field (e.g. tuples seen)
  int64_t ts_us; // producer timestamp (for tracing)
  int64_t n;     // payload size (sparse push: number of touched features)
};

class CtrlQueue {
 public:
  // create=true: the server creates (and later unlinks) the segment.
  CtrlQueue(const std::string& name, uint32_t capacity, bool create);
  ~CtrlQueue();
  CtrlQueue(const CtrlQueue&) = delete;
  CtrlQueue& operator=(const CtrlQueue&) = delete;

  // Non-blocking; false when the ring is full.
  bool try_push(const CtrlToken& t);
  // Spins (then sleeps) until pushed or timeout; false on timeout.
  bool push(const CtrlToken& t, double timeout_s);
  bool try_pop(CtrlToken* out);
  // Blocks until a token arrives or timeout_s elapses; false on timeout.
  bool pop(CtrlToken* out, double timeout_s);
  uint32_t capacity() const;
  const std::string& name() const { return name_; }
  void unlink();
  // (diagnostics) tokens pushed / popped so far and the segment's inode
  uint64_t enqueued() const { return hdr_->enq.load(std::memory_order_relaxed); }
  uint64_t dequeued() const { return hdr_->deq.load(std::memory_order_relaxed); }
  uint64_t inode() const { return ino_; }

 private:
  struct Slot {
    std::atomic<uint64_t> seq;
    CtrlToken tok;
  };
  struct alignas(64) Header {
    uint64_t magic;
    uint32_t capacity;
    uint32_t pad0;
    alignas(64) std::atomic<uint64_t> enq;
    alignas(64) std::atomic<uint64_t> deq;
  };
  std::string name_;
  bool owner_;
  size_t bytes_ = 0;
  uint64_t ino_ = 0;
  void* base_ = nullptr;
  Header* hdr_ = nullptr;
  Slot* slots_ = nullptr;
};

}  // namespace psx
