#include "ctrl.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <cstring>
#include <stdexcept>
#include <thread>

namespace psx {

namespace {
constexpr uint64_t kMagic = 0x5053584354524c31ull;  // "PSXCTRL1"

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

inline void backoff(int& spins) {
  if (spins < 256) {
    ++spins;
#if defined(__x86_64__)
    __builtin_ia32_pause();
#endif
  } else if (spins < 1024) {
    ++spins;
    std::this_thread::yield();
  } else {
    std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
}
}  // namespace

CtrlQueue::CtrlQueue(const std::string& name, uint32_t capacity, bool create) : name_(name), owner_(create) {
  if (capacity == 0 || (capacity & (capacity - 1)) != 0) throw std::invalid_argument("capacity must be a power of 2");
  bytes_ = sizeof(Header) + sizeof(Slot) * capacity;
  int fd;
  if (create) {
    shm_unlink(name.c_str());
    fd = shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
    if (fd < 0) throw std::runtime_error("shm_open(create) failed for " + name);
    if (ftruncate(fd, static_cast<off_t>(bytes_)) != 0) {
      ::close(fd);
      throw std::runtime_error("ftruncate failed for " + name);
    }
  } else {
    fd = -1;
    double t0 = now_s();
    while (fd < 0) {  // the server may not have created it yet
      fd = shm_open(name.c_str(), O_RDWR, 0600);
      if (fd < 0) {
        if (now_s() - t0 > 60.0) throw std::runtime_error("shm_open(attach) timed out for " + name);
        std::this_thread::sleep_for(std::chrono::milliseconds(5));
      }
    }
    struct stat st;
    // wait until the creator has sized it
    double t1 = now_s();
    while (fstat(fd, &st) == 0 && static_cast<size_t>(st.st_size) < bytes_) {
      if (now_s() - t1 > 60.0) throw std::runtime_error("shm segment never sized: " + name);
      std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
  }
  {
    struct stat st;
    if (fstat(fd, &st) == 0) ino_ = (uint64_t)st.st_ino;
  }
  base_ = mmap(nullptr, bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  ::close(fd);
  if (base_ == MAP_FAILED) throw std::runtime_error("mmap failed for " + name);
  hdr_ = static_cast<Header*>(base_);
  slots_ = reinterpret_cast<Slot*>(static_cast<char*>(base_) + sizeof(Header));
  if (create) {
    hdr_->capacity = capacity;
    hdr_->enq.store(0, std::memory_order_relaxed);
    hdr_->deq.store(0, std::memory_order_relaxed);
    for (uint32_t i = 0; i < capacity; ++i) slots_[i].seq.store(i, std::memory_order_relaxed);
    std::atomic_thread_fence(std::memory_order_release);
    reinterpret_cast<std::atomic<uint64_t>*>(&hdr_->magic)->store(kMagic, std::memory_order_release);
  } else {
    double t0 = now_s();
    while (reinterpret_cast<std::atomic<uint64_t>*>(&hdr_->magic)->load(std::memory_order_acquire) != kMagic) {
      if (now_s() - t0 > 60.0) throw std::runtime_error("control queue never initialised: " + name);
      std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
    if (hdr_->capacity != capacity) throw std::runtime_error("control queue capacity mismatch: " + name);
  }
}

CtrlQueue::~CtrlQueue() {
  if (base_ && base_ != MAP_FAILED) munmap(base_, bytes_);
  if (owner_) shm_unlink(name_.c_str());
}

void CtrlQueue::unlink() {
  shm_unlink(name_.c_str());
  owner_ = false;
}

uint32_t CtrlQueue::capacity() const { return hdr_->capacity; }

bool CtrlQueue::try_push(const CtrlToken& t) {
  const uint64_t mask = hdr_->capacity - 1;
  uint64_t pos = hdr_->enq.load(std::memory_order_relaxed);
  for (;;) {
    Slot& s = slots_[pos & mask];
    uint64_t seq = s.seq.load(std::memory_order_acquire);
    int64_t dif = static_cast<int64_t>(seq) - static_cast<int64_t>(pos);
    if (dif == 0) {
      if (hdr_->enq.compare_exchange_weak(pos, pos + 1, std::memory_order_relaxed)) {
        s.tok = t;
        s.seq.store(pos + 1, std::memory_order_release);
        return true;
      }
    } else if (dif < 0) {
      return false;  // full
    } else {
      pos = hdr_->enq.load(std::memory_order_relaxed);
    }
  }
}

bool CtrlQueue::try_pop(CtrlToken* out) {
  const uint64_t mask = hdr_->capacity - 1;
  uint64_t pos = hdr_->deq.load(std::memory_order_relaxed);
  for (;;) {
    Slot& s = slots_[pos & mask];
    uint64_t seq = s.seq.load(std::memory_order_acquire);
    int64_t dif = static_cast<int64_t>(seq) - static_cast<int64_t>(pos + 1);
    if (dif == 0) {
      if (hdr_->deq.compare_exchange_weak(pos, pos + 1, std::memory_order_relaxed)) {
        *out = s.tok;
        s.seq.store(pos + mask + 1, std::memory_order_release);
        return true;
      }
    } else if (dif < 0) {
      return false;  // empty
    } else {
      pos = hdr_->deq.load(std::memory_order_relaxed);
    }
  }
}

bool CtrlQueue::push(const CtrlToken& t, double timeout_s) {
  int spins = 0;
  double t0 = now_s();
  while (!try_push(t)) {
    if (timeout_s >= 0 && (spins & 63) == 0 && now_s() - t0 > timeout_s) return false;
    backoff(spins);
  }
  return true;
}

bool CtrlQueue::pop(CtrlToken* out, double timeout_s) {
  int spins = 0;
  double t0 = now_s();
  while (!try_pop(out)) {
    if (timeout_s >= 0 && (spins & 63) == 0 && now_s() - t0 > timeout_s) return false;
    backoff(spins);
  }
  return true;
}

}  // namespace psx
