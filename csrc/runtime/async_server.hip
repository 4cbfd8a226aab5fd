// Native asynchronous server loop (see async_server.h).
#include "async_server.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>

#include "../kernels/lr_kernels.h"
#include "../kernels/wide_kernels.h"
#include "../solver/solver.h"

namespace psx {
namespace {

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
int64_t epoch_ms() {
  return std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::system_clock::now().time_since_epoch())
      .count();
}
constexpr int kKindDelta = 0, kKindFinal = 1, kKindError = 2;

}  // namespace

// ---- HostP2P: byte FIFOs in one POSIX shared-memory segment ----------------
namespace {
constexpr uint64_t kShmMagic = 0x70737832703270ull;  // "psx2p2p"
constexpr size_t kSegHdr = 256, kChanHdr = 256;
size_t dtype_bytes(int dtype) { return dtype == RcclComm::kU8 ? 1 : 4; }
}  // namespace

struct HostP2P::Chan {
  alignas(128) std::atomic<uint64_t> head;  // bytes written (the producer's)
  alignas(128) std::atomic<uint64_t> tail;  // bytes read (the consumer's)
};
static_assert(sizeof(std::atomic<uint64_t>) == 8, "lock-free 64-bit counters");

HostP2P::HostP2P(const std::string& name, int nworkers, int rank, bool create, bool device, size_t cap_bytes,
                 double timeout_s)
    : name_(name), n_(nworkers), rank_(rank), owner_(create), device_(device), cap_(cap_bytes),
      timeout_s_(timeout_s) {
  if (nworkers < 1 || rank < 0 || rank > nworkers || cap_bytes < 4096 || name.empty() || name[0] != '/')
    throw std::invalid_argument("HostP2P: bad arguments");
  map_bytes_ = kSegHdr + (size_t)2 * nworkers * (kChanHdr + cap_);
  int fd;
  if (create) {
    fd = shm_open(name.c_str(), O_CREAT | O_RDWR | O_TRUNC, 0600);
    if (fd < 0) throw std::runtime_error("HostP2P: shm_open(create) " + name);
    if (ftruncate(fd, (off_t)map_bytes_) != 0) {
      close(fd);
      throw std::runtime_error("HostP2P: ftruncate");
    }
  } else {
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {  // the server creates the segment before the rendezvous barrier; tolerate a race
      fd = shm_open(name.c_str(), O_RDWR, 0600);
      struct stat st {};
      if (fd >= 0 && fstat(fd, &st) == 0 && (size_t)st.st_size >= map_bytes_) break;
      if (fd >= 0) close(fd);
      if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s_)
        throw std::runtime_error("HostP2P: no segment " + name);
      std::this_thread::sleep_for(std::chrono::milliseconds(2));
    }
  }
  void* p = mmap(nullptr, map_bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) throw std::runtime_error("HostP2P: mmap");
  base_ = static_cast<char*>(p);
  auto* magic = reinterpret_cast<std::atomic<uint64_t>*>(base_);
  if (create) {
    for (int i = 0; i < 2 * n_; ++i) {
      new (&chan(i)->head) std::atomic<uint64_t>(0);
      new (&chan(i)->tail) std::atomic<uint64_t>(0);
    }
    reinterpret_cast<uint64_t*>(base_)[1] = (uint64_t)n_;
    reinterpret_cast<uint64_t*>(base_)[2] = (uint64_t)cap_;
    magic->store(kShmMagic, std::memory_order_release);
  } else {
    const auto t0 = std::chrono::steady_clock::now();
    while (magic->load(std::memory_order_acquire) != kShmMagic) {
      if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s_)
        throw std::runtime_error("HostP2P: segment never initialised");
      std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
    if (reinterpret_cast<uint64_t*>(base_)[1] != (uint64_t)n_ || reinterpret_cast<uint64_t*>(base_)[2] != cap_)
      throw std::runtime_error("HostP2P: segment shape differs");
  }
}

HostP2P::~HostP2P() {
  if (bounce_) (void)hipHostFree(bounce_);
  if (base_) munmap(base_, map_bytes_);
  if (owner_) shm_unlink(name_.c_str());
}

void HostP2P::unlink() {
  if (owner_) shm_unlink(name_.c_str());
  owner_ = false;
}

HostP2P::Chan* HostP2P::chan(int idx) const {
  return reinterpret_cast<Chan*>(base_ + kSegHdr + (size_t)idx * (kChanHdr + cap_));
}
// channel 2k: worker k -> server, 2k + 1: server -> worker k
int HostP2P::out_chan(int peer) const {
  if (rank_ == 0) {
    if (peer < 1 || peer > n_) throw std::invalid_argument("HostP2P::send: peer");
    return 2 * (peer - 1) + 1;
  }
  if (peer != 0) throw std::invalid_argument("HostP2P: workers talk to the server only");
  return 2 * (rank_ - 1);
}
int HostP2P::in_chan(int peer) const {
  if (rank_ == 0) {
    if (peer < 1 || peer > n_) throw std::invalid_argument("HostP2P::recv: peer");
    return 2 * (peer - 1);
  }
  if (peer != 0) throw std::invalid_argument("HostP2P: workers talk to the server only");
  return 2 * (rank_ - 1) + 1;
}

void HostP2P::write(Chan* c, const char* src, size_t n) {
  char* data = reinterpret_cast<char*>(c) + kChanHdr;
  uint64_t head = c->head.load(std::memory_order_relaxed);
  auto t0 = std::chrono::steady_clock::now();
  int spins = 0;
  while (n > 0) {
    const uint64_t tail = c->tail.load(std::memory_order_acquire);
    const size_t room = cap_ - (size_t)(head - tail);
    if (room == 0) {
      if (++spins > 64) std::this_thread::sleep_for(std::chrono::microseconds(spins < 4096 ? 2 : 100));
      if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s_)
        throw std::runtime_error("HostP2P: send timed out (peer not receiving)");
      continue;
    }
    const size_t off = (size_t)(head % cap_);
    const size_t m = std::min({n, room, cap_ - off});
    std::memcpy(data + off, src, m);
    head += m;
    src += m;
    n -= m;
    c->head.store(head, std::memory_order_release);
    spins = 0;
    t0 = std::chrono::steady_clock::now();
  }
}

void HostP2P::read(Chan* c, char* dst, size_t n) {
  const char* data = reinterpret_cast<const char*>(c) + kChanHdr;
  uint64_t tail = c->tail.load(std::memory_order_relaxed);
  auto t0 = std::chrono::steady_clock::now();
  int spins = 0;
  while (n > 0) {
    const uint64_t head = c->head.load(std::memory_order_acquire);
    const size_t avail = (size_t)(head - tail);
    if (avail == 0) {
      if (++spins > 64) std::this_thread::sleep_for(std::chrono::microseconds(spins < 4096 ? 2 : 100));
      if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s_)
        throw std::runtime_error("HostP2P: recv timed out (peer not sending)");
      continue;
    }
    const size_t off = (size_t)(tail % cap_);
    const size_t m = std::min({n, avail, cap_ - off});
    std::memcpy(dst, data + off, m);
    tail += m;
    dst += m;
    n -= m;
    c->tail.store(tail, std::memory_order_release);
    spins = 0;
    t0 = std::chrono::steady_clock::now();
  }
}

void HostP2P::send(const void* buf, size_t count, int dtype, int peer, hipStream_t s) {
  const size_t bytes = count * dtype_bytes(dtype);
  Chan* c = chan(out_chan(peer));
  if (!device_) {
    write(c, static_cast<const char*>(buf), bytes);
    return;
  }
  char* st = staging(bytes);  // stream order: behind the producer of buf on s
  hip_check(hipMemcpyAsync(st, buf, bytes, hipMemcpyDeviceToHost, s), "HostP2P send staging");
  hip_check(hipStreamSynchronize(s), "HostP2P send sync");
  write(c, st, bytes);
}

char* HostP2P::staging(size_t bytes) {
  if (bytes > bounce_bytes_) {
    if (bounce_) hip_check(hipHostFree(bounce_), "hipHostFree");
    bounce_ = nullptr;
    hip_check(hipHostMalloc((void**)&bounce_, bytes, hipHostMallocDefault), "HostP2P staging");
    bounce_bytes_ = bytes;
  }
  return bounce_;
}

void HostP2P::recv(void* buf, size_t count, int dtype, int peer, hipStream_t s) {
  const size_t bytes = count * dtype_bytes(dtype);
  Chan* c = chan(in_chan(peer));
  if (!device_) {
    read(c, static_cast<char*>(buf), bytes);
    return;
  }
  char* st = staging(bytes);
  hip_check(hipStreamSynchronize(s), "HostP2P recv sync");  // (the staging buffer's previous copy)
  read(c, st, bytes);
  hip_check(hipMemcpyAsync(buf, st, bytes, hipMemcpyHostToDevice, s), "HostP2P recv staging");
  hip_check(hipStreamSynchronize(s), "HostP2P recv sync");
}

RcclP2P::RcclP2P(RcclComm* c) : c_(c) {
  if (!c_) throw std::invalid_argument("RcclP2P: null communicator");
  if (c_->rank() != 0) throw std::invalid_argument("the asynchronous server runs on rank 0");
}

LocalP2P::LocalP2P(int nworkers, const std::vector<uintptr_t>& out_f32, const std::vector<uintptr_t>& out_i32,
                   const std::vector<uintptr_t>& inbox)
    : n_(nworkers), out_f32_(out_f32), out_i32_(out_i32), inbox_(inbox),
      released_(new std::atomic<int64_t>[nworkers > 0 ? nworkers : 1]) {
  if (nworkers < 1 || (int)out_f32.size() != nworkers || (int)inbox.size() != nworkers ||
      (!out_i32.empty() && (int)out_i32.size() != nworkers))
    throw std::invalid_argument("LocalP2P: one outbox / inbox per worker");
  for (int k = 0; k < nworkers; ++k) released_[k].store(0);
}

void LocalP2P::send(const void* buf, size_t count, int dtype, int peer, hipStream_t s) {
  if (peer < 1 || peer > n_ || dtype == RcclComm::kU8) throw std::invalid_argument("LocalP2P::send: peer / dtype");
  // the inbox is sized for the dense weights: every pull piece fits (stand-in
  // workers read only the release counter); one release per group
  hip_check(hipMemcpyAsync(reinterpret_cast<void*>(inbox_[peer - 1]), buf, count * 4, hipMemcpyDeviceToDevice, s),
            "LocalP2P send copy");
  if (!in_group_) released_[peer - 1].fetch_add(1, std::memory_order_release);
  else group_peers_.push_back(peer - 1);
}

void LocalP2P::group_start() {
  in_group_ = true;
  group_peers_.clear();
}

void LocalP2P::group_end() {
  in_group_ = false;
  std::sort(group_peers_.begin(), group_peers_.end());
  group_peers_.erase(std::unique(group_peers_.begin(), group_peers_.end()), group_peers_.end());
  for (int k : group_peers_) released_[k].fetch_add(1, std::memory_order_release);
  group_peers_.clear();
}

void LocalP2P::recv(void* buf, size_t count, int dtype, int peer, hipStream_t s) {
  if (peer < 1 || peer > n_) throw std::invalid_argument("LocalP2P::recv: peer");
  uintptr_t src = dtype == RcclComm::kI32 ? (out_i32_.empty() ? 0 : out_i32_[peer - 1]) : out_f32_[peer - 1];
  if (!src) throw std::invalid_argument("LocalP2P::recv: no outbox of that dtype");
  hip_check(hipMemcpyAsync(buf, reinterpret_cast<const void*>(src), count * 4, hipMemcpyDeviceToDevice, s),
            "LocalP2P recv copy");
}

int64_t LocalP2P::released(int k) const { return released_[k].load(std::memory_order_acquire); }

LocalFeeder::LocalFeeder(uintptr_t api, uintptr_t ctrl, LocalP2P* p2p, int nworkers, int64_t iters, int64_t token_n,
                         double timeout_s, const std::vector<int64_t>& vc0, const std::vector<uintptr_t>& replies)
    : api_(reinterpret_cast<const HostApi*>(api)), ctrl_(ctrl), p2p_(p2p), n_(nworkers), iters_(iters),
      token_n_(token_n), timeout_s_(timeout_s), vc0_(vc0), base_(nworkers, 0), replies_(replies) {
  if (!replies_.empty() && (int)replies_.size() != nworkers)
    throw std::invalid_argument("LocalFeeder: one reply queue per worker");
  if (!api_ || api_->version != kHostApiVersion || !ctrl || !p2p || nworkers < 1 || iters < 1)
    throw std::invalid_argument("LocalFeeder: bad arguments");
  if (vc0_.empty()) vc0_.assign(nworkers, 0);
  if ((int)vc0_.size() != nworkers) throw std::invalid_argument("LocalFeeder: one start clock per worker");
  // construct BEFORE the server's begin(): its bootstrap sends count as releases
  for (int k = 0; k < n_; ++k) base_[k] = p2p_->released(k);
}

LocalFeeder::~LocalFeeder() { join(); }

void LocalFeeder::start() {
  for (int k = 0; k < n_; ++k) th_.emplace_back([this, k] { run(k); });
}

bool LocalFeeder::join() {
  for (auto& t : th_)
    if (t.joinable()) t.join();
  th_.clear();
  return failed_.load() == 0;
}

void LocalFeeder::run(int k) {
  for (int64_t it = 0; it < iters_; ++it) {
    const double t0 = now_s();
    while (p2p_->released(k) < base_[k] + it + 1) {  // the weights of this clock were sent to k
      if (now_s() - t0 > timeout_s_) {
        failed_.fetch_add(1);
        return;
      }
      std::this_thread::yield();
    }
    if (!replies_.empty()) {  // sparse pull: consume the release's reply token
      CtrlToken r{};
      if (api_->ctrl_pop((void*)replies_[k], &r, timeout_s_) != 1) {
        failed_.fetch_add(1);
        return;
      }
      if (r.kind == 1) sparse_.fetch_add(1);
    }
    CtrlToken t{};
    t.worker = k;
    t.kind = it + 1 == iters_ ? kKindFinal : kKindDelta;
    t.vc = vc0_[k] + it;
    t.n = token_n_;
    if (api_->ctrl_push((void*)ctrl_, &t, timeout_s_) != 1) {
      failed_.fetch_add(1);
      return;
    }
  }
}

AsyncServer::AsyncServer(P2P* comm, const AsyncServerCfg& cfg, hipStream_t stream)
    : comm_(comm), cfg_(cfg), stream_(stream) {
  if (!comm_) throw std::invalid_argument("AsyncServer: null transport");
  // one rank per worker, or (peer map) several workers per worker rank: every
  // worker's rank in [1, size)
  if (cfg.nworkers < 1 || (cfg.peer.empty() ? comm_->size() != cfg.nworkers + 1 : comm_->size() < 2))
    throw std::invalid_argument("AsyncServer: the communicator must hold the server + every worker");
  for (int p : cfg.peer)
    if (p < 1 || p >= comm_->size()) throw std::invalid_argument("AsyncServer: a worker's peer rank is outside the communicator");
  if (!cfg.api || !cfg.tracker || !cfg.ctrl) throw std::invalid_argument("AsyncServer: missing host runtime handles");
  api_ = reinterpret_cast<const HostApi*>(cfg.api);
  if (api_->version != kHostApiVersion) throw std::runtime_error("AsyncServer: host runtime C ABI version mismatch");
  if (!cfg.w || cfg.P <= 0) throw std::invalid_argument("AsyncServer: no weights");
  if (cfg.model == kAsyncWideSparse) {
    if (!cfg.ubuf || !cfg.dbuf || cfg.KP < 1 || cfg.umax < 0) throw std::invalid_argument("AsyncServer: sparse buffers");
  } else if (!cfg.buf) {
    throw std::invalid_argument("AsyncServer: no receive buffer");
  }
  if (cfg.model == kAsyncDense && cfg.sink && !cfg.cpu && (!cfg.fhi || !cfg.flo || !cfg.fb || !cfg.Xt || !cfg.yt))
    throw std::invalid_argument("AsyncServer: dense evaluation needs fragments and a test set");
  if (cfg.sink && (!cfg.acc || !cfg.ticket)) throw std::invalid_argument("AsyncServer: evaluation scratch");
  if (!cfg.peer.empty() && (int)cfg.peer.size() != cfg.nworkers)
    throw std::invalid_argument("AsyncServer: one peer per worker");
  if (!cfg.replies.empty() && (int)cfg.replies.size() != cfg.nworkers)
    throw std::invalid_argument("AsyncServer: one reply queue per worker");
  finished_.assign(cfg.nworkers, 0);
  failed_.assign(cfg.nworkers, 0);
  dead_.assign(cfg.nworkers, 0);
  last_pos_.assign(cfg.nworkers, -1);
  since_dense_.assign(cfg.nworkers, 0);
  if (cfg.sparse_pull) {
    if (cfg.model != kAsyncWideSparse) throw std::invalid_argument("AsyncServer: sparse pull needs sparse pushes");
    if (!cfg.lids || !cfg.lvals || cfg.logcap < 1 || (int)cfg.replies.size() != cfg.nworkers)
      throw std::invalid_argument("AsyncServer: sparse pull needs the ring log and one reply queue per worker");
  }
  busy_since_.assign(cfg.nworkers, -1.0);
  rel_k_.resize(cfg.nworkers + 1);
  rel_v_.resize(cfg.nworkers + 1);
}

void AsyncServer::check_api(int rc, const char* what) const {
  if (rc < 0) throw std::runtime_error(std::string("AsyncServer: ") + what + ": " + api_->last_error());
}

int AsyncServer::log_worker() const {
  // server rows follow the deltas of worker 0 (ServerProcessor.java:154-165), or of
  // the lowest surviving worker once 0 has failed
  for (int j = 0; j < cfg_.nworkers; ++j)
    if (!failed_[j]) return j;
  return -1;
}

std::vector<int> AsyncServer::failed() const {
  std::vector<int> out;
  for (int j = 0; j < cfg_.nworkers; ++j)
    if (failed_[j]) out.push_back(j);
  return out;
}

void AsyncServer::send_weights(const int* ks, const int64_t* vs, int n) {
  bool any = false;
  for (int i = 0; i < n; ++i) any |= !finished_[ks[i]];
  if (!any) return;
  const double t = now_s();
  const int KP = cfg_.KP;
  comm_->group_start();
  for (int i = 0; i < n; ++i) {
    const int j = ks[i];
    if (finished_[j]) continue;
    busy_since_[j] = t;
    if (!cfg_.sparse_pull) {
      if (!cfg_.replies.empty()) {  // several workers per rank: which one the weights are for
        CtrlToken r{};
        r.worker = j;
        r.vc = vs[i];
        if (api().ctrl_push((void*)cfg_.replies[j], &r, cfg_.worker_timeout_s) != 1)
          throw std::runtime_error("AsyncServer: reply queue of worker " + std::to_string(j) + " full");
      }
      comm_->send(cfg_.w, (size_t)cfg_.P, RcclComm::kF32, peer_of(j), stream_);
      pull_floats_ += cfg_.P;
      ++dense_pulls_;
      continue;
    }
    // the entries [last_pos_[j], log_pos_) of the ring log, or the dense vector
    const int64_t m = last_pos_[j] < 0 ? -1 : log_pos_ - last_pos_[j];
    const bool sparse = m >= 0 && m <= cfg_.logcap && m * (KP + 1) * 2 < cfg_.P && since_dense_[j] < cfg_.dense_every;
    CtrlToken r{};
    r.worker = j;
    r.vc = vs[i];
    if (sparse) {
      const int64_t start = last_pos_[j] % cfg_.logcap;
      const int64_t len1 = m < cfg_.logcap - start ? m : cfg_.logcap - start, len2 = m - len1;
      r.kind = 1;
      r.n = m;
      r.aux = len1;
      if (api().ctrl_push((void*)cfg_.replies[j], &r, cfg_.worker_timeout_s) != 1)
        throw std::runtime_error("AsyncServer: reply queue of worker " + std::to_string(j) + " full");
      if (len1) {
        comm_->send(cfg_.lids + start, (size_t)len1, RcclComm::kI32, peer_of(j), stream_);
        comm_->send(cfg_.lvals + start * KP, (size_t)(len1 * KP), RcclComm::kF32, peer_of(j), stream_);
      }
      if (len2) {
        comm_->send(cfg_.lids, (size_t)len2, RcclComm::kI32, peer_of(j), stream_);
        comm_->send(cfg_.lvals, (size_t)(len2 * KP), RcclComm::kF32, peer_of(j), stream_);
      }
      ++since_dense_[j];
      ++sparse_pulls_;
      pull_floats_ += m * (KP + 1);
    } else {
      r.kind = 0;
      if (api().ctrl_push((void*)cfg_.replies[j], &r, cfg_.worker_timeout_s) != 1)
        throw std::runtime_error("AsyncServer: reply queue of worker " + std::to_string(j) + " full");
      comm_->send(cfg_.w, (size_t)cfg_.P, RcclComm::kF32, peer_of(j), stream_);
      since_dense_[j] = 0;
      ++dense_pulls_;
      pull_floats_ += cfg_.P;
    }
    last_pos_[j] = log_pos_;
  }
  comm_->group_end();
}

void AsyncServer::begin() {
  std::fill(last_pos_.begin(), last_pos_.end(), -1);  // every run starts with a dense pull
  std::fill(finished_.begin(), finished_.end(), 0);
  std::fill(failed_.begin(), failed_.end(), 0);
  std::fill(busy_since_.begin(), busy_since_.end(), -1.0);
  int n = 0;
  for (int j = 0; j < cfg_.nworkers; ++j) {
    int live = api().tracker_is_live((void*)cfg_.tracker, j);
    check_api(live, "tracker is_live");
    if (!live && !dead_[j]) {  // retired because it finished the previous run: rejoins
      check_api(api().tracker_revive((void*)cfg_.tracker, j), "tracker revive");
      live = 1;
    }
    if (!live) {  // failed in an earlier run (or retired in a resumed checkpoint)
      failed_[j] = finished_[j] = dead_[j] = 1;
      continue;
    }
    const int64_t u = api().tracker_clock((void*)cfg_.tracker, j);
    if (u > 0) api().tracker_sent((void*)cfg_.tracker, j, u);  // a later run resumes at the tracked clocks
    rel_k_[n] = j;
    rel_v_[n] = u;
    ++n;
  }
  send_weights(rel_k_.data(), rel_v_.data(), n);  // the bootstrap (ServerProcessor.java:75-87)
}

// Host-memory update (CPU ranks): the same arithmetic as the update kernels
// (server_apply / axpy: w += lr * delta; wide_apply_sparse: the pushed ids'
// values and the intercepts; the pull log), without evaluation fragments.
void AsyncServer::apply_cpu(const CtrlToken& t) {
  const int peer = peer_of(t.worker);
  float* w = cfg_.w;
  const float lr = cfg_.lr;
  if (cfg_.model == kAsyncWideSparse) {
    const int64_t U = t.n, KP = cfg_.KP;
    if (U < 0 || U > cfg_.umax) throw std::runtime_error("AsyncServer: sparse push larger than the buffer");
    if (U) comm_->recv(cfg_.ubuf, (size_t)U, RcclComm::kI32, peer, stream_);
    comm_->recv(cfg_.dbuf, (size_t)(KP + U * KP), RcclComm::kF32, peer, stream_);
    for (int64_t p = 0; p < KP + U * KP; ++p) {
      const float v = cfg_.dbuf[p];
      if (v == 0.f) continue;
      if (p < KP)
        w[cfg_.Fw * KP + p] += lr * v;
      else
        w[(int64_t)cfg_.ubuf[(p - KP) / KP] * KP + (p - KP) % KP] += lr * v;
    }
    if (cfg_.sparse_pull) {
      if (U + 1 > cfg_.logcap) throw std::runtime_error("AsyncServer: push larger than the pull log");
      for (int64_t l = 0; l <= U; ++l) {
        const int64_t slot = (log_pos_ + l) % cfg_.logcap;
        cfg_.lids[slot] = l == 0 ? (int32_t)cfg_.Fw : cfg_.ubuf[l - 1];
        for (int64_t c = 0; c < KP; ++c) cfg_.lvals[slot * KP + c] = cfg_.dbuf[l * KP + c];
      }
      log_pos_ += U + 1;
    }
    return;
  }
  comm_->recv(cfg_.buf, (size_t)cfg_.P, RcclComm::kF32, peer, stream_);
  for (int64_t i = 0; i < cfg_.P; ++i) w[i] += lr * cfg_.buf[i];
}

// Host-memory evaluation of the global model on the test set (CPU ranks): the
// argmax confusion counts published into the metrics slot like the kernels do.
void AsyncServer::eval_cpu(char* slot, uint64_t seq) {
  int32_t conf[256] = {0};
  const float* w = cfg_.w;
  if (cfg_.model == kAsyncDense) {
    const int K = cfg_.K, FP = cfg_.FP;
    for (int t = 0; t < cfg_.T; ++t) {
      int best = 0;
      float bz = -INFINITY;
      for (int c = 0; c < K; ++c) {
        float z = w[(int64_t)K * FP + c];
        const uint16_t* x = cfg_.Xt + (int64_t)t * FP;
        const float* wc = w + (int64_t)c * FP;
        for (int f = 0; f < cfg_.F; ++f) {
          uint32_t u = (uint32_t)x[f] << 16;
          float xf;
          std::memcpy(&xf, &u, 4);
          z += xf * wc[f];
        }
        if (z > bz) {
          bz = z;
          best = c;
        }
      }
      const int y = std::min(15, std::max(0, (int)cfg_.yt[t]));
      ++conf[y * 16 + best];
    }
  } else {
    const int K = cfg_.K, KP = cfg_.KP;
    std::vector<float> z(KP);
    for (int t = 0; t < cfg_.T; ++t) {
      for (int k = 0; k < KP; ++k) z[k] = w[cfg_.Fw * KP + k];
      for (int64_t e = cfg_.t_indptr[t]; e < cfg_.t_indptr[t + 1]; ++e) {
        uint32_t u = (uint32_t)cfg_.t_val[e] << 16;
        float v;
        std::memcpy(&v, &u, 4);
        for (int k = 0; k < KP; ++k) z[k] += v * w[(int64_t)cfg_.t_idx[e] * KP + k];
      }
      int best = 0;
      if (K == 1) {
        best = z[0] > 0.f ? 1 : 0;
      } else {
        float bz = -INFINITY;
        for (int k = 0; k < K; ++k)
          if (z[k] > bz) {
            bz = z[k];
            best = k;
          }
      }
      int y = cfg_.t_y[t];
      if (K == 1) y = y > 0 ? 1 : 0;
      y = std::min(15, std::max(0, y));
      ++conf[y * 16 + best];
    }
  }
  std::memcpy(slot, conf, sizeof(conf));
  const float zero = 0.f;
  std::memcpy(slot + 1024, &zero, 4);
  __atomic_store_n(reinterpret_cast<uint64_t*>(slot + 1032), (uint64_t)seq, __ATOMIC_RELEASE);
}

void AsyncServer::apply_and_log(const CtrlToken& t) {
  const int k = t.worker;
  const int peer = peer_of(k);
  const int64_t v = t.vc;
  if (cfg_.cpu) {
    apply_cpu(t);
    ++updates_;
    ++updates_run_;
    if (cfg_.sink && k == log_worker()) {
      uint64_t seq = 0;
      uintptr_t addr = 0;
      const int slot = api().sink_acquire((void*)cfg_.sink, &seq, &addr);
      check_api(slot, "metrics sink acquire");
      eval_cpu(reinterpret_cast<char*>(addr), seq);
      api().sink_submit((void*)cfg_.sink, slot, seq, 1, -1, -1, v, 0);
    }
    return;
  }
  if (cfg_.model == kAsyncWideSparse) {
    const int64_t U = t.n;
    if (U < 0 || U > cfg_.umax) throw std::runtime_error("AsyncServer: sparse push larger than the buffer");
    if (U) comm_->recv(cfg_.ubuf, (size_t)U, RcclComm::kI32, peer, stream_);
    comm_->recv(cfg_.dbuf, (size_t)(cfg_.KP + U * cfg_.KP), RcclComm::kF32, peer, stream_);
    launch_wide_apply_sparse(cfg_.w, cfg_.Fw, cfg_.KP, nullptr, (int)U, cfg_.ubuf, cfg_.dbuf, cfg_.lr, cfg_.umax,
                             stream_);
    if (cfg_.sparse_pull) {  // stream-ordered after every send that reads the slots it overwrites
      if (U + 1 > cfg_.logcap) throw std::runtime_error("AsyncServer: push larger than the pull log");
      launch_log_append(cfg_.ubuf, cfg_.dbuf, (int)U, cfg_.Fw, cfg_.KP, cfg_.lids, cfg_.lvals,
                        log_pos_ % cfg_.logcap, cfg_.logcap, stream_);
      log_pos_ += U + 1;
    }
  } else {
    comm_->recv(cfg_.buf, (size_t)cfg_.P, RcclComm::kF32, peer, stream_);
    if (cfg_.model == kAsyncDense)
      launch_server_apply(cfg_.K, cfg_.F, cfg_.FP, cfg_.w, cfg_.buf, cfg_.lr, cfg_.fhi, cfg_.flo, cfg_.fb, stream_,
                          cfg_.coff);
    else
      launch_axpy(cfg_.w, cfg_.buf, cfg_.lr, cfg_.P, stream_);
  }
  ++updates_;
  ++updates_run_;
  if (cfg_.sink && k == log_worker()) {  // the global model's test metrics, one server row
    uint64_t seq = 0;
    uintptr_t addr = 0;
    const int slot = api().sink_acquire((void*)cfg_.sink, &seq, &addr);
    check_api(slot, "metrics sink acquire");
    if (cfg_.model == kAsyncDense)
      launch_test_eval(cfg_.FP, cfg_.K, cfg_.Xt, cfg_.yt, cfg_.T, cfg_.fhi, cfg_.flo, cfg_.fb, cfg_.acc, stream_,
                       cfg_.ticket, reinterpret_cast<void*>(addr), nullptr, seq, cfg_.coff);
    else
      launch_wide_eval(cfg_.K, cfg_.KP, cfg_.Fw, cfg_.t_indptr, cfg_.t_idx, cfg_.t_val, cfg_.t_y, cfg_.T, cfg_.w,
                       nullptr, 0u, nullptr, cfg_.acc, cfg_.ticket, reinterpret_cast<void*>(addr), nullptr, seq, stream_);
    api().sink_submit((void*)cfg_.sink, slot, seq, 1, -1, -1, v, 0);  // stamped when the evaluation lands
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("AsyncServer launch: ") + hipGetErrorString(e));
}

void AsyncServer::fail(int k) {
  if (k < 0 || k >= cfg_.nworkers) throw std::out_of_range("AsyncServer::fail: worker id");
  failed_[k] = finished_[k] = dead_[k] = 1;
  busy_since_[k] = -1.0;
  const int n = api().tracker_retire((void*)cfg_.tracker, k, rel_k_.data(), rel_v_.data(), (int)rel_k_.size());
  check_api(n, "tracker retire");
  send_weights(rel_k_.data(), rel_v_.data(), n);
}

AsyncStatus AsyncServer::run(int64_t checkpoint_every) {
  AsyncStatus st;
  const double poll = cfg_.worker_timeout_s < 1.0 ? cfg_.worker_timeout_s : 1.0;
  for (;;) {
    int open = 0;
    for (int j = 0; j < cfg_.nworkers; ++j) open += !finished_[j];
    if (open == 0) break;
    CtrlToken t;
    const int got = api().ctrl_pop((void*)cfg_.ctrl, &t, poll);
    check_api(got, "token pop");
    if (!got) {  // watchdog: a worker holding weights that stays silent has failed
      const double now = now_s();
      for (int j = 0; j < cfg_.nworkers; ++j)
        if (!finished_[j] && busy_since_[j] >= 0.0 && now - busy_since_[j] > cfg_.worker_timeout_s) {
          st.code = kAsyncWatchdog;
          st.worker = j;
          st.updates = updates_;
          return st;
        }
      continue;
    }
    const auto h0 = std::chrono::steady_clock::now();
    ++tokens_;
    const int k = t.worker;
    if (k < 0 || k >= cfg_.nworkers) throw std::runtime_error("AsyncServer: token from an unknown worker");
    if (t.kind == kKindError) {
      st.code = kAsyncErrorToken;
      st.worker = k;
      st.updates = updates_;
      return st;
    }
    if (finished_[k]) throw std::runtime_error("AsyncServer: delta from a finished worker " + std::to_string(k));
    busy_since_[k] = -1.0;
    apply_and_log(t);
    int n = api().tracker_on_delta((void*)cfg_.tracker, k, t.vc, rel_k_.data(), rel_v_.data(), (int)rel_k_.size());
    check_api(n, "tracker on_delta");
    if (t.kind == kKindFinal) {
      // a finished worker no longer holds the others back (its frozen clock would
      // stall an SSP worker D ahead forever)
      finished_[k] = 1;
      const int m = api().tracker_retire((void*)cfg_.tracker, k, rel_k_.data() + n, rel_v_.data() + n,
                                         (int)rel_k_.size() - n);
      check_api(m, "tracker retire");
      n += m;
    }
    send_weights(rel_k_.data(), rel_v_.data(), n);
    host_ns_ += std::chrono::duration<double, std::nano>(std::chrono::steady_clock::now() - h0).count();
    if (checkpoint_every > 0 && updates_ % checkpoint_every == 0) {
      st.code = kAsyncCheckpoint;
      st.updates = updates_;
      return st;
    }
  }
  st.code = kAsyncDone;
  st.updates = updates_;
  return st;
}

}  // namespace psx
