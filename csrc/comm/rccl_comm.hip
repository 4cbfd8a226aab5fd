// Native RCCL communicator (see rccl_comm.h).
#include "rccl_comm.h"

#include <dlfcn.h>
#include <rccl/rccl.h>

#include <cstring>
#include <mutex>
#include <stdexcept>

namespace psx {
namespace {

struct Api {
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) init_rank = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  decltype(&ncclCommAbort) abort = nullptr;
  decltype(&ncclGetErrorString) err = nullptr;
  decltype(&ncclAllReduce) all_reduce = nullptr;
  decltype(&ncclReduce) reduce = nullptr;
  decltype(&ncclBroadcast) broadcast = nullptr;
  decltype(&ncclReduceScatter) reduce_scatter = nullptr;
  decltype(&ncclAllGather) all_gather = nullptr;
  decltype(&ncclSend) send = nullptr;
  decltype(&ncclRecv) recv = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  bool ok = false;
};

template <class T>
bool resolve(void* h, const char* name, T* out) {
  *out = reinterpret_cast<T>(dlsym(h, name));
  return *out != nullptr;
}

const Api& api() {
  static Api a;
  static std::once_flag once;
  std::call_once(once, [] {
    // the RCCL PyTorch already mapped (same SONAME) first; else load it
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD | RTLD_GLOBAL);
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
    if (!h) return;
    bool ok = resolve(h, "ncclGetUniqueId", &a.get_unique_id) && resolve(h, "ncclCommInitRank", &a.init_rank) &&
              resolve(h, "ncclCommDestroy", &a.destroy) && resolve(h, "ncclCommAbort", &a.abort) &&
              resolve(h, "ncclGetErrorString", &a.err) && resolve(h, "ncclAllReduce", &a.all_reduce) &&
              resolve(h, "ncclReduce", &a.reduce) && resolve(h, "ncclBroadcast", &a.broadcast) &&
              resolve(h, "ncclReduceScatter", &a.reduce_scatter) && resolve(h, "ncclAllGather", &a.all_gather) &&
              resolve(h, "ncclSend", &a.send) && resolve(h, "ncclRecv", &a.recv) &&
              resolve(h, "ncclGroupStart", &a.group_start) && resolve(h, "ncclGroupEnd", &a.group_end);
    a.ok = ok;
  });
  return a;
}

const Api& need() {
  const Api& a = api();
  if (!a.ok) throw std::runtime_error("RCCL library not found in the process");
  return a;
}

void check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) throw std::runtime_error(std::string("RCCL ") + what + ": " + need().err(r));
}

ncclDataType_t dt(int d) {
  switch (d) {
    case RcclComm::kF32: return ncclFloat32;
    case RcclComm::kI32: return ncclInt32;
    case RcclComm::kU8: return ncclUint8;
  }
  throw std::invalid_argument("RcclComm: unsupported dtype");
}

}  // namespace

bool RcclComm::available() { return api().ok; }

std::string RcclComm::unique_id() {
  ncclUniqueId id;
  check(need().get_unique_id(&id), "get unique id");
  return std::string(id.internal, NCCL_UNIQUE_ID_BYTES);
}

RcclComm::RcclComm(const std::string& id, int nranks, int rank, int device) : nranks_(nranks), rank_(rank) {
  if (id.size() != NCCL_UNIQUE_ID_BYTES) throw std::invalid_argument("RcclComm: unique id must be 128 bytes");
  if (nranks < 1 || rank < 0 || rank >= nranks) throw std::invalid_argument("RcclComm: bad rank / size");
  if (hipSetDevice(device) != hipSuccess) throw std::runtime_error("RcclComm: hipSetDevice failed");
  ncclUniqueId uid;
  std::memcpy(uid.internal, id.data(), NCCL_UNIQUE_ID_BYTES);
  ncclComm_t c = nullptr;
  check(need().init_rank(&c, nranks, uid, rank), "comm init");
  comm_ = c;
  if (hipStreamCreateWithFlags(&side_, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&ev_fork_, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&ev_join_, hipEventDisableTiming) != hipSuccess) {
    abort();
    throw std::runtime_error("RcclComm: stream / event creation failed");
  }
}

// a communicator still open at destruction (error paths, interpreter exit) is
// aborted, not destroyed: destroy can block on peers that are already gone
RcclComm::~RcclComm() { abort(); }

void RcclComm::release_stream() {
  if (ev_fork_) (void)hipEventDestroy(ev_fork_);
  if (ev_join_) (void)hipEventDestroy(ev_join_);
  if (side_) (void)hipStreamDestroy(side_);
  ev_fork_ = ev_join_ = nullptr;
  side_ = nullptr;
}

void RcclComm::close() {
  if (!comm_) return;
  if (side_) (void)hipStreamSynchronize(side_);
  ncclComm_t c = static_cast<ncclComm_t>(comm_);
  comm_ = nullptr;
  release_stream();
  check(need().destroy(c), "comm destroy");
}

void RcclComm::abort() {
  if (comm_) {
    ncclComm_t c = static_cast<ncclComm_t>(comm_);
    comm_ = nullptr;
    (void)need().abort(c);
  }
  release_stream();
}

void RcclComm::fork(hipStream_t compute) {
  if (hipEventRecord(ev_fork_, compute) != hipSuccess || hipStreamWaitEvent(side_, ev_fork_, 0) != hipSuccess)
    throw std::runtime_error("RcclComm::fork failed");
}

void RcclComm::join(hipStream_t compute) {
  if (hipEventRecord(ev_join_, side_) != hipSuccess || hipStreamWaitEvent(compute, ev_join_, 0) != hipSuccess)
    throw std::runtime_error("RcclComm::join failed");
}

#define PSX_COMM static_cast<ncclComm_t>(comm_)
#define PSX_LIVE() \
  if (!comm_) throw std::runtime_error("RcclComm used after close")

void RcclComm::all_reduce(const void* send, void* recv, size_t count, int dtype, hipStream_t s) {
  PSX_LIVE();
  check(need().all_reduce(send, recv, count, dt(dtype), ncclSum, PSX_COMM, s), "all_reduce");
}
void RcclComm::reduce(const void* send, void* recv, size_t count, int dtype, int root, hipStream_t s) {
  PSX_LIVE();
  check(need().reduce(send, recv, count, dt(dtype), ncclSum, root, PSX_COMM, s), "reduce");
}
void RcclComm::broadcast(const void* send, void* recv, size_t count, int dtype, int root, hipStream_t s) {
  PSX_LIVE();
  check(need().broadcast(send, recv, count, dt(dtype), root, PSX_COMM, s), "broadcast");
}
void RcclComm::reduce_scatter(const void* send, void* recv, size_t recvcount, int dtype, hipStream_t s) {
  PSX_LIVE();
  check(need().reduce_scatter(send, recv, recvcount, dt(dtype), ncclSum, PSX_COMM, s), "reduce_scatter");
}
void RcclComm::all_gather(const void* send, void* recv, size_t sendcount, int dtype, hipStream_t s) {
  PSX_LIVE();
  check(need().all_gather(send, recv, sendcount, dt(dtype), PSX_COMM, s), "all_gather");
}
void RcclComm::send(const void* buf, size_t count, int dtype, int peer, hipStream_t s) {
  PSX_LIVE();
  check(need().send(buf, count, dt(dtype), peer, PSX_COMM, s), "send");
}
void RcclComm::recv(void* buf, size_t count, int dtype, int peer, hipStream_t s) {
  PSX_LIVE();
  check(need().recv(buf, count, dt(dtype), peer, PSX_COMM, s), "recv");
}
void RcclComm::group_start() { check(need().group_start(), "group start"); }
void RcclComm::group_end() { check(need().group_end(), "group end"); }

}  // namespace psx
