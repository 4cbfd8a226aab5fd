// Same-device multi-process transport (see ipc_comm.h).
#include "ipc_comm.h"

#include <cstring>
#include <stdexcept>

namespace psx {
namespace {

void ck(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("IpcComm: ") + what + ": " + hipGetErrorString(e));
}

// dst[i] = sum over ranks r (in rank order) of src[r][i]
template <typename T>
__global__ void ipc_sum_kernel(const T* const* __restrict__ src, int n, T* __restrict__ dst, size_t count) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += (size_t)gridDim.x * blockDim.x) {
    T v = src[0][i];
    for (int r = 1; r < n; ++r) v += src[r][i];
    dst[i] = v;
  }
}

size_t elem_bytes(int dtype) {
  switch (dtype) {
    case Comm::kF32:
    case Comm::kI32: return 4;
    case Comm::kU8: return 1;
  }
  throw std::invalid_argument("IpcComm: unsupported dtype");
}

}  // namespace

IpcComm::IpcComm(int nranks, int rank, int device, size_t max_bytes)
    : nranks_(nranks), rank_(rank), max_((max_bytes + 255) / 256 * 256) {
  if (nranks < 1 || rank < 0 || rank >= nranks) throw std::invalid_argument("IpcComm: bad rank / size");
  ck(hipSetDevice(device), "hipSetDevice");
  ck(hipMalloc((void**)&own_, kFlagBytes + 2 * max_), "hipMalloc(area)");
  ck(hipMemset(own_, 0, kFlagBytes + 2 * max_), "hipMemset(area)");
  ck(hipMalloc(&srcs_dev_, 2 * (size_t)nranks * sizeof(void*)), "hipMalloc(sources)");
  ck(hipDeviceSynchronize(), "sync");
  base_.assign(nranks, nullptr);
  base_[rank] = own_;
}

IpcComm::~IpcComm() {
  try {
    close();
  } catch (...) {
  }
  if (srcs_dev_) (void)hipFree(srcs_dev_);
  if (own_) (void)hipFree(own_);
}

std::string IpcComm::handle() const {
  hipIpcMemHandle_t h;
  ck(hipIpcGetMemHandle(&h, own_), "hipIpcGetMemHandle");
  return std::string(reinterpret_cast<const char*>(&h), sizeof(h));
}

void IpcComm::connect(const std::vector<std::string>& handles) {
  if ((int)handles.size() != nranks_) throw std::invalid_argument("IpcComm::connect: one handle per rank");
  for (int r = 0; r < nranks_; ++r) {
    if (r == rank_) continue;
    if (handles[r].size() != sizeof(hipIpcMemHandle_t)) throw std::invalid_argument("IpcComm::connect: bad handle");
    hipIpcMemHandle_t h;
    std::memcpy(&h, handles[r].data(), sizeof(h));
    void* p = nullptr;
    ck(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
    base_[r] = static_cast<char*>(p);
  }
  std::vector<void*> srcs(2 * (size_t)nranks_);
  for (int q = 0; q < 2; ++q)
    for (int r = 0; r < nranks_; ++r) srcs[(size_t)q * nranks_ + r] = box(r, (uint64_t)q);
  ck(hipMemcpy(srcs_dev_, srcs.data(), srcs.size() * sizeof(void*), hipMemcpyHostToDevice), "sources upload");
  connected_ = true;
}

void IpcComm::close() {
  if (!connected_) return;
  connected_ = false;
  (void)hipDeviceSynchronize();
  for (int r = 0; r < nranks_; ++r)
    if (r != rank_ && base_[r]) {
      (void)hipIpcCloseMemHandle(base_[r]);
      base_[r] = nullptr;
    }
}

void IpcComm::live() const {
  if (!connected_) throw std::runtime_error("IpcComm used before connect() / after close()");
}

void IpcComm::wait_posted(int r, uint64_t q, hipStream_t s) {
  ck(hipStreamWaitValue64(s, posted(r), q, hipStreamWaitValueGte, ~0ull), "wait posted");
}

void IpcComm::post(const void* src, size_t bytes, uint64_t q, hipStream_t s) {
  if (bytes > max_) throw std::invalid_argument("IpcComm: contribution larger than the staging box");
  if (q > 2)  // the box of this parity was read by the peers' collective q - 2
    for (int r = 0; r < nranks_; ++r)
      if (r != rank_) ck(hipStreamWaitValue64(s, consumed(r), q - 2, hipStreamWaitValueGte, ~0ull), "wait consumed");
  ck(hipMemcpyAsync(box(rank_, q), src, bytes, hipMemcpyDeviceToDevice, s), "stage contribution");
  ck(hipStreamWriteValue64(s, posted(rank_), q, 0), "post");
}

void IpcComm::finish(uint64_t q, hipStream_t s) { ck(hipStreamWriteValue64(s, consumed(rank_), q, 0), "consumed"); }

void IpcComm::sum(void* dst, size_t count, int dtype, uint64_t q, hipStream_t s) {
  const int grid = (int)((count + 255) / 256 < 64 ? (count + 255) / 256 : 64);
  void* const* srcs = static_cast<void* const*>(srcs_dev_) + (q & 1) * nranks_;
  if (dtype == kF32)
    ipc_sum_kernel<float><<<grid > 0 ? grid : 1, 256, 0, s>>>((const float* const*)srcs, nranks_, (float*)dst, count);
  else if (dtype == kI32)
    ipc_sum_kernel<int><<<grid > 0 ? grid : 1, 256, 0, s>>>((const int* const*)srcs, nranks_, (int*)dst, count);
  else
    throw std::invalid_argument("IpcComm: sums of float / int32 only");
  ck(hipGetLastError(), "sum launch");
}

void IpcComm::all_reduce(const void* send, void* recv, size_t count, int dtype, hipStream_t s) {
  live();
  const uint64_t q = ++seq_;
  post(send, count * elem_bytes(dtype), q, s);
  for (int r = 0; r < nranks_; ++r)
    if (r != rank_) wait_posted(r, q, s);
  sum(recv, count, dtype, q, s);
  finish(q, s);
}

void IpcComm::reduce(const void* send, void* recv, size_t count, int dtype, int root, hipStream_t s) {
  live();
  const uint64_t q = ++seq_;
  post(send, count * elem_bytes(dtype), q, s);
  if (rank_ == root) {
    for (int r = 0; r < nranks_; ++r)
      if (r != rank_) wait_posted(r, q, s);
    sum(recv, count, dtype, q, s);
  }
  finish(q, s);
}

void IpcComm::broadcast(const void* send, void* recv, size_t count, int dtype, int root, hipStream_t s) {
  live();
  const uint64_t q = ++seq_;
  const size_t bytes = count * elem_bytes(dtype);
  if (rank_ == root) {
    post(send, bytes, q, s);
    if (recv != send) ck(hipMemcpyAsync(recv, send, bytes, hipMemcpyDeviceToDevice, s), "broadcast copy");
  } else {
    wait_posted(root, q, s);
    ck(hipMemcpyAsync(recv, box(root, q), bytes, hipMemcpyDeviceToDevice, s), "broadcast receive");
  }
  finish(q, s);
}

}  // namespace psx
