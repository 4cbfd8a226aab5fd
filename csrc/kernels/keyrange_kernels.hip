// Key-range shard gather / apply (see keyrange_kernels.h).  Both are pure
// bandwidth: one thread per (feature, class) element, consecutive threads on
// consecutive classes of a feature so a KP-wide row is one contiguous access.
#include <hip/hip_runtime.h>

#include "keyrange_kernels.h"

namespace psx {

namespace {

__global__ __launch_bounds__(256) void kr_gather_kernel(const float* __restrict__ shard, int64_t lo, int KP,
                                                        const int32_t* __restrict__ ids, const unsigned* n_dev,
                                                        int n_host, float* __restrict__ out) {
  const int64_t n = n_dev ? (int64_t)*n_dev : (int64_t)n_host;
  const int64_t tot = n * KP;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < tot; e += (int64_t)gridDim.x * 256) {
    const int64_t i = e / KP, c = e - i * KP;
    out[e] = shard[((int64_t)ids[i] - lo) * KP + c];
  }
}

__global__ __launch_bounds__(256) void kr_apply_kernel(float* __restrict__ shard, int64_t lo, int KP,
                                                       const int32_t* __restrict__ ids, const unsigned* n_dev,
                                                       int n_host, const float* __restrict__ vals, float lr,
                                                       float* __restrict__ b, const float* __restrict__ db) {
  const int64_t n = n_dev ? (int64_t)*n_dev : (int64_t)n_host;
  const int64_t tot = n * KP;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < tot; e += (int64_t)gridDim.x * 256) {
    const int64_t i = e / KP, c = e - i * KP;
    shard[((int64_t)ids[i] - lo) * KP + c] += lr * vals[e];
  }
  if (db && blockIdx.x == 0 && threadIdx.x < KP) b[threadIdx.x] += lr * db[threadIdx.x];
}

int kr_grid(int64_t elems) {
  int64_t g = (elems + 255) / 256;
  if (g < 1) g = 1;
  return g > 2048 ? 2048 : (int)g;
}

}  // namespace

void launch_kr_gather(const float* shard, int64_t lo, int KP, const int32_t* ids, const unsigned* n_dev, int n_host,
                      float* out, int nmax, hipStream_t s) {
  const int64_t n = n_dev ? nmax : n_host;
  if (n <= 0) return;
  kr_gather_kernel<<<kr_grid(n * KP), 256, 0, s>>>(shard, lo, KP, ids, n_dev, n_host, out);
}

void launch_kr_apply(float* shard, int64_t lo, int KP, const int32_t* ids, const unsigned* n_dev, int n_host,
                     const float* vals, float lr, float* b, const float* db, int nmax, hipStream_t s) {
  const int64_t n = n_dev ? nmax : n_host;
  if (n <= 0 && !db) return;
  kr_apply_kernel<<<kr_grid(n * KP), 256, 0, s>>>(shard, lo, KP, ids, n_dev, n_host, vals, lr, b, db);
}

}  // namespace psx
