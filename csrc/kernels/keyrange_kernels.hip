// Key-range shard gather / apply (see keyrange_kernels.h).  Both are pure
// bandwidth: one thread per (feature, class) element, consecutive threads on
// consecutive classes of a feature so a KP-wide row is one contiguous access.
#include <hip/hip_runtime.h>

#include "common.h"
#include "keyrange_kernels.h"
#include "wide_kernels.h"

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

// Confusion counts of this workgroup (LDS [256]) -> the private accumulators;
// the last workgroup of the launch publishes them into the pinned EvalSlot:
// drained system-scope stores, then the sequence number (the test_eval_kernel
// protocol).  Every thread of every workgroup calls it.
__device__ __forceinline__ void kr_publish(int* cl, int* acc, unsigned* ticket, char* slot, const float* loss,
                                           unsigned long long seq) {
  __shared__ int last;
  __syncthreads();
  const int tid = threadIdx.x;
  const int v = cl[tid];
  if (v) atomicAdd(acc + tid * kAccStride, v);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0)
    last = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
  __syncthreads();
  if (!last) return;
  const int tot = __hip_atomic_exchange(acc + tid * kAccStride, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store((int*)slot + tid, tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (tid == 0)
    __hip_atomic_store((float*)(slot + 1024), loss ? *loss : 0.f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store((unsigned long long*)(slot + 1032), seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

template <int KP>
__device__ __forceinline__ int kr_argmax(int K, const float (&z)[KP]) {
  if (K == 1) return z[0] > 0.f ? 1 : 0;
  int best = 0;
  float bz = -INFINITY;
#pragma unroll
  for (int k = 0; k < KP; ++k)
    if (k < K && z[k] > bz) {
      bz = z[k];
      best = k;
    }
  return best;
}

__device__ __forceinline__ int kr_label(int K, int y) {
  if (K == 1) y = y > 0 ? 1 : 0;
  return y < 0 ? 0 : (y > 15 ? 15 : y);
}

// 16 lanes per test row, 16 rows per workgroup pass; each lane keeps 4 entries'
// loads in flight (ids / values, then the table probes, then the deltas).
template <int KP>
__global__ __launch_bounds__(256) void kr_worker_rows_kernel(
    int K, const int64_t* __restrict__ indptr, const int32_t* __restrict__ idx, const uint16_t* __restrict__ val,
    const int32_t* __restrict__ y, int T, const float* __restrict__ z, const int2* __restrict__ htab, unsigned hmask,
    const float* __restrict__ dloc, const float* __restrict__ wloc_b, float* __restrict__ dz, int* acc,
    unsigned* ticket, char* slot, const float* loss, unsigned long long seq) {
  __shared__ int cl[256];
  const int tid = threadIdx.x, l = tid & 15;
  cl[tid] = 0;
  __syncthreads();
  float bv[KP];
#pragma unroll
  for (int k = 0; k < KP; ++k) bv[k] = wloc_b ? wloc_b[k] : 0.f;
  for (int64_t r0 = (int64_t)blockIdx.x * 16; r0 < T; r0 += (int64_t)gridDim.x * 16) {
    const int64_t r = r0 + (tid >> 4);
    float s[KP];
#pragma unroll
    for (int k = 0; k < KP; ++k) s[k] = 0.f;
    if (r < T && htab) {
      const int64_t a = indptr[r], b = indptr[r + 1];
      for (int64_t e0 = a + l; e0 < b; e0 += 64) {
        int f[4], li[4];
        float v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int64_t e = e0 + 16 * u;
          f[u] = e < b ? idx[e] : -1;
          v[u] = e < b ? bf2f(val[e]) : 0.f;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) li[u] = f[u] >= 0 ? wide_find(htab, hmask, f[u]) : -1;
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (li[u] >= 0) {
#pragma unroll
            for (int k = 0; k < KP; ++k) s[k] += v[u] * dloc[KP + (int64_t)li[u] * KP + k];
          }
      }
    }
#pragma unroll
    for (int k = 0; k < KP; ++k)
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) s[k] += __shfl_xor(s[k], o, 64);
    if (l == 0 && r < T) {
      float zw[KP];
#pragma unroll
      for (int k = 0; k < KP; ++k) {
        dz[r * KP + k] = s[k];
        zw[k] = z[r * KP + k] + s[k] + bv[k];
      }
      if (slot) atomicAdd(&cl[kr_label(K, y[r]) * 16 + kr_argmax<KP>(K, zw)], 1);
    }
  }
  if (slot) kr_publish(cl, acc, ticket, slot, loss, seq);
}

template <int KP>
__global__ __launch_bounds__(256) void kr_server_rows_kernel(int K, const int32_t* __restrict__ y, int T,
                                                             float* __restrict__ z, const float* __restrict__ dz,
                                                             float lr, const float* __restrict__ b, int* acc,
                                                             unsigned* ticket, char* slot, unsigned long long seq) {
  __shared__ int cl[256];
  const int tid = threadIdx.x;
  cl[tid] = 0;
  __syncthreads();
  float bv[KP];
#pragma unroll
  for (int k = 0; k < KP; ++k) bv[k] = b[k];
  for (int64_t r = (int64_t)blockIdx.x * 256 + tid; r < T; r += (int64_t)gridDim.x * 256) {
    float zs[KP];
#pragma unroll
    for (int k = 0; k < KP; ++k) {
      const float zn = z[r * KP + k] + lr * dz[r * KP + k];
      z[r * KP + k] = zn;
      zs[k] = zn + bv[k];
    }
    if (slot) atomicAdd(&cl[kr_label(K, y[r]) * 16 + kr_argmax<KP>(K, zs)], 1);
  }
  if (slot) kr_publish(cl, acc, ticket, slot, nullptr, seq);
}

}  // namespace

void launch_kr_worker_rows(int K, int KP, const int64_t* indptr, const int32_t* idx, const uint16_t* val,
                           const int32_t* y, int T, const float* z, const int2* htab, unsigned hmask,
                           const float* dloc, const float* wloc_b, float* dz, int* acc, unsigned* ticket, void* slot,
                           const float* loss, unsigned long long seq, hipStream_t s) {
  if (T <= 0) return;
  const int grid = kr_grid((int64_t)T * 16);
  char* sl = static_cast<char*>(slot);
  switch (KP) {
    case 1: kr_worker_rows_kernel<1><<<grid, 256, 0, s>>>(K, indptr, idx, val, y, T, z, htab, hmask, dloc, wloc_b, dz, acc, ticket, sl, loss, seq); break;
    case 2: kr_worker_rows_kernel<2><<<grid, 256, 0, s>>>(K, indptr, idx, val, y, T, z, htab, hmask, dloc, wloc_b, dz, acc, ticket, sl, loss, seq); break;
    case 4: kr_worker_rows_kernel<4><<<grid, 256, 0, s>>>(K, indptr, idx, val, y, T, z, htab, hmask, dloc, wloc_b, dz, acc, ticket, sl, loss, seq); break;
    case 8: kr_worker_rows_kernel<8><<<grid, 256, 0, s>>>(K, indptr, idx, val, y, T, z, htab, hmask, dloc, wloc_b, dz, acc, ticket, sl, loss, seq); break;
    default: kr_worker_rows_kernel<16><<<grid, 256, 0, s>>>(K, indptr, idx, val, y, T, z, htab, hmask, dloc, wloc_b, dz, acc, ticket, sl, loss, seq); break;
  }
}

void launch_kr_server_rows(int K, int KP, const int32_t* y, int T, float* z, const float* dz, float lr, const float* b,
                           int* acc, unsigned* ticket, void* slot, unsigned long long seq, hipStream_t s) {
  if (T <= 0) return;
  const int grid = kr_grid(T) < 256 ? kr_grid(T) : 256;
  char* sl = static_cast<char*>(slot);
  switch (KP) {
    case 1: kr_server_rows_kernel<1><<<grid, 256, 0, s>>>(K, y, T, z, dz, lr, b, acc, ticket, sl, seq); break;
    case 2: kr_server_rows_kernel<2><<<grid, 256, 0, s>>>(K, y, T, z, dz, lr, b, acc, ticket, sl, seq); break;
    case 4: kr_server_rows_kernel<4><<<grid, 256, 0, s>>>(K, y, T, z, dz, lr, b, acc, ticket, sl, seq); break;
    case 8: kr_server_rows_kernel<8><<<grid, 256, 0, s>>>(K, y, T, z, dz, lr, b, acc, ticket, sl, seq); break;
    default: kr_server_rows_kernel<16><<<grid, 256, 0, s>>>(K, y, T, z, dz, lr, b, acc, ticket, sl, seq); break;
  }
}

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
