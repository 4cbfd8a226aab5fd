// Does a persistent kernel on a stream of the greatest priority (or with a CU mask) get a
// hardware queue of its own, or does it share one with the process's normal streams?
// A kernel on stream S spins until a host flag is set (or 2 s pass); meanwhile a tiny
// kernel on each of 12 normal-priority streams writes its done word.  Every normal
// stream finishing before the flag is released = no normal stream shares S's queue.
//   hipcc --offload-arch=gfx950 -O2 tools/hwq_probe.hip -o tools/hwq_probe
//   ./tools/hwq_probe [normal|prio|cumask]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      std::printf("%s: %s\n", #x, hipGetErrorString(e_));                  \
      return 2;                                                            \
    }                                                                      \
  } while (0)

__global__ void spin_kernel(const volatile int* flag, int* out) {
  const long long t0 = __builtin_amdgcn_s_memrealtime();
  // every wave reaches the exit: the flag, or 2 s of the 100 MHz clock
  while (*flag == 0 && __builtin_amdgcn_s_memrealtime() - t0 < 200000000ll) __builtin_amdgcn_s_sleep(16);
  if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = 1;
}

__global__ void mark_kernel(int* done, int i) {
  if (threadIdx.x == 0) done[i] = 1;
}

int main(int argc, char** argv) {
  const char* mode = argc > 1 ? argv[1] : "prio";
  int lo = 0, hi = 0;
  CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
  hipStream_t s;
  if (!std::strcmp(mode, "prio")) {
    CK(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, hi));
  } else if (!std::strcmp(mode, "cumask")) {
    std::vector<uint32_t> m(8, 0xffffffffu);
    CK(hipExtStreamCreateWithCUMask(&s, (uint32_t)m.size(), m.data()));
  } else {
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  }
  const int N = 12;
  std::vector<hipStream_t> ns(N);
  for (int i = 0; i < N; ++i) CK(hipStreamCreateWithFlags(&ns[i], hipStreamNonBlocking));
  int* flag = nullptr;
  CK(hipHostMalloc((void**)&flag, 64, hipHostMallocCoherent));
  flag[0] = 0;
  int *done = nullptr, *out = nullptr;
  CK(hipHostMalloc((void**)&done, 4 * N, hipHostMallocCoherent));
  CK(hipMalloc((void**)&out, 64));
  std::memset(done, 0, 4 * N);
  spin_kernel<<<1, 64, 0, s>>>(flag, out);
  CK(hipGetLastError());
  std::this_thread::sleep_for(std::chrono::milliseconds(50));
  for (int i = 0; i < N; ++i) mark_kernel<<<1, 64, 0, ns[i]>>>(done, i);
  CK(hipGetLastError());
  std::this_thread::sleep_for(std::chrono::milliseconds(500));
  int fin = 0;
  std::printf("{\"mode\": \"%s\", \"priority_range\": [%d, %d], \"done_before_release\": [", mode, lo, hi);
  for (int i = 0; i < N; ++i) {
    const int d = __atomic_load_n(done + i, __ATOMIC_ACQUIRE);
    fin += d;
    std::printf("%s%d", i ? ", " : "", d);
  }
  __atomic_store_n(flag, 1, __ATOMIC_RELEASE);
  CK(hipDeviceSynchronize());
  std::printf("], \"all_free\": %s}\n", fin == N ? "true" : "false");
  return 0;
}
