// Probe of the peer-mapped data plane (csrc/comm/peer_bus.h) on one GPU: two
// processes exchange 16 KB messages through HIP IPC mappings of each other's
// device memory, with system-scope stores / loads and a tag word per message.
//
//   build: hipcc -O3 --offload-arch=gfx950 tools/peer_probe.hip -o tools/peer_probe
//   run:   ./tools/peer_probe [iters]      (JSON on stdout)
//
// For each allocation flavour (hipMalloc, fine-grained, uncached) the parent
// exports a region, the child maps it (hipIpcOpenMemHandle) and exports its
// own; then a one-workgroup kernel in each process ping-pongs `iters` messages:
// the parent writes payload i + tag i into the child's region, the child checks
// the payload, answers into the parent's region.  Reported: whether IPC export
// / open works per flavour, payload errors, spin timeouts and the round-trip
// time (s_memrealtime, 100 MHz).  Every wait is bounded.
#include <hip/hip_runtime.h>
#include <sys/wait.h>
#include <unistd.h>

#include <cstdio>
#include <cstring>
#include <string>

#define CK(x)                                                                             \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) {                                                               \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      return 2;                                                                           \
    }                                                                                     \
  } while (0)

typedef __attribute__((address_space(1))) unsigned g_u32;
constexpr int kWords = 4096;  // 16 KB payload
constexpr int kSpin = 1 << 22;

__device__ __forceinline__ unsigned ld_sys(const unsigned* p) {
  return __hip_atomic_load((g_u32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys(unsigned* p, unsigned v) {
  __hip_atomic_store((g_u32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// region layout: [0] tag, [64 ..) payload
// role 0 (parent): send i -> wait answer i; role 1 (child): wait i -> check -> answer i
__global__ void pingpong(unsigned* mine, unsigned* peer, int iters, int role, unsigned* out) {
  __shared__ int ok_s;
  unsigned errs = 0, timeouts = 0;
  long long t0 = 0, t1 = 0;
  for (int i = 1; i <= iters; ++i) {
    if (role == 0) {
      if (i == 2) t0 = __builtin_amdgcn_s_memrealtime();
      for (int w = threadIdx.x; w < kWords; w += blockDim.x) st_sys(peer + 64 + w, (unsigned)i * 7919u + (unsigned)w);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        st_sys(peer, (unsigned)i);
      }
    }
    if (threadIdx.x == 0) {  // wait for message i in my region
      int s = 0;
      while (ld_sys(mine) < (unsigned)i && ++s < kSpin) __builtin_amdgcn_s_sleep(1);
      ok_s = s < kSpin;
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    }
    __syncthreads();
    if (!ok_s) {
      ++timeouts;
      break;
    }
    const unsigned salt = role == 0 ? 104729u : 7919u;
    for (int w = threadIdx.x; w < kWords; w += blockDim.x)
      errs += ld_sys(mine + 64 + w) != (unsigned)i * salt + (unsigned)w;
    if (role == 1) {
      for (int w = threadIdx.x; w < kWords; w += blockDim.x) st_sys(peer + 64 + w, (unsigned)i * 104729u + (unsigned)w);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        st_sys(peer, (unsigned)i);
      }
    }
    __syncthreads();
  }
  t1 = __builtin_amdgcn_s_memrealtime();
  atomicAdd(out + 0, errs);
  if (threadIdx.x == 0) {
    out[1] = timeouts;
    *(long long*)(out + 2) = t1 - t0;
  }
}

static int alloc(int flavour, void** p, size_t bytes) {
  if (flavour == 0) return hipMalloc(p, bytes) == hipSuccess ? 0 : 1;
  const unsigned fl = flavour == 1 ? hipDeviceMallocFinegrained : hipDeviceMallocUncached;
  return hipExtMallocWithFlags(p, bytes, fl) == hipSuccess ? 0 : 1;
}

static bool rd(int fd, void* b, size_t n) {
  char* c = (char*)b;
  while (n) {
    ssize_t k = read(fd, c, n);
    if (k <= 0) return false;
    c += k;
    n -= (size_t)k;
  }
  return true;
}
static bool wr(int fd, const void* b, size_t n) {
  const char* c = (const char*)b;
  while (n) {
    ssize_t k = write(fd, c, n);
    if (k <= 0) return false;
    c += k;
    n -= (size_t)k;
  }
  return true;
}

// one flavour, one side.  to / from: pipes.  Returns 0 and fills res.
struct Res {
  int alloc_rc, export_rc, open_rc;
  unsigned errs, timeouts;
  long long ticks;
};

static int side(int role, int flavour, int iters, int to, int from, Res* res) {
  memset(res, 0, sizeof(*res));
  const size_t bytes = (64 + kWords) * 4;
  void* mine = nullptr;
  res->alloc_rc = alloc(flavour, &mine, bytes);
  hipIpcMemHandle_t h{};
  if (!res->alloc_rc) {
    CK(hipMemset(mine, 0, bytes));
    CK(hipDeviceSynchronize());
    res->export_rc = hipIpcGetMemHandle(&h, mine) == hipSuccess ? 0 : 1;
  }
  int okme = !res->alloc_rc && !res->export_rc, okpeer = 0;
  hipIpcMemHandle_t ph{};
  if (!wr(to, &okme, sizeof(okme)) || !wr(to, &h, sizeof(h))) return 3;
  if (!rd(from, &okpeer, sizeof(okpeer)) || !rd(from, &ph, sizeof(ph))) return 3;
  void* peer = nullptr;
  if (okme && okpeer) res->open_rc = hipIpcOpenMemHandle(&peer, ph, hipIpcMemLazyEnablePeerAccess) == hipSuccess ? 0 : 1;
  else res->open_rc = -1;
  int go = res->open_rc == 0, pgo = 0;
  if (!wr(to, &go, sizeof(go)) || !rd(from, &pgo, sizeof(pgo))) return 3;
  if (go && pgo) {
    unsigned* out = nullptr;
    CK(hipMalloc(&out, 64));
    CK(hipMemset(out, 0, 64));
    hipLaunchKernelGGL(pingpong, dim3(1), dim3(256), 0, 0, (unsigned*)mine, (unsigned*)peer, iters, role, out);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    unsigned o[4];
    CK(hipMemcpy(o, out, 16, hipMemcpyDeviceToHost));
    res->errs = o[0];
    res->timeouts = o[1];
    memcpy(&res->ticks, o + 2, 8);
    CK(hipFree(out));
    int done = 1, pdone = 0;
    if (!wr(to, &done, sizeof(done)) || !rd(from, &pdone, sizeof(pdone))) return 3;
  }
  if (peer) (void)hipIpcCloseMemHandle(peer);
  int fin = 1, pfin = 0;
  if (!wr(to, &fin, sizeof(fin)) || !rd(from, &pfin, sizeof(pfin))) return 3;
  if (mine) (void)hipFree(mine);
  return 0;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 2000;
  int p2c[2], c2p[2], res_pipe[2];
  if (pipe(p2c) || pipe(c2p) || pipe(res_pipe)) return 4;
  const pid_t pid = fork();  // before any HIP call
  if (pid < 0) return 4;
  const int role = pid == 0 ? 1 : 0;
  const int to = role == 0 ? p2c[1] : c2p[1], from = role == 0 ? c2p[0] : p2c[0];
  if (hipSetDevice(0) != hipSuccess) return 5;
  Res r[3];
  int rc = 0;
  for (int f = 0; f < 3 && rc == 0; ++f) rc = side(role, f, iters, to, from, &r[f]);
  if (role == 1) {
    (void)wr(res_pipe[1], r, sizeof(r));
    _exit(rc);
  }
  Res cr[3];
  memset(cr, 0, sizeof(cr));
  const bool got = rd(res_pipe[0], cr, sizeof(cr));
  int st = 0;
  waitpid(pid, &st, 0);
  const char* names[3] = {"hipMalloc", "finegrained", "uncached"};
  printf("{\"iters\": %d, \"rc\": %d, \"child_status\": %d, \"flavours\": {", iters, rc, st);
  for (int f = 0; f < 3; ++f) {
    const double us = r[f].ticks > 0 ? r[f].ticks / 100.0 / (iters - 1) : -1.0;
    printf("%s\"%s\": {\"alloc\": %d, \"export\": %d, \"open\": %d, \"errs\": %u, \"timeouts\": %u, "
           "\"child_errs\": %u, \"child_timeouts\": %u, \"round_trip_us\": %.3f}",
           f ? ", " : "", names[f], r[f].alloc_rc, r[f].export_rc, r[f].open_rc, r[f].errs, r[f].timeouts,
           got ? cr[f].errs : 999u, got ? cr[f].timeouts : 999u, us);
  }
  printf("}}\n");
  return rc;
}
