// XCD probe (MI355X): where do a launch's workgroups land, and what does a
// grid-wide hand-off cost when every participant shares one XCD's L2 instead
// of being spread over the 8 XCDs?
//
//   1. map: blockIdx -> XCC_ID (hwreg) for a 2048-workgroup launch.
//   2. barrier: NG workgroups run R rounds of {store a word per thread, drain,
//      arrive on a counter, spin, read a neighbour's words and check them}.
//        spread/agent : blockIdx 0..NG-1 (all XCDs), sc1 stores / loads, agent atomics
//        xcd/l2       : blockIdx 8*i (one XCD), plain stores, sc0 loads (L1 bypass,
//                       L2 hit), workgroup-scope atomics (executed in that L2)
//   3. load: 2 MB read by 32 workgroups on one XCD vs 32 spread vs 256 spread.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/xcd_probe tools/xcd_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                \
    }                                                                              \
  } while (0)

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) unsigned long long g_u64;

__device__ __forceinline__ unsigned xcc_id() { return __builtin_amdgcn_s_getreg((3 << 11) | 20) & 15u; }
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* b, unsigned n) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(b), (short)0, (int)n, 0x00020000);
}

__global__ void map_kernel(unsigned* out) {
  if (threadIdx.x == 0) out[blockIdx.x] = xcc_id();
}

// mode 0: spread, agent atomic counter, sc1 polling
// mode 1: one XCD, flag array (plain stores -> L2), sc0 polling (L1 bypass, L2 hit)
// mode 2: spread, flag array, sc1 stores + sc1 polling
// mode 3: one XCD, agent atomic counter, sc1 polling
template <int MODE>
__global__ __launch_bounds__(256) void barrier_kernel(unsigned long long* ctr, unsigned* flags, unsigned* data, int NG,
                                                      int R, unsigned* errs, long long* t, unsigned* xccs) {
  constexpr bool one = MODE == 1 || MODE == 3 || MODE >= 4;
  int wg;
  if (!one) {
    if ((int)blockIdx.x >= NG) return;
    wg = blockIdx.x;
  } else {
    if (blockIdx.x % 8 != 0 || (int)blockIdx.x / 8 >= NG) return;
    wg = blockIdx.x / 8;
  }
  if (threadIdx.x == 0) xccs[wg] = xcc_id();
  const auto rd = rsrc(data, (unsigned)(NG * 2 * 256 * 4));
  const auto rf = rsrc(flags, (unsigned)(NG * 64 * 4));  // one 256-B line per workgroup's flag
  // loads: sc0 (1, 4) | nt (5) | sc1;  stores: plain (1, 5) | sc0 (4) | sc1
  const int laux = (MODE == 1 || MODE == 4) ? 1 : MODE == 5 ? 2 : 16;
  const int saux = (MODE == 1 || MODE == 5) ? 0 : MODE == 4 ? 1 : 16;
  unsigned bad = 0;
  __shared__ int quit;
  if (threadIdx.x == 0) quit = 0;
  __syncthreads();
  int total = 0;  // spins over the whole run: a hand-off that never becomes visible ends the run
  long long t0 = wall_clock64();
  for (int r = 0; r < R; ++r) {
    const unsigned v = (unsigned)(r * 4096 + wg);
    const unsigned off = (unsigned)((((r & 1) * NG + wg) * 256 + threadIdx.x) * 4);
    __builtin_amdgcn_raw_buffer_store_b32(v, rd, (int)off, 0, saux);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (MODE == 0 || MODE == 3) {
      if (threadIdx.x == 0) {
        const unsigned long long target = (unsigned long long)NG * (r + 1);
        (void)__hip_atomic_fetch_add((g_u64*)ctr, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        while (__hip_atomic_load((g_u64*)ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
          if (++total > (1 << 20)) {
            quit = 1;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
      }
    } else {
      if (threadIdx.x == 0) __builtin_amdgcn_raw_buffer_store_b32((unsigned)(r + 1), rf, wg * 256, 0, saux);
      if ((int)threadIdx.x < NG) {  // thread i waits for workgroup i's flag
        while (true) {
          const unsigned f = __builtin_amdgcn_raw_buffer_load_b32(rf, (int)threadIdx.x * 256, 0, laux);
          if (f >= (unsigned)(r + 1)) break;
          if (++total > (1 << 20)) {
            quit = 1;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
      }
    }
    __syncthreads();
    if (quit) {
      bad += 1000000;
      break;
    }
    const int nb = (wg + 1) % NG;
    const unsigned noff = (unsigned)((((r & 1) * NG + nb) * 256 + threadIdx.x) * 4);
    const unsigned got = __builtin_amdgcn_raw_buffer_load_b32(rd, (int)noff, 0, laux);
    if (got != (unsigned)(r * 4096 + nb)) ++bad;
  }
  long long t1 = wall_clock64();
  if (bad) atomicAdd(errs, bad);
  if (wg == 0 && threadIdx.x == 0) t[0] = t1 - t0;
}

// every participating workgroup reads its share of a 2 MB region (16-B loads, all in flight)
template <int MODE>
__global__ __launch_bounds__(256) void load_kernel(const u32x4* src, int NG, u32x4* sink) {
  int wg;
  if (MODE == 1) {
    if (blockIdx.x % 8 != 0 || (int)blockIdx.x / 8 >= NG) return;
    wg = blockIdx.x / 8;
  } else {
    if ((int)blockIdx.x >= NG) return;
    wg = blockIdx.x;
  }
  const int per = (2 << 20) / 16 / NG;  // 16-B pieces per workgroup
  const u32x4* p = src + (size_t)wg * per;
  u32x4 acc = {0, 0, 0, 0};
  constexpr int U = 16;
  for (int i = threadIdx.x; i < per; i += 256 * U) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = i + 256 * u < per ? p[i + 256 * u] : u32x4{0, 0, 0, 0};
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u];
  }
  if (acc[0] == 0x12345678u) sink[threadIdx.x] = acc;
}

int main() {
  int dev = 0;
  CK(hipSetDevice(dev));
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, dev));
  std::printf("device %s CUs %d\n", prop.gcnArchName, prop.multiProcessorCount);
  // 1. map
  const int NM = 2048;
  unsigned* dmap;
  CK(hipMalloc(&dmap, NM * 4));
  std::vector<unsigned> hmap(NM);
  bool rr = true;
  for (int rep = 0; rep < 3; ++rep) {
    map_kernel<<<NM, 64>>>(dmap);
    CK(hipMemcpy(hmap.data(), dmap, NM * 4, hipMemcpyDeviceToHost));
    for (int b = 0; b < NM; ++b) rr = rr && hmap[b] == (unsigned)(b % 8);
  }
  std::printf("map: blockIdx %% 8 == XCC_ID for all %d workgroups x 3 launches: %s (first 16:", NM, rr ? "yes" : "NO");
  for (int b = 0; b < 16; ++b) std::printf(" %u", hmap[b]);
  std::printf(")\n");
  // 2. barrier
  unsigned long long* ctr;
  unsigned *data, *errs, *xccs, *flags;
  long long* t;
  CK(hipMalloc(&ctr, 64));
  CK(hipMalloc(&flags, 64 * 256));
  CK(hipMalloc(&data, 64 * 2 * 256 * 4));
  CK(hipMalloc(&errs, 4));
  CK(hipMalloc(&xccs, 64 * 4));
  CK(hipMalloc(&t, 8));
  const int R = 500;
  const char* names[6] = {"spread/atomic", "xcd/flags-l2", "spread/flags", "xcd/atomic", "xcd/flags-sc0", "xcd/flags-nt"};
  for (int NG : {8, 32}) {
    for (int mode = 0; mode < 6; ++mode) {
      for (int rep = 0; rep < 2; ++rep) {
        CK(hipMemset(ctr, 0, 64));
        CK(hipMemset(flags, 0, 64 * 256));
        CK(hipMemset(errs, 0, 4));
        CK(hipMemset(xccs, 0xff, 64 * 4));
        CK(hipDeviceSynchronize());
        switch (mode) {
          case 0: barrier_kernel<0><<<NG, 256>>>(ctr, flags, data, NG, R, errs, t, xccs); break;
          case 1: barrier_kernel<1><<<8 * NG, 256>>>(ctr, flags, data, NG, R, errs, t, xccs); break;
          case 2: barrier_kernel<2><<<NG, 256>>>(ctr, flags, data, NG, R, errs, t, xccs); break;
          case 3: barrier_kernel<3><<<8 * NG, 256>>>(ctr, flags, data, NG, R, errs, t, xccs); break;
          case 4: barrier_kernel<4><<<8 * NG, 256>>>(ctr, flags, data, NG, R, errs, t, xccs); break;
          default: barrier_kernel<5><<<8 * NG, 256>>>(ctr, flags, data, NG, R, errs, t, xccs); break;
        }
        CK(hipDeviceSynchronize());
        long long ht;
        unsigned he;
        std::vector<unsigned> hx(NG);
        CK(hipMemcpy(&ht, t, 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(&he, errs, 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(hx.data(), xccs, NG * 4, hipMemcpyDeviceToHost));
        bool one = true;
        for (int i = 0; i < NG; ++i) one = one && hx[i] == hx[0];
        // wall_clock64 runs at 100 MHz on MI300-class parts
        std::printf("barrier %-14s NG=%2d rep %d: %.3f us per hand-off, %u stale reads, one XCD: %s\n", names[mode],
                    NG, rep, (double)ht * 10.0 / 1000.0 / R, he, one ? "yes" : "no");
      }
    }
  }
  // 3. load 2 MB: regions rotate over 256 MB so that no run starts warm in the L2s
  const size_t region = 2 << 20, nreg = 128;
  u32x4* src;
  u32x4* sink;
  CK(hipMalloc(&src, region * nreg));
  CK(hipMemset(src, 1, region * nreg));
  CK(hipMalloc(&sink, 256 * 16));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  struct Cfg {
    const char* name;
    int mode, NG, grid;
  } cfgs[] = {{"32 WG one XCD", 1, 32, 256}, {"32 WG spread", 0, 32, 32}, {"256 WG spread", 0, 256, 256},
              {"64 WG one XCD", 1, 64, 512}};
  for (auto& c : cfgs) {
    const int N = 512;
    for (int warm = 0; warm < 2; ++warm) {
      CK(hipEventRecord(e0));
      for (int i = 0; i < N; ++i) {
        const u32x4* s = src + (size_t)(i % nreg) * (region / 16);
        if (c.mode == 1)
          load_kernel<1><<<c.grid, 256>>>(s, c.NG, sink);
        else
          load_kernel<0><<<c.grid, 256>>>(s, c.NG, sink);
      }
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (warm) std::printf("load 2 MB %-14s: %.2f us per launch (back to back)\n", c.name, ms * 1000.f / N);
    }
  }
  return 0;
}
