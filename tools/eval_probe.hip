// Device time of the riders' test-set evaluation, standalone (one MI355X): the
// pair-major riders (lanes_detail::eval_multi_body, the round-3 form) against the
// tile-resident riders (lanes_detail::eval_tile_body), 9 models (8 local + the
// global one, K = 6) over the 4,877 x 1,024 test set.  Checks that both publish
// the same counts into the slots, then times each form over `reps` launches.
//
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -munsafe-fp-atomics -I csrc/kernels \
//     tools/eval_probe.hip -o tools/eval_probe && ./tools/eval_probe [reps]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "lanes_body.h"

using namespace psx;
using namespace psx::lanes_detail;

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                        \
    }                                                                                      \
  } while (0)

constexpr int FP = 1024;

__global__ __launch_bounds__(256) void pair_major_kernel(EvalMulti ev, int nride) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  eval_multi_body<FP>(lds, ev, (int)blockIdx.x, nride);
}

// q != nullptr: the tiles popped from q[32 * par] (cleared for the other parity, as the
// round kernel's claim counters)
template <int kStop = 3>
__global__ __launch_bounds__(256) void tile_resident_kernel(EvalMulti ev, int nride, unsigned* q, int par) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  if (q && blockIdx.x == 0 && threadIdx.x == 0) q[32 * (par ^ 1)] = 0u;
  ev.xq = q ? q + 32 * par : nullptr;
  eval_tile_body<FP, kStop>(lds, ev, (int)blockIdx.x, nride);
}

__global__ __launch_bounds__(256) void empty_kernel(EvalMulti ev, int nride) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  if (threadIdx.x == 0 && ev.nmodels < 0) lds[0] = (char)nride;  // (never: keeps the arguments live)
}

// the flush alone: every workgroup adds its (here: constant) counts into the shared
// accumulators and arrives on the ticket, as a rider's tail does
__global__ __launch_bounds__(256) void flush_only_kernel(EvalMulti ev, int nride) {
  const int tid = threadIdx.x;
  for (int m = 0; m < ev.nmodels; ++m)
    if ((tid & 15) < ev.K && (tid >> 4) < ev.K) atomicAdd(acc_cell(ev.acc, xcd_copy(), m, tid), 1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) (void)__hip_atomic_fetch_add(ev.ticket + 8, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// the ticket alone: one device-scope atomic per workgroup on one address
__global__ __launch_bounds__(256) void ticket_only_kernel(EvalMulti ev, int nride) {
  if (threadIdx.x == 0) (void)__hip_atomic_fetch_add(ev.ticket + 8, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

static uint16_t bf16_bits(float v) {
  uint32_t u;
  std::memcpy(&u, &v, 4);
  return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? std::atoi(argv[1]) : 200;
  const int T = 4877, K = 6, M = 9;
  std::mt19937 rng(1);
  std::normal_distribution<float> nd(0.f, 1.f);
  std::vector<uint16_t> X((size_t)T * FP);
  for (auto& v : X) v = bf16_bits(nd(rng) * 0.05f);
  std::vector<int32_t> y(T);
  for (auto& v : y) v = 1 + (int)(rng() % 5);
  uint16_t* dX;
  int32_t* dy;
  CK(hipMalloc(&dX, X.size() * 2));
  CK(hipMalloc(&dy, T * 4));
  CK(hipMemcpy(dX, X.data(), X.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dy, y.data(), T * 4, hipMemcpyHostToDevice));
  // model m: fragments [FP/8][16][8] (hi, lo), class columns 0..K-1, intercepts [16]
  const size_t fr = (size_t)FP / 8 * 16 * 8;
  std::vector<uint16_t*> hi(M), lo(M);
  std::vector<float*> b(M);
  for (int m = 0; m < M; ++m) {
    std::vector<uint16_t> h(fr, 0), l(fr, 0);
    for (int g = 0; g < FP / 8; ++g)
      for (int c = 0; c < K; ++c)
        for (int e = 0; e < 8; ++e) {
          const float wv = nd(rng);
          const uint16_t hb = bf16_bits(wv);
          uint32_t hu = (uint32_t)hb << 16;
          float hf;
          std::memcpy(&hf, &hu, 4);
          h[((size_t)g * 16 + c) * 8 + e] = hb;
          l[((size_t)g * 16 + c) * 8 + e] = bf16_bits(wv - hf);
        }
    std::vector<float> bb(16, 0.f);
    for (int c = 0; c < K; ++c) bb[c] = nd(rng) * 0.1f;
    CK(hipMalloc(&hi[m], fr * 2));
    CK(hipMalloc(&lo[m], fr * 2));
    CK(hipMalloc(&b[m], 64));
    CK(hipMemcpy(hi[m], h.data(), fr * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(lo[m], l.data(), fr * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(b[m], bb.data(), 64, hipMemcpyHostToDevice));
  }
  int* acc;
  unsigned* ticket;
  CK(hipMalloc(&acc, kEvalAccInts * 4));
  CK(hipMalloc(&ticket, 64));
  CK(hipMemset(acc, 0, kEvalAccInts * 4));
  CK(hipMemset(ticket, 0, 64));
  unsigned* q;
  CK(hipMalloc(&q, 64 * 4));
  CK(hipMemset(q, 0, 64 * 4));
  char* slots;
  CK(hipHostMalloc(&slots, 2 * M * 1088, hipHostMallocDefault));
  std::memset(slots, 0, 2 * M * 1088);

  auto make = [&](int set, int nride) {
    EvalMulti ev;
    std::memset(&ev, 0, sizeof(ev));
    ev.Xt = dX;
    ev.yt = dy;
    ev.T = T;
    ev.K = K;
    ev.nmodels = M;
    for (int m = 0; m < M; ++m) {
      ev.m[m].hi = hi[m];
      ev.m[m].lo = lo[m];
      ev.m[m].b = b[m];
      ev.m[m].coff = 0;
      ev.m[m].loss = nullptr;
      ev.m[m].slot = slots + (size_t)(set * M + m) * 1088;
      ev.m[m].seq = 100 + m;
    }
    ev.acc = acc;
    ev.ticket = ticket;
    ev.nticket = (unsigned)nride;
    return ev;
  };
  const int nT = (T + 31) / 32;
  const size_t lds_pm = (size_t)32 * FP * 2 + 8192 + kMaxEvalModels * 256 * 4 + 16 + 64;
  const size_t lds_tr = kEvalTileLds;
  CK(hipFuncSetAttribute((const void*)pair_major_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_pm));
  CK(hipFuncSetAttribute((const void*)tile_resident_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_tr));
  CK(hipFuncSetAttribute((const void*)tile_resident_kernel<2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_tr));
  CK(hipFuncSetAttribute((const void*)tile_resident_kernel<3>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_tr));
  CK(hipFuncSetAttribute((const void*)empty_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_pm));

  // correctness: one launch of each into its own slot set
  pair_major_kernel<<<256, 256, lds_pm>>>(make(0, 256), 256);
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  tile_resident_kernel<3><<<nT, 256, lds_tr>>>(make(1, nT), nT, nullptr, 0);
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  const bool same = std::memcmp(slots, slots + (size_t)M * 1088, (size_t)M * 1088) == 0;
  long long total = 0;
  for (int m = 0; m < M; ++m) {
    const unsigned* s = (const unsigned*)(slots + (size_t)m * 1088);
    for (int i = 1; i < 1 + (K * K + 2) / 3; ++i) total += s[4 * i + 1] + s[4 * i + 2] + s[4 * i + 3];
  }
  std::printf("{\"slots_equal\": %s, \"counted_rows\": %lld, \"expected_rows\": %d", same ? "true" : "false", total,
              T * M);

  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto time_it = [&](const char* name, auto launch) {
    for (int i = 0; i < 10; ++i) launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::printf(", \"%s_us\": %.2f", name, ms * 1000.f / reps);
  };
  const EvalMulti pm = make(0, 256), tr = make(1, nT), tr256 = make(1, 256);
  time_it("pair_major_256", [&] { pair_major_kernel<<<256, 256, lds_pm>>>(pm, 256); });
  int par = 0;
  time_it("tile_resident_153", [&] { tile_resident_kernel<3><<<nT, 256, lds_tr>>>(tr, nT, nullptr, 0); });
  time_it("tile_resident_256", [&] { tile_resident_kernel<3><<<256, 256, lds_tr>>>(tr256, 256, nullptr, 0); });
  time_it("tile_queue_256", [&] { tile_resident_kernel<3><<<256, 256, lds_tr>>>(tr256, 256, q, par); par ^= 1; });
  CK(hipDeviceSynchronize());
  std::printf(", \"queue_slots_equal\": %s",
              std::memcmp(slots, slots + (size_t)M * 1088, (size_t)M * 1088) == 0 ? "true" : "false");
  for (int ppi : {1, 2}) {
    EvalMulti e = tr256;
    e.ppi = ppi;
    char name[64];
    std::snprintf(name, sizeof(name), "tile_queue_ppi%d_256", ppi);
    time_it(name, [&] { tile_resident_kernel<3><<<256, 256, lds_tr>>>(e, 256, q, par); par ^= 1; });
    CK(hipDeviceSynchronize());
    std::printf(", \"ppi%d_slots_equal\": %s", ppi,
                std::memcmp(slots, slots + (size_t)M * 1088, (size_t)M * 1088) == 0 ? "true" : "false");
  }
  time_it("tile_tiles_only_153", [&] { tile_resident_kernel<1><<<nT, 256, lds_tr>>>(tr, nT, nullptr, 0); });
  time_it("tile_plus_flush_153", [&] { tile_resident_kernel<2><<<nT, 256, lds_tr>>>(tr, nT, nullptr, 0); });
  time_it("empty_256_lds83k", [&] { empty_kernel<<<256, 256, lds_pm>>>(pm, 256); });
  time_it("flush_only_256", [&] { flush_only_kernel<<<256, 256>>>(pm, 256); });
  time_it("ticket_only_256", [&] { ticket_only_kernel<<<256, 256>>>(pm, 256); });
  // (the flush-only kernels leave counts in the accumulators: zero them for the next run)
  CK(hipMemset(acc, 0, kEvalAccInts * 4));
  CK(hipDeviceSynchronize());
  std::printf("}\n");
  return same ? 0 : 3;
}
