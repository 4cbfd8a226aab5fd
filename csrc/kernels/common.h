// Shared device helpers for the psx HIP kernels (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace psx {

// Private evaluation accumulators (EvalSlot mode): cell i at acc[i * kAccStride],
// one 128-B cache line per cell; [2 models][256 cells] -> 2*256*kAccStride ints.
constexpr int kAccStride = 32;

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));
typedef unsigned short u16x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef double double2v __attribute__((ext_vector_type(2)));

__device__ __forceinline__ unsigned short f2bf(float f) {
  unsigned u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (unsigned short)((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (unsigned short)(u >> 16);
}
__device__ __forceinline__ float bf2f(unsigned short h) { return __uint_as_float(((unsigned)h) << 16); }

// Split an fp32 value into bf16 hi + lo so that hi + lo carries ~16 mantissa
// bits: two bf16 MFMAs then give near-fp32 products against exact-bf16 data.
__device__ __forceinline__ void split_bf16(float v, unsigned short& hi, unsigned short& lo) {
  hi = f2bf(v);
  lo = f2bf(v - bf2f(hi));
}

__device__ __forceinline__ bf16x8 as_bf16x8(u16x8 v) { return __builtin_bit_cast(bf16x8, v); }

__device__ __forceinline__ f32x4 mfma16x16x32(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// 32 values per lane summed over the wave's 64 lanes at once: a reduce-scatter
// butterfly (xor 32, 16, 8, 4, 2 halve the values a lane carries, xor 1 completes
// the sum) -- 31 shuffles for all 32 sums instead of 6 per value.  Lane l returns
// the sum of v[l >> 1].  Fixed order: bitwise reproducible.
__device__ __forceinline__ double wave_sum_scatter32(const double (&v)[32]) {
  const int lane = threadIdx.x & 63;
  double a[16], b[8], c[4], d[2];
  {
    const bool hi = (lane & 32) != 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const double keep = hi ? v[16 + j] : v[j], send = hi ? v[j] : v[16 + j];
      a[j] = keep + __shfl_xor(send, 32, 64);
    }
  }
  {
    const bool hi = (lane & 16) != 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const double keep = hi ? a[8 + j] : a[j], send = hi ? a[j] : a[8 + j];
      b[j] = keep + __shfl_xor(send, 16, 64);
    }
  }
  {
    const bool hi = (lane & 8) != 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const double keep = hi ? b[4 + j] : b[j], send = hi ? b[j] : b[4 + j];
      c[j] = keep + __shfl_xor(send, 8, 64);
    }
  }
  {
    const bool hi = (lane & 4) != 0;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const double keep = hi ? c[2 + j] : c[j], send = hi ? c[j] : c[2 + j];
      d[j] = keep + __shfl_xor(send, 4, 64);
    }
  }
  const bool hi = (lane & 2) != 0;
  double r = (hi ? d[1] : d[0]) + __shfl_xor(hi ? d[0] : d[1], 2, 64);
  return r + __shfl_xor(r, 1, 64);
}

// Copy N 8-byte words global -> LDS with all of a thread's loads in flight
// before its first store (a load -> wait -> store loop pays one memory round
// trip per word).  NTHR threads take words tid, tid + NTHR, ...
template <int N, int NTHR>
__device__ __forceinline__ void copy_words_to_lds(unsigned long long* dst, const unsigned long long* src) {
  constexpr int PER = (N + NTHR - 1) / NTHR;
  unsigned long long v[PER];
#pragma unroll
  for (int c = 0; c < PER; ++c) {
    const int i = (int)threadIdx.x + NTHR * c;
    v[c] = i < N ? src[i] : 0ull;
  }
#pragma unroll
  for (int c = 0; c < PER; ++c) {
    const int i = (int)threadIdx.x + NTHR * c;
    if (i < N) dst[i] = v[c];
  }
}

// ---- in-launch hand-offs between workgroups (persistent solve) ----------
// Write-through (sc1) stores and L1-bypassing (sc1) loads: the R1 form of the
// CDNA4 playbook's hand-off -- every handed-off byte is stored sc1 and drained
// (s_waitcnt vmcnt(0)) before the arrival that publishes it, and EVERY load of
// it is an sc1 load, so no release / acquire fence (buffer_wbl2 / buffer_inv)
// is needed.  4- and 8-byte accesses: agent-scope relaxed atomics on global
// pointers; 16 bytes: raw buffer ops with aux = sc1.
typedef __attribute__((address_space(1))) float g_f32;
typedef __attribute__((address_space(1))) unsigned long long g_u64;
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
constexpr int kAuxSc1 = 16;

__device__ __forceinline__ float ld_sc1(const float* p) {
  return __hip_atomic_load((g_f32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(float* p, float v) {
  __hip_atomic_store((g_f32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_sc1(const double* p) {
  return __builtin_bit_cast(double, __hip_atomic_load((g_u64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ void st_sc1(double* p, double v) {
  __hip_atomic_store((g_u64*)p, __builtin_bit_cast(unsigned long long, v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const void* base, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ u16x8 ld_sc1_b128(__amdgpu_buffer_rsrc_t r, unsigned byte_off) {
  return __builtin_bit_cast(u16x8, __builtin_amdgcn_raw_buffer_load_b128(r, (int)byte_off, 0, kAuxSc1));
}
__device__ __forceinline__ void st_sc1_b128(__amdgpu_buffer_rsrc_t r, unsigned byte_off, u16x8 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, (int)byte_off, 0, kAuxSc1);
}
__device__ __forceinline__ void st_sc1_f32(__amdgpu_buffer_rsrc_t r, unsigned byte_off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, (int)byte_off, 0, kAuxSc1);
}
__device__ __forceinline__ float ld_sc1_f32(__amdgpu_buffer_rsrc_t r, unsigned byte_off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)byte_off, 0, kAuxSc1));
}

// Hand-off accessors by the parties' scope.  S = 1: the workgroups are spread
// over the XCDs -- sc1 accesses as above.  S = 2: every party runs on ONE XCD
// (blockIdx % 8 == XCC_ID on MI355X) and so shares one L2: a plain store reaches
// that L2 through the write-through vector L1, an nt load misses the L1 and
// reads it.  Measured (tools/xcd_probe.hip, profiles/r02_v5/): a 32-workgroup
// hand-off costs 0.64 us that way, 1.7 us with sc1 flags and 2.7 us with sc1 + an
// atomic arrival counter (sc0 loads and L2-executed counters do NOT work: device
// memory's atomics are performed past the L2).
constexpr int kAuxNt = 2;
template <int S>
__device__ __forceinline__ float ld_h(const float* p) {
  if constexpr (S == 2) return __builtin_nontemporal_load(p);
  else return ld_sc1(p);
}
template <int S>
__device__ __forceinline__ double ld_h(const double* p) {
  if constexpr (S == 2) return __builtin_nontemporal_load(p);
  else return ld_sc1(p);
}
template <int S>
__device__ __forceinline__ void st_h(float* p, float v) {
  if constexpr (S == 2) *p = v;
  else st_sc1(p, v);
}
template <int S>
__device__ __forceinline__ u16x8 ld_h_b128(__amdgpu_buffer_rsrc_t r, unsigned byte_off) {
  return __builtin_bit_cast(u16x8,
                            __builtin_amdgcn_raw_buffer_load_b128(r, (int)byte_off, 0, S == 2 ? kAuxNt : kAuxSc1));
}
template <int S>
__device__ __forceinline__ void st_h_b128(__amdgpu_buffer_rsrc_t r, unsigned byte_off, u16x8 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, (int)byte_off, 0, S == 2 ? 0 : kAuxSc1);
}
template <int S>
__device__ __forceinline__ unsigned long long ld_h64(unsigned long long* p) {
  if constexpr (S == 2) {
    asm volatile("" ::: "memory");  // a spin re-reads: never fold the load out of the loop
    return __builtin_nontemporal_load(p);
  } else {
    return __hip_atomic_load((g_u64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
template <int S>
__device__ __forceinline__ void st_h64(unsigned long long* p, unsigned long long v) {
  if constexpr (S == 2) *(volatile unsigned long long*)p = v;
  else __hip_atomic_store((g_u64*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Dual-use LDS image of a [rows][128 x bf16] sub-tile with 256-B rows: row
// reads (ds_read_b128) and transposed reads (ds_read_b64_tr_b16) share one
// copy.  Byte offset of 16-B chunk `ch` (0..15) of `row`:
__device__ __forceinline__ int lds_off(int row, int ch) {
  return 256 * row + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
}

}  // namespace psx
