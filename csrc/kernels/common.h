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

// Dual-use LDS image of a [rows][128 x bf16] sub-tile with 256-B rows: row
// reads (ds_read_b128) and transposed reads (ds_read_b64_tr_b16) share one
// copy.  Byte offset of 16-B chunk `ch` (0..15) of `row`:
__device__ __forceinline__ int lds_off(int row, int ch) {
  return 256 * row + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
}

}  // namespace psx
