// Tile machinery shared by the solve, evaluation and logits kernels (gfx950).
//
// A 32-row x FP-feature bf16 tile is staged into a dual-use LDS image
// (FP/128 sub-images of [32][128] with 256-B rows, XOR-swizzled so that row
// reads with ds_read_b128 and hardware-transposed reads with
// ds_read_b64_tr_b16 share one copy).  The forward product
// Z[32][16] = X_tile . W^T uses v_mfma_f32_16x16x32_bf16 with the weights
// split into bf16 hi + lo (two MFMAs, ~16-bit mantissa), so logits carry
// near-fp32 accuracy while X stays exact bf16.
#pragma once
#include "common.h"

namespace psx {

constexpr int kTileRowsT = 32;

__device__ __forceinline__ void write_frag(uint16_t* hi, uint16_t* lo, int c, int f, float w) {
  unsigned short h, l;
  split_bf16(w, h, l);
  const size_t o = ((size_t)(f >> 3) * 16 + c) * 8 + (f & 7);
  hi[o] = h;
  lo[o] = l;
}

// Stage rows [row0, row0+nrows) (ring-wrapped when ring) into the LDS image.
// All global loads of a batch are issued before any LDS write, so a thread
// keeps up to 16 x 16 B in flight instead of serialising on HBM latency.
template <int FP>
__device__ __forceinline__ void stage_tile(char* lds, const uint16_t* __restrict__ X, int64_t row0, int nrows,
                                           int64_t cap, bool ring) {
  constexpr int CPR = FP / 8;              // 16-B chunks per row
  constexpr int TOTAL = 32 * CPR;          // chunks per tile
  constexpr int PER_T = TOTAL / 256;       // chunks per thread (>= 2)
  constexpr int BATCH = PER_T < 16 ? PER_T : 16;
#pragma unroll
  for (int b0 = 0; b0 < PER_T; b0 += BATCH) {
    u16x8 v[BATCH];
#pragma unroll
    for (int j = 0; j < BATCH; ++j) {
      const int q = threadIdx.x + 256 * (b0 + j);
      const int row = q / CPR, cg = q - row * CPR;
      v[j] = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
      if (row < nrows) {
        int64_t r = row0 + row;
        if (ring && r >= cap) r -= cap;
        v[j] = *(const u16x8*)(X + r * FP + cg * 8);
      }
    }
#pragma unroll
    for (int j = 0; j < BATCH; ++j) {
      const int q = threadIdx.x + 256 * (b0 + j);
      const int row = q / CPR, cg = q - row * CPR;
      *(u16x8*)(lds + (cg >> 4) * 8192 + lds_off(row, cg & 15)) = v[j];
    }
  }
}

// fp32 rows: stage a 32-row tile split into TWO bf16 images, hi = bf16(x) and
// lo = bf16(x - hi) (x = hi + lo to ~16 mantissa bits), same layout as stage_tile.
template <int FP>
__device__ __forceinline__ void stage_tile_f32(char* lds_hi, char* lds_lo, const float* __restrict__ X, int64_t row0) {
  constexpr int CPR = FP / 8;           // 8-feature chunks per row
  constexpr int PER_T = 32 * CPR / 256;  // chunks per thread
  constexpr int BATCH = PER_T < 8 ? PER_T : 8;
#pragma unroll
  for (int b0 = 0; b0 < PER_T; b0 += BATCH) {
    f32x4 v[BATCH][2];
#pragma unroll
    for (int j = 0; j < BATCH; ++j) {
      const int q = threadIdx.x + 256 * (b0 + j);
      const int row = q / CPR, cg = q - row * CPR;
      const float* src = X + (row0 + row) * FP + cg * 8;
      v[j][0] = *(const f32x4*)src;
      v[j][1] = *(const f32x4*)(src + 4);
    }
#pragma unroll
    for (int j = 0; j < BATCH; ++j) {
      const int q = threadIdx.x + 256 * (b0 + j);
      const int row = q / CPR, cg = q - row * CPR;
      u16x8 h, l;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        unsigned short hh, ll;
        split_bf16(v[j][e >> 2][e & 3], hh, ll);
        h[e] = hh;
        l[e] = ll;
      }
      const int o = (cg >> 4) * 8192 + lds_off(row, cg & 15);
      *(u16x8*)(lds_hi + o) = h;
      *(u16x8*)(lds_lo + o) = l;
    }
  }
}

template <int FP>
__device__ __forceinline__ void forward_tile(const char* lds, const uint16_t* __restrict__ wf_hi,
                                             const uint16_t* __restrict__ wf_lo, f32x4& acc0, f32x4& acc1) {
  constexpr int KS_PER_WAVE = FP / 128;  // 32-feature k-steps per wave
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 15, kq = lane >> 4;
  acc0 = f32x4{0, 0, 0, 0};
  acc1 = f32x4{0, 0, 0, 0};
  constexpr int KB = KS_PER_WAVE < 8 ? KS_PER_WAVE : 8;  // k-steps whose weights are in flight together
#pragma unroll
  for (int k0 = 0; k0 < KS_PER_WAVE; k0 += KB) {
    u16x8 bh[KB], bl[KB];
#pragma unroll
    for (int kk = 0; kk < KB; ++kk) {  // weight fragments first: all loads in flight
      const int cg = (w * KS_PER_WAVE + k0 + kk) * 4 + kq;
      const size_t fo = ((size_t)cg * 16 + r) * 8;
      bh[kk] = *(const u16x8*)(wf_hi + fo);
      bl[kk] = *(const u16x8*)(wf_lo + fo);
    }
#pragma unroll
    for (int kk = 0; kk < KB; ++kk) {
      const int cg = (w * KS_PER_WAVE + k0 + kk) * 4 + kq;
      const char* sub = lds + (cg >> 4) * 8192;
      const u16x8 a0 = *(const u16x8*)(sub + lds_off(r, cg & 15));
      const u16x8 a1 = *(const u16x8*)(sub + lds_off(16 + r, cg & 15));
      acc0 = mfma16x16x32(as_bf16x8(a0), as_bf16x8(bh[kk]), acc0);
      acc0 = mfma16x16x32(as_bf16x8(a0), as_bf16x8(bl[kk]), acc0);
      acc1 = mfma16x16x32(as_bf16x8(a1), as_bf16x8(bh[kk]), acc1);
      acc1 = mfma16x16x32(as_bf16x8(a1), as_bf16x8(bl[kk]), acc1);
    }
  }
}

// Weight fragments of one wave's K-slice held in registers, so they can be
// fetched before (and overlap with) the X-tile staging.
template <int FP>
struct WFrag {
  static constexpr int KS = FP / 128;
  u16x8 h[KS], l[KS];
};

// Lanes of classes >= K hold zero fragments without fetching them (the
// fragment layout pads classes to 16; for K = 6 that skips 10/16 of the bytes).
template <int FP>
__device__ __forceinline__ void load_wfrag(WFrag<FP>& wf, const uint16_t* __restrict__ wf_hi,
                                           const uint16_t* __restrict__ wf_lo, int K = 16) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const bool live = (lane & 15) < K;
#pragma unroll
  for (int kk = 0; kk < WFrag<FP>::KS; ++kk) {
    const int cg = (w * WFrag<FP>::KS + kk) * 4 + (lane >> 4);
    const size_t fo = ((size_t)cg * 16 + (lane & 15)) * 8;
    wf.h[kk] = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
    wf.l[kk] = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
    if (live) {
      wf.h[kk] = *(const u16x8*)(wf_hi + fo);
      wf.l[kk] = *(const u16x8*)(wf_lo + fo);
    }
  }
}

// The same with hand-off loads (fragments handed off inside a persistent launch;
// S: the hand-off scope of common.h's ld_h_b128).
template <int FP, int S = 1>
__device__ __forceinline__ void load_wfrag_sc1(WFrag<FP>& wf, const uint16_t* wf_hi, const uint16_t* wf_lo, int K = 16) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const bool live = (lane & 15) < K;
  const auto rh = rsrc_of(wf_hi, 16u * FP * 2u), rl = rsrc_of(wf_lo, 16u * FP * 2u);
#pragma unroll
  for (int kk = 0; kk < WFrag<FP>::KS; ++kk) {
    const int cg = (w * WFrag<FP>::KS + kk) * 4 + (lane >> 4);
    const unsigned fo = (unsigned)((cg * 16 + (lane & 15)) * 8) * 2u;
    wf.h[kk] = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
    wf.l[kk] = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
    if (live) {
      wf.h[kk] = ld_h_b128<S>(rh, fo);
      wf.l[kk] = ld_h_b128<S>(rl, fo);
    }
  }
}

template <int FP>
__device__ __forceinline__ void forward_tile_pre(const char* lds, const WFrag<FP>& wf, f32x4& acc0, f32x4& acc1) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 15, kq = lane >> 4;
  acc0 = f32x4{0, 0, 0, 0};
  acc1 = f32x4{0, 0, 0, 0};
#pragma unroll
  for (int kk = 0; kk < WFrag<FP>::KS; ++kk) {
    const int cg = (w * WFrag<FP>::KS + kk) * 4 + kq;
    const char* sub = lds + (cg >> 4) * 8192;
    const u16x8 a0 = *(const u16x8*)(sub + lds_off(r, cg & 15));
    const u16x8 a1 = *(const u16x8*)(sub + lds_off(16 + r, cg & 15));
    acc0 = mfma16x16x32(as_bf16x8(a0), as_bf16x8(wf.h[kk]), acc0);
    acc0 = mfma16x16x32(as_bf16x8(a0), as_bf16x8(wf.l[kk]), acc0);
    acc1 = mfma16x16x32(as_bf16x8(a1), as_bf16x8(wf.h[kk]), acc1);
    acc1 = mfma16x16x32(as_bf16x8(a1), as_bf16x8(wf.l[kk]), acc1);
  }
}

// The lo image's share of the forward (x_lo . W_hi; x_lo . W_lo is below the
// precision of the hi + lo split), accumulated onto forward_tile_pre's result.
template <int FP>
__device__ __forceinline__ void forward_tile_pre_lo(const char* lds, const WFrag<FP>& wf, f32x4& acc0, f32x4& acc1) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 15, kq = lane >> 4;
#pragma unroll
  for (int kk = 0; kk < WFrag<FP>::KS; ++kk) {
    const int cg = (w * WFrag<FP>::KS + kk) * 4 + kq;
    const char* sub = lds + (cg >> 4) * 8192;
    const u16x8 a0 = *(const u16x8*)(sub + lds_off(r, cg & 15));
    const u16x8 a1 = *(const u16x8*)(sub + lds_off(16 + r, cg & 15));
    acc0 = mfma16x16x32(as_bf16x8(a0), as_bf16x8(wf.h[kk]), acc0);
    acc1 = mfma16x16x32(as_bf16x8(a1), as_bf16x8(wf.h[kk]), acc1);
  }
}

// Cross-wave logits reduction buffer [4 waves][2 m-tiles][64 lanes] f32x4.
__device__ __forceinline__ void store_partial_logits(char* red_base, const f32x4& acc0, const f32x4& acc1) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  f32x4* red = (f32x4*)red_base;
  red[(w * 2 + 0) * 64 + lane] = acc0;
  red[(w * 2 + 1) * 64 + lane] = acc1;
}

__device__ __forceinline__ float load_logit(const char* red_base, int row, int c) {
  const float* red = (const float*)red_base;
  const int mt = row >> 4, rr = row & 15;
  const int lane = (rr >> 2) * 16 + c, reg = rr & 3;
  float z = 0.f;
#pragma unroll
  for (int w = 0; w < 4; ++w) z += red[((w * 2 + mt) * 64 + lane) * 4 + reg];
  return z;
}

}  // namespace psx
