// Device bodies of the worker local solve, shared by the launch chain and the
// persistent solve (solve_kernels.hip) and the multi-lane round kernel
// (lanes_kernels.hip): forward / backward / controller / finalisation pieces
// and the in-launch barriers.  See solve_kernels.hip for the algorithm.
#pragma once
#include <hip/hip_runtime.h>

#include "eval_body.h"
#include "lr_kernels.h"
#include "solve_kernels.h"
#include "tile.h"

namespace psx {

// Debug timeline (tools/bench_solver.py --stamps): s_memrealtime (100 MHz) per
// phase of slot `slot`, written by one lane; no effect when dv.dbg is null.
__device__ __forceinline__ void stamp(const SolveDev& dv, int slot, int k) {
  if (dv.dbg && slot < 32) dv.dbg[slot * 16 + k] = (long long)__builtin_amdgcn_s_memrealtime();
}
// Per-workgroup phase stamps of slot 1's bwd_update (rows 16..23: phase p,
// workgroup wg < 32) -- arrival-skew diagnosis.
__device__ __forceinline__ void wg_stamp(const SolveDev& dv, int slot, int p, int wg) {
  if (dv.dbg && slot == 1 && wg < 32 && threadIdx.x == 0)
    dv.dbg[(16 + p * 2 + (wg >> 4)) * 16 + (wg & 15)] = (long long)__builtin_amdgcn_s_memrealtime();
}

// ---------------------------------------------------------------------------
// Cross-workgroup exchange area of bwd_update_kernel: 64-bit words written
// with agent-scope atomic stores (sc1 write-through) and read with agent-scope
// atomic loads (sc1, bypass L1) -- the write-through hand-off form (R1) of the
// CDNA4 playbook: every storing wave drains vmcnt before the signal (ticket RMW
// or flag store), every consumer load is sc1, so no fences are needed.  Only
// the arrival ticket is a read-modify-write.
constexpr size_t ctrl_lds_bytes() { return ((sizeof(Ctrl) + 15) / 16) * 16; }
constexpr int kND = 3 + 2 * kMaxHist;  // dot products: gt.gt, gt.d, gt.gc, S_i.gt, Y_i.gt
constexpr int kNDX = kND + 1;          // + loss
constexpr int kMaxSlices = 2048 / 32;
constexpr int kXchBar = kMaxSlices * 2 * kNDX;  // [slices][2*kNDX] dot granules, then the tail barrier counter
constexpr int kXchErr = kXchBar + 1;
constexpr int kXchPhase = kXchErr + 1;  // persistent solve: the controller phase after a slot (wg 0 -> row-only wgs)
constexpr int kXchGen = kXchPhase + 1;  // persistent solve: the barrier counters of even / odd runs
constexpr int kXchRide = kXchGen + 2;   // persistent solve: riding workgroups done, even / odd runs
// one-XCD persistent solve: workgroup i's arrival word at kXchFlags + 32 i (own 256-B line)
constexpr int kXchFlags = (kXchRide + 2 + 31) / 32 * 32;
constexpr int kMaxXcdWg = 32;  // CUs of one MI355X XCD
constexpr int kPartStride = 32;  // fwd partials per workgroup: rsum[16], loss

typedef __attribute__((address_space(1))) unsigned long long gu64;
__device__ __forceinline__ unsigned long long xload(unsigned long long* p) {
  return __hip_atomic_load((gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void xstore(unsigned long long* p, unsigned long long v) {
  __hip_atomic_store((gu64*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// The window [start, start+B) of the ring (cap % 32 == 0) as a run of ring-
// aligned 32-row tiles: window tile i is ring tile (start/32 + i) mod cap/32,
// its row rr is in the window iff 0 <= 32*i + rr - start%32 < B.
struct WinTiles {
  int s0, t0, T, nt;
  __device__ __forceinline__ WinTiles(int start, int B, int cap)
      : s0(start & 31), t0(start >> 5), T(cap >> 5), nt(((start & 31) + B + 31) >> 5) {}
  __device__ __forceinline__ int ring_tile(int i) const { return t0 + i >= T ? t0 + i - T : t0 + i; }
};
// Physical history slot i holds one of the m stored pairs (ring head = newest);
// no integer modulo (H is a runtime value: each % costs ~40 instructions).
__device__ __forceinline__ bool pair_valid(int i, int m, int head, int H) {
  if (i >= H || m <= 0) return false;
  if (m >= H) return true;
  int d = i - (head - m + 1);  // in [-(H-1), 2H-3]: (d mod H) < m
  if (d < 0) d += H;
  if (d >= H) d -= H;
  return d < m;
}
__device__ __forceinline__ unsigned long long d2u(double v) { return __builtin_bit_cast(unsigned long long, v); }
__device__ __forceinline__ double u2d(unsigned long long v) { return __builtin_bit_cast(double, v); }
// Spin budget of a cross-workgroup wait (SolveDev::spin_max; 0 = the default 2^22
// polls, seconds: a timeout means a workgroup was not co-resident).
__device__ __forceinline__ int spin_limit(const SolveDev& dv) { return dv.spin_max > 0 ? dv.spin_max : 1 << 22; }


// ---------------------------------------------------------------------------
// fwd_kernel: loss and residuals at the trial point (row-parallel).
// Body shared by fwd_kernel and tail_kernel: workgroup `wg` of `G` takes the
// window tiles wg, wg+G, ...
// Rows mode: G^T partial of one tile, acc[n] (this wave's N-tiles of 16 features)
// += R_tile^T X_tile on MFMA.  A = R^T (class x 8 rows, bf16 hi + lo from the
// LDS residual tile rt[c][32 rows]); B = 8 rows x 16 features of the staged X
// image, read TRANSPOSED by ds_read_b64_tr_b16 from the same dual-use image the
// forward reads row-wise (no feature-major copy of the ring).
template <int FP, bool kHiOnly = false>
__device__ __forceinline__ void bwd_tile_acc(const char* lds, const unsigned short* rt, f32x4* acc) {
  constexpr int NT = FP / 64;  // 16-feature N-tiles per wave
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const u16x8 ah = *(const u16x8*)(rt + i * 32 + 8 * g);  // class i, rows 8g..8g+7
  const u16x8 al = *(const u16x8*)(rt + 512 + i * 32 + 8 * g);
  const int r0 = 8 * g + q;  // lane 4q+p of the group supplies row q of the 4-row block
#pragma unroll
  for (int n = 0; n < NT; ++n) {
    const int f0 = (w * NT + n) * 16;
    const char* sub = lds + (f0 >> 7) * 8192;
    const int ch = ((f0 & 127) >> 3) + (p >> 1);
    const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(sub + lds_off(r0, ch) + 8 * (p & 1)));
    const s16x4 v2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(sub + lds_off(r0 + 4, ch) + 8 * (p & 1)));
    const u16x8 b = u16x8{(unsigned short)v1[0], (unsigned short)v1[1], (unsigned short)v1[2], (unsigned short)v1[3],
                          (unsigned short)v2[0], (unsigned short)v2[1], (unsigned short)v2[2], (unsigned short)v2[3]};
    acc[n] = mfma16x16x32(as_bf16x8(ah), as_bf16x8(b), acc[n]);
    if constexpr (!kHiOnly) acc[n] = mfma16x16x32(as_bf16x8(al), as_bf16x8(b), acc[n]);
  }
}

// kF32 (rows mode only): fp32 ring rows staged as hi + lo bf16 images (the lo
// image right after the hi one), forward x_hi.(W_hi + W_lo) + x_lo.W_hi and
// backward (R_hi + R_lo)^T x_hi + R_hi^T x_lo -- near-fp32 products on bf16 MFMA.
// kP (persistent solve): the tile and its labels are already resident in LDS,
// and the trial point (fragments, intercepts) is read / the partials written
// with sc1 accesses (an in-launch hand-off, see common.h).
// kModRows (multi-lane round kernel): workgroup tiles are the window's RING tiles
// (at most cap/32 of them: a window that wraps onto its own first ring tile is one
// tile, not two) and a row is in the window iff (slot - start) mod cap < B.
template <int FP, bool kRows = false, bool kF32 = false, int kP = 0, bool kModRows = false, bool kRestage = false>
__device__ __forceinline__ void fwd_body(const SolverCfg& cfg, const SolveParams pr, int slot, const SolveDev& dv,
                                         char* lds, const int wg, const int G, f32x4* gacc = nullptr,
                                         const int entry_phase = -1) {
  static_assert(!kF32 || (kRows && FP <= 1024), "fp32 rows: rows mode, FP <= 1024 (two tile images in LDS)");
  const int B = pr.B, K = cfg.K;
  const WinTiles wt(pr.start, B, cfg.cap);
  const int ntiles = kModRows ? (wt.nt < wt.T ? wt.nt : wt.T) : wt.nt;
  if (wg >= ntiles) return;
  if (wg == 0 && threadIdx.x == 0) stamp(dv, slot, 0);
  char* lds_lo = lds + 32 * FP * 2;  // kF32: the lo image
  char* red_base = lds + (kF32 ? 2 : 1) * 32 * FP * 2;
  unsigned short* rt = (unsigned short*)(red_base + 8192);  // [2][16][32]
  int* ylds = (int*)(red_base + 8192 + 2048);
  float* rsum = (float*)(ylds + 32);  // [4 waves][16] per-wave residual sums
  float* lred = rsum + 64;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;

  float loss = 0.f;
  const int sr = tid >> 3, sc0 = (tid & 7) * 2;
  float rs0 = 0.f, rs1 = 0.f;
  static_assert(!kP || (FP <= 1024 && kRows && !kF32), "persistent solve: rows-form bodies, FP <= 1024");
  float bz0, bz1;
  if constexpr (kP != 0) {
    bz0 = ld_h<kP>(dv.b_eff + sc0);
    bz1 = ld_h<kP>(dv.b_eff + sc0 + 1);
  } else {
    bz0 = dv.b_eff[sc0];
    bz1 = dv.b_eff[sc0 + 1];
  }
  // the trial weights do not depend on the tile: fetch them before staging so
  // the two memory latencies overlap (register budget allows it up to FP 1024)
  constexpr bool kPre = FP <= 1024;
  WFrag<kPre ? FP : 128> wf;
  auto fetch_w = [&]() {
    if constexpr (kPre && kP != 0)
      load_wfrag_sc1<FP, kP>(wf, dv.whi, dv.wlo, K);
    else if constexpr (kPre)
      load_wfrag<FP>(wf, dv.whi, dv.wlo, K);
  };
  // (kRestage: fetched per tile, after its staging loads -- both sets of registers
  // live at once would spill)
  if constexpr (kPre && !kRestage) fetch_w();
  // persistent: the tile staged once, at the start of the solve -- unless the window
  // has more ring tiles than row workgroups (kRestage: every slot stages each of them)
  for (int tile = wg; tile < ntiles; tile += G) {
    const int64_t row0 = (int64_t)wt.ring_tile(tile) * 32;
    if constexpr (kP == 0 || kRestage) {
      const int yv = tid < 32 ? dv.y[row0 + tid] : 0;  // issued with the tile's loads (one round trip)
      if constexpr (kF32)
        stage_tile_f32<FP>(lds, lds_lo, dv.Xf, row0);
      else
        stage_tile<FP>(lds, dv.X, row0, 32, cfg.cap, false);
      if (tid < 32) ylds[tid] = yv;
    }
    if constexpr (kPre && kRestage) fetch_w();
    __syncthreads();
    // converged in an earlier slot: exit (the phase word was loaded at kernel
    // entry, so its latency overlapped the tile staging; nothing written yet)
    if (entry_phase == kPhDone) return;
    if (wg == 0 && tid == 0) stamp(dv, slot, 9);
    f32x4 a0, a1;
    if constexpr (kPre)
      forward_tile_pre<FP>(lds, wf, a0, a1);
    else
      forward_tile<FP>(lds, dv.whi, dv.wlo, a0, a1);
    if constexpr (kF32) forward_tile_pre_lo<FP>(lds_lo, wf, a0, a1);
    store_partial_logits(red_base, a0, a1);
    __syncthreads();
    if (wg == 0 && tid == 0) stamp(dv, slot, 10);
    {  // softmax + cross entropy: 8 threads per row, 2 classes each
      const bool v0 = sc0 < K, v1 = sc0 + 1 < K;
      const float z0 = v0 ? load_logit(red_base, sr, sc0) + bz0 : -INFINITY;
      const float z1 = v1 ? load_logit(red_base, sr, sc0 + 1) + bz1 : -INFINITY;
      float mx = fmaxf(z0, z1);
      mx = fmaxf(mx, __shfl_xor(mx, 1, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 2, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 4, 64));
      const float e0 = v0 ? __expf(z0 - mx) : 0.f, e1 = v1 ? __expf(z1 - mx) : 0.f;
      float se = e0 + e1;
      se += __shfl_xor(se, 1, 64);
      se += __shfl_xor(se, 2, 64);
      se += __shfl_xor(se, 4, 64);
      int orow = tile * 32 + sr - wt.s0;  // offset in the window
      if (kModRows && orow < 0) orow += wt.T * 32;  // a wrapped window's newest rows share its first ring tile
      const bool valid = orow >= 0 && orow < B;
      const int yl = ylds[sr];
      const float inv = 1.f / se;
      const float r0 = valid && v0 ? e0 * inv - (yl == sc0 ? 1.f : 0.f) : 0.f;
      const float r1 = valid && v1 ? e1 * inv - (yl == sc0 + 1 ? 1.f : 0.f) : 0.f;
      if (valid) {
        const float lse = mx + __logf(se);
        if (yl == sc0) loss += lse - z0;
        if (yl == sc0 + 1) loss += lse - z1;
      }
      rs0 += r0;
      rs1 += r1;
      unsigned short h, l;
      split_bf16(r0, h, l);
      rt[sc0 * 32 + sr] = h;
      rt[512 + sc0 * 32 + sr] = l;
      split_bf16(r1, h, l);
      rt[(sc0 + 1) * 32 + sr] = h;
      rt[512 + (sc0 + 1) * 32 + sr] = l;
    }
    __syncthreads();
    if constexpr (kRows) {  // the backward of this tile while it is in LDS
      bwd_tile_acc<FP>(lds, rt, gacc);
      if constexpr (kF32) bwd_tile_acc<FP, true>(lds_lo, rt, gacc);
      __syncthreads();  // the next tile's staging overwrites the image and rt
    } else {
      // residual tile -> global, in the A-operand layout of the backward MFMA
      // (rows of the padding classes >= K are never read by the backward)
      if ((((tid * 4) & 511) >> 5) < K)
        *(u16x4*)(dv.R + (size_t)tile * 1024 + tid * 4) = *(const u16x4*)(rt + tid * 4);
    }
    if (wg == 0 && tid == 0) stamp(dv, slot, 11);
  }
  // per-class residual sums over the rows, in a fixed order (a butterfly over the
  // lanes of one class pair, then the waves in order): the solve is bitwise
  // reproducible -- LDS float atomics would sum in arrival order
#pragma unroll
  for (int o = 8; o < 64; o <<= 1) {
    rs0 += __shfl_xor(rs0, o, 64);
    rs1 += __shfl_xor(rs1, o, 64);
  }
  if (lane < 8) {
    rsum[w * 16 + sc0] = rs0;
    rsum[w * 16 + sc0 + 1] = rs1;
  }
  loss = wave_sum(loss);
  if (lane == 0) lred[w] = loss;
  __syncthreads();
  float* part = dv.part + (size_t)wg * kPartStride;
  float pv = 0.f;
  if (tid < 16) pv = ((rsum[tid] + rsum[16 + tid]) + rsum[32 + tid]) + rsum[48 + tid];
  if (tid == 16) pv = lred[0] + lred[1] + lred[2] + lred[3];
  if (tid < 17) {
    if constexpr (kP != 0)
      st_h<kP>(part + tid, pv);
    else
      part[tid] = pv;
  }
  if (wg == 0 && tid == 0) stamp(dv, slot, 1);
}

// The window arrives as a kernel argument (win.B > 0; eager launches) or from
// device memory (win.B <= 0: graph replays, whose arguments are fixed at capture)
// -- the argument form takes one dependent load off the head of the chain.
__device__ __forceinline__ SolveParams window_of(const SolveParams& win, const SolveParams* prm) {
  return win.B > 0 ? win : *prm;
}

// A forward workgroup's partial gradient sums R^T X (classes < KP) -> gpf[wg][f][KP]:
// a lane's 4 classes of one feature are contiguous -> one 16-B store (sc1 inside
// the persistent solve, plain behind a kernel boundary).
template <int FP, bool kSc1>
__device__ __forceinline__ void store_gpf(const SolveDev& dv, int wg, int G, const f32x4* acc) {
  constexpr int NT = FP / 64;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, KP = dv.KP;
  const int c0 = (lane >> 4) * 4;
  const auto rg = rsrc_of(dv.gpf, (unsigned)((size_t)G * KP * FP * 4));
#pragma unroll
  for (int n = 0; n < NT; ++n) {
    const int f = (w * NT + n) * 16 + (lane & 15);
    const size_t eo = ((size_t)wg * FP + f) * KP + c0;
    if (KP >= 4) {
      if (c0 < KP) {
        if constexpr (kSc1)
          st_sc1_b128(rg, (unsigned)(eo * 4), __builtin_bit_cast(u16x8, acc[n]));
        else
          *(f32x4*)(dv.gpf + eo) = acc[n];
      }
    } else if (c0 == 0) {
      if constexpr (kSc1) {
        st_sc1_f32(rg, (unsigned)(eo * 4), acc[n][0]);
        st_sc1_f32(rg, (unsigned)(eo * 4) + 4, acc[n][1]);
      } else {
        dv.gpf[eo] = acc[n][0];
        dv.gpf[eo + 1] = acc[n][1];
      }
    }
  }
}

// Forward of the slot's trial point; with dv.gpf also the backward's partial
// sums R^T X of the workgroup's tile, while the tile is in LDS.
template <int FP, bool kGpf>
__device__ __forceinline__ void fwd_slot(const SolverCfg& cfg, const SolveParams pr, int slot, const SolveDev& dv,
                                         char* lds, const int wg, const int G, const int entry_phase) {
  if constexpr (kGpf) {
    constexpr int NT = FP / 64;
    f32x4 acc[NT];
#pragma unroll
    for (int n = 0; n < NT; ++n) acc[n] = f32x4{0, 0, 0, 0};
    const WinTiles wt(pr.start, pr.B, cfg.cap);
    if (wg >= wt.nt) return;
    fwd_body<FP, true>(cfg, pr, slot, dv, lds, wg, G, acc, entry_phase);
    if (entry_phase == kPhDone) return;  // (converged earlier: fwd_body left after staging)
    store_gpf<FP, false>(dv, wg, G, acc);
  } else {
    fwd_body<FP>(cfg, pr, slot, dv, lds, wg, G, nullptr, entry_phase);
  }
}

// ---------------------------------------------------------------------------
// Finalisation (after the last slot): back to the unstandardised space,
// multinomial centring across classes, delta = w_new - w_old, eval fragments,
// loss and solver statistics.  One thread per feature (all classes).
// Per-feature inputs of the finalisation, loadable ahead of the phase check.
template <int KP>
struct FinIn {
  float iv, xv[KP], fx[KP], wo[KP];
  __device__ __forceinline__ void load(const SolverCfg& cfg, const SolveDev& dv, int blk) {
    load_f(cfg, dv, blk * 256 + threadIdx.x);
  }
  __device__ __forceinline__ void load_f(const SolverCfg& cfg, const SolveDev& dv, int f) {
    const int FP = cfg.Fp, FPI = dv.FPI, K = cfg.K;
    if (f >= FP) return;
    iv = dv.inv_std[f];
#pragma unroll
    for (int c = 0; c < KP; ++c) {
      xv[c] = dv.x[c * FPI + f];
      fx[c] = dv.wfix[c * FPI + f];
      wo[c] = (c < K && f < cfg.F) ? dv.w_old[c * FP + f] : 0.f;
    }
  }
};

template <int KP>
__device__ __forceinline__ void finalize_feature(const SolverCfg& cfg, const SolveDev& dv, int f, const FinIn<KP>& in,
                                                 bool sc1_delta = false) {
  const int FP = cfg.Fp, K = cfg.K;
  if (f < FP) {
    const float iv = in.iv;
    const float *xv = in.xv, *fx = in.fx, *wo = in.wo;
    float wv[KP];
    float mean = 0.f;
#pragma unroll
    for (int c = 0; c < KP; ++c) {
      wv[c] = f < cfg.F ? (iv > 0.f ? xv[c] * iv : fx[c]) : 0.f;
      mean += wv[c];
    }
    mean = (cfg.center && f < cfg.F) ? mean / (float)K : 0.f;
#pragma unroll
    for (int c = 0; c < KP; ++c) {
      const float v = c < K ? wv[c] - mean : 0.f;
      write_frag(dv.out_hi, dv.out_lo, c, f, v);
      if (c < K) {
        const float dl = v - wo[c];
        if (sc1_delta)
          st_sc1(dv.delta + c * FP + f, dl);
        else
          dv.delta[c * FP + f] = dl;
        if (dv.w_new) dv.w_new[c * FP + f] = v;
        if (dv.ap_w) {  // fused server update: w += lr * delta (ServerProcessor.java:148-151)
          // (ap_w may alias w_old: this thread alone reads and writes element (c, f))
          const float nw = wo[c] + dv.ap_lr * dl;
          dv.ap_w[c * FP + f] = nw;
          write_frag(dv.ap_hi, dv.ap_lo, dv.ap_coff + c, f, f < cfg.F ? nw : 0.f);
        }
      }
    }
  }
}

// The intercepts, the loss and the solver statistics (one thread).  Every load
// is issued before the first store (they are independent): one memory round
// trip instead of a chain of them -- this is most of the tail launch's time
// when the last bwd_update launch finalised the features.
struct FinScal {
  float bv[16], wo[16];
  double f_c;
  int evals, nacc, ls_fail, dir_reset, st4;
  unsigned run;
  unsigned long long err;
  __device__ __forceinline__ void load(const SolverCfg& cfg, const Ctrl* ctrl, const SolveDev& dv) {
    const int K = cfg.K, IB = dv.KP * dv.FPI, KF = K * cfg.Fp;
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      bv[c] = c < K ? dv.x[IB + c] : 0.f;
      wo[c] = c < K ? dv.w_old[KF + c] : 0.f;
    }
    f_c = ctrl->f_c;
    evals = ctrl->evals;
    nacc = ctrl->nacc;
    ls_fail = ctrl->ls_fail;
    dir_reset = ctrl->dir_reset;
    run = *dv.prm_count;
    // a cross-workgroup wait that timed out (a workgroup was not co-resident):
    // this solve's result is garbage -- sticky flag for the host, NaN loss in the logs
    err = dv.stats ? xload(dv.xch + kXchErr) : 0ull;
    st4 = dv.stats ? dv.stats[4] : 0;
  }
  // sc1_delta: the delta is read by workgroups of other XCDs in this launch (the
  // multi-lane round kernel's cross-lane sum): write-through stores
  // clear_err = false: the caller owns the sticky error word (the lanes kernel)
  __device__ __forceinline__ void store(const SolverCfg& cfg, const SolveDev& dv, bool sc1_delta = false,
                                        bool clear_err = true) const {
    const int K = cfg.K, KF = K * cfg.Fp;
    float mean = 0.f;
#pragma unroll
    for (int c = 0; c < 16; ++c) mean += c < K ? bv[c] : 0.f;
    mean = cfg.center ? mean / (float)K : 0.f;
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      if (c >= K) continue;
      const float v = bv[c] - mean;
      const float dl = v - wo[c];
      if (sc1_delta)
        st_sc1(dv.delta + KF + c, dl);
      else
        dv.delta[KF + c] = dl;
      if (dv.w_new) dv.w_new[KF + c] = v;
      dv.b_fin[c] = v;
      if (dv.ap_w) {
        const float nw = wo[c] + dv.ap_lr * dl;
        dv.ap_w[KF + c] = nw;
        dv.ap_b[dv.ap_coff + c] = nw;
      }
    }
    *dv.loss = err ? __builtin_nanf("") : (float)f_c;
    *dv.prm_count = run + 1;  // run counter: makes the all-gather tags unique per run
    if (dv.stats) {
      dv.stats[0] = evals;
      dv.stats[1] = nacc;
      dv.stats[2] = ls_fail;
      dv.stats[3] = dir_reset;
      if (err) {
        dv.stats[4] = st4 | (int)err;
        if (clear_err) xstore(dv.xch + kXchErr, 0ull);
      }
    }
    if (err && dv.err_host) {  // pinned host word: the host loop sees the failure without a sync
      __hip_atomic_store(dv.err_host, (unsigned long long)(run + 1) << 8 | (err & 0xffull), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
};

template <int KP>
__device__ __forceinline__ void finalize_scalars(const SolverCfg& cfg, const Ctrl* ctrl, const SolveDev& dv) {
  FinScal sc;
  sc.load(cfg, ctrl, dv);
  sc.store(cfg, dv);
}

// Finalisation over 32-feature slices (FP/32 workgroups, one (class, feature)
// element per thread): the scattered fragment / delta stores spread over 32 CUs
// instead of 4.  Same arithmetic (and class order of the centring mean) as
// finalize_feature.
template <int KP>
struct FinSl {
  static constexpr int NE = KP > 8 ? KP / 8 : 1;
  float iv, xv[NE], fx[NE], wo[NE];
  __device__ __forceinline__ void load(const SolverCfg& cfg, const SolveDev& dv, int blk) {
    const int FP = cfg.Fp, FPI = dv.FPI, K = cfg.K;
    const int f = blk * 32 + (threadIdx.x & 31), cg = threadIdx.x >> 5;
    iv = dv.inv_std[f];
#pragma unroll
    for (int e = 0; e < NE; ++e) {
      const int c = cg + 8 * e;
      xv[e] = fx[e] = wo[e] = 0.f;
      if (c < KP) {
        xv[e] = dv.x[c * FPI + f];
        fx[e] = dv.wfix[c * FPI + f];
        wo[e] = (c < K && f < cfg.F) ? dv.w_old[c * FP + f] : 0.f;
      }
    }
  }
};

// sc1_delta: the delta is stored write-through (agent scope) for readers on other
// XCDs (the lanes kernel's cross-lane sum), as finalize_feature's flag.
template <int KP>
__device__ __forceinline__ void finalize_slice(const SolverCfg& cfg, const SolveDev& dv, int blk, const FinSl<KP>& in,
                                               float* wvl /* LDS [16][32] */, bool sc1_delta = false) {
  constexpr int NE = FinSl<KP>::NE;
  const int FP = cfg.Fp, K = cfg.K;
  const int fl = threadIdx.x & 31, cg = threadIdx.x >> 5, f = blk * 32 + fl;
  float wv[NE];
#pragma unroll
  for (int e = 0; e < NE; ++e) {
    const int c = cg + 8 * e;
    wv[e] = (c < KP && f < cfg.F) ? (in.iv > 0.f ? in.xv[e] * in.iv : in.fx[e]) : 0.f;
    if (c < KP) wvl[c * 32 + fl] = wv[e];
  }
  __syncthreads();
  float mean = 0.f;
#pragma unroll
  for (int c = 0; c < KP; ++c) mean += wvl[c * 32 + fl];  // class order: as finalize_feature
  mean = (cfg.center && f < cfg.F) ? mean / (float)K : 0.f;
#pragma unroll
  for (int e = 0; e < NE; ++e) {
    const int c = cg + 8 * e;
    if (c >= KP) continue;
    const float v = c < K ? wv[e] - mean : 0.f;
    write_frag(dv.out_hi, dv.out_lo, c, f, v);
    if (c < K) {
      const float dl = v - in.wo[e];
      if (sc1_delta)
        st_sc1(dv.delta + c * FP + f, dl);
      else
        dv.delta[c * FP + f] = dl;
      if (dv.w_new) dv.w_new[c * FP + f] = v;
      if (dv.ap_w) {  // fused server update (see finalize_feature)
        const float nw = in.wo[e] + dv.ap_lr * dl;
        dv.ap_w[c * FP + f] = nw;
        write_frag(dv.ap_hi, dv.ap_lo, dv.ap_coff + c, f, f < cfg.F ? nw : 0.f);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// bwd_update_kernel: gradient of a 32-feature slice, controller step, update.
// Both MFMA operands come straight from global memory in fragment shape: the
// residual tiles R (class x 8 rows = 16 B per lane) and the feature-major ring
// copy XT (feature x 8 consecutive rows = 16 B per lane), so no LDS staging.
constexpr int kBwdBatch = 8;  // k-steps (32-row tiles) per wave whose loads are in flight together

// persistent solve: the slice's curvature pairs in LDS, [kMaxHist][S | Y][KP <= 8 classes x 32 features + 16 intercepts]
constexpr int kSyStride = 8 * 32 + 16;
constexpr size_t kSyBytes = (size_t)kMaxHist * 2 * kSyStride * sizeof(float);
constexpr size_t kBwdLdsBytes = (size_t)4 * 16 * 32 * 4 + 2 * 512 * 2 + ctrl_lds_bytes() +
                                (4 * kNDX + kNDX + kMaxSlices * kNDX) * sizeof(double) + 256 * sizeof(float) +
                                sizeof(CtrlScratch);

// Body shared by bwd_update_kernel, tail_kernel and the persistent solve: slice
// `wg` of `NS`.  kP (persistent solve): the controller copy in LDS persists
// across slots (no copy-in / write-back), the partials written by other
// workgroups of the launch are read with sc1 loads and the next trial point is
// published with sc1 stores (common.h).
template <int FP, int KP, int kP = 0, int kXs = (kP == 2 ? 2 : 1)>
__device__ __forceinline__ void bwd_body(const SolverCfg& cfg, const SolveParams win, Ctrl* gctrl, int slot,
                                         const SolveDev& dv, int fwd_grid, char* lds, const int wg, const int NS,
                                         const bool check_done = false, const int fin_slot = kNoFinSlot,
                                         const bool fin_sc1 = false) {
  constexpr int FPI = FP > 256 ? FP : 256;
  constexpr int IB = KP * FPI;              // internal intercept base
  constexpr int NE = KP >= 8 ? KP / 8 : 1;  // elements per thread
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  if (wg == 0 && tid == 0) stamp(dv, slot, 2);
  wg_stamp(dv, slot, 0, wg);
  // (kMaxSlots tags per run: the LocalSolver / lanes loop reject nslots >= kMaxSlots, so a
  // word left from the previous run never carries this run's tag)
  const unsigned run_tag = *dv.prm_count * (unsigned)kMaxSlots;  // early: needed by the all-gather
  float* gw = (float*)lds;                             // [4 waves][16 classes][32]
  unsigned short* frl = (unsigned short*)(gw + 4 * 16 * 32);  // [2][512] fragment staging
  Ctrl* cl = (Ctrl*)(frl + 1024);
  double* sdot = (double*)((char*)cl + ctrl_lds_bytes());  // [4 waves][kNDX]
  double* dots = sdot + 4 * kNDX;                          // [kNDX]
  double* gat = dots + kNDX;                               // [slices][kNDX]
  float* pr = (float*)(gat + kMaxSlices * kNDX);           // [15][17] fwd-partial stripes
  CtrlScratch* csw = (CtrlScratch*)(pr + 256);
  unsigned long long* xch = dv.xch;

  const int B = win.B, cap = cfg.cap, K = cfg.K, H = cfg.hist;
  const WinTiles wt(win.start, B, cap);
  const size_t PI = dv.PI;
  const float invB = 1.f / (float)B;
  const int fs = wg * 32;
  const int fl = tid & 31, cgp = tid >> 5;
  const int f = fs + fl;
  const bool wg0 = wg == 0;
  const int ntiles = wt.nt;

  // ---- the backward's operands first: the residual tiles R (fwd output) and
  // the feature-major window XT of this slice, kBwdBatch k-steps per wave in
  // flight -- issued ahead of every other load so that one memory round trip
  // covers them, the controller copy and the per-element state together ----
  // partials of the forward workgroups [g][f][KP] (always, in the persistent solve)
  const bool gpf = kP != 0 || dv.gpf != nullptr;
  const bool gred = kP == 0 && !gpf && dv.gpart != nullptr;  // rows mode: partials [g][KP][FP]
  const int m16 = lane & 15, kg = (lane >> 4) * 8;
  const unsigned short* xt0 = dv.XT + (size_t)(fs + m16) * cap + kg;  // N-tile 0 (features fs..fs+15)
  const unsigned short* xt1 = xt0 + (size_t)16 * cap;                  // N-tile 1
  const unsigned short* rp0 = dv.R + m16 * 32 + kg;
  const bool live = m16 < K;  // padding-class rows of R are neither written nor read
  u16x8 ah[kBwdBatch], al[kBwdBatch], b0[kBwdBatch], b1[kBwdBatch];
  auto load_batch = [&](int kb) {
#pragma unroll
    for (int u = 0; u < kBwdBatch; ++u) {  // every load of the batch in flight together
      const int i = kb + w + 4 * u;
      const int ic = i < ntiles ? i : ntiles - 1;
      const size_t ro = (size_t)wt.ring_tile(ic) * 32;
      ah[u] = al[u] = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
      if (live) {
        ah[u] = *(const u16x8*)(rp0 + (size_t)ic * 1024);
        al[u] = *(const u16x8*)(rp0 + (size_t)ic * 1024 + 512);
      }
      b0[u] = *(const u16x8*)(xt0 + ro);
      b1[u] = *(const u16x8*)(xt1 + ro);
    }
  };
  if (!gred && !gpf) load_batch(0);
  // every workgroup runs the (deterministic) controller on its own LDS copy
  if constexpr (kP == 0)
    copy_words_to_lds<sizeof(Ctrl) / 8, 256>((unsigned long long*)cl, (const unsigned long long*)gctrl);

  // ---- per-element state first (independent of the backward) ----
  float DD[NE], GC[NE], XO[NE], FX[NE];
  int idx[NE];
  bool own[NE];
#pragma unroll
  for (int e = 0; e < NE; ++e) {
    const int c = cgp + 8 * e;
    own[e] = c < KP;
    idx[e] = (own[e] ? c : 0) * FPI + f;
    DD[e] = dv.d[idx[e]];
    GC[e] = dv.g_c[idx[e]];
    XO[e] = dv.x[idx[e]];
    FX[e] = dv.wfix[idx[e]];
  }
  const float iv = dv.inv_std[f];
  const bool ib0 = wg0 && tid < 16;
  // stored curvature pairs of this slice (measured: prefetching them with the
  // backward's operands lengthens the load phase by ~1 us and saves nothing
  // later -- profiles/r02_v5/README.md -- so they are read where needed)
  // (persistent solve: the slice's pairs stay in LDS for the whole solve -- each
  // element is written and read by the same thread -- at lsy[(2 i + {0: S, 1: Y})
  // * kSyStride + c * 32 + fl], intercepts at [... + 256 + tid])
  float* lsy = kP != 0 ? (float*)(lds + (kBwdLdsBytes + 15) / 16 * 16) : nullptr;
  auto s_at = [&](int i, int e) {
    return kP != 0 ? lsy[2 * i * kSyStride + (cgp + 8 * e) * 32 + fl] : dv.S[(size_t)i * PI + idx[e]];
  };
  auto y_at = [&](int i, int e) {
    return kP != 0 ? lsy[(2 * i + 1) * kSyStride + (cgp + 8 * e) * 32 + fl] : dv.Y[(size_t)i * PI + idx[e]];
  };
  auto sb_at = [&](int i) { return kP != 0 ? lsy[2 * i * kSyStride + 256 + tid] : dv.S[(size_t)i * PI + IB + tid]; };
  auto yb_at = [&](int i) {
    return kP != 0 ? lsy[(2 * i + 1) * kSyStride + 256 + tid] : dv.Y[(size_t)i * PI + IB + tid];
  };
  // a launch that may finish the solve finalises its slice in place (below):
  // its w_old elements travel with the per-element state
  const bool may_fin = slot >= fin_slot;
  float WO[NE];
#pragma unroll
  for (int e = 0; e < NE; ++e) {
    const int c = cgp + 8 * e;
    WO[e] = (may_fin && c < K && f < cfg.F) ? dv.w_old[c * FP + f] : 0.f;
  }
  const int nfw = ntiles < fwd_grid ? ntiles : fwd_grid;
  float db0 = 0.f, gcb0 = 0.f, xb0 = 0.f;
  if (wg0 && tid < 255) {  // intercept gradient / loss partials: 15 stripes x 17 values, fixed order
    const int k = tid % 17, g0 = tid / 17;
    float a = 0.f;
#pragma unroll 4
    for (int s = g0; s < nfw; s += 15) {
      const float* pp = dv.part + (size_t)s * kPartStride + k;
      if constexpr (kP != 0)
        a += ld_h<kP>(pp);
      else
        a += *pp;
    }
    pr[g0 * 17 + k] = a;
  }
  if (wg0 && tid < 16) {
    db0 = dv.d[IB + tid];
    gcb0 = dv.g_c[IB + tid];
    xb0 = dv.x[IB + tid];
  }
  if (tid < 128) *(u16x8*)(frl + tid * 8) = u16x8{0, 0, 0, 0, 0, 0, 0, 0};

  // ---- backward G[c][slice] = sum_r R[r][c] X[r][slice] ----
  // (rows mode: partial sums of the fwdbwd_rows workgroups, already reduced by
  // reduce_g into dv.gred for large grids, summed here in a fixed order otherwise)
  f32x4 acc[2] = {f32x4{0, 0, 0, 0}, f32x4{0, 0, 0, 0}};
  if (!gred && !gpf) {
    for (int kb = 0; kb < ntiles; kb += 4 * kBwdBatch) {
      if (kb > 0) load_batch(kb);  // (batch 0 was issued at entry)
#pragma unroll
      for (int u = 0; u < kBwdBatch; ++u) {
        const int i = kb + w + 4 * u;
        if (i >= ntiles) ah[u] = al[u] = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
        acc[0] = mfma16x16x32(as_bf16x8(ah[u]), as_bf16x8(b0[u]), acc[0]);
        acc[0] = mfma16x16x32(as_bf16x8(al[u]), as_bf16x8(b0[u]), acc[0]);
        acc[1] = mfma16x16x32(as_bf16x8(ah[u]), as_bf16x8(b1[u]), acc[1]);
        acc[1] = mfma16x16x32(as_bf16x8(al[u]), as_bf16x8(b1[u]), acc[1]);
      }
    }
  }
  if (gpf) {
    // the slice's [32 f][KP c] partials of every tile are contiguous (1 KB for KP 8):
    // thread = (16-B piece p, tile group q of 4); all its tiles' loads in flight,
    // summed in tile order, then the 4 groups in order -> gw[c][f]
    constexpr int NP = 32 * KP / 4;  // 16-B pieces of a slice (KP >= 4); KP 2: 8-B pieces
    const int nfw_g = wt.nt < fwd_grid ? wt.nt : fwd_grid;
    const int p = tid % 64, q = tid / 64;
    float* red = (float*)(gw + 16 * 32);  // [4 groups][64 pieces][4] (gw's other waves' rows)
    f32x4 a = f32x4{0, 0, 0, 0};
    if (p < NP && KP >= 4) {
      // (persistent solve: sc1 loads of the in-launch hand-off; chain: plain loads
      // behind the kernel boundary)
      const auto rg = rsrc_of(dv.gpf, (unsigned)((size_t)fwd_grid * KP * FP * 4));
      constexpr int UG = 17;
      for (int g0 = q; g0 < nfw_g; g0 += 4 * UG) {
        u16x8 v[UG];
#pragma unroll
        for (int u = 0; u < UG; ++u) {
          const int g = g0 + 4 * u;
          const size_t eo = ((size_t)g * FP + fs) * KP + p * 4;
          v[u] = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
          if (g < nfw_g) {
            if constexpr (kP != 0)
              v[u] = ld_h_b128<kP>(rg, (unsigned)(eo * 4));
            else
              v[u] = *(const u16x8*)(dv.gpf + eo);
          }
        }
#pragma unroll
        for (int u = 0; u < UG; ++u) a += __builtin_bit_cast(f32x4, v[u]);
      }
    } else if (p < 16 && KP == 2) {  // 32 features x 2 classes = 16 x 16 B as well
      for (int g = q; g < nfw_g; g += 4) {
        const float* src = dv.gpf + ((size_t)g * FP + fs) * KP + p * 4;
        if constexpr (kP != 0)
          a += f32x4{ld_h<kP>(src), ld_h<kP>(src + 1), ld_h<kP>(src + 2), ld_h<kP>(src + 3)};
        else
          a += *(const f32x4*)src;
      }
    }
    *(f32x4*)(red + (q * 64 + p) * 4) = a;
    __syncthreads();
    // thread (cgp = class, fl = feature): element (f, c) sits in piece (fl * KP + c) / 4
    if (cgp < KP && cgp < 8) {
      const int pc = fl * KP + cgp, pp = pc >> 2, lanei = pc & 3;
      gw[cgp * 32 + fl] = ((red[(0 * 64 + pp) * 4 + lanei] + red[(1 * 64 + pp) * 4 + lanei]) +
                           red[(2 * 64 + pp) * 4 + lanei]) + red[(3 * 64 + pp) * 4 + lanei];
    }
  }
  if (wg0 && tid == 0) stamp(dv, slot, 3);
  wg_stamp(dv, slot, 1, wg);
  // cross-wave reduction of the accumulators (D[class][feature])
  if (!gred && !gpf) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int c = (lane >> 4) * 4 + rr;
        gw[(w * 16 + c) * 32 + j * 16 + (lane & 15)] = acc[j][rr];
      }
  }
  __syncthreads();
  // converged in an earlier slot (standalone launch): exit.  Checked here, on the
  // LDS copy of the controller, so the phase load overlapped the backward's loads;
  // nothing global has been written yet.
  if (check_done && cl->phase == kPhDone) return;
  float g[NE];
#pragma unroll
  for (int e = 0; e < NE; ++e) {
    const int c = (cgp + 8 * e) & 15;
    float s;
    if (gpf) {  // reduced from the forward partials above
      s = own[e] ? gw[c * 32 + fl] : 0.f;
    } else if (!gred) {
      s = gw[c * 32 + fl] + gw[(16 + c) * 32 + fl] + gw[(32 + c) * 32 + fl] + gw[(48 + c) * 32 + fl];
    } else if (dv.gred) {
      s = own[e] ? dv.gred[idx[e]] : 0.f;
    } else {  // small grid: sum the workgroups' partials here (fixed order)
      s = 0.f;
      if (own[e]) {
        const int nfw_g = wt.nt < fwd_grid ? wt.nt : fwd_grid;
        const size_t stride = (size_t)dv.KP * cfg.Fp;
        const float* src = dv.gpart + (size_t)(cgp + 8 * e) * cfg.Fp + f;
        constexpr int U = 8;
        for (int g0 = 0; g0 < nfw_g; g0 += U) {
          float v[U];
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const float* q = src + (size_t)(g0 + u) * stride;
            if constexpr (kP != 0)
              v[u] = g0 + u < nfw_g ? ld_h<kP>(q) : 0.f;
            else
              v[u] = g0 + u < nfw_g ? *q : 0.f;
          }
#pragma unroll
          for (int u = 0; u < U; ++u) s += v[u];
        }
      }
    }
    g[e] = own[e] ? s * invB * iv : 0.f;
  }
  float rpart = 0.f;  // the cross-wave barrier above also published pr[]
  if (wg0 && tid < 17)
#pragma unroll
    for (int g0 = 0; g0 < 15; ++g0) rpart += pr[g0 * 17 + tid];
  const float gb = (wg0 && tid < 16) ? rpart * invB : 0.f;
  if (wg0 && tid == 0) stamp(dv, slot, 4);

  // ---- partial dot products -> exchange area ----
  // The wave's values in the all-gather's order (k < nv = 4 + 2m): gt.gt, gt.d, gt.gc,
  // loss, then per stored pair j (oldest first, ring slot (hbase + j) mod H) S_j.gt,
  // Y_j.gt.  Up to 32 values go through ONE multi-value butterfly per wave (a
  // reduce-scatter over the lanes: 31 shuffles of doubles for all of them instead of
  // 6 per value -- the dots phase was 1.5-2.3 us of every 12-us slot, profiles/r05).
  const int m = cl->m, head = cl->head;
  const int nv = 4 + 2 * m;  // gt.gt, gt.d, gt.gc, loss, (S_j.gt, Y_j.gt) x m
  const int hbase = head - m + 1 < 0 ? head - m + 1 + H : head - m + 1;  // (head - m + 1) mod H: > -H
  double tt = (double)gb * gb, td = (double)gb * db0, tc = (double)gb * gcb0;
#pragma unroll
  for (int e = 0; e < NE; ++e) {
    tt += (double)g[e] * g[e];
    td += (double)g[e] * DD[e];
    tc += (double)g[e] * GC[e];
  }
  const double lsum = (wg0 && tid == 16) ? (double)rpart : 0.0;
  auto pair_dots = [&](int j, double& si, double& yi) {
    int i = hbase + j;
    if (i >= H) i -= H;
    si = 0.0;
    yi = 0.0;
#pragma unroll
    for (int e = 0; e < NE; ++e) {
      si += (double)s_at(i, e) * g[e];
      yi += (double)y_at(i, e) * g[e];
    }
    if (ib0) {
      si += (double)sb_at(i) * gb;
      yi += (double)yb_at(i) * gb;
    }
  };
  if (nv <= 32) {
    double v[32];
    v[0] = tt;
    v[1] = td;
    v[2] = tc;
    v[3] = lsum;
#pragma unroll
    for (int j = 0; j < 14; ++j) {
      double si = 0.0, yi = 0.0;
      if (j < m) pair_dots(j, si, yi);  // (wave-uniform)
      v[4 + 2 * j] = si;
      v[5 + 2 * j] = yi;
    }
    const double r = wave_sum_scatter32(v);  // lane l: the wave's sum of value l >> 1
    const int k = lane >> 1;
    if ((lane & 1) == 0 && k < nv) sdot[w * kNDX + k] = r;
  } else {  // (more than 14 stored pairs: one reduction per value)
    tt = wave_sum(tt);
    td = wave_sum(td);
    tc = wave_sum(tc);
    const double ls = wave_sum(lsum);
    if (lane == 0) {
      sdot[w * kNDX + 0] = tt;
      sdot[w * kNDX + 1] = td;
      sdot[w * kNDX + 2] = tc;
      sdot[w * kNDX + 3] = ls;
    }
    for (int j = 0; j < m; ++j) {  // wave-uniform loop over the stored pairs
      double si, yi;
      pair_dots(j, si, yi);
      si = wave_sum(si);
      yi = wave_sum(yi);
      if (lane == 0) {
        sdot[w * kNDX + 4 + 2 * j] = si;
        sdot[w * kNDX + 5 + 2 * j] = yi;
      }
    }
  }
  __syncthreads();
  if (wg0 && tid == 0) stamp(dv, slot, 12);
  // ---- all-gather of the partial dots as tagged granules (the data is its
  // own flag: R2 of the CDNA4 playbook).  Each workgroup stores its nv partial
  // sums as 2*nv 8-byte words {tag, 32-bit half of the fp64 value} with sc1
  // stores; every workgroup sweeps all slices' words with sc1 loads until each
  // carries this (run, slot)'s tag, which never repeats (no reset needed) ----
  const int ns = NS;
  // the slices share one XCD (one L2) unless the solver spreads them (cfg.xcd < 0)
  const bool xs2 = kXs == 2 && (kP == 2 || cfg.xcd >= 0);
  // only the m stored pairs' dots travel, in the order above
  const unsigned tag = run_tag + (unsigned)slot + 1u;
  unsigned* gat32 = (unsigned*)gat;  // [ns][2*nv]
  if (tid < 2 * nv) {
    const int k = tid >> 1;
    const double v = sdot[k] + sdot[kNDX + k] + sdot[2 * kNDX + k] + sdot[3 * kNDX + k];
    const unsigned long long u = d2u(v);
    const unsigned half = (tid & 1) ? (unsigned)(u >> 32) : (unsigned)u;
    if (ns > 1) {
      unsigned long long* dst = xch + (size_t)wg * (2 * kNDX) + tid;
      const unsigned long long v = ((unsigned long long)tag << 32) | half;
      if (xs2)
        st_h64<2>(dst, v);
      else
        st_h64<1>(dst, v);
    }
    else
      gat32[tid] = half;
  }
  wg_stamp(dv, slot, 2, wg);
  // The storing wave (wave 0) does not sweep: vmcnt retires in order, so its
  // loads would wait for its own write-through stores to complete.
  if (ns > 1 && tid >= 64) {
    const int total = ns * 2 * nv, st = tid - 64;
    for (int i0 = 0; i0 < total; i0 += 192 * 8) {
      unsigned long long x[8];
      int spins = 0;
      bool ok;
      do {  // all 8 loads of the sweep in flight, then check the tags
        ok = true;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int i = i0 + st + 192 * j;
          if (i < total) {
            const int b = i / (2 * nv), r = i - b * (2 * nv);
            x[j] = xs2 ? ld_h64<2>(xch + (size_t)b * (2 * kNDX) + r) : ld_h64<1>(xch + (size_t)b * (2 * kNDX) + r);
            ok &= (unsigned)(x[j] >> 32) == tag;
          }
        }
        if (!ok) {
          __builtin_amdgcn_s_sleep(1);
          if (++spins > spin_limit(dv)) {  // never expected: record and fall through rather than hang
            xstore(xch + kXchErr, 1ull);
            break;
          }
        }
      } while (!ok);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int i = i0 + st + 192 * j;
        if (i < total) gat32[i] = (unsigned)x[j];
      }
    }
  }
  __syncthreads();
  wg_stamp(dv, slot, 3, wg);
  if (wg0 && tid == 0) stamp(dv, slot, 13);
  if (tid < kNDX) dots[tid] = 0.0;  // pairs not stored stay 0
  __syncthreads();
  if (tid < nv) {
    double v = 0.0;
    for (int b = 0; b < ns; ++b) {  // fixed order: identical in every workgroup
      const unsigned long long u =
          (unsigned long long)gat32[b * 2 * nv + 2 * tid] | ((unsigned long long)gat32[b * 2 * nv + 2 * tid + 1] << 32);
      v += u2d(u);
    }
    // order expected by ctrl_step: 3 scalars, S_i.g (H ring slots), Y_i.g (H); loss in dots[kND]
    const int rr = hbase + ((tid - 4) >> 1), ring = tid < 4 ? 0 : (rr >= H ? rr - H : rr);
    const int pos = tid < 3 ? tid : (tid == 3 ? kND : (((tid - 4) & 1) == 0 ? 3 + ring : 3 + H + ring));
    dots[pos] = v;
  }
  __syncthreads();
  if (wg0 && tid == 0) stamp(dv, slot, 14);
  if (tid == 0) {
    if (wg0) stamp(dv, slot, 5);
    ctrl_step(*cl, cfg, dots[kND] / (double)B, dots, slot, *csw);
    cl->fin = (may_fin && cl->phase == kPhDone) ? 1 : 0;  // finalised by this launch (tail: scalars only)
    if (wg0) stamp(dv, slot, 6);
  }
  __syncthreads();
  if (kP == 0 && wg0) {  // the next launches read the controller from global memory
    constexpr int CW = sizeof(Ctrl) / 8;
    for (int i = tid; i < CW; i += 256) ((unsigned long long*)gctrl)[i] = ((const unsigned long long*)cl)[i];
  }
  if (wg0 && tid == 0) stamp(dv, slot, 7);

  // ---- apply the controller's action to this slice ----
  const int act = cl->action_slot == slot ? cl->action : kActNone;
  const bool done = cl->phase == kPhDone;
  const float t_next = (float)cl->t, t_acc = (float)cl->t_acc, cg = (float)cl->cg;
  const int ps = cl->push_slot;
  const bool accept = act == kActAccept || act == kActAcceptDone;
  const bool more = act == kActAccept;
  float dn[NE];
#pragma unroll
  for (int e = 0; e < NE; ++e) dn[e] = DD[e];
  float dbv = db0, xbv = xb0;
  const bool ib = wg0 && tid < 16;
  if (act == kActInit) {
#pragma unroll
    for (int e = 0; e < NE; ++e) {
      dn[e] = cg * g[e];
      if (own[e]) {
        dv.g_c[idx[e]] = g[e];
        dv.d[idx[e]] = dn[e];
      }
    }
    if (ib) {
      dbv = cg * gb;
      dv.g_c[IB + tid] = gb;
      dv.d[IB + tid] = dbv;
    }
  } else if (accept) {
#pragma unroll
    for (int e = 0; e < NE; ++e) {
      XO[e] += t_acc * DD[e];
      if (own[e]) {
        dv.x[idx[e]] = XO[e];
        if (more) {
          if (ps >= 0) {
            if constexpr (kP != 0) {
              lsy[2 * ps * kSyStride + (cgp + 8 * e) * 32 + fl] = t_acc * DD[e];
              lsy[(2 * ps + 1) * kSyStride + (cgp + 8 * e) * 32 + fl] = g[e] - GC[e];
            } else {
              dv.S[(size_t)ps * PI + idx[e]] = t_acc * DD[e];
              dv.Y[(size_t)ps * PI + idx[e]] = g[e] - GC[e];
            }
          }
          dv.g_c[idx[e]] = g[e];
        }
      }
      if (more) dn[e] = cg * g[e];
    }
    if (ib) {
      xbv = xb0 + t_acc * db0;
      dv.x[IB + tid] = xbv;
      if (more) {
        if (ps >= 0) {
          if constexpr (kP != 0) {
            lsy[2 * ps * kSyStride + 256 + tid] = t_acc * db0;
            lsy[(2 * ps + 1) * kSyStride + 256 + tid] = gb - gcb0;
          } else {
            dv.S[(size_t)ps * PI + IB + tid] = t_acc * db0;
            dv.Y[(size_t)ps * PI + IB + tid] = gb - gcb0;
          }
        }
        dv.g_c[IB + tid] = gb;
        dbv = cg * gb;
      }
    }
  }
  if (more) {  // new direction d = cg*g + sum_i cs_i S_i + cy_i Y_i
    for (int i = 0; i < H; ++i) {
      const float cs = (float)cl->cs[i], cy = (float)cl->cy[i];
      if (cs == 0.f && cy == 0.f) continue;  // uniform
      if (i == ps) {  // the pair pushed just now is still in registers
#pragma unroll
        for (int e = 0; e < NE; ++e) dn[e] += cs * (t_acc * DD[e]) + cy * (g[e] - GC[e]);
        if (ib) dbv += cs * (t_acc * db0) + cy * (gb - gcb0);
        continue;
      }
#pragma unroll
      for (int e = 0; e < NE; ++e) dn[e] += cs * s_at(i, e) + cy * y_at(i, e);
      if (ib) dbv += cs * sb_at(i) + cy * yb_at(i);
    }
#pragma unroll
    for (int e = 0; e < NE; ++e)
      if (own[e]) dv.d[idx[e]] = dn[e];
    if (ib) dv.d[IB + tid] = dbv;
  }
  // ---- the solve ended in this launch: finalise this slice in place (no
  // launch reads the fragments it rewrites: the riding evaluation workgroups
  // are all in launches before fin_slot) ----
  if (done && may_fin) {
    FinSl<KP> in;
    in.iv = iv;
#pragma unroll
    for (int e = 0; e < NE; ++e) {
      in.xv[e] = own[e] ? XO[e] : 0.f;
      in.fx[e] = own[e] ? FX[e] : 0.f;
      in.wo[e] = WO[e];
    }
    __syncthreads();  // gw (the gradient's LDS) is free: its last reads preceded the dots
    finalize_slice<KP>(cfg, dv, wg, in, gw, fin_sc1);
  }
  // ---- next trial point: this slice of the MFMA weight fragments (16-B stores) ----
  if (!done) {
#pragma unroll
    for (int e = 0; e < NE; ++e) {
      const int c = cgp + 8 * e;
      if (own[e]) {
        unsigned short h, l;
        split_bf16((XO[e] + t_next * dn[e]) * iv + FX[e], h, l);
        const int o = (fl >> 3) * 128 + c * 8 + (fl & 7);
        frl[o] = h;
        frl[512 + o] = l;
      }
    }
    if (ib) {
      if constexpr (kP != 0)
        st_h<kP>(dv.b_eff + tid, xbv + t_next * dbv);
      else
        dv.b_eff[tid] = xbv + t_next * dbv;
    }
    __syncthreads();
    if (tid < 128) {
      const size_t go = (size_t)(fs >> 3) * 128 + (tid & 63) * 8;
      uint16_t* dst = tid < 64 ? dv.whi : dv.wlo;
      if constexpr (kP != 0) {  // (wave-uniform buffer: wave 0 the hi, wave 1 the lo fragments)
        const u16x8 v = *(const u16x8*)(frl + tid * 8);
        if (tid < 64)
          st_h_b128<kP>(rsrc_of(dv.whi, 16u * FP * 2u), (unsigned)(go * 2), v);
        else
          st_h_b128<kP>(rsrc_of(dv.wlo, 16u * FP * 2u), (unsigned)(go * 2), v);
      } else
        *(u16x8*)(dst + go) = *(const u16x8*)(frl + tid * 8);
    }
  }
  if (wg0 && tid == 0) stamp(dv, slot, 8);
}

__device__ __forceinline__ void p_barrier(unsigned long long* ctr, unsigned long long target, unsigned long long* err,
                                          int spin_max = 1 << 22) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 stores
  __syncthreads();
  if (threadIdx.x == 0) {
    (void)__hip_atomic_fetch_add((g_u64*)ctr, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int spins = 0;
    while (xload(ctr) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > spin_max) {  // never expected: record and fall through rather than hang
        xstore(err, 3ull);
        break;
      }
    }
  }
  __syncthreads();
}

// The one-XCD form (S = 2): no read-modify-write (device memory's atomics run
// past the L2, 2 us at 32 workgroups): workgroup wg stores the arrival word
// (run << 16 | n) into its own 256-B flag line, and thread i of every workgroup
// polls workgroup i's line with nt loads (the L2 of the shared XCD), so all
// arrivals are observed in one round trip.  The words only grow over the runs
// (the run counter advances per solve): nothing is reset.
// drain = false: the workgroup publishes nothing through this barrier (its outstanding
// stores -- e.g. system-scope stores into pinned host memory -- need not complete first).
__device__ __forceinline__ void x_barrier(unsigned long long* flags, int wg, int G, unsigned long long word,
                                          unsigned long long* err, int spin_max = 1 << 22, bool drain = true) {
  if (drain) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave's stores reached the L2
  __syncthreads();
  if (threadIdx.x == 0) st_h64<2>(flags + (size_t)wg * 32, word);
  if ((int)threadIdx.x < G) {
    int spins = 0;
    while (ld_h64<2>(flags + (size_t)threadIdx.x * 32) < word) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > spin_max) {  // never expected: record and fall through rather than hang
        xstore(err, 5ull);
        break;
      }
    }
  }
  __syncthreads();
}

PSX_HD constexpr size_t persist_fwd_bytes(int FP) { return (eval_lds_bytes(FP) + 15) / 16 * 16; }

}  // namespace psx
