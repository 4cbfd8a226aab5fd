// Fused worker local-solve kernels (gfx950).
//
//   stats_prep_kernel : window statistics (per-feature mean/std, fp64) and the
//                       initial point x0 = w_old * std, one workgroup per 128
//                       features (no cross-workgroup reduction, deterministic).
//   slot_kernel       : ONE function evaluation of the line search:
//       eval part (all workgroups): 32-row tiles staged once in LDS, forward
//         Z = X W_eff^T on MFMA, softmax / cross entropy, backward G = R^T X on
//         MFMA through hardware-transposed LDS reads; partial G / intercept /
//         loss sums accumulate with no-return fp32 atomics (memory side);
//       tail (the LAST workgroup to arrive, split-K seam recipe): reads and
//         zeroes the sums, builds g_t in the standardised space plus the dot
//         products the L-BFGS controller needs, advances the controller on an
//         LDS copy (csrc/kernels/solver_ctrl.h), applies the accepted step /
//         curvature pair / new direction elementwise, writes W_eff for the
//         next trial, and when the controller is done finalises (unscale,
//         multinomial centring, delta, eval fragments).
// A local solve is therefore 1 + nslots launches in one hipGraph; slots after
// convergence exit on their first instruction.
//
// The tail is latency-bound (one workgroup), so it is written in explicit
// phases: every global load of a feature group is issued before any result
// is consumed and before any store (stores to possibly-aliasing vectors would
// otherwise pin each load behind the previous store), and the bf16 weight
// fragments are assembled in LDS and leave in 16-byte stores.
//
// Solver-private vectors use a padded layout so the tail's loops are
// branch-free (a guarded load/atomic makes hipcc wait vmcnt(0) per element):
// class count KP = next power of two >= K (compile time), feature stride
// FPI = max(FP, 256); coefficient (c, f) at c*FPI + f, intercept c at
// KP*FPI + c (c < 16).  Padded entries are identically zero.
//
// Reference semantics: LogisticRegressionTaskSpark.java:142-221 (Spark fit
// with setMaxIter(2), standardisation, centring, delta = w_new - w_old).
#include <hip/hip_runtime.h>

#include "lr_kernels.h"
#include "solve_kernels.h"
#include "tile.h"

namespace psx {

// Debug timeline (tools/bench_solver.py --stamps): s_memrealtime (100 MHz) per
// phase of slot `slot`, written by one lane; no effect when dv.dbg is null.
__device__ __forceinline__ void stamp(const SolveDev& dv, int slot, int k) {
  if (dv.dbg && slot < 31) dv.dbg[slot * 16 + k] = (long long)__builtin_amdgcn_s_memrealtime();
}

// ---------------------------------------------------------------------------
// stats + prep: grid = FP/128 workgroups of 1024 threads (16 chunks x 64 rows)
__global__ __launch_bounds__(1024) void stats_prep_kernel(SolverCfg cfg, const SolveParams* prm, SolveDev dv,
                                                          Ctrl* ctrl) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* rs = (float*)smem;   // [64][128]
  float* rq = rs + 64 * 128;  // [64][128]
  float* sdl = rq + 64 * 128; // [128]
  float* ivl = sdl + 128;     // [128]
  const int B = prm->B, start = prm->start, cap = cfg.cap, FP = cfg.Fp;
  const int t = threadIdx.x, ch = t & 15, rl = t >> 4;
  const int fb = blockIdx.x * 128;
  float s[8], q[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s[j] = q[j] = 0.f;
  for (int i0 = rl; i0 < B; i0 += 64 * 4) {
    u16x8 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = i0 + 64 * u;
      int r = start + (i < B ? i : 0);
      if (r >= cap) r -= cap;
      v[u] = *(const u16x8*)(dv.X + (size_t)r * FP + fb + ch * 8);
      if (i >= B) v[u] = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float x = bf2f(v[u][j]);
        s[j] += x;
        q[j] += x * x;
      }
  }
  // fold the 4 row lanes of each wave with shuffles, then 16 waves through LDS
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    s[j] += __shfl_xor(s[j], 16, 64);
    s[j] += __shfl_xor(s[j], 32, 64);
    q[j] += __shfl_xor(q[j], 16, 64);
    q[j] += __shfl_xor(q[j], 32, 64);
  }
  const int wv = t >> 6;
  if ((t & 63) < 16) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      rs[wv * 128 + ch * 8 + j] = s[j];
      rq[wv * 128 + ch * 8 + j] = q[j];
    }
  }
  (void)rl;
  __syncthreads();
  if (t < 128) {
    double a = 0.0, b = 0.0;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      a += rs[r * 128 + t];
      b += rq[r * 128 + t];
    }
    const int f = fb + t;
    const double n = (double)B;
    double sd = 0.0;
    if (f < cfg.F && n > 1.0) {
      const double mean = a / n;
      const double var = (b - n * mean * mean) / (n - 1.0);
      sd = var > 0.0 ? sqrt(var) : 0.0;
    }
    const float sdf = (float)sd, inv = sd > 0.0 ? (float)(1.0 / sd) : 0.f;
    sdl[t] = sdf;
    ivl[t] = inv;
    dv.std_[f] = sdf;
    dv.inv_std[f] = inv;
  }
  __syncthreads();
  const int K = cfg.K, KP = dv.KP, FPI = dv.FPI;
  for (int e = t; e < 128 * KP; e += 1024) {
    const int c = e >> 7, fl = e & 127, f = fb + fl;
    const int pi = c * FPI + f;
    const float wo = (c < K && f < cfg.F) ? dv.w_old[c * FP + f] : 0.f;
    const float xv = wo * sdl[fl];
    dv.x[pi] = xv;
    dv.d[pi] = 0.f;
    dv.g_c[pi] = 0.f;
    const float fix = (sdl[fl] > 0.f || cfg.zero_const) ? 0.f : wo;
    dv.wfix[pi] = fix;
    write_frag(dv.whi, dv.wlo, c, f, xv * ivl[fl] + fix);
  }
  if (blockIdx.x == 0) {
    if (t < 16) {
      const int pi = KP * FPI + t;
      const float b = t < K ? dv.w_old[K * FP + t] : 0.f;
      dv.x[pi] = b;
      dv.d[pi] = 0.f;
      dv.g_c[pi] = 0.f;
      dv.b_eff[t] = b;
    }
    if (t == 0) ctrl_init(*ctrl);
  }
}

// ---------------------------------------------------------------------------
// LDS layout of the tail: [Ctrl copy] [dots] [controller workspace]
constexpr size_t ctrl_lds_bytes() { return ((sizeof(Ctrl) + 15) / 16) * 16; }
constexpr int kND = 3 + 2 * kMaxHist;

// N consecutive floats <-> registers with the widest vector accesses.
template <int N>
__device__ __forceinline__ void vload(float (&d)[N], const float* __restrict__ p) {
  if constexpr (N % 4 == 0) {
#pragma unroll
    for (int i = 0; i < N / 4; ++i) {
      const float4 t = *(const float4*)(p + 4 * i);
      d[4 * i] = t.x;
      d[4 * i + 1] = t.y;
      d[4 * i + 2] = t.z;
      d[4 * i + 3] = t.w;
    }
  } else if constexpr (N == 2) {
    const float2 t = *(const float2*)p;
    d[0] = t.x;
    d[1] = t.y;
  } else {
#pragma unroll
    for (int i = 0; i < N; ++i) d[i] = p[i];
  }
}

template <int N>
__device__ __forceinline__ void vstore(float* __restrict__ p, const float (&s)[N]) {
  if constexpr (N % 4 == 0) {
#pragma unroll
    for (int i = 0; i < N / 4; ++i) *(float4*)(p + 4 * i) = make_float4(s[4 * i], s[4 * i + 1], s[4 * i + 2], s[4 * i + 3]);
  } else if constexpr (N == 2) {
    *(float2*)p = make_float2(s[0], s[1]);
  } else {
#pragma unroll
    for (int i = 0; i < N; ++i) p[i] = s[i];
  }
}

// Write N consecutive features (f0 % N == 0, N <= 8) of class c into the MFMA
// fragment layout: they sit in one 16-B chunk, so this is one store per array.
template <int N>
__device__ __forceinline__ void frag_store(uint16_t* hi, uint16_t* lo, int c, int f0, const float (&v)[N]) {
  unsigned short h[N], l[N];
#pragma unroll
  for (int i = 0; i < N; ++i) split_bf16(v[i], h[i], l[i]);
  const size_t o = ((size_t)(f0 >> 3) * 16 + c) * 8 + (f0 & 7);
  if constexpr (N == 8) {
    *(u16x8*)(hi + o) = u16x8{h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7]};
    *(u16x8*)(lo + o) = u16x8{l[0], l[1], l[2], l[3], l[4], l[5], l[6], l[7]};
  } else if constexpr (N == 4) {
    *(u16x4*)(hi + o) = u16x4{h[0], h[1], h[2], h[3]};
    *(u16x4*)(lo + o) = u16x4{l[0], l[1], l[2], l[3]};
  } else {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      hi[o + i] = h[i];
      lo[o + i] = l[i];
    }
  }
}

// The tail.  Thread t owns the FPT consecutive features [t*FPT, t*FPT+FPT) of
// every class (and intercept t when t < 16), so every vector access is a 16-B
// (or 8-B) per-lane load/store: the single tail workgroup is bound by memory
// instructions in flight, and wide accesses move 4x the bytes per instruction.
template <int FP, int KP>
__device__ __forceinline__ void solve_tail(const SolverCfg& cfg, const SolveParams* prm, Ctrl* gctrl, int slot,
                                           const SolveDev& dv, char* lds) {
  constexpr int FPI = FP > 256 ? FP : 256;
  constexpr int FPT = FPI / 256;  // consecutive features owned per thread
  constexpr int IB = KP * FPI;    // internal intercept base
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int f0 = tid * FPT;
  const int K = cfg.K, H = cfg.hist;
  const size_t PI = dv.PI;
  Ctrl* cl = (Ctrl*)lds;
  double* sdot = (double*)(lds + ctrl_lds_bytes());  // [4 waves][kND]
  double* dots = sdot + 4 * kND;
  CtrlScratch* csw = (CtrlScratch*)(dots + kND);  // controller workspace (LDS)
  // ---- 0) controller to LDS; read-and-zero the sums; every per-element input ----
  constexpr int CW = sizeof(Ctrl) / 8;
  {
    const unsigned long long* src = (const unsigned long long*)gctrl;
    unsigned long long* dst = (unsigned long long*)cl;
    for (int i = tid; i < CW; i += 256) dst[i] = src[i];
  }
  float g[KP][FPT];
#pragma unroll
  for (int c = 0; c < KP; ++c)
#pragma unroll
    for (int j = 0; j < FPT; ++j)
      g[c][j] = __hip_atomic_exchange(dv.Gacc + c * FPI + f0 + j, 0.f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  float gb = 0.f;
  if (tid < 16) gb = __hip_atomic_exchange(dv.Racc + tid, 0.f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  float DD[KP][FPT], GC[KP][FPT], XO[KP][FPT], FX[KP][FPT], ivs[FPT];
  vload<FPT>(ivs, dv.inv_std + f0);
#pragma unroll
  for (int c = 0; c < KP; ++c) {
    vload<FPT>(DD[c], dv.d + c * FPI + f0);
    vload<FPT>(GC[c], dv.g_c + c * FPI + f0);
    vload<FPT>(XO[c], dv.x + c * FPI + f0);
    vload<FPT>(FX[c], dv.wfix + c * FPI + f0);
  }
  float db0 = 0.f, gcb0 = 0.f, xb0 = 0.f;
  if (tid < 16) {
    db0 = dv.d[IB + tid];
    gcb0 = dv.g_c[IB + tid];
    xb0 = dv.x[IB + tid];
  }
  __syncthreads();  // controller copy complete
  const int m = cl->m, head = cl->head;
  const float invB = 1.f / (float)prm->B;
  if (tid == 0) stamp(dv, slot, 3);
  // ---- 1) gradient in the standardised space + dot products ----
  double tt = 0.0, td = 0.0, tc = 0.0;
#pragma unroll
  for (int c = 0; c < KP; ++c)
#pragma unroll
    for (int j = 0; j < FPT; ++j) {
      const float gv = g[c][j] * invB * ivs[j];
      g[c][j] = gv;
      tt += (double)gv * gv;
      td += (double)gv * DD[c][j];
      tc += (double)gv * GC[c][j];
    }
  if (tid < 16) {
    gb *= invB;
    tt += (double)gb * gb;
    td += (double)gb * db0;
    tc += (double)gb * gcb0;
  }
  tt = wave_sum(tt);
  td = wave_sum(td);
  tc = wave_sum(tc);
  if (lane == 0) {
    sdot[w * kND + 0] = tt;
    sdot[w * kND + 1] = td;
    sdot[w * kND + 2] = tc;
  }
  for (int i = 0; i < H; ++i) {  // wave-uniform loop over stored pairs
    const bool valid = m > 0 && (m == H || (((i - (head - m + 1)) % H + H) % H) < m);
    double si = 0.0, yi = 0.0;
    if (valid) {
      const float* Si = dv.S + (size_t)i * PI;
      const float* Yi = dv.Y + (size_t)i * PI;
      float sv[KP][FPT], yv[KP][FPT];
#pragma unroll
      for (int c = 0; c < KP; ++c) {
        vload<FPT>(sv[c], Si + c * FPI + f0);
        vload<FPT>(yv[c], Yi + c * FPI + f0);
      }
#pragma unroll
      for (int c = 0; c < KP; ++c)
#pragma unroll
        for (int j = 0; j < FPT; ++j) {
          si += (double)sv[c][j] * g[c][j];
          yi += (double)yv[c][j] * g[c][j];
        }
      if (tid < 16) {
        si += (double)Si[IB + tid] * gb;
        yi += (double)Yi[IB + tid] * gb;
      }
      si = wave_sum(si);
      yi = wave_sum(yi);
    }
    if (lane == 0) {
      sdot[w * kND + 3 + i] = si;
      sdot[w * kND + 3 + H + i] = yi;
    }
  }
  __syncthreads();
  if (tid < 3 + 2 * H) dots[tid] = sdot[tid] + sdot[kND + tid] + sdot[2 * kND + tid] + sdot[3 * kND + tid];
  __syncthreads();
  if (tid == 0) {
    const float L = __hip_atomic_exchange(dv.Lacc, 0.f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    stamp(dv, slot, 4);
    ctrl_step(*cl, cfg, (double)L / (double)prm->B, dots, slot, *csw);
    stamp(dv, slot, 5);
  }
  __syncthreads();
  // ---- 2) apply the controller's action ----
  const int act = cl->action_slot == slot ? cl->action : kActNone;
  const bool done = cl->phase == kPhDone;
  const float t_next = (float)cl->t, t_acc = (float)cl->t_acc, cg = (float)cl->cg;
  const int ps = cl->push_slot;
  const bool accept = act == kActAccept || act == kActAcceptDone;
  const bool more = act == kActAccept;
  float (&xv)[KP][FPT] = XO;  // updated in place
  float (&dn)[KP][FPT] = DD;  // DD holds the previous direction until overwritten
  float dold[KP][FPT];
#pragma unroll
  for (int c = 0; c < KP; ++c)
#pragma unroll
    for (int j = 0; j < FPT; ++j) dold[c][j] = DD[c][j];
  if (act == kActInit) {
#pragma unroll
    for (int c = 0; c < KP; ++c) {
#pragma unroll
      for (int j = 0; j < FPT; ++j) dn[c][j] = cg * g[c][j];
      vstore<FPT>(dv.g_c + c * FPI + f0, g[c]);
      vstore<FPT>(dv.d + c * FPI + f0, dn[c]);
    }
  } else if (accept) {
#pragma unroll
    for (int c = 0; c < KP; ++c) {
#pragma unroll
      for (int j = 0; j < FPT; ++j) xv[c][j] += t_acc * dold[c][j];
      vstore<FPT>(dv.x + c * FPI + f0, xv[c]);
      if (more) {
        if (ps >= 0) {
          float sn[FPT], yn[FPT];
#pragma unroll
          for (int j = 0; j < FPT; ++j) {
            sn[j] = t_acc * dold[c][j];
            yn[j] = g[c][j] - GC[c][j];
          }
          vstore<FPT>(dv.S + (size_t)ps * PI + c * FPI + f0, sn);
          vstore<FPT>(dv.Y + (size_t)ps * PI + c * FPI + f0, yn);
        }
        vstore<FPT>(dv.g_c + c * FPI + f0, g[c]);
#pragma unroll
        for (int j = 0; j < FPT; ++j) dn[c][j] = cg * g[c][j];
      }
    }
  }
  float dbv = db0, xbv = xb0;
  if (tid < 16) {
    if (act == kActInit) {
      dbv = cg * gb;
      dv.g_c[IB + tid] = gb;
      dv.d[IB + tid] = dbv;
    } else if (accept) {
      xbv = xb0 + t_acc * db0;
      dv.x[IB + tid] = xbv;
      if (more) {
        if (ps >= 0) {
          dv.S[(size_t)ps * PI + IB + tid] = t_acc * db0;
          dv.Y[(size_t)ps * PI + IB + tid] = gb - gcb0;
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
        for (int c = 0; c < KP; ++c)
#pragma unroll
          for (int j = 0; j < FPT; ++j) dn[c][j] += cs * (t_acc * dold[c][j]) + cy * (g[c][j] - GC[c][j]);
        if (tid < 16) dbv += cs * (t_acc * db0) + cy * (gb - gcb0);
        continue;
      }
      const float* Si = dv.S + (size_t)i * PI;
      const float* Yi = dv.Y + (size_t)i * PI;
      float sv[KP][FPT], yv[KP][FPT];
#pragma unroll
      for (int c = 0; c < KP; ++c) {
        vload<FPT>(sv[c], Si + c * FPI + f0);
        vload<FPT>(yv[c], Yi + c * FPI + f0);
      }
#pragma unroll
      for (int c = 0; c < KP; ++c)
#pragma unroll
        for (int j = 0; j < FPT; ++j) dn[c][j] += cs * sv[c][j] + cy * yv[c][j];
      if (tid < 16) dbv += cs * Si[IB + tid] + cy * Yi[IB + tid];
    }
#pragma unroll
    for (int c = 0; c < KP; ++c) vstore<FPT>(dv.d + c * FPI + f0, dn[c]);
    if (tid < 16) dv.d[IB + tid] = dbv;
  }
  if (tid == 0) stamp(dv, slot, 6);
  // ---- 3) next trial point as MFMA weight fragments (finalize_kernel runs
  //         after the last slot when the controller is done) ----
  if (!done) {
    if (f0 < FP) {
#pragma unroll
      for (int c = 0; c < KP; ++c) {
        float v[FPT];
#pragma unroll
        for (int j = 0; j < FPT; ++j) v[j] = (xv[c][j] + t_next * dn[c][j]) * ivs[j] + FX[c][j];
        if constexpr (FPT <= 8) frag_store<FPT>(dv.whi, dv.wlo, c, f0, v);
      }
    }
    if (tid < 16) dv.b_eff[tid] = xbv + t_next * dbv;
  }
  if (tid == 0) stamp(dv, slot, 7);
  // ---- controller back to global memory (ticket re-armed) ----
  if (tid == 0) cl->ticket = 0;
  __syncthreads();
  {
    const unsigned long long* src = (const unsigned long long*)cl;
    unsigned long long* dst = (unsigned long long*)gctrl;
    for (int i = tid; i < CW; i += 256) dst[i] = src[i];
  }
}

// ---------------------------------------------------------------------------
template <int FP, int KP>
__global__ __launch_bounds__(256) void slot_kernel(SolverCfg cfg, const SolveParams* prm, Ctrl* ctrl, int slot,
                                                   SolveDev dv) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  constexpr int NTW = FP / 64;  // 16-feature N-tiles per wave in the backward
  constexpr int FPI = FP > 256 ? FP : 256;
  if (ctrl->phase == kPhDone) return;  // converged in an earlier slot: exit at once
  if (blockIdx.x == 0 && threadIdx.x == 0) stamp(dv, slot, 0);
  const int B = prm->B, start = prm->start, cap = cfg.cap, K = cfg.K;
  const int ntiles = (B + 31) / 32;
  char* red_base = lds + 32 * FP * 2;
  unsigned short* rt = (unsigned short*)(red_base + 8192);  // [2][16][32]
  int* ylds = (int*)(red_base + 8192 + 2048);
  float* rsum = (float*)(ylds + 32);
  float* lred = rsum + 16;
  int* flag = (int*)(lred + 4);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;

  if ((int)blockIdx.x < ntiles) {
    if (tid < 16) rsum[tid] = 0.f;
    f32x4 accb[NTW];
#pragma unroll
    for (int j = 0; j < NTW; ++j) accb[j] = f32x4{0, 0, 0, 0};
    float loss = 0.f;
    const int sr = tid >> 3, sc0 = (tid & 7) * 2;
    float rs0 = 0.f, rs1 = 0.f;
    const float bz0 = dv.b_eff[sc0], bz1 = dv.b_eff[sc0 + 1];
    // the trial weights do not depend on the tile: fetch them before staging so
    // the two memory latencies overlap (register budget allows it up to FP 1024)
    constexpr bool kPre = FP <= 1024;
    WFrag<kPre ? FP : 128> wf;
    if constexpr (kPre) load_wfrag<FP>(wf, dv.whi, dv.wlo);
    for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
      const int nrows = min(32, B - tile * 32);
      int64_t row0 = (int64_t)start + (int64_t)tile * 32;
      if (row0 >= cap) row0 -= cap;
      stage_tile<FP>(lds, dv.X, row0, nrows, cap, true);
      if (tid < 32) {
        int yy = 0;
        if (tid < nrows) {
          int64_t r = row0 + tid;
          if (r >= cap) r -= cap;
          yy = dv.y[r];
        }
        ylds[tid] = yy;
      }
      __syncthreads();
      if (blockIdx.x == 0 && tid == 0) stamp(dv, slot, 9);
      f32x4 a0, a1;
      if constexpr (kPre)
        forward_tile_pre<FP>(lds, wf, a0, a1);
      else
        forward_tile<FP>(lds, dv.whi, dv.wlo, a0, a1);
      store_partial_logits(red_base, a0, a1);
      __syncthreads();
      if (blockIdx.x == 0 && tid == 0) stamp(dv, slot, 10);
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
        const bool valid = sr < nrows;
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
      if (blockIdx.x == 0 && tid == 0) stamp(dv, slot, 11);
      {  // backward G[c][f] += sum_r R[r][c] X[r][f] (M = classes, N = features, K = rows)
        const u16x8 ah = *(const u16x8*)(rt + (lane & 15) * 32 + (lane >> 4) * 8);
        const u16x8 al = *(const u16x8*)(rt + 512 + (lane & 15) * 32 + (lane >> 4) * 8);
        const int gq = lane >> 4, il = lane & 15, q = il >> 2, pp = il & 3;
#pragma unroll
        for (int j = 0; j < NTW; ++j) {
          const int nt = w * NTW + j, f0 = nt * 16;
          const int sub = f0 >> 7, c0 = (f0 & 127) >> 3;
          const int chk = c0 + (pp >> 1), inb = 8 * (pp & 1);
          const char* base = lds + sub * 8192;
          const s16x4 b0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) s16x4*)(base + lds_off(8 * gq + q, chk) + inb));
          const s16x4 b1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) s16x4*)(base + lds_off(8 * gq + 4 + q, chk) + inb));
          u16x8 bv;
          bv[0] = b0[0]; bv[1] = b0[1]; bv[2] = b0[2]; bv[3] = b0[3];
          bv[4] = b1[0]; bv[5] = b1[1]; bv[6] = b1[2]; bv[7] = b1[3];
          accb[j] = mfma16x16x32(as_bf16x8(ah), as_bf16x8(bv), accb[j]);
          accb[j] = mfma16x16x32(as_bf16x8(al), as_bf16x8(bv), accb[j]);
        }
      }
      __syncthreads();
      if (blockIdx.x == 0 && tid == 0) stamp(dv, slot, 12);
    }
    // ---- accumulate partial sums (no-return fp32 atomics at the memory side) ----
    // The accumulator fragments hold 4 class rows x 16 features per lane group,
    // half of them padding for K = 6; transposing through LDS turns them into
    // K*FP/64 fully populated wave-instructions of 256 contiguous bytes each
    // (the shape the memory-side atomic units serve at full rate).
    float* gs = (float*)lds;  // [K][FP] (the X image is no longer needed)
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
      const int f = (w * NTW + j) * 16 + (lane & 15);
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int c = (lane >> 4) * 4 + rr;
        if (c < K) gs[c * FP + f] = accb[j][rr];
      }
    }
    atomicAdd(&rsum[sc0], rs0);
    atomicAdd(&rsum[sc0 + 1], rs1);
    loss = wave_sum(loss);
    if (lane == 0) lred[w] = loss;
    __syncthreads();
    for (int e = tid; e < K * FP; e += 256) {
      const int c = e / FP, f = e - c * FP;
      atomicAdd(dv.Gacc + c * FPI + f, gs[e]);
    }
    if (tid < K) atomicAdd(dv.Racc + tid, rsum[tid]);
    if (tid == 0) atomicAdd(dv.Lacc, lred[0] + lred[1] + lred[2] + lred[3]);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) stamp(dv, slot, 1);
  // ---- arrival ----
  // Every wave drains its no-return atomics (vmcnt counts them until the memory
  // side has performed them), then one lane takes a ticket.  No agent release /
  // acquire pair is needed: this launch publishes nothing through plain
  // stores -- the tail consumes only memory-side atomic sums (read back with
  // atomic exchanges) and data written by EARLIER launches (kernel-boundary
  // visibility); the eval part never reads a line the tail writes.
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    const unsigned prev = __hip_atomic_fetch_add(&ctrl->ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = prev == gridDim.x - 1;
  }
  __syncthreads();
  if (!*flag) return;
  if (tid == 0) stamp(dv, slot, 2);
  solve_tail<FP, KP>(cfg, prm, ctrl, slot, dv, lds);
  if (tid == 0) stamp(dv, slot, 8);
}

// ---------------------------------------------------------------------------
// Finalisation (after the last slot): back to the unstandardised space,
// multinomial centring across classes, delta = w_new - w_old, eval fragments,
// loss and solver statistics.  One thread per feature (all classes).
template <int KP>
__global__ __launch_bounds__(256) void finalize_kernel(SolverCfg cfg, const Ctrl* ctrl, SolveDev dv) {
  const int FP = cfg.Fp, FPI = dv.FPI, K = cfg.K;
  const int f = blockIdx.x * 256 + threadIdx.x;
  if (f < FP) {
    const float iv = dv.inv_std[f];
    float xv[KP], fx[KP], wo[KP];
#pragma unroll
    for (int c = 0; c < KP; ++c) {
      xv[c] = dv.x[c * FPI + f];
      fx[c] = dv.wfix[c * FPI + f];
      wo[c] = (c < K && f < cfg.F) ? dv.w_old[c * FP + f] : 0.f;
    }
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
        dv.delta[c * FP + f] = v - wo[c];
        if (dv.w_new) dv.w_new[c * FP + f] = v;
      }
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    const int IB = dv.KP * FPI;
    float bv[16];
    float mean = 0.f;
    for (int c = 0; c < K; ++c) {
      bv[c] = dv.x[IB + c];
      mean += bv[c];
    }
    mean = cfg.center ? mean / (float)K : 0.f;
    const int KF = K * FP;
    for (int c = 0; c < K; ++c) {
      const float v = bv[c] - mean;
      dv.delta[KF + c] = v - dv.w_old[KF + c];
      if (dv.w_new) dv.w_new[KF + c] = v;
      dv.b_fin[c] = v;
    }
    *dv.loss = (float)ctrl->f_c;
    if (dv.stats) {
      dv.stats[0] = ctrl->evals;
      dv.stats[1] = ctrl->nacc;
      dv.stats[2] = ctrl->ls_fail;
      dv.stats[3] = ctrl->dir_reset;
    }
  }
}

void launch_finalize(const SolverCfg& cfg, const Ctrl* ctrl, const SolveDev& dv, hipStream_t s) {
  const int grid = (cfg.Fp + 255) / 256;
  switch (dv.KP) {
    case 2: finalize_kernel<2><<<grid, 256, 0, s>>>(cfg, ctrl, dv); break;
    case 4: finalize_kernel<4><<<grid, 256, 0, s>>>(cfg, ctrl, dv); break;
    case 8: finalize_kernel<8><<<grid, 256, 0, s>>>(cfg, ctrl, dv); break;
    default: finalize_kernel<16><<<grid, 256, 0, s>>>(cfg, ctrl, dv); break;
  }
}

// ---------------------------------------------------------------------------
size_t stats_prep_lds_bytes() { return (size_t)(2 * 64 * 128 + 256) * sizeof(float); }

void launch_stats_prep(const SolverCfg& cfg, const SolveParams* prm, const SolveDev& dv, Ctrl* ctrl, hipStream_t s) {
  stats_prep_kernel<<<cfg.Fp / 128, 1024, stats_prep_lds_bytes(), s>>>(cfg, prm, dv, ctrl);
}

size_t slot_lds_bytes(int FP) {
  size_t a = eval_lds_bytes(FP);
  size_t b = 2 * (size_t)16 * FP * 2 + ctrl_lds_bytes() + 5 * kND * sizeof(double) + sizeof(CtrlScratch) + 64;
  return a > b ? a : b;
}

int padded_classes(int K) { return K <= 2 ? 2 : K <= 4 ? 4 : K <= 8 ? 8 : 16; }
int padded_stride(int FP) { return FP > 256 ? FP : 256; }

template <int FP>
static void launch_slot_fp(const SolverCfg& cfg, const SolveParams* prm, Ctrl* ctrl, int slot, const SolveDev& dv,
                           int nwg, size_t lds, hipStream_t s) {
  switch (dv.KP) {
    case 2: slot_kernel<FP, 2><<<nwg, 256, lds, s>>>(cfg, prm, ctrl, slot, dv); break;
    case 4: slot_kernel<FP, 4><<<nwg, 256, lds, s>>>(cfg, prm, ctrl, slot, dv); break;
    case 8: slot_kernel<FP, 8><<<nwg, 256, lds, s>>>(cfg, prm, ctrl, slot, dv); break;
    default: slot_kernel<FP, 16><<<nwg, 256, lds, s>>>(cfg, prm, ctrl, slot, dv); break;
  }
}

void launch_slot(const SolverCfg& cfg, const SolveParams* prm, Ctrl* ctrl, int slot, const SolveDev& dv, int nwg,
                 hipStream_t s) {
  const size_t lds = slot_lds_bytes(cfg.Fp);
  switch (cfg.Fp) {
    case 128: launch_slot_fp<128>(cfg, prm, ctrl, slot, dv, nwg, lds, s); break;
    case 256: launch_slot_fp<256>(cfg, prm, ctrl, slot, dv, nwg, lds, s); break;
    case 512: launch_slot_fp<512>(cfg, prm, ctrl, slot, dv, nwg, lds, s); break;
    case 1024: launch_slot_fp<1024>(cfg, prm, ctrl, slot, dv, nwg, lds, s); break;
    case 2048: launch_slot_fp<2048>(cfg, prm, ctrl, slot, dv, nwg, lds, s); break;
    default: break;
  }
}

template <int FP>
static void set_slot_attr() {
  const int b = (int)slot_lds_bytes(FP);
  (void)hipFuncSetAttribute((const void*)slot_kernel<FP, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, b);
  (void)hipFuncSetAttribute((const void*)slot_kernel<FP, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, b);
  (void)hipFuncSetAttribute((const void*)slot_kernel<FP, 8>, hipFuncAttributeMaxDynamicSharedMemorySize, b);
  (void)hipFuncSetAttribute((const void*)slot_kernel<FP, 16>, hipFuncAttributeMaxDynamicSharedMemorySize, b);
}

void prepare_solve_kernels() {
  static bool done = false;
  if (done) return;
  set_slot_attr<128>();
  set_slot_attr<256>();
  set_slot_attr<512>();
  set_slot_attr<1024>();
  set_slot_attr<2048>();
  (void)hipFuncSetAttribute((const void*)stats_prep_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)stats_prep_lds_bytes());
  done = true;
}

}  // namespace psx
