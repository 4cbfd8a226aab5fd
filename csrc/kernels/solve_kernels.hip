// Worker local-solve kernels (gfx950).
//
//   stats_prep_kernel : window statistics (per-feature mean/std, fp64) and the
//                       initial point x0 = w_old * std; one workgroup per
//                       32-feature slice.
//   per line-search slot, two launches:
//   fwd_kernel        : ROW-parallel.  Each workgroup owns whole 32-row tiles:
//                       stage in LDS, forward Z = X W_eff^T on MFMA (bf16 hi/lo
//                       weights), softmax / cross entropy.  The residuals
//                       R = softmax - onehot leave as bf16 hi/lo tiles already
//                       in the MFMA A-operand layout (2 KB per tile), plus
//                       per-workgroup intercept-gradient / loss partials.
//   bwd_update_kernel : FEATURE-parallel.  Each workgroup owns a 32-feature
//                       slice of every class for ALL rows: G = R^T X on MFMA,
//                       fed from the feature-major ring copy XT, needs no
//                       cross-workgroup reduction; only the handful of dot
//                       products the L-BFGS controller needs cross workgroups
//                       (one all-gather: write-through stores + an arrival
//                       counter).  Every workgroup then advances its own copy
//                       of the (deterministic) controller (csrc/kernels/
//                       solver_ctrl.h) -- no decision broadcast -- applies it
//                       to its slice and writes that slice of the next trial
//                       point's MFMA weight fragments.
//   finalize_kernel   : unscale, multinomial centring, delta, eval fragments.
// A local solve is 2 + 2*nslots launches captured in one hipGraph; slots after
// convergence exit on their first instruction.  The ring capacity is a multiple
// of 32 and the window is processed as ring-aligned 32-row tiles (WinTiles), so
// every tile and every 8-row XT fragment is contiguous (no wrap inside a tile).
//
// Solver-private vectors use a padded layout: class count KP = next power of
// two >= K (compile time), feature stride FPI = max(FP, 256); coefficient
// (c, f) at c*FPI + f, intercept c at KP*FPI + c (c < 16).  Padded entries are
// identically zero.
//
// Reference semantics: LogisticRegressionTaskSpark.java:142-221 (Spark fit
// with setMaxIter(2), standardisation, centring, delta = w_new - w_old).
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "eval_body.h"
#include "lr_kernels.h"
#include "solve_kernels.h"
#include "tile.h"
#include "solve_body.h"

namespace psx {

int xch_words() { return kXchFlags + 32 * kMaxXcdWg; }
// ---------------------------------------------------------------------------
// stats + prep: grid = FP/kStatW workgroups of 256 threads; kStatL = 256/kStatW
// lanes per feature read the feature-major ring copy XT in contiguous 16-B
// pieces of 8 rows (8 features per workgroup: 128 workgroups for FP 1024, each
// with few loads per lane, so the window read is not latency-serialised).
constexpr int kStatW = 8;
constexpr int kStatL = 256 / kStatW;
// Shared tail of the window-statistics kernels: rs / rq (LDS) hold the kStatW
// features' column sums and sums of squares over the window; derive std /
// 1/std, the initial point x0 = w_old * std (Spark standardisation), reset the
// solver vectors, write the first trial fragments and initialise the controller.
__device__ __forceinline__ void prep_epilogue(const SolverCfg& cfg, const SolveDev& dv, Ctrl* ctrl, int B, int fs,
                                              const double* rs, const double* rq, float* sdl, float* ivl, float wo_pre,
                                              float b_pre) {
  const int t = threadIdx.x;
  if (t < kStatW) {
    const double a = rs[t];
    const double b = rq[t];
    const int f = fs + t;
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
  static_assert(kStatW * 16 <= 256, "one element per thread");
  if (t < kStatW * KP) {
    const int e = t;
    const int c = e / kStatW, fl = e % kStatW, f = fs + fl;
    const int pi = c * FPI + f;
    const float wo = wo_pre;
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
      const float b = b_pre;
      dv.x[pi] = b;
      dv.d[pi] = 0.f;
      dv.g_c[pi] = 0.f;
      dv.b_eff[t] = b;
    }
    if (t == 32) ctrl_init(*ctrl);
    if (t == 0) stamp(dv, 30, 1);
    if (t == 65) xstore(dv.xch + kXchBar, 0ull);
  }
}

// With a fused ingest (ing.n > 0) each workgroup first copies its kStatW-feature
// slice of the new rows into X / XT (and workgroup 0 the labels); the new rows'
// statistics come from an LDS copy, the old rows' from XT as before.
__global__ __launch_bounds__(256) void stats_prep_kernel(SolverCfg cfg, SolveParams* prm, SolveDev dv, Ctrl* ctrl,
                                                         int B_arg, int start_arg, RingIngest ing) {
  static_assert(kStatW == 8, "the ingest copy moves one 16-B chunk (8 features) per row");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  double* rs = (double*)smem;          // [kStatW]
  double* rq = rs + kStatW;            // [kStatW]
  float* sdl = (float*)(rq + kStatW);  // [kStatW]
  float* ivl = sdl + kStatW;           // [kStatW]
  unsigned short* nv = (unsigned short*)(ivl + kStatW);  // [kMaxFusedIngest][kStatW] new rows of this slice
  // this run's window arrives as kernel arguments (the host rewrites this graph
  // node's parameters per run); later launches read it from device memory
  const SolveParams pr{B_arg, start_arg, 0, 0};
  const int B = pr.B, cap = cfg.cap, FP = cfg.Fp;
  const WinTiles wt(pr.start, B, cap);
  const int t = threadIdx.x, j = t % kStatL, fl0 = t / kStatL;
  if (blockIdx.x == 0 && t == 0) *prm = pr;  // the later launches read it from device memory
  if (blockIdx.x == 0 && t == 0) stamp(dv, 30, 0);
  // XCD-aware slice order: workgroups are dealt round-robin over the 8 XCDs, so
  // workgroup b takes slice (b % 8) * (G / 8) + b / 8 -- each XCD owns a
  // contiguous feature range and fetches every 128-B line of the new rows
  // once, instead of all 8 XCDs fetching each line for their 8-feature pieces
  const int G = gridDim.x;
  const int sl = (G & 7) == 0 ? (int)(blockIdx.x & 7) * (G >> 3) + (int)(blockIdx.x >> 3) : (int)blockIdx.x;
  const int fs = sl * kStatW;
  const int nin = ing.n;
  // the pulled weights were just written by the server update: fetch them now so
  // their latency overlaps the window read (one element per thread: kStatW*KP <= 256)
  const int KP0 = dv.KP;
  float wo_pre = 0.f, b_pre = 0.f;
  if (t < kStatW * KP0) {
    const int c = t / kStatW, f = fs + t % kStatW;
    if (c < cfg.K && f < cfg.F) wo_pre = dv.w_old[c * FP + f];
  }
  if (blockIdx.x == 0 && t < 16 && t < cfg.K) b_pre = dv.w_old[cfg.K * FP + t];
  // the newest min(nin, B) window rows are the fused ones (counted from LDS);
  // only the pieces holding older rows are read from XT
  const int bold = B - (nin < B ? nin : B);
  const unsigned short* xt = dv.XT + (size_t)(fs + fl0) * cap;
  const int nq_all = wt.nt * 4;  // 8-row pieces of the window tiles (piece qq starts at window row qq*8 - s0)
  const int nq = min(nq_all, (bold + wt.s0 + 7) >> 3);
  constexpr int U = 4;  // pieces per lane in flight
  u16x8 v[U];
  auto load_pieces = [&](int q0) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int qq = q0 + kStatL * u;
      const int qc = qq < nq ? qq : nq - 1;
      v[u] = *(const u16x8*)(xt + wt.ring_tile(qc >> 2) * 32 + (qc & 3) * 8);
    }
  };
  // the first batch of the window read is issued before the ingest copy: the
  // old rows' XT pieces do not depend on it
  if (nq > 0) load_pieces(j);
  // fused ingest: one 16-B chunk (this slice) of each new row; every chunk's
  // load is issued before the first store
  constexpr int kIU = kMaxFusedIngest / 256;
  u16x8 iv[kIU];
  int iy[kIU];
#pragma unroll
  for (int u = 0; u < kIU; ++u) {
    const int i = t + 256 * u;
    if (i < nin) {
      const long long sr = ing.first + (long long)i * ing.step;
      iv[u] = *(const u16x8*)(ing.src + sr * FP + fs);
      if (blockIdx.x == 0) iy[u] = ing.ysrc[sr];
    }
  }
  if (nin > 0 && blockIdx.x == 0 && t == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    stamp(dv, 30, 5);  // this thread's ingest loads arrived
  }
#pragma unroll
  for (int u = 0; u < kIU; ++u) {
    const int i = t + 256 * u;
    if (i < nin) {
      int dr = ing.dst + i;
      dr = dr >= cap ? dr - cap : dr;
      *(u16x8*)(const_cast<uint16_t*>(dv.X) + (size_t)dr * FP + fs) = iv[u];
      *(u16x8*)(nv + i * kStatW) = iv[u];
#pragma unroll
      for (int e = 0; e < 8; ++e) const_cast<uint16_t*>(dv.XT)[(size_t)(fs + e) * cap + dr] = iv[u][e];
      if (blockIdx.x == 0) const_cast<int32_t*>(dv.y)[dr] = iy[u];
    }
  }
  float s = 0.f, q = 0.f;
  for (int q0 = j; q0 < nq; q0 += kStatL * U) {
    if (q0 != j) load_pieces(q0);  // (the first batch was issued at entry)
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int qq = q0 + kStatL * u;
      const int o0 = (qq >> 2) * 32 + (qq & 3) * 8 - wt.s0;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const bool in = qq < nq && o0 + e >= 0 && o0 + e < bold;
        const float x = in ? bf2f(v[u][e]) : 0.f;
        s += x;
        q += x * x;
      }
    }
  }
  if (nin > 0) {
    __syncthreads();
    if (blockIdx.x == 0 && t == 0) stamp(dv, 30, 6);  // copies issued, old-row sums done
    for (int i = nin - (B - bold) + j; i < nin; i += kStatL) {
      const float x = bf2f(nv[i * kStatW + fl0]);
      s += x;
      q += x * x;
    }
  }
  double a = s, b2 = q;
#pragma unroll
  for (int o = 1; o < kStatL; o <<= 1) {
    a += __shfl_xor(a, o, 64);
    b2 += __shfl_xor(b2, o, 64);
  }
  if (j == 0) {
    rs[fl0] = a;
    rq[fl0] = b2;
  }
  __syncthreads();
  prep_epilogue(cfg, dv, ctrl, B, fs, rs, rq, sdl, ivl, wo_pre, b_pre);
}

// Launch geometry of a grid whose G <= 32 cooperating workgroups hand off
// through one L2 (S = 2): they are blockIdx 0, 8, .., 8 (G - 1) -- all on XCD 0
// (blockIdx % 8 == XCC_ID on MI355X) -- and the riding evaluation workgroups
// fill the other blockIdx, i.e. XCDs 1..7: they never compete with the
// cooperating ones for XCD 0's CUs.  S = 1: workgroups 0..G-1 spread over the
// XCDs (sc1 hand-offs), riding workgroups after them.
template <int S>
__device__ __forceinline__ int xcd_role(int b, int G, int x) {  // >= 0: cooperating workgroup; < 0: -(ride index) - 1
  if constexpr (S == 2) {  // cooperating workgroup i is blockIdx 8 i + x (XCD x)
    if ((b & 7) == x && (b >> 3) < G) return b >> 3;
    int before = b > x ? (b - x + 7) >> 3 : 0;  // cooperating workgroups with blockIdx < b
    before = before < G ? before : G;
    return -(b - before) - 1;
  } else {
    return b < G ? b : -(b - G) - 1;
  }
}
int xcd_grid(int G, int nride, bool one_xcd, int x) {
  if (!one_xcd) return G + nride;
  const int a = 8 * (G - 1) + x + 1, b = G + nride;
  return a > b ? a : b;
}


template <int FP>
__global__ __launch_bounds__(256) void fwd_kernel(SolverCfg cfg, const SolveParams* prm, const Ctrl* ctrl, int slot,
                                                  SolveDev dv, SolveParams win) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int phase = ctrl->phase;  // checked once the first tile is staged
  if constexpr (FP <= 1024) {
    if (dv.gpf) {
      fwd_slot<FP, true>(cfg, window_of(win, prm), slot, dv, lds, blockIdx.x, gridDim.x, phase);
      return;
    }
  }
  fwd_slot<FP, false>(cfg, window_of(win, prm), slot, dv, lds, blockIdx.x, gridDim.x, phase);
}



size_t bwd_lds_bytes();
// a bwd_update launch with riding evaluation workgroups sizes its LDS for both bodies
size_t bwd_ride_lds_bytes(int FP) {
  const size_t a = bwd_lds_bytes(), b = eval_lds_bytes(FP);
  return a > b ? a : b;
}

size_t bwd_lds_bytes() { return kBwdLdsBytes; }


// The ns = FP/32 slice workgroups all-gather their dots: for FP <= 1024 (ns <=
// 32) they run on one XCD and the all-gather goes through its L2 (xcd_role).
template <int FP>
constexpr int bwd_scope() { return FP <= 1024 ? 2 : 1; }

template <int FP, int KP>
__global__ __launch_bounds__(256) void bwd_update_kernel(SolverCfg cfg, const SolveParams* prm, Ctrl* gctrl, int slot,
                                                         SolveDev dv, int fwd_grid, SolveParams win, int ns,
                                                         EvalRide ride, int ride_t0, int nride, int fin_slot) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  constexpr int S = bwd_scope<FP>();
  const int role = (S == 2 && cfg.xcd >= 0) ? xcd_role<2>((int)blockIdx.x, ns, cfg.xcd & 7)
                                            : xcd_role<1>((int)blockIdx.x, ns, 0);
  if (role < 0) {  // an evaluation workgroup riding in this launch: one test tile
    if (-role - 1 >= nride) return;  // (a gap of the one-XCD geometry)
    const int t = ride_t0 - role - 1;
    eval_body<FP>(lds, ride, t, 1, t + 1);
    return;
  }
  bwd_body<FP, KP, 0, S>(cfg, window_of(win, prm), gctrl, slot, dv, fwd_grid, lds, role, ns, true, fin_slot);
}

// ---------------------------------------------------------------------------
// tail_kernel: the line-search retry slots [slot_begin, slot_end) in ONE
// persistent launch.  The usual solve is done after 1 + iters evaluations
// (every line search accepts its first trial), so this launch exits on its
// first instruction; when a line search does need more evaluations they run
// here as fwd phase -> grid barrier -> bwd phase -> grid barrier, instead of
// as 2 launches per budgeted slot that are almost always empty.
// Grid = max(fwd grid, slices); all workgroups are co-resident (<= 512).
// Barriers: plain stores -> every wave drains -> __syncthreads -> lane 0
// agent release fence -> drain -> arrival RMW on a monotone counter -> relaxed
// poll -> agent acquire fence (the CDNA4 playbook's counter barrier); the
// controller phase is re-read with sc1 loads (never through the scalar cache).
__device__ __forceinline__ void grid_barrier(unsigned long long* ctr, unsigned long long target,
                                             unsigned long long* err) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    (void)__hip_atomic_fetch_add(ctr, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int spins = 0;
    while (xload(ctr) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > (1 << 24)) {
        xstore(err, 2ull);
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
}

template <int KP>
__device__ __forceinline__ void finalize_body(const SolverCfg& cfg, const Ctrl* ctrl, const SolveDev& dv, int blk,
                                              const FinIn<KP>& in) {
  if (blk == 0 && threadIdx.x == 0) stamp(dv, 30, 2);
  finalize_feature<KP>(cfg, dv, blk * 256 + threadIdx.x, in);
  if (blk == 0 && threadIdx.x == 0) finalize_scalars<KP>(cfg, ctrl, dv);
}

template <int KP>
__global__ __launch_bounds__(256) void finalize_kernel(SolverCfg cfg, const Ctrl* ctrl, SolveDev dv) {
  if (ctrl->fin) {  // the last bwd_update launch finalised the features
    if (blockIdx.x == 0 && threadIdx.x == 0) finalize_scalars<KP>(cfg, ctrl, dv);
    return;
  }
  FinIn<KP> in;
  in.load(cfg, dv, blockIdx.x);
  finalize_body<KP>(cfg, ctrl, dv, blockIdx.x, in);
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

template <int FP, int KP>
__global__ __launch_bounds__(256) void tail_kernel(SolverCfg cfg, const SolveParams* prm, Ctrl* gctrl,
                                                   int slot_begin, int slot_end, SolveDev dv, int ns, int lds_flag,
                                                   int nfin) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  int& phase_s = *(int*)(lds + lds_flag);  // past both bodies' LDS (no static __shared__: keeps the base aligned)
  // the finalisation's inputs are fetched before the phase word is known, so
  // the two load latencies overlap (the common case is phase == done)
  // the scalars' inputs travel with the phase words (one round trip); they are
  // re-read below when slots run here
  FinScal sc;
  const bool t0 = blockIdx.x == 0 && threadIdx.x == 0;
  if (t0 && nfin > 0) sc.load(cfg, gctrl, dv);
  if (gctrl->fin) {  // the common case: the last bwd_update launch finished and finalised the solve
    if (t0) {
      stamp(dv, 30, 2);
      if (nfin > 0) sc.store(cfg, dv);
    }
    return;
  }
  FinSl<KP> in;
  float* wvl = (float*)lds;  // finalisation scratch (the slots' LDS is dead by then)
  if ((int)blockIdx.x < nfin) in.load(cfg, dv, blockIdx.x);
  if (gctrl->phase == kPhDone) {  // written by the previous launch
    // the finalisation is folded into this launch (one graph node less per solve)
    if ((int)blockIdx.x < nfin) {
      if (blockIdx.x == 0 && threadIdx.x == 0) stamp(dv, 30, 2);
      finalize_slice<KP>(cfg, dv, blockIdx.x, in, wvl);
      if (blockIdx.x == 0 && threadIdx.x == 0) finalize_scalars<KP>(cfg, gctrl, dv);
    }
    return;
  }
  const int G = gridDim.x, wg = blockIdx.x;
  unsigned long long* bar = dv.xch + kXchBar;
  unsigned long long nb = 0;
  for (int slot = slot_begin; slot < slot_end; ++slot) {
    if (slot > slot_begin) {
      if (threadIdx.x == 0) phase_s = (int)(unsigned)xload((unsigned long long*)&gctrl->phase);
      __syncthreads();
      if (phase_s == kPhDone) break;  // uniform: every workgroup read the same word after the barrier
    }
    if constexpr (FP <= 1024) {
      if (dv.gpf)
        fwd_slot<FP, true>(cfg, *prm, slot, dv, lds, wg, G, -1);
      else
        fwd_slot<FP, false>(cfg, *prm, slot, dv, lds, wg, G, -1);
    } else {
      fwd_body<FP>(cfg, *prm, slot, dv, lds, wg, G);
    }
    grid_barrier(bar, (unsigned long long)G * ++nb, dv.xch + kXchErr);
    if (wg < ns) bwd_body<FP, KP>(cfg, *prm, gctrl, slot, dv, G, lds, wg, ns);
    grid_barrier(bar, (unsigned long long)G * ++nb, dv.xch + kXchErr);
  }
  // every exit of the loop follows a grid barrier: all slots' updates are visible
  if (wg < nfin) {
    in.load(cfg, dv, wg);  // re-read: the slots above moved x
    __syncthreads();       // (wvl overlaps the slots' LDS)
    finalize_slice<KP>(cfg, dv, wg, in, wvl);
    if (wg == 0 && threadIdx.x == 0) finalize_scalars<KP>(cfg, gctrl, dv);
  }
}

// ---------------------------------------------------------------------------
size_t stats_prep_lds_bytes() {
  return 2 * kStatW * sizeof(double) + 2 * kStatW * sizeof(float) + kMaxFusedIngest * kStatW * sizeof(uint16_t);
}

void launch_stats_prep(const SolverCfg& cfg, SolveParams* prm, const SolveDev& dv, Ctrl* ctrl, int B, int start,
                       const RingIngest& ing, hipStream_t s) {
  stats_prep_kernel<<<cfg.Fp / kStatW, 256, stats_prep_lds_bytes(), s>>>(cfg, prm, dv, ctrl, B, start, ing);
}
const void* stats_prep_symbol() { return (const void*)stats_prep_kernel; }

size_t fwd_lds_bytes(int FP) { return eval_lds_bytes(FP); }
int padded_classes(int K) { return K <= 2 ? 2 : K <= 4 ? 4 : K <= 8 ? 8 : 16; }
int padded_stride(int FP) { return FP > 256 ? FP : 256; }
int bwd_grid(int FP) { return FP / 32; }

template <int FP>
static void launch_bwd_fp(const SolverCfg& cfg, const SolveParams* prm, Ctrl* ctrl, int slot, const SolveDev& dv,
                          int nwg, hipStream_t s, const SolveParams& win, const EvalRide& ride = EvalRide{},
                          int ride_t0 = 0, int nride = 0, int fin_slot = kNoFinSlot) {
  const int ns = bwd_grid(FP), ng = xcd_grid(ns, nride, bwd_scope<FP>() == 2 && cfg.xcd >= 0, cfg.xcd & 7);
  const size_t bl = nride > 0 ? bwd_ride_lds_bytes(FP) : bwd_lds_bytes();
  switch (dv.KP) {
    case 2:
      bwd_update_kernel<FP, 2><<<ng, 256, bl, s>>>(cfg, prm, ctrl, slot, dv, nwg, win, ns, ride, ride_t0, nride, fin_slot);
      break;
    case 4:
      bwd_update_kernel<FP, 4><<<ng, 256, bl, s>>>(cfg, prm, ctrl, slot, dv, nwg, win, ns, ride, ride_t0, nride, fin_slot);
      break;
    case 8:
      bwd_update_kernel<FP, 8><<<ng, 256, bl, s>>>(cfg, prm, ctrl, slot, dv, nwg, win, ns, ride, ride_t0, nride, fin_slot);
      break;
    default:
      bwd_update_kernel<FP, 16><<<ng, 256, bl, s>>>(cfg, prm, ctrl, slot, dv, nwg, win, ns, ride, ride_t0, nride, fin_slot);
      break;
  }
}

template <int FP>
static void launch_slot_fp(const SolverCfg& cfg, const SolveParams* prm, Ctrl* ctrl, int slot, const SolveDev& dv,
                           int nwg, hipStream_t s, const SolveParams& win, int fin_slot,
                           const EvalRide& ride = EvalRide{}, int ride_t0 = 0, int nride = 0) {
  fwd_kernel<FP><<<nwg, 256, fwd_lds_bytes(FP), s>>>(cfg, prm, ctrl, slot, dv, win);
  launch_bwd_fp<FP>(cfg, prm, ctrl, slot, dv, nwg, s, win, ride, ride_t0, nride, fin_slot);
}

void launch_bwd(const SolverCfg& cfg, const SolveParams* prm, Ctrl* ctrl, int slot, const SolveDev& dv, int fwd_grid,
                hipStream_t s, const SolveParams& win) {
  switch (cfg.Fp) {
    case 128: launch_bwd_fp<128>(cfg, prm, ctrl, slot, dv, fwd_grid, s, win); break;
    case 256: launch_bwd_fp<256>(cfg, prm, ctrl, slot, dv, fwd_grid, s, win); break;
    case 512: launch_bwd_fp<512>(cfg, prm, ctrl, slot, dv, fwd_grid, s, win); break;
    case 1024: launch_bwd_fp<1024>(cfg, prm, ctrl, slot, dv, fwd_grid, s, win); break;
    case 2048: launch_bwd_fp<2048>(cfg, prm, ctrl, slot, dv, fwd_grid, s, win); break;
    default: break;
  }
}

void launch_slot_ride(const SolverCfg& cfg, const SolveParams* prm, Ctrl* ctrl, int slot, const SolveDev& dv, int nwg,
                      hipStream_t s, const SolveParams& win, const EvalRide& ride, int ride_t0, int nride,
                      int fin_slot) {
  switch (cfg.Fp) {
    case 128: launch_slot_fp<128>(cfg, prm, ctrl, slot, dv, nwg, s, win, fin_slot, ride, ride_t0, nride); break;
    case 256: launch_slot_fp<256>(cfg, prm, ctrl, slot, dv, nwg, s, win, fin_slot, ride, ride_t0, nride); break;
    case 512: launch_slot_fp<512>(cfg, prm, ctrl, slot, dv, nwg, s, win, fin_slot, ride, ride_t0, nride); break;
    case 1024: launch_slot_fp<1024>(cfg, prm, ctrl, slot, dv, nwg, s, win, fin_slot, ride, ride_t0, nride); break;
    case 2048: launch_slot_fp<2048>(cfg, prm, ctrl, slot, dv, nwg, s, win, fin_slot, ride, ride_t0, nride); break;
    default: break;
  }
}

void launch_slot(const SolverCfg& cfg, const SolveParams* prm, Ctrl* ctrl, int slot, const SolveDev& dv, int nwg,
                 hipStream_t s, const SolveParams& win, int fin_slot) {
  switch (cfg.Fp) {
    case 128: launch_slot_fp<128>(cfg, prm, ctrl, slot, dv, nwg, s, win, fin_slot); break;
    case 256: launch_slot_fp<256>(cfg, prm, ctrl, slot, dv, nwg, s, win, fin_slot); break;
    case 512: launch_slot_fp<512>(cfg, prm, ctrl, slot, dv, nwg, s, win, fin_slot); break;
    case 1024: launch_slot_fp<1024>(cfg, prm, ctrl, slot, dv, nwg, s, win, fin_slot); break;
    case 2048: launch_slot_fp<2048>(cfg, prm, ctrl, slot, dv, nwg, s, win, fin_slot); break;
    default: break;
  }
}

size_t tail_lds_bytes(int FP) {
  const size_t a = fwd_lds_bytes(FP), b = bwd_lds_bytes();
  return ((a > b ? a : b) + 15) / 16 * 16 + 16;
}
int tail_grid(int FP, int nwg) {
  const int ns = bwd_grid(FP), g = nwg < 64 ? nwg : 64;
  return g > ns ? g : ns;
}

template <int FP>
static void launch_tail_fp(const SolverCfg& cfg, const SolveParams* prm, Ctrl* ctrl, int s0, int s1,
                           const SolveDev& dv, int nwg, int fin, hipStream_t s) {
  const int G = tail_grid(FP, nwg), ns = bwd_grid(FP);
  const size_t lb = tail_lds_bytes(FP);
  const int flag = (int)(lb - 16);
  const int nfin = fin ? cfg.Fp / 32 : 0;  // 32-feature slices; <= G: G >= FP/32 workgroups
  switch (dv.KP) {
    case 2: tail_kernel<FP, 2><<<G, 256, lb, s>>>(cfg, prm, ctrl, s0, s1, dv, ns, flag, nfin); break;
    case 4: tail_kernel<FP, 4><<<G, 256, lb, s>>>(cfg, prm, ctrl, s0, s1, dv, ns, flag, nfin); break;
    case 8: tail_kernel<FP, 8><<<G, 256, lb, s>>>(cfg, prm, ctrl, s0, s1, dv, ns, flag, nfin); break;
    default: tail_kernel<FP, 16><<<G, 256, lb, s>>>(cfg, prm, ctrl, s0, s1, dv, ns, flag, nfin); break;
  }
}

void launch_tail(const SolverCfg& cfg, const SolveParams* prm, Ctrl* ctrl, int slot_begin, int slot_end,
                 const SolveDev& dv, int nwg, hipStream_t s, int with_finalize) {
  switch (cfg.Fp) {
    case 128: launch_tail_fp<128>(cfg, prm, ctrl, slot_begin, slot_end, dv, nwg, with_finalize, s); break;
    case 256: launch_tail_fp<256>(cfg, prm, ctrl, slot_begin, slot_end, dv, nwg, with_finalize, s); break;
    case 512: launch_tail_fp<512>(cfg, prm, ctrl, slot_begin, slot_end, dv, nwg, with_finalize, s); break;
    case 1024: launch_tail_fp<1024>(cfg, prm, ctrl, slot_begin, slot_end, dv, nwg, with_finalize, s); break;
    case 2048: launch_tail_fp<2048>(cfg, prm, ctrl, slot_begin, slot_end, dv, nwg, with_finalize, s); break;
    default: break;
  }
}

// ---------------------------------------------------------------------------
// Large-window ("rows") mode.  A window of up to tens of millions of ring rows
// (the reference's -max, WorkerAppRunner.java:56-57) is streamed
// row-parallel by G workgroups, each taking ring tiles wg, wg+G, ...:
//   stats_rows_kernel   partial column sums / squares          -> spart[G]
//   prep_rows_kernel    reduce them (fixed order), std, x0, controller
//   per slot: fwdbwd_rows_kernel  forward + softmax + backward of each tile
//                                 while it sits in LDS        -> gpart[G]
//             reduce_g_kernel     G = sum over workgroups (fixed order)
//             bwd_update_kernel   (gred mode) dots, controller, update
// Every evaluation reads the window ONCE (the small-window path reads X for the
// forward and the feature-major copy XT for the backward), no XT copy exists,
// and no residual buffer is materialised.  Deterministic: every reduction runs
// in a fixed order.
bool rows_mode_for(int cap) {
  const char* e = std::getenv("PSX_SOLVER_ROWS");
  if (e && *e) return e[0] == '1';
  return cap > kRowsModeMinCap;
}

template <int FP, bool kF32 = false>
__global__ __launch_bounds__(256) void stats_rows_kernel(SolverCfg cfg, SolveParams* prm, SolveDev dv, int B,
                                                         int start) {
  constexpr int C = FP / 8;   // 16-B chunks per row
  constexpr int L = 256 / C;  // row lanes
  static_assert(C * L == 256, "FP in {128..2048}");
  constexpr int RPL = 32 / L;  // rows of a tile per lane
  extern __shared__ __attribute__((aligned(16))) char smem[];
  double* red = (double*)smem;  // [L][C][16]
  if (blockIdx.x == 0 && threadIdx.x == 0) *prm = SolveParams{B, start, 0, 0};
  const WinTiles wt(start, B, cfg.cap);
  const int t = threadIdx.x, ch = t % C, rl = t / C;
  double s[8], q[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) s[e] = q[e] = 0.0;
  for (int tile = blockIdx.x; tile < wt.nt; tile += gridDim.x) {
    const int64_t row0 = (int64_t)wt.ring_tile(tile) * 32;
    float fs[8], fq[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) fs[e] = fq[e] = 0.f;
    if constexpr (kF32) {
      constexpr int RB = RPL < 8 ? RPL : 8;  // rows whose 32 B are in flight together
#pragma unroll
      for (int j0 = 0; j0 < RPL; j0 += RB) {
        f32x4 v[RB][2];
#pragma unroll
        for (int j = 0; j < RB; ++j) {
          const float* src = dv.Xf + (row0 + rl + L * (j0 + j)) * FP + ch * 8;
          v[j][0] = *(const f32x4*)src;
          v[j][1] = *(const f32x4*)(src + 4);
        }
#pragma unroll
        for (int j = 0; j < RB; ++j) {
          const int o = tile * 32 + rl + L * (j0 + j) - wt.s0;
          const bool in = o >= 0 && o < B;
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float x = in ? v[j][e >> 2][e & 3] : 0.f;
            fs[e] += x;
            fq[e] += x * x;
          }
        }
      }
    } else {
      u16x8 v[RPL];
#pragma unroll
      for (int j = 0; j < RPL; ++j) v[j] = *(const u16x8*)(dv.X + (row0 + rl + L * j) * FP + ch * 8);
#pragma unroll
      for (int j = 0; j < RPL; ++j) {
        const int o = tile * 32 + rl + L * j - wt.s0;  // offset in the window
        const bool in = o >= 0 && o < B;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float x = in ? bf2f(v[j][e]) : 0.f;
          fs[e] += x;
          fq[e] += x * x;
        }
      }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      s[e] += fs[e];
      q[e] += fq[e];
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    red[(rl * C + ch) * 16 + e] = s[e];
    red[(rl * C + ch) * 16 + 8 + e] = q[e];
  }
  __syncthreads();
  for (int k = t; k < C * 16; k += 256) {  // k = chunk * 16 + {sum e | square e}
    double a = 0.0;
    for (int r = 0; r < L; ++r) a += red[r * C * 16 + k];
    const int c = k >> 4, e = k & 15, f = c * 8 + (e & 7);
    dv.spart[((size_t)blockIdx.x * 2 + (e >> 3)) * FP + f] = a;
  }
}

__global__ __launch_bounds__(256) void prep_rows_kernel(SolverCfg cfg, const SolveParams* prm, SolveDev dv,
                                                        Ctrl* ctrl, int G) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  double* rs = (double*)smem;          // [kStatW]
  double* rq = rs + kStatW;            // [kStatW]
  float* sdl = (float*)(rq + kStatW);  // [kStatW]
  float* ivl = sdl + kStatW;           // [kStatW]
  double* part = (double*)(ivl + kStatW);  // [16 lanes][16]
  const int t = threadIdx.x, FP = cfg.Fp, B = prm->B;
  const int fs = blockIdx.x * kStatW;
  const int KP0 = dv.KP;
  float wo_pre = 0.f, b_pre = 0.f;
  if (t < kStatW * KP0) {
    const int c = t / kStatW, f = fs + t % kStatW;
    if (c < cfg.K && f < cfg.F) wo_pre = dv.w_old[c * FP + f];
  }
  if (blockIdx.x == 0 && t < 16 && t < cfg.K) b_pre = dv.w_old[cfg.K * FP + t];
  {  // thread: (feature fl, sum|square) x 16 lanes over the G partials
    const int fl = t & 7, kind = (t >> 3) & 1, lane = t >> 4;
    double a = 0.0;
    for (int g = lane; g < G; g += 16) a += dv.spart[((size_t)g * 2 + kind) * FP + fs + fl];
    part[lane * 16 + kind * 8 + fl] = a;
  }
  __syncthreads();
  if (t < 16) {
    double a = 0.0;
    for (int lane = 0; lane < 16; ++lane) a += part[lane * 16 + t];  // fixed order
    if (t < 8)
      rs[t] = a;
    else
      rq[t - 8] = a;
  }
  __syncthreads();
  prep_epilogue(cfg, dv, ctrl, B, fs, rs, rq, sdl, ivl, wo_pre, b_pre);
}

template <int FP, bool kF32 = false>
__global__ __launch_bounds__(256) void fwdbwd_rows_kernel(SolverCfg cfg, const SolveParams* prm, const Ctrl* ctrl,
                                                          int slot, SolveDev dv) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  if (ctrl->phase == kPhDone) return;  // converged in an earlier slot
  constexpr int NT = FP / 64;
  f32x4 acc[NT];
#pragma unroll
  for (int n = 0; n < NT; ++n) acc[n] = f32x4{0, 0, 0, 0};
  const int wg = blockIdx.x;
  const WinTiles wt(prm->start, prm->B, cfg.cap);
  if (wg >= wt.nt) return;
  fwd_body<FP, true, kF32>(cfg, *prm, slot, dv, lds, wg, gridDim.x, acc);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, KP = dv.KP;
#pragma unroll
  for (int n = 0; n < NT; ++n) {
    const int f = (w * NT + n) * 16 + (lane & 15);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = (lane >> 4) * 4 + i;
      if (c < KP) dv.gpart[((size_t)wg * KP + c) * FP + f] = acc[n][i];
    }
  }
}

// gred[c][f] = sum over the forward workgroups of gpart (fixed order): 64
// elements per workgroup, 4 partial sums per element combined in order.
__global__ __launch_bounds__(256) void reduce_g_kernel(SolverCfg cfg, const SolveParams* prm, const Ctrl* ctrl,
                                                       SolveDev dv, int G) {
  __shared__ float red[4][64];
  if (ctrl->phase == kPhDone) return;
  const WinTiles wt(prm->start, prm->B, cfg.cap);
  const int nfw = wt.nt < G ? wt.nt : G;
  const int FP = cfg.Fp, KP = dv.KP;
  const int t = threadIdx.x, e = blockIdx.x * 64 + (t & 63), sub = t >> 6;
  const int c = e / FP, f = e - c * FP;
  float a = 0.f;
  if (c < KP) {
    const float* src = dv.gpart + (size_t)c * FP + f;
    const size_t stride = (size_t)KP * FP;
    constexpr int U = 8;
    for (int g0 = sub; g0 < nfw; g0 += 4 * U) {
      float v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int g = g0 + 4 * u;
        v[u] = g < nfw ? src[(size_t)g * stride] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) a += v[u];
    }
  }
  red[sub][t & 63] = a;
  __syncthreads();
  if (t < 64 && c < KP) dv.gred[c * dv.FPI + f] = red[0][t] + red[1][t] + red[2][t] + red[3][t];
}

size_t stats_rows_lds_bytes() { return (size_t)256 * 16 * sizeof(double); }

// fp32 ring ingest: one workgroup per row group, 16 B per thread per step.
__global__ __launch_bounds__(256) void ring_ingest_f32_kernel(const float* src, const int32_t* ysrc, int64_t first,
                                                              int64_t step, int64_t n, float* ring, int32_t* yring,
                                                              int64_t dst, int64_t cap, int FP) {
  const int64_t q = FP / 4;  // float4 chunks per row
  const int64_t total = n * q;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int64_t r = i / q, c = i - r * q;
    int64_t d = dst + r;
    d = d >= cap ? d % cap : d;
    const int64_t sr = first + r * step;
    *(f32x4*)(ring + d * FP + c * 4) = *(const f32x4*)(src + sr * FP + c * 4);
    if (c == 0) yring[d] = ysrc[sr];
  }
}

void launch_ring_ingest_f32(const float* src, const int32_t* ysrc, int64_t src_first, int64_t src_step, int64_t n,
                            float* ring, int32_t* yring, int64_t dst_first, int64_t cap, int FP, hipStream_t s) {
  if (n <= 0) return;
  const int64_t total = n * (FP / 4);
  int64_t grid = (total + 255) / 256;
  if (grid > 4096) grid = 4096;
  ring_ingest_f32_kernel<<<(unsigned)grid, 256, 0, s>>>(src, ysrc, src_first, src_step, n, ring, yring, dst_first,
                                                         cap, FP);
}

void launch_stats_rows(const SolverCfg& cfg, SolveParams* prm, const SolveDev& dv, int B, int start, int G,
                       hipStream_t s) {
  const size_t lb = stats_rows_lds_bytes();
  if (cfg.xf32) {
    switch (cfg.Fp) {
      case 128: stats_rows_kernel<128, true><<<G, 256, lb, s>>>(cfg, prm, dv, B, start); break;
      case 256: stats_rows_kernel<256, true><<<G, 256, lb, s>>>(cfg, prm, dv, B, start); break;
      case 512: stats_rows_kernel<512, true><<<G, 256, lb, s>>>(cfg, prm, dv, B, start); break;
      case 1024: stats_rows_kernel<1024, true><<<G, 256, lb, s>>>(cfg, prm, dv, B, start); break;
      default: break;
    }
    return;
  }
  switch (cfg.Fp) {
    case 128: stats_rows_kernel<128><<<G, 256, lb, s>>>(cfg, prm, dv, B, start); break;
    case 256: stats_rows_kernel<256><<<G, 256, lb, s>>>(cfg, prm, dv, B, start); break;
    case 512: stats_rows_kernel<512><<<G, 256, lb, s>>>(cfg, prm, dv, B, start); break;
    case 1024: stats_rows_kernel<1024><<<G, 256, lb, s>>>(cfg, prm, dv, B, start); break;
    case 2048: stats_rows_kernel<2048><<<G, 256, lb, s>>>(cfg, prm, dv, B, start); break;
    default: break;
  }
}

void launch_prep_rows(const SolverCfg& cfg, const SolveParams* prm, const SolveDev& dv, Ctrl* ctrl, int G,
                      hipStream_t s) {
  const size_t lb = 2 * kStatW * sizeof(double) + 2 * kStatW * sizeof(float) + 16 * 16 * sizeof(double);
  prep_rows_kernel<<<cfg.Fp / kStatW, 256, lb, s>>>(cfg, prm, dv, ctrl, G);
}

size_t fwdbwd_rows_lds_bytes(int FP, bool f32) { return fwd_lds_bytes(FP) + (f32 ? (size_t)32 * FP * 2 : 0); }

void launch_fwdbwd_rows(const SolverCfg& cfg, const SolveParams* prm, const Ctrl* ctrl, int slot, const SolveDev& dv,
                        int G, hipStream_t s) {
  if (cfg.xf32) {
    const size_t lb = fwdbwd_rows_lds_bytes(cfg.Fp, true);
    switch (cfg.Fp) {
      case 128: fwdbwd_rows_kernel<128, true><<<G, 256, lb, s>>>(cfg, prm, ctrl, slot, dv); break;
      case 256: fwdbwd_rows_kernel<256, true><<<G, 256, lb, s>>>(cfg, prm, ctrl, slot, dv); break;
      case 512: fwdbwd_rows_kernel<512, true><<<G, 256, lb, s>>>(cfg, prm, ctrl, slot, dv); break;
      case 1024: fwdbwd_rows_kernel<1024, true><<<G, 256, lb, s>>>(cfg, prm, ctrl, slot, dv); break;
      default: break;
    }
    return;
  }
  const size_t lb = fwd_lds_bytes(cfg.Fp);
  switch (cfg.Fp) {
    case 128: fwdbwd_rows_kernel<128><<<G, 256, lb, s>>>(cfg, prm, ctrl, slot, dv); break;
    case 256: fwdbwd_rows_kernel<256><<<G, 256, lb, s>>>(cfg, prm, ctrl, slot, dv); break;
    case 512: fwdbwd_rows_kernel<512><<<G, 256, lb, s>>>(cfg, prm, ctrl, slot, dv); break;
    case 1024: fwdbwd_rows_kernel<1024><<<G, 256, lb, s>>>(cfg, prm, ctrl, slot, dv); break;
    case 2048: fwdbwd_rows_kernel<2048><<<G, 256, lb, s>>>(cfg, prm, ctrl, slot, dv); break;
    default: break;
  }
}

void launch_reduce_g(const SolverCfg& cfg, const SolveParams* prm, const Ctrl* ctrl, const SolveDev& dv, int G,
                     hipStream_t s) {
  const int n = dv.KP * cfg.Fp;
  reduce_g_kernel<<<(n + 63) / 64, 256, 0, s>>>(cfg, prm, ctrl, dv, G);
}


// ---------------------------------------------------------------------------
// Persistent small-window solve: the WHOLE local solve in ONE launch.
//
// The launch chain above (stats_prep, 2 launches per slot, tail) pays a kernel
// boundary (~1.5-2 us) per phase, and every launch re-reads its operands from
// memory: each kernel start meets cold caches, so the per-slot chain is bounded
// by memory round trips, not by work (profiles/r02_v3).  The persistent solve is
// TWO launches: stats_prep_kernel (the fused ingest, window statistics, x0, the
// first trial point, the controller -- as in the chain), then one launch in
// which G = max(window tiles, FP/32) co-resident workgroups keep their 32-row
// window tile (and its labels) resident in LDS for the whole solve and run
//   per slot:  row role   forward + softmax + R^T X of the resident tile -> gpf[wg]
//              slice role  G = sum of the partials (fixed order), the dots
//                          all-gather, controller step, update, next fragments
//   F  slice owners finalise their features (+ the fused server update)
// with a grid-wide arrival between the phases.  When G <= 32 (every window of
// <= 1024 rows that starts on a 32-row boundary) all solve workgroups run on
// ONE XCD and every hand-off goes through its L2 (S = 2 below: plain stores, nt
// loads, a flag-line barrier; 0.64 us per hand-off, tools/xcd_probe.hip);
// otherwise they spread over the XCDs with the R1 form of the CDNA4 playbook
// (S = 1: sc1 write-through stores, each storing wave drained before the
// arrival on a monotone counter, sc1 loads; 1.7-2.7 us per hand-off).  Spins
// are bounded (a timeout sets the sticky error word).  The riding evaluation's
// workgroups (one test tile each) never wait.
size_t persist_lds_bytes(int FP) { return persist_fwd_bytes(FP) + (bwd_lds_bytes() + 15) / 16 * 16 + kSyBytes; }
int persist_grid(int FP, int ntiles) { return ntiles > FP / 32 ? ntiles : FP / 32; }

template <int FP, int KP, int S>
__global__ __launch_bounds__(256) void solve_persist_kernel(SolverCfg cfg, SolveDev dv, Ctrl* gctrl, SolveParams win,
                                                            int G, EvalRide ride, int nride) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int role = xcd_role<S>((int)blockIdx.x, G, cfg.xcd & 7), tid = threadIdx.x;
  if (role < 0) {  // an evaluation workgroup riding in this launch: one test tile, no waiting
    const int t = -role - 1;
    if (t >= nride) return;
    eval_body<FP>(lds, ride, t, 1, t + 1);
    // arrival once this workgroup's loads (the models' fragments) are complete: the
    // finalisation rewrites those fragments only after every riding workgroup arrived
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0)
      (void)__hip_atomic_fetch_add((g_u64*)(dv.xch + kXchRide + (*dv.prm_count & 1u)), 1ull, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  const int wg = role;
  constexpr int NS = FP / 32;  // feature slices
  char* lf = lds;                          // row role: the resident tile + forward scratch
  char* lb = lds + persist_fwd_bytes(FP);  // slice role: bwd_body's region
  unsigned short* frl = (unsigned short*)(lb + 4 * 16 * 32 * 4);
  Ctrl* cl = (Ctrl*)(frl + 1024);          // bwd_body's controller copy (persists across slots)
  const int B = win.B;
  const WinTiles wt(win.start, B, cfg.cap);
  const int ntiles = wt.nt;
  const unsigned run = *dv.prm_count;
  unsigned long long* xch = dv.xch;
  unsigned long long* bar = xch + kXchGen + (run & 1u);
  unsigned long long* err = xch + kXchErr;
  unsigned long long nb = 0;
  auto barrier = [&]() {
    ++nb;
    if constexpr (S == 2)
      x_barrier(xch + kXchFlags, wg, G, ((unsigned long long)run << 16) | nb, err, spin_limit(dv));
    else
      p_barrier(bar, (unsigned long long)G * nb, err, spin_limit(dv));
  };
  const bool row = wg < ntiles, owner = wg < NS;
  if (wg == 0 && tid == 0) stamp(dv, 30, 3);
  // ---- the window statistics, x0, the first trial point's fragments and the
  // controller come from stats_prep_kernel, the launch before (with the fused
  // ingest of the new rows): here the tile is staged once and stays resident ----
  if (row) {
    const int64_t row0 = (int64_t)wt.ring_tile(wg) * 32;
    const int yv = tid < 32 ? dv.y[row0 + tid] : 0;  // issued with the tile's loads
    stage_tile<FP>(lf, dv.X, row0, 32, cfg.cap, false);
    if (tid < 32) ((int*)(lf + 32 * FP * 2 + 8192 + 2048))[tid] = yv;  // fwd_body's label slots
  }
  if (owner) copy_words_to_lds<sizeof(Ctrl) / 8, 256>((unsigned long long*)cl, (const unsigned long long*)gctrl);
  __syncthreads();
  if (wg == 0 && tid == 0) stamp(dv, 30, 4);
  // ---- slots ----
  int phase = kPhInit;
  for (int slot = 0; slot < cfg.nslots; ++slot) {
    if (phase == kPhDone) break;  // uniform: every workgroup holds the same phase
    if (row) {
      constexpr int NT = FP / 64;
      f32x4 acc[NT];
#pragma unroll
      for (int n = 0; n < NT; ++n) acc[n] = f32x4{0, 0, 0, 0};
      fwd_body<FP, true, false, S>(cfg, win, slot, dv, lf, wg, G, acc);
      store_gpf<FP, S == 1>(dv, wg, G, acc);  // this tile's R^T X partials (sc1 | plain: in-XCD)
    }
    barrier();
    if (owner) bwd_body<FP, KP, S>(cfg, win, gctrl, slot, dv, G, lb, wg, NS);
    if (wg == 0 && tid == 0) st_h64<S>(xch + kXchPhase, (unsigned long long)(unsigned)cl->phase);
    barrier();
    phase = owner ? cl->phase : (int)(unsigned)ld_h64<S>(xch + kXchPhase);
  }
  // ---- F: slice owners finalise their features ----
  if (owner) {
    if (nride > 0) {  // the riding evaluation still reads the fragments written below
      if (tid == 0) {
        unsigned long long* rc = xch + kXchRide + (run & 1u);
        int spins = 0;
        while (xload(rc) < (unsigned long long)nride) {
          __builtin_amdgcn_s_sleep(2);
          if (++spins > spin_limit(dv)) {
            xstore(err, 4ull);
            break;
          }
        }
      }
      __syncthreads();
    }
    FinIn<KP> in;
    const int f = wg * 32 + tid;
    if (tid < 32) in.load_f(cfg, dv, f);
    if (wg == 0 && tid == 0) stamp(dv, 30, 2);
    if (tid < 32) finalize_feature<KP>(cfg, dv, f, in);
    if (wg == 0) {
      __syncthreads();  // (the intercept entries of x were written by this workgroup's threads)
      if (tid == 0) {
        finalize_scalars<KP>(cfg, cl, dv);
        xstore(xch + kXchGen + ((run + 1u) & 1u), 0ull);  // re-arm the next run's counters
        xstore(xch + kXchRide + ((run + 1u) & 1u), 0ull);
      }
      // the controller state for the host / later launches
      constexpr int CW = sizeof(Ctrl) / 8;
      for (int i = tid; i < CW; i += 256) ((unsigned long long*)gctrl)[i] = ((const unsigned long long*)cl)[i];
    }
  }
}

template <int FP, int S>
static void launch_persist_fps(const SolverCfg& cfg, const SolveDev& dv, Ctrl* ctrl, const SolveParams& win, int G,
                               const EvalRide& ride, int nride, hipStream_t s) {
  const size_t lb = persist_lds_bytes(FP);
  const int grid = xcd_grid(G, nride, S == 2, cfg.xcd & 7);
  switch (dv.KP) {
    case 2: solve_persist_kernel<FP, 2, S><<<grid, 256, lb, s>>>(cfg, dv, ctrl, win, G, ride, nride); break;
    case 4: solve_persist_kernel<FP, 4, S><<<grid, 256, lb, s>>>(cfg, dv, ctrl, win, G, ride, nride); break;
    default: solve_persist_kernel<FP, 8, S><<<grid, 256, lb, s>>>(cfg, dv, ctrl, win, G, ride, nride); break;
  }
}

template <int FP>
static void launch_persist_fp(const SolverCfg& cfg, const SolveDev& dv, Ctrl* ctrl, const SolveParams& win, int G,
                              const EvalRide& ride, int nride, hipStream_t s) {
  // one XCD when the solve workgroups fit its CUs (PSX_PERSIST_XCD=0: always spread)
  static const bool xcd_ok = [] {
    const char* e = std::getenv("PSX_PERSIST_XCD");
    return !(e && e[0] == '0');
  }();
  if (xcd_ok && G <= kMaxXcdWg && cfg.xcd >= 0)
    launch_persist_fps<FP, 2>(cfg, dv, ctrl, win, G, ride, nride, s);
  else
    launch_persist_fps<FP, 1>(cfg, dv, ctrl, win, G, ride, nride, s);
}

bool persist_supported(int FP, int KP) { return FP >= 128 && FP <= 1024 && KP <= 8; }

void launch_persist(const SolverCfg& cfg, const SolveDev& dv, Ctrl* ctrl, const SolveParams& win, int G,
                    const EvalRide& ride, int nride, hipStream_t s) {
  switch (cfg.Fp) {
    case 128: launch_persist_fp<128>(cfg, dv, ctrl, win, G, ride, nride, s); break;
    case 256: launch_persist_fp<256>(cfg, dv, ctrl, win, G, ride, nride, s); break;
    case 512: launch_persist_fp<512>(cfg, dv, ctrl, win, G, ride, nride, s); break;
    case 1024: launch_persist_fp<1024>(cfg, dv, ctrl, win, G, ride, nride, s); break;
    default: break;
  }
}

template <int FP>
static void set_persist_attr() {
  const int b = (int)persist_lds_bytes(FP);
  (void)hipFuncSetAttribute((const void*)solve_persist_kernel<FP, 2, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, b);
  (void)hipFuncSetAttribute((const void*)solve_persist_kernel<FP, 4, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, b);
  (void)hipFuncSetAttribute((const void*)solve_persist_kernel<FP, 8, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, b);
  (void)hipFuncSetAttribute((const void*)solve_persist_kernel<FP, 2, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, b);
  (void)hipFuncSetAttribute((const void*)solve_persist_kernel<FP, 4, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, b);
  (void)hipFuncSetAttribute((const void*)solve_persist_kernel<FP, 8, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, b);
}

template <int FP>
static void set_slot_attr() {
  const int tb = (int)tail_lds_bytes(FP);
  (void)hipFuncSetAttribute((const void*)tail_kernel<FP, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, tb);
  (void)hipFuncSetAttribute((const void*)tail_kernel<FP, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, tb);
  (void)hipFuncSetAttribute((const void*)tail_kernel<FP, 8>, hipFuncAttributeMaxDynamicSharedMemorySize, tb);
  (void)hipFuncSetAttribute((const void*)tail_kernel<FP, 16>, hipFuncAttributeMaxDynamicSharedMemorySize, tb);
  (void)hipFuncSetAttribute((const void*)fwd_kernel<FP>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)fwd_lds_bytes(FP));
  (void)hipFuncSetAttribute((const void*)fwdbwd_rows_kernel<FP>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)fwd_lds_bytes(FP));
  if constexpr (FP <= 1024)
    (void)hipFuncSetAttribute((const void*)fwdbwd_rows_kernel<FP, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)fwdbwd_rows_lds_bytes(FP, true));
  const int b = (int)bwd_ride_lds_bytes(FP);
  (void)hipFuncSetAttribute((const void*)bwd_update_kernel<FP, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, b);
  (void)hipFuncSetAttribute((const void*)bwd_update_kernel<FP, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, b);
  (void)hipFuncSetAttribute((const void*)bwd_update_kernel<FP, 8>, hipFuncAttributeMaxDynamicSharedMemorySize, b);
  (void)hipFuncSetAttribute((const void*)bwd_update_kernel<FP, 16>, hipFuncAttributeMaxDynamicSharedMemorySize, b);
}

void prepare_solve_kernels() {
  static bool done = false;
  if (done) return;
  set_slot_attr<128>();
  set_slot_attr<256>();
  set_slot_attr<512>();
  set_slot_attr<1024>();
  set_slot_attr<2048>();
  set_persist_attr<128>();
  set_persist_attr<256>();
  set_persist_attr<512>();
  set_persist_attr<1024>();
  done = true;
}

}  // namespace psx
