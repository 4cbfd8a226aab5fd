// Multi-lane BSP round kernel (see lanes_kernels.h).
#include "lanes_kernels.h"

#include <cstdlib>

#include "lanes_body.h"
#include "solve_body.h"

namespace psx {

bool lanes_supported(int FP, int K, int cap) {
  // (rings over 32 tiles: each row workgroup stages several tiles every slot)
  return FP >= 128 && FP <= 1024 && (FP & (FP - 1)) == 0 && K >= 2 && K <= 8 && cap >= 32 && cap % 32 == 0 &&
         cap <= kLanesMaxCap;
}
size_t lanes_lds_bytes(int FP) { return persist_fwd_bytes(FP) + (kBwdLdsBytes + 15) / 16 * 16 + kSyBytes; }
int lanes_grid(int L, int min_riders) {
  const int g = L * kLaneWg + min_riders;
  return g > 8 * kLaneWg ? g : 8 * kLaneWg;
}

namespace {
using namespace lanes_detail;

constexpr int kSkipRole = -(1 << 30);  // a workgroup on an XCD of LanesArgs::xcd_skip

// LE: the lanes evaluate their own models after the solve (LanesArgs::lane_eval).  A
// template flag, not a run-time test: the evaluation tail compiled into the kernel
// costs the solve its registers (1208 B of scratch against 120 B without it).
template <int FP, int KP, int S, bool LE>
__global__ __launch_bounds__(256) void lanes_round_kernel(SolverCfg cfg, const LaneDev* __restrict__ lanes,
                                                          LanesArgs a) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int b = (int)blockIdx.x, tid = threadIdx.x, L = a.L;
  int l, wg;
  {
    __shared__ int role;
    if (tid == 0) {
      if (a.ev.dbg)  // PSX_LANES_STAMPS: the earliest workgroup entry of the launch ([15])
        atomicMin((unsigned long long*)(a.ev.dbg + 15), (unsigned long long)__builtin_amdgcn_s_memrealtime());
      unsigned* c = a.claim + 32 * a.cpar;
      const int xcc = (int)(__builtin_amdgcn_s_getreg((3 << 11) | 20) & 15u);  // HW_REG_XCC_ID
      const bool skip = ((a.xcd_skip >> xcc) & 1u) != 0u;
      // (a skipped workgroup -- another process's XCD -- may be placed late: it touches
      // nothing, and the first workgroup of every other XCD resets the counters instead)
      if (b < 8 && !skip) {  // the other parity's counters (the previous launch has claimed) for the next launch
        for (int j = 0; j < 32; ++j)
          __hip_atomic_store(a.claim + 32 * (a.cpar ^ 1) + j, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (reset before this launch counts as dispatched)
      }
      // every workgroup not skipped: the launch is fully dispatched once this reaches the
      // grid less the skipped XCDs' share (the next overlapped launch waits for that)
      if (!skip) (void)__hip_atomic_fetch_add(c + 9, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      int r = -1;
      if (skip) {
        r = kSkipRole;  // another process's XCD (shared-GPU rehearsals): leave at once
      } else if constexpr (S == 2) {  // the XCD this workgroup runs on decides its lane
        const int lx = xcc - a.xcd0;
        if (lx >= 0 && lx < L) {
          const unsigned k = __hip_atomic_fetch_add(c + lx, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (k < (unsigned)kLaneWg) r = lx * kLaneWg + (int)k;
        }
      } else if (b < 8 * kLaneWg && (b & 7) - a.xcd0 >= 0 && (b & 7) - a.xcd0 < L) {  // spread: any placement works
        r = ((b & 7) - a.xcd0) * kLaneWg + (b >> 3);
      }
      if (r == -1) r = -(int)__hip_atomic_fetch_add(c + 8, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - 1;
      role = r;
    }
    __syncthreads();
    const int r = __builtin_amdgcn_readfirstlane(role);  // (uniform: lane / workgroup indices in SGPRs)
    __syncthreads();
    if (r == kSkipRole) return;
    if (r < 0) {  // a rider: the previous round's evaluation
      if (a.ovl && a.ev.nmodels > 0)  // round - 1's launch complete: its fragments written back
        wait_ge(a.evdone, a.round, (unsigned long long*)nullptr, a.spin_max > 0 ? a.spin_max : 1 << 22);
      if (a.ev.form == 1)
        eval_tile_body<FP>(lds, a.ev, -r - 1, a.lane_riders ? (int)a.ev.nticket : a.nride);
      else
        eval_multi_body<FP>(lds, a.ev, -r - 1, a.nride);
      return;
    }
    l = r / kLaneWg;
    wg = r - l * kLaneWg;
  }
  // a lane workgroup whose part of the round is done joins the evaluation (lane_riders)
  auto join_eval = [&]() {
    if (!a.lane_riders) return;
    if (a.ovl && a.ev.nmodels > 0)  // round - 1's launch complete: its fragments written back
      wait_ge(a.evdone, a.round, (unsigned long long*)nullptr, a.spin_max > 0 ? a.spin_max : 1 << 22);
    eval_tile_body<FP>(lds, a.ev, a.nride + l * kLaneWg + wg, (int)a.ev.nticket);
  };
  constexpr int NS = FP / 32;
  const LaneRound rr = pick(a.r, l);
  const SolveParams win{rr.B, rr.start, 0, 0};
  const WinTiles wt(win.start, win.B, cfg.cap);
  const int ntt = wt.nt < wt.T ? wt.nt : wt.T;   // ring tiles of the window
  const int ntr = ntt < kLaneWg ? ntt : kLaneWg;  // row workgroups (tiles wg, wg + ntr, ...)
  const int G = ntr > NS ? ntr : NS;
  if (wg >= G) {
    join_eval();
    return;
  }
  SolveDev dv = lanes[l].dv;
  dv.out_hi = lanes[l].ohi[a.par];
  dv.out_lo = lanes[l].olo[a.par];
  dv.b_fin = lanes[l].ob[a.par];
  dv.loss = lanes[l].loss2 + a.par;
  dv.w_old = a.ovl ? lanes[l].wpull : a.w;  // (overlapped: the slice's copy pulled below)
  dv.w_new = nullptr;
  dv.ap_w = nullptr;
  dv.spin_max = a.spin_max;
  char* lf = lds;                          // row role: the resident tile + forward scratch
  char* lb = lds + persist_fwd_bytes(FP);  // slice role: bwd_body's region
  float* lsy = (float*)(lb + (kBwdLdsBytes + 15) / 16 * 16);  // curvature pairs (phase I: scratch)
  unsigned short* frl = (unsigned short*)(lb + 4 * 16 * 32 * 4);
  Ctrl* cl = (Ctrl*)(frl + 1024);  // bwd_body's controller copy (persists across slots)
  int* flag = (int*)(lsy + 8192);
  const bool owner = wg < NS;
  __shared__ int ovl_late;
  if (a.ovl) {
    // Overlapped launches: the previous round's launch may still run (its evaluation).
    // Every slice of its update applied means every lane is past that round (the last
    // lane to arrive on a slice applies it; each lane's workgroup 0 arrives on slice 0
    // after advancing its run counter), so its rings, workspaces and counters are free
    // and w holds the update (written through).  Then an acquire: this CU's L1 may hold
    // lines of them cached by the previous round's workgroups after this launch began.
    if (tid == 0) ovl_late = 0;
    __syncthreads();
    if (tid < NS) {
      if (a.rx_tag) {
        // peer_sum: this slice of the server's update of round - 1, written into this
        // rank's receive slot over xGMI (system scope), then its tag; a wall-clock budget
        // (the slowest rank's round, which may wait for its rows, gates the update)
        const long long t_end = rt_now() + a.peer_ticks;
        while ((int)(ld_sys_u32(a.rx_tag + tid) - a.round) < 0) {
          if (rt_now() > t_end) {
            ovl_late = 1;
            break;
          }
          __builtin_amdgcn_s_sleep(2);
        }
      } else {
        const int sp = spin_limit(dv);
        int spins = 0;
        while ((int)(__hip_atomic_load(a.applied + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - a.round) < 0) {
          __builtin_amdgcn_s_sleep(2);
          if (++spins > sp) {  // never expected: reported below (after this round's error word is cleared)
            ovl_late = 1;
            break;
          }
        }
      }
    }
    // (one wave: the L1 is the CU's, and four waves fencing queue four invalidates;
    // behind every polling wave)
    if constexpr (NS > 64) __syncthreads();
    // (peer_sum: the receive slot is read with system-scope loads below, which the
    // server's sc0 sc1 stores + tag need no acquire for; this CU's L1 still needs the
    // agent acquire for the previous round's rings and workspaces)
    if (tid < 64) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
  }
  const unsigned run = a.ovl ? __hip_atomic_load(dv.prm_count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                             : *dv.prm_count;
  unsigned long long* xch = dv.xch;
  unsigned long long* bar = xch + kXchGen + (run & 1u);
  unsigned long long* err = xch + kXchErr;
  const int spin = spin_limit(dv);
  unsigned long long nb = 0;
  auto barrier = [&]() {
    ++nb;
    if constexpr (S == 2)
      x_barrier(xch + kXchFlags, wg, G, ((unsigned long long)run << 16) | nb, err, spin);
    else
      p_barrier(bar, (unsigned long long)G * nb, err, spin);
  };
  const bool row = wg < ntr;
  const int K = cfg.K, FPr = FP;
  if (wg == 0 && tid == 0) {
    xstore(err, 0ull);  // this round's sticky error word (set by any timed-out wait below)
    if constexpr (S == 1) xstore(xch + kXchGen + ((run + 1u) & 1u), 0ull);  // re-arm the next run's counter
    if (rr.delay_us > 0) {  // injected straggler (--inject_worker_delay): the lane's solve starts late
      const long long t0 = rt_now();
      while (rt_now() - t0 < (long long)rr.delay_us * (kRtTicksPerS / 1000000)) __builtin_amdgcn_s_sleep(64);
    }
  }
  // the pulled weights of this slice, fetched first (their latency overlaps the staging)
  float wo_pre = 0.f, b_pre = 0.f;
  if (owner) {
    const int c = tid >> 5, f = wg * 32 + (tid & 31);
    if (a.ovl) {  // the previous round's update of this slice is in w (written through, waited for above)
      if (a.rx) {  // peer_sum: in this rank's receive slot (the server GPU's system-scope stores)
        if (c < K && f < cfg.F) wo_pre = ld_sys_f32(a.rx + (size_t)c * FPr + f);
        if (wg == 0 && tid < K) b_pre = ld_sys_f32(a.rx + (size_t)K * FPr + tid);
      } else {
        if (c < K && f < cfg.F) wo_pre = ld_sc1(a.w + (size_t)c * FPr + f);
        if (wg == 0 && tid < K) b_pre = ld_sc1(a.w + (size_t)K * FPr + tid);
      }
      if (c < K) lanes[l].wpull[(size_t)c * FPr + f] = wo_pre;  // the solve's w_old (this slice)
      if (wg == 0 && tid < K) lanes[l].wpull[(size_t)K * FPr + tid] = b_pre;
    } else {
      if (c < K && f < cfg.F) wo_pre = a.w[(size_t)c * FPr + f];
      if (wg == 0 && tid < K) b_pre = a.w[(size_t)K * FPr + tid];
    }
  }
  // --trace: the lane's phase times of this round (one lane thread)
  auto trace = [&](int k) {
    if (a.tr && wg == 0 && tid == 0) a.tr[((size_t)a.tr_slot * kMaxLanes + l) * 4 + k] = rt_now();
  };
  // ---- phase I: stage + ingest + window statistics, then x0 / first trial point ----
  if (wg == 0 && tid == 0) stamp(dv, 30, 0);
  trace(0);
  if (row) {
    lane_stage_stats<FP, S>(lf, lsy, cfg, dv, rr, a.dsX, a.dsy, wt, wg, ntr, ntt,
                            lanes[l].spart + (size_t)wg * FP * 2);
  }
  if (wg == 0 && tid == 0) stamp(dv, 30, 1);
  barrier();
  if (wg == 0 && tid == 0) stamp(dv, 30, 2);
  if (a.ovl && tid == 0 && ovl_late) xstore(err, 9ull);  // (after workgroup 0 cleared the error word)
  if (owner) {
    lane_prep<FP, KP, S>(lb, cfg, dv, lanes[l].spart, ntr, win.B, wg, wo_pre, b_pre);
    if (tid == 0) ctrl_init(*cl);
  }
  barrier();
  if (wg == 0 && tid == 0) stamp(dv, 30, 3);
  trace(1);
  // ---- slots (as solve_persist_kernel) ----
  // Every workgroup a slice owner (G == NS: the window has no more tiles than the
  // model has 32-feature slices): the controller's phase is in every workgroup's
  // LDS copy, so the slot that ends the solve finalises each slice in place, from
  // the registers of its backward (delta written through for the cross-lane sum),
  // and skips the last grid barrier -- no later forward reads its trial point.
  const bool inplace = G == NS;
  int phase = kPhInit;
  for (int slot = 0; slot < cfg.nslots; ++slot) {
    if (phase == kPhDone) break;  // uniform: every workgroup holds the same phase
    if (row) {
      constexpr int NT = FP / 64;
      f32x4 acc[NT];
#pragma unroll
      for (int n = 0; n < NT; ++n) acc[n] = f32x4{0, 0, 0, 0};
      if (ntt > kLaneWg)  // (several ring tiles per row workgroup: staged every slot)
        fwd_body<FP, true, false, S, true, true>(cfg, win, slot, dv, lf, wg, G, acc);
      else
        fwd_body<FP, true, false, S, true>(cfg, win, slot, dv, lf, wg, G, acc);
      store_gpf<FP, S == 1>(dv, wg, G, acc);
      if (wg == 0 && tid == 0) stamp(dv, slot, 15);
    }
    barrier();
    if (owner)
      bwd_body<FP, KP, S>(cfg, win, lanes[l].ctrl, slot, dv, G, lb, wg, NS, false, inplace ? 0 : kNoFinSlot,
                          /*fin_sc1=*/true);
    if (inplace && cl->phase == kPhDone) {
      phase = kPhDone;
      break;
    }
    if (wg == 0 && tid == 0) st_h64<S>(xch + kXchPhase, (unsigned long long)(unsigned)cl->phase);
    barrier();
    phase = owner ? cl->phase : (int)(unsigned)ld_h64<S>(xch + kXchPhase);
  }
  if (!owner && !LE) {
    join_eval();
    return;
  }
  if (owner) {
    if (wg == 0 && tid == 0) stamp(dv, 30, 4);
    trace(2);
    // ---- finalisation of this slice (delta written through for the cross-lane sum) ----
    if (!inplace) {
      FinIn<KP> in;
      const int f = wg * 32 + tid;
      if (tid < 32) {
        in.load_f(cfg, dv, f);
        finalize_feature<KP>(cfg, dv, f, in, /*sc1_delta=*/true);
      }
    }
    if (wg == 0) {
      __syncthreads();  // (the intercept entries of x were written by this workgroup's threads)
      if (tid == 0) {
        FinScal sc;
        sc.load(cfg, cl, dv);
        sc.store(cfg, dv, /*sc1_delta=*/true, /*clear_err=*/false);
      }
      constexpr int CW = sizeof(Ctrl) / 8;
      for (int k = tid; k < CW; k += 256) ((unsigned long long*)lanes[l].ctrl)[k] = ((const unsigned long long*)cl)[k];
    }
    // ---- the BSP update: the last lane to finish a slice applies the sum ----
    if (wg == 0 && tid == 0) stamp(dv, 30, 5);
    if (lane_arrive(a.arrive, wg, L, flag)) {
      lane_apply_slice<FP>(cfg, lanes,
                           ApplyArgs{L, a.w, a.lr, a.dsum, a.shi, a.slo, a.sb, a.scoff, a.ovl ? a.applied : nullptr,
                                     a.round, a.push, a.push_tag, a.round + 1u},
                           wg);
    }
    if (wg == 0 && tid == 0) stamp(dv, 30, 6);
    trace(3);
  }
  if constexpr (!LE) {
    join_eval();
    return;
  }
  // ---- the lane's own evaluation of this round's local model (+ the previous update's
  // global model on lane 0), while the other lanes still solve ----
  if constexpr (S == 1) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");  // fragments across XCDs
  barrier();
  if constexpr (S == 1) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  {
    const EvalModel Am = pick(a.ev.m, l), Bm = a.ev.m[kMaxEvalModels - 1];
    PairModels pm;
    pm.ah = Am.hi;
    pm.al = Am.lo;
    pm.ab = Am.b;
    pm.aloss = Am.loss;
    pm.aslot = Am.slot;
    pm.aseq = (unsigned)Am.seq;
    pm.acoff = Am.coff;
    pm.bh = Bm.hi;
    pm.bl = Bm.lo;
    pm.bb = Bm.b;
    pm.bslot = l == 0 ? Bm.slot : nullptr;
    pm.bseq = (unsigned)Bm.seq;
    pm.bcoff = Bm.coff;
    if (wg == 0 && tid == 0) stamp(dv, 30, 7);
    lane_pair_eval<FP>(lds, cfg.K, a.ev.Xt, a.ev.yt, a.ev.T, wg, G, pm,
                       a.lacc + (size_t)l * 2 * 256 * kAccStride, a.lticket + 32 * l);
    if (wg == 0 && tid == 0) stamp(dv, 30, 8);
  }
}

__global__ void xcc_probe_kernel(int* ids, int n) {
  if (threadIdx.x == 0 && (int)blockIdx.x < n)
    ids[blockIdx.x] = (int)(__builtin_amdgcn_s_getreg((3 << 11) | 20) & 15u);  // HW_REG_XCC_ID
}

template <int FP, int KP, int S, bool LE>
void set_lanes_attr() {
  (void)hipFuncSetAttribute((const void*)lanes_round_kernel<FP, KP, S, LE>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lanes_lds_bytes(FP));
}

template <int FP, int KP, int S, bool LE>
void launch_fks(const SolverCfg& cfg, const LaneDev* lanes, const LanesArgs& a, hipStream_t s) {
  static const bool prepared = (set_lanes_attr<FP, KP, S, LE>(), true);
  (void)prepared;
  const int grid = lanes_grid(a.L, a.nride);
  lanes_round_kernel<FP, KP, S, LE><<<grid, 256, lanes_lds_bytes(FP), s>>>(cfg, lanes, a);
}

// Lane evaluation is only built for the XCD-resident form (S == 2, the MI355X
// default); LanesLoop never asks for it with S == 1.
template <int FP, int KP>
void launch_fk(const SolverCfg& cfg, const LaneDev* lanes, const LanesArgs& a, int S, hipStream_t s) {
  if (S == 2 && a.lane_eval)
    launch_fks<FP, KP, 2, true>(cfg, lanes, a, s);
  else if (S == 2)
    launch_fks<FP, KP, 2, false>(cfg, lanes, a, s);
  else
    launch_fks<FP, KP, 1, false>(cfg, lanes, a, s);
}

template <int FP>
void launch_f(const SolverCfg& cfg, const LaneDev* lanes, const LanesArgs& a, int S, hipStream_t s) {
  const int KP = padded_classes(cfg.K);
  if (KP <= 2)
    launch_fk<FP, 2>(cfg, lanes, a, S, s);
  else if (KP <= 4)
    launch_fk<FP, 4>(cfg, lanes, a, S, s);
  else
    launch_fk<FP, 8>(cfg, lanes, a, S, s);
}

}  // namespace

void launch_lanes_round(const SolverCfg& cfg, const LaneDev* lanes_dev, const LanesArgs& a, int S, hipStream_t s) {
  switch (cfg.Fp) {
    case 128: launch_f<128>(cfg, lanes_dev, a, S, s); break;
    case 256: launch_f<256>(cfg, lanes_dev, a, S, s); break;
    case 512: launch_f<512>(cfg, lanes_dev, a, S, s); break;
    case 1024: launch_f<1024>(cfg, lanes_dev, a, S, s); break;
    default: break;
  }
}

void launch_xcc_probe(int* ids, int n, hipStream_t s) { xcc_probe_kernel<<<n, 64, 0, s>>>(ids, n); }

namespace {
// Workgroup m: model m's counts summed over the riders' slab rows (4 row groups of
// 64 cells, integer sums: any order gives the same counts), then its slot as tagged
// 16-B system-scope chunks (publish_counts' format).  Block 0 clears the tile queue.
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8))) void lanes_publish_kernel(EvalMulti ev) {
  __shared__ int part[4][kSlabCells];
  __shared__ int cells[kSlabCells];
  const int m = (int)blockIdx.x, tid = threadIdx.x, K = ev.K, KK = K * K;
  const int c = tid & 63, g = tid >> 6;
  int t = 0;
  const int* col = ev.slab + (size_t)m * kSlabCells + c;
  for (int r = g; r < (int)ev.nticket; r += 4) t += col[(size_t)r * kMaxEvalModels * kSlabCells];
  part[g][c] = t;
  __syncthreads();
  if (tid < KK) {
    const int yl = tid / K, p = tid - yl * K, cc = yl * 8 + p;
    cells[tid] = part[0][cc] + part[1][cc] + part[2][cc] + part[3][cc];
  }
  if (m == 0 && ev.xq && tid < (ev.gq ? kEvalGroups : 1))
    __hip_atomic_store(ev.xq + tid, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  if (tid < 64) {
    const EvalModel E = pick(ev.m, m);
    const unsigned tag = eval_tag(E.seq);
    const int nch = 1 + (KK + 2) / 3;
    TagChunk ch;
    if (tid == 0) {
      const float lv = E.loss ? *E.loss : 0.f;
      ch = TagChunk{tag, (unsigned)__float_as_int(lv), (unsigned)K, 0u};
    } else {
      const int c0 = 3 * (tid - 1);
      auto cv = [&](int q) { return q < KK ? (unsigned)cells[q] : 0u; };
      ch = TagChunk{tag, cv(c0), cv(c0 + 1), cv(c0 + 2)};
    }
    if (tid < nch) st_sys_chunk(E.slot, 1088u, (unsigned)tid * 16u, ch);
  }
}
}  // namespace

namespace {
__global__ void clock_probe_kernel(long long* out) {
  if (threadIdx.x == 0) __hip_atomic_store(out, rt_now(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
}  // namespace

void launch_clock_probe(long long* out, hipStream_t s) { clock_probe_kernel<<<1, 64, 0, s>>>(out); }

void launch_lanes_publish(const EvalMulti& ev, hipStream_t s) {
  if (ev.nmodels <= 0 || !ev.slab) return;
  lanes_publish_kernel<<<ev.nmodels, 256, 0, s>>>(ev);
}

namespace {
// grid (blocks per lane, L): the lane's delta in float4 pieces, its loss by block 0
__global__ __launch_bounds__(256) void lanes_copy_out_kernel(LanesCopyOut c) {
  const int l = (int)blockIdx.y;
  const LanesCopyOut& cc = c;
  const float* sd = pick(cc.src_d, l);
  float* dd = pick(cc.dst_d, l);
  if (dd) {
    const int n4 = c.P / 4;
    for (int i = (int)(blockIdx.x * blockDim.x + threadIdx.x); i < n4; i += (int)(gridDim.x * blockDim.x))
      ((f32x4*)dd)[i] = ((const f32x4*)sd)[i];
    if (blockIdx.x == 0 && (int)threadIdx.x < c.P - 4 * n4) dd[4 * n4 + threadIdx.x] = sd[4 * n4 + threadIdx.x];
  }
  float* dl = pick(cc.dst_l, l);
  if (dl && blockIdx.x == 0 && threadIdx.x == 0) *dl = *pick(cc.src_l, l);
}
}  // namespace

namespace {
// block s: slice s of w (32 features x K classes; block 0 also the intercepts) from the
// receive slot once its tag reached `want`
__global__ __launch_bounds__(256) void peer_pull_kernel(const float* rx, const unsigned* rx_tag, unsigned want,
                                                        float* w, int K, int FP, long long ticks,
                                                        unsigned long long* err_host) {
  const int s = (int)blockIdx.x, tid = threadIdx.x;
  __shared__ int late;
  if (tid == 0) {
    const long long t_end = rt_now() + ticks;
    bool l = false;
    while ((int)(ld_sys_u32(rx_tag + s) - want) < 0 && !(l = rt_now() > t_end)) __builtin_amdgcn_s_sleep(4);
    late = l ? 1 : 0;
    if (l && err_host) __hip_atomic_store(err_host, 10ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __syncthreads();
  if (late) return;
  const int c = tid >> 5, f = s * 32 + (tid & 31);
  if (c < K) w[(size_t)c * FP + f] = ld_sys_f32(rx + (size_t)c * FP + f);
  if (s == 0 && tid < K) w[(size_t)K * FP + tid] = ld_sys_f32(rx + (size_t)K * FP + tid);
}
}  // namespace

void launch_peer_pull(const float* rx, const unsigned* rx_tag, unsigned want, float* w, int K, int FP,
                      long long ticks, unsigned long long* err_host, hipStream_t s) {
  if (K < 1 || K > 8 || FP < 32 || FP % 32) return;
  peer_pull_kernel<<<FP / 32, 256, 0, s>>>(rx, rx_tag, want, w, K, FP, ticks, err_host);
}

void launch_lanes_copy_out(const LanesCopyOut& c, hipStream_t s) {
  if (c.L < 1 || c.L > kMaxLanes) return;
  lanes_copy_out_kernel<<<dim3(8, c.L), 256, 0, s>>>(c);
}

namespace {

// ---------------------------------------------------------------------------
// Side-stream evaluation (8 lanes: every XCD solves, so in-launch riders could
// only start once the solves have freed their CUs).  The same models and
// EvalSlot protocol as eval_multi_body, in a launch sized to CO-RUN with the
// next round's kernel: a lane workgroup leaves ~14.5 KB of LDS and ~150 VGPRs
// per SIMD lane free on its CU, and this kernel needs 8.6 KB of LDS and no LDS
// staging -- each wave streams its 256-feature slice of a 16-row test tile from
// global memory straight into the MFMA A operand, against the pair's weight
// fragments held in registers.  Items = (model pair, 16-row tile), pair-major
// contiguous chunks per workgroup.  Co-residence with a lane workgroup needs the
// registers it leaves: 512 - (256 VGPR + 128 AGPR) = 128 per SIMD lane, hence
// waves_per_eu(4) (FP 1024: 128 VGPRs, 5 spilled; without it 134 + 4 did not fit).
template <int FP>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void lanes_eval_kernel(EvalMulti ev) {
  __shared__ f32x4 red[4][64];
  __shared__ int cl[kMaxEvalModels][16][8];  // (>= kMaxEvalModels * 64 + kMaxEvalModels ints: publish_counts' cells)
  __shared__ int last;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int K = ev.K, T = ev.T, M = ev.nmodels;
  if (M <= 0) return;
  const int nT = (T + 15) / 16, npairs = (M + 1) / 2;
  for (int i = tid; i < kMaxEvalModels * 128; i += 256) (&cl[0][0][0])[i] = 0;
  const int items = npairs * nT, chunk = (items + (int)gridDim.x - 1) / (int)gridDim.x;
  const int i0 = (int)blockIdx.x * chunk, i1 = i0 + chunk < items ? i0 + chunk : items;
  const int r = lane & 15, kq = lane >> 4;
  int curp = -1;
  WFrag<FP> wf;
  __syncthreads();
  for (int it = i0; it < i1; ++it) {
    const int p = it / nT, tile = it - p * nT;
    const int ma = 2 * p, mb = 2 * p + 1 < M ? 2 * p + 1 : -1;
    const EvalModel A = pick(ev.m, ma), Bm = pick(ev.m, mb >= 0 ? mb : 0);
    if (p != curp) {  // (workgroup-uniform)
      load_pair_frags<FP>(wf, A, Bm, mb >= 0, K);
      curp = p;
    }
    const int64_t row = (int64_t)tile * 16 + r;
    u16x8 a[WFrag<FP>::KS];
#pragma unroll
    for (int kk = 0; kk < WFrag<FP>::KS; ++kk) {  // the slice's loads all in flight
      const int cg = (w * WFrag<FP>::KS + kk) * 4 + kq;
      a[kk] = row < T ? *(const u16x8*)(ev.Xt + row * FP + cg * 8) : u16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
    f32x4 acc = f32x4{0, 0, 0, 0};
#pragma unroll
    for (int kk = 0; kk < WFrag<FP>::KS; ++kk) {
      acc = mfma16x16x32(as_bf16x8(a[kk]), as_bf16x8(wf.h[kk]), acc);
      acc = mfma16x16x32(as_bf16x8(a[kk]), as_bf16x8(wf.l[kk]), acc);
    }
    red[w][lane] = acc;
    __syncthreads();
    if (tid < 32) {  // (row, model) of the tile: rows 0..15 x models {a, b}
      const int rr = tid & 15, which = tid >> 4;
      const int m = which == 0 ? ma : mb;
      const int64_t grow = (int64_t)tile * 16 + rr;
      if (m >= 0 && grow < T) {
        const float* bb = which == 0 ? A.b + A.coff : Bm.b + Bm.coff;
        int best = 0;
        float bz = -INFINITY;
        for (int c = 0; c < K; ++c) {
          const int ln = (rr >> 2) * 16 + which * 8 + c, reg = rr & 3;
          const float z = red[0][ln][reg] + red[1][ln][reg] + red[2][ln][reg] + red[3][ln][reg] + bb[c];
          if (z > bz) {
            bz = z;
            best = c;
          }
        }
        const int y = ev.yt[grow];
        atomicAdd(&cl[m][y < 0 ? 0 : (y > 15 ? 15 : y)][best], 1);
      }
    }
    __syncthreads();
  }
  const int cp = xcd_copy();
  for (int m = 0; m < M; ++m)
    if (tid < 128) {
      const int v = cl[m][tid >> 3][tid & 7];
      if (v) atomicAdd(acc_cell(ev.acc, cp, m, (tid >> 3) * 16 + (tid & 7)), v);
    }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0)
    last = __hip_atomic_fetch_add(ev.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
  __syncthreads();
  if (!last) return;
  publish_counts(ev, M, tid, &cl[0][0][0]);
}

}  // namespace

int lanes_eval_grid() {  // PSX_SIDE_GRID: workgroups of the evaluation launch (default 256)
  static const int g = [] {
    const char* e = std::getenv("PSX_SIDE_GRID");
    const int v = e ? std::atoi(e) : 256;
    return v >= 1 && v <= 4096 ? v : 256;
  }();
  return g;
}

void launch_lanes_eval(const SolverCfg& cfg, const EvalMulti& ev, hipStream_t s) {
  if (ev.nmodels <= 0) return;
  const int g = lanes_eval_grid();
  switch (cfg.Fp) {
    case 128: lanes_eval_kernel<128><<<g, 256, 0, s>>>(ev); break;
    case 256: lanes_eval_kernel<256><<<g, 256, 0, s>>>(ev); break;
    case 512: lanes_eval_kernel<512><<<g, 256, 0, s>>>(ev); break;
    case 1024: lanes_eval_kernel<1024><<<g, 256, 0, s>>>(ev); break;
    default: break;
  }
}

}  // namespace psx
