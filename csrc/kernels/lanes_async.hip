// Asynchronous (SSP / ASP) multi-lane kernel: ONE persistent launch in which
// every lane (logical worker, one XCD each) loops
//
//   release record (host) -> stage + solve -> push (ticket, serial slice
//   updates, snapshot, token) -> evaluation of its local model (+ the global
//   model on the logging lane) -> next release record
//
// See lanes_kernels.h for the protocol.  Reference: ServerProcessor.java:143-183
// (apply on arrival, one partition = serial updates, server row on worker-0
// deltas, reply to whom the tracker releases), WorkerTrainingProcessor.java:
// 63-98 (pull -> train on the buffer -> log -> push), MessageTracker.java:69-87.
#include <cstdlib>

#include "lanes_body.h"
#include "lanes_kernels.h"
#include "solve_body.h"

namespace psx {
namespace {
using namespace lanes_detail;

// system-coherent 16-B loads of pinned host memory (sc0 | sc1)
__device__ __forceinline__ TagChunk ld_sys_chunk(const void* base, unsigned bytes, unsigned off) {
  return __builtin_bit_cast(TagChunk,
                            __builtin_amdgcn_raw_buffer_load_b128(rsrc_of(base, bytes), (int)off, 0, kAuxSys));
}
__device__ __forceinline__ TagChunk ld_nt_chunk(const void* p) {
  return __builtin_bit_cast(TagChunk, __builtin_nontemporal_load((const u32x4*)p));
}

// The lane's leader waits for its next release record (pinned, written by the
// host loop); wave 0's lanes 0..7 load one 16-B chunk each per poll, so one
// PCIe round trip sees the whole record.  The record goes to the lane's
// broadcast area (its XCD's L2); a timeout becomes a stop record (code 2).
// A record is complete when its 8 chunks carry one tag; it is new when that tag
// is at least the one the lane expects (a stop record written over an unread
// release on the host's error path is newer still).
__device__ __forceinline__ void leader_wait_release(const AsyncLaneDev& A, unsigned want, long long ticks,
                                                    unsigned long long* err_host) {
  const int tid = threadIdx.x;
  if (tid >= 64) return;
  TagChunk c = TagChunk{0, 0, 0, 0};
  bool ok = false;
  const long long t_end = rt_now() + ticks;
  for (;;) {
    if (tid < kRelChunks) c = ld_sys_chunk(A.rel, (unsigned)sizeof(AsyncRelease), (unsigned)tid * 16u);
    const unsigned t0 = __shfl(c.tag, 0, 64);
    ok = __all(tid >= kRelChunks || c.tag == t0) && (int)(t0 - want) >= 0;
    if (ok || rt_now() > t_end) break;
    __builtin_amdgcn_s_sleep(8);
  }
  if (!ok) {  // the host never answered: leave the launch, and say so
    c = TagChunk{want, tid == 0 ? 2u : 0u, 0u, 0u};
    if (tid == 0 && err_host)
      __hip_atomic_store(err_host, (unsigned long long)7, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (tid < kRelChunks) ((TagChunk*)A.rec)[tid] = c;
}

// The lane's sticky error word -> its pinned host word ((solves + 1) << 8 | code,
// the format of FinScal::store), then cleared.  One thread.
__device__ __forceinline__ void report_and_clear(const SolveDev& dv, unsigned long long* err, unsigned run) {
  const unsigned long long e = xload(err);
  if (e) {
    if (dv.err_host)
      __hip_atomic_store(dv.err_host, (unsigned long long)run << 8 | (e & 0xffull), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
    xstore(err, 0ull);
  }
}

// Peer data plane push (remote mode with a mapped server inbox): slice `wg` of
// the lane's delta straight into its slot of the server GPU's inbox over xGMI,
// then the slice's tag = vc + 1 (WorkerTrainingProcessor.java:95-97: the
// GradientMessage of clock vc).  A solve whose wait timed out pushes zeros.
template <int FP>
__device__ __forceinline__ void peer_push_slice(const SolverCfg& cfg, const SolveDev& dv, const AsyncLaneDev& A,
                                                int wg, long long vc, unsigned long long* err) {
  const int tid = threadIdx.x, K = cfg.K;
  const int c = tid >> 5, f = wg * 32 + (tid & 31);
  const bool bad = xload(err) != 0ull;
  if (c < K) {
    const size_t e = (size_t)c * FP + f;
    st_sys_f32(A.inbox + e, bad ? 0.f : ld_sc1(dv.delta + e));
  }
  if (wg == 0 && tid < K) {
    const size_t e = (size_t)K * FP + tid;
    st_sys_f32(A.inbox + e, bad ? 0.f : ld_sc1(dv.delta + e));
  }
  publish_sys_tag(A.inbox_tag + wg, (unsigned)(vc + 1));
}

// The update of slice `wg` by the delta of ticket t, after slice wg of ticket
// t - 1 (serial per slice, in ticket order: the single GRADIENTS_TOPIC
// partition), w += lr * delta (ServerProcessor.java:148-151, 225-228).  The new
// slice also goes to snapshot slot t % R (the weights a release after ticket t
// pulls) and, on the logging lane, to the server-row evaluation fragments.
template <int FP>
__device__ __forceinline__ void async_apply_slice(const SolverCfg& cfg, const SolveDev& dv, const AsyncLaneDev& A,
                                                  const AsyncArgs& a, int wg, unsigned long long t, bool logl,
                                                  unsigned long long* err, int spin, int* flag) {
  const int tid = threadIdx.x, K = cfg.K;
  const int c = tid >> 5, f = wg * 32 + (tid & 31);
  const bool coef = c < K;
  const bool icpt = wg == 0 && tid < K;
  const size_t e = (size_t)c * FP + f, ei = (size_t)K * FP + tid;
  // a solve whose cross-workgroup wait timed out contributes nothing (its loss is NaN)
  const bool bad = xload(err) != 0ull;
  float dl = 0.f, di = 0.f;
  if (coef && !bad) dl = ld_sc1(dv.delta + e);
  if (icpt && !bad) di = ld_sc1(dv.delta + ei);
  if (a.dbg_delta) {  // (tests) the delta of ticket t as applied
    float* dd = a.dbg_delta + (size_t)((t - 1ull) % (unsigned long long)a.dbg_cap) * (size_t)cfg.P;
    if (coef) dd[e] = dl;
    if (icpt) dd[ei] = di;
  }
  unsigned long long* turn = a.turn + (size_t)wg * 32;
  if (tid == 0) {
    int spins = 0;
    while (xload(turn) + 1ull != t) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > spin) {  // never expected: record and go on
        xstore(err, 6ull);
        break;
      }
    }
  }
  __syncthreads();
  const size_t so = (size_t)(t % (unsigned long long)a.R) * (size_t)a.sstride;
  if (coef) {
    const float nw = ld_sc1(a.w + e) + a.lr * dl;
    st_sc1(a.w + e, nw);
    st_sc1(a.snap + so + e, nw);
    if (logl) write_frag(A.shi, A.slo, c, f, f < cfg.F ? nw : 0.f);
  }
  if (icpt) {
    const float nw = ld_sc1(a.w + ei) + a.lr * di;
    st_sc1(a.w + ei, nw);
    st_sc1(a.snap + so + ei, nw);
    if (logl) A.sb[tid] = nw;
  }
  if (tid == 0)
    __hip_atomic_store(a.snap_tag + (size_t)(t % (unsigned long long)a.R) * (FP / 32) + wg, (unsigned)t,
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) xstore(turn, t);
  (void)flag;
}

// A pointer the compiler must treat as new on every loop iteration: the loads
// through it stay inside the iteration instead of being hoisted in front of the
// persistent loop (where their values would be live across it -- hundreds of
// registers of structure fields, spilled).
template <typename T>
__device__ __forceinline__ const T* fresh(const T* p) {
  asm volatile("" : "+s"(p));
  return p;
}

// One iteration of lane l's loop (workgroup wg): release -> solve -> push ->
// evaluation.  false: the lane got its stop record.
// MT: rings over 32 tiles possible (a build of its own: the restaging forward's
// registers would spill in the resident form -- 192 B of scratch, 62.6k -> 58.0k
// updates/s, profiles/r04/s19)
template <int FP, int KP, int S, bool MT>
__device__ __forceinline__ bool async_iteration(char* lds, const SolverCfg& cfg_mem, const AsyncArgs& a,
                                                const AsyncLaneDev& A, int l, int wg, unsigned& run,
                                                unsigned long long& relc, unsigned long long& lw) {
  constexpr int NS = FP / 32;
  const SolverCfg& cfg = cfg_mem;  // (by value: 300 B of scratch, no faster -- profiles/r05/README.md)
  const int tid = threadIdx.x, K = cfg.K;
  // The solver's pointers BY VALUE (registers), not a reference into the launch's device
  // table: every spin loop's memory clobber and every acquire fence of the hand-offs
  // would otherwise re-issue their loads -- a memory round trip ahead of each phase's
  // data loads (measured: 78-96 us per solve by reference, 63-76 by value, against 56-66
  // in the BSP round kernel, which holds its SolveDev by value; profiles/r05/README.md)
  const SolveDev dv = A.dv;
  unsigned long long* const xch = dv.xch;
  unsigned long long* const err = xch + kXchErr;
  // ---- 1. the release record ----
  // (PSX_LANES_STAMPS, slot 30 of the lane's table: 0 released, 4 solved, 5 ticket,
  // 6 applied, 7 token out / evaluation starts, 8 evaluation done)
  // (PSX_LANES_STAMPS: the iteration's start and the release record seen, kept as stamps 9
  // / 10 of a real release -- the final stop record does not overwrite them)
  const long long t_it = dv.dbg ? (long long)__builtin_amdgcn_s_memrealtime() : 0;
  if (wg == 0) leader_wait_release(A, (unsigned)(relc + 1), a.rel_ticks, dv.err_host);
  const long long t_rel = dv.dbg ? (long long)__builtin_amdgcn_s_memrealtime() : 0;
  // The lane's sticky error word: a wait that timed out after the previous solve's
  // report (FinScal::store) -- its push (turn words, barriers) or its evaluation --
  // is reported here, then the word is cleared BEFORE the barrier every workgroup
  // of this iteration passes, so nothing stored in this iteration is wiped.
  if (wg == 0 && tid == 0) report_and_clear(dv, err, run);
  // (only the leader publishes through this barrier -- the release record; the others'
  // outstanding stores, e.g. the last evaluation's pinned-slot chunks, need not land first)
  // (no budget of their own for the others: the leader's release wait is bounded and
  // ends in a stop record)
  // (the broadcast area's address in a register across the barrier: read from the lane
  // table behind the acquire it would be one more memory round trip, after the invalidate)
  const unsigned long long* const rec = A.rec;
  x_barrier(A.flags, wg, kLaneWg, ++lw, err, 0x7fffffff, /*drain=*/wg == 0);
  const long long t_bar = dv.dbg ? rt_now() : 0;
  RelRec q;
  {
    // The record BEFORE the acquire: nt loads are served by the XCD's L2, which the
    // leader's stores reached before its barrier word (drain), so they need no
    // invalidate -- and their round trip no longer waits behind it (the record read
    // behind the fence took 7.5 us of the lane's ~100-us iteration, profiles/r05/s39)
    TagChunk ch[kRelChunks];
    // every chunk must carry one tag at least the one the leader waited for: a line of
    // an older record still in this CU's L1 would otherwise replay the previous window
    // silently -- re-read until they do (bounded: a persistent mismatch is error 12)
    const unsigned want = (unsigned)(relc + 1ull);
    for (int tries = 0;; ++tries) {
#pragma unroll
      for (int i = 0; i < kRelChunks; ++i) ch[i] = ld_nt_chunk(rec + 2 * i);
      bool fresh = (int)(ch[0].tag - want) >= 0;
#pragma unroll
      for (int i = 1; i < kRelChunks; ++i) fresh &= ch[i].tag == ch[0].tag;
      if (__syncthreads_and(fresh ? 1 : 0)) break;
      if (tries >= 4096) {
        if (tid == 0) xstore(err, 12ull);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    // the lane's rows, state and the pulled snapshot were written by other CUs
    // (other XCDs for the snapshot) since this CU last read them.  ONE wave invalidates
    // the CU's L1 and waits for it, the others wait at the workgroup barrier: four
    // waves fencing queue four invalidates (6-7.8 us measured, profiles/r05/s41)
    if (tid < 64) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    unpack_release(ch, q);
    relc = ch[0].tag;  // the record consumed
  }
  const long long t_acq = dv.dbg ? rt_now() : 0;
  if (q.stop) {
    if (wg == 0 && tid == 0) {
      *A.relc = relc;
      report_and_clear(dv, err, run);  // (a wait of this iteration's barrier)
    }
    return false;
  }
  if (wg == 0 && tid == 0 && dv.dbg) {
    dv.dbg[30 * 16 + 9] = t_it;
    dv.dbg[30 * 16 + 10] = t_rel;
    dv.dbg[30 * 16 + 11] = t_bar;
    dv.dbg[30 * 16 + 12] = t_acq;
  }
  if (wg == 0 && tid == 0) stamp(dv, 30, 0);
  // --trace: released / solved parked in the lane's two words behind the ring (no
  // registers held across the solve), copied to the ticket's entry after the push
  long long* tr_park = a.tr ? a.tr + (size_t)a.tr_cap * 4 + 2 * l : nullptr;
  if (tr_park && wg == 0 && tid == 0) tr_park[0] = rt_now();
  // ---- 2. the solve (as lanes_round_kernel) ----
  {
    char* lf = lds;
    char* lb = lds + persist_fwd_bytes(FP);
    float* lsy = (float*)(lb + (kBwdLdsBytes + 15) / 16 * 16);
    unsigned short* frl = (unsigned short*)(lb + 4 * 16 * 32 * 4);
    Ctrl* cl = (Ctrl*)(frl + 1024);
    const int spin = spin_limit(dv);
    const SolveParams win{q.r.B, q.r.start, 0, 0};
    const WinTiles wt(win.start, win.B, cfg.cap);
    const int ntt = wt.nt < wt.T ? wt.nt : wt.T;   // ring tiles of the window
    const int ntr = ntt < kLaneWg ? ntt : kLaneWg;  // row workgroups (tiles wg, wg + ntr, ...)
    const int G = ntr > NS ? ntr : NS;
    const bool row = wg < ntr, owner = wg < NS;
    const unsigned rn = run;
    unsigned long long nb = 0;
    auto barrier = [&]() {
      ++nb;
      if constexpr (S == 2)
        x_barrier(xch + kXchFlags, wg, G, ((unsigned long long)rn << 16) | nb, err, spin);
      else
        p_barrier(xch + kXchGen + (rn & 1u), (unsigned long long)G * nb, err, spin);
    };
    if (wg < G) {
      float wo_pre = 0.f, b_pre = 0.f;
      if (owner) {  // the pulled weights of this slice: snapshot -> this solve's private copy
        const int c = tid >> 5, f = wg * 32 + (tid & 31);
        const size_t so = (size_t)(q.snap % (long long)a.R) * (size_t)a.sstride;
        if (a.peer_rx) {
          // peer data plane: the server GPU writes this slice of the lane's receive
          // slot over xGMI and then its tag (system scope); wait for the tag of this
          // pull, acquire, read the slice with system-scope loads
          if (tid == 0) {
            const unsigned* tg = a.snap_tag + (size_t)(q.snap % (long long)a.R) * NS + wg;
            const long long t_end = rt_now() + a.rel_ticks;
            bool late = false;
            while ((int)(ld_sys_u32(tg) - q.pull_tag) < 0 && !(late = rt_now() > t_end)) __builtin_amdgcn_s_sleep(2);
            if (late) xstore(err, 10ull);  // the server's weights never arrived
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
          }
          __syncthreads();
          if (c < K && f < cfg.F) wo_pre = ld_sys_f32(a.snap + so + (size_t)c * FP + f);
          if (wg == 0 && tid < K) b_pre = ld_sys_f32(a.snap + so + (size_t)K * FP + tid);
        } else {
          if (c < K && f < cfg.F) wo_pre = a.snap[so + (size_t)c * FP + f];
          if (wg == 0 && tid < K) b_pre = a.snap[so + (size_t)K * FP + tid];
        }
        if (c < K) A.wpull[(size_t)c * FP + f] = wo_pre;
        if (wg == 0 && tid < K) A.wpull[(size_t)K * FP + tid] = b_pre;
        if (wg == 0 && tid == 0) stamp(dv, 30, 13);  // (the pulled weights read)
        // (the error word was cleared before this iteration's first barrier: this
        // store is not wiped and FinScal::store reports it with the solve)
        if (!a.remote && tid == 0 &&
            a.snap_tag[(size_t)(q.snap % (long long)a.R) * NS + wg] != (unsigned)(unsigned long long)q.snap)
          xstore(err, 8ull);  // the snapshot slot was reused before this lane pulled it
      }
      if (wg == 0 && tid == 0) {
        if constexpr (S == 1) xstore(xch + kXchGen + ((rn + 1u) & 1u), 0ull);
      }
      if (row) {
        lane_stage_stats<FP, S>(lf, lsy, cfg, dv, q.r, a.dsX, a.dsy, wt, wg, ntr, ntt, A.spart + (size_t)wg * FP * 2);
      }
      if (wg == 0 && tid == 0) stamp(dv, 30, 14);  // (staged)
      barrier();
      if (wg == 0 && tid == 0) stamp(dv, 30, 15);  // (every row workgroup staged)
      if (owner) {
        lane_prep<FP, KP, S>(lb, cfg, dv, A.spart, ntr, win.B, wg, wo_pre, b_pre);
        if (tid == 0) ctrl_init(*cl);
      }
      barrier();
      const bool inplace = G == NS;
      int phase = kPhInit;
      for (int slot = 0; slot < cfg.nslots; ++slot) {
        if (phase == kPhDone) break;
        if (row) {
          constexpr int NT = FP / 64;
          f32x4 acc[NT];
#pragma unroll
          for (int n = 0; n < NT; ++n) acc[n] = f32x4{0, 0, 0, 0};
          if (MT && ntt > kLaneWg)  // (several ring tiles per row workgroup: staged every slot)
            fwd_body<FP, true, false, S, true, true>(cfg, win, slot, dv, lf, wg, G, acc);
          else
            fwd_body<FP, true, false, S, true>(cfg, win, slot, dv, lf, wg, G, acc);
          store_gpf<FP, S == 1>(dv, wg, G, acc);
        }
        barrier();
        if (owner)
          bwd_body<FP, KP, S>(cfg, win, A.ctrl, slot, dv, G, lb, wg, NS, false, inplace ? 0 : kNoFinSlot,
                              /*fin_sc1=*/true);
        if (inplace && cl->phase == kPhDone) {
          phase = kPhDone;
          break;
        }
        if (wg == 0 && tid == 0) st_h64<S>(xch + kXchPhase, (unsigned long long)(unsigned)cl->phase);
        barrier();
        phase = owner ? cl->phase : (int)(unsigned)ld_h64<S>(xch + kXchPhase);
      }
      if (owner) {
        if (!inplace) {
          FinIn<KP> in;
          const int f = wg * 32 + tid;
          if (tid < 32) {
            in.load_f(cfg, dv, f);
            finalize_feature<KP>(cfg, dv, f, in, /*sc1_delta=*/true);
          }
        }
        if (wg == 0) {
          __syncthreads();
          if (tid == 0) {
            FinScal sc;
            sc.load(cfg, cl, dv);
            sc.store(cfg, dv, /*sc1_delta=*/true, /*clear_err=*/false);
          }
          constexpr int CW = sizeof(Ctrl) / 8;
          for (int k = tid; k < CW; k += 256) ((unsigned long long*)A.ctrl)[k] = ((const unsigned long long*)cl)[k];
        }
      }
    }
  }
  ++run;
  if (wg == 0 && tid == 0) stamp(dv, 30, 4);
  if (a.tr && wg == 0 && tid == 0) a.tr[(size_t)a.tr_cap * 4 + 2 * l + 1] = rt_now();
  // the record's late fields again from the broadcast area (nothing but the window and
  // the snapshot is kept live across the solve: registers for the solve's pointers)
  {
    TagChunk ch[kRelChunks];
#pragma unroll
    for (int i = 0; i < kRelChunks; ++i) ch[i] = ld_nt_chunk(A.rec + 2 * i);
    unpack_release(ch, q);
  }
  // ---- 3. push: ticket, serial slice updates, snapshot, token ----
  if (wg == 0 && tid == 0) {
    if (q.delay_us > 0) {  // injected straggler (tests): the solve "took" delay_us longer
      const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();  // 100 MHz
      while ((long long)__builtin_amdgcn_s_memrealtime() - t0 < (long long)q.delay_us * 100)
        __builtin_amdgcn_s_sleep(64);
    }
    const unsigned long long t =
        __hip_atomic_fetch_add(a.ticket, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1ull;
    *(volatile unsigned long long*)(A.rec + 16) = t;
  }
  const int spin = spin_limit(dv);
  x_barrier(A.flags, wg, kLaneWg, ++lw, err, spin);
  const unsigned long long t = ld_h64<2>(A.rec + 16);
  if (wg == 0 && tid == 0) stamp(dv, 30, 5);
  // the logging lane: the host asks this release for a server row (the lowest live
  // worker's deltas, ServerProcessor.java:154-165 -- it moves when that worker fails)
  const bool logl = !a.remote && q.slot_s != 0ull;
  if (!a.remote) {  // the server is this launch: serial slice updates in ticket order
    if (wg < NS) async_apply_slice<FP>(cfg, dv, A, a, wg, t, logl, err, spin, nullptr);
    x_barrier(A.flags, wg, kLaneWg, ++lw, err, spin);
  } else if (A.inbox) {  // the server GPU's inbox: the delta goes out with the token
    if (wg < NS) peer_push_slice<FP>(cfg, dv, A, wg, q.vc, err);
    x_barrier(A.flags, wg, kLaneWg, ++lw, err, spin);
  }
  if (wg == 0 && tid == 0) stamp(dv, 30, 6);
  if (a.tr && wg == 0 && tid == 0) {
    long long* e = a.tr + (size_t)(t % (unsigned long long)a.tr_cap) * 4;
    const long long* pk = a.tr + (size_t)a.tr_cap * 4 + 2 * l;
    e[0] = l;
    e[1] = pk[0];
    e[2] = pk[1];
    e[3] = rt_now();
  }
  if (wg == 0 && tid == 0)
    st_sys_chunk(a.tok, (unsigned)(a.ring * 16), (unsigned)((t % (unsigned long long)a.ring) * 16ull),
                 TagChunk{(unsigned)t, (unsigned)l, (unsigned)(unsigned long long)q.vc,
                          (unsigned)((unsigned long long)q.vc >> 32)});
  // ---- 4. evaluation: the local model (worker row, LogisticRegressionTaskSpark.java:186)
  // paired on the logging lane with the global model right after this update (server
  // row, ServerProcessor.java:154-165) ----
  {
    PairModels pm;
    pm.ah = dv.out_hi;
    pm.al = dv.out_lo;
    pm.ab = dv.b_fin;
    pm.aloss = dv.loss;
    pm.aslot = (char*)q.slot_w;
    pm.aseq = q.seq_w;
    pm.bh = A.shi;
    pm.bl = A.slo;
    pm.bb = A.sb;
    pm.bslot = logl ? (char*)q.slot_s : nullptr;
    pm.bseq = q.seq_s;
    if (wg == 0 && tid == 0) stamp(dv, 30, 7);
    if (dv.dbg && tid == 0 && wg < 32)  // (every workgroup's evaluation start: rows 26-27)
      dv.dbg[(26 + (wg >> 4)) * 16 + (wg & 15)] = (long long)__builtin_amdgcn_s_memrealtime();
    if (a.tnz > 0)  // (the hashed bag-of-words test rows in ELL form: 1.3 instead of 10 MB per pass)
      lane_pair_eval_ell<FP>(lds, K, a.Ti, a.Tv, a.tnz, a.yt, a.T, wg, kLaneWg, pm, A.acc, A.eticket, A.eslab);
    else
      lane_pair_eval<FP>(lds, K, a.Xt, a.yt, a.T, wg, kLaneWg, pm, A.acc, A.eticket);
    if (wg == 0 && tid == 0) stamp(dv, 30, 8);
    if (dv.dbg && tid == 0 && wg < 32)  // (every workgroup's evaluation end: rows 24-25 of the table)
      dv.dbg[(24 + (wg >> 4)) * 16 + (wg & 15)] = (long long)__builtin_amdgcn_s_memrealtime();
  }
  return true;
}

// The launch's {cfg, args} is its first kernel argument, read in place in the kernarg
// segment (constant address space: scalar loads) through fresh_k per iteration.
typedef const __attribute__((address_space(4))) AsyncPack KPack;
__device__ __forceinline__ KPack* fresh_k(KPack* p) {
  asm volatile("" : "+s"(p));
  return p;
}

template <int FP, int KP, int S, bool MT>
__global__ __launch_bounds__(256) void lanes_async_kernel(const AsyncPack pkv,
                                                          const AsyncLaneDev* __restrict__ als) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  KPack* const pk4 = (KPack*)__builtin_amdgcn_kernarg_segment_ptr();  // = &pkv (argument 0)
  const AsyncPack* const pk = (const AsyncPack*)pk4;
  const int b = (int)blockIdx.x, tid = threadIdx.x;
  int l, wg;
  {  // roles as lanes_round_kernel: a lane's workgroups claim its XCD's slots; no riders
    const AsyncArgs& a = pk->a;
    const int L = a.L;
    __shared__ int role;
    if (tid == 0) {
      unsigned* c = a.claim + 32 * a.cpar;
      int r = -1;
      if constexpr (S == 2) {
        const int lx = (int)(__builtin_amdgcn_s_getreg((3 << 11) | 20) & 15u) - a.xcd0;  // HW_REG_XCC_ID
        if (lx >= 0 && lx < L) {
          const unsigned k = __hip_atomic_fetch_add(c + lx, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (k < (unsigned)kLaneWg) r = lx * kLaneWg + (int)k;
        }
      } else if (b < 8 * kLaneWg && (b & 7) - a.xcd0 >= 0 && (b & 7) - a.xcd0 < L) {
        r = ((b & 7) - a.xcd0) * kLaneWg + (b >> 3);
      }
      if (b == 0)
        for (int j = 0; j < 32; ++j)
          __hip_atomic_store(a.claim + 32 * (a.cpar ^ 1) + j, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      (void)__hip_atomic_fetch_add(c + 9, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // (diagnostics)
      role = r;
    }
    __syncthreads();
    const int r = __builtin_amdgcn_readfirstlane(role);  // (uniform: lane / workgroup indices in SGPRs)
    __syncthreads();
    if (r < 0) return;
    l = r / kLaneWg;
    wg = r - l * kLaneWg;
  }
  unsigned run = *als[l].dv.prm_count;           // solves so far (kernel entry: coherent)
  unsigned long long relc = *als[l].relc;        // release records consumed so far
  unsigned long long lw = (unsigned long long)pk->a.launch << 40;  // lane-wide barrier words
  for (;;) {
    const AsyncPack* p = (const AsyncPack*)fresh_k(pk4);
    const AsyncLaneDev* A = fresh(als + l);
    if (!async_iteration<FP, KP, S, MT>(lds, p->cfg, p->a, *A, l, wg, run, relc, lw)) return;
  }
}

__global__ void async_init_kernel(const float* __restrict__ w, float* snap, unsigned* snap_tag,
                                  unsigned long long* turn, unsigned long long* ticket, int P, int NS, int R,
                                  unsigned long long t, long long sstride) {
  const size_t so = (size_t)(t % (unsigned long long)R) * (size_t)sstride;
  if (w) {  // (remote mode: the ticket only)
    for (int i = (int)(blockIdx.x * blockDim.x + threadIdx.x); i < P; i += (int)(gridDim.x * blockDim.x))
      snap[so + i] = w[i];
    if (blockIdx.x == 0)
      for (int s = threadIdx.x; s < NS; s += blockDim.x) {
        snap_tag[(size_t)(t % (unsigned long long)R) * NS + s] = (unsigned)t;
        turn[(size_t)s * 32] = t;
      }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) *ticket = t;
}

template <int FP, int KP, int S, bool MT>
void launch_afks(const AsyncPack& pk, const AsyncLaneDev* al, hipStream_t s) {
  static const bool prepared = ((void)hipFuncSetAttribute((const void*)lanes_async_kernel<FP, KP, S, MT>,
                                                          hipFuncAttributeMaxDynamicSharedMemorySize,
                                                          (int)lanes_lds_bytes(FP)),
                                true);
  (void)prepared;
  lanes_async_kernel<FP, KP, S, MT><<<8 * kLaneWg, 256, lanes_lds_bytes(FP), s>>>(pk, al);
}

template <int FP, int KP>
void launch_afk(const SolverCfg& cfg, const AsyncPack& pk, const AsyncLaneDev* al, int S, hipStream_t s) {
  const bool mt = cfg.cap > 32 * kLaneWg;
  if (S == 2 && mt)
    launch_afks<FP, KP, 2, true>(pk, al, s);
  else if (S == 2)
    launch_afks<FP, KP, 2, false>(pk, al, s);
  else if (mt)
    launch_afks<FP, KP, 1, true>(pk, al, s);
  else
    launch_afks<FP, KP, 1, false>(pk, al, s);
}

template <int FP>
void launch_af(const SolverCfg& cfg, const AsyncPack& pk, const AsyncLaneDev* al, int S, hipStream_t s) {
  const int KP = padded_classes(cfg.K);
  if (KP <= 2)
    launch_afk<FP, 2>(cfg, pk, al, S, s);
  else if (KP <= 4)
    launch_afk<FP, 4>(cfg, pk, al, S, s);
  else
    launch_afk<FP, 8>(cfg, pk, al, S, s);
}

}  // namespace

void launch_async_init(const SolverCfg& cfg, const AsyncArgs& a, unsigned long long t, hipStream_t s) {
  async_init_kernel<<<8, 256, 0, s>>>(a.w, a.snap, a.snap_tag, a.turn, a.ticket, cfg.P, cfg.Fp / 32, a.R, t,
                                      a.sstride);
}

void launch_lanes_async(const SolverCfg& cfg, const AsyncPack& pk, const AsyncLaneDev* al, int S, hipStream_t s) {
  switch (cfg.Fp) {
    case 128: launch_af<128>(cfg, pk, al, S, s); break;
    case 256: launch_af<256>(cfg, pk, al, S, s); break;
    case 512: launch_af<512>(cfg, pk, al, S, s); break;
    case 1024: launch_af<1024>(cfg, pk, al, S, s); break;
    default: break;
  }
}

}  // namespace psx
