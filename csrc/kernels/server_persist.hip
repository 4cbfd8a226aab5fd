// Persistent server kernel of the peer data plane (see server_persist.h).
#include "lanes_body.h"
#include "server_persist.h"
#include "solve_body.h"
#include "tile.h"

namespace psx {
namespace {
using namespace lanes_detail;

__device__ __forceinline__ TagChunk srv_ld_sys_chunk(const void* base, unsigned bytes, unsigned off) {
  return __builtin_bit_cast(TagChunk,
                            __builtin_amdgcn_raw_buffer_load_b128(rsrc_of(base, bytes), (int)off, 0, kAuxSys));
}

// The leader (workgroup 0, wave 0) waits for command `want` (1-based) in the
// pinned ring and copies it into the broadcast area (this XCD's L2).  A timeout
// becomes a stop command (error 7 on the host word).
__device__ __forceinline__ void srv_wait_cmd(const SrvArgs& a, unsigned long long want) {
  const int tid = threadIdx.x;
  if (tid >= 64) return;
  const TagChunk* slot = a.cmd + (size_t)((want - 1) % (unsigned long long)a.ring) * kCmdChunks;
  TagChunk c = TagChunk{0, 0, 0, 0};
  bool ok = false;
  const long long t_end = rt_now() + a.cmd_ticks;
  for (;;) {
    if (tid < kCmdChunks) c = srv_ld_sys_chunk(slot, (unsigned)(kCmdChunks * 16), (unsigned)tid * 16u);
    const unsigned t0 = __shfl(c.tag, 0, 64);
    ok = __all(tid >= kCmdChunks || c.tag == t0) && t0 == (unsigned)want;
    if (ok || rt_now() > t_end) break;
    __builtin_amdgcn_s_sleep(8);
  }
  if (!ok) {
    c = TagChunk{(unsigned)want, tid == 0 ? 1u : 0u, 0u, 0u};  // stop
    if (tid == 0) __hip_atomic_store(a.err_host, (want << 8) | 7ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  // a batch command: its entries too, every lane one 16-B chunk per pass (all in flight),
  // into the entry broadcast area -- the barrier behind this publishes both
  const int k0 = (int)__shfl(c.b, 0, 64);
  if (ok && k0 == kSrvBatch) {
    const int m = (int)__shfl(c.c, 0, 64);
    const unsigned long long e0 = ((unsigned long long)__shfl(c.c, 1, 64) << 32) | __shfl(c.b, 1, 64);
    const int nch = (m < kSrvMaxBatch ? m : kSrvMaxBatch) * kEntChunks;
    for (int i0 = 0; i0 < nch && ok; i0 += 64) {
      const int i = i0 + tid;
      const bool mine = i < nch;
      const unsigned long long e = e0 + (unsigned long long)(i / kEntChunks);
      const TagChunk* es = a.ent + (size_t)(e % (unsigned long long)a.ent_cap) * kEntChunks + (i % kEntChunks);
      TagChunk v = TagChunk{0, 0, 0, 0};
      for (;;) {
        if (mine) v = srv_ld_sys_chunk(es, 16u, 0u);
        ok = __all(!mine || v.tag == (unsigned)(e + 1ull));
        if (ok || rt_now() > t_end) break;
        __builtin_amdgcn_s_sleep(2);
      }
      if (mine) ((TagChunk*)a.erec)[i] = v;
    }
    if (!ok) {  // (never expected: the host writes the entries before their command)
      c = TagChunk{(unsigned)want, tid == 0 ? 1u : 0u, 0u, 0u};
      if (tid == 0) __hip_atomic_store(a.err_host, (want << 8) | 8ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  if (tid < kCmdChunks) ((TagChunk*)a.rec)[tid] = c;
}

// Slice s of a batch command: the entries' deltas in entry order, each entry's releases
// written right after its update (ServerProcessor.java:143-183: apply, then answer).  The
// deltas' loads go out kBChunk at a time; w is stored once, after the last.
template <int FP>
__device__ __forceinline__ void srv_batch_slice(const SrvArgs& a, const SrvCmd& cmd, int s, unsigned long long* err) {
  constexpr int NS = FP / 32;
  constexpr int kBChunk = 8;
  const int tid = threadIdx.x, K = a.K;
  const int c = tid >> 5, f = s * 32 + (tid & 31);
  const bool coef = c < K, icpt = s == 0 && tid < K;
  const size_t e = (size_t)c * FP + f, ei = (size_t)K * FP + tid;
  const int m = (int)(cmd.dtag < (unsigned)kSrvMaxBatch ? cmd.dtag : (unsigned)kSrvMaxBatch);
  __shared__ SrvEnt ents[kSrvMaxBatch];
  __shared__ int ok_s;
  if (tid < m) {
    TagChunk ch[kEntChunks];
#pragma unroll
    for (int q = 0; q < kEntChunks; ++q)
      ch[q] = __builtin_bit_cast(TagChunk, __builtin_nontemporal_load((const u32x4*)(a.erec + 2 * (tid * kEntChunks + q))));
    unpack_ent(ch, ents[tid]);
  }
  __syncthreads();
  // every entry's tag of this slice, one lane per entry (wave 0), then the acquire
  if (tid < 64) {
    bool late = false;
    if (tid < m) {
      const unsigned* tg = a.inbox_tag + (size_t)ents[tid].k * NS + s;
      const long long t_end = rt_now() + a.tag_ticks;
      while ((int)(ld_sys_u32(tg) - ents[tid].dtag) < 0 && !(late = rt_now() > t_end)) __builtin_amdgcn_s_sleep(2);
    }
    const bool any_late = __any(late);
    if (tid == 0) {
      ok_s = any_late ? 0 : 1;
      if (any_late) xstore(err, 11ull);  // a delta never arrived: apply none of the batch's
      // (no acquire: the deltas are read with system-scope loads below)
    }
  }
  __syncthreads();
  float nw = coef ? ld_sc1(a.w + e) : 0.f;
  float nb = icpt ? ld_sc1(a.w + ei) : 0.f;
  if (ok_s) {
    for (int j0 = 0; j0 < m; j0 += kBChunk) {
      float dl[kBChunk], di[kBChunk];
#pragma unroll
      for (int u = 0; u < kBChunk; ++u) {  // this chunk's loads all in flight
        dl[u] = di[u] = 0.f;
        if (j0 + u < m) {
          const float* d = a.inbox + (size_t)ents[j0 + u].k * (size_t)a.in_stride;
          if (coef) dl[u] = ld_sys_f32(d + e);
          if (icpt) di[u] = ld_sys_f32(d + ei);
        }
      }
#pragma unroll
      for (int u = 0; u < kBChunk; ++u) {
        if (j0 + u >= m) break;
        nw += a.lr * dl[u];
        nb += a.lr * di[u];
        for (unsigned long long rm = ents[j0 + u].relmask; rm; rm &= rm - 1) {  // the weights right after it
          float* dst = a.rx[__builtin_ctzll(rm)];
          if (coef) st_sys_f32(dst + e, nw);
          if (icpt) st_sys_f32(dst + ei, nb);
        }
      }
    }
    if (coef) st_sc1(a.w + e, nw);
    if (icpt) st_sc1(a.w + ei, nb);
  }
  if (cmd.log) {  // the global model after the batch's last (logging) delta
    if (coef) write_frag(a.shi, a.slo, c, f, f < a.F ? nw : 0.f);
    if (icpt) a.sb[tid] = nb;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    // (no release fence: the receive slots were written with sc0 sc1 stores, drained by
    // every wave's vmcnt(0) above -- a system-scope release would write back the XCD's L2)
    for (int j = 0; j < m; ++j)
      for (unsigned long long rm = ents[j].relmask; rm; rm &= rm - 1) {
        const int r = __builtin_ctzll(rm);
        unsigned* pt = a.ptag + (size_t)r * NS + s;
        const unsigned t = __hip_atomic_load((g_u32*)pt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
        __hip_atomic_store((g_u32*)pt, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        st_sys_u32(a.rx_tag[r] + s, t);
      }
  }
  __syncthreads();  // (ents / ok_s: the next slice of this workgroup)
}

// A BSP round (kSrvBspSum) on workgroup wg's slices wg, wg + nwg, ... -- up to kBspSl of them
// in ONE pass: every (slice, rank) tag polled by a lane of its own, all the ranks' slice loads
// in flight, the receive slots' stores drained together, then every (slice, rank) tag by a
// thread of its own.  A launch with fewer workgroups than slices (the colocated rank 0 and
// the shared-GPU rehearsals keep half of the XCD's CUs free) then pays each xGMI / memory
// round trip once per round, not once per slice.  The sums are the per-slice ones of
// srv_slice: ranks in rank order, w += lr * sum.
template <int FP>
__device__ __forceinline__ void srv_bsp_slices(const SrvArgs& a, const SrvCmd& cmd, int wg, unsigned long long* err) {
  constexpr int NS = FP / 32;
  constexpr int kBspSl = 4;
  const int tid = threadIdx.x, K = a.K, N = a.N;
  __shared__ int ok_s;
  for (int s0 = wg; s0 < NS; s0 += kBspSl * a.nwg) {
    int nsl = 0;
    for (int j = 0; j < kBspSl; ++j) nsl += s0 + j * a.nwg < NS ? 1 : 0;
    // the (slice, rank) tags: wave 0, one lane each (a wall-clock budget per pass)
    if (tid < 64) {
      bool late = false;
      const long long t_end = rt_now() + a.tag_ticks;
      for (int i = tid; i < nsl * N; i += 64) {
        const int j = i / N, r = i - j * N;
        const unsigned* tg = a.inbox_tag + (size_t)r * NS + (s0 + j * a.nwg);
        while ((int)(ld_sys_u32(tg) - cmd.dtag) < 0 && !(late = rt_now() > t_end)) __builtin_amdgcn_s_sleep(2);
        if (late) break;
      }
      const bool any_late = __any(late);
      if (tid == 0) {
        ok_s = any_late ? 0 : 1;
        if (any_late) xstore(err, 11ull);  // a rank's sum never arrived: apply nothing
      }
    }
    __syncthreads();
    const int c = tid >> 5;
    const bool coef = c < K;
    float nw[kBspSl], nb = 0.f;
#pragma unroll
    for (int j = 0; j < kBspSl; ++j) {
      const int sj = s0 + j * a.nwg;
      nw[j] = (j < nsl && coef) ? ld_sc1(a.w + (size_t)c * FP + sj * 32 + (tid & 31)) : 0.f;
    }
    const bool icpt = s0 == 0 && tid < K;  // (slice 0 is always the pass's first)
    if (icpt) nb = ld_sc1(a.w + (size_t)K * FP + tid);
    if (ok_s) {
      float sum[kBspSl], sumi = 0.f;
#pragma unroll
      for (int j = 0; j < kBspSl; ++j) sum[j] = 0.f;
      for (int r = 0; r < N; ++r) {  // ranks in rank order (the loads of a rank's slices in flight together)
        const float* d = a.inbox + (size_t)r * (size_t)a.in_stride;
        float v[kBspSl];
#pragma unroll
        for (int j = 0; j < kBspSl; ++j)
          v[j] = (j < nsl && coef) ? ld_sys_f32(d + (size_t)c * FP + (s0 + j * a.nwg) * 32 + (tid & 31)) : 0.f;
        const float vi = icpt ? ld_sys_f32(d + (size_t)K * FP + tid) : 0.f;
#pragma unroll
        for (int j = 0; j < kBspSl; ++j) sum[j] += v[j];
        sumi += vi;
      }
#pragma unroll
      for (int j = 0; j < kBspSl; ++j)
        if (j < nsl && coef) {
          nw[j] += a.lr * sum[j];
          st_sc1(a.w + (size_t)c * FP + (s0 + j * a.nwg) * 32 + (tid & 31), nw[j]);
        }
      if (icpt) {
        nb += a.lr * sumi;
        st_sc1(a.w + (size_t)K * FP + tid, nb);
      }
    }
#pragma unroll
    for (int j = 0; j < kBspSl; ++j) {
      if (j >= nsl) break;
      const int f = (s0 + j * a.nwg) * 32 + (tid & 31);
      if (cmd.log && coef) write_frag(a.shi, a.slo, c, f, f < a.F ? nw[j] : 0.f);
      for (unsigned long long m = cmd.relmask; m; m &= m - 1) {  // the new slice into every rank's receive slot
        float* dst = a.rx[__builtin_ctzll(m)];
        if (coef) st_sys_f32(dst + (size_t)c * FP + f, nw[j]);
      }
    }
    if (icpt) {
      if (cmd.log) a.sb[tid] = nb;
      for (unsigned long long m = cmd.relmask; m; m &= m - 1) st_sys_f32(a.rx[__builtin_ctzll(m)] + (size_t)K * FP + tid, nb);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    // the (slice, rank) tags, a thread each (no release fence: sc0 sc1 stores, drained above)
    for (int i = tid; i < nsl * 64; i += 256) {
      const int j = i >> 6, r = i & 63;
      if (!((cmd.relmask >> r) & 1ull)) continue;
      const int sj = s0 + j * a.nwg;
      __hip_atomic_store((g_u32*)(a.ptag + (size_t)r * NS + sj), cmd.dtag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      st_sys_u32(a.rx_tag[r] + sj, cmd.dtag);
    }
    __syncthreads();  // (ok_s: the next pass)
  }
}

// Slice s of command `cmd` (one workgroup; every thread calls it).
template <int FP>
__device__ __forceinline__ void srv_slice(const SrvArgs& a, const SrvCmd& cmd, int s, unsigned long long* err) {
  constexpr int NS = FP / 32;
  const int tid = threadIdx.x, K = a.K;
  const int c = tid >> 5, f = s * 32 + (tid & 31);
  const bool coef = c < K, icpt = s == 0 && tid < K;
  const size_t e = (size_t)c * FP + f, ei = (size_t)K * FP + tid;
  // this slice of w (only this workgroup role touches it; sc1: the role may have run on
  // another CU in an earlier launch)
  float nw = coef ? ld_sc1(a.w + e) : 0.f;
  float nb = icpt ? ld_sc1(a.w + ei) : 0.f;
  __shared__ int ok_s;
  if (cmd.k == kSrvBspSum || cmd.k >= 0) {
    // the delta(s) in the inbox: worker k's (ServerProcessor.java:148-151), or under a BSP
    // round every worker rank's lane sum (waited for in rank order)
    if (tid == 0) {
      const long long t_end = rt_now() + a.tag_ticks;
      bool late = false;
      const int j0 = cmd.k == kSrvBspSum ? 0 : cmd.k, j1 = cmd.k == kSrvBspSum ? a.N : cmd.k + 1;
      for (int j = j0; j < j1 && !late; ++j) {
        const unsigned* tg = a.inbox_tag + (size_t)j * NS + s;
        while ((int)(ld_sys_u32(tg) - cmd.dtag) < 0 && !(late = rt_now() > t_end)) __builtin_amdgcn_s_sleep(2);
      }
      ok_s = !late;
      if (late) xstore(err, 11ull);  // a delta never arrived: apply nothing
      // (no acquire: the inbox is read with system-scope loads, and its writers drained
      // their stores before the tag)
    }
    __syncthreads();
    if (ok_s) {
      const int j0 = cmd.k == kSrvBspSum ? 0 : cmd.k, j1 = cmd.k == kSrvBspSum ? a.N : cmd.k + 1;
      float sum = 0.f, sumi = 0.f;  // (a BSP round: the ranks' sums added in rank order)
      for (int j = j0; j < j1; ++j) {
        const float* d = a.inbox + (size_t)j * (size_t)a.in_stride;
        if (coef) sum += ld_sys_f32(d + e);
        if (icpt) sumi += ld_sys_f32(d + ei);
      }
      if (coef) {
        nw += a.lr * sum;
        st_sc1(a.w + e, nw);
      }
      if (icpt) {
        nb += a.lr * sumi;
        st_sc1(a.w + ei, nb);
      }
    }
  }
  if (cmd.log) {  // the global model's fragments for the server row
    if (coef) write_frag(a.shi, a.slo, c, f, f < a.F ? nw : 0.f);
    if (icpt) a.sb[tid] = nb;
  }
  // the weights right after this update to every released worker's receive slot
  // (ServerProcessor.java:172-182), then ONE release and the slots' slice tags
  if (cmd.relmask) {
    for (unsigned long long m = cmd.relmask; m; m &= m - 1) {
      const int j = __builtin_ctzll(m);
      float* dst = a.rx[j];
      if (coef) st_sys_f32(dst + e, nw);
      if (icpt) st_sys_f32(dst + ei, nb);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      // (no release fence: the slices are sc0 sc1 stores, drained above -- a system-scope
      // release would write back this XCD's L2 on the path to the released workers)
      for (unsigned long long m = cmd.relmask; m; m &= m - 1) {
        const int j = __builtin_ctzll(m);
        unsigned* pt = a.ptag + (size_t)j * NS + s;
        // (a BSP round's tag is the round's own: the ranks wait for tag >= round)
        const unsigned t = cmd.k == kSrvBspSum
                               ? cmd.dtag
                               : __hip_atomic_load((g_u32*)pt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
        __hip_atomic_store((g_u32*)pt, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        st_sys_u32(a.rx_tag[j] + s, t);
      }
    }
  }
}

template <int FP>
__device__ __forceinline__ void srv_command(char* lds, const SrvArgs& a, const SrvCmd& cmd, int wg,
                                            unsigned long long n, unsigned long long& lw, unsigned long long* err) {
  constexpr int NS = FP / 32;
  const int K = a.K;
  // workgroup wg owns slices wg, wg + nwg, ... (nwg < NS: a server launch that leaves CUs of
  // its XCD to other processes on a shared GPU)
  if (cmd.k == kSrvBspSum) {
    srv_bsp_slices<FP>(a, cmd, wg, err);
  } else {
    for (int s = wg; s < NS; s += a.nwg) {
      if (cmd.k == kSrvBatch) {
        srv_batch_slice<FP>(a, cmd, s, err);
      } else {
        srv_slice<FP>(a, cmd, s, err);
        if (a.nwg < NS) __syncthreads();  // (ok_s / the tag lanes of the next slice)
      }
    }
  }
  long long* trn = (a.tr && wg == 0 && threadIdx.x == 0) ? a.tr + (size_t)(n % (unsigned long long)a.tr_cap) * 4 : nullptr;
  if (trn) trn[1] = rt_now();
  if (cmd.log && cmd.slot_s) {  // the server row: every workgroup on the test tiles
    x_barrier(a.flags, wg, a.nwg, ++lw, err, a.spin);
    PairModels pm;
    pm.ah = a.shi;
    pm.al = a.slo;
    pm.ab = a.sb;
    pm.aloss = nullptr;
    pm.aslot = nullptr;
    pm.aseq = 0;
    pm.bh = a.shi;
    pm.bl = a.slo;
    pm.bb = a.sb;
    pm.bslot = (char*)cmd.slot_s;
    pm.bseq = cmd.seq_s;
    lane_pair_eval_at<FP>(lds, K, a.Xt, a.yt, a.T, wg, a.nwg, pm, a.acc, a.eticket);
  }
  if (trn) {
    trn[2] = rt_now();
    trn[3] = (long long)n;
  }
}

template <int FP>
__global__ __launch_bounds__(256) void server_persist_kernel(const SrvArgs pa) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int b = (int)blockIdx.x, tid = threadIdx.x;
  int wg;
  {
    __shared__ int role;
    if (tid == 0) {
      unsigned* cl = pa.claim + 32 * pa.cpar;
      int r = -1;
      const int x = (int)(__builtin_amdgcn_s_getreg((3 << 11) | 20) & 15u);  // HW_REG_XCC_ID
      if (x == pa.sxcd) {
        const unsigned k = __hip_atomic_fetch_add(cl, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (k < (unsigned)pa.nwg) r = (int)k;
      }
      if (b == 0)
        for (int j = 0; j < 32; ++j)
          __hip_atomic_store(pa.claim + 32 * (pa.cpar ^ 1) + j, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      role = r;
    }
    __syncthreads();
    wg = __builtin_amdgcn_readfirstlane(role);
    __syncthreads();
    if (wg < 0) return;
  }
  const SrvArgs& a = pa;
  unsigned long long* err = a.flags + (size_t)kSrvWg * 32;  // (the line behind the barrier lines)
  unsigned long long lw = (unsigned long long)a.launch << 40;
  // a timed-out wait (the sticky word `err`) -> the pinned host word as (command << 8) |
  // code, then cleared; before the barrier every workgroup of the next command passes
  auto report = [&](unsigned long long cmdno) {
    const unsigned long long e = xload(err);
    if (e) {
      __hip_atomic_store(a.err_host, (cmdno << 8) | (e & 0xffull), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      xstore(err, 0ull);
    }
  };
  for (unsigned long long n = a.cmd0 + 1;; ++n) {
    if (wg == 0) srv_wait_cmd(a, n);
    if (wg == 0 && tid == 0) report(n - 1);
    // (the others wait for the leader without a budget of their own: the leader's command
    // wait is bounded and ends in a stop command -- with the same poll budget the others'
    // faster polls would give up first during a long idle period)
    x_barrier(a.flags, wg, a.nwg, ++lw, err, 0x7fffffff);
    if (wg == 0 && tid == 0) {  // (its ring slot may be reused: the record is in the broadcast area)
      __hip_atomic_store(a.consumed_host, n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      if (a.tr) a.tr[(size_t)(n % (unsigned long long)a.tr_cap) * 4] = rt_now();
    }
    SrvCmd cmd;
    {
      TagChunk ch[kCmdChunks];
#pragma unroll
      for (int i = 0; i < kCmdChunks; ++i)
        ch[i] = __builtin_bit_cast(TagChunk, __builtin_nontemporal_load((const u32x4*)(a.rec + 2 * i)));
      unpack_cmd(ch, cmd);
    }
    if (cmd.stop) {
      if (wg == 0 && tid == 0) report(n);
      break;
    }
    srv_command<FP>(lds, a, cmd, wg, n, lw, err);
  }
}

}  // namespace

size_t server_persist_lds_bytes() { return (size_t)kPairEvalLds; }

void launch_server_persist(const SrvArgs& a, int FP, hipStream_t s) {
  const size_t lds = server_persist_lds_bytes();
  if (a.nwg < 1 || a.nwg > kSrvWg) return;
  switch (FP) {
    case 128: server_persist_kernel<128><<<8 * a.nwg, 256, lds, s>>>(a); break;
    case 256: server_persist_kernel<256><<<8 * a.nwg, 256, lds, s>>>(a); break;
    case 512: server_persist_kernel<512><<<8 * a.nwg, 256, lds, s>>>(a); break;
    case 1024: server_persist_kernel<1024><<<8 * a.nwg, 256, lds, s>>>(a); break;
    default: break;
  }
}

}  // namespace psx
