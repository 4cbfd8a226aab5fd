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
  if (tid < kCmdChunks) ((TagChunk*)a.rec)[tid] = c;
}

template <int FP>
__device__ __forceinline__ void srv_command(char* lds, const SrvArgs& a, const SrvCmd& cmd, int wg,
                                            unsigned long long n, unsigned long long& lw, unsigned long long* err) {
  constexpr int NS = FP / 32;
  const int tid = threadIdx.x, K = a.K;
  const int c = tid >> 5, f = wg * 32 + (tid & 31);
  const bool coef = c < K, icpt = wg == 0 && tid < K;
  const size_t e = (size_t)c * FP + f, ei = (size_t)K * FP + tid;
  if (wg < NS) {
    // this slice of w (only this workgroup role touches it; sc1: the role may have
    // run on another CU in an earlier launch)
    float nw = coef ? ld_sc1(a.w + e) : 0.f;
    float nb = icpt ? ld_sc1(a.w + ei) : 0.f;
    if (cmd.k >= 0) {  // w += lr * delta_k (ServerProcessor.java:148-151)
      __shared__ int ok_s;
      if (tid == 0) {
        const unsigned* tg = a.inbox_tag + (size_t)cmd.k * NS + wg;
        const long long t_end = rt_now() + a.tag_ticks;
        bool late = false;
        while ((int)(ld_sys_u32(tg) - cmd.dtag) < 0 && !(late = rt_now() > t_end)) __builtin_amdgcn_s_sleep(2);
        ok_s = !late;
        if (!ok_s) xstore(err, 11ull);  // the delta never arrived: apply nothing
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
      }
      __syncthreads();
      if (ok_s) {
        const float* d = a.inbox + (size_t)cmd.k * (size_t)a.in_stride;
        if (coef) {
          nw += a.lr * ld_sys_f32(d + e);
          st_sc1(a.w + e, nw);
        }
        if (icpt) {
          nb += a.lr * ld_sys_f32(d + ei);
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
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        for (unsigned long long m = cmd.relmask; m; m &= m - 1) {
          const int j = __builtin_ctzll(m);
          unsigned* pt = a.ptag + (size_t)j * NS + wg;
          const unsigned t = __hip_atomic_load((g_u32*)pt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
          __hip_atomic_store((g_u32*)pt, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          st_sys_u32(a.rx_tag[j] + wg, t);
        }
      }
    }
  }
  if (cmd.log && cmd.slot_s) {  // the server row: every workgroup on the test tiles
    x_barrier(a.flags, wg, kSrvWg, ++lw, err, a.spin);
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
    lane_pair_eval_at<FP>(lds, K, a.Xt, a.yt, a.T, wg, kSrvWg, pm, a.acc, a.eticket);
  }
  (void)n;
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
        if (k < (unsigned)kSrvWg) r = (int)k;
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
    x_barrier(a.flags, wg, kSrvWg, ++lw, err, 0x7fffffff);
    if (wg == 0 && tid == 0)  // (its ring slot may be reused: the record is in the broadcast area)
      __hip_atomic_store(a.consumed_host, n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
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
  switch (FP) {
    case 128: server_persist_kernel<128><<<8 * kSrvWg, 256, lds, s>>>(a); break;
    case 256: server_persist_kernel<256><<<8 * kSrvWg, 256, lds, s>>>(a); break;
    case 512: server_persist_kernel<512><<<8 * kSrvWg, 256, lds, s>>>(a); break;
    case 1024: server_persist_kernel<1024><<<8 * kSrvWg, 256, lds, s>>>(a); break;
    default: break;
  }
}

}  // namespace psx
