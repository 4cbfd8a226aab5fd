// Device body of one evaluation pass (K8/K9: test-set argmax + confusion
// counts), shared by the standalone evaluation launch (lr_kernels.hip:
// test_eval_kernel) and the evaluation workgroups that ride in the solver's
// bwd_update launches (solve_kernels.hip).  See EvalRide in lr_kernels.h.
//
// Reference math: LogisticRegressionTaskSpark.java:236-251 (predict the test
// set, MulticlassMetrics), Metrics.java:15-24 (weighted F1 / accuracy from the
// confusion counts -- computed on the host by MetricsSink).
#pragma once
#include "lr_kernels.h"
#include "tile.h"

namespace psx {

// LDS bytes the body needs (the X tile image + logits + two 16x16 count tables).
// Equal to eval_lds_bytes(FP).
//
// Workgroup-uniform arguments: tiles [tile0, tend) step tstep of the test set.
// Every calling workgroup arrives at the ticket exactly once (with zero tiles
// too), so r.nticket must count all of them.
template <int FP>
__device__ __forceinline__ void eval_body(char* lds, const EvalRide& r, int tile0, int tstep, int tend) {
  char* red_base = lds + 32 * FP * 2;
  int* cl = (int*)(red_base + 8192);  // [16][16]
  int* last = cl + 256;
  int* cl2 = last + 4;                // [16][16] (paired mode)
  const int tid = threadIdx.x, K = r.K, T = r.T;
  const bool pair = r.slot2 != nullptr;
  const int coff1 = r.coff1, coff2 = r.coff2;
  cl[tid] = 0;
  if (pair) cl2[tid] = 0;
  // per-lane B-operand source: the second model's columns from its own buffer
  const bool split = r.shi != nullptr;
  const int lcls = tid & 15;
  const uint16_t* fh = (split && lcls >= coff2) ? r.shi : r.whi;
  const uint16_t* fl = (split && lcls >= coff2) ? r.slo : r.wlo;
  const float* b = r.wb;
  const float* b2 = split ? r.sb : r.wb;
  // The weight fragments are usually fresh (written by the solve / update just
  // before, so not in this XCD's L2): fetch them into registers BEFORE staging
  // the first tile so the two memory latencies overlap; only the columns of the
  // evaluated models are fetched.
  constexpr bool kPre = FP <= 1024;
  WFrag<kPre ? FP : 128> wf;
  if constexpr (kPre) {
    if (tile0 < tend) {
      const bool live = (lcls >= coff1 && lcls < coff1 + K) || (pair && lcls >= coff2 && lcls < coff2 + K);
      load_wfrag<FP>(wf, fh, fl, live ? 16 : 0);
    }
  }
  for (int tile = tile0; tile < tend; tile += tstep) {
    const int nrows = min(32, T - tile * 32);
    // the labels travel with the tile's loads (one memory round trip, not two)
    const int ylab = tid < nrows ? r.yt[(size_t)tile * 32 + tid] : 0;
    stage_tile<FP>(lds, r.Xt, (int64_t)tile * 32, nrows, 0, false);
    __syncthreads();
    f32x4 a0, a1;
    if constexpr (kPre)
      forward_tile_pre<FP>(lds, wf, a0, a1);
    else
      forward_tile<FP>(lds, fh, fl, a0, a1);
    store_partial_logits(red_base, a0, a1);
    __syncthreads();
    if (tid < nrows) {
      int best = 0;
      float bz = -INFINITY;
      for (int c = 0; c < K; ++c) {
        const float z = load_logit(red_base, tid, coff1 + c) + b[coff1 + c];
        if (z > bz) {
          bz = z;
          best = c;
        }
      }
      const int yl = ylab < 0 ? 0 : (ylab > 15 ? 15 : ylab);
      atomicAdd(&cl[yl * 16 + best], 1);
      if (pair) {
        int best2 = 0;
        float bz2 = -INFINITY;
        for (int c = 0; c < K; ++c) {
          const float z = load_logit(red_base, tid, coff2 + c) + b2[coff2 + c];
          if (z > bz2) {
            bz2 = z;
            best2 = c;
          }
        }
        atomicAdd(&cl2[yl * 16 + best2], 1);
      }
    }
    __syncthreads();
  }
  __syncthreads();
  int* acc = r.acc;
  const int v = cl[tid];
  // the private accumulator (slot mode) spreads its cells one per 128-B line, so
  // the workgroups' atomics are not serialised on a few cache lines (kAccStride)
  const int ast = r.slot ? kAccStride : 1;
  if (v) atomicAdd(acc + tid * ast, v);
  if (pair) {
    const int v2 = cl2[tid];
    if (v2) atomicAdd(acc + (256 + tid) * ast, v2);
  }
  if (r.slot == nullptr) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0)
    *last = __hip_atomic_fetch_add(r.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == r.nticket - 1;
  __syncthreads();
  if (!*last) return;
  // Publication into the pinned (fine-grained, uncached) host slot: the counts
  // go out as system-scope relaxed stores, every wave drains them (vmcnt), and
  // only then is the sequence number stored.  No release fence: it would write
  // back this XCD's whole L2 (the solver's dirty lines included), and nothing
  // cached is being published.
  const int tot = __hip_atomic_exchange(acc + tid * ast, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store((int*)r.slot + tid, tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (tid == 0)
    __hip_atomic_store((float*)(r.slot + 1024), r.loss ? *r.loss : 0.f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (pair) {
    const int tot2 = __hip_atomic_exchange(acc + (256 + tid) * ast, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store((int*)r.slot2 + tid, tot2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (tid == 0) __hip_atomic_store((float*)(r.slot2 + 1024), 0.f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    __hip_atomic_store(r.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store((unsigned long long*)(r.slot + 1032), r.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (pair)
      __hip_atomic_store((unsigned long long*)(r.slot2 + 1032), r.seq2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

}  // namespace psx
