// Device bodies shared by the multi-lane round kernels (gfx950):
// lanes_kernels.hip (BSP: one launch per round) and lanes_async.hip (SSP / ASP:
// one persistent launch that serves many releases).  Phase I of a lane's solve
// (staging + ingest + window statistics, x0 / first trial point) and the
// test-set evaluation helpers.
#pragma once
#include <hip/hip_runtime.h>

#include "lanes_kernels.h"
#include "solve_body.h"

namespace psx {
namespace lanes_detail {

// Element i of a kernel-argument array with a wave-uniform runtime index.  Each
// candidate is read with a constant index and passed through readfirstlane word by
// word: a plain select chain is folded by the compiler into ONE load from a selected
// address, which needs the argument struct in memory -- every lane of every
// workgroup then copies the kernel arguments into scratch at entry (measured: 1208
// B per lane, 79 MB of scratch writes per round launch).  The index must be
// uniform across the wave (it is read from the first lane).
template <typename T, int N>
__device__ __forceinline__ T pick(const T (&arr)[N], int i) {
  static_assert(sizeof(T) % 4 == 0, "pick: word-sized structs");
  constexpr int W = sizeof(T) / 4;
  i = __builtin_amdgcn_readfirstlane(i);
  struct Words {
    unsigned w[W];
  } v;
#pragma unroll
  for (int k = 0; k < W; ++k) v.w[k] = 0u;
#pragma unroll
  for (int j = 0; j < N; ++j)
    if (i == j) {
      const unsigned* src = reinterpret_cast<const unsigned*>(&arr[j]);
#pragma unroll
      for (int k = 0; k < W; ++k) v.w[k] = __builtin_amdgcn_readfirstlane(src[k]);
    }
  return __builtin_bit_cast(T, v);
}

// system-coherent 16-B stores into pinned host memory (sc0 | sc1)
constexpr int kAuxSys = 17;
__device__ __forceinline__ void st_sys_chunk(void* base, unsigned bytes, unsigned off, TagChunk v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rsrc_of(base, bytes), (int)off, 0, kAuxSys);
}

// Peer data plane (csrc/comm/peer_bus.h): words another GPU writes over xGMI into
// fine-grained memory, or this GPU writes into another's.  System-scope relaxed
// atomics = global loads / stores with sc0 sc1 (no L1 / L2 reuse); the hand-off
// is payload stores -> s_waitcnt vmcnt(0) -> barrier -> one lane: release fence
// (system) + tag store; the reader polls the tag, acquires (system), then loads.
typedef __attribute__((address_space(1))) unsigned g_u32;
// Wall-clock budgets of the cross-device waits (another process answers them, so a
// poll count would make the budget depend on the poll's latency): s_memrealtime
// is the constant 100 MHz clock.
constexpr long long kRtTicksPerS = 100000000ll;
__device__ __forceinline__ long long rt_now() { return (long long)__builtin_amdgcn_s_memrealtime(); }
__device__ __forceinline__ unsigned ld_sys_u32(const unsigned* p) {
  asm volatile("" ::: "memory");  // a spin re-reads
  return __hip_atomic_load((g_u32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys_u32(unsigned* p, unsigned v) {
  __hip_atomic_store((g_u32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ float ld_sys_f32(const float* p) {
  return __hip_atomic_load((g_f32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys_f32(float* p, float v) {
  __hip_atomic_store((g_f32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// One lane publishes `tag` for the stores of its whole workgroup (call from every
// thread: the wait / barrier are the workgroup's).
__device__ __forceinline__ void publish_sys_tag(unsigned* tagp, unsigned tag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    st_sys_u32(tagp, tag);
  }
}

static_assert(kEvalAccInts == (size_t)kAccCopies * kMaxEvalModels * 256 * kAccStride, "EvalMulti::acc size");

// Accumulator cell of model m in copy `copy` (EvalMulti::acc)
__device__ __forceinline__ int* acc_cell(int* acc, int copy, int m, int cell) {
  return acc + ((size_t)(copy * kMaxEvalModels + m) * 256 + cell) * kAccStride;
}
__device__ __forceinline__ int xcd_copy() {
  return kAccCopies == 1 ? 0 : (int)((__builtin_amdgcn_s_getreg((3 << 11) | 20) & 7u) % kAccCopies);
}

// ---------------------------------------------------------------------------
// Riders: evaluation of up to kMaxEvalModels models (the previous round's
// local models and global model) over the test tiles.  Work items = (model
// pair, test tile), pair-major, dealt to the riders in contiguous chunks so that
// a rider keeps one pair's fragments in registers across its tiles.  Every
// rider arrives on the ticket once; the last one publishes every model's
// counts (and its loss) into its pinned slot, then the sequence number.
template <int FP>
// (the per-lane choice between the two models selects field values, not struct
// addresses: a pointer select would keep both structs in scratch memory)
__device__ __forceinline__ void load_pair_frags(WFrag<FP>& wf, const EvalModel& ma, const EvalModel& mb, bool has_b,
                                                int K) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int col = lane & 15, c = col & 7;
  const bool a = col < 8;
  const uint16_t* hi = a ? ma.hi : mb.hi;
  const uint16_t* lo = a ? ma.lo : mb.lo;
  const int coff = a ? ma.coff : mb.coff;
  const bool live = (a || has_b) && c < K;
#pragma unroll
  for (int kk = 0; kk < WFrag<FP>::KS; ++kk) {
    const int cg = (w * WFrag<FP>::KS + kk) * 4 + (lane >> 4);
    const size_t fo = ((size_t)cg * 16 + (live ? coff + c : 0)) * 8;
    wf.h[kk] = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
    wf.l[kk] = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
    if (live) {
      wf.h[kk] = *(const u16x8*)(hi + fo);
      wf.l[kk] = *(const u16x8*)(lo + fo);
    }
  }
}

// The last arriving workgroup publishes every model's counts into its pinned slot
// as tagged 16-B chunks (sink kind | kSinkTagged, eval_tag(seq)): all M
// accumulator exchanges are issued before the first store (one L2 round trip), the
// counts go through LDS (cells: [M][K*K] ints) into chunk form, and each chunk is
// ONE system-scope store carrying its own tag -- no store-completion wait before a
// sequence number, so the publication costs the workgroup no PCIe round trip.
__device__ __forceinline__ void publish_counts(const EvalMulti& ev, int M, int tid, int* cells) {
  const int K = ev.K, KK = K * K;
  // the counts of the kAccCopies accumulator copies: thread = (model, cell), its
  // copies' sc1 loads (past this XCD's L2: the adds were performed in memory) all in
  // flight, summed in registers; then the copies zeroed
  float lv = 0.f;  // (constant model indices: a per-thread index would copy ev.m into scratch)
#pragma unroll
  for (int m = 0; m < kMaxEvalModels; ++m)
    if (m < M && tid == m && ev.m[m].loss) lv = *ev.m[m].loss;
  if (tid < M) cells[kMaxEvalModels * 64 + tid] = __float_as_int(lv);
  const auto ra = rsrc_of(ev.acc, (unsigned)(kEvalAccInts * 4));
  constexpr unsigned kCopyBytes = (unsigned)kMaxEvalModels * 256 * kAccStride * 4;
  constexpr int kPer = (kMaxEvalModels * 64 + 255) / 256;  // (model, cell) items per thread (K <= 8)
  unsigned o[kPer];
  int v[kPer][kAccCopies];
#pragma unroll
  for (int j = 0; j < kPer; ++j) {  // every load of the thread in flight before any use
    const int q = tid + 256 * j;
    const int m = q / KK, ci = q - m * KK, t16 = ci / K, p16 = ci - t16 * K;
    o[j] = (unsigned)((m * 256 + t16 * 16 + p16) * kAccStride * 4);
#pragma unroll
    for (int c = 0; c < kAccCopies; ++c)
      v[j][c] = q < M * KK ? (int)__builtin_amdgcn_raw_buffer_load_b32(ra, (int)(o[j] + c * kCopyBytes), 0, kAuxSc1) : 0;
  }
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    const int q = tid + 256 * j;
    if (q >= M * KK) continue;
    int t = 0;
#pragma unroll
    for (int c = 0; c < kAccCopies; ++c) {
      t += v[j][c];
      if (v[j][c]) __builtin_amdgcn_raw_buffer_store_b32(0u, ra, (int)(o[j] + c * kCopyBytes), 0, kAuxSc1);
    }
    cells[q] = t;  // (the caller's counts were flushed before the ticket)
  }
  __syncthreads();
  if (tid == 0) __hip_atomic_store(ev.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // wave w publishes models w, w + 4, ... (nch <= 23 chunks: one per lane); the model
  // index is wave-uniform, so pick() stays a scalar select of kernel arguments
  const int nch = 1 + (KK + 2) / 3, i = tid & 63;
  for (int m = __builtin_amdgcn_readfirstlane(tid >> 6); m < M; m += 4) {
    const EvalModel E = pick(ev.m, m);
    const unsigned tag = eval_tag(E.seq);
    TagChunk ch;
    if (i == 0) {
      ch = TagChunk{tag, (unsigned)cells[kMaxEvalModels * 64 + m], (unsigned)K, 0u};
    } else {
      const int c0 = 3 * (i - 1);
      auto cv = [&](int c) { return c < KK ? (unsigned)cells[m * KK + c] : 0u; };
      ch = TagChunk{tag, cv(c0), cv(c0 + 1), cv(c0 + 2)};
    }
    if (i < nch) st_sys_chunk(E.slot, 1088u, (unsigned)i * 16u, ch);
  }
}

// A 32-row test tile held in registers (stage_tile's loads, split from its LDS
// stores so that the next tile's loads fly while the current one is evaluated).
template <int FP>
struct TileRegs {
  static constexpr int CPR = FP / 8, PER_T = 32 * CPR / 256;
  u16x8 v[PER_T];
  int y;
  __device__ __forceinline__ void load(const uint16_t* __restrict__ X, const int32_t* __restrict__ yt, int tile,
                                       int T) {
    const int64_t row0 = (int64_t)tile * 32;
    const int nrows = T - tile * 32 < 32 ? T - tile * 32 : 32;
#pragma unroll
    for (int j = 0; j < PER_T; ++j) {
      const int q = threadIdx.x + 256 * j;
      const int row = q / CPR, cg = q - row * CPR;
      v[j] = row < nrows ? *(const u16x8*)(X + (row0 + row) * FP + cg * 8) : u16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
    y = (int)threadIdx.x < nrows ? yt[row0 + threadIdx.x] : 0;
  }
  __device__ __forceinline__ void store(char* lds) const {  // stage_tile's LDS layout
#pragma unroll
    for (int j = 0; j < PER_T; ++j) {
      const int q = threadIdx.x + 256 * j;
      const int row = q / CPR, cg = q - row * CPR;
      *(u16x8*)(lds + (cg >> 4) * 8192 + lds_off(row, cg & 15)) = v[j];
    }
  }
};

template <int FP>
__device__ __forceinline__ void eval_multi_body(char* lds, const EvalMulti& ev, int rid, int nride) {
  if (ev.nmodels <= 0 || rid >= nride) return;
  rid = __builtin_amdgcn_readfirstlane(rid);  // (workgroup-uniform: keeps the item indices scalar)
  long long* dbg = ev.dbg;
  auto rstamp = [&](int k) {
    if (dbg && threadIdx.x == 0) dbg[k] = (long long)__builtin_amdgcn_s_memrealtime();
  };
  if (dbg && threadIdx.x == 0) {
    const long long t = (long long)__builtin_amdgcn_s_memrealtime();
    atomicMin((unsigned long long*)(dbg + 12), (unsigned long long)t);
    atomicMax((unsigned long long*)(dbg + 13), (unsigned long long)t);
  }
  if (rid == 0) rstamp(0);
  char* red_base = lds + 32 * FP * 2;
  int* cl = (int*)(red_base + 8192);  // [kMaxEvalModels][256]
  int* lastp = cl + kMaxEvalModels * 256;
  float* bl = (float*)(lastp + 4);  // [16]: the current pair's intercepts (model A: 0..7, B: 8..15)
  const int tid = threadIdx.x, K = ev.K, T = ev.T, M = ev.nmodels;
  const int nT = (T + 31) / 32, npairs = (M + 1) / 2;
  for (int m = 0; m < M; ++m) cl[m * 256 + tid] = 0;
  const int items = npairs * nT, chunk = (items + nride - 1) / nride;
  int curp = -1;
  WFrag<FP> wf;
  TileRegs<FP> tr;  // the next item's tile, in flight during the current item
  // items [j0, j1) of the tile range [t0, t0 + ntx): item j = (pair j / ntx, tile t0 + j % ntx)
  auto run_items = [&](int t0, int ntx, int j0, int j1, bool first) {
    if (j0 < j1) tr.load(ev.Xt, ev.yt, t0 + j0 % ntx, T);
    __syncthreads();
    for (int it = j0; it < j1; ++it) {
      const int p = it / ntx, tile = t0 + (it - p * ntx);
      const int ma = 2 * p, mb = 2 * p + 1 < M ? 2 * p + 1 : -1;
      if (p != curp) {  // (workgroup-uniform)
        const EvalModel A = pick(ev.m, ma), Bm = pick(ev.m, mb >= 0 ? mb : 0);
        load_pair_frags<FP>(wf, A, Bm, mb >= 0, K);
        if (tid < 16) {  // the intercepts into LDS once per pair, not a global load per class and row
          const int h = tid >> 3, c = tid & 7;
          const float* bp = h == 0 ? A.b + A.coff : Bm.b + Bm.coff;
          bl[tid] = (c < K && (h == 0 || mb >= 0)) ? bp[c] : 0.f;
        }
        curp = p;
      }
      const int nrows = T - tile * 32 < 32 ? T - tile * 32 : 32;
      tr.store(lds);
      const int ylab = tr.y;
      if (it + 1 < j1) tr.load(ev.Xt, ev.yt, t0 + (it + 1) % ntx, T);
      __syncthreads();
      if (first && rid == 0 && it == j0) rstamp(1);
      f32x4 a0, a1;
      forward_tile_pre<FP>(lds, wf, a0, a1);
      store_partial_logits(red_base, a0, a1);
      __syncthreads();
      {  // thread (row, model): rows 0..31 x models {A, B} -- both models' argmax at once
        const int row = tid & 31, h = (tid >> 5) & 1;
        const int yrow = __shfl(ylab, row, 64);  // the row's label (held by thread `row` of wave 0)
        if (tid < 64 && row < nrows && (h == 0 || mb >= 0)) {
          const int yl = yrow < 0 ? 0 : (yrow > 15 ? 15 : yrow);
          int best = 0;
          float bz = -INFINITY;
          for (int c = 0; c < K; ++c) {
            const float z = load_logit(red_base, row, 8 * h + c) + bl[8 * h + c];
            if (z > bz) {
              bz = z;
              best = c;
            }
          }
          atomicAdd(&cl[(h == 0 ? ma : mb) * 256 + yl * 16 + best], 1);
        }
      }
      __syncthreads();
      if (first && rid == 0 && it - j0 < 4) rstamp(2 + (it - j0));
    }
  };
  if (!ev.xq) {  // rider rid: items [rid * chunk, (rid + 1) * chunk), pair-major over the whole test set
    const int i0 = rid * chunk, i1 = i0 + chunk < items ? i0 + chunk : items;
    run_items(0, nT, i0, i1, true);
  } else {
    // XCD-local slices: the test set split into 8 tile ranges, range x evaluated by riders
    // running on XCD x (its tiles stay in that XCD's L2 from round to round), in chunks
    // popped from a per-XCD counter; a rider whose range is done pops the next XCD's --
    // every chunk exactly once whatever the placement
    const int xcc = (int)(__builtin_amdgcn_s_getreg((3 << 11) | 20) & 7u);  // HW_REG_XCC_ID
    int* cp = lastp + 1;
    bool first = true;
    for (int probe = 0; probe < 8;) {
      const int x = (xcc + probe) & 7;
      const int t0 = x * nT / 8, ntx = (x + 1) * nT / 8 - t0, itx = npairs * ntx;
      const int chx = (itx + chunk - 1) / chunk;
      if (tid == 0) *cp = (int)__hip_atomic_fetch_add(ev.xq + x, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __syncthreads();
      const int c = __builtin_amdgcn_readfirstlane(*cp);  // (uniform: scalar item indices)
      __syncthreads();
      if (c >= chx) {
        ++probe;
        continue;
      }
      const int j0 = c * chunk, j1 = j0 + chunk < itx ? j0 + chunk : itx;
      curp = -1;
      run_items(t0, ntx, j0, j1, first);
      first = false;
    }
  }
  __syncthreads();
  {
    const int cp = xcd_copy();
    for (int m = 0; m < M; ++m) {
      const int v = cl[m * 256 + tid];
      if (v) atomicAdd(acc_cell(ev.acc, cp, m, tid), v);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (rid == 0) rstamp(8);
  if (dbg && tid == 0)
    atomicMax((unsigned long long*)(dbg + 14), (unsigned long long)__builtin_amdgcn_s_memrealtime());
  if (tid == 0)
    *lastp = __hip_atomic_fetch_add(ev.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ev.nticket - 1;
  __syncthreads();
  if (!*lastp) return;
  rstamp(10);
  publish_counts(ev, M, tid, cl);
  rstamp(11);
}

// LDS of eval_tile_body: [pairs][4 waves][2 m-tiles][64 lanes] f32x4 partial logits,
// then [kMaxEvalModels][256] counts, the publisher flag, [kMaxEvalModels][8]
// intercepts and [32] labels.
constexpr int kEvalPairs = (kMaxEvalModels + 1) / 2;
constexpr size_t kEvalTileLds = (size_t)kEvalPairs * 8192 + kMaxEvalModels * 256 * 4 + 16 +
                                kMaxEvalModels * 8 * 4 + 32 * 4 + 16;

// Riders, tile-resident form: rider rid evaluates EVERY model on test tiles rid,
// rid + nride, ...  The 32-row tile's MFMA A operands are loaded straight from
// global memory into registers (no LDS staging) and stay there while the waves run
// the model pairs' fragments past them, the next pair's fragments in flight during
// the current pair's MFMAs; the test set is read once per round.  Each wave owns
// the same K-slice and issues the same MFMA sequence as forward_tile_pre, and the
// cross-wave sums run in the same order (load_logit), so the rows equal the
// pair-major riders' bit for bit.  Counts: LDS atomics per tile, one flush per
// rider, the last arrival publishes (publish_counts).
// (kStop < 3: tools/eval_probe.hip's cost split -- 1: the tiles only, 2: + the flush)
template <int FP, int kStop = 3>
__device__ __forceinline__ void eval_tile_body(char* lds, const EvalMulti& ev, int rid, int nride) {
  if (ev.nmodels <= 0 || rid >= nride) return;
  rid = __builtin_amdgcn_readfirstlane(rid);
  long long* dbg = ev.dbg;
  auto rstamp = [&](int k) {
    if (dbg && threadIdx.x == 0) dbg[k] = (long long)__builtin_amdgcn_s_memrealtime();
  };
  if (dbg && threadIdx.x == 0) {
    const long long t = (long long)__builtin_amdgcn_s_memrealtime();
    atomicMin((unsigned long long*)(dbg + 12), (unsigned long long)t);
    atomicMax((unsigned long long*)(dbg + 13), (unsigned long long)t);
  }
  if (rid == 0) rstamp(0);
  constexpr int KS = WFrag<FP>::KS;
  char* red = lds;                                             // [kEvalPairs][8 KB]
  int* cl = (int*)(lds + (size_t)kEvalPairs * 8192);           // [kMaxEvalModels][256]
  int* lastp = cl + kMaxEvalModels * 256;
  float* bl = (float*)(lastp + 4);                             // [kMaxEvalModels][8]
  int* ylab = (int*)(bl + kMaxEvalModels * 8);                 // [32]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r = lane & 15, kq = lane >> 4;
  const int K = ev.K, T = ev.T, M = ev.nmodels, npairs = (M + 1) / 2;
  const int nT = (T + 31) / 32;
  for (int m = 0; m < M; ++m) cl[m * 256 + tid] = 0;
#pragma unroll
  for (int m = 0; m < kMaxEvalModels; ++m)  // (constant model indices: scalar kernel-argument loads)
    if (m < M && tid < 8) bl[m * 8 + tid] = tid < K ? ev.m[m].b[ev.m[m].coff + tid] : 0.f;
  auto load_pair = [&](WFrag<FP>& wf, int p) {
    const int ma = 2 * p, mb = 2 * p + 1;
    const EvalModel A = pick(ev.m, ma), Bm = pick(ev.m, mb < M ? mb : ma);
    load_pair_frags<FP>(wf, A, Bm, mb < M, K);
  };
  bool first = true;
  // tiles popped from ev.xq[0] (riders entering early take more of them); without a
  // queue, tiles rid, rid + nride, ...
  int* tq = ylab + 32;
  auto pop = [&](int fallback) {
    if (!ev.xq) return fallback;
    if (tid == 0) *tq = (int)__hip_atomic_fetch_add(ev.xq, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const int t = __builtin_amdgcn_readfirstlane(*tq);
    __syncthreads();
    return t;
  };
  // items = (tile, group of ev.ppi model pairs; 0: every pair), tile-major
  const int ppi = ev.ppi > 0 && ev.ppi < npairs ? ev.ppi : npairs, ngr = (npairs + ppi - 1) / ppi;
  u16x8 a0[KS], a1[KS];  // the tile's A operands: rows r and 16 + r, wave w's k-steps (forward_tile_pre's)
  auto load_tile = [&](int tile, int nrows) {
    const int64_t row0 = (int64_t)tile * 32;
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) {
      const int cg = (w * KS + kk) * 4 + kq;
      a0[kk] = r < nrows ? *(const u16x8*)(ev.Xt + (row0 + r) * FP + cg * 8) : u16x8{0, 0, 0, 0, 0, 0, 0, 0};
      a1[kk] = 16 + r < nrows ? *(const u16x8*)(ev.Xt + (row0 + 16 + r) * FP + cg * 8)
                              : u16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
    if (tid < 32) ylab[tid] = tid < nrows ? ev.yt[row0 + tid] : 0;
  };
  auto mfma_pair = [&](const WFrag<FP>& wf, int p) {
    f32x4 acc0 = f32x4{0, 0, 0, 0}, acc1 = f32x4{0, 0, 0, 0};
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) {
      acc0 = mfma16x16x32(as_bf16x8(a0[kk]), as_bf16x8(wf.h[kk]), acc0);
      acc0 = mfma16x16x32(as_bf16x8(a0[kk]), as_bf16x8(wf.l[kk]), acc0);
      acc1 = mfma16x16x32(as_bf16x8(a1[kk]), as_bf16x8(wf.h[kk]), acc1);
      acc1 = mfma16x16x32(as_bf16x8(a1[kk]), as_bf16x8(wf.l[kk]), acc1);
    }
    store_partial_logits(red + (size_t)p * 8192, acc0, acc1);
  };
  auto count_tile = [&](int m0, int m1, int nrows) {
    __syncthreads();
    if (first && rid == 0) rstamp(1);
    for (int it = tid; it < 32 * (m1 - m0); it += 256) {  // thread (row, model)
      const int row = it & 31, m = m0 + (it >> 5);
      if (row < nrows) {
        const char* rb = red + (size_t)(m >> 1) * 8192;
        const int c0 = 8 * (m & 1);
        int best = 0;
        float bz = -INFINITY;
        for (int c = 0; c < K; ++c) {
          const float z = load_logit(rb, row, c0 + c) + bl[m * 8 + c];
          if (z > bz) {
            bz = z;
            best = c;
          }
        }
        const int yrow = ylab[row], yl = yrow < 0 ? 0 : (yrow > 15 ? 15 : yrow);
        atomicAdd(&cl[m * 256 + yl * 16 + best], 1);
      }
    }
    __syncthreads();  // (red / ylab are rewritten by the next tile)
    first = false;
  };
  if (ev.gq && ev.xq && ppi <= 2 && ngr <= kEvalGroups) {
    // Group queues (EvalMulti::gq): rider rid starts on group rid % ngr and pops that
    // group's tiles from ev.xq[group]; the group's (<= 2) model pairs stay in registers
    // across its tiles, so a tile costs its own 64 KB and no fragment reloads.  An
    // exhausted group sends the rider to the next one.
    WFrag<FP> h0, h1;
    int g = rid % ngr, cur = -1;
    for (int left = ngr; left > 0;) {
      if (tid == 0) *tq = (int)__hip_atomic_fetch_add(ev.xq + g, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __syncthreads();
      const int tile = __builtin_amdgcn_readfirstlane(*tq);
      __syncthreads();
      if (tile >= nT) {
        g = g + 1 == ngr ? 0 : g + 1;
        --left;
        continue;
      }
      const int p0 = g * ppi, p1 = p0 + ppi < npairs ? p0 + ppi : npairs;
      const int nrows = T - tile * 32 < 32 ? T - tile * 32 : 32;
      load_tile(tile, nrows);
      if (g != cur) {  // (uniform)
        load_pair(h0, p0);
        if (p0 + 1 < p1) load_pair(h1, p0 + 1);
        cur = g;
      }
      mfma_pair(h0, p0);
      if (p0 + 1 < p1) mfma_pair(h1, p0 + 1);
      count_tile(2 * p0, 2 * p1 < M ? 2 * p1 : M, nrows);
    }
  } else {
    for (int item = pop(rid); item < nT * ngr; item = pop(item + nride)) {
      const int tile = item / ngr, gr = item - tile * ngr;
      const int p0 = gr * ppi, p1 = p0 + ppi < npairs ? p0 + ppi : npairs;
      const int nrows = T - tile * 32 < 32 ? T - tile * 32 : 32;
      load_tile(tile, nrows);
      WFrag<FP> wc, wn;
      load_pair(wc, p0);
      for (int p = p0; p < p1; ++p) {  // (uniform)
        if (p + 1 < p1) load_pair(wn, p + 1);
        mfma_pair(wc, p);
        if (p + 1 < p1) wc = wn;
      }
      count_tile(2 * p0, 2 * p1 < M ? 2 * p1 : M, nrows);
    }
  }
  if constexpr (kStop == 1) return;
  if (ev.slab) {  // slab form: this rider's counts, every cell (zeros included); no ticket
    int* row = ev.slab + (size_t)rid * kMaxEvalModels * kSlabCells;
    for (int q = tid; q < M * kSlabCells; q += 256) {
      const int m = q >> 6, c = q & 63;
      row[q] = cl[m * 256 + (c >> 3) * 16 + (c & 7)];
    }
    if (rid == 0) rstamp(8);
    return;
  }
  {
    const int cp = xcd_copy();
    for (int m = 0; m < M; ++m) {
      const int v = cl[m * 256 + tid];
      if (v) atomicAdd(acc_cell(ev.acc, cp, m, tid), v);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if constexpr (kStop == 2) return;
  if (rid == 0) rstamp(8);
  if (dbg && tid == 0)
    atomicMax((unsigned long long*)(dbg + 14), (unsigned long long)__builtin_amdgcn_s_memrealtime());
  if (tid == 0)
    *lastp = __hip_atomic_fetch_add(ev.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ev.nticket - 1;
  __syncthreads();
  if (!*lastp) return;
  rstamp(10);
  // (every rider has popped its last item: the queue is free for the next pass)
  if (ev.xq && tid < (ev.gq ? kEvalGroups : 1)) __hip_atomic_store(ev.xq + tid, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  publish_counts(ev, M, tid, cl);
  rstamp(11);
}

// The BSP update of one slice by the last lane to finish it: w += lr * (sum of
// the lanes' deltas, lane order) and the server's evaluation fragments, or the
// plain sum into dsum (multi-rank).  A lane whose solve reported a timed-out
// wait (sticky error word) contributes nothing.  Slice 0 also carries the
// intercepts (each lane's workgroup 0 stored them before arriving).  Every
// lane's error word and delta element are loaded before the first is used: one
// round trip to the other XCDs' data, not one per lane.
struct ApplyArgs {
  int L;
  float* w;
  float lr;
  float* dsum;  // != nullptr: the lane sum goes here (multi-rank), w untouched
  uint16_t *shi, *slo;  // the server's evaluation fragments of this update
  float* sb;
  int scoff;
  // overlapped launches (LanesArgs::ovl): w read and written through (its readers
  // run on other XCDs in a launch that overlaps this one), then applied[slice] = round + 1
  unsigned* applied = nullptr;
  unsigned round = 0;
  // peer_sum (LanesArgs::push): the lane sum goes to this rank's inbox slot on the server
  // GPU (system-scope stores over xGMI), then the slice's tag push_val; w untouched
  float* push = nullptr;
  unsigned* push_tag = nullptr;
  unsigned push_val = 0;
};

// Spin until *p >= want (device-scope loads); a timeout sets the sticky error word
__device__ __forceinline__ void wait_ge(unsigned* p, unsigned want, unsigned long long* err, int spin_max) {
  if (threadIdx.x == 0) {
    int spins = 0;
    while ((int)(__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - want) < 0) {
      __builtin_amdgcn_s_sleep(2);
      if (++spins > spin_max) {  // never expected: record and fall through rather than hang
        if (err) xstore(err, 9ull);
        break;
      }
    }
  }
  __syncthreads();
}

template <int FP>
__device__ __forceinline__ void lane_apply_slice(const SolverCfg& cfg, const LaneDev* lanes, const ApplyArgs& a,
                                                 int wg) {
  const int tid = threadIdx.x, K = cfg.K, L = a.L;
  const int c = tid >> 5, f = wg * 32 + (tid & 31);
  const bool coef = c < K;
  const bool icpt = wg == 0 && tid < K;  // (threads 0..K-1 carry one intercept each as well)
  const size_t e = (size_t)c * FP + f, ei = (size_t)K * FP + tid;
  unsigned long long er[kMaxLanes];
  float dl[kMaxLanes], di[kMaxLanes];
#pragma unroll
  for (int l = 0; l < kMaxLanes; ++l) {
    er[l] = 0ull;
    dl[l] = di[l] = 0.f;
    if (l < L) {
      er[l] = xload(lanes[l].dv.xch + kXchErr);
      if (coef) dl[l] = ld_sc1(lanes[l].dv.delta + e);
      if (icpt) di[l] = ld_sc1(lanes[l].dv.delta + ei);
    }
  }
  const bool wt = a.applied != nullptr;  // (write-through: overlapped launches)
  float sum = 0.f, sumi = 0.f;
#pragma unroll
  for (int l = 0; l < kMaxLanes; ++l)
    if (l < L && er[l] == 0ull) {
      sum += dl[l];
      sumi += di[l];
    }
  if (a.push) {  // the rank's push (WorkerTrainingProcessor.java:95-97): the server sums the ranks
    // system-scope stores (sc0 sc1: written through to the server GPU's memory), every
    // wave's vmcnt(0), a barrier, then the tag: no release fence -- nothing of the hand-off
    // sits dirty in an L2 (the sc0 sc1 form of the CDNA4 playbook, at system scope), and a
    // system-scope release would write back this XCD's whole L2 on the round's critical path
    if (coef) st_sys_f32(a.push + e, sum);
    if (icpt) st_sys_f32(a.push + ei, sumi);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) st_sys_u32(a.push_tag + wg, a.push_val);
    return;
  }
  if (coef) {
    if (a.dsum) {
      a.dsum[e] = sum;
    } else {
      const float nw = (wt ? ld_sc1(a.w + e) : a.w[e]) + a.lr * sum;
      if (wt)
        st_sc1(a.w + e, nw);
      else
        a.w[e] = nw;
      write_frag(a.shi, a.slo, a.scoff + c, f, f < cfg.F ? nw : 0.f);
    }
  }
  if (icpt) {
    if (a.dsum) {
      a.dsum[ei] = sumi;
    } else {
      const float nw = (wt ? ld_sc1(a.w + ei) : a.w[ei]) + a.lr * sumi;
      if (wt)
        st_sc1(a.w + ei, nw);
      else
        a.w[ei] = nw;
      a.sb[a.scoff + tid] = nw;
    }
  }
  if (wt) {  // the slice's new weights are out: the next round's owners may read them
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) __hip_atomic_store(a.applied + wg, a.round + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Arrive on slice `idx`'s lane counter (every store of this workgroup drained
// first); true for the last lane, which resets the counter for the next launch.
__device__ __forceinline__ bool lane_arrive(unsigned* arrive, int idx, int L, int* flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned old = __hip_atomic_fetch_add(arrive + idx, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const bool last = old == (unsigned)L - 1u;
    if (last) __hip_atomic_store(arrive + idx, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = last ? 1 : 0;
  }
  __syncthreads();
  return *flag != 0;
}

// ---------------------------------------------------------------------------
// Phase I of a lane's solve, row role: row workgroup `wg` of `ntr` takes window ring
// tiles wg, wg + ntr, ... (of `ntt`: one each up to 32 tiles, a 1,024-row ring; more
// for longer windows), stages them into the LDS image (the last one stays: resident
// when it is the only one), the round's new rows straight from the dataset (also
// written into the ring), and publishes its tiles' column sums / sums of squares
// over their window rows.  Thread t holds chunk cg = t % CPR (8 features) of rows
// g + NG j (g = t / CPR), so the sums come from the staging registers (tile order);
// the NG row groups are combined in LDS (fixed order).
template <int FP, int S>
__device__ __forceinline__ void lane_stage_stats(char* lf, float* scratch, const SolverCfg& cfg, const SolveDev& dv,
                                                 const LaneRound& r, const uint16_t* dsX, const int32_t* dsy,
                                                 const WinTiles& wt, int wg, int ntr, int ntt, float* spart_wg) {
  constexpr int CPR = FP / 8, NG = 256 / CPR, PER_T = 32 * CPR / 256;
  const int tid = threadIdx.x, cap = cfg.cap;
  const int cg = tid % CPR, g = tid / CPR;
  uint16_t* X = const_cast<uint16_t*>(dv.X);
  int32_t* Y = const_cast<int32_t*>(dv.y);
  // the dataset row of ring slot s when it holds one of this round's new rows, else -1
  auto new_src = [&](int s) -> long long {
    int dn = s - r.dst;
    if (dn < 0) dn += cap;
    if (dn < r.n) return r.first + (long long)dn * r.step;
    if (dn - r.n < r.n2) return r.first2 + (long long)(dn - r.n) * r.step;
    return -1;
  };
  float sm[8], sq[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) sm[e] = sq[e] = 0.f;
  for (int ti = wg; ti < ntt; ti += ntr) {
    const int rt = wt.ring_tile(ti);
    // labels travel with the first loads
    int yv = 0;
    bool ynew = false;
    if (tid < 32) {
      const int s = rt * 32 + tid;
      const long long src = new_src(s);
      ynew = src >= 0;
      yv = ynew ? dsy[src] : dv.y[s];
    }
    u16x8 v[PER_T];
    bool isnew[PER_T], valid[PER_T];
#pragma unroll
    for (int j = 0; j < PER_T; ++j) {
      const int row = g + NG * j, s = rt * 32 + row;
      const long long sr = new_src(s);
      isnew[j] = sr >= 0;
      int dw = s - r.start;
      if (dw < 0) dw += cap;
      valid[j] = dw < r.B;
      const uint16_t* src = isnew[j] ? dsX + (size_t)sr * FP : dv.X + (size_t)s * FP;
      v[j] = *(const u16x8*)(src + cg * 8);
    }
#pragma unroll
    for (int j = 0; j < PER_T; ++j) {
      const int row = g + NG * j, s = rt * 32 + row;
      *(u16x8*)(lf + (cg >> 4) * 8192 + lds_off(row, cg & 15)) = v[j];
      if (isnew[j]) *(u16x8*)(X + (size_t)s * FP + cg * 8) = v[j];  // the ring keeps the new row
      if (valid[j]) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float x = bf2f(v[j][e]);
          sm[e] += x;
          sq[e] += x * x;
        }
      }
    }
    if (tid < 32) {
      ((int*)(lf + 32 * FP * 2 + 8192 + 2048))[tid] = yv;  // fwd_body's label slots
      if (ynew) Y[rt * 32 + tid] = yv;
    }
    if (ti + ntr < ntt) __syncthreads();  // (the next tile's image over this one)
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    scratch[(g * CPR + cg) * 16 + e] = sm[e];
    scratch[(g * CPR + cg) * 16 + 8 + e] = sq[e];
  }
  __syncthreads();
  if (tid < CPR) {
    float a[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) a[e] = 0.f;
    for (int gg = 0; gg < NG; ++gg)  // fixed order
#pragma unroll
      for (int e = 0; e < 16; ++e) a[e] += scratch[(gg * CPR + tid) * 16 + e];
    // 8 features x (sum, sum of squares) = 64 contiguous bytes of spart[wg][f][2]
    const auto rs = rsrc_of(spart_wg, (unsigned)(FP * 2 * 4));
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const f32x4 o = f32x4{a[2 * q], a[8 + 2 * q], a[2 * q + 1], a[8 + 2 * q + 1]};
      st_h_b128<S>(rs, (unsigned)((tid * 8 + 2 * q) * 2 * 4), __builtin_bit_cast(u16x8, o));
    }
  }
}

// Phase I, slice role: the window statistics of features [fs, fs + 32) from the
// row workgroups' partials, then x0 = w_old * std (Spark standardisation), the
// solver vectors and the first trial point's fragments (as prep_epilogue).
template <int FP, int KP, int S>
__device__ __forceinline__ void lane_prep(char* lb, const SolverCfg& cfg, const SolveDev& dv, const float* spart,
                                          int ntr, int B, int wg, float wo_pre, float b_pre) {
  constexpr int FPI = FP > 256 ? FP : 256;
  const int tid = threadIdx.x, fl = tid & 31, grp = tid >> 5, fs = wg * 32, K = cfg.K;
  double* red = (double*)lb;                  // [8 groups][32][2]
  float* sdl = (float*)(red + 8 * 32 * 2);    // [32]
  float* ivl = sdl + 32;                      // [32]
  unsigned short* frl = (unsigned short*)(lb + 4 * 16 * 32 * 4);  // [2][512] (bwd_body's staging)
  double s = 0.0, q = 0.0;
  {  // the (<= 4) row tiles' partials of this thread all in flight, then summed in tile order
    constexpr int NPT = (kLaneWg + 7) / 8;
    double pv[NPT];
#pragma unroll
    for (int i = 0; i < NPT; ++i) {
      const int gg = grp + 8 * i;
      pv[i] = gg < ntr ? ld_h<S>((const double*)(spart + ((size_t)gg * FP + fs + fl) * 2)) : 0.0;
    }
#pragma unroll
    for (int i = 0; i < NPT; ++i)
      if (grp + 8 * i < ntr) {
        const float2 u = __builtin_bit_cast(float2, pv[i]);
        s += (double)u.x;
        q += (double)u.y;
      }
  }
  red[(grp * 32 + fl) * 2] = s;
  red[(grp * 32 + fl) * 2 + 1] = q;
  if (tid < 128) *(u16x8*)(frl + tid * 8) = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
  __syncthreads();
  if (tid < 32) {
    double a = 0.0, b = 0.0;
    for (int gg = 0; gg < 8; ++gg) {
      a += red[(gg * 32 + tid) * 2];
      b += red[(gg * 32 + tid) * 2 + 1];
    }
    const int f = fs + tid;
    const double n = (double)B;
    double sd = 0.0;
    if (f < cfg.F && n > 1.0) {
      const double mean = a / n;
      const double var = (b - n * mean * mean) / (n - 1.0);
      sd = var > 0.0 ? sqrt(var) : 0.0;
    }
    const float sdf = (float)sd, inv = sd > 0.0 ? (float)(1.0 / sd) : 0.f;
    sdl[tid] = sdf;
    ivl[tid] = inv;
    dv.std_[f] = sdf;
    dv.inv_std[f] = inv;
  }
  __syncthreads();
  {  // element (c = tid / 32, feature fs + fl): x0, d, g_c, wfix, trial fragment
    const int c = grp;
    if (c < KP) {
      const int f = fs + fl, pi = c * FPI + f;
      const float xv = wo_pre * sdl[fl];
      dv.x[pi] = xv;
      dv.d[pi] = 0.f;
      dv.g_c[pi] = 0.f;
      const float fix = (sdl[fl] > 0.f || cfg.zero_const) ? 0.f : wo_pre;
      dv.wfix[pi] = fix;
      unsigned short h, l;
      split_bf16(xv * ivl[fl] + fix, h, l);
      const int o = (fl >> 3) * 128 + c * 8 + (fl & 7);
      frl[o] = h;
      frl[512 + o] = l;
    }
  }
  if (wg == 0 && tid < 16) {  // intercepts: x0 = the pulled intercepts (not standardised)
    const int pi = KP * FPI + tid;
    dv.x[pi] = b_pre;
    dv.d[pi] = 0.f;
    dv.g_c[pi] = 0.f;
    st_h<S>(dv.b_eff + tid, b_pre);
  }
  (void)K;
  __syncthreads();
  if (tid < 128) {  // this slice of the trial fragments: 16-B hand-off stores (wave 0 hi, wave 1 lo)
    const size_t go = (size_t)(fs >> 3) * 128 + (tid & 63) * 8;
    const u16x8 vv = *(const u16x8*)(frl + tid * 8);
    if (tid < 64)
      st_h_b128<S>(rsrc_of(dv.whi, 16u * FP * 2u), (unsigned)(go * 2), vv);
    else
      st_h_b128<S>(rsrc_of(dv.wlo, 16u * FP * 2u), (unsigned)(go * 2), vv);
  }
}

// ---------------------------------------------------------------------------
// A lane's own evaluation pass (both the BSP round kernel and the asynchronous
// launch): model A (the lane's local model -- the worker row,
// LogisticRegressionTaskSpark.java:186) and optionally model B (a global model --
// the server row, ServerProcessor.java:154-165) in one MFMA pass (A in columns
// 0..7, B in 8..15) over the test tiles wg, wg + G, ... of the lane's G
// workgroups, while the other lanes still solve on their XCDs.  Counts go to the
// lane's accumulators; the last of the G arrivals publishes each row into its
// pinned slot as tagged 16-B chunks (sink kind | kSinkTagged): no wait for the
// system-scope stores to complete on the lane's path.
// Fragments written in this launch by the lane's own workgroups (one XCD): nt loads.
struct PairModels {
  const uint16_t *ah, *al;  // model A fragments (columns acoff .. acoff + K - 1)
  const float* ab;          // A's intercepts
  const float* aloss;       // A's training loss (the worker row's), nullptr: 0
  char* aslot;              // nullptr: no A row
  unsigned aseq;
  const uint16_t *bh, *bl;  // model B (columns 0..K-1 of its buffers)
  const float* bb;
  char* bslot;              // nullptr: no B row
  unsigned bseq;
  int acoff = 0, bcoff = 0;  // first class column of each model in its buffers
};


// The counts of a pair pass: this workgroup's LDS counts cl[2][256] into the lane's
// accumulators, then the last of the G arrivals writes each row into its pinned slot as
// tagged 16-B chunks (sink kind | kSinkTagged): no wait for the system-scope stores to
// complete on the lane's path.
__device__ __forceinline__ void pair_eval_publish(int* cl, int* lastp, int K, const PairModels& pm, int* acc,
                                                  unsigned* ticket, int G, bool wrow, bool srow) {
  const int tid = threadIdx.x;
  for (int m = 0; m < 2; ++m) {
    const int v = cl[m * 256 + tid];
    if (v) atomicAdd(acc + (m * 256 + tid) * kAccStride, v);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0)
    *lastp = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)G - 1u;
  __syncthreads();
  if (!*lastp) return;
  // the last workgroup: the lane's counts -> LDS [K][K], then tagged chunks to the slots
  const int t16 = tid >> 4, p16 = tid & 15;
  const bool cell = t16 < K && p16 < K;
  for (int m = 0; m < 2; ++m) {
    const int v = cell ? __hip_atomic_exchange(acc + (m * 256 + tid) * kAccStride, 0, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT)
                       : 0;
    if (cell) cl[m * 256 + t16 * K + p16] = v;
  }
  const float lv = (tid == 0 && wrow && pm.aloss) ? ld_h<2>(pm.aloss) : 0.f;
  if (tid == 0) __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const int nch = 1 + (K * K + 2) / 3;
  const int m = tid >> 6, i = tid & 63;  // wave 0: row A, wave 1: row B
  if (m < 2 && i < nch && (m == 0 ? wrow : srow)) {
    const unsigned tag = eval_tag(m == 0 ? pm.aseq : pm.bseq);
    TagChunk ch;
    if (i == 0) {
      ch = TagChunk{tag, __float_as_uint(m == 0 ? __shfl(lv, 0, 64) : 0.f), (unsigned)K, 0u};
    } else {
      const int c0 = 3 * (i - 1);
      auto cv = [&](int c) { return c < K * K ? (unsigned)cl[m * 256 + c] : 0u; };
      ch = TagChunk{tag, cv(c0), cv(c0 + 1), cv(c0 + 2)};
    }
    st_sys_chunk(m == 0 ? pm.aslot : pm.bslot, 1088u, (unsigned)i * 16u, ch);
  }
}

// The slab form of pair_eval_publish (no device-scope atomics): each workgroup stores its
// K x K counts of both models into its row of `slab` [G][2][64] ints, arrives on the
// ticket, and the last one sums the G rows in workgroup order (nt loads: the lane's
// workgroups share one XCD's L2) and publishes the rows as tagged chunks.
__device__ __forceinline__ void pair_eval_publish_slab(int* cl, int* lastp, int K, const PairModels& pm, int* slab,
                                                       unsigned* ticket, int wg, int G, bool wrow, bool srow) {
  const int tid = threadIdx.x, KK = K * K;
  if (tid < 128) {
    const int m = tid >> 6, c = tid & 63;
    slab[(size_t)wg * 128 + tid] = c < KK ? cl[m * 256 + (c / K) * 16 + (c - (c / K) * K)] : 0;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0)
    *lastp = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)G - 1u;
  __syncthreads();
  if (!*lastp) return;
  if (tid < 128) {
    int v[kLaneWg];
#pragma unroll
    for (int g = 0; g < kLaneWg; ++g) v[g] = g < G ? __builtin_nontemporal_load(slab + (size_t)g * 128 + tid) : 0;
    int t = 0;
#pragma unroll
    for (int g = 0; g < kLaneWg; ++g) t += v[g];
    cl[(tid >> 6) * 256 + (tid & 63)] = t;  // [model][cell k = true * K + pred]
  }
  const float lv = (tid == 0 && wrow && pm.aloss) ? ld_h<2>(pm.aloss) : 0.f;
  if (tid == 0) __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const int nch = 1 + (KK + 2) / 3;
  const int m = tid >> 6, i = tid & 63;  // wave 0: row A, wave 1: row B
  if (m < 2 && i < nch && (m == 0 ? wrow : srow)) {
    const unsigned tag = eval_tag(m == 0 ? pm.aseq : pm.bseq);
    TagChunk ch;
    if (i == 0) {
      ch = TagChunk{tag, __float_as_uint(m == 0 ? __shfl(lv, 0, 64) : 0.f), (unsigned)K, 0u};
    } else {
      const int c0 = 3 * (i - 1);
      auto cv = [&](int c) { return c < KK ? (unsigned)cl[m * 256 + c] : 0u; };
      ch = TagChunk{tag, cv(c0), cv(c0 + 1), cv(c0 + 2)};
    }
    st_sys_chunk(m == 0 ? pm.aslot : pm.bslot, 1088u, (unsigned)i * 16u, ch);
  }
}

// red_base: kPairEvalLds bytes of LDS (the logits' exchange, the counts)
constexpr int kPairEvalLds = 8192 + 2 * 256 * 4 + 16 + 16 * 4;
template <int FP>
__device__ __forceinline__ void lane_pair_eval_at(char* red_base, int K, const uint16_t* Xt, const int32_t* yt, int T,
                                                  int wg, int G, const PairModels& pm, int* acc, unsigned* ticket) {
  const int tid = threadIdx.x;
  const bool wrow = pm.aslot != nullptr, srow = pm.bslot != nullptr;
  if (!wrow && !srow) return;  // (uniform)
  int* cl = (int*)(red_base + 8192);  // [2][256]
  int* lastp = cl + 512;
  float* bl = (float*)(lastp + 4);    // [16]: model A 0..7, model B 8..15
  cl[tid] = 0;
  cl[256 + tid] = 0;
  WFrag<FP> wf;
  {
    const int lane = tid & 63, w = tid >> 6, col = lane & 15, cc = col & 7;
    const bool live = cc < K && (col < 8 ? wrow : srow);
    const uint16_t* fh = col < 8 ? pm.ah : pm.bh;
    const uint16_t* fo = col < 8 ? pm.al : pm.bl;
    const auto rh = rsrc_of(live ? fh : pm.ah, 16u * FP * 2u), rl = rsrc_of(live ? fo : pm.al, 16u * FP * 2u);
#pragma unroll
    for (int kk = 0; kk < WFrag<FP>::KS; ++kk) {
      const int cg = (w * WFrag<FP>::KS + kk) * 4 + (lane >> 4);
      const int co = col < 8 ? pm.acoff : pm.bcoff;
      const unsigned off = (unsigned)((cg * 16 + (live ? cc + co : 0)) * 8) * 2u;
      wf.h[kk] = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
      wf.l[kk] = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
      if (live) {
        wf.h[kk] = ld_h_b128<2>(rh, off);
        wf.l[kk] = ld_h_b128<2>(rl, off);
      }
    }
  }
  if (tid < 16) {
    const int cc = tid & 7;
    const bool live = cc < K && (tid < 8 ? wrow : srow);
    bl[tid] = live ? ld_h<2>((tid < 8 ? pm.ab + pm.acoff : pm.bb + pm.bcoff) + cc) : 0.f;
  }
  // the tile's MFMA A operands straight from global memory into registers (rows r
  // and 16 + r, wave w's k-steps, as forward_tile_pre reads them from LDS), the next
  // tile's in flight during the current tile's MFMAs -- no LDS staging
  const int nT = (T + 31) / 32;
  constexpr int KS = WFrag<FP>::KS;
  const int lane = tid & 63, w = tid >> 6, r = lane & 15, kq = lane >> 4;
  u16x8 a0[KS], a1[KS];
  int ylab = 0;
  auto load_tile = [&](int tile) {
    const int64_t row0 = (int64_t)tile * 32;
    const int nr = T - tile * 32 < 32 ? T - tile * 32 : 32;
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) {
      const int cg = (w * KS + kk) * 4 + kq;
      a0[kk] = r < nr ? *(const u16x8*)(Xt + (row0 + r) * FP + cg * 8) : u16x8{0, 0, 0, 0, 0, 0, 0, 0};
      a1[kk] = 16 + r < nr ? *(const u16x8*)(Xt + (row0 + 16 + r) * FP + cg * 8) : u16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
    ylab = tid < nr ? yt[row0 + tid] : 0;
  };
  if (wg < nT) load_tile(wg);
  __syncthreads();
  for (int tile = wg; tile < nT; tile += G) {
    const int nrows = T - tile * 32 < 32 ? T - tile * 32 : 32;
    f32x4 acc0 = f32x4{0, 0, 0, 0}, acc1 = f32x4{0, 0, 0, 0};
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) {
      acc0 = mfma16x16x32(as_bf16x8(a0[kk]), as_bf16x8(wf.h[kk]), acc0);
      acc0 = mfma16x16x32(as_bf16x8(a0[kk]), as_bf16x8(wf.l[kk]), acc0);
      acc1 = mfma16x16x32(as_bf16x8(a1[kk]), as_bf16x8(wf.h[kk]), acc1);
      acc1 = mfma16x16x32(as_bf16x8(a1[kk]), as_bf16x8(wf.l[kk]), acc1);
    }
    const int ycur = ylab;
    if (tile + G < nT) load_tile(tile + G);  // (the MFMAs above consumed a0 / a1)
    store_partial_logits(red_base, acc0, acc1);
    __syncthreads();
    {  // thread (row, model)
      const int row = tid & 31, h = (tid >> 5) & 1;
      const int yrow = __shfl(ycur, row, 64);
      if (tid < 64 && row < nrows && (h == 0 ? wrow : srow)) {
        const int yl = yrow < 0 ? 0 : (yrow > 15 ? 15 : yrow);
        int best = 0;
        float bz = -INFINITY;
        for (int c = 0; c < K; ++c) {
          const float z = load_logit(red_base, row, 8 * h + c) + bl[8 * h + c];
          if (z > bz) {
            bz = z;
            best = c;
          }
        }
        atomicAdd(&cl[h * 256 + yl * 16 + best], 1);
      }
    }
    __syncthreads();
  }
  pair_eval_publish(cl, lastp, K, pm, acc, ticket, G, wrow, srow);
}
// (the lane kernels: the exchange sits behind the row workgroups' 32-row tile image)
template <int FP>
__device__ __forceinline__ void lane_pair_eval(char* lds, int K, const uint16_t* Xt, const int32_t* yt, int T, int wg,
                                               int G, const PairModels& pm, int* acc, unsigned* ticket) {
  lane_pair_eval_at<FP>(lds + 32 * FP * 2, K, Xt, yt, T, wg, G, pm, acc, ticket);
}


// The same pair pass over the test set in ELL form (EvalSet.ell: [T][nz] feature ids +
// bf16 values, nz a multiple of 8; the hashed bag-of-words rows are ~3 % dense, so 1.3 MB
// instead of the 10 MB dense tiles): both models' weights w = hi + lo (exact in fp32)
// staged into LDS feature-major, [model][FP][8 classes] (one feature's classes = two
// 16-B LDS reads), then one thread per row -- z_c = b_c + sum_j x_j w_c[id_j] in feature
// order -- and the argmax counts.  Every product x * w is exact as in the MFMA form (8 x
// 16 significant bits); only the summation order differs.
// LDS: ell_eval_lds_bytes(FP).
constexpr size_t ell_eval_lds_bytes(int FP) { return (size_t)2 * 8 * FP * 4 + 2 * 256 * 4 + 16 + 16 * 4; }
template <int FP>
__device__ __forceinline__ void lane_pair_eval_ell(char* lds, int K, const uint16_t* Ti, const uint16_t* Tv, int nz,
                                                   const int32_t* yt, int T, int wg, int G, const PairModels& pm,
                                                   int* acc, unsigned* ticket, int* slab = nullptr) {
  const int tid = threadIdx.x;
  const bool wrow = pm.aslot != nullptr, srow = pm.bslot != nullptr;
  if (!wrow && !srow) return;  // (uniform)
  float* wl = (float*)lds;                         // [2][FP][8]
  int* cl = (int*)(lds + (size_t)2 * 8 * FP * 4);  // [2][256]
  int* lastp = cl + 512;
  float* bl = (float*)(lastp + 4);  // [16]: model A 0..7, model B 8..15
  cl[tid] = 0;
  cl[256 + tid] = 0;
  constexpr int NCH = FP / 8;  // 8-feature chunks of a fragment column
  // thread -> (model, chunk of 8 features): every class column of that chunk (hi + lo)
  for (int i = tid; i < 2 * NCH; i += 256) {
    const int m = i / NCH, ch = i - m * NCH;
    const bool mine = m == 0 ? wrow : srow;
    const int co = m == 0 ? pm.acoff : pm.bcoff;
    float v[8][8];  // [class][feature in chunk]
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const bool live = mine && c < K;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[c][j] = 0.f;
      if (live) {
        const size_t o = ((size_t)ch * 16 + co + c) * 8;
        const u16x8 h = __builtin_nontemporal_load((const u16x8*)((m == 0 ? pm.ah : pm.bh) + o));
        const u16x8 l = __builtin_nontemporal_load((const u16x8*)((m == 0 ? pm.al : pm.bl) + o));
#pragma unroll
        for (int j = 0; j < 8; ++j) v[c][j] = bf2f(h[j]) + bf2f(l[j]);
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float* dst = wl + ((size_t)m * FP + ch * 8 + j) * 8;
      *(f32x4*)dst = f32x4{v[0][j], v[1][j], v[2][j], v[3][j]};
      *(f32x4*)(dst + 4) = f32x4{v[4][j], v[5][j], v[6][j], v[7][j]};
    }
  }
  if (tid < 16) {
    const int cc = tid & 7;
    const bool live = cc < K && (tid < 8 ? wrow : srow);
    bl[tid] = live ? ld_h<2>((tid < 8 ? pm.ab + pm.acoff : pm.bb + pm.bcoff) + cc) : 0.f;
  }
  __syncthreads();
  const f32x4* wv = (const f32x4*)wl;
  // a contiguous block of rows per workgroup (every workgroup busy: 4,877 rows over 32
  // workgroups, not 256-row blocks over the first 19), a thread per row
  const int per = (T + G - 1) / G, r1 = (wg + 1) * per < T ? (wg + 1) * per : T;
  for (int r = wg * per + tid; r < r1; r += 256) {
    f32x4 a0 = f32x4{bl[0], bl[1], bl[2], bl[3]}, a1 = f32x4{bl[4], bl[5], bl[6], bl[7]};
    f32x4 b0 = f32x4{bl[8], bl[9], bl[10], bl[11]}, b1 = f32x4{bl[12], bl[13], bl[14], bl[15]};
    const uint16_t* ip = Ti + (size_t)r * nz;
    const uint16_t* vp = Tv + (size_t)r * nz;
    for (int q = 0; q < nz; q += 8) {
      const u16x8 iv = *(const u16x8*)(ip + q);
      const u16x8 vv = *(const u16x8*)(vp + q);
      if (vv[0] == 0) break;  // (the row's nonzeros come first: the rest is padding)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float x = bf2f(vv[j]);
        const int f = iv[j];
        a0 += x * wv[f * 2];
        a1 += x * wv[f * 2 + 1];
        b0 += x * wv[(FP + f) * 2];
        b1 += x * wv[(FP + f) * 2 + 1];
      }
    }
    const int y = yt[r];
    const int yl = y < 0 ? 0 : (y > 15 ? 15 : y);
    const float za[8] = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
    const float zb[8] = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
    int ba = 0, bb = 0;
    float za_best = -INFINITY, zb_best = -INFINITY;
#pragma unroll
    for (int c = 0; c < 8; ++c)
      if (c < K) {
        if (za[c] > za_best) {
          za_best = za[c];
          ba = c;
        }
        if (zb[c] > zb_best) {
          zb_best = zb[c];
          bb = c;
        }
      }
    if (wrow) atomicAdd(&cl[yl * 16 + ba], 1);
    if (srow) atomicAdd(&cl[256 + yl * 16 + bb], 1);
  }
  __syncthreads();
  if (slab)
    pair_eval_publish_slab(cl, lastp, K, pm, slab, ticket, wg, G, wrow, srow);
  else
    pair_eval_publish(cl, lastp, K, pm, acc, ticket, G, wrow, srow);
}

}  // namespace lanes_detail
}  // namespace psx
