// Wide / sparse logistic-regression kernels (gfx950 / CDNA4).  See
// wide_kernels.h for the design and layouts.
//
// Reference math being replaced: the worker's Spark fit on its buffer
// (LogisticRegressionTaskSpark.java:142-221), test-set metrics
// (LogisticRegressionTaskSpark.java:236-251, Metrics.java:15-24) and the
// server's per-key update loop (ServerProcessor.java:148-151, 225-228).
#include <hip/hip_runtime.h>

#include "common.h"
#include "wide_kernels.h"

namespace psx {

namespace {

typedef __attribute__((address_space(1))) unsigned long long gu64w;

__device__ __forceinline__ double ld_agent_f64(const double* p) {
  return __builtin_bit_cast(double, __hip_atomic_load((gu64w*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

template <int KP>
__device__ __forceinline__ void ldk(const float* __restrict__ p, float (&o)[KP]) {
  if constexpr (KP % 4 == 0) {
#pragma unroll
    for (int q = 0; q < KP / 4; ++q) {
      const f32x4 t = *(const f32x4*)(p + 4 * q);
      o[4 * q] = t[0];
      o[4 * q + 1] = t[1];
      o[4 * q + 2] = t[2];
      o[4 * q + 3] = t[3];
    }
  } else if constexpr (KP == 2) {
    const float2 t = *(const float2*)p;
    o[0] = t.x;
    o[1] = t.y;
  } else {
    o[0] = p[0];
  }
}

// Class probabilities -> residual r = (p - onehot(y)) * invB and the row loss.
// K == 1: binary sigmoid model (label y in {0,1}).
template <int KP>
__device__ __forceinline__ float row_residual(const float (&z)[KP], int K, int y, float invB, float (&r)[KP]) {
  if (K == 1) {
    const float zz = z[0];
    const float yy = y > 0 ? 1.f : 0.f;
    const float p = 1.f / (1.f + __expf(-zz));
    r[0] = (p - yy) * invB;
#pragma unroll
    for (int c = 1; c < KP; ++c) r[c] = 0.f;
    // softplus(z) - y z, stable for both signs
    return fmaxf(zz, 0.f) + log1pf(__expf(-fabsf(zz))) - yy * zz;
  }
  const int yc = y < 0 ? 0 : (y >= K ? K - 1 : y);
  float m = -INFINITY;
#pragma unroll
  for (int c = 0; c < KP; ++c)
    if (c < K) m = fmaxf(m, z[c]);
  float e[KP];
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < KP; ++c) {
    e[c] = c < K ? __expf(z[c] - m) : 0.f;
    s += e[c];
  }
  const float is = 1.f / s;
  float zy = 0.f;
#pragma unroll
  for (int c = 0; c < KP; ++c) {
    r[c] = c < K ? (e[c] * is - (c == yc ? 1.f : 0.f)) * invB : 0.f;
    if (c == yc) zy = z[c];
  }
  return __logf(s) + m - zy;
}

}  // namespace

// ---------------------------------------------------------------------------
// begin: reset the previous solve's feature map entries, publish the window.
__device__ __forceinline__ void wide_begin_body(const WideDev& d, int B, int start, int blk, int nblk) {
  const unsigned prevU = d.cnt[2];
  const unsigned nthr = blockDim.x;
  if (blk == 0 && threadIdx.x == 0) {
    d.prm->B = B;
    d.prm->start = start;
    d.cnt[0] = 0u;  // not read by anybody else in this phase
    d.cnt[1] = 0u;
    *d.gbar = 0ull;  // grid-barrier counter of this solve's tail launch
  }
  for (unsigned i = blk * nthr + threadIdx.x; i < prevU; i += nblk * nthr) d.htab[d.hslot[i]] = make_int2(-1, -1);
  if (blk == 0 && threadIdx.x < 2 * kMaxOwners) d.own[threadIdx.x] = 0u;
}

__global__ __launch_bounds__(256) void wide_begin_kernel(WideDev d, int B, int start) {
  wide_begin_body(d, B, start, blockIdx.x, gridDim.x);
}

// plan: per group of RB window rows, dedup the entries' features in an LDS
// hash table (linear probing), give every entry its group slot, and give every
// feature new to the window a compact id (first CAS of its key into the
// window table htab wins; winners of a wave take consecutive ids with ONE
// atomic per wave).  A hot feature thus costs one global CAS per group instead
// of one per row.
__device__ __forceinline__ unsigned wide_hash(int f) { return (unsigned)f * 2654435761u; }

// Group `b` of the window (any block size; LDS: (2 TS + EB) ints at plan_lds).
__device__ __forceinline__ void wide_plan_body(const WideCfg& c, const WideDev& d, int b, int* plan_lds) {
  const int TS = d.TS, EB = d.EB, RB = d.RB, NZ = c.NZ, cap = c.cap;
  const int nthr = blockDim.x;
  int* keys = plan_lds;        // [TS]
  int* sidx = keys + TS;       // [TS]
  int* bf = sidx + TS;         // [EB]
  __shared__ int nuq;
  const int B = d.prm->B, start = d.prm->start;
  const int t = threadIdx.x, lane = __lane_id();
  const int r0 = b * RB;
  if (r0 >= B) return;
  const int rows = min(RB, B - r0);
  for (int h = t; h < TS; h += nthr) keys[h] = -1;
  if (t == 0) nuq = 0;
  __syncthreads();
  const int ne = rows * NZ;
  for (int el = t; el < ne; el += nthr) {
    const int r = el / NZ, j = el - r * NZ;
    int sl = start + r0 + r;
    if (sl >= cap) sl -= cap;
    if (j >= d.rnnz[sl]) continue;
    const int f = d.ridx[(size_t)sl * NZ + j];
    unsigned h = wide_hash(f) & (TS - 1);
    while (true) {
      const int old = atomicCAS(&keys[h], -1, f);
      if (old == -1 || old == f) break;
      h = (h + 1) & (TS - 1);
    }
  }
  __syncthreads();
  for (int h = t; h < TS; h += nthr) {
    const int k = keys[h];
    if (k != -1) {
      const int sidx_h = atomicAdd(&nuq, 1);
      sidx[h] = sidx_h;
      bf[sidx_h] = k;
    }
  }
  __syncthreads();
  const int n = nuq;
  for (int el = t; el < ne; el += nthr) {
    const int r = el / NZ, j = el - r * NZ;
    int sl = start + r0 + r;
    if (sl >= cap) sl -= cap;
    if (j >= d.rnnz[sl]) continue;
    const int f = d.ridx[(size_t)sl * NZ + j];
    unsigned h = wide_hash(f) & (TS - 1);
    while (keys[h] != f) h = (h + 1) & (TS - 1);
    d.pslot[(int64_t)(r0 + r) * NZ + j] = (uint16_t)sidx[h];
  }
  int32_t* gfeat = d.bfeat + (int64_t)b * EB;
  for (int base = 0; base < n; base += nthr) {  // uniform trip count: every lane reaches the ballot
    const int si = base + t;
    bool win = false;
    int f = 0;
    if (si < n) {
      f = bf[si];
      gfeat[si] = f;
      unsigned h = wide_gslot(f, d.hmask);
      while (true) {
        const int old = atomicCAS(&d.htab[h].x, -1, f);
        if (old == -1) {
          win = true;
          break;
        }
        if (old == f) break;
        h = (h + 1) & d.hmask;
      }
    }
    const unsigned long long mask = __ballot(win);
    if (mask) {
      const int leader = __ffsll((long long)mask) - 1;
      unsigned b0 = 0;
      if (lane == leader) b0 = atomicAdd(&d.cnt[0], (unsigned)__popcll(mask));
      b0 = __shfl(b0, leader, 64);
      if (win) d.uniq[b0 + __popcll(mask & ((1ull << lane) - 1ull))] = f;
    }
  }
  if (t == 0) d.bcount[b] = n;
  __syncthreads();  // the LDS table is reused by the block's next group
}

__global__ __launch_bounds__(256) void wide_plan_kernel(WideCfg c, WideDev d) {
  extern __shared__ __attribute__((aligned(16))) int plan_lds[];
  wide_plan_body(c, d, blockIdx.x, plan_lds);
}

// owner order (pull mode, own_W > 1): per-owner counts of the window's
// features, then every feature scattered to its owner's segment of uniq_alt
// (assign copies it back): the pull and push segments of owner j are then the
// contiguous local ids [off_j, off_j + cnt_j).
__device__ __forceinline__ int wide_owner(const WideCfg& c, int f) {
  const int64_t o = (int64_t)f / c.own_S;
  return o < c.own_W - 1 ? (int)o : c.own_W - 1;
}

__global__ __launch_bounds__(256) void wide_owner_count_kernel(WideCfg c, WideDev d) {
  __shared__ unsigned cnt_s[kMaxOwners];
  const unsigned U = d.cnt[0];
  if (threadIdx.x < kMaxOwners) cnt_s[threadIdx.x] = 0u;
  __syncthreads();
  for (unsigned i = blockIdx.x * 256 + threadIdx.x; i < U; i += gridDim.x * 256) {
    const int f = d.uniq[i];
    atomicAdd(&cnt_s[wide_owner(c, f)], 1u);
    d.uniq_alt[i] = f;
  }
  __syncthreads();
  if (threadIdx.x < c.own_W && cnt_s[threadIdx.x]) atomicAdd(&d.own[threadIdx.x], cnt_s[threadIdx.x]);
}

__global__ __launch_bounds__(256) void wide_owner_scatter_kernel(WideCfg c, WideDev d) {
  __shared__ unsigned base_s[kMaxOwners];
  const unsigned U = d.cnt[0];
  if (threadIdx.x == 0) {
    unsigned o = 0;
    for (int j = 0; j < c.own_W; ++j) {
      base_s[j] = o;
      o += d.own[j];
    }
  }
  __syncthreads();
  unsigned* cur = d.own + kMaxOwners;
  for (unsigned i = blockIdx.x * 256 + threadIdx.x; i < U; i += gridDim.x * 256) {
    const int f = d.uniq_alt[i];
    const int j = wide_owner(c, f);
    d.uniq[base_s[j] + atomicAdd(&cur[j], 1u)] = f;
  }
}

// assign: table entry of every local id, gather the old weights of the
// window's features (the dense pulled vector, or the pulled values in pull mode).
__device__ __forceinline__ void wide_assign_body(const WideCfg& c, const WideDev& d, int blk, int nblk) {
  const unsigned U = d.cnt[0];
  const int KP = c.KP;
  const unsigned nthr = blockDim.x;
  for (unsigned i = blk * nthr + threadIdx.x; i < U; i += nblk * nthr) {
    const int f = d.uniq[i];
    unsigned h = wide_gslot(f, d.hmask);
    while (d.htab[h].x != f) h = (h + 1) & d.hmask;
    d.htab[h].y = (int)i;
    d.hslot[i] = (int)h;
    const float* src = c.pulled ? d.w_pull + (int64_t)i * KP : d.w_old + (int64_t)f * KP;
    float* dst = d.w0 + KP + (int64_t)i * KP;
    for (int k = 0; k < KP; ++k) dst[k] = src[k];
    d.s1[i] = 0.f;
    d.s2[i] = 0.f;
  }
  if (blk == 0 && threadIdx.x < KP)  // intercepts: kept apart (w_pull_b) or after the coefficients
    d.w0[threadIdx.x] = d.w_pull_b ? d.w_pull_b[threadIdx.x] : d.w_old[c.F * KP + threadIdx.x];
}

__global__ __launch_bounds__(256) void wide_assign_kernel(WideCfg c, WideDev d) {
  wide_assign_body(c, d, blockIdx.x, gridDim.x);
}

// stats: local ids of the group's features, every entry's local id, and the
// feature sums for the 1/std scaling aggregated per group in LDS.
__device__ __forceinline__ void wide_stats_body(const WideCfg& c, const WideDev& d, int b, int* st_lds) {
  const int EB = d.EB, RB = d.RB, NZ = c.NZ, cap = c.cap;
  const int nthr = blockDim.x;
  int* lid_s = st_lds;                  // [EB]
  float* s1l = (float*)(lid_s + EB);    // [EB]
  float* s2l = s1l + EB;                // [EB]
  const int B = d.prm->B, start = d.prm->start;
  const int t = threadIdx.x;
  const int r0 = b * RB;
  if (r0 >= B) return;
  const int rows = min(RB, B - r0);
  const int n = d.bcount[b];
  const int32_t* gfeat = d.bfeat + (int64_t)b * EB;
  int32_t* glid = d.blid + (int64_t)b * EB;
  for (int si = t; si < n; si += nthr) {
    const int l = wide_find(d.htab, d.hmask, gfeat[si]);
    lid_s[si] = l;
    glid[si] = l;
    s1l[si] = 0.f;
    s2l[si] = 0.f;
  }
  __syncthreads();
  const int ne = rows * NZ;
  for (int el = t; el < ne; el += nthr) {
    const int r = el / NZ, j = el - r * NZ;
    int sl = start + r0 + r;
    if (sl >= cap) sl -= cap;
    if (j >= d.rnnz[sl]) continue;
    const int64_t e = (int64_t)(r0 + r) * NZ + j;
    const int ps = d.pslot[e];
    d.lid[e] = lid_s[ps];
    if (c.standardize) {
      const float v = bf2f(d.rval[(size_t)sl * NZ + j]);
      atomicAdd(&s1l[ps], v);
      atomicAdd(&s2l[ps], v * v);
    }
  }
  __syncthreads();
  if (c.standardize) {
    for (int si = t; si < n; si += nthr) {
      atomicAdd(&d.s1[lid_s[si]], s1l[si]);
      atomicAdd(&d.s2[lid_s[si]], s2l[si]);
    }
  }
  __syncthreads();  // the block's next group reuses the LDS
}

__global__ __launch_bounds__(256) void wide_stats_kernel(WideCfg c, WideDev d) {
  extern __shared__ __attribute__((aligned(16))) int st_lds[];
  wide_stats_body(c, d, blockIdx.x, st_lds);
}

// prep: per-feature scaling, starting point x, zeroed direction / gradients,
// controller init.
__device__ __forceinline__ void wide_prep_body(const WideCfg& c, const WideDev& d, int blk, int nblk) {
  const unsigned U = d.cnt[0];
  const int KP = c.KP, K = c.K;
  const int B = d.prm->B;
  const int64_t PL = KP + (int64_t)U * KP;
  const int64_t gid = (int64_t)blk * blockDim.x + threadIdx.x, gs = (int64_t)nblk * blockDim.x;
  for (int64_t i = gid; i < U; i += gs) {
    float sc = 1.f, gsc = 1.f, xs = 1.f;
    if (c.standardize) {
      const double n = (double)B;
      double sd = 0.0;
      if (n > 1.0) {
        const double mean = (double)d.s1[i] / n;
        const double var = ((double)d.s2[i] - n * mean * mean) / (n - 1.0);
        sd = var > 0.0 ? sqrt(var) : 0.0;
      }
      if (sd > 0.0) {
        sc = gsc = (float)(1.0 / sd);
        xs = (float)sd;
      } else {
        gsc = 0.f;
        sc = xs = c.zero_const ? 0.f : 1.f;
      }
    }
    d.scale[i] = sc;
    d.gscale[i] = gsc;
    for (int k = 0; k < KP; ++k) {
      const int64_t p = KP + i * KP + k;
      d.x[p] = k < K ? d.w0[p] * xs : 0.f;
    }
  }
  for (int64_t p = gid; p < PL; p += gs) {
    d.d[p] = 0.f;
    d.g_t[p] = 0.f;
    d.g_c[p] = 0.f;
    if (p < KP) d.x[p] = p < K ? d.w0[p] : 0.f;
  }
  if (gid == 0) {
    ctrl_init(*d.ctrl);
    d.ctrl->t = 0.0;
    for (int s = 0; s < c.sc.nslots; ++s) d.loss_acc[s] = 0.0;
  }
}

__global__ __launch_bounds__(256) void wide_prep_kernel(WideCfg c, WideDev d) {
  wide_prep_body(c, d, blockIdx.x, gridDim.x);
}

// ---------------------------------------------------------------------------
// Shared-memory blocks of the slot phases (static in each kernel that runs them).
struct WideFwdShared {
  float red_r[8][16];
  double red_l[8];
};
struct WideDotsShared {
  double red[8][kWideND];
  double dots[kWideND];
  int last;
  CtrlScratch ws;
  Ctrl ctrl;
};

// One function evaluation at x + t d: margins, softmax/CE, gradient.  One
// wavefront per window row, RB rows (one group of the plan) per workgroup; the
// rows' gradient contributions are summed in LDS per distinct feature of the
// group and flushed with one global atomic per (feature, class).
template <int KP, int NQ>
__device__ __forceinline__ void wide_fwdbwd_body(const WideCfg& c, const WideDev& d, int slot, int grp, float* gacc,
                                                 WideFwdShared& sh) {
  const Ctrl* ctrl = d.ctrl;
  const int B = d.prm->B, start = d.prm->start, NZ = c.NZ, cap = c.cap, K = c.K, RB = d.RB;
  const int r0 = grp * RB;
  if (r0 >= B) return;  // uniform per workgroup
  const float t = (float)ctrl->t;
  const float invB = 1.f / (float)B;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nthr = blockDim.x;
  const int n = d.bcount[grp];
  for (int i = threadIdx.x; i < n * KP; i += nthr) gacc[i] = 0.f;
  __syncthreads();
  const float* __restrict__ X = d.x;
  const float* __restrict__ D = d.d;
  float rr[KP];
#pragma unroll
  for (int k = 0; k < KP; ++k) rr[k] = 0.f;
  double lrow = 0.0;
  const int r = r0 + wv;
  if (wv < RB && r < B) {
    int sl = start + r;
    if (sl >= cap) sl -= cap;
    const int nnz = d.rnnz[sl];
    const int64_t e0 = (int64_t)r * NZ;
    const uint16_t* __restrict__ vals = d.rval + (int64_t)sl * NZ;
    float z[KP];
#pragma unroll
    for (int k = 0; k < KP; ++k) z[k] = 0.f;
    int lq[NQ], pq[NQ];
    float vq[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int j = lane + 64 * q;
      lq[q] = -1;
      pq[q] = 0;
      vq[q] = 0.f;
      if (j < nnz) {
        const int l = d.lid[e0 + j];
        const float v = bf2f(vals[j]);
        lq[q] = l;
        pq[q] = d.pslot[e0 + j];
        vq[q] = v;
        const float sv = v * d.scale[l];
        float xv[KP], dv[KP];
        ldk<KP>(X + KP + (int64_t)l * KP, xv);
        ldk<KP>(D + KP + (int64_t)l * KP, dv);
#pragma unroll
        for (int k = 0; k < KP; ++k) z[k] += sv * (xv[k] + t * dv[k]);
      }
    }
#pragma unroll
    for (int k = 0; k < KP; ++k) z[k] = wave_sum(z[k]);
    {
      float xb[KP], db[KP];
      ldk<KP>(X, xb);
      ldk<KP>(D, db);
#pragma unroll
      for (int k = 0; k < KP; ++k) z[k] += xb[k] + t * db[k];
    }
    lrow = (double)row_residual<KP>(z, K, d.ry[sl], invB, rr);
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      if (lq[q] < 0) continue;
      const float g = vq[q] * d.gscale[lq[q]];
      if (g == 0.f) continue;
      float* gp = gacc + pq[q] * KP;
#pragma unroll
      for (int k = 0; k < KP; ++k)
        if (k < K) atomicAdd(gp + k, g * rr[k]);
    }
  }
  if (lane == 0 && wv < 8) {
#pragma unroll
    for (int k = 0; k < KP; ++k) sh.red_r[wv][k] = rr[k];
    sh.red_l[wv] = lrow;
  }
  __syncthreads();
  const int nw = nthr >> 6;
  if (threadIdx.x < KP && threadIdx.x < K) {
    float sr = 0.f;
    for (int w = 0; w < nw; ++w) sr += sh.red_r[w][threadIdx.x];
    if (sr != 0.f) atomicAdd(d.g_t + threadIdx.x, sr);
  }
  if (threadIdx.x == 0) {
    double sl = 0.0;
    for (int w = 0; w < nw; ++w) sl += sh.red_l[w];
    if (sl != 0.0) atomicAdd(d.loss_acc + slot, sl);
  }
  const int32_t* glid = d.blid + (int64_t)grp * d.EB;
  for (int i = threadIdx.x; i < n * K; i += nthr) {
    const int si = i / K, k = i - si * K;
    const float v = gacc[si * KP + k];
    if (v != 0.f) atomicAdd(d.g_t + KP + (int64_t)glid[si] * KP + k, v);
  }
  __syncthreads();  // gacc is reused by the workgroup's next group
}

template <int KP, int NQ>
__global__ __launch_bounds__(512) void wide_fwdbwd_kernel(WideCfg c, WideDev d, int slot) {
  extern __shared__ __attribute__((aligned(16))) float gacc[];  // [EB][KP]
  __shared__ WideFwdShared sh;
  if (d.ctrl->phase == kPhDone) return;
  wide_fwdbwd_body<KP, NQ>(c, d, slot, blockIdx.x, gacc, sh);
}

// Dot products of the new gradient (ctrl dots layout, solver_ctrl.h) + the
// controller step in the last-arriving workgroup (of nblk; workgroup `blk`).
__device__ __forceinline__ void wide_dots_body(const WideCfg& c, const WideDev& d, int slot, int blk, int nblk,
                                               WideDotsShared& sh) {
  Ctrl* ctrl = d.ctrl;
  static_assert(sizeof(Ctrl) % 8 == 0, "Ctrl is copied as 64-bit words");
  const int H = c.sc.hist;
  const int m = ctrl->m;
  const unsigned U = d.cnt[0];
  const int nthr = blockDim.x, nw = nthr >> 6;
  const int64_t PL = c.KP + (int64_t)U * c.KP, PLmax = d.PLmax;
  long long* stp = d.dbg ? d.dbg + slot * 8 : nullptr;
  if (stp && blk == 0 && threadIdx.x == 0) stp[0] = (long long)__builtin_amdgcn_s_memrealtime();
  double a0 = 0.0, a1 = 0.0, a2 = 0.0;
  double aS[kMaxHist], aY[kMaxHist];
#pragma unroll
  for (int i = 0; i < kMaxHist; ++i) aS[i] = aY[i] = 0.0;
  for (int64_t p = (int64_t)blk * nthr + threadIdx.x; p < PL; p += (int64_t)nblk * nthr) {
    const float g = d.g_t[p];
    a0 += (double)g * g;
    a1 += (double)g * d.d[p];
    a2 += (double)g * d.g_c[p];
#pragma unroll
    for (int i = 0; i < kMaxHist; ++i) {
      if (i < m) {
        aS[i] += (double)g * d.S[(int64_t)i * PLmax + p];
        aY[i] += (double)g * d.Y[(int64_t)i * PLmax + p];
      }
    }
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  a0 = wave_sum(a0);
  a1 = wave_sum(a1);
  a2 = wave_sum(a2);
  if (lane == 0) {
    sh.red[wv][0] = a0;
    sh.red[wv][1] = a1;
    sh.red[wv][2] = a2;
  }
#pragma unroll
  for (int i = 0; i < kMaxHist; ++i) {
    if (i < m) {
      const double s = wave_sum(aS[i]);
      const double y = wave_sum(aY[i]);
      if (lane == 0) {
        sh.red[wv][3 + i] = s;
        sh.red[wv][3 + H + i] = y;
      }
    }
  }
  __syncthreads();
  const int nd = 3 + 2 * H;
  if (threadIdx.x < nd) {
    const int k = threadIdx.x;
    const bool used = k < 3 || (k < 3 + H ? k - 3 < m : k - 3 - H < m);
    double s = 0.0;
    if (used)
      for (int w = 0; w < nw; ++w) s += sh.red[w][k];
    // write-through hand-off: agent-scope stores, drained before the ticket,
    // agent-scope loads by the last workgroup -- no L2 writeback fence
    __hip_atomic_store((gu64w*)(d.part + (int64_t)blk * kWideND + k), __builtin_bit_cast(unsigned long long, s),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0)
    sh.last = __hip_atomic_fetch_add(&d.cnt[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)nblk - 1;
  __syncthreads();
  if (!sh.last) return;
  if (stp && threadIdx.x == 0) stp[1] = (long long)__builtin_amdgcn_s_memrealtime();
  // thread b loads workgroup b's partials -- only the dots the controller
  // reads (3 + 2m of them), all loads in flight together -- then one wave
  // reduction per dot in a fixed order (deterministic)
  double v[kWideND];
#pragma unroll
  for (int k = 0; k < kWideND; ++k) {
    const bool used = k < nd && (k < 3 || (k < 3 + H ? k - 3 < m : k - 3 - H < m));
    v[k] = (used && threadIdx.x < nblk) ? ld_agent_f64(d.part + (int64_t)threadIdx.x * kWideND + k) : 0.0;
  }
#pragma unroll
  for (int k = 0; k < kWideND; ++k) {
    const bool used = k < nd && (k < 3 || (k < 3 + H ? k - 3 < m : k - 3 - H < m));
    if (used) {  // uniform across the block
      const double w = wave_sum(v[k]);
      if (lane == 0) sh.red[wv][k] = w;
    }
  }
  __syncthreads();
  if (threadIdx.x < nd) {
    const int k = threadIdx.x;
    const bool used = k < 3 || (k < 3 + H ? k - 3 < m : k - 3 - H < m);
    double s = 0.0;
    if (used)
      for (int w = 0; w < nw; ++w) s += sh.red[w][k];
    sh.dots[k] = s;
  }
  __syncthreads();
  if (stp && threadIdx.x == 0) stp[2] = (long long)__builtin_amdgcn_s_memrealtime();
  // the controller is a single thread doing dependent scalar work: run it on
  // an LDS copy of the state (an L2 round trip per access otherwise)
  constexpr int kCW = (int)(sizeof(Ctrl) / 8);
  unsigned long long* cg = reinterpret_cast<unsigned long long*>(ctrl);
  unsigned long long* cs = reinterpret_cast<unsigned long long*>(&sh.ctrl);
  {  // all of a thread's words in flight before its first store (nthr >= 256)
    constexpr int kPer = (kCW + 255) / 256;
    unsigned long long cv[kPer];
#pragma unroll
    for (int c2 = 0; c2 < kPer; ++c2) {
      const int i = (int)threadIdx.x + nthr * c2;
      cv[c2] = i < kCW ? cg[i] : 0ull;
    }
#pragma unroll
    for (int c2 = 0; c2 < kPer; ++c2) {
      const int i = (int)threadIdx.x + nthr * c2;
      if (i < kCW) cs[i] = cv[c2];
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    if (stp) stp[3] = (long long)__builtin_amdgcn_s_memrealtime();
    __hip_atomic_store(&d.cnt[1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const double f = ld_agent_f64(d.loss_acc + slot) / (double)d.prm->B;
    ctrl_step(sh.ctrl, c.sc, f, sh.dots, slot, sh.ws);
    if (stp) stp[4] = (long long)__builtin_amdgcn_s_memrealtime();
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kCW; i += nthr) cg[i] = cs[i];
  if (stp && threadIdx.x == 0) stp[5] = (long long)__builtin_amdgcn_s_memrealtime();
}

__global__ __launch_bounds__(256) void wide_dots_kernel(WideCfg c, WideDev d, int slot) {
  __shared__ WideDotsShared sh;
  if (d.ctrl->phase == kPhDone) return;
  wide_dots_body(c, d, slot, blockIdx.x, gridDim.x, sh);
}

// Apply the controller's decision of `slot` to the local vectors; clears g_t
// for the next evaluation.
__device__ __forceinline__ void wide_apply_body(const WideCfg& c, const WideDev& d, int slot, int blk, int nblk) {
  const Ctrl* ctrl = d.ctrl;
  if (ctrl->action_slot != slot) return;
  const int act = ctrl->action;
  if (act == kActDone) return;
  const unsigned U = d.cnt[0];
  const int nthr = blockDim.x;
  const int64_t PL = c.KP + (int64_t)U * c.KP, PLmax = d.PLmax;
  const float ta = (float)ctrl->t_acc;
  const int ps = ctrl->push_slot;
  const int m = ctrl->m;
  const float cg = (float)ctrl->cg;
  float cs[kMaxHist], cy[kMaxHist];
#pragma unroll
  for (int i = 0; i < kMaxHist; ++i) {
    cs[i] = i < m ? (float)ctrl->cs[i] : 0.f;
    cy[i] = i < m ? (float)ctrl->cy[i] : 0.f;
  }
  for (int64_t p = (int64_t)blk * nthr + threadIdx.x; p < PL; p += (int64_t)nblk * nthr) {
    const float gt = d.g_t[p];
    d.g_t[p] = 0.f;
    if (act == kActInit) {
      d.g_c[p] = gt;
      d.d[p] = -gt;
    } else if (act == kActAccept || act == kActAcceptDone) {
      const float dp = d.d[p];
      d.x[p] += ta * dp;
      if (act == kActAccept) {
        if (ps >= 0) {
          d.S[(int64_t)ps * PLmax + p] = ta * dp;
          d.Y[(int64_t)ps * PLmax + p] = gt - d.g_c[p];
        }
        d.g_c[p] = gt;
        float nd = cg * gt;
#pragma unroll
        for (int i = 0; i < kMaxHist; ++i)
          if (i < m) nd += cs[i] * d.S[(int64_t)i * PLmax + p] + cy[i] * d.Y[(int64_t)i * PLmax + p];
        d.d[p] = nd;
      }
    }
  }
}

__global__ __launch_bounds__(256) void wide_apply_kernel(WideCfg c, WideDev d, int slot) {
  wide_apply_body(c, d, slot, blockIdx.x, gridDim.x);
}

// ---------------------------------------------------------------------------
// wide_tail_kernel: the line-search retry slots [s0, s1) in ONE persistent
// launch.  The usual solve is over after 1 + iters evaluations (every line
// search accepts its first trial), so this launch exits at once; otherwise each
// slot runs fwdbwd -> grid barrier -> dots + controller -> grid barrier ->
// apply -> grid barrier, instead of three mostly-empty launches per budgeted
// slot.  Grid <= 64 workgroups of 512 threads: co-resident on 256 CUs.
// Barrier: every wave drains its stores, lane 0 releases at agent scope,
// arrives on a monotone counter and polls it (agent-scope loads), acquires.
__device__ __forceinline__ void wide_grid_barrier(unsigned long long* ctr, unsigned long long target,
                                                  unsigned* err) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    (void)__hip_atomic_fetch_add(ctr, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int spins = 0;
    while (__hip_atomic_load((gu64w*)ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > (1 << 24)) {  // never expected: a workgroup was not co-resident
        __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
}

template <int KP, int NQ>
__global__ __launch_bounds__(512) void wide_tail_kernel(WideCfg c, WideDev d, int s0, int s1) {
  extern __shared__ __attribute__((aligned(16))) float gacc[];  // [EB][KP]
  __shared__ WideFwdShared fsh;
  __shared__ WideDotsShared dsh;
  __shared__ int phase_s;
  const int G = gridDim.x;
  unsigned long long nb = 0;
  for (int slot = s0; slot < s1; ++slot) {
    if (threadIdx.x == 0)
      phase_s = __hip_atomic_load(&d.ctrl->phase, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    if (phase_s == kPhDone) break;  // uniform: every workgroup read the word after the last barrier
    const int B = d.prm->B;
    for (int grp = blockIdx.x; grp * d.RB < B; grp += G) wide_fwdbwd_body<KP, NQ>(c, d, slot, grp, gacc, fsh);
    wide_grid_barrier(d.gbar, (unsigned long long)G * ++nb, d.cnt + 3);
    wide_dots_body(c, d, slot, blockIdx.x, G, dsh);
    wide_grid_barrier(d.gbar, (unsigned long long)G * ++nb, d.cnt + 3);
    wide_apply_body(c, d, slot, blockIdx.x, G);
    wide_grid_barrier(d.gbar, (unsigned long long)G * ++nb, d.cnt + 3);
  }
}

// finalize: effective coefficients, centring, local delta (+ dense scatter).
__device__ __forceinline__ void wide_finalize_body(const WideCfg& c, const WideDev& d, int blk, int nblk) {
  const unsigned U = d.cnt[0];
  const int KP = c.KP, K = c.K;
  const int64_t gid = (int64_t)blk * blockDim.x + threadIdx.x;
  for (int64_t i = gid; i <= (int64_t)U; i += (int64_t)nblk * blockDim.x) {
    // i < U: feature i ; i == U: the intercepts
    const bool icpt = i == (int64_t)U;
    const int64_t p0 = icpt ? 0 : KP + i * KP;
    const float sc = icpt ? 1.f : d.scale[i];
    float v[16];
    float mean = 0.f;
    for (int k = 0; k < KP; ++k) {
      v[k] = k < K ? sc * d.x[p0 + k] : 0.f;
      mean += v[k];
    }
    if (c.center && K >= 2) {
      mean /= (float)K;
      for (int k = 0; k < K; ++k) v[k] -= mean;
    }
    const int64_t dst = icpt ? c.F * KP : (int64_t)d.uniq[i] * KP;
    for (int k = 0; k < KP; ++k) {
      const float dl = k < K ? v[k] - d.w0[p0 + k] : 0.f;
      d.wloc[p0 + k] = k < K ? v[k] : 0.f;
      d.dloc[p0 + k] = dl;
      if (c.dense_delta) d.delta_dense[dst + k] = dl;
    }
  }
  if (gid == 0) {
    const Ctrl* ctrl = d.ctrl;
    *d.loss = (float)ctrl->f_c;
    d.stats[0] = ctrl->evals;
    d.stats[1] = ctrl->nacc;
    d.stats[2] = ctrl->ls_fail;
    d.stats[3] = ctrl->dir_reset;
    // a grid barrier that timed out (a workgroup was not co-resident): sticky flag
    // for the host, NaN loss in the logs
    const unsigned err = __hip_atomic_load(d.cnt + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (err) {
      d.stats[4] |= (int)err;
      __hip_atomic_store(d.cnt + 3, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *d.loss = __builtin_nanf("");
    }
    d.cnt[2] = U;
    // read by the host after a stream synchronisation: no release (an L2 writeback) needed
    if (d.host_u) __hip_atomic_store(d.host_u, U, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

__global__ __launch_bounds__(256) void wide_finalize_kernel(WideCfg c, WideDev d) {
  wide_finalize_body(c, d, blockIdx.x, gridDim.x);
}

// ---------------------------------------------------------------------------
// wide_persist_kernel: the whole solve (or, in pull mode, its second phase) in
// ONE launch of co-resident workgroups, the phases separated by a
// self-resetting grid barrier (arrival count + generation word: the last
// arriver zeroes the count and bumps the generation, the others poll the
// generation).  On MI355X a kernel boundary of the launch chain costs ~4.5-5 us
// of device time even for an empty phase (profiles/r03_v4), a barrier ~2-3 us.
// phases: bit 0 = begin + plan, bit 1 = assign .. finalize.
// xl (XCD-local): every party runs on ONE XCD and shares its L2 -- the drained stores
// have reached that L2 through the write-through L1, so the release (an L2 write-back
// of the XCD's dirty lines, 1.7-6.5 us, MI355X_MICROARCH.md) is skipped; the acquire
// (this CU's L1 invalidated) stays.
__device__ __forceinline__ void wide_gen_barrier(unsigned* bar, unsigned G, unsigned* err, bool xl = false) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned g = __hip_atomic_load(bar + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (!xl) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned old = __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old == G - 1) {
      __hip_atomic_store(bar, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      (void)__hip_atomic_fetch_add(bar + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      int spins = 0;
      while (__hip_atomic_load(bar + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == g) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > (1 << 24)) {  // never expected: a workgroup was not co-resident
          __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
}

// The persistent solve's phases for workgroup blk of G (the whole grid of
// wide_persist_kernel, or one lane's XCD in wide_lanes_kernel).
template <int KP, int NQ>
__device__ __forceinline__ void wide_persist_body(const WideCfg& c, const WideDev& d, int B, int start, int phases,
                                                  int G, int blk, int* pl_lds, WideFwdShared& fsh,
                                                  WideDotsShared& dsh, int& phase_s, bool xl = false) {
  const int ngr = (c.cap + d.RB - 1) / d.RB;
  unsigned* err = d.cnt + 3;
  // PSX_WIDE_STAMPS: [7] the body's entry, [slot * 8 + 6] slot's forward begins, [15] finalize
  // (next to wide_dots_body's [slot * 8 + 0..5]; nslots >= 2 in every configuration)
  const bool st = d.dbg && blk == 0 && threadIdx.x == 0;
  if (st) d.dbg[7] = (long long)__builtin_amdgcn_s_memrealtime();
  if (phases & 1) {
    wide_begin_body(d, B, start, blk, G);
    wide_gen_barrier(d.pbar, G, err, xl);
    for (int grp = blk; grp < ngr; grp += G) wide_plan_body(c, d, grp, pl_lds);
    wide_gen_barrier(d.pbar, G, err, xl);
  }
  // (stamps of the prefix's phases, where nslots >= 6: [23] planned, [31] assigned,
  // [39] window statistics, [47] prepared)
  const bool stp = st && c.sc.nslots >= 6;
  if (stp) d.dbg[23] = (long long)__builtin_amdgcn_s_memrealtime();
  if (!(phases & 2)) return;
  wide_assign_body(c, d, blk, G);
  wide_gen_barrier(d.pbar, G, err, xl);
  if (stp) d.dbg[31] = (long long)__builtin_amdgcn_s_memrealtime();
  for (int grp = blk; grp < ngr; grp += G) wide_stats_body(c, d, grp, pl_lds);
  wide_gen_barrier(d.pbar, G, err, xl);
  if (stp) d.dbg[39] = (long long)__builtin_amdgcn_s_memrealtime();
  wide_prep_body(c, d, blk, G);
  wide_gen_barrier(d.pbar, G, err, xl);
  if (stp) d.dbg[47] = (long long)__builtin_amdgcn_s_memrealtime();
  for (int slot = 0; slot < c.sc.nslots; ++slot) {
    if (threadIdx.x == 0)
      phase_s = __hip_atomic_load(&d.ctrl->phase, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    if (phase_s == kPhDone) break;  // uniform: every workgroup read the word after the last barrier
    const int Bw = d.prm->B;
    if (st) d.dbg[slot * 8 + 6] = (long long)__builtin_amdgcn_s_memrealtime();
    for (int grp = blk; grp * d.RB < Bw; grp += G) wide_fwdbwd_body<KP, NQ>(c, d, slot, grp, (float*)pl_lds, fsh);
    wide_gen_barrier(d.pbar, G, err, xl);
    wide_dots_body(c, d, slot, blk, G, dsh);
    wide_gen_barrier(d.pbar, G, err, xl);
    wide_apply_body(c, d, slot, blk, G);
    wide_gen_barrier(d.pbar, G, err, xl);
  }
  if (st && c.sc.nslots >= 2) d.dbg[15] = (long long)__builtin_amdgcn_s_memrealtime();
  wide_finalize_body(c, d, blk, G);
}

template <int KP, int NQ>
__global__ __launch_bounds__(512) void wide_persist_kernel(WideCfg c, WideDev d, int B, int start, int phases) {
  extern __shared__ __attribute__((aligned(16))) int pl_lds[];
  __shared__ WideFwdShared fsh;
  __shared__ WideDotsShared dsh;
  __shared__ int phase_s;
  wide_persist_body<KP, NQ>(c, d, B, start, phases, (int)gridDim.x, (int)blockIdx.x, pl_lds, fsh, dsh, phase_s);
}

// wide_lanes_kernel: up to 8 workers' persistent solves in one launch, lane l on
// XCD xcd0 + l.  Two workers' separate persistent launches deadlock (each waits for
// CUs the other's workgroups hold: the dispatcher places a launch's workgroups in
// order, profiles/r02_v5), and the launch chain is ~14 kernels per solve on the
// workers' streams, which HIP's 4 hardware queues serialise pairwise
// (profiles/r06/README.md section 7).  One launch of 8 x 32 workgroups instead: a
// workgroup claims the next of the 32 slots of its XCD's lane, so the lane's grid
// barriers and dot-product tickets stay inside one L2, and surplus workgroups
// (an XCD dealt more than 32, or no lane) leave at once.
template <int KP, int NQ>
__global__ __launch_bounds__(512) void wide_lanes_kernel(WideCfg c, const WideDev* __restrict__ devs,
                                                         WideLanesArgs a) {
  extern __shared__ __attribute__((aligned(16))) int pl_lds[];
  __shared__ WideFwdShared fsh;
  __shared__ WideDotsShared dsh;
  __shared__ int phase_s;
  __shared__ int role_s;
  if (threadIdx.x == 0) {
    // the other parity's counters (the previous launch, complete in stream order) for the next launch
    if (blockIdx.x < 16)
      __hip_atomic_store(a.claim + 16 * (a.cpar ^ 1) + blockIdx.x, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int xcc = (int)(__builtin_amdgcn_s_getreg((3 << 11) | 20) & 15u);  // HW_REG_XCC_ID
    const int lx = xcc - a.xcd0;
    const int G = a.gpx * a.per;
    int r = -1;
    if (lx >= 0 && lx < a.L * a.per) {
      const int lane = lx / a.per;
      const unsigned k = __hip_atomic_fetch_add(a.claim + 16 * a.cpar + lane, 1u, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
      if (k < (unsigned)G) r = lane * G + (int)k;
    }
    role_s = r;
  }
  __syncthreads();
  const int r = __builtin_amdgcn_readfirstlane(role_s);
  if (r < 0) return;
  // (a lane over several XCDs: its barriers and tickets are agent-scope atomics and its
  // hand-offs agent-scope fences, coherent across the XCDs' L2s)
  const int G = a.gpx * a.per;
  const int l = r / G, blk = r - l * G;
  // the lane's window: constant-index reads of the kernel argument (a runtime index
  // would copy the argument block into scratch, lanes_body.h pick())
  int B = a.B[0], start = a.start[0];
#pragma unroll
  for (int i = 1; i < kWideMaxLanes; ++i)
    if (l == i) {
      B = a.B[i];
      start = a.start[i];
    }
  const WideDev& d = devs[l];
  wide_persist_body<KP, NQ>(c, d, B, start, 3, G, blk, pl_lds, fsh, dsh, phase_s, a.per == 1);
  if (a.pres) {
    // the lane's rows of the evaluation's overlay table: the same thread-to-feature map as
    // wide_finalize_body's, so every thread reads back the wloc rows it has just written
    const unsigned U = d.cnt[0];
    const int64_t gs = (int64_t)G * blockDim.x;
    for (int64_t i = (int64_t)blk * blockDim.x + threadIdx.x; i < (int64_t)U; i += gs) {
      const int f = d.uniq[i];
      float* dst = a.ov + ((int64_t)f * kWideMaxLanes + l) * KP;
      const float* src = d.wloc + KP + i * KP;
#pragma unroll
      for (int k = 0; k < KP; ++k) dst[k] = src[k];
      a.lidt[(int64_t)f * kWideMaxLanes + l] = (int)i;
      atomicOr(a.pres + f, 1u << l);
    }
  }
}

// ---------------------------------------------------------------------------
static int grid_for(int64_t n, int cap_blocks) {
  int64_t g = (n + 255) / 256;
  if (g < 1) g = 1;
  if (g > cap_blocks) g = cap_blocks;
  return (int)g;
}

int wide_dots_blocks(int64_t PLmax) { return grid_for(PLmax / 4, 256); }  // <= 256: one partial per thread

void wide_launch_begin(const WideCfg& c, const WideDev& d, int B, int start, hipStream_t s) {
  wide_begin_kernel<<<grid_for(c.umax, 1024), 256, 0, s>>>(d, B, start);
}

int wide_rows_per_group(int NZ, int KP) {
  int rb = 8;
  while (rb > 1 && (rb * NZ > 2048 || rb * NZ * KP * 4 > 64512)) --rb;  // + static LDS < 64 KiB
  return rb;
}

static int ngroups(const WideCfg& c, const WideDev& d) { return (c.cap + d.RB - 1) / d.RB; }

void wide_launch_plan(const WideCfg& c, const WideDev& d, hipStream_t s) {
  wide_plan_kernel<<<ngroups(c, d), 256, (size_t)(2 * d.TS + d.EB) * 4, s>>>(c, d);
  if (c.pulled && c.own_W > 1) {
    wide_owner_count_kernel<<<grid_for(c.umax, 1024), 256, 0, s>>>(c, d);
    wide_owner_scatter_kernel<<<grid_for(c.umax, 1024), 256, 0, s>>>(c, d);
  }
}

void wide_launch_prepare(const WideCfg& c, const WideDev& d, hipStream_t s) {
  const int G = ngroups(c, d);
  wide_assign_kernel<<<grid_for(c.umax, 1024), 256, 0, s>>>(c, d);
  wide_stats_kernel<<<G, 256, (size_t)d.EB * 12, s>>>(c, d);
  wide_prep_kernel<<<grid_for(d.PLmax, 1024), 256, 0, s>>>(c, d);
}

template <int KP>
static void launch_fwdbwd_kp(const WideCfg& c, const WideDev& d, int slot, int grid, hipStream_t s) {
  const int nq = (c.NZ + 63) / 64;
  const int thr = 64 * d.RB;
  const size_t lds = (size_t)d.EB * KP * 4;
  if (nq <= 1)
    wide_fwdbwd_kernel<KP, 1><<<grid, thr, lds, s>>>(c, d, slot);
  else if (nq <= 2)
    wide_fwdbwd_kernel<KP, 2><<<grid, thr, lds, s>>>(c, d, slot);
  else if (nq <= 4)
    wide_fwdbwd_kernel<KP, 4><<<grid, thr, lds, s>>>(c, d, slot);
  else
    wide_fwdbwd_kernel<KP, 8><<<grid, thr, lds, s>>>(c, d, slot);
}

void wide_launch_slot(const WideCfg& c, const WideDev& d, int slot, int nblk_dots, hipStream_t s) {
  const int rows_grid = ngroups(c, d);  // one workgroup per group of RB rows
  switch (c.KP) {
    case 1: launch_fwdbwd_kp<1>(c, d, slot, rows_grid, s); break;
    case 2: launch_fwdbwd_kp<2>(c, d, slot, rows_grid, s); break;
    case 4: launch_fwdbwd_kp<4>(c, d, slot, rows_grid, s); break;
    case 8: launch_fwdbwd_kp<8>(c, d, slot, rows_grid, s); break;
    default: launch_fwdbwd_kp<16>(c, d, slot, rows_grid, s); break;
  }
  wide_dots_kernel<<<nblk_dots, 256, 0, s>>>(c, d, slot);
  wide_apply_kernel<<<grid_for(d.PLmax, 1024), 256, 0, s>>>(c, d, slot);
}

int wide_tail_grid(const WideCfg& c, const WideDev& d) {
  const int g = ngroups(c, d);
  return g < 64 ? g : 64;
}

template <int KP>
static void launch_tail_kp(const WideCfg& c, const WideDev& d, int s0, int s1, hipStream_t s) {
  const int nq = (c.NZ + 63) / 64;
  const int G = wide_tail_grid(c, d);
  const size_t lds = (size_t)d.EB * KP * 4;
  if (nq <= 1)
    wide_tail_kernel<KP, 1><<<G, 512, lds, s>>>(c, d, s0, s1);
  else if (nq <= 2)
    wide_tail_kernel<KP, 2><<<G, 512, lds, s>>>(c, d, s0, s1);
  else if (nq <= 4)
    wide_tail_kernel<KP, 4><<<G, 512, lds, s>>>(c, d, s0, s1);
  else
    wide_tail_kernel<KP, 8><<<G, 512, lds, s>>>(c, d, s0, s1);
}

void wide_launch_tail(const WideCfg& c, const WideDev& d, int s0, int s1, hipStream_t s) {
  switch (c.KP) {
    case 1: launch_tail_kp<1>(c, d, s0, s1, s); break;
    case 2: launch_tail_kp<2>(c, d, s0, s1, s); break;
    case 4: launch_tail_kp<4>(c, d, s0, s1, s); break;
    case 8: launch_tail_kp<8>(c, d, s0, s1, s); break;
    default: launch_tail_kp<16>(c, d, s0, s1, s); break;
  }
}

template <int KP, int NQ>
static void set_tail_attr() {
  (void)hipFuncSetAttribute((const void*)wide_tail_kernel<KP, NQ>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            96 * 1024);
}
template <int KP, int NQ>
static void set_persist_attr() {
  (void)hipFuncSetAttribute((const void*)wide_persist_kernel<KP, NQ>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            96 * 1024);
}
template <int KP>
static void set_tail_attr_kp() {
  set_tail_attr<KP, 1>();
  set_tail_attr<KP, 2>();
  set_tail_attr<KP, 4>();
  set_tail_attr<KP, 8>();
  set_persist_attr<KP, 1>();
  set_persist_attr<KP, 2>();
  set_persist_attr<KP, 4>();
  set_persist_attr<KP, 8>();
}
void wide_prepare_kernels() {
  static bool done = false;
  if (done) return;
  set_tail_attr_kp<1>();
  set_tail_attr_kp<2>();
  set_tail_attr_kp<4>();
  set_tail_attr_kp<8>();
  set_tail_attr_kp<16>();
  done = true;
}

size_t wide_persist_lds(const WideCfg& c, const WideDev& d) {
  const size_t plan = (size_t)(2 * d.TS + d.EB) * 4, stats = (size_t)d.EB * 12, fb = (size_t)d.EB * c.KP * 4;
  size_t m = plan > stats ? plan : stats;
  return m > fb ? m : fb;
}

int wide_persist_grid() { return 256; }

template <int KP>
static void launch_persist_kp(const WideCfg& c, const WideDev& d, int B, int start, int phases, hipStream_t s) {
  const int nq = (c.NZ + 63) / 64;
  const size_t lds = wide_persist_lds(c, d);
  const int G = wide_persist_grid();
  if (nq <= 1)
    wide_persist_kernel<KP, 1><<<G, 512, lds, s>>>(c, d, B, start, phases);
  else if (nq <= 2)
    wide_persist_kernel<KP, 2><<<G, 512, lds, s>>>(c, d, B, start, phases);
  else if (nq <= 4)
    wide_persist_kernel<KP, 4><<<G, 512, lds, s>>>(c, d, B, start, phases);
  else
    wide_persist_kernel<KP, 8><<<G, 512, lds, s>>>(c, d, B, start, phases);
}

void wide_launch_persist(const WideCfg& c, const WideDev& d, int B, int start, int phases, hipStream_t s) {
  switch (c.KP) {
    case 1: launch_persist_kp<1>(c, d, B, start, phases, s); break;
    case 2: launch_persist_kp<2>(c, d, B, start, phases, s); break;
    case 4: launch_persist_kp<4>(c, d, B, start, phases, s); break;
    case 8: launch_persist_kp<8>(c, d, B, start, phases, s); break;
    default: launch_persist_kp<16>(c, d, B, start, phases, s); break;
  }
}

// 8 XCDs x 32 lanes' workgroups, twice over: an XCD the dispatcher deals fewer than
// 32 of the first 256 still gets its lane's 32 (the surplus leaves at once)
int wide_lanes_grid(int gpx) { return 2 * 8 * gpx; }

__global__ __launch_bounds__(256) void wide_lanes_bitmap_kernel(const WideDev* __restrict__ devs, int L, unsigned* bm,
                                                                int64_t nw) {
  for (int l = 0; l < L; ++l) {
    const WideDev& d = devs[l];
    const unsigned U = d.cnt[0];
    unsigned* b = bm + (int64_t)l * nw;
    for (unsigned i = blockIdx.x * 256 + threadIdx.x; i < U; i += gridDim.x * 256) {
      const unsigned f = (unsigned)d.uniq[i];
      atomicOr(b + (f >> 5), 1u << (f & 31));
    }
  }
}

// blockIdx.y = lane.  set: lane l's row of every window feature f (and its local id) into
// the table, bit l into pres[f]; clear: pres[f] = 0.
__global__ __launch_bounds__(256) void wide_lanes_overlay_kernel(const WideDev* __restrict__ devs, int KP,
                                                                 unsigned* pres, float* ov, int* lidt, int set) {
  const int l = (int)blockIdx.y;
  const WideDev& d = devs[l];
  const unsigned U = d.cnt[0];
  for (unsigned i = blockIdx.x * 256 + threadIdx.x; i < U; i += gridDim.x * 256) {
    const int f = d.uniq[i];
    if (set) {
      float* dst = ov + ((int64_t)f * kWideMaxLanes + l) * KP;
      const float* src = d.wloc + KP + (int64_t)i * KP;
      if (KP % 4 == 0) {
        for (int k = 0; k < KP; k += 4) *(float4*)(dst + k) = *(const float4*)(src + k);
      } else {
        for (int k = 0; k < KP; ++k) dst[k] = src[k];
      }
      lidt[(int64_t)f * kWideMaxLanes + l] = (int)i;
      atomicOr(pres + f, 1u << l);
    } else {
      pres[f] = 0u;
    }
  }
}

void wide_lanes_overlay(const WideDev* devs, int L, int KP, unsigned* pres, float* ov, int* lidt, bool set,
                        hipStream_t s) {
  wide_lanes_overlay_kernel<<<dim3(128, (unsigned)L), 256, 0, s>>>(devs, KP, pres, ov, lidt, set ? 1 : 0);
}

// The lanes' sparse pushes in ONE launch, in the order `ord` (= one launch per push in that
// order, bit for bit): every window feature is updated by ONE thread -- the one of the lowest
// lane holding it (pres bits) -- which adds the lanes' deltas in `ord`, then clears pres[f];
// the intercepts by one thread per class.  w[f * KP + c] += lr * dloc_j[KP + lid * KP + c].
__global__ __launch_bounds__(256) void wide_lanes_apply_kernel(const WideDev* __restrict__ devs, WideLanesOrder o,
                                                               int64_t F, int KP, float* w, float lr, unsigned* pres,
                                                               const int* __restrict__ lidt) {
  const int l = (int)blockIdx.y;
  const WideDev& d = devs[l];
  const unsigned U = d.cnt[0];
  for (unsigned i = blockIdx.x * 256 + threadIdx.x; i < U; i += gridDim.x * 256) {
    const int f = d.uniq[i];
    const unsigned bits = pres[f];
    if (bits == 0u || (int)__builtin_ctz(bits) != l) continue;  // another lane's thread owns f
    float* wf = w + (int64_t)f * KP;
    float acc[16];  // (constant indices only: registers)
#pragma unroll
    for (int k = 0; k < 16; ++k) acc[k] = k < KP ? wf[k] : 0.f;
#pragma unroll
    for (int q = 0; q < kWideMaxLanes; ++q) {
      if (q < o.n) {
        const int j = o.ord[q];
        if ((bits >> j) & 1u) {
          const int li = lidt[(int64_t)f * kWideMaxLanes + j];
          const float* dl = devs[j].dloc + KP + (int64_t)li * KP;
#pragma unroll
          for (int k = 0; k < 16; ++k)
            if (k < KP) acc[k] += lr * dl[k];
        }
      }
    }
#pragma unroll
    for (int k = 0; k < 16; ++k)
      if (k < KP) wf[k] = acc[k];
    pres[f] = 0u;
  }
  if (l == 0 && blockIdx.x == 0 && (int)threadIdx.x < KP) {  // the intercepts
    float b = w[F * KP + threadIdx.x];
#pragma unroll
    for (int q = 0; q < kWideMaxLanes; ++q)
      if (q < o.n) b += lr * devs[o.ord[q]].dloc[threadIdx.x];
    w[F * KP + threadIdx.x] = b;
  }
}

void wide_lanes_apply(const WideDev* devs, int L, const WideLanesOrder& o, int64_t F, int KP, float* w, float lr,
                      unsigned* pres, const int* lidt, hipStream_t s) {
  wide_lanes_apply_kernel<<<dim3(128, (unsigned)L), 256, 0, s>>>(devs, o, F, KP, w, lr, pres, lidt);
}

void wide_lanes_bitmap(const WideDev* devs, int L, unsigned* bm, int64_t nw, hipStream_t s) {
  wide_lanes_bitmap_kernel<<<256, 256, 0, s>>>(devs, L, bm, nw);
}

template <int KP, int NQ>
static int lanes_per_cu_kp(size_t lds) {
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, (const void*)wide_lanes_kernel<KP, NQ>, 512, lds) != hipSuccess)
    return 1;
  return n >= 2 ? 2 : 1;
}

int wide_lanes_per_cu(const WideCfg& c, size_t lds) {
  const int nq = (c.NZ + 63) / 64;
#define PSX_OCC(KV)                                                                                          \
  case KV:                                                                                                   \
    return nq <= 1 ? lanes_per_cu_kp<KV, 1>(lds)                                                             \
                   : (nq <= 2 ? lanes_per_cu_kp<KV, 2>(lds)                                                  \
                              : (nq <= 4 ? lanes_per_cu_kp<KV, 4>(lds) : lanes_per_cu_kp<KV, 8>(lds)));
  switch (c.KP) {
    PSX_OCC(1)
    PSX_OCC(2)
    PSX_OCC(4)
    PSX_OCC(8)
    default:
      PSX_OCC(16)
  }
#undef PSX_OCC
}

template <int KP, int NQ>
static void set_lanes_attr() {
  (void)hipFuncSetAttribute((const void*)wide_lanes_kernel<KP, NQ>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            96 * 1024);
}

template <int KP>
static void launch_lanes_kp(const WideCfg& c, const WideDev* devs, const WideLanesArgs& a, size_t lds,
                            hipStream_t s) {
  static const bool prepared = (set_lanes_attr<KP, 1>(), set_lanes_attr<KP, 2>(), set_lanes_attr<KP, 4>(),
                                set_lanes_attr<KP, 8>(), true);
  (void)prepared;
  const int nq = (c.NZ + 63) / 64;
  const int G = wide_lanes_grid(a.gpx);
  if (nq <= 1)
    wide_lanes_kernel<KP, 1><<<G, 512, lds, s>>>(c, devs, a);
  else if (nq <= 2)
    wide_lanes_kernel<KP, 2><<<G, 512, lds, s>>>(c, devs, a);
  else if (nq <= 4)
    wide_lanes_kernel<KP, 4><<<G, 512, lds, s>>>(c, devs, a);
  else
    wide_lanes_kernel<KP, 8><<<G, 512, lds, s>>>(c, devs, a);
}

void wide_launch_lanes(const WideCfg& c, const WideDev* devs, const WideLanesArgs& a, size_t lds, hipStream_t s) {
  switch (c.KP) {
    case 1: launch_lanes_kp<1>(c, devs, a, lds, s); break;
    case 2: launch_lanes_kp<2>(c, devs, a, lds, s); break;
    case 4: launch_lanes_kp<4>(c, devs, a, lds, s); break;
    case 8: launch_lanes_kp<8>(c, devs, a, lds, s); break;
    default: launch_lanes_kp<16>(c, devs, a, lds, s); break;
  }
}

void wide_launch_finalize(const WideCfg& c, const WideDev& d, hipStream_t s) {
  wide_finalize_kernel<<<grid_for((int64_t)c.umax + 1, 1024), 256, 0, s>>>(c, d);
}

const void* wide_begin_symbol() { return (const void*)wide_begin_kernel; }

// ---------------------------------------------------------------------------
// Ring ingest: one wavefront per row.
__global__ __launch_bounds__(256) void sparse_ring_ingest_kernel(const int64_t* __restrict__ indptr,
                                                                 const int32_t* __restrict__ idx,
                                                                 const uint16_t* __restrict__ val,
                                                                 const int32_t* __restrict__ y, int64_t src_first,
                                                                 int64_t src_step, int64_t n, int32_t* ridx,
                                                                 uint16_t* rval, int32_t* rnnz, int32_t* ry,
                                                                 int64_t dst_first, int cap, int NZ, int* trunc) {
  const int lane = threadIdx.x & 63;
  for (int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); i < n; i += (int64_t)gridDim.x * 4) {
    const int64_t sr = src_first + i * src_step;
    const int64_t dr = (dst_first + i) % cap;
    const int64_t a = indptr[sr], b = indptr[sr + 1];
    const int64_t len = b - a;
    const int nz = len < NZ ? (int)len : NZ;
    for (int j = lane; j < nz; j += 64) {
      ridx[dr * NZ + j] = idx[a + j];
      rval[dr * NZ + j] = val[a + j];
    }
    if (lane == 0) {
      rnnz[dr] = nz;
      ry[dr] = y[sr];
      if (len > NZ && trunc) atomicAdd(trunc, 1);
    }
  }
}

void launch_sparse_ring_ingest(const int64_t* indptr, const int32_t* idx, const uint16_t* val, const int32_t* y,
                               int64_t src_first, int64_t src_step, int64_t n, int32_t* ridx, uint16_t* rval,
                               int32_t* rnnz, int32_t* ry, int64_t dst_first, int cap, int NZ, int* trunc,
                               hipStream_t s) {
  if (n <= 0) return;
  sparse_ring_ingest_kernel<<<grid_for(n * 64, 2048), 256, 0, s>>>(indptr, idx, val, y, src_first, src_step, n, ridx,
                                                                   rval, rnnz, ry, dst_first, cap, NZ, trunc);
}

// Several rings' deliveries from one dataset in one launch (the wide lanes' ingest:
// blockIdx.y = job).  A job's fields are read with constant indices (unrolled selects
// on the uniform job id): a run-time index into the argument block would copy it into
// scratch (lanes_body.h pick()).
__global__ __launch_bounds__(256) void sparse_ring_ingest_many_kernel(const int64_t* __restrict__ indptr,
                                                                      const int32_t* __restrict__ idx,
                                                                      const uint16_t* __restrict__ val,
                                                                      const int32_t* __restrict__ y,
                                                                      SparseIngestJobs a) {
  const int jy = (int)blockIdx.y;
  SparseIngestJob j = a.job[0];
#pragma unroll
  for (int q = 1; q < kMaxIngestJobs; ++q)
    if (q == jy) j = a.job[q];
  const int lane = threadIdx.x & 63;
  const int cap = a.cap, NZ = a.NZ;
  for (int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); i < j.n; i += (int64_t)gridDim.x * 4) {
    const int64_t sr = j.src_first + i * j.src_step;
    const int64_t dr = (j.dst_first + i) % cap;
    const int64_t a0 = indptr[sr], b0 = indptr[sr + 1];
    const int64_t len = b0 - a0;
    const int nz = len < NZ ? (int)len : NZ;
    for (int e = lane; e < nz; e += 64) {
      j.ridx[dr * NZ + e] = idx[a0 + e];
      j.rval[dr * NZ + e] = val[a0 + e];
    }
    if (lane == 0) {
      j.rnnz[dr] = nz;
      j.ry[dr] = y[sr];
      if (len > NZ && j.trunc) atomicAdd(j.trunc, 1);
    }
  }
}

void launch_sparse_ring_ingest_many(const int64_t* indptr, const int32_t* idx, const uint16_t* val, const int32_t* y,
                                    const SparseIngestJobs& a, hipStream_t s) {
  if (a.njobs <= 0) return;
  int64_t nmax = 0;
  for (int q = 0; q < a.njobs; ++q) nmax = a.job[q].n > nmax ? a.job[q].n : nmax;
  if (nmax <= 0) return;
  const dim3 grid((unsigned)grid_for(nmax * 64, 512), (unsigned)a.njobs);
  sparse_ring_ingest_many_kernel<<<grid, 256, 0, s>>>(indptr, idx, val, y, a);
}

// ---------------------------------------------------------------------------
// Test-set evaluation: one wavefront per row, LDS confusion counts, last
// workgroup publishes into the pinned EvalSlot (protocol of test_eval_kernel).
template <int KP>
__device__ __forceinline__ void wide_row_margins(int64_t F, const int64_t* __restrict__ indptr,
                                                 const int32_t* __restrict__ idx, const uint16_t* __restrict__ val,
                                                 int64_t row, const float* __restrict__ w, float (&z)[KP]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int k = 0; k < KP; ++k) z[k] = 0.f;
  const int64_t a = indptr[row], b = indptr[row + 1];
  for (int64_t e = a + lane; e < b; e += 64) {
    const int f = idx[e];
    const float v = bf2f(val[e]);
    float wv[KP];
    ldk<KP>(w + (int64_t)f * KP, wv);
#pragma unroll
    for (int k = 0; k < KP; ++k) z[k] += v * wv[k];
  }
#pragma unroll
  for (int k = 0; k < KP; ++k) z[k] = wave_sum(z[k]);
  float bv[KP];
  ldk<KP>(w + F * KP, bv);
#pragma unroll
  for (int k = 0; k < KP; ++k) z[k] += bv[k];
}

// Margins of up to 4 rows per wave for the evaluation: 16 lanes per row, each
// lane with 4 entries' loads in flight (ids/values, then the local-model map,
// then the weight rows), so a wave keeps 4 rows x 64 gathers outstanding
// instead of walking one row's dependent load chain at a time.
// PAIR: also the margins zb of the plain model w (no overlay) from the same
// gathers -- the worker's local model and the global model it was trained from
// differ only on the window's features.
// Key-range form (w == nullptr): only overlay entries contribute, on top of
// zbase[row] (the caller adds it), with the intercepts from `bias`.
template <int KP, bool PAIR>
__device__ __forceinline__ void wide_rows4_margins(int64_t F, const int64_t* __restrict__ indptr,
                                                  const int32_t* __restrict__ idx,
                                                  const uint16_t* __restrict__ val, int64_t row, bool valid,
                                                  const float* __restrict__ w, const int2* __restrict__ htab,
                                                  unsigned hmask, const float* __restrict__ wloc,
                                                  const float* __restrict__ bias, float (&z)[KP], float (&zb)[KP]) {
  const int l = threadIdx.x & 15;
#pragma unroll
  for (int k = 0; k < KP; ++k) z[k] = zb[k] = 0.f;
  if (valid && (w || htab)) {  // (key-range server row: margins base + intercepts only)
    const int64_t a = indptr[row], b = indptr[row + 1];
    for (int64_t e0 = a + l; e0 < b; e0 += 64) {
      int f[4];
      float v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t e = e0 + 16 * u;
        const bool ok = e < b;
        f[u] = ok ? idx[e] : -1;
        v[u] = ok ? bf2f(val[e]) : 0.f;
      }
      const float* src[4];
      bool ov[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        src[u] = f[u] >= 0 && w ? w + (int64_t)f[u] * KP : nullptr;
        ov[u] = false;
        if (htab && f[u] >= 0) {
          const int li = wide_find(htab, hmask, f[u]);
          if (li >= 0) {
            src[u] = wloc + KP + (int64_t)li * KP;
            ov[u] = true;
          }
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (src[u]) {
          float wv[KP];
          ldk<KP>(src[u], wv);
#pragma unroll
          for (int k = 0; k < KP; ++k) z[k] += v[u] * wv[k];
          if constexpr (PAIR) {
            if (ov[u]) ldk<KP>(w + (int64_t)f[u] * KP, wv);
#pragma unroll
            for (int k = 0; k < KP; ++k) zb[k] += v[u] * wv[k];
          }
        }
      }
    }
  }
#pragma unroll
  for (int k = 0; k < KP; ++k) {
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      z[k] += __shfl_xor(z[k], o, 64);
      if constexpr (PAIR) zb[k] += __shfl_xor(zb[k], o, 64);
    }
  }
  float bv[KP];
  ldk<KP>(bias ? bias : (htab ? wloc : w + F * KP), bv);
#pragma unroll
  for (int k = 0; k < KP; ++k) z[k] += bv[k];
  if constexpr (PAIR) {
    ldk<KP>(w + F * KP, bv);
#pragma unroll
    for (int k = 0; k < KP; ++k) zb[k] += bv[k];
  }
}

template <int KP>
__device__ __forceinline__ int wide_argmax(int K, const float (&z)[KP]) {
  if (K == 1) return z[0] > 0.f ? 1 : 0;
  int best = 0;
  float bz = -INFINITY;
#pragma unroll
  for (int k = 0; k < KP; ++k)
    if (k < K && z[k] > bz) {
      bz = z[k];
      best = k;
    }
  return best;
}

// Paired mode (slot2 != nullptr, needs the overlay): row 1 = the overlay model
// (the worker's local model), row 2 = the plain model w (the global model it was
// trained from), one pass.
template <int KP, bool PAIR>
__global__ __launch_bounds__(256) void wide_eval_kernel(int K, int64_t F, const int64_t* __restrict__ indptr,
                                                        const int32_t* __restrict__ idx,
                                                        const uint16_t* __restrict__ val,
                                                        const int32_t* __restrict__ y, int T,
                                                        const float* __restrict__ w, const int2* __restrict__ htab,
                                                        unsigned hmask, const float* __restrict__ wloc, int* acc,
                                                        unsigned* ticket, char* slot, const float* loss,
                                                        unsigned long long seq, char* slot2, unsigned long long seq2,
                                                        const float* __restrict__ zbase,
                                                        const float* __restrict__ bias) {
  __shared__ int cl[2][256];
  __shared__ int last;
  const int tid = threadIdx.x, lane = tid & 63;
  cl[0][tid] = 0;
  cl[1][tid] = 0;
  __syncthreads();
  // 16 rows per workgroup pass: wave (tid >> 6), lane group (lane >> 4)
  for (int64_t r0 = (int64_t)blockIdx.x * 16; r0 < T; r0 += (int64_t)gridDim.x * 16) {
    const int64_t r = r0 + (tid >> 4);
    float z[KP], zb[KP];
    wide_rows4_margins<KP, PAIR>(F, indptr, idx, val, r, r < T, w, htab, hmask, wloc, bias, z, zb);
    if (zbase && r < T) {
#pragma unroll
      for (int k = 0; k < KP; ++k) z[k] += zbase[r * KP + k];
    }
    if ((lane & 15) == 0 && r < T) {
      int yl = y[r];
      if (K == 1) yl = yl > 0 ? 1 : 0;
      yl = yl < 0 ? 0 : (yl > 15 ? 15 : yl);
      atomicAdd(&cl[0][yl * 16 + wide_argmax<KP>(K, z)], 1);
      if constexpr (PAIR) atomicAdd(&cl[1][yl * 16 + wide_argmax<KP>(K, zb)], 1);
    }
  }
  __syncthreads();
  const int ast = slot ? kAccStride : 1;  // slot mode: one cell per 128-B line (see test_eval_kernel)
  // slot mode: workgroup b adds into copy b % kWideEvalCopies of the [2][256] cells (one
  // copy serialises every workgroup's atomics on the same few cells)
  int* accb = slot ? acc + (int)(blockIdx.x % kWideEvalCopies) * 512 * kAccStride : acc;
  const int v = cl[0][tid];
  if (v) atomicAdd(accb + tid * ast, v);
  if constexpr (PAIR) {
    const int v2 = cl[1][tid];
    if (v2) atomicAdd(accb + (256 + tid) * ast, v2);
  }
  if (slot == nullptr) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0)
    last = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
  __syncthreads();
  if (!last) return;
  // publication as in test_eval_kernel: drained system-scope stores into the
  // uncached host slot, then the sequence number (no L2-writeback fence)
  int part[kWideEvalCopies];
#pragma unroll
  for (int q = 0; q < kWideEvalCopies; ++q)
    part[q] = __hip_atomic_exchange(acc + (q * 512 + tid) * ast, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  int tot = 0;
#pragma unroll
  for (int q = 0; q < kWideEvalCopies; ++q) tot += part[q];
  __hip_atomic_store((int*)slot + tid, tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (tid == 0) __hip_atomic_store((float*)(slot + 1024), loss ? *loss : 0.f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if constexpr (PAIR) {
    int tot2 = 0;
#pragma unroll
    for (int q = 0; q < kWideEvalCopies; ++q)
      part[q] = __hip_atomic_exchange(acc + (q * 512 + 256 + tid) * ast, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
    for (int q = 0; q < kWideEvalCopies; ++q) tot2 += part[q];
    __hip_atomic_store((int*)slot2 + tid, tot2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (tid == 0) __hip_atomic_store((float*)(slot2 + 1024), 0.f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store((unsigned long long*)(slot + 1032), seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if constexpr (PAIR)
      __hip_atomic_store((unsigned long long*)(slot2 + 1032), seq2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// wide_eval_multi_kernel: see launch_wide_eval_multi.  16 lanes per row (4 rows per
// wave), two non-zeros per lane in flight: the row of w gathered once per non-zero,
// every overlay's table probed for the feature at its home slot (independent loads, in
// flight together; a collision walks on), the lane's local coefficients where it maps
// the feature.  Every model loop is unrolled over kWideMaxEval with run-time guards, so
// the margins stay in registers (a runtime model index would put them in scratch).
template <int KP>
__global__ __launch_bounds__(256) void wide_eval_multi_kernel(int K, int64_t F, const int64_t* __restrict__ indptr,
                                                              const int32_t* __restrict__ idx,
                                                              const uint16_t* __restrict__ val,
                                                              const int32_t* __restrict__ y, int T,
                                                              const float* __restrict__ w, WideEvalModels m, int* acc,
                                                              unsigned* ticket) {
  constexpr int NE = 2;  // non-zeros per lane in flight (4: the same 116 us, profiles/r06/README.md section 9)
  __shared__ int cl[kWideMaxEval][256];
  __shared__ int last;
  const int tid = threadIdx.x, lane = tid & 63;
  const int nov = m.nov, M = m.nov + m.plain;
#pragma unroll
  for (int j = 0; j < kWideMaxEval; ++j) cl[j][tid] = 0;
  __syncthreads();
  for (int64_t r0 = (int64_t)blockIdx.x * 16; r0 < T; r0 += (int64_t)gridDim.x * 16) {
    const int64_t row = r0 + (tid >> 4);
    const bool valid = row < T;
    float z[kWideMaxEval][KP];
#pragma unroll
    for (int j = 0; j < kWideMaxEval; ++j)
#pragma unroll
      for (int k = 0; k < KP; ++k) z[j][k] = 0.f;
    if (valid) {
      const int64_t a0 = indptr[row], b0 = indptr[row + 1];
      for (int64_t e0 = a0 + (lane & 15); e0 < b0; e0 += 16 * NE) {
        int f[NE];
        float v[NE];
#pragma unroll
        for (int u = 0; u < NE; ++u) {
          const int64_t e = e0 + 16 * u;
          const bool ok = e < b0;
          f[u] = ok ? idx[e] : -1;
          v[u] = ok ? bf2f(val[e]) : 0.f;
        }
        if (m.pres) {  // the lanes' overlay table: one presence word + the lanes' rows of f
          float wv[NE][KP];
          unsigned pm[NE];
#pragma unroll
          for (int u = 0; u < NE; ++u) {
            if (f[u] >= 0) {
              ldk<KP>(w + (int64_t)f[u] * KP, wv[u]);
              pm[u] = m.pres[f[u]];
            } else {
#pragma unroll
              for (int k = 0; k < KP; ++k) wv[u][k] = 0.f;
              pm[u] = 0u;
            }
          }
#pragma unroll
          for (int u = 0; u < NE; ++u) {
#pragma unroll
            for (int j = 0; j < kWideMaxLanes; ++j) {
              if (j < nov) {
                if ((pm[u] >> j) & 1u) {
                  float ov[KP];
                  ldk<KP>(m.ov + ((int64_t)f[u] * kWideMaxLanes + j) * KP, ov);
#pragma unroll
                  for (int k = 0; k < KP; ++k) z[j][k] += v[u] * ov[k];
                } else {
#pragma unroll
                  for (int k = 0; k < KP; ++k) z[j][k] += v[u] * wv[u][k];
                }
              }
            }
#pragma unroll
            for (int j = 0; j < kWideMaxEval; ++j)
              if (m.plain && j == nov) {
#pragma unroll
                for (int k = 0; k < KP; ++k) z[j][k] += v[u] * wv[u][k];
              }
          }
          continue;
        }
        float wv[NE][KP];
        int2 pr[NE][kWideMaxLanes];
#pragma unroll
        for (int u = 0; u < NE; ++u) {
          if (f[u] >= 0) {
            ldk<KP>(w + (int64_t)f[u] * KP, wv[u]);
          } else {
#pragma unroll
            for (int k = 0; k < KP; ++k) wv[u][k] = 0.f;
          }
          bool in[kWideMaxLanes];  // the feature is in lane j's window (bitmap; no bitmap: maybe)
#pragma unroll
          for (int j = 0; j < kWideMaxLanes; ++j)
            in[j] = j < nov && f[u] >= 0 &&
                    (m.bm == nullptr || ((m.bm[(int64_t)j * m.nw + (f[u] >> 5)] >> (f[u] & 31)) & 1u));
#pragma unroll
          for (int j = 0; j < kWideMaxLanes; ++j)
            pr[u][j] = in[j] ? m.htab[j][wide_gslot(f[u], m.hmask[j])] : make_int2(-1, -1);
        }
#pragma unroll
        for (int u = 0; u < NE; ++u) {
#pragma unroll
          for (int j = 0; j < kWideMaxLanes; ++j) {
            if (j < nov) {
              int li = -1;
              if (f[u] >= 0 && pr[u][j].x != -1) {
                if (pr[u][j].x == f[u]) {
                  li = pr[u][j].y;
                } else if (pr[u][j].x != -1) {  // collision: walk on from the home slot
                  unsigned h = wide_gslot(f[u], m.hmask[j]);
                  while (true) {
                    h = (h + 1) & m.hmask[j];
                    const int2 e = m.htab[j][h];
                    if (e.x == f[u]) {
                      li = e.y;
                      break;
                    }
                    if (e.x == -1) break;
                  }
                }
              }
              if (li >= 0) {
                float ov[KP];
                ldk<KP>(m.wloc[j] + KP + (int64_t)li * KP, ov);
#pragma unroll
                for (int k = 0; k < KP; ++k) z[j][k] += v[u] * ov[k];
              } else {
#pragma unroll
                for (int k = 0; k < KP; ++k) z[j][k] += v[u] * wv[u][k];
              }
            }
          }
#pragma unroll
          for (int j = 0; j < kWideMaxEval; ++j)
            if (m.plain && j == nov) {
#pragma unroll
              for (int k = 0; k < KP; ++k) z[j][k] += v[u] * wv[u][k];
            }
        }
      }
    }
#pragma unroll
    for (int j = 0; j < kWideMaxEval; ++j) {
      if (j < M) {
#pragma unroll
        for (int k = 0; k < KP; ++k)
#pragma unroll
          for (int o = 1; o < 16; o <<= 1) z[j][k] += __shfl_xor(z[j][k], o, 64);
      }
    }
    if ((lane & 15) == 0 && valid) {
      int yl = y[row];
      if (K == 1) yl = yl > 0 ? 1 : 0;
      yl = yl < 0 ? 0 : (yl > 15 ? 15 : yl);
#pragma unroll
      for (int j = 0; j < kWideMaxEval; ++j) {
        if (j < M) {
          // the intercepts: the overlay's own, or w's
          const float* bsrc = (j < kWideMaxLanes && j < nov) ? m.wloc[j < kWideMaxLanes ? j : 0] : w + F * KP;
          float bv[KP];
          ldk<KP>(bsrc, bv);
#pragma unroll
          for (int k = 0; k < KP; ++k) z[j][k] += bv[k];
          atomicAdd(&cl[j][yl * 16 + wide_argmax<KP>(K, z[j])], 1);
        }
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kWideMaxEval; ++j) {
    if (j < M) {
      const int v = cl[j][tid];
      if (v) atomicAdd(acc + (((int)(blockIdx.x % kWideEvalCopies) * kWideMaxEval + j) * 256 + tid) * kAccStride, v);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0)
    last = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
  __syncthreads();
  if (!last) return;
  // publication as in wide_eval_kernel: drained system-scope stores into the uncached
  // host slots, then each slot's sequence number
#pragma unroll
  for (int j = 0; j < kWideMaxEval; ++j) {
    if (j < M) {
      char* slot = m.slot[j];
      const float* loss = m.loss[j];
      int part[kWideEvalCopies];  // every copy's exchange in flight before the sum
#pragma unroll
      for (int q = 0; q < kWideEvalCopies; ++q)
        part[q] = __hip_atomic_exchange(acc + ((q * kWideMaxEval + j) * 256 + tid) * kAccStride, 0, __ATOMIC_RELAXED,
                                        __HIP_MEMORY_SCOPE_AGENT);
      int tot = 0;
#pragma unroll
      for (int q = 0; q < kWideEvalCopies; ++q) tot += part[q];
      __hip_atomic_store((int*)slot + tid, tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      if (tid == 0)
        __hip_atomic_store((float*)(slot + 1024), loss ? *loss : 0.f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
    for (int j = 0; j < kWideMaxEval; ++j)
      if (j < M)
        __hip_atomic_store((unsigned long long*)(m.slot[j] + 1032), m.seq[j], __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

template <int KP>
__global__ __launch_bounds__(256) void wide_logits_kernel(int64_t F, const int64_t* __restrict__ indptr,
                                                          const int32_t* __restrict__ idx,
                                                          const uint16_t* __restrict__ val, int T,
                                                          const float* __restrict__ w, float* out) {
  const int lane = threadIdx.x & 63;
  for (int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < T; r += (int64_t)gridDim.x * 4) {
    float z[KP];
    wide_row_margins<KP>(F, indptr, idx, val, r, w, z);
    if (lane < KP) {
      float o = 0.f;
#pragma unroll
      for (int k = 0; k < KP; ++k)
        if (k == lane) o = z[k];
      out[r * KP + lane] = o;
    }
  }
}

void launch_wide_eval(int K, int KP, int64_t F, const int64_t* indptr, const int32_t* idx, const uint16_t* val,
                      const int32_t* y, int T, const float* w, const int2* htab, unsigned hmask, const float* wloc,
                      int* acc, unsigned* ticket, void* slot, const float* loss, unsigned long long seq, hipStream_t s,
                      void* slot2, unsigned long long seq2, const float* zbase, const float* bias) {
  if (T <= 0) return;
  const int grid = grid_for((int64_t)T * 16, 1024);  // 16 rows per workgroup pass
  char* sl = static_cast<char*>(slot);
  char* sl2 = static_cast<char*>(slot2);
  const bool pair = sl2 != nullptr;
#define PSX_WE(KV)                                                                                             \
  case KV:                                                                                                     \
    if (pair)                                                                                                  \
      wide_eval_kernel<KV, true><<<grid, 256, 0, s>>>(K, F, indptr, idx, val, y, T, w, htab, hmask, wloc, acc, \
                                                      ticket, sl, loss, seq, sl2, seq2, nullptr, nullptr);     \
    else                                                                                                        \
      wide_eval_kernel<KV, false><<<grid, 256, 0, s>>>(K, F, indptr, idx, val, y, T, w, htab, hmask, wloc, acc, \
                                                       ticket, sl, loss, seq, nullptr, 0, zbase, bias);        \
    break;
  switch (KP) {
    PSX_WE(1)
    PSX_WE(2)
    PSX_WE(4)
    PSX_WE(8)
    PSX_WE(16)
    default:
      break;
  }
#undef PSX_WE
}

void launch_wide_eval_multi(int K, int KP, int64_t F, const int64_t* indptr, const int32_t* idx, const uint16_t* val,
                            const int32_t* y, int T, const float* w, const WideEvalModels& m, int* acc,
                            unsigned* ticket, hipStream_t s) {
  if (T <= 0 || m.nov + m.plain <= 0) return;
  const int grid = grid_for((int64_t)T * 16, 1024);  // 16 rows per workgroup pass
#define PSX_WM(KV)                                                                                         \
  case KV:                                                                                                 \
    wide_eval_multi_kernel<KV><<<grid, 256, 0, s>>>(K, F, indptr, idx, val, y, T, w, m, acc, ticket); \
    break;
  switch (KP) {
    PSX_WM(1)
    PSX_WM(2)
    PSX_WM(4)
    PSX_WM(8)
    PSX_WM(16)
    default:
      break;
  }
#undef PSX_WM
}

void launch_wide_logits(int K, int KP, int64_t F, const int64_t* indptr, const int32_t* idx, const uint16_t* val,
                        int T, const float* w, float* out, hipStream_t s) {
  (void)K;
  if (T <= 0) return;
  const int grid = grid_for((int64_t)T * 64, 1024);
#define PSX_WL(KV)                                                                      \
  case KV:                                                                              \
    wide_logits_kernel<KV><<<grid, 256, 0, s>>>(F, indptr, idx, val, T, w, out); \
    break;
  switch (KP) {
    PSX_WL(1)
    PSX_WL(2)
    PSX_WL(4)
    PSX_WL(8)
    PSX_WL(16)
    default:
      break;
  }
#undef PSX_WL
}

// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void wide_apply_sparse_kernel(float* w, int64_t F, int KP, const unsigned* Ud,
                                                                int Uh, const int32_t* __restrict__ uniq,
                                                                const float* __restrict__ dloc, float lr) {
  const int64_t U = Ud ? (int64_t)*Ud : (int64_t)Uh;
  const int64_t n = KP + U * KP;
  for (int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x; p < n; p += (int64_t)gridDim.x * 256) {
    const float v = dloc[p];
    if (v == 0.f) continue;
    if (p < KP) {
      w[F * KP + p] += lr * v;
    } else {
      const int64_t l = (p - KP) / KP, k = (p - KP) - l * KP;
      w[(int64_t)uniq[l] * KP + k] += lr * v;
    }
  }
}

void launch_wide_apply_sparse(float* w, int64_t F, int KP, const unsigned* U_dev, int U_host, const int32_t* uniq,
                              const float* dloc, float lr, int umax, hipStream_t s) {
  const int64_t n = KP + (int64_t)(U_dev ? umax : U_host) * KP;
  wide_apply_sparse_kernel<<<grid_for(n, 2048), 256, 0, s>>>(w, F, KP, U_dev, U_host, uniq, dloc, lr);
}

__global__ __launch_bounds__(256) void axpy_kernel(float* __restrict__ w, const float* __restrict__ x, float a,
                                                   int64_t n) {
  const int64_t n4 = n >> 2;
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += stride) {
    f32x4 v = ((f32x4*)w)[i];
    const f32x4 d = ((const f32x4*)x)[i];
    v += a * d;
    ((f32x4*)w)[i] = v;
  }
  for (int64_t i = (n4 << 2) + (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) w[i] += a * x[i];
}

// ---------------------------------------------------------------------------
// Sparse pull (asynchronous wide model): the server keeps the applied deltas in
// a ring log -- entry = ids [F (the intercepts' pseudo-feature), uniq[0..U)] and
// the push payload dloc [(U+1) * KP] unchanged, value block l <-> id l -- and a
// released worker receives the log entries since its previous pull instead of
// the dense weight vector (KeyRange-addressed payloads, BaseMessage.java:24-27).
__global__ __launch_bounds__(256) void log_append_kernel(const int32_t* __restrict__ uniq,
                                                         const float* __restrict__ dloc, int U, int64_t F, int KP,
                                                         int32_t* lids, float* lvals, int64_t pos, int64_t cap) {
  const int64_t nid = (int64_t)U + 1, nv = nid * KP;
  for (int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x; p < nv; p += (int64_t)gridDim.x * 256) {
    const int64_t l = p / KP, k = p - l * KP;
    const int64_t slot = (pos + l) % cap;
    lvals[slot * KP + k] = dloc[p];
    if (k == 0) lids[slot] = l == 0 ? (int32_t)F : uniq[l - 1];
  }
}

void launch_log_append(const int32_t* uniq, const float* dloc, int U, int64_t F, int KP, int32_t* lids, float* lvals,
                       int64_t pos, int64_t cap, hipStream_t s) {
  const int64_t nv = ((int64_t)U + 1) * KP;
  log_append_kernel<<<grid_for(nv, 2048), 256, 0, s>>>(uniq, dloc, U, F, KP, lids, lvals, pos, cap);
}

// w[ids[l] * KP + k] += lr * vals[l * KP + k]: ids repeat across log entries, so
// the adds are atomic (hardware fp32 atomics; the order of equal-id adds varies).
__global__ __launch_bounds__(256) void log_apply_kernel(float* w, const int32_t* __restrict__ ids,
                                                        const float* __restrict__ vals, int64_t n, int KP, float lr) {
  const int64_t nv = n * KP;
  for (int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x; p < nv; p += (int64_t)gridDim.x * 256) {
    const float v = vals[p];
    if (v == 0.f) continue;
    const int64_t l = p / KP, k = p - l * KP;
    atomicAdd(w + (int64_t)ids[l] * KP + k, lr * v);
  }
}

void launch_log_apply(float* w, const int32_t* ids, const float* vals, int64_t n, int KP, float lr, hipStream_t s) {
  if (n <= 0) return;
  log_apply_kernel<<<grid_for(n * KP, 4096), 256, 0, s>>>(w, ids, vals, n, KP, lr);
}

void launch_axpy(float* w, const float* delta, float lr, int64_t n, hipStream_t s) {
  if (n <= 0) return;
  axpy_kernel<<<grid_for(n / 4 + 1, 4096), 256, 0, s>>>(w, delta, lr, n);
}

}  // namespace psx
