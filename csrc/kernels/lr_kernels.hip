// Multinomial logistic-regression kernels for the worker local solve, the
// server update and test-set evaluation (gfx950 / CDNA4).
//
// Reference math being replaced (all Spark MLlib local mode on the JVM):
//   * standardisation statistics + multinomial loss/gradient inside
//     LogisticRegression.fit  (LogisticRegressionTaskSpark.java:179-184)
//   * delta extraction w_new - w_old (:195-218)
//   * server update w += (1/N) delta (ServerProcessor.java:148-151, 225-228)
//   * test-set predict + weighted F1/accuracy (:236-251, Metrics.java:15-24)
//
// Layout conventions (device):
//   X ring   : bf16 [cap][FP], FP = features padded to a multiple of 128
//   vectors  : fp32 [P] with P = K*FP + K: coefficient (c, f) at c*FP + f,
//              intercept c at K*FP + c (the reference's column-major flat
//              index is only used at the checkpoint/log boundary)
//   W frags  : bf16 hi/lo [FP/8][16][8]: element (c, f) at ((f>>3)*16+c)*8+(f&7),
//              i.e. exactly the B-operand fragment order of
//              v_mfma_f32_16x16x32_bf16, so one 16-B load per lane per k-step.
#include <hip/hip_runtime.h>

#include "common.h"
#include "lr_kernels.h"

namespace psx {

bool fp_supported(int FP) { return FP == 128 || FP == 256 || FP == 512 || FP == 1024 || FP == 2048; }

template <int FP> __global__ void eval_kernel(SolverCfg, const SolveParams*, const Ctrl*, int, const uint16_t*,
                                              const int32_t*, const uint16_t*, const uint16_t*, const float*, float*,
                                              float*, float*);
template <int FP> __global__ void test_eval_kernel(int, const uint16_t*, const int32_t*, int, const uint16_t*,
                                                   const uint16_t*, const float*, int*);
template <int FP> __global__ void logits_kernel(int, const uint16_t*, int, const uint16_t*, const uint16_t*,
                                                const float*, float*);

#define PSX_CHECK_LAUNCH() (void)hipGetLastError()

// ---------------------------------------------------------------------------
__global__ void set_params_kernel(SolveParams* p, int B, int start) {
  p->B = B;
  p->start = start;
}

void launch_set_params(SolveParams* p, int B, int start, hipStream_t s) {
  set_params_kernel<<<1, 1, 0, s>>>(p, B, start);
}

// ---------------------------------------------------------------------------
// K2: per-feature sum / sum of squares over the window (fp64 atomics).
// grid (FP/128, row_blocks); 256 threads = 16 chunks (8 features) x 16 rows.
__global__ __launch_bounds__(256) void stats_kernel(const uint16_t* __restrict__ X, const SolveParams* prm,
                                                    int cap, int FP, double* __restrict__ acc) {
  __shared__ float red[2][16][129];
  const int B = prm->B, start = prm->start;
  const int t = threadIdx.x, ch = t & 15, rs = t >> 4;
  const int f0 = blockIdx.x * 128 + ch * 8;
  float s[8], q[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s[j] = q[j] = 0.f;
  for (int i = blockIdx.y * 16 + rs; i < B; i += gridDim.y * 16) {
    int r = start + i;
    if (r >= cap) r -= cap;
    u16x8 v = *(const u16x8*)(X + (size_t)r * FP + f0);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float x = bf2f(v[j]);
      s[j] += x;
      q[j] += x * x;
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    red[0][rs][ch * 8 + j] = s[j];
    red[1][rs][ch * 8 + j] = q[j];
  }
  __syncthreads();
  if (t < 128) {
    double a = 0, b = 0;
    for (int r = 0; r < 16; ++r) {
      a += red[0][r][t];
      b += red[1][r][t];
    }
    // per-row-block partials; prep sums them in a fixed order (deterministic)
    acc[((size_t)blockIdx.y * 2 + 0) * FP + blockIdx.x * 128 + t] = a;
    acc[((size_t)blockIdx.y * 2 + 1) * FP + blockIdx.x * 128 + t] = b;
  }
}

void launch_stats(const uint16_t* X, const SolveParams* prm, int cap, int FP, double* acc, int row_blocks,
                  hipStream_t s) {
  dim3 grid(FP / 128, row_blocks);
  stats_kernel<<<grid, 256, 0, s>>>(X, prm, cap, FP, acc);
}

// ---------------------------------------------------------------------------
__device__ __forceinline__ void write_frag(uint16_t* hi, uint16_t* lo, int c, int f, float w) {
  unsigned short h, l;
  split_bf16(w, h, l);
  size_t o = ((size_t)(f >> 3) * 16 + c) * 8 + (f & 7);
  hi[o] = h;
  lo[o] = l;
}

// Initial point in the standardised space: x0 = w_old * std, std from the
// window statistics (sample variance, n-1), W_eff for the first evaluation.
__global__ __launch_bounds__(256) void prep_kernel(SolverCfg cfg, const SolveParams* prm,
                                                   const double* __restrict__ acc, const float* __restrict__ w_old,
                                                   float* x, float* d, float* g_c, float* std_, float* inv_std,
                                                   float* wfix, uint16_t* wf_hi, uint16_t* wf_lo, float* b_eff,
                                                   Ctrl* ctrl, int nrb) {
  const int p = blockIdx.x * 256 + threadIdx.x;
  const int KF = cfg.K * cfg.Fp;
  if (p == 0) ctrl_init(*ctrl);
  if (p >= cfg.P) return;
  d[p] = 0.f;
  g_c[p] = 0.f;
  if (p < KF) {
    const int c = p / cfg.Fp, f = p - c * cfg.Fp;
    const double n = (double)prm->B;
    double sd = 0.0;
    if (f < cfg.F && n > 1.0) {
      double s1 = 0.0, s2 = 0.0;
      for (int rb = 0; rb < nrb; ++rb) {
        s1 += acc[((size_t)rb * 2 + 0) * cfg.Fp + f];
        s2 += acc[((size_t)rb * 2 + 1) * cfg.Fp + f];
      }
      double mean = s1 / n;
      double var = (s2 - n * mean * mean) / (n - 1.0);
      sd = var > 0.0 ? sqrt(var) : 0.0;
    }
    float sdf = (float)sd, inv = sd > 0.0 ? (float)(1.0 / sd) : 0.f;
    if (c == 0) {
      std_[f] = sdf;
      inv_std[f] = inv;
    }
    const float wo = f < cfg.F ? w_old[p] : 0.f;
    const float xv = wo * sdf;
    x[p] = xv;
    const float fix = (sd > 0.0 || cfg.zero_const) ? 0.f : wo;
    wfix[p] = fix;
    write_frag(wf_hi, wf_lo, c, f, xv * inv + fix);
  } else {
    const int c = p - KF;
    x[p] = w_old[p];
    b_eff[c] = w_old[p];
  }
}

void launch_prep(const SolverCfg& cfg, const SolveParams* prm, const double* acc, const float* w_old, float* x,
                 float* d, float* g_c, float* std_, float* inv_std, float* wfix, uint16_t* wf_hi, uint16_t* wf_lo,
                 float* b_eff, Ctrl* ctrl, int nrb, hipStream_t s) {
  prep_kernel<<<(cfg.P + 255) / 256, 256, 0, s>>>(cfg, prm, acc, w_old, x, d, g_c, std_, inv_std, wfix, wf_hi,
                                                  wf_lo, b_eff, ctrl, nrb);
}

// ---------------------------------------------------------------------------
// Shared tile machinery: stage a 32-row tile into the dual-use LDS image and
// run the forward product Z[32][16] = X_tile . W^T with bf16 hi/lo weights.

// LDS map: [0, 32*FP*2)       X image (FP/128 sub-images of 8 KB)
//          +8192              cross-wave logits reduction [4][2][64][4] f32
//          +2048              R^T hi/lo  [2][16][32] bf16
//          +512               labels [32] i32, rsum [16] f32, misc
template <int FP>
__device__ __forceinline__ void stage_tile(char* lds, const uint16_t* __restrict__ X, int64_t row0, int nrows,
                                           int cap, bool ring) {
  constexpr int CPR = FP / 8;  // 16-B chunks per row
  for (int q = threadIdx.x; q < 32 * CPR; q += 256) {
    const int row = q / CPR, cg = q - row * CPR;
    u16x8 v = {0, 0, 0, 0, 0, 0, 0, 0};
    if (row < nrows) {
      int64_t r = row0 + row;
      if (ring && r >= cap) r -= cap;
      v = *(const u16x8*)(X + r * FP + cg * 8);
    }
    *(u16x8*)(lds + (cg >> 4) * 8192 + lds_off(row, cg & 15)) = v;
  }
}

template <int FP>
__device__ __forceinline__ void forward_tile(const char* lds, const uint16_t* __restrict__ wf_hi,
                                             const uint16_t* __restrict__ wf_lo, f32x4& acc0, f32x4& acc1) {
  constexpr int KS_PER_WAVE = FP / 128;  // 32-feature k-steps per wave
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 15, kq = lane >> 4;
  acc0 = f32x4{0, 0, 0, 0};
  acc1 = f32x4{0, 0, 0, 0};
#pragma unroll
  for (int kk = 0; kk < KS_PER_WAVE; ++kk) {
    const int ks = w * KS_PER_WAVE + kk;
    const int cg = ks * 4 + kq;
    const char* sub = lds + (cg >> 4) * 8192;
    const u16x8 a0 = *(const u16x8*)(sub + lds_off(r, cg & 15));
    const u16x8 a1 = *(const u16x8*)(sub + lds_off(16 + r, cg & 15));
    const size_t fo = ((size_t)cg * 16 + r) * 8;
    const u16x8 bh = *(const u16x8*)(wf_hi + fo);
    const u16x8 bl = *(const u16x8*)(wf_lo + fo);
    acc0 = mfma16x16x32(as_bf16x8(a0), as_bf16x8(bh), acc0);
    acc0 = mfma16x16x32(as_bf16x8(a0), as_bf16x8(bl), acc0);
    acc1 = mfma16x16x32(as_bf16x8(a1), as_bf16x8(bh), acc1);
    acc1 = mfma16x16x32(as_bf16x8(a1), as_bf16x8(bl), acc1);
  }
}

// Sum the 4 waves' partial logits; returns z(row, c) from LDS after a barrier.
__device__ __forceinline__ void store_partial_logits(char* red_base, const f32x4& acc0, const f32x4& acc1) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  f32x4* red = (f32x4*)red_base;
  red[(w * 2 + 0) * 64 + lane] = acc0;
  red[(w * 2 + 1) * 64 + lane] = acc1;
}

__device__ __forceinline__ float load_logit(const char* red_base, int row, int c) {
  const float* red = (const float*)red_base;
  const int mt = row >> 4, rr = row & 15;
  const int lane = (rr >> 2) * 16 + c, reg = rr & 3;
  float z = 0.f;
#pragma unroll
  for (int w = 0; w < 4; ++w) z += red[((w * 2 + mt) * 64 + lane) * 4 + reg];
  return z;
}

// ---------------------------------------------------------------------------
// K3: fused multinomial forward + softmax/CE + backward for the current trial
// point.  One workgroup per 32-row tile (grid-stride), X tile staged once in
// LDS and consumed twice: row reads for Z = X W^T, hardware-transposed reads
// (ds_read_b64_tr_b16) for G = R^T X.  Per-workgroup partial G / loss slabs
// are reduced by the next kernel (deterministic, no float atomics).
template <int FP>
__global__ __launch_bounds__(256) void eval_kernel(SolverCfg cfg, const SolveParams* prm, const Ctrl* ctrl,
                                                   int slot, const uint16_t* __restrict__ X,
                                                   const int32_t* __restrict__ y, const uint16_t* __restrict__ wf_hi,
                                                   const uint16_t* __restrict__ wf_lo,
                                                   const float* __restrict__ b_eff, float* __restrict__ Gpart,
                                                   float* __restrict__ Rpart, float* __restrict__ Lpart) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  constexpr int NTW = FP / 64;  // 16-feature N-tiles per wave in the backward
  if (ctrl->phase == kPhDone) return;
  const int B = prm->B, start = prm->start, cap = cfg.cap, K = cfg.K;
  const int ntiles = (B + 31) / 32;
  const int nact = min((int)gridDim.x, ntiles);
  if ((int)blockIdx.x >= nact) return;

  char* red_base = lds + 32 * FP * 2;
  unsigned short* rt = (unsigned short*)(red_base + 8192);  // [2][16][32]
  int* ylds = (int*)(red_base + 8192 + 2048);
  float* rsum = (float*)(ylds + 32);

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  if (tid < 16) rsum[tid] = 0.f;

  f32x4 accb[NTW];
#pragma unroll
  for (int j = 0; j < NTW; ++j) accb[j] = f32x4{0, 0, 0, 0};
  float loss = 0.f;
  // softmax role: row sr, classes sc0, sc0+1
  const int sr = tid >> 3, sc0 = (tid & 7) * 2;
  float rs0 = 0.f, rs1 = 0.f;
  const float bz0 = sc0 < K ? b_eff[sc0] : 0.f, bz1 = sc0 + 1 < K ? b_eff[sc0 + 1] : 0.f;

  for (int tile = blockIdx.x; tile < ntiles; tile += nact) {
    const int nrows = min(32, B - tile * 32);
    int64_t row0 = (int64_t)start + (int64_t)tile * 32;
    if (row0 >= cap) row0 -= cap;
    stage_tile<FP>(lds, X, row0, nrows, cap, true);
    if (tid < 32) {
      int yy = 0;
      if (tid < nrows) {
        int64_t r = row0 + tid;
        if (r >= cap) r -= cap;
        yy = y[r];
      }
      ylds[tid] = yy;
    }
    __syncthreads();
    f32x4 a0, a1;
    forward_tile<FP>(lds, wf_hi, wf_lo, a0, a1);
    store_partial_logits(red_base, a0, a1);
    __syncthreads();
    // softmax + cross entropy, 8 threads per row
    {
      const bool v0 = sc0 < K, v1 = sc0 + 1 < K;
      float z0 = v0 ? load_logit(red_base, sr, sc0) + bz0 : -INFINITY;
      float z1 = v1 ? load_logit(red_base, sr, sc0 + 1) + bz1 : -INFINITY;
      float mx = fmaxf(z0, z1);
      mx = fmaxf(mx, __shfl_xor(mx, 1, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 2, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 4, 64));
      float e0 = v0 ? __expf(z0 - mx) : 0.f, e1 = v1 ? __expf(z1 - mx) : 0.f;
      float se = e0 + e1;
      se += __shfl_xor(se, 1, 64);
      se += __shfl_xor(se, 2, 64);
      se += __shfl_xor(se, 4, 64);
      const bool valid = sr < nrows;
      const int yl = ylds[sr];
      const float inv = 1.f / se;
      float r0 = valid && v0 ? e0 * inv - (yl == sc0 ? 1.f : 0.f) : 0.f;
      float r1 = valid && v1 ? e1 * inv - (yl == sc0 + 1 ? 1.f : 0.f) : 0.f;
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
    // backward: G[c][f] += sum_r R[r][c] X[r][f]  (M = classes, N = features, K = rows)
    {
      const u16x8 ah = *(const u16x8*)(rt + (lane & 15) * 32 + (lane >> 4) * 8);
      const u16x8 al = *(const u16x8*)(rt + 512 + (lane & 15) * 32 + (lane >> 4) * 8);
      const int g = lane >> 4, il = lane & 15, q = il >> 2, pp = il & 3;
#pragma unroll
      for (int j = 0; j < NTW; ++j) {
        const int nt = w * NTW + j, f0 = nt * 16;
        const int sub = f0 >> 7, c0 = (f0 & 127) >> 3;
        const int chk = c0 + (pp >> 1), inb = 8 * (pp & 1);
        const char* base = lds + sub * 8192;
        const s16x4 b0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s16x4*)(base + lds_off(8 * g + q, chk) + inb));
        const s16x4 b1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s16x4*)(base + lds_off(8 * g + 4 + q, chk) + inb));
        u16x8 bv;
        bv[0] = b0[0]; bv[1] = b0[1]; bv[2] = b0[2]; bv[3] = b0[3];
        bv[4] = b1[0]; bv[5] = b1[1]; bv[6] = b1[2]; bv[7] = b1[3];
        accb[j] = mfma16x16x32(as_bf16x8(ah), as_bf16x8(bv), accb[j]);
        accb[j] = mfma16x16x32(as_bf16x8(al), as_bf16x8(bv), accb[j]);
      }
    }
    __syncthreads();
  }
  // ---- partial slabs ----
  float* G = Gpart + (size_t)blockIdx.x * K * FP;
#pragma unroll
  for (int j = 0; j < NTW; ++j) {
    const int f = (w * NTW + j) * 16 + (lane & 15);
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int c = (lane >> 4) * 4 + rr;
      if (c < K) G[(size_t)c * FP + f] = accb[j][rr];
    }
  }
  atomicAdd(&rsum[sc0], rs0);
  if (sc0 + 1 < 16) atomicAdd(&rsum[sc0 + 1], rs1);
  loss = wave_sum(loss);
  float* lred = rsum + 16;
  if (lane == 0) lred[w] = loss;
  __syncthreads();
  if (tid < 16) Rpart[blockIdx.x * 16 + tid] = rsum[tid];
  if (tid == 0) Lpart[blockIdx.x] = lred[0] + lred[1] + lred[2] + lred[3];
}

void launch_eval(const SolverCfg& cfg, const SolveParams* prm, const Ctrl* ctrl, int slot, const uint16_t* X,
                 const int32_t* y, const uint16_t* wf_hi, const uint16_t* wf_lo, const float* b_eff, float* Gpart,
                 float* Rpart, float* Lpart, int nwg, hipStream_t s) {
  const size_t lds = eval_lds_bytes(cfg.Fp);
#define PSX_EVAL(FPV)                                                                                    \
  case FPV:                                                                                              \
    eval_kernel<FPV><<<nwg, 256, lds, s>>>(cfg, prm, ctrl, slot, X, y, wf_hi, wf_lo, b_eff, Gpart, Rpart, \
                                           Lpart);                                                       \
    break;
  switch (cfg.Fp) {
    PSX_EVAL(128)
    PSX_EVAL(256)
    PSX_EVAL(512)
    PSX_EVAL(1024)
    PSX_EVAL(2048)
    default:
      break;
  }
#undef PSX_EVAL
}

// ---------------------------------------------------------------------------
// K4 reduction + controller: sums the eval slabs into the gradient g_t (in the
// standardised space), produces the dot products the line search / L-BFGS
// need, and the LAST workgroup to arrive advances the solver state machine
// (split-K seam recipe: slab stores -> vmcnt(0) -> barrier -> agent release ->
// ticket; last arriver: agent acquire -> plain loads).
__global__ __launch_bounds__(256) void reduce_kernel(SolverCfg cfg, const SolveParams* prm, Ctrl* ctrl, int slot,
                                                     const float* __restrict__ Gpart, const float* __restrict__ Rpart,
                                                     const float* __restrict__ Lpart, int nwg_eval,
                                                     const float* __restrict__ inv_std, const float* __restrict__ d,
                                                     const float* __restrict__ g_c, float* __restrict__ g_t,
                                                     const float* __restrict__ S, const float* __restrict__ Y,
                                                     double* __restrict__ dotpart) {
  __shared__ double sred[4][3 + 2 * kMaxHist];
  __shared__ double sdots[3 + 2 * kMaxHist];
  __shared__ int s_last;
  if (ctrl->phase == kPhDone) return;
  const int H = cfg.hist, ND = num_dots(H);
  const int B = prm->B, K = cfg.K, FP = cfg.Fp, KF = K * FP;
  const int nact = min(nwg_eval, (B + 31) / 32);
  const int m = ctrl->m, head = ctrl->head;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int p = blockIdx.x * 256 + tid;
  const float invB = 1.f / (float)B;
  float gv = 0.f, dv = 0.f, gcv = 0.f;
  if (p < cfg.P) {
    float s = 0.f;
    if (p < KF) {
      const int c = p / FP, f = p - c * FP;
      for (int e = 0; e < nact; ++e) s += Gpart[((size_t)e * K + c) * FP + f];
      gv = s * invB * inv_std[f];
    } else {
      const int c = p - KF;
      for (int e = 0; e < nact; ++e) s += Rpart[e * 16 + c];
      gv = s * invB;
    }
    g_t[p] = gv;
    dv = d[p];
    gcv = g_c[p];
  }
  {
    double v0 = wave_sum((double)gv * gv), v1 = wave_sum((double)gv * dv), v2 = wave_sum((double)gv * gcv);
    if (lane == 0) {
      sred[w][0] = v0;
      sred[w][1] = v1;
      sred[w][2] = v2;
    }
  }
  for (int i = 0; i < H; ++i) {
    const bool valid = m > 0 && (m == H || (((i - (head - m + 1)) % H + H) % H) < m);
    double si = 0.0, yi = 0.0;
    if (valid) {  // wave-uniform
      if (p < cfg.P) {
        si = (double)S[(size_t)i * cfg.P + p] * gv;
        yi = (double)Y[(size_t)i * cfg.P + p] * gv;
      }
      si = wave_sum(si);
      yi = wave_sum(yi);
    }
    if (lane == 0) {
      sred[w][3 + i] = si;
      sred[w][3 + H + i] = yi;
    }
  }
  __syncthreads();
  if (tid < ND) dotpart[(size_t)blockIdx.x * ND + tid] = sred[0][tid] + sred[1][tid] + sred[2][tid] + sred[3][tid];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    unsigned prev = __hip_atomic_fetch_add(&ctrl->ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = prev == gridDim.x - 1;
  }
  __syncthreads();
  if (!s_last) return;
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  if (tid < ND) {
    double s = 0.0;
    for (unsigned b = 0; b < gridDim.x; ++b) s += dotpart[(size_t)b * ND + tid];
    sdots[tid] = s;
  }
  __syncthreads();
  if (tid == 0) {
    double L = 0.0;
    for (int e = 0; e < nact; ++e) L += Lpart[e];
    ctrl_step(*ctrl, cfg, L / (double)B, sdots, slot);
    ctrl->ticket = 0;
  }
}

void launch_reduce(const SolverCfg& cfg, const SolveParams* prm, Ctrl* ctrl, int slot, const float* Gpart,
                   const float* Rpart, const float* Lpart, int nwg_eval, const float* inv_std, const float* d,
                   const float* g_c, float* g_t, const float* S, const float* Y, double* dotpart, hipStream_t s) {
  reduce_kernel<<<(cfg.P + 255) / 256, 256, 0, s>>>(cfg, prm, ctrl, slot, Gpart, Rpart, Lpart, nwg_eval, inv_std, d,
                                                    g_c, g_t, S, Y, dotpart);
}

// ---------------------------------------------------------------------------
// K4' elementwise solver update: applies the controller's action (accept step,
// push curvature pair, new direction) and materialises W_eff for the next
// trial point in MFMA fragment order.
__global__ __launch_bounds__(256) void update_kernel(SolverCfg cfg, const Ctrl* ctrl, int slot, float* x, float* d,
                                                     float* g_c, const float* __restrict__ g_t, float* S, float* Y,
                                                     const float* __restrict__ inv_std,
                                                     const float* __restrict__ wfix, uint16_t* wf_hi,
                                                     uint16_t* wf_lo, float* b_eff) {
  if (ctrl->action_slot != slot) return;
  const int act = ctrl->action;
  if (act == kActDone) return;
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= cfg.P) return;
  const int H = cfg.hist;
  float xv, dn;
  if (act == kActInit) {
    const float gc = g_t[p];
    g_c[p] = gc;
    dn = (float)ctrl->cg * gc;
    d[p] = dn;
    xv = x[p];
  } else if (act == kActTrial) {
    xv = x[p];
    dn = d[p];
  } else {  // accept
    const float dold = d[p];
    const float ta = (float)ctrl->t_acc;
    xv = x[p] + ta * dold;
    x[p] = xv;
    if (act == kActAcceptDone) return;
    const float gt = g_t[p];
    const int ps = ctrl->push_slot;
    if (ps >= 0) {
      S[(size_t)ps * cfg.P + p] = ta * dold;
      Y[(size_t)ps * cfg.P + p] = gt - g_c[p];
    }
    g_c[p] = gt;
    float acc = (float)ctrl->cg * gt;
    for (int i = 0; i < H; ++i) {
      const double cs = ctrl->cs[i], cy = ctrl->cy[i];
      if (cs != 0.0) acc += (float)cs * S[(size_t)i * cfg.P + p];
      if (cy != 0.0) acc += (float)cy * Y[(size_t)i * cfg.P + p];
    }
    dn = acc;
    d[p] = dn;
  }
  const float v = xv + (float)ctrl->t * dn;
  const int KF = cfg.K * cfg.Fp;
  if (p < KF) {
    const int c = p / cfg.Fp, f = p - c * cfg.Fp;
    write_frag(wf_hi, wf_lo, c, f, v * inv_std[f] + wfix[p]);
  } else {
    b_eff[p - KF] = v;
  }
}

void launch_update(const SolverCfg& cfg, const Ctrl* ctrl, int slot, float* x, float* d, float* g_c,
                   const float* g_t, float* S, float* Y, const float* inv_std, const float* wfix, uint16_t* wf_hi,
                   uint16_t* wf_lo, float* b_eff, hipStream_t s) {
  update_kernel<<<(cfg.P + 255) / 256, 256, 0, s>>>(cfg, ctrl, slot, x, d, g_c, g_t, S, Y, inv_std, wfix, wf_hi,
                                                    wf_lo, b_eff);
}

// ---------------------------------------------------------------------------
// K5/K6: back to the unstandardised space, multinomial centering, delta.
__global__ __launch_bounds__(256) void finalize_kernel(SolverCfg cfg, const Ctrl* ctrl, const float* __restrict__ x,
                                                       const float* __restrict__ inv_std,
                                                       const float* __restrict__ wfix,
                                                       const float* __restrict__ w_old, float* delta, float* w_new,
                                                       uint16_t* wf_hi, uint16_t* wf_lo, float* b_fin,
                                                       float* loss_out, int* stats_out) {
  const int f = blockIdx.x * 256 + threadIdx.x;
  const int K = cfg.K, FP = cfg.Fp, KF = K * FP;
  if (f < FP) {
    float wv[16];
    float mean = 0.f;
    for (int c = 0; c < K; ++c) {
      const int p = c * FP + f;
      float v = 0.f;
      if (f < cfg.F) v = inv_std[f] > 0.f ? x[p] * inv_std[f] : wfix[p];
      wv[c] = v;
      mean += v;
    }
    mean = (cfg.center && f < cfg.F) ? mean / (float)K : 0.f;
    for (int c = 0; c < K; ++c) {
      const int p = c * FP + f;
      const float v = wv[c] - mean;
      delta[p] = v - (f < cfg.F ? w_old[p] : 0.f);
      if (w_new) w_new[p] = v;
      write_frag(wf_hi, wf_lo, c, f, v);
    }
  }
  if (f == 0) {
    float bv[16];
    float mean = 0.f;
    for (int c = 0; c < K; ++c) {
      bv[c] = x[KF + c];
      mean += bv[c];
    }
    mean = cfg.center ? mean / (float)K : 0.f;
    for (int c = 0; c < K; ++c) {
      const float v = bv[c] - mean;
      delta[KF + c] = v - w_old[KF + c];
      if (w_new) w_new[KF + c] = v;
      b_fin[c] = v;
    }
    *loss_out = (float)ctrl->f_c;
    if (stats_out) {
      stats_out[0] = ctrl->evals;
      stats_out[1] = ctrl->nacc;
      stats_out[2] = ctrl->ls_fail;
      stats_out[3] = ctrl->dir_reset;
    }
  }
}

void launch_finalize(const SolverCfg& cfg, const Ctrl* ctrl, const float* x, const float* inv_std,
                     const float* wfix, const float* w_old, float* delta, float* w_new, uint16_t* wf_hi,
                     uint16_t* wf_lo, float* b_fin, float* loss_out, int* stats_out, hipStream_t s) {
  finalize_kernel<<<(cfg.Fp + 255) / 256, 256, 0, s>>>(cfg, ctrl, x, inv_std, wfix, w_old, delta, w_new, wf_hi, wf_lo,
                                                       b_fin, loss_out, stats_out);
}

// ---------------------------------------------------------------------------
// K8/K9: test-set argmax + confusion matrix (LDS counts, one global atomic per
// non-zero cell per workgroup).
template <int FP>
__global__ __launch_bounds__(256) void test_eval_kernel(int K, const uint16_t* __restrict__ Xt,
                                                        const int32_t* __restrict__ yt, int T,
                                                        const uint16_t* __restrict__ wf_hi,
                                                        const uint16_t* __restrict__ wf_lo,
                                                        const float* __restrict__ b, int* conf) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  char* red_base = lds + 32 * FP * 2;
  int* cl = (int*)(red_base + 8192);  // [16][16]
  const int tid = threadIdx.x;
  cl[tid] = 0;
  const int ntiles = (T + 31) / 32;
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int nrows = min(32, T - tile * 32);
    stage_tile<FP>(lds, Xt, (int64_t)tile * 32, nrows, 0, false);
    __syncthreads();
    f32x4 a0, a1;
    forward_tile<FP>(lds, wf_hi, wf_lo, a0, a1);
    store_partial_logits(red_base, a0, a1);
    __syncthreads();
    if (tid < nrows) {
      int best = 0;
      float bz = -INFINITY;
      for (int c = 0; c < K; ++c) {
        const float z = load_logit(red_base, tid, c) + b[c];
        if (z > bz) {
          bz = z;
          best = c;
        }
      }
      int yl = yt[(size_t)tile * 32 + tid];
      yl = yl < 0 ? 0 : (yl > 15 ? 15 : yl);
      atomicAdd(&cl[yl * 16 + best], 1);
    }
    __syncthreads();
  }
  __syncthreads();
  const int v = cl[tid];
  if (v) atomicAdd(conf + tid, v);
}

void launch_test_eval(int FP, int K, const uint16_t* Xt, const int32_t* yt, int T, const uint16_t* wf_hi,
                      const uint16_t* wf_lo, const float* b, int* conf, hipStream_t s) {
  const size_t lds = eval_lds_bytes(FP);
  const int ntiles = (T + 31) / 32;
  const int grid = ntiles < 1024 ? ntiles : 1024;
  if (grid <= 0) return;
#define PSX_TE(FPV)                                                                                  \
  case FPV:                                                                                          \
    test_eval_kernel<FPV><<<grid, 256, lds, s>>>(K, Xt, yt, T, wf_hi, wf_lo, b, conf); \
    break;
  switch (FP) {
    PSX_TE(128)
    PSX_TE(256)
    PSX_TE(512)
    PSX_TE(1024)
    PSX_TE(2048)
    default:
      break;
  }
#undef PSX_TE
}

// Logits for T rows (tests / debugging): logits[T][K].
template <int FP>
__global__ __launch_bounds__(256) void logits_kernel(int K, const uint16_t* __restrict__ Xt, int T,
                                                     const uint16_t* __restrict__ wf_hi,
                                                     const uint16_t* __restrict__ wf_lo,
                                                     const float* __restrict__ b, float* out) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  char* red_base = lds + 32 * FP * 2;
  const int tid = threadIdx.x;
  const int ntiles = (T + 31) / 32;
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int nrows = min(32, T - tile * 32);
    stage_tile<FP>(lds, Xt, (int64_t)tile * 32, nrows, 0, false);
    __syncthreads();
    f32x4 a0, a1;
    forward_tile<FP>(lds, wf_hi, wf_lo, a0, a1);
    store_partial_logits(red_base, a0, a1);
    __syncthreads();
    for (int e = tid; e < nrows * K; e += 256) {
      const int r = e / K, c = e - r * K;
      out[((size_t)tile * 32 + r) * K + c] = load_logit(red_base, r, c) + b[c];
    }
    __syncthreads();
  }
}

void launch_logits(int FP, int K, const uint16_t* X, int T, const uint16_t* wf_hi, const uint16_t* wf_lo,
                   const float* b, float* logits, hipStream_t s) {
  const size_t lds = eval_lds_bytes(FP);
  const int ntiles = (T + 31) / 32;
  const int grid = ntiles < 1024 ? ntiles : 1024;
  if (grid <= 0) return;
#define PSX_LG(FPV)                                                                      \
  case FPV:                                                                              \
    logits_kernel<FPV><<<grid, 256, lds, s>>>(K, X, T, wf_hi, wf_lo, b, logits); \
    break;
  switch (FP) {
    PSX_LG(128)
    PSX_LG(256)
    PSX_LG(512)
    PSX_LG(1024)
    PSX_LG(2048)
    default:
      break;
  }
#undef PSX_LG
}

// ---------------------------------------------------------------------------
// K7: server update w += lr * delta over ALL P entries (the reference skips the
// last intercept, quirk Q1) + bf16 hi/lo fragments for the server-side eval.
__global__ __launch_bounds__(256) void server_apply_kernel(int K, int F, int FP, float* w,
                                                           const float* __restrict__ delta, float lr,
                                                           uint16_t* wf_hi, uint16_t* wf_lo, float* b_eff,
                                                           int apply) {
  const int P = K * FP + K, KF = K * FP;
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= P) return;
  float v = w[p];
  if (apply) {
    v += lr * delta[p];
    w[p] = v;
  }
  if (p < KF) {
    const int c = p / FP, f = p - c * FP;
    write_frag(wf_hi, wf_lo, c, f, f < F ? v : 0.f);
  } else {
    b_eff[p - KF] = v;
  }
}

void launch_server_apply(int K, int F, int FP, float* w, const float* delta, float lr, uint16_t* wf_hi,
                         uint16_t* wf_lo, float* b_eff, hipStream_t s) {
  const int P = K * FP + K;
  server_apply_kernel<<<(P + 255) / 256, 256, 0, s>>>(K, F, FP, w, delta, lr, wf_hi, wf_lo, b_eff, 1);
}

void launch_make_fragments(int K, int F, int FP, const float* w, uint16_t* wf_hi, uint16_t* wf_lo, float* b_eff,
                           hipStream_t s) {
  const int P = K * FP + K;
  server_apply_kernel<<<(P + 255) / 256, 256, 0, s>>>(K, F, FP, const_cast<float*>(w), nullptr, 0.f, wf_hi, wf_lo,
                                                      b_eff, 0);
}

// ---------------------------------------------------------------------------
// K1/K10: ring ingest (gather of round-robin rows into consecutive ring slots).
__global__ __launch_bounds__(256) void ring_ingest_kernel(const uint16_t* __restrict__ src,
                                                          const int32_t* __restrict__ ysrc, int64_t src_first,
                                                          int64_t src_step, int64_t n, uint16_t* ring,
                                                          int32_t* yring, int64_t dst_first, int64_t cap, int FP) {
  const int CPR = FP / 8;
  const int64_t total = n * CPR;
  for (int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x; q < total; q += (int64_t)gridDim.x * 256) {
    const int64_t i = q / CPR;
    const int cg = (int)(q - i * CPR);
    const int64_t sr = src_first + i * src_step;
    int64_t dr = dst_first + i;
    dr %= cap;
    *(u16x8*)(ring + dr * FP + cg * 8) = *(const u16x8*)(src + sr * FP + cg * 8);
    if (cg == 0) yring[dr] = ysrc[sr];
  }
}

// Allow the wide tiles to use more than the default 64 KiB of dynamic LDS
// (gfx950: 160 KiB per CU).  Must run before any launch / graph capture.
template <int FP>
static void set_lds_attr() {
  const int bytes = (int)eval_lds_bytes(FP);
  (void)hipFuncSetAttribute((const void*)eval_kernel<FP>, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  (void)hipFuncSetAttribute((const void*)test_eval_kernel<FP>, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  (void)hipFuncSetAttribute((const void*)logits_kernel<FP>, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
}

void prepare_kernels() {
  static bool done = false;
  if (done) return;
  set_lds_attr<128>();
  set_lds_attr<256>();
  set_lds_attr<512>();
  set_lds_attr<1024>();
  set_lds_attr<2048>();
  done = true;
}

void launch_ring_ingest(const uint16_t* src, const int32_t* ysrc, int64_t src_first, int64_t src_step, int64_t n,
                        uint16_t* ring, int32_t* yring, int64_t dst_first, int64_t cap, int FP, hipStream_t s) {
  if (n <= 0) return;
  const int64_t total = n * (FP / 8);
  int64_t grid = (total + 255) / 256;
  if (grid > 2048) grid = 2048;
  ring_ingest_kernel<<<(int)grid, 256, 0, s>>>(src, ysrc, src_first, src_step, n, ring, yring, dst_first, cap, FP);
}

}  // namespace psx
