// Evaluation, server-update and ingest kernels for the logistic-regression
// parameter server (gfx950 / CDNA4).
//
// Reference math being replaced (Spark MLlib local mode / boxed HashMaps):
//   * server update w += (1/N) delta (ServerProcessor.java:148-151, 225-228)
//   * test-set predict + weighted F1/accuracy (LogisticRegressionTaskSpark.java:
//     236-251, Metrics.java:15-24)
//   * buffer insert (WorkerSamplingProcessor.java:110-112)
//
// Layout conventions (device):
//   X rows   : bf16 [rows][FP], FP = features padded to a multiple of 128
//   vectors  : fp32 [P] with P = K*FP + K: coefficient (c, f) at c*FP + f,
//              intercept c at K*FP + c
//   W frags  : bf16 hi/lo [FP/8][16][8]: element (c, f) at ((f>>3)*16+c)*8+(f&7),
//              the B-operand fragment order of v_mfma_f32_16x16x32_bf16.
#include <hip/hip_runtime.h>

#include "eval_body.h"
#include "lr_kernels.h"
#include "solve_kernels.h"
#include "tile.h"

namespace psx {

bool fp_supported(int FP) { return FP == 128 || FP == 256 || FP == 512 || FP == 1024 || FP == 2048; }

// ---------------------------------------------------------------------------

// ---------------------------------------------------------------------------
// K8/K9: test-set argmax + confusion matrix (LDS counts, one global atomic per
// non-zero cell per workgroup).  With an EvalSlot destination the workgroups
// accumulate into a private device accumulator, and the last one to arrive
// (ticket after draining its memory-side atomics) reads-and-zeroes it, writes
// the counts (+ the worker's loss) into the pinned host slot, and publishes the
// record's sequence number with a system-scope release store -- the host-side
// MetricsSink picks it up with no copy, event or fill launch.
//
// The model's classes sit at columns [coff1, coff1 + K) of the fragments.
// Paired mode (slot2 != nullptr): the 16 MFMA columns carry TWO models -- the
// worker's locally trained model at [coff1, coff1 + K) and the server's global
// model at [coff2, coff2 + K) of the same fragment buffer -- so the worker row
// of this round and the server row of the previous round cost one pass over
// the test set instead of two.
//
// eval_apply (ea.shi != nullptr): the server model's columns come from their own
// fragment buffer, and the launch also performs the round's server update into
// the other buffer of the server's pair (see lr_kernels.h: EvalApply) -- one
// launch per round for the worker row, the server row and the update.
template <int FP>
__global__ __launch_bounds__(256) void test_eval_kernel(EvalRide r, EvalApply ea) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  // workgroups [0, tgrid) evaluate test tiles; the extra workgroups [tgrid, grid)
  // perform the round's server update (independent of everything this launch
  // reads) on otherwise idle CUs, beside the evaluation
  const int tgrid = ea.tgrid > 0 ? ea.tgrid : gridDim.x;
  const int K = r.K;
  if (ea.dl.n > 0 && (int)blockIdx.x >= tgrid) {
    const int P = K * FP + K, KF = K * FP;
    for (int p = (blockIdx.x - tgrid) * 256 + threadIdx.x; p < P; p += (gridDim.x - tgrid) * 256) {
      float sum = 0.f;
      for (int i = 0; i < ea.dl.n; ++i) sum += ea.dl.p[i][p];
      const float v = ea.w[p] + ea.lr * sum;
      ea.w[p] = v;
      if (p < KF) {
        const int c = p / FP, f = p - c * FP;
        write_frag(ea.ohi, ea.olo, r.coff2 + c, f, f < ea.F ? v : 0.f);
      } else {
        ea.ob[r.coff2 + p - KF] = v;
      }
    }
  }
  const int ntiles = (int)blockIdx.x < tgrid ? r.ntiles() : 0;
  eval_body<FP>(lds, r, blockIdx.x, tgrid, ntiles);  // every workgroup arrives at the ticket
}

void launch_test_eval(int FP, int K, const uint16_t* Xt, const int32_t* yt, int T, const uint16_t* wf_hi,
                      const uint16_t* wf_lo, const float* b, int* conf, hipStream_t s, unsigned* ticket, void* slot,
                      const float* loss, unsigned long long seq, int coff1, int coff2, void* slot2,
                      unsigned long long seq2) {
  EvalApply none{};
  launch_eval_apply(FP, K, Xt, yt, T, wf_hi, wf_lo, b, conf, s, ticket, slot, loss, seq, coff1, coff2, slot2, seq2,
                    none);
}

void launch_eval_apply(int FP, int K, const uint16_t* Xt, const int32_t* yt, int T, const uint16_t* wf_hi,
                       const uint16_t* wf_lo, const float* b, int* conf, hipStream_t s, unsigned* ticket, void* slot,
                       const float* loss, unsigned long long seq, int coff1, int coff2, void* slot2,
                       unsigned long long seq2, const EvalApply& ea) {
  const size_t lds = eval_lds_bytes(FP);
  const int ntiles = (T + 31) / 32;
  const int tgrid = ntiles < 1024 ? ntiles : 1024;
  int grid = tgrid;
  EvalApply a = ea;
  a.tgrid = tgrid;
  if (ea.dl.n > 0) grid += (K * FP + K + 255) / 256;  // update workgroups
  if (grid <= 0) return;
  EvalRide r{};
  r.Xt = Xt;
  r.yt = yt;
  r.T = T;
  r.K = K;
  r.whi = wf_hi;
  r.wlo = wf_lo;
  r.wb = b;
  r.shi = ea.shi;
  r.slo = ea.slo;
  r.sb = ea.sb;
  r.coff1 = coff1;
  r.coff2 = coff2;
  r.acc = conf;
  r.ticket = ticket;
  r.slot = static_cast<char*>(slot);
  r.loss = loss;
  r.seq = seq;
  r.slot2 = static_cast<char*>(slot2);
  r.seq2 = seq2;
  r.nticket = (unsigned)grid;
#define PSX_TE(FPV)                                             \
  case FPV:                                                     \
    test_eval_kernel<FPV><<<grid, 256, lds, s>>>(r, a);         \
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
#define PSX_LG(FPV)                                                                  \
  case FPV:                                                                          \
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
                                                           int apply, int coff) {
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
    write_frag(wf_hi, wf_lo, coff + c, f, f < F ? v : 0.f);
  } else {
    b_eff[coff + p - KF] = v;
  }
}

// BSP round with N colocated workers: w += lr * (delta_0 + ... + delta_{n-1}) in ONE pass
// (instead of a copy + N-1 adds + the update), fragments refreshed.
__global__ __launch_bounds__(256) void server_apply_n_kernel(int K, int F, int FP, float* w, DeltaList dl, float lr,
                                                             uint16_t* wf_hi, uint16_t* wf_lo, float* b_eff,
                                                             int coff) {
  const int P = K * FP + K, KF = K * FP;
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= P) return;
  float sum = 0.f;
  for (int i = 0; i < dl.n; ++i) sum += dl.p[i][p];
  const float v = w[p] + lr * sum;
  w[p] = v;
  if (p < KF) {
    const int c = p / FP, f = p - c * FP;
    write_frag(wf_hi, wf_lo, coff + c, f, f < F ? v : 0.f);
  } else {
    b_eff[coff + p - KF] = v;
  }
}

void launch_server_apply_n(int K, int F, int FP, float* w, const DeltaList& dl, float lr, uint16_t* wf_hi,
                           uint16_t* wf_lo, float* b_eff, hipStream_t s, int coff) {
  const int P = K * FP + K;
  server_apply_n_kernel<<<(P + 255) / 256, 256, 0, s>>>(K, F, FP, w, dl, lr, wf_hi, wf_lo, b_eff, coff);
}

void launch_server_apply(int K, int F, int FP, float* w, const float* delta, float lr, uint16_t* wf_hi,
                         uint16_t* wf_lo, float* b_eff, hipStream_t s, int coff) {
  const int P = K * FP + K;
  server_apply_kernel<<<(P + 255) / 256, 256, 0, s>>>(K, F, FP, w, delta, lr, wf_hi, wf_lo, b_eff, 1, coff);
}

void launch_make_fragments(int K, int F, int FP, const float* w, uint16_t* wf_hi, uint16_t* wf_lo, float* b_eff,
                           hipStream_t s, int coff) {
  const int P = K * FP + K;
  server_apply_kernel<<<(P + 255) / 256, 256, 0, s>>>(K, F, FP, const_cast<float*>(w), nullptr, 0.f, wf_hi, wf_lo,
                                                      b_eff, 0, coff);
}

// ---------------------------------------------------------------------------
// K1/K10: ring ingest (gather of round-robin rows into consecutive ring slots).
// Rows land in the row-major ring (16-B chunks) and, when XT is given, in the
// feature-major copy: each thread owns one 8-feature chunk of one row and
// writes its 8 values to 8 feature rows of XT (the bwd/stats kernels then read
// every 32-feature slice of a window contiguously).
__global__ __launch_bounds__(256) void ring_ingest_kernel(const uint16_t* __restrict__ src,
                                                          const int32_t* __restrict__ ysrc, int64_t src_first,
                                                          int64_t src_step, int64_t n, uint16_t* ring,
                                                          uint16_t* ringT, int32_t* yring, int64_t dst_first,
                                                          int64_t cap, int FP) {
  const int CPR = FP / 8;
  const int64_t total = n * CPR;
  for (int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x; q < total; q += (int64_t)gridDim.x * 256) {
    // consecutive threads take consecutive ROWS of one chunk, so the 2-B XT
    // stores of a wave land in contiguous runs of each feature row
    const int cg = (int)(q / n);
    const int64_t i = q - (int64_t)cg * n;
    const int64_t sr = src_first + i * src_step;
    const int64_t dr = (dst_first + i) % cap;
    const u16x8 v = *(const u16x8*)(src + sr * FP + cg * 8);
    *(u16x8*)(ring + dr * FP + cg * 8) = v;
    if (ringT) {
#pragma unroll
      for (int e = 0; e < 8; ++e) ringT[(int64_t)(cg * 8 + e) * cap + dr] = v[e];
    }
    if (cg == 0) yring[dr] = ysrc[sr];
  }
}

void launch_ring_ingest(const uint16_t* src, const int32_t* ysrc, int64_t src_first, int64_t src_step, int64_t n,
                        uint16_t* ring, uint16_t* ringT, int32_t* yring, int64_t dst_first, int64_t cap, int FP,
                        hipStream_t s) {
  if (n <= 0) return;
  const int64_t total = n * (FP / 8);
  int64_t grid = (total + 255) / 256;
  if (grid > 2048) grid = 2048;
  ring_ingest_kernel<<<(int)grid, 256, 0, s>>>(src, ysrc, src_first, src_step, n, ring, ringT, yring, dst_first, cap,
                                               FP);
}

// ---------------------------------------------------------------------------
// Allow the wide tiles to use more than the default 64 KiB of dynamic LDS
// (gfx950: 160 KiB per CU).  Must run before any launch / graph capture.
template <int FP>
static void set_lds_attr() {
  const int bytes = (int)eval_lds_bytes(FP);
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
  prepare_solve_kernels();
  done = true;
}

}  // namespace psx
