// Wide / sparse logistic regression on gfx950: CSR feature rows, a dense
// weight vector of F*KP + KP floats (F up to ~10^8 hashed features).
//
// BASELINE.json configs 4 (10M rows x 1M sparse features, ASP) and 5 (sharded
// 100M-dim dense weight vector).  The reference has no sparse path: its worker
// densifies 1024 hashed features into Spark rows
// (LogisticRegressionTaskSpark.java:146-162) and the server loops over a boxed
// HashMap (ServerProcessor.java:148-151).  The MI355X design:
//
//  * the window of a worker touches only U << F features, so the local solve
//    runs in that U-dimensional subspace: a plan pass gives every distinct
//    feature of the window a compact local id (wave-aggregated atomics), the
//    old weights of those features are gathered once, and every L-BFGS vector
//    (x, d, g, S_i, Y_i) is KP + U*KP floats instead of F*KP;
//  * hashed text is Zipf-distributed: the few hottest features occur in most
//    rows, and one global atomic per occurrence serialises on their cache
//    lines.  The plan therefore groups the window's rows RB at a time and
//    dedups each group's features in an LDS hash table once per solve; every
//    later pass (feature sums, gradients) accumulates per group in LDS and
//    issues ONE global atomic per (group, feature);
//  * one wavefront per row: lanes gather the row's non-zeros, the K margins are
//    reduced across the wave, softmax / cross-entropy in registers, and the
//    same wave adds the row's gradient into its group's LDS accumulators
//    (forward and backward fused, no residual round trip);
//  * the line-search / L-BFGS control is the same on-device state machine as
//    the dense solver (solver_ctrl.h), advanced by the last workgroup of the
//    dot-product reduction; the whole solve is one hipGraph replay;
//  * the output is sparse (U ids + U*KP deltas) with an optional dense scatter
//    for the collective schedules.
//
// Device layouts:
//   dense weights / deltas : [F][KP] coefficient (f, c) at f*KP + c, then KP
//                            intercepts at F*KP + c (classes c >= K stay 0)
//   local vectors          : KP intercepts first, then feature l at KP + l*KP
//   ring (ELL)             : idx [cap][NZ] int32, val [cap][NZ] bf16,
//                            nnz [cap] int32, y [cap] int32
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "solver_ctrl.h"

namespace psx {

struct WideCfg {
  SolverCfg sc;       // iters / hist / ls_max / mode / nslots / gd_lr / tol (K F Fp P cap unused)
  int K;              // logits (1 = binary sigmoid model, >= 2 softmax incl. phantom class)
  int KP;             // padded classes: 1, 2, 4, 8 or 16
  int64_t F;          // features
  int cap;            // ring rows
  int NZ;             // ring entries per row (<= 512)
  int umax;           // max distinct features of a window = min(F, cap*NZ)
  int standardize;    // Spark's feature scaling by 1/std over the window
  int center;         // multinomial centring (Spark, regParam == 0)
  int zero_const;     // zero-std features get coefficient 0 (Spark) instead of keeping w_old
  int dense_delta;    // also scatter the delta into a dense [F*KP + KP] vector
  // key-range pull mode (csrc/runtime/keyrange_loop.h): the old weights of the
  // window's features arrive as w_pull [U][KP] in local-id order, and the local
  // ids are grouped by owner rank min(f / own_S, own_W - 1) (own_W > 1)
  int pulled;
  int own_W;
  int64_t own_S;
  // the whole solve in one persistent launch (wide_persist_kernel) instead of the
  // launch chain; only for a solver alone on the GPU (its workgroups must be co-resident)
  int persist;
};

constexpr int kMaxOwners = 64;

// Feature -> local id of the window: open-addressing table of H = pow2 >=
// 2*umax int2 entries {feature, local id} (key -1 = empty).  Sized by the
// window, not by F, so a 10^8-feature model carries no F-sized index.
__device__ __forceinline__ unsigned wide_gslot(int f, unsigned mask) {
  unsigned x = (unsigned)f;
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x & mask;
}

__device__ __forceinline__ int wide_find(const int2* __restrict__ tab, unsigned mask, int f) {
  unsigned h = wide_gslot(f, mask);
  while (true) {
    const int2 e = tab[h];
    if (e.x == f) return e.y;
    if (e.x == -1) return -1;
    h = (h + 1) & mask;
  }
}

struct WideParams {
  int B, start, pad0, pad1;
};

// Everything the solve kernels touch (device pointers; passed by value).
struct WideDev {
  // ring (caller-owned)
  const int32_t* ridx;
  const uint16_t* rval;
  const int32_t* rnnz;
  const int32_t* ry;
  const float* w_old;  // dense pulled weights [F*KP + KP] (null in pull mode)
  const float* w_pull;    // pull mode: [umax][KP] old weights of local id i
  const float* w_pull_b;  // pull mode: [KP] old intercepts
  // workspace
  WideParams* prm;
  Ctrl* ctrl;
  unsigned* cnt;       // [0] U, [1] dots ticket, [2] U of the previous solve, [3] tail barrier error
  int2* htab;          // [H] {feature, local id} (see wide_find)
  unsigned hmask;      // H - 1
  int32_t* hslot;      // [umax] table slot of local id i (cleared by the next solve's begin)
  int32_t* uniq;       // [umax] local id -> feature
  int32_t* uniq_alt;   // [umax] owner-order scratch (pull mode with own_W > 1)
  unsigned* own;       // [2 * kMaxOwners] per-owner counts, then cursors
  int32_t* lid;        // [cap*NZ] window entry -> local id
  // block plan (built once per solve): window rows are processed in groups of
  // RB rows; every group dedups its entries' features in LDS so that hot
  // features cost one global atomic per group instead of one per row
  uint16_t* pslot;     // [cap*NZ] window entry -> distinct slot within its group
  int32_t* bfeat;      // [ngroups][EB] distinct features of a group
  int32_t* blid;       // [ngroups][EB] their local ids
  int32_t* bcount;     // [ngroups] distinct features per group
  int RB, EB, TS;      // rows per group, EB = RB*NZ, LDS hash size (pow2 >= 2*EB)
  unsigned long long* gbar;  // grid-barrier counter of the tail launch (reset per solve)
  unsigned* pbar;            // [2] self-resetting grid barrier of the persistent solve: count, generation
  float* s1;           // [umax] feature sums over the window
  float* s2;           // [umax] feature sums of squares
  float* scale;        // [umax] effective coefficient = scale * x
  float* gscale;       // [umax] gradient scale (0 for frozen features)
  float *x, *d, *g_t, *g_c, *w0;  // [PLmax]
  float *S, *Y;        // [hist][PLmax]
  double* part;        // [nblk][kWideND] dot partials
  double* loss_acc;    // [nslots]
  // outputs (caller-owned)
  float* dloc;         // [PLmax] local delta (intercepts first)
  float* wloc;         // [PLmax] local new weights
  float* loss;         // [1]
  int* stats;          // [4] evals, accepted steps, ls failures, direction resets
  float* delta_dense;  // [F*KP + KP] (dense_delta)
  long long* dbg;      // [nslots][8] s_memrealtime stamps of the dots kernel (PSX_WIDE_STAMPS), or null
  unsigned* host_u;    // pinned host mirror of U (optional)
  int64_t PLmax;
};

constexpr int kWideND = 3 + 2 * kMaxHist;

// Rows per group of the block plan for ring rows of NZ entries and KP classes
// (LDS budgets: hash 8*TS + 4*EB bytes in the plan kernel, EB*KP*4 in fwdbwd).
int wide_rows_per_group(int NZ, int KP);

// Launchers (stream order; the solver captures them into one hipGraph).
void wide_launch_begin(const WideCfg& c, const WideDev& d, int B, int start, hipStream_t s);  // cleanup + params
// plan: window features -> local ids (+ owner order in pull mode); the old
// weights are read from here on (prepare: assign, stats, prep)
void wide_launch_plan(const WideCfg& c, const WideDev& d, hipStream_t s);
void wide_launch_prepare(const WideCfg& c, const WideDev& d, hipStream_t s);
void wide_launch_slot(const WideCfg& c, const WideDev& d, int slot, int nblk_dots, hipStream_t s);
// Line-search retry slots [s0, s1) in one persistent launch (grid barriers).
void wide_launch_tail(const WideCfg& c, const WideDev& d, int s0, int s1, hipStream_t s);
void wide_prepare_kernels();  // LDS attributes of the tail kernels (call before capture)
// The solve (phases 3) or one of its phases (1: begin + plan, 2: the rest) in one
// persistent launch of wide_persist_grid() co-resident workgroups.
void wide_launch_persist(const WideCfg& c, const WideDev& d, int B, int start, int phases, hipStream_t s);
int wide_persist_grid();
void wide_launch_finalize(const WideCfg& c, const WideDev& d, hipStream_t s);
int wide_dots_blocks(int64_t PLmax);
size_t wide_persist_lds(const WideCfg& c, const WideDev& d);

// ---------------------------------------------------------------------------
// Wide lanes: the local solves of up to kWideMaxLanes in-process workers in ONE
// launch, lane l on the `per` XCDs xcd0 + l * per .. with per * kWideLaneWg
// co-resident workgroups (the persistent solve's phases; per = 8 / L, so fewer
// workers still fill the GPU).  Workgroups claim their lane from their XCC_ID
// (lanes_kernels.hip's claim), so the dispatch order of the grid does not matter.  devs: [L] WideDev table in device memory (each
// lane's own workspace and ring; w_old = the server weights every lane pulled).
constexpr int kWideMaxLanes = 8;
constexpr int kWideLaneWg = 32;
struct WideLanesArgs {
  int L;
  int xcd0;
  int per;          // XCDs per lane (L * per <= 8 - xcd0)
  int gpx;          // workgroups per XCD and lane: 32 x the CU's co-resident lane workgroups (1 or 2)
  unsigned* claim;  // [2][16] per-lane slot counters; launch parity cpar, the other one cleared
  int cpar;
  int B[kWideMaxLanes];
  int start[kWideMaxLanes];
  // the evaluation's overlay table (WideEvalModels::pres / ov, lidt [F][kWideMaxLanes]),
  // built by each lane right after its finalisation (null: not built here); the table
  // must be clear (every pres word 0) at launch
  unsigned* pres;
  float* ov;
  int* lidt;
};
void wide_launch_lanes(const WideCfg& c, const WideDev* devs, const WideLanesArgs& a, size_t lds, hipStream_t s);
int wide_lanes_grid(int gpx);
// co-resident lane workgroups per CU of the lanes kernel for this configuration (LDS,
// registers), capped at 2 -- a lane may only count on workgroups that ARE co-resident
int wide_lanes_per_cu(const WideCfg& c, size_t lds);
// bm [L][nw] (nw = (F + 31) / 32 words, zeroed by the caller): bit f of lane l set for
// every feature of lane l's last window (devs[l].uniq[0 .. U))
void wide_lanes_bitmap(const WideDev* devs, int L, unsigned* bm, int64_t nw, hipStream_t s);
// the overlay table of the lanes' last windows (set: pres bits + rows + local ids lidt
// [F][kWideMaxLanes]; clear: pres words of those features back to 0 -- the rows need no
// clearing, pres guards them)
void wide_lanes_overlay(const WideDev* devs, int L, int KP, unsigned* pres, float* ov, int* lidt, bool set,
                        hipStream_t s);
// the lanes' pushes in order ord[0 .. n) in one launch, reading the overlay table (which it
// clears): one thread per window feature adds the deltas in that order (= one launch per
// push, bit for bit); needs the table of THESE solves (wide_lanes_overlay set)
struct WideLanesOrder {
  int n;
  int ord[kWideMaxLanes];
};
void wide_lanes_apply(const WideDev* devs, int L, const WideLanesOrder& o, int64_t F, int KP, float* w, float lr,
                      unsigned* pres, const int* lidt, hipStream_t s);

// Test-set evaluation of up to kWideMaxEval models of the wide model in ONE pass:
// model m < nov = the common weights w overlaid with lane m's window solution
// (htab / hmask / wloc, the worker row of a lane), and with `plain` one more model, w
// itself (a server row).  Each non-zero's row of w is gathered once.  The last
// workgroup publishes every model's counts into its pinned EvalSlot (+ the loss).
constexpr int kWideMaxEval = kWideMaxLanes + 1;
struct WideEvalModels {
  int nov;    // overlay models
  int plain;  // 1: model nov is w itself
  // optional [nov][nw] bitmaps of the overlays' window features (wide_lanes_bitmap): a
  // table is probed only for a feature whose bit is set (null: always probed)
  const unsigned* bm;
  int64_t nw;
  // optional overlay table (wide_lanes_overlay): pres[f] bit j = f is in lane j's window,
  // ov[(f * kWideMaxLanes + j) * KP ..] = lane j's local coefficients of f; replaces the
  // bitmaps and table probes (one presence word + one contiguous row block per non-zero)
  const unsigned* pres;
  const float* ov;
  const int2* htab[kWideMaxLanes];
  unsigned hmask[kWideMaxLanes];
  const float* wloc[kWideMaxLanes];
  const float* loss[kWideMaxEval];
  char* slot[kWideMaxEval];
  unsigned long long seq[kWideMaxEval];
};
// acc: [kWideEvalCopies][kWideMaxEval][256] cells at stride kAccStride (zero between
// passes): workgroup b adds into copy b % kWideEvalCopies -- one copy took every
// workgroup's atomics on the same 9 x 36 cells, serialised (135 us for 9 models)
constexpr int kWideEvalCopies = 8;
void launch_wide_eval_multi(int K, int KP, int64_t F, const int64_t* indptr, const int32_t* idx, const uint16_t* val,
                            const int32_t* y, int T, const float* w, const WideEvalModels& m, int* acc,
                            unsigned* ticket, hipStream_t s);

// Ring ingest: rows src_first + i*src_step of a CSR matrix (i < n) -> ring
// slots (dst_first + i) % cap; rows longer than NZ are truncated and counted
// in *trunc.
void launch_sparse_ring_ingest(const int64_t* indptr, const int32_t* idx, const uint16_t* val, const int32_t* y,
                               int64_t src_first, int64_t src_step, int64_t n, int32_t* ridx, uint16_t* rval,
                               int32_t* rnnz, int32_t* ry, int64_t dst_first, int cap, int NZ, int* trunc,
                               hipStream_t s);

// The same for several rings of one geometry (cap, NZ) fed from one dataset, in ONE
// launch: job q = rows src_first + i*src_step (i < n) -> its ring's slots (dst_first + i) % cap.
constexpr int kMaxIngestJobs = 16;
struct SparseIngestJob {
  int64_t src_first, src_step, n, dst_first;
  int32_t* ridx;
  uint16_t* rval;
  int32_t* rnnz;
  int32_t* ry;
  int* trunc;
};
struct SparseIngestJobs {
  int njobs, cap, NZ;
  SparseIngestJob job[kMaxIngestJobs];
};
void launch_sparse_ring_ingest_many(const int64_t* indptr, const int32_t* idx, const uint16_t* val, const int32_t* y,
                                    const SparseIngestJobs& a, hipStream_t s);

// Test-set evaluation of a dense wide model (optionally overlaid with a
// worker's local solution: features the solver's table htab maps to a local id
// l read wloc[KP + l*KP]).  Same EvalSlot protocol as launch_test_eval.
// Key-range form (w == nullptr): margins = zbase[r] (the reduced partial
// margins of the sharded model) + the overlay's entries + bias[0..KP).
void launch_wide_eval(int K, int KP, int64_t F, const int64_t* indptr, const int32_t* idx, const uint16_t* val,
                      const int32_t* y, int T, const float* w, const int2* htab, unsigned hmask, const float* wloc,
                      int* acc, unsigned* ticket, void* slot, const float* loss, unsigned long long seq, hipStream_t s,
                      void* slot2 = nullptr, unsigned long long seq2 = 0, const float* zbase = nullptr,
                      const float* bias = nullptr);
// Margins of T rows (tests): out[T][KP].
void launch_wide_logits(int K, int KP, int64_t F, const int64_t* indptr, const int32_t* idx, const uint16_t* val,
                        int T, const float* w, float* out, hipStream_t s);

// Server updates.  Sparse: w[uniq[l]*KP + c] += lr * dloc[KP + l*KP + c] for
// l < *U (device count) or U_host when U_dev is null, and the intercepts.
void launch_wide_apply_sparse(float* w, int64_t F, int KP, const unsigned* U_dev, int U_host, const int32_t* uniq,
                              const float* dloc, float lr, int umax, hipStream_t s);
// Sparse pull: append a push (uniq[U], dloc[(U+1)*KP]) to the server's ring log
// at id position pos (mod cap); a worker applies n received log ids / values.
void launch_log_append(const int32_t* uniq, const float* dloc, int U, int64_t F, int KP, int32_t* lids, float* lvals,
                       int64_t pos, int64_t cap, hipStream_t s);
void launch_log_apply(float* w, const int32_t* ids, const float* vals, int64_t n, int KP, float lr, hipStream_t s);
// Dense: w += lr * delta over n floats.
void launch_axpy(float* w, const float* delta, float lr, int64_t n, hipStream_t s);

}  // namespace psx
