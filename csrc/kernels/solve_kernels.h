// Fused local-solve kernels (see solve_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lr_kernels.h"
#include "solver_ctrl.h"

namespace psx {

// Device pointers of one solver instance (passed by value as a kernel argument).
struct SolveDev {
  const uint16_t* X;    // ring [cap][Fp] bf16
  const uint16_t* XT;   // the same ring feature-major [Fp][cap] (cap % 32 == 0)
  const int32_t* y;     // ring labels
  const float* w_old;   // [P]
  float *x, *d, *g_c;   // [P] iterate, direction, gradient at x
  float *S, *Y;         // [hist][P] curvature pairs
  float *std_, *inv_std;  // [Fp]
  float* wfix;          // [P] frozen contributions (zero-variance features, non-Spark mode)
  float* b_eff;         // [16] trial intercepts
  uint16_t *whi, *wlo;  // trial weight fragments [16*Fp]
  unsigned short* R;          // [tiles][2][16][32] bf16 hi/lo residuals (fwd -> bwd)
  float* part;                // [fwd grid][32] per-workgroup intercept-gradient / loss partials
  unsigned long long* xch;    // bwd_update_kernel cross-workgroup exchange words
  // outputs
  float* delta;
  float* w_new;
  uint16_t *out_hi, *out_lo;
  float* b_fin;
  float* loss;
  int* stats;
  // padded internal layout: KP classes (power of two >= K), feature stride FPI
  int KP, FPI, PI, pad_;
  long long* dbg;  // optional phase timeline (debug)
  unsigned* prm_count;  // runs completed (finalize advances it): all-gather tag base
  // large-window ("rows") mode: row-parallel fused forward+backward with
  // per-workgroup partials instead of the feature-major ring copy XT
  float* gpart;   // [G][KP][FP] partial gradients (raw sums of R^T X)
  double* spart;  // [G][2][FP] partial column sums / sums of squares
  float* gred;    // [KP][FPI] reduced gradient sums (bwd_update reads them when non-null)
  const float* Xf;  // fp32 ring rows [cap][Fp] (cfg.xf32; X is then unused)
  // feature-major gradient partials [fwd workgroup][FP][KP] (the "gpf" backward of
  // the small-window solve: each forward workgroup's R^T X of its LDS tile; the
  // slice owners reduce them with 16-B loads).  nullptr: the XT backward.
  float* gpf;
  // optional server update fused into the finalisation (a colocated server whose
  // model is this worker's pulled w_old, e.g. BSP with one worker): ap_w (may be
  // w_old itself) = w_old + ap_lr * delta, fragments at columns ap_coff of
  // (ap_hi, ap_lo, ap_b).  ap_w == nullptr: no update.
  float* ap_w;
  uint16_t *ap_hi, *ap_lo;
  float* ap_b;
  float ap_lr;
  int ap_coff;
  // pinned host word (nullptr: none): a solve whose cross-workgroup wait timed
  // out stores ((run + 1) << 8 | code) there, so host loops notice without a sync
  unsigned long long* err_host;
  int spin_max;  // cross-workgroup wait budget in polls (0: 2^22)
  int pad_sd;
};

// Server update fused into a solve (see SolveDev::ap_w).
struct FusedApply {
  float* w = nullptr;
  float lr = 1.f;
  uint16_t *hi = nullptr, *lo = nullptr;
  float* b = nullptr;
  int coff = 0;
};

int padded_classes(int K);
int padded_stride(int FP);
void prepare_solve_kernels();
size_t stats_prep_lds_bytes();
size_t fwd_lds_bytes(int FP);
size_t bwd_lds_bytes();
int bwd_grid(int FP);
int xch_words();
void launch_stats_prep(const SolverCfg& cfg, SolveParams* prm, const SolveDev& dv, Ctrl* ctrl, int B, int start,
                       const RingIngest& ing, hipStream_t s);
const void* stats_prep_symbol();
void launch_finalize(const SolverCfg& cfg, const Ctrl* ctrl, const SolveDev& dv, hipStream_t s);
// win.B > 0: the window as kernel arguments (eager launches); otherwise the
// kernels read it from prm (graph replays).
// fin_slot: a bwd_update launch of slot >= fin_slot that ends the solve finalises
// its slice in place (the tail / finalize launch then writes the scalars only);
// riding evaluation workgroups must all be in launches of earlier slots.
void launch_slot(const SolverCfg& cfg, const SolveParams* prm, Ctrl* ctrl, int slot, const SolveDev& dv, int nwg,
                 hipStream_t s, const SolveParams& win, int fin_slot = kNoFinSlot);
// Line-search retry slots [slot_begin, slot_end) in one persistent launch.
// with_finalize: the finalisation runs inside the tail launch (no separate finalize node).
void launch_tail(const SolverCfg& cfg, const SolveParams* prm, Ctrl* ctrl, int slot_begin, int slot_end,
                 const SolveDev& dv, int nwg, hipStream_t s, int with_finalize = 0);
size_t tail_lds_bytes(int FP);
int tail_grid(int FP, int nwg);

// ---- large-window ("rows") mode: every pass over the window is row-parallel
// over G workgroups (no XT copy, no residual buffer); see solve_kernels.hip ----
// Windows of more than this many ring rows use it (PSX_SOLVER_ROWS=0/1 forces).
constexpr int kRowsModeMinCap = 8192;
// rows-mode grids up to this many workgroups reduce their partials inside bwd_update
constexpr int kRowsReduceInBwd = 64;
bool rows_mode_for(int cap);
void launch_stats_rows(const SolverCfg& cfg, SolveParams* prm, const SolveDev& dv, int B, int start, int G,
                       hipStream_t s);
void launch_prep_rows(const SolverCfg& cfg, const SolveParams* prm, const SolveDev& dv, Ctrl* ctrl, int G,
                      hipStream_t s);
void launch_fwdbwd_rows(const SolverCfg& cfg, const SolveParams* prm, const Ctrl* ctrl, int slot, const SolveDev& dv,
                        int G, hipStream_t s);
void launch_reduce_g(const SolverCfg& cfg, const SolveParams* prm, const Ctrl* ctrl, const SolveDev& dv, int G,
                     hipStream_t s);
void launch_bwd(const SolverCfg& cfg, const SolveParams* prm, Ctrl* ctrl, int slot, const SolveDev& dv, int fwd_grid,
                hipStream_t s, const SolveParams& win);
// One function-evaluation slot (fwd + bwd_update launches) with `nride` extra
// workgroups in the bwd_update launch evaluating test tiles [ride_t0, ride_t0 +
// nride) of `ride` (see EvalRide, lr_kernels.h); nride == 0: none.
void launch_slot_ride(const SolverCfg& cfg, const SolveParams* prm, Ctrl* ctrl, int slot, const SolveDev& dv, int nwg,
                      hipStream_t s, const SolveParams& win, const struct EvalRide& ride, int ride_t0, int nride,
                      int fin_slot = kNoFinSlot);
size_t stats_rows_lds_bytes();

// ---- persistent small-window solve: every slot and the finalisation in ONE
// launch after launch_stats_prep (see solve_kernels.hip); G = persist_grid(FP,
// window tiles) co-resident workgroups (on XCD cfg.xcd when G <= 32) + `nride`
// evaluation workgroups of `ride` (tiles [0, nride)) ----
bool persist_supported(int FP, int KP);
int persist_grid(int FP, int ntiles);
size_t persist_lds_bytes(int FP);
void launch_persist(const SolverCfg& cfg, const SolveDev& dv, Ctrl* ctrl, const SolveParams& win, int G,
                    const EvalRide& ride, int nride, hipStream_t s);
// fp32 ring rows: rows src_first + i*src_step -> slots (dst_first + i) % cap
void launch_ring_ingest_f32(const float* src, const int32_t* ysrc, int64_t src_first, int64_t src_step, int64_t n,
                            float* ring, int32_t* yring, int64_t dst_first, int64_t cap, int FP, hipStream_t s);

}  // namespace psx
