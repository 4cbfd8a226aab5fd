// Host launchers for the multinomial logistic-regression kernels (gfx950).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "solver_ctrl.h"

namespace psx {

// Eval-kernel row tile and its dynamic LDS footprint for a padded width FP.
constexpr int kTileRows = 32;
inline size_t eval_lds_bytes(int FP) { return (size_t)kTileRows * FP * 2 + 8192 + 2048 + 512; }
bool fp_supported(int FP);
// Raise dynamic-LDS limits for the wide tile kernels (call before capture).
void prepare_kernels();

void launch_set_params(SolveParams* p, int B, int start, hipStream_t s);
void launch_stats(const uint16_t* X, const SolveParams* prm, int cap, int FP, double* acc, int row_blocks,
                  hipStream_t s);
void launch_prep(const SolverCfg& cfg, const SolveParams* prm, const double* acc, const float* w_old, float* x,
                 float* d, float* g_c, float* std_, float* inv_std, float* wfix, uint16_t* wf_hi, uint16_t* wf_lo,
                 float* b_eff, Ctrl* ctrl, int nrb, hipStream_t s);
void launch_eval(const SolverCfg& cfg, const SolveParams* prm, const Ctrl* ctrl, int slot, const uint16_t* X,
                 const int32_t* y, const uint16_t* wf_hi, const uint16_t* wf_lo, const float* b_eff, float* Gpart,
                 float* Rpart, float* Lpart, int nwg, hipStream_t s);
void launch_reduce(const SolverCfg& cfg, const SolveParams* prm, Ctrl* ctrl, int slot, const float* Gpart,
                   const float* Rpart, const float* Lpart, int nwg_eval, const float* inv_std, const float* d,
                   const float* g_c, float* g_t, const float* S, const float* Y, double* dotpart, hipStream_t s);
void launch_update(const SolverCfg& cfg, const Ctrl* ctrl, int slot, float* x, float* d, float* g_c,
                   const float* g_t, float* S, float* Y, const float* inv_std, const float* wfix, uint16_t* wf_hi,
                   uint16_t* wf_lo, float* b_eff, hipStream_t s);
void launch_finalize(const SolverCfg& cfg, const Ctrl* ctrl, const float* x, const float* inv_std,
                     const float* wfix, const float* w_old, float* delta, float* w_new, uint16_t* wf_hi,
                     uint16_t* wf_lo, float* b_fin, float* loss_out, int* stats_out, hipStream_t s);
// Test-set prediction + KxK confusion counts (conf must be zeroed, int[16*16]).
void launch_test_eval(int FP, int K, const uint16_t* Xt, const int32_t* yt, int T, const uint16_t* wf_hi,
                      const uint16_t* wf_lo, const float* b, int* conf, hipStream_t s);
// Server update w += lr * delta (all P entries) and refresh the eval fragments.
void launch_server_apply(int K, int F, int FP, float* w, const float* delta, float lr, uint16_t* wf_hi,
                         uint16_t* wf_lo, float* b_eff, hipStream_t s);
// Refresh fragments from w without updating (bootstrap / after a pull).
void launch_make_fragments(int K, int F, int FP, const float* w, uint16_t* wf_hi, uint16_t* wf_lo, float* b_eff,
                           hipStream_t s);
// Copy n rows (row i of the batch = src row src_first + i*src_step) into ring
// slots (dst_first + i) % cap, labels alongside.
void launch_ring_ingest(const uint16_t* src, const int32_t* ysrc, int64_t src_first, int64_t src_step, int64_t n,
                        uint16_t* ring, int32_t* yring, int64_t dst_first, int64_t cap, int FP, hipStream_t s);
// Dense predict/loss for arbitrary w (used by tests): loss (sum) and logits.
void launch_logits(int FP, int K, const uint16_t* X, int T, const uint16_t* wf_hi, const uint16_t* wf_lo,
                   const float* b, float* logits, hipStream_t s);

}  // namespace psx
