// Host launchers for the evaluation / server / ingest kernels (gfx950).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "solver_ctrl.h"

namespace psx {

// Row tile and dynamic LDS footprint of the tile kernels for a padded width FP.
constexpr int kTileRows = 32;
PSX_HD constexpr size_t eval_lds_bytes(int FP) { return (size_t)kTileRows * FP * 2 + 8192 + 2048 + 1024 + 512; }
bool fp_supported(int FP);
// Raise dynamic-LDS limits for the wide tile kernels (call before capture).
void prepare_kernels();


// Test-set prediction + KxK confusion counts (conf: zeroed int[16*16]).
// Confusion counts of the test set.  slot == nullptr: accumulate into conf
// (must be zeroed by the caller).  Otherwise conf is a private accumulator
// (zero, left zero) with its `ticket` word, and the counts + *loss land in the
// pinned host EvalSlot `slot`, published with sequence number `seq`.
struct DeltaList {
  const float* p[16];
  int n;
};

// Paired evaluation fused with the server update of the same round.
//   * worker row: the locally trained model, fragment columns [coff1, coff1+K)
//     of (whi, wlo, wb);
//   * server row (slot2 != nullptr): the global model of the PREVIOUS round,
//     columns [coff2, coff2+K) of (shi, slo, sb) -- a separate buffer;
//   * apply (dl.n > 0): w += lr * sum(dl) and the new global model's fragments
//     into (ohi, olo, ob) at coff2 -- the other buffer of the server's pair, so
//     nothing this launch reads is written.
struct EvalApply {
  const uint16_t *shi, *slo;
  const float* sb;
  float* w;
  DeltaList dl;
  float lr;
  uint16_t *ohi, *olo;
  float* ob;
  int F;
  int tgrid;  // workgroups evaluating test tiles (set by the launcher); the rest update
};
// One evaluation pass described as data, so that it can run either as its own
// launch (test_eval_kernel) or "ride" in spare workgroups of the worker's solve
// launches (bwd_update_kernel, see LocalSolver::run): the solve's latency-bound
// kernels leave >200 of the 256 CUs idle, and the test-set pass of the previous
// round fits beside them instead of adding a launch to the round.
//   * model 1: columns [coff1, coff1+K) of (whi, wlo, wb) -> counts acc[0..256)
//   * model 2 (slot2 != nullptr): columns [coff2, coff2+K), from (shi, slo, sb)
//     when shi != nullptr (else the same buffer) -> acc[256..512)
//   * slot != nullptr: the last of `nticket` arriving workgroups (over every
//     launch the pass spans) publishes the counts (+ *loss) to the pinned host
//     slot(s) with the sequence numbers; slot == nullptr: counts stay in acc.
struct EvalRide {
  const uint16_t* Xt;
  const int32_t* yt;
  int T, K;
  const uint16_t *whi, *wlo;
  const float* wb;
  const uint16_t *shi, *slo;
  const float* sb;
  int coff1, coff2;
  int* acc;
  unsigned* ticket;
  char* slot;
  const float* loss;
  unsigned long long seq;
  char* slot2;
  unsigned long long seq2;
  unsigned nticket;  // arriving workgroups that complete the pass
  PSX_HD int ntiles() const { return (T + kTileRows - 1) / kTileRows; }
};

void launch_eval_apply(int FP, int K, const uint16_t* Xt, const int32_t* yt, int T, const uint16_t* whi,
                       const uint16_t* wlo, const float* wb, int* conf, hipStream_t s, unsigned* ticket, void* slot,
                       const float* loss, unsigned long long seq, int coff1, int coff2, void* slot2,
                       unsigned long long seq2, const EvalApply& ea);
void launch_test_eval(int FP, int K, const uint16_t* Xt, const int32_t* yt, int T, const uint16_t* wf_hi,
                      const uint16_t* wf_lo, const float* b, int* conf, hipStream_t s, unsigned* ticket = nullptr,
                      void* slot = nullptr, const float* loss = nullptr, unsigned long long seq = 0, int coff1 = 0,
                      int coff2 = 0, void* slot2 = nullptr, unsigned long long seq2 = 0);
void launch_logits(int FP, int K, const uint16_t* X, int T, const uint16_t* wf_hi, const uint16_t* wf_lo,
                   const float* b, float* logits, hipStream_t s);
// Server update w += lr * delta (all P entries) and refresh the eval fragments.

// w += lr * sum_i dl.p[i] (all P entries) + fragments, one kernel (n <= 16).
void launch_server_apply_n(int K, int F, int FP, float* w, const DeltaList& dl, float lr, uint16_t* wf_hi,
                           uint16_t* wf_lo, float* b_eff, hipStream_t s, int coff = 0);
// coff: first class column of this model in the (shared) fragment buffer.
void launch_server_apply(int K, int F, int FP, float* w, const float* delta, float lr, uint16_t* wf_hi,
                         uint16_t* wf_lo, float* b_eff, hipStream_t s, int coff = 0);
void launch_make_fragments(int K, int F, int FP, const float* w, uint16_t* wf_hi, uint16_t* wf_lo, float* b_eff,
                           hipStream_t s, int coff = 0);
// Copy n rows (row i of the batch = src row src_first + i*src_step) into ring
// slots (dst_first + i) % cap, labels alongside.
// ringT (optional): feature-major copy [FP][cap] kept in step with the ring.
void launch_ring_ingest(const uint16_t* src, const int32_t* ysrc, int64_t src_first, int64_t src_step, int64_t n,
                        uint16_t* ring, uint16_t* ringT, int32_t* yring, int64_t dst_first, int64_t cap, int FP,
                        hipStream_t s);

}  // namespace psx
