// One BSP round of up to 8 in-process workers ("lanes") in ONE launch (gfx950).
//
// Reference round (sequential consistency, ServerProcessor.java:143-183 +
// WorkerTrainingProcessor.java:63-98, BaseKafkaApp.java:25 numWorkers workers in
// one process): every worker ingests its new tuples into its buffer
// (WorkerSamplingProcessor.java:50-113), fits the buffer from the pulled weights
// (LogisticRegressionTaskSpark.java:142-221: standardisation, 2 L-BFGS
// iterations, centring, delta), the server applies w += (1/N) * delta of every
// worker (ServerProcessor.java:148-151) and evaluates the global model; each
// worker also evaluates its local model (LogisticRegressionTaskSpark.java:186).
//
// MI355X mapping (lanes_kernels.hip):
//   * lane l (worker) owns XCD l: its <= 32 cooperating workgroups are blockIdx
//     8 i + l (blockIdx % 8 == XCC_ID), one per CU, so every hand-off of its
//     solve goes through that XCD's L2;
//   * phase I inside the launch: each row workgroup stages its ring tile -- the new
//     tuples straight from the resident dataset (and writes them into the ring) --
//     and publishes the tile's column sums; the slice owners reduce them (window
//     standardisation), form x0 and the first trial point: no separate ingest /
//     statistics launch;
//   * the slots (forward + R^T X | gradient slice, dots all-gather, controller,
//     update) and the finalisation exactly as the persistent solve
//     (solve_body.h);
//   * the BSP update: each lane's slice owner writes its delta slice write-through
//     and arrives on the slice's counter; the LAST lane to arrive sums the L deltas
//     in lane order and applies w += lr * sum (or writes the sum for an RCCL
//     reduce) plus the server's evaluation fragments -- nobody waits;
//   * the evaluation of the PREVIOUS round's models (L local models + the global
//     model: the reference's worker and server rows) runs in "rider" workgroups
//     on the XCDs no lane uses (and after the lanes when all 8 XCDs solve), from
//     double-buffered fragments, and publishes into the pinned metrics slots.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lr_kernels.h"
#include "solve_kernels.h"

namespace psx {

constexpr int kMaxLanes = 8;
constexpr int kLaneWg = 32;  // cooperating workgroups per lane: the CUs of one XCD
constexpr int kMaxEvalModels = kMaxLanes + 1;

// Per-lane device state (a device-resident table read by the lane's workgroups).
struct LaneDev {
  SolveDev dv;        // solver workspace + the lane's ring (dv.X, dv.y); dv.delta = delta
  float* spart;       // [32 tiles][FP][2] window column sums / sums of squares (phase I hand-off)
  uint16_t* ohi[2];   // local model fragments by round parity (class columns 0..K-1)
  uint16_t* olo[2];
  float* ob[2];
  float* loss2;       // [2] training loss by round parity
  Ctrl* ctrl;         // the lane's controller after the round (host diagnostics)
};

// Per-round arguments of one lane: the window and the new rows of this round:
// dataset rows first + i * step (i < n) into ring slots (dst + i) % cap, then (a
// delivery that wraps the worker's shard) first2 + i * step (i < n2) into slots
// (dst + n + i) % cap.
struct LaneRound {
  int B, start, n, dst;
  long long first, step, first2;
  int n2, pad;
};

struct EvalModel {
  const uint16_t *hi, *lo;  // fragments, class columns coff..coff+K-1
  const float* b;           // intercepts b[coff + c]
  int coff;                 // first class column of the model in its buffers
  const float* loss;        // worker rows: the training loss; nullptr: 0
  char* slot;               // pinned EvalSlot
  unsigned long long seq;
};

// Test-set evaluation of up to kMaxEvalModels models in one pass over the test
// tiles: models are paired (model 2j in MFMA columns 0..7, 2j+1 in 8..15).
struct EvalMulti {
  const uint16_t* Xt;
  const int32_t* yt;
  int T, K;
  int nmodels;  // 0: nothing to evaluate
  EvalModel m[kMaxEvalModels];
  int* acc;          // [kMaxEvalModels][256] private accumulators (stride kAccStride), zero between passes
  unsigned* ticket;  // arrivals of the riders (reset by the last)
  unsigned nticket;
  // PSX_LANES_STAMPS: s_memrealtime stamps of the riders (nullptr: none): [0] rider 0
  // enters, [1] its first tile staged, [2..5] its items done, [8] it arrives on the
  // ticket, [10] the last rider is known, [11] its publication done, [12] / [13] the
  // earliest / latest rider entry, [14] the latest ticket arrival
  long long* dbg;
};

struct LanesArgs {
  int L;    // lanes (0: evaluation only)
  int par;  // round parity: lanes write fragments / loss of buffer `par`
  LaneRound r[kMaxLanes];
  const uint16_t* dsX;  // resident dataset [rows][FP] bf16
  const int32_t* dsy;
  float* w;             // server weights = every lane's pulled w_old [P]
  float lr;
  float* dsum;          // != nullptr: the lane sum is written here (multi-rank: RCCL reduce), w untouched
  uint16_t *shi, *slo;  // server fragments written by this round's update (columns scoff..)
  float* sb;
  int scoff;
  unsigned* arrive;     // [FP/32 + 1] per-slice lane arrival counters (zero between launches)
  // workgroup roles are CLAIMED at run time: a workgroup reads its XCC_ID and takes
  // the next slot of that XCD's lane (< kLaneWg of them), else the next rider id,
  // so a lane's workgroups share one L2 whatever order the dispatcher deals the
  // workgroups to the XCDs in.  claim: [2 launch parities][16] counters (XCD
  // lane slots 0..7, riders at 8); this launch uses parity cpar and clears the other.
  unsigned* claim;
  int cpar;
  int spin_max;         // cross-workgroup wait budget (0: default)
  int nride;            // rider workgroups
  EvalMulti ev;
};

bool lanes_supported(int FP, int K, int cap);
size_t lanes_lds_bytes(int FP);
// Grid of a round with L lanes and at least `min_riders` riders (>= 8 * kLaneWg);
// its riders are grid - L * kLaneWg.
int lanes_grid(int L, int min_riders);
// S = 2: one-XCD hand-offs (blockIdx % 8 == XCC_ID verified); S = 1: sc1 hand-offs.
void launch_lanes_round(const SolverCfg& cfg, const LaneDev* lanes_dev, const LanesArgs& a, int S, hipStream_t s);
// XCC_ID of every workgroup of a 2048-workgroup launch -> ids[2048] (device).
void launch_xcc_probe(int* ids, int n, hipStream_t s);
// Evaluation of ev's models as a launch of its own that co-runs with a lanes
// round (side stream; 8.6 KB LDS per workgroup, lanes_eval_grid() workgroups,
// ev.nticket must equal that grid).  Same EvalSlot publication.
int lanes_eval_grid();
void launch_lanes_eval(const SolverCfg& cfg, const EvalMulti& ev, hipStream_t s);

}  // namespace psx
