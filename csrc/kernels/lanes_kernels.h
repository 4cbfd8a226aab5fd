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
// longest ring (window) of a lane: up to 32 tiles (1,024 rows) stay resident in the
// row workgroups' LDS; longer rings are staged tile by tile every slot
constexpr int kLanesMaxCap = 8192;
constexpr int kMaxEvalModels = kMaxLanes + 1;
// model buffers per lane (local fragments, intercepts, loss) and of the server
// fragments, by round: r % 2, or r % 3 with overlapped launches (round r's
// evaluation of round r - 1 can still run while round r + 1 writes its models)
constexpr int kLaneBufs = 3;
// EvalMulti accumulators: [kAccCopies][kMaxEvalModels][256 cells] at stride kAccStride;
// a rider adds into copy XCC_ID % kAccCopies.  One copy: measured best end to end
// (tools/eval_probe, profiles/r04_s8-s9): 8 per-XCD copies cut the riders' flush from
// 3.3 to 1.25 us but the publication's reads of every copy cost ~7 us more
constexpr int kAccCopies = 1;
constexpr size_t kEvalAccInts = (size_t)kAccCopies * kMaxEvalModels * 256 * 32;

// Per-lane device state (a device-resident table read by the lane's workgroups).
struct LaneDev {
  SolveDev dv;        // solver workspace + the lane's ring (dv.X, dv.y); dv.delta = delta
  float* spart;       // [32 tiles][FP][2] window column sums / sums of squares (phase I hand-off)
  uint16_t* ohi[kLaneBufs];  // local model fragments by round buffer (class columns 0..K-1)
  uint16_t* olo[kLaneBufs];
  float* ob[kLaneBufs];
  float* loss2;       // [kLaneBufs] training loss by round buffer
  Ctrl* ctrl;         // the lane's controller after the round (host diagnostics)
  float* wpull;       // [P] overlapped launches: the lane's copy of the pulled weights (LanesArgs::ovl)
};

// Per-round arguments of one lane: the window and the new rows of this round:
// dataset rows first + i * step (i < n) into ring slots (dst + i) % cap, then (a
// delivery that wraps the worker's shard) first2 + i * step (i < n2) into slots
// (dst + n + i) % cap.
struct LaneRound {
  int B, start, n, dst;
  long long first, step, first2;
  int n2;
  int delay_us;  // BSP round kernel: injected straggler delay before the lane's solve (0: none)
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
  int* acc;          // [kAccCopies][kMaxEvalModels][256] accumulators (stride kAccStride), zero between passes
  unsigned* ticket;  // arrivals of the riders (reset by the last)
  unsigned nticket;
  // != nullptr: XCD-local evaluation -- [8] chunk counters (zero at launch): riders on
  // XCD x take chunks of the x-th eighth of the test tiles first (eval_multi_body)
  unsigned* xq;
  // 0: pair-major riders (eval_multi_body: items = (model pair, tile)); 1: tile-resident
  // riders (eval_tile_body: every model on a rider's tiles, the test set read once; the
  // tiles popped from xq[0], zero at launch)
  int form;
  int ppi;  // tile-resident form: model pairs per work item (0: all; items = (tile, pair group))
  // tile-resident form, gq = 1: one tile queue per pair group (xq[0 .. kEvalGroups)), a
  // rider keeps its group's fragments in registers across the group's tiles
  int gq;
  // != nullptr (tile-resident form, overlapped launches): no ticket -- every rider
  // stores its counts, [rider][kMaxEvalModels][64] ints (cell = label * 8 + predicted),
  // and a publish launch behind the round (launch_lanes_publish, co-running with the
  // next round) sums them and fills the slots; its nticket riders write their rows
  int* slab;
  // PSX_LANES_STAMPS: s_memrealtime stamps of the riders (nullptr: none): [0] rider 0
  // enters, [1] its first tile staged, [2..5] its items done, [8] it arrives on the
  // ticket, [10] the last rider is known, [11] its publication done, [12] / [13] the
  // earliest / latest rider entry, [14] the latest ticket arrival
  long long* dbg;
};

struct LanesArgs {
  int L;    // lanes (0: evaluation only)
  int par;  // round buffer (r % 2, or r % 3 with ovl): lanes write fragments / loss of buffer `par`
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
  // workgroups to the XCDs in.  claim: [2 launch parities][32] counters (XCD
  // lane slots 0..7, riders at 8, every workgroup at 9 -- the launch is fully
  // dispatched once it reaches the grid, XCD-local evaluation chunks / the
  // tile-resident riders' queue at 16..23, EvalMulti::xq); this launch uses parity
  // cpar and clears the other.
  unsigned* claim;
  int cpar;
  int xcd0;             // lane l runs on XCD xcd0 + l (processes sharing a GPU take disjoint XCDs)
  int spin_max;         // cross-workgroup wait budget (0: default)
  // --trace / --perf_log: each lane's phase times of this round (s_memrealtime ticks) ->
  // tr[(tr_slot * kMaxLanes + lane) * 4 + {0 stage, 1 solve, 2 solved, 3 updated}]; null: off
  long long* tr;
  int tr_slot;
  int nride;            // rider workgroups
  EvalMulti ev;
  // lane_eval = 1: each lane evaluates its own local model of THIS round right after
  // its solve (ev.m[l], worker row) with its own workgroups, lane 0 paired with the
  // global model of the previous update (ev.m[kMaxEvalModels - 1], server row); the
  // riders evaluate nothing.  0: the riders evaluate ev's models (the previous round's).
  int lane_eval;
  // ovl = 1 (LanesLoop with PSX_LANES_OVERLAP=1): consecutive round launches alternate
  // between two streams, launch n + 1 enqueued once every workgroup of launch n has
  // claimed its role (claim counter 9 at the grid: a stream wait on it), so launch n +
  // 1's workgroups take the CUs launch n's leave while its evaluation still runs, with
  // no kernel boundary in between.  The cross-round hand-offs go through counters
  // instead: the last lane's update of slice s writes w through and then sets
  // applied[s] = round + 1; the lane workgroups of launch `round` start once every
  // slice reads >= round (every lane is then past round - 1: its rings, workspaces and
  // run counter are free), pull their slice of w with write-through loads into
  // LaneDev::wpull and acquire.  The fragments rotate over three buffers (par = round
  // % 3): launch n evaluates buffer (n - 1) % 3 while launch n + 1 writes (n + 1) % 3.
  // evdone = n + 1 is a stream write behind launch n: launch n + 1's evaluation (same
  // accumulators, ticket and tile queue) starts only once evdone >= its round.
  int ovl;
  unsigned round;
  unsigned* applied;  // [FP/32]
  unsigned* evdone;
  // lane_riders = 1 (tile-resident form, ev.form == 1): every lane workgroup joins the
  // evaluation as a rider once its part of the round is done (ev.nticket counts the
  // nride riders + L * kLaneWg lane workgroups); the tiles come from ev.xq[0]
  int lane_riders;
  int* lacc;            // [kMaxLanes][2][256] accumulators (stride kAccStride), zero between launches
  unsigned* lticket;    // [kMaxLanes][32] per-lane evaluation arrivals
  // peer_sum (multi-rank BSP over the peer data plane, LanesLoop::set_peer_sum; needs ovl):
  // the last lane of slice s stores this rank's lane sum into its inbox slot on the server
  // GPU (system-scope stores over xGMI, csrc/comm/peer_bus.h) and tags it round + 1 (the
  // push); the launch's lane workgroups start once every slice of this rank's receive slot
  // carries a tag >= round (the server kernel's update of round - 1, written over xGMI) and
  // pull w from there -- no collective, no host and no kernel boundary between a round's
  // push and the next round's pull.  push == nullptr: off
  float* push;
  unsigned* push_tag;
  const float* rx;
  const unsigned* rx_tag;
  long long peer_ticks;  // the pull wait's wall-clock budget (s_memrealtime ticks, 100 MHz)
  // workgroups on an XCD whose bit is set leave at once (no role, no count): ranks that
  // share one GPU (the one-GPU rehearsals) keep off each other's and the server kernel's
  // XCDs, so no rider spins on a CU another process's persistent launch needs
  unsigned xcd_skip;
};

bool lanes_supported(int FP, int K, int cap);
size_t lanes_lds_bytes(int FP);
// Grid of a round with L lanes and at least `min_riders` riders (>= 8 * kLaneWg);
// its riders are grid - L * kLaneWg.
int lanes_grid(int L, int min_riders);
// S = 2: one-XCD hand-offs (blockIdx % 8 == XCC_ID verified); S = 1: sc1 hand-offs.
void launch_lanes_round(const SolverCfg& cfg, const LaneDev* lanes_dev, const LanesArgs& a, int S, hipStream_t s);
// The slab form's publication (EvalMulti::slab): one small workgroup per model sums the
// ev.nticket riders' counts and writes the model's slot; it also clears the tile queue
// ev.xq.  Sized to co-run with a round kernel (a few KB of LDS, <= 64 VGPRs).
constexpr int kSlabCells = 64;
constexpr int kEvalGroups = 8;  // EvalMulti::gq: tile queues (pair groups) at most
constexpr int kSlabRiders = 1024;  // slab rows allocated (riders of one launch at most)
void launch_lanes_publish(const EvalMulti& ev, hipStream_t s);
// --trace: the device clock (s_memrealtime, 100 MHz) into *out (pinned host memory).
void launch_clock_probe(long long* out, hipStream_t s);
// XCC_ID of every workgroup of a 2048-workgroup launch -> ids[2048] (device).
void launch_xcc_probe(int* ids, int n, hipStream_t s);
// Every lane's last delta [P] and training loss to caller buffers in ONE launch (the
// end of a run: 2 L memcpy launches of ~5 us each otherwise)
struct LanesCopyOut {
  int L, P;
  const float* src_d[kMaxLanes];
  float* dst_d[kMaxLanes];
  const float* src_l[kMaxLanes];
  float* dst_l[kMaxLanes];
};
void launch_lanes_copy_out(const LanesCopyOut& c, hipStream_t s);
// peer_sum, the end of a run: w[P] <- this rank's receive slot once every slice's tag is >=
// want (the server's last update); a wait beyond `ticks` sets *err_host (code 10)
void launch_peer_pull(const float* rx, const unsigned* rx_tag, unsigned want, float* w, int K, int FP,
                      long long ticks, unsigned long long* err_host, hipStream_t s);
// Evaluation of ev's models as a launch of its own that co-runs with a lanes
// round (side stream; 8.6 KB LDS per workgroup, lanes_eval_grid() workgroups,
// ev.nticket must equal that grid).  Same EvalSlot publication.
int lanes_eval_grid();
void launch_lanes_eval(const SolverCfg& cfg, const EvalMulti& ev, hipStream_t s);

// ---------------------------------------------------------------------------
// Asynchronous consistency (SSP / ASP) on one GPU: ONE persistent launch in
// which every lane loops release -> solve -> push -> evaluate (lanes_async.hip).
//
// Reference: ServerProcessor.process (ServerProcessor.java:143-183) applies each
// gradient on arrival -- GRADIENTS_TOPIC has ONE partition, so updates are
// serial in arrival order -- and answers the workers MessageTracker releases
// (MessageTracker.java:69-87) with the weights right after that update.
// MI355X mapping:
//   * arrival order = a device ticket taken when a lane's delta is final; slice
//     s of the update of ticket t waits until slice s of ticket t - 1 is applied
//     (per-slice turn words), so updates are serial per slice and pipelined
//     across slices; each applied slice is also written to snapshot slot t % R
//     (the weights "right after the update" a release refers to);
//   * the tracker decision stays on the HOST (the C++ VectorClockTracker): a
//     lane publishes a token (ticket, lane, vc) into a pinned ring once all its
//     slices are applied; the host loop consumes tokens in ticket order, runs
//     on_delta, and answers each released lane with a release record (pinned,
//     polled by the lane's leader): its clock, the snapshot ticket, its window
//     and new stream rows, the metrics slots of its rows;
//   * a lane evaluates its local model (the worker row) -- paired with the
//     global model after its own update on the logging lane (the server row) --
//     with its own 32 workgroups right after its push, and publishes the counts
//     as tagged 16-B chunks (no store-completion wait on the lane's path).
// Host <-> device records are 16-B chunks {tag, 3 x u32 payload}: a chunk is
// written by ONE 16-B store, so a reader that sees every chunk carry the
// expected tag has the whole record, without ordering between the stores.
struct alignas(16) TagChunk {
  unsigned tag, a, b, c;
};
constexpr int kRelChunks = 8;
struct alignas(16) AsyncRelease {  // host -> lane (pinned), tag = the lane's record count
  TagChunk ch[kRelChunks];
};
// release record payload (unpacked on both sides by the same layout)
struct RelRec {
  int stop;              // 1: leave the launch (no solve)
  long long vc;          // the pulled weights' version (tracker clock)
  long long snap;        // ticket whose snapshot holds the pulled weights
  LaneRound r;           // window + this solve's new stream rows
  unsigned long long slot_w, slot_s;  // pinned EvalSlot addresses (0: no row)
  unsigned seq_w, seq_s;              // their sequence numbers (low 32 bits)
  int delay_us;          // injected straggler delay before the push (tests)
  unsigned pull_tag;     // peer data plane: the receive slot's tag that carries these weights
};
PSX_HD inline void pack_release(const RelRec& q, unsigned tag, TagChunk* ch) {
  auto lo = [](long long v) { return (unsigned)(unsigned long long)v; };
  auto hi = [](long long v) { return (unsigned)((unsigned long long)v >> 32); };
  ch[0] = TagChunk{tag, (unsigned)q.stop, lo(q.vc), hi(q.vc)};
  ch[1] = TagChunk{tag, lo(q.snap), hi(q.snap), (unsigned)q.r.B};
  ch[2] = TagChunk{tag, (unsigned)q.r.start, (unsigned)q.r.n, (unsigned)q.r.dst};
  ch[3] = TagChunk{tag, lo(q.r.first), hi(q.r.first), (unsigned)q.r.n2};
  ch[4] = TagChunk{tag, lo(q.r.step), hi(q.r.step), lo(q.r.first2)};
  ch[5] = TagChunk{tag, hi(q.r.first2), lo((long long)q.slot_w), hi((long long)q.slot_w)};
  ch[6] = TagChunk{tag, q.seq_w, lo((long long)q.slot_s), hi((long long)q.slot_s)};
  ch[7] = TagChunk{tag, q.seq_s, (unsigned)q.delay_us, q.pull_tag};
}
PSX_HD inline void unpack_release(const TagChunk* ch, RelRec& q) {
  auto j = [](unsigned l, unsigned h) { return (long long)(((unsigned long long)h << 32) | l); };
  q.stop = (int)ch[0].a;
  q.vc = j(ch[0].b, ch[0].c);
  q.snap = j(ch[1].a, ch[1].b);
  q.r.B = (int)ch[1].c;
  q.r.start = (int)ch[2].a;
  q.r.n = (int)ch[2].b;
  q.r.dst = (int)ch[2].c;
  q.r.first = j(ch[3].a, ch[3].b);
  q.r.n2 = (int)ch[3].c;
  q.r.step = j(ch[4].a, ch[4].b);
  q.r.first2 = j(ch[4].c, ch[5].a);
  q.slot_w = (unsigned long long)j(ch[5].b, ch[5].c);
  q.seq_w = ch[6].a;
  q.slot_s = (unsigned long long)j(ch[6].b, ch[6].c);
  q.seq_s = ch[7].a;
  q.delay_us = (int)ch[7].b;
  q.pull_tag = ch[7].c;
  q.r.delay_us = 0;
}
// token: lane -> host (pinned ring, slot t % ring): {tag = ticket (low 32 bits,
// tickets start at 1), lane, vc low, vc high}
typedef TagChunk AsyncToken;
// the tag of a tagged evaluation slot's chunks (never 0)
PSX_HD inline unsigned eval_tag(unsigned long long seq) { return (unsigned)seq | 0x80000000u; }

// Per-lane device state of the asynchronous launch (a device table prepared by
// the host: the kernel reads it through a pointer it re-loads every iteration).
struct AsyncLaneDev {
  SolveDev dv;           // the lane's solver (LaneDev::dv with the buffers of this launch's mode)
  float* spart;          // LaneDev::spart
  Ctrl* ctrl;            // LaneDev::ctrl
  float* wpull;          // [P] the pulled weights of the current solve (copied from the snapshot)
  uint16_t *shi, *slo;   // server fragments of the logging lane's update (columns 0..K-1)
  float* sb;             // [16]
  int* acc;              // [2 models][256][kAccStride] evaluation accumulators (zero between solves)
  unsigned* eticket;     // evaluation arrivals
  unsigned long long* flags;  // [kLaneWg][32] lane-wide barrier words (own 256-B line each)
  unsigned long long* rec;    // [kRelChunks * 2] the release record broadcast (+ the ticket at [16])
  unsigned long long* relc;   // release records consumed by this lane (persists across launches)
  AsyncRelease* rel;     // pinned release record (host -> device)
  // peer data plane (remote mode, csrc/comm/peer_bus.h): this lane's worker's slot in
  // the server GPU's inbox (an IPC mapping over xGMI) -- [P] delta + [FP/32] slice tags
  float* inbox;
  unsigned* inbox_tag;
  int* eslab;            // [kLaneWg][2][64] the evaluation's per-workgroup counts (slab form)
};

struct AsyncArgs {
  int L;
  const uint16_t* dsX;  // resident dataset [rows][FP] bf16
  const int32_t* dsy;
  float* w;             // server master weights [P]
  float lr;
  float* snap;          // [R][sstride] w after ticket t at slot t % R
  unsigned* snap_tag;   // [R][FP/32] ticket of each slot's slices (sanity check)
  int R;
  long long sstride;    // floats between snapshot slots (P; a peer region's padded stride)
  unsigned long long* ticket;  // last ticket handed out (device counter)
  unsigned long long* turn;    // [FP/32][32] last ticket applied to slice s (own 256-B line each)
  AsyncToken* tok;             // pinned token ring
  int ring;
  const uint16_t* Xt;  // test set
  const int32_t* yt;
  int T;
  // the test set in ELL form (EvalSet.ell: [T][tnz] feature ids + bf16 values); tnz == 0:
  // the dense MFMA pass over Xt
  const uint16_t* Ti;
  const uint16_t* Tv;
  int tnz;
  int log_lane;        // lane whose deltas produce server rows (-1: none)
  long long launch;    // launch number (> every earlier one): lane-wide barrier words
  long long rel_ticks; // release / pull wait budget (s_memrealtime ticks, 100 MHz)
  unsigned* claim;     // [2][16] role claim counters
  int cpar;
  // remote = 1: the server is another rank (worker GPUs of a multi-rank job): a
  // push only publishes the token (the host sends the delta, ticket = this rank's
  // push order); a release's snapshot is the lane's receive slot (snap = slot)
  int remote;
  int xcd0;            // lane l runs on XCD xcd0 + l
  // peer_rx = 1 (remote mode, peer data plane): snap / snap_tag are this rank's
  // receive slots [L][P] / [L][FP/32] in fine-grained memory the server GPU writes
  // over xGMI; a release's pull_tag says which slice tags carry its weights
  int peer_rx;
  // debug (tests: the float64 replay of an asynchronous run): the delta every ticket t
  // applied, at dbg_delta[(t - 1) % dbg_cap][P]; nullptr: off
  float* dbg_delta;
  int dbg_cap;
  // --trace / --perf_log: per ticket t -> tr[(t % tr_cap) * 4 + {0 lane, 1 released,
  // 2 solved, 3 pushed}] (s_memrealtime ticks); null: off
  long long* tr;
  int tr_cap;
};

// The launch's uniform arguments, in device memory (see AsyncLaneDev).
struct AsyncPack {
  SolverCfg cfg;
  AsyncArgs a;
};

// Initialise the snapshot slot of ticket t (= w) and the slices' turn words (t).
void launch_async_init(const SolverCfg& cfg, const AsyncArgs& a, unsigned long long t, hipStream_t s);
// pk: {cfg, a} of THIS launch (a.launch / a.cpar), passed as the kernel argument -- no
// copy before the launch (on a GPU shared with other processes' persistent launches
// a copy can wait behind them for minutes); al: device table [L]
void launch_lanes_async(const SolverCfg& cfg, const AsyncPack& pk, const AsyncLaneDev* al, int S, hipStream_t s);

}  // namespace psx
