// Native multi-lane BSP round loop (see lanes_loop.h).
#include "lanes_loop.h"

#include <immintrin.h>

#include <algorithm>
#include <ctime>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>

#include "../kernels/common.h"
#include "../kernels/lr_kernels.h"
#include "../solver/solver.h"

namespace psx {

namespace {
double epoch_ms() {
  using namespace std::chrono;
  return (double)duration_cast<microseconds>(system_clock::now().time_since_epoch()).count() / 1000.0;
}
int64_t steady_ns() {
  using namespace std::chrono;
  return duration_cast<nanoseconds>(steady_clock::now().time_since_epoch()).count();
}
size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }
}  // namespace

bool LanesLoop::probe_placement(hipStream_t stream) {
  static int cached = -1;  // one probe per process
  if (const char* e = std::getenv("PSX_FAKE_XCD_MISMATCH"))
    if (e[0] == '1') return false;
  if (cached >= 0) return cached == 1;
  constexpr int n = 2048;
  int* ids = nullptr;
  hip_check(hipMalloc(&ids, n * sizeof(int)), "hipMalloc(xcc probe)");
  launch_xcc_probe(ids, n, stream);
  hip_check(hipGetLastError(), "xcc probe launch");
  std::vector<int> h(n);
  hip_check(hipMemcpyAsync(h.data(), ids, n * sizeof(int), hipMemcpyDeviceToHost, stream), "xcc probe copy");
  hip_check(hipStreamSynchronize(stream), "xcc probe sync");
  (void)hipFree(ids);
  bool ok = true;
  for (int b = 0; b < n; ++b) ok &= h[b] == (b & 7);
  cached = ok ? 1 : 0;
  return ok;
}

LanesLoop::LanesLoop(const LanesLoopCfg& cfg, Comm* comm)
    : cfg_(cfg), comm_(comm), api_(reinterpret_cast<const HostApi*>(cfg.api)) {
  const SolverCfg& s = cfg_.scfg;
  if (!api_ || api_->version != kHostApiVersion) throw std::invalid_argument("LanesLoop: host runtime API mismatch");
  if (cfg_.L < 0 || cfg_.L > kMaxLanes) throw std::invalid_argument("LanesLoop: 0..8 lanes per process");
  if (cfg_.xcd0 < 0 || cfg_.xcd0 + cfg_.L > kMaxLanes) throw std::invalid_argument("LanesLoop: lanes beyond XCD 7");
  if (cfg_.L == 0 && !comm_) throw std::invalid_argument("LanesLoop: a rank without lanes needs a communicator");
  if (!lanes_supported(s.Fp, s.K, s.cap)) throw std::invalid_argument("LanesLoop: unsupported model / ring shape");
  if (s.P != s.K * s.Fp + s.K) throw std::invalid_argument("LanesLoop: P mismatch");
  if (s.nslots < 1 || s.nslots >= kMaxSlots || s.hist < 1 || s.hist > kMaxHist)
    throw std::invalid_argument("LanesLoop: slots / history out of range");
  if ((int)cfg_.k.size() != cfg_.L || (int)cfg_.X.size() != cfg_.L || (int)cfg_.y.size() != cfg_.L ||
      (int)cfg_.window.size() != cfg_.L)
    throw std::invalid_argument("LanesLoop: one worker id / ring / window per lane");
  if (cfg_.XT.empty()) cfg_.XT.assign(cfg_.L, 0);
  if (cfg_.L > 0 && (!cfg_.dsX || !cfg_.dsy || cfg_.ds_rows <= 0 || cfg_.N < cfg_.L))
    throw std::invalid_argument("LanesLoop: bad dataset / worker count");
  if (cfg_.per_iter_rows <= 0 && !(cfg_.p_ms > 0.0) && cfg_.L > 0)
    throw std::invalid_argument("LanesLoop: need rows per round or a producer period");
  if (!cfg_.w) throw std::invalid_argument("LanesLoop: no server weights");
  if (cfg_.new_rows < 0 || cfg_.new_frac < 0.0 || cfg_.new_cap < 0 || cfg_.new_ramp < 0)
    throw std::invalid_argument("LanesLoop: negative cadence");
  const bool evaluates = cfg_.sink && (cfg_.log_server || cfg_.log_workers);
  if (evaluates && (!cfg_.Xt || !cfg_.yt || cfg_.T <= 0)) throw std::invalid_argument("LanesLoop: no test set");
  if (cfg_.log_server && evaluates && (!cfg_.shi[0] || !cfg_.shi[1] || !cfg_.slo[0] || !cfg_.slo[1] || !cfg_.sb[0] ||
                                       !cfg_.sb[1] || cfg_.scoff < 0 || cfg_.scoff + s.K > 16))
    throw std::invalid_argument("LanesLoop: server evaluation fragments");
  if (comm_ && comm_->rank() == cfg_.server_rank && (!cfg_.shi[0] || !cfg_.shi[1]))
    throw std::invalid_argument("LanesLoop: the server rank needs its fragments");
  P_ = s.P;
  for (int l = 0; l < cfg_.L; ++l) {
    const int k = cfg_.k[l];
    if (k < 0 || k >= cfg_.N || !cfg_.X[l] || !cfg_.y[l] || !cfg_.window[l])
      throw std::invalid_argument("LanesLoop: bad lane " + std::to_string(l));
    const int64_t tot = cfg_.ds_rows > k ? (cfg_.ds_rows - k + cfg_.N - 1) / cfg_.N : 0;
    if (tot == 0) throw std::invalid_argument("LanesLoop: worker " + std::to_string(k) + " has no rows");
    local_total_.push_back(tot);
    next_local_.push_back(0);
    seen_at_solve_.push_back(0);
  }
  prepare_kernels();
  // the lanes claim their XCD at run time (LanesArgs::claim), so placement needs no
  // assumption; PSX_FAKE_XCD_MISMATCH=1 / PSX_LANES_SPREAD=1 select the spread form
  const char* sp = std::getenv("PSX_LANES_SPREAD");
  const char* fk = std::getenv("PSX_FAKE_XCD_MISMATCH");
  S_ = ((sp && sp[0] == '1') || (fk && fk[0] == '1')) ? 1 : 2;

  // ---- device workspace: per lane + shared ----
  const int KP = padded_classes(s.K), FPI = padded_stride(s.Fp), PI = KP * FPI + 16, FP = s.Fp;
  size_t off = 0;
  auto take = [&](size_t bytes) {
    const size_t o = off;
    off = align_up(off + bytes, 256);
    return o;
  };
  struct Offs {
    size_t x, d, gc, wfix, std_, istd, beff, whi, wlo, part, xch, gpf, spart, delta, ohi[kLaneBufs], olo[kLaneBufs],
        ob[kLaneBufs], loss2, stats, cnt, ctrl, dbg, wpull;
  };
  const bool stamps = std::getenv("PSX_LANES_STAMPS") != nullptr;
  std::vector<Offs> o(cfg_.L);
  for (int l = 0; l < cfg_.L; ++l) {
    Offs& q = o[l];
    q.x = take(PI * 4);
    q.d = take(PI * 4);
    q.gc = take(PI * 4);
    q.wfix = take(PI * 4);
    q.std_ = take(FPI * 4);
    q.istd = take(FPI * 4);
    q.beff = take(16 * 4);
    q.whi = take(16 * FP * 2);
    q.wlo = take(16 * FP * 2);
    q.part = take(kLaneWg * 32 * 4);
    q.xch = take((size_t)xch_words() * 8);
    q.gpf = take((size_t)kLaneWg * KP * FP * 4);
    q.spart = take((size_t)kLaneWg * FP * 2 * 4);
    q.delta = take((size_t)P_ * 4);
    for (int p = 0; p < kLaneBufs; ++p) {
      q.ohi[p] = take(16 * FP * 2);
      q.olo[p] = take(16 * FP * 2);
      q.ob[p] = take(16 * 4);
    }
    q.loss2 = take(kLaneBufs * 4);
    q.wpull = take((size_t)P_ * 4);
    q.stats = take(8 * 4);
    q.cnt = take(16);
    q.ctrl = take(sizeof(Ctrl));
    q.dbg = stamps ? take(32 * 16 * sizeof(long long)) : 0;
  }
  const size_t o_tab = take(sizeof(LaneDev) * (cfg_.L > 0 ? cfg_.L : 1));
  const size_t o_arr = take((FP / 32 + 1) * sizeof(unsigned));
  const size_t o_acc = take(kEvalAccInts * sizeof(int));
  const size_t o_tic = take(8 * sizeof(unsigned));
  const size_t o_claim = take(64 * sizeof(unsigned));
  const size_t o_dsum = take((size_t)P_ * 4);
  const size_t o_uhi = take((size_t)16 * FP * 2), o_ulo = take((size_t)16 * FP * 2), o_ub = take(16 * 4);
  const size_t o_acc2 = take(kEvalAccInts * sizeof(int));
  const size_t o_tic2 = take(8 * sizeof(unsigned));
  const size_t o_sfl = take(8 * sizeof(unsigned));
  const size_t o_lacc = take((size_t)kMaxLanes * 2 * 256 * kAccStride * sizeof(int));
  const size_t o_ltic = take((size_t)kMaxLanes * 32 * sizeof(unsigned));
  const size_t o_rdbg = stamps ? take(64 * sizeof(long long)) : 0;
  const size_t o_ovl = take(64 * sizeof(unsigned));  // applied [0, 32), evdone [32], tile queue [48]
  const size_t o_slab = take((size_t)kSlabRiders * kMaxEvalModels * kSlabCells * sizeof(int));
  hip_check(hipMalloc(&ws_, off), "hipMalloc(lanes workspace)");
  hip_check(hipMemset(ws_, 0, off), "hipMemset(lanes workspace)");
  char* b = static_cast<char*>(ws_);
  hip_check(hipHostMalloc((void**)&err_host_, kMaxLanes * sizeof(unsigned long long),
                          hipHostMallocCoherent | hipHostMallocMapped),
            "hipHostMalloc(error words)");
  std::memset(err_host_, 0, kMaxLanes * sizeof(unsigned long long));
  lanes_.resize(cfg_.L);
  for (int l = 0; l < cfg_.L; ++l) {
    const Offs& q = o[l];
    LaneDev& ld = lanes_[l];
    std::memset(&ld, 0, sizeof(ld));
    SolveDev& dv = ld.dv;
    dv.X = reinterpret_cast<const uint16_t*>(cfg_.X[l]);
    dv.XT = reinterpret_cast<const uint16_t*>(cfg_.XT[l]);
    dv.y = reinterpret_cast<const int32_t*>(cfg_.y[l]);
    dv.w_old = cfg_.w;
    dv.x = reinterpret_cast<float*>(b + q.x);
    dv.d = reinterpret_cast<float*>(b + q.d);
    dv.g_c = reinterpret_cast<float*>(b + q.gc);
    dv.wfix = reinterpret_cast<float*>(b + q.wfix);
    dv.std_ = reinterpret_cast<float*>(b + q.std_);
    dv.inv_std = reinterpret_cast<float*>(b + q.istd);
    dv.b_eff = reinterpret_cast<float*>(b + q.beff);
    dv.whi = reinterpret_cast<uint16_t*>(b + q.whi);
    dv.wlo = reinterpret_cast<uint16_t*>(b + q.wlo);
    dv.part = reinterpret_cast<float*>(b + q.part);
    dv.xch = reinterpret_cast<unsigned long long*>(b + q.xch);
    dv.gpf = reinterpret_cast<float*>(b + q.gpf);
    dv.delta = reinterpret_cast<float*>(b + q.delta);
    dv.out_hi = reinterpret_cast<uint16_t*>(b + q.ohi[0]);
    dv.out_lo = reinterpret_cast<uint16_t*>(b + q.olo[0]);
    dv.b_fin = reinterpret_cast<float*>(b + q.ob[0]);
    dv.loss = reinterpret_cast<float*>(b + q.loss2);
    dv.stats = reinterpret_cast<int*>(b + q.stats);
    dv.prm_count = reinterpret_cast<unsigned*>(b + q.cnt);
    dv.KP = KP;
    dv.FPI = FPI;
    dv.PI = PI;
    dv.err_host = err_host_ + l;
    dv.dbg = stamps ? reinterpret_cast<long long*>(b + q.dbg) : nullptr;
    ld.spart = reinterpret_cast<float*>(b + q.spart);
    for (int p = 0; p < kLaneBufs; ++p) {
      ld.ohi[p] = reinterpret_cast<uint16_t*>(b + q.ohi[p]);
      ld.olo[p] = reinterpret_cast<uint16_t*>(b + q.olo[p]);
      ld.ob[p] = reinterpret_cast<float*>(b + q.ob[p]);
    }
    ld.loss2 = reinterpret_cast<float*>(b + q.loss2);
    ld.wpull = reinterpret_cast<float*>(b + q.wpull);
    ld.ctrl = reinterpret_cast<Ctrl*>(b + q.ctrl);
  }
  lanes_dev_ = reinterpret_cast<LaneDev*>(b + o_tab);
  arrive_ = reinterpret_cast<unsigned*>(b + o_arr);
  acc_ = reinterpret_cast<int*>(b + o_acc);
  ticket_ = reinterpret_cast<unsigned*>(b + o_tic);
  claim_ = reinterpret_cast<unsigned*>(b + o_claim);
  dsum_ = reinterpret_cast<float*>(b + o_dsum);
  upd_hi_ = reinterpret_cast<uint16_t*>(b + o_uhi);
  upd_lo_ = reinterpret_cast<uint16_t*>(b + o_ulo);
  upd_b_ = reinterpret_cast<float*>(b + o_ub);
  acc2_ = reinterpret_cast<int*>(b + o_acc2);
  ticket2_ = reinterpret_cast<unsigned*>(b + o_tic2);
  sflags_ = reinterpret_cast<unsigned*>(b + o_sfl);
  lacc_ = reinterpret_cast<int*>(b + o_lacc);
  lticket_ = reinterpret_cast<unsigned*>(b + o_ltic);
  rider_dbg_ = stamps ? reinterpret_cast<long long*>(b + o_rdbg) : nullptr;
  applied_ = reinterpret_cast<unsigned*>(b + o_ovl);
  evdone_ = applied_ + 32;
  ovlq_ = applied_ + 48;
  slab_ = reinterpret_cast<int*>(b + o_slab);
  if (const char* ss = std::getenv("PSX_SIDE_SYNC"))
    side_sync_ = std::string(ss) == "value" ? 1 : (std::string(ss) == "nowait" ? 2 : (std::string(ss) == "inline" ? 3 : 0));
  // PSX_LANES_SIDE_EVAL=1: the rows go to a co-running side launch instead of riders
  // of the round kernel.  Off by default: with 8 lanes (no XCD left for riders) the
  // two forms measured the same, 69.4k vs 69.2k updates/s (profiles/r03_v5), and
  // the riders keep a round at one launch
  const char* se = std::getenv("PSX_LANES_SIDE_EVAL");
  side_eval_ = se ? (se[0] == '1' && cfg_.L > 0) : false;
  // PSX_LANES_LANE_EVAL=1: each lane evaluates its own local model after its solve.  Off
  // by default: with 8 lanes every XCD then streams the whole test set per round (8 x
  // 10 MB): 101.2 against 95.8 us per round for the riders (profiles/r04_s3, same box)
  // PSX_RIDERS_XCD=1: riders take XCD-local slices of the test set from per-XCD chunk
  // queues (EvalMulti::xq) instead of contiguous chunks of the whole set.  Off by
  // default: 113.1 against 95.8 us per round (profiles/r04_s3) -- the queue pops and
  // the per-slice pair reloads cost more than the L2 locality returns
  // The riders' form, PSX_RIDERS_TILE: 2 (default) = tile-resident riders (eval_tile_body:
  // a work item's 32-row test tile held in registers, its model pairs run past it, items
  // popped from a queue) that every lane workgroup joins once its part of the round is
  // done (LanesArgs::lane_riders); 1 = the tile-resident riders alone; 0 = the pair-major
  // riders (eval_multi_body).  Same box, driver-form bench, 8 lanes (profiles/r04/s10,
  // s11): 84.0 / 80.5k updates/s for 2 / 0, 85.3k with 2 model pairs per item
  // (PSX_RIDERS_PPI; 1: 82.3k; 0 = all 5 pairs: 85.0k).  With overlapped launches and
  // the slab form every pair per item (0, the default) is best: 86.7 / 86.4k against
  // 84.3 / 84.5k for 2 pairs, 86.3 / 86.0k for 3, 80.0 / 80.1k for 1 (profiles/r04/s35)
  const char* rt = std::getenv("PSX_RIDERS_TILE");
  const char tf = rt && rt[0] ? rt[0] : '2';
  tile_riders_ = tf == '1' || tf == '2';
  lane_riders_ = tf == '2';
  const char* rp = std::getenv("PSX_RIDERS_PPI");
  riders_ppi_ = rp ? std::atoi(rp) : 0;
  // PSX_RIDERS_GQ=1: tile queues per pair group, the group's fragments held in
  // registers across its tiles (EvalMulti::gq).  Off by default: 80.6-80.9k against
  // 83.3-83.5k updates/s (profiles/r04/s27) -- the tile-major queue has a tile's groups
  // popped back to back, so the 64 KB tile comes from L2 after the first; fragment
  // reloads cost less than the lost tile locality
  const char* rg = std::getenv("PSX_RIDERS_GQ");
  riders_gq_ = rg && rg[0] == '1';
  const char* rx = std::getenv("PSX_RIDERS_XCD");
  xcd_riders_ = rx && rx[0] == '1';
  const char* le = std::getenv("PSX_LANES_LANE_EVAL");
  lane_eval_ = cfg_.L > 0 && S_ == 2 && !side_eval_ && le && le[0] == '1';  // (built for S == 2 only)
  // PSX_LANES_OVERLAP (default 1; 0: one launch after the other on the caller's
  // stream): overlapped round launches (LanesArgs::ovl).  One rank (the multi-rank
  // rounds end in collectives on the caller's stream), rider evaluation in the
  // tile-resident or pair-major form without the XCD chunk counters (the claim block is
  // reset while the previous launch runs), the XCD-resident form, and a third server
  // fragment buffer.  Same box, driver-form A/B: 83.5 / 83.4 / 84.1k against 82.2 /
  // 82.1 / 83.2k updates/s (profiles/r04/s19, s21, s22); the rocprofv3 trace shows
  // each launch dispatched ~46 us before the previous one ends (s23)
  const char* ov = std::getenv("PSX_LANES_OVERLAP");
  const bool sfr = !cfg_.shi[0] || (cfg_.shi[2] && cfg_.slo[2] && cfg_.sb[2]);  // (a sink may come later)
  ovl_ = !(ov && ov[0] == '0') && !comm_ && cfg_.L > 0 && S_ == 2 && !side_eval_ && !lane_eval_ && !xcd_riders_ && sfr;
  // PSX_RIDERS_SLAB (default 1, overlapped launches with tile-resident riders): the
  // riders store their counts (EvalMulti::slab) instead of flushing them with atomics
  // and waiting on a ticket; a publish launch behind each round sums them and fills
  // the slots while the next round runs
  const char* sl = std::getenv("PSX_RIDERS_SLAB");
  slab_on_ = ovl_ && tile_riders_ && !(sl && sl[0] == '0');
  if (ovl_) {
    // The two streams of the overlapped launches must not share a hardware queue (packets
    // of one queue run in order: the next round's launch would wait for the previous one to
    // END, the very thing the overlap removes).  HIP spreads a process's streams of one
    // priority over GPU_MAX_HW_QUEUES (4) queues, and every solver holds a capture stream,
    // RCCL / torch.distributed a few more: the second stream takes the least priority,
    // whose queue pool is its own (PSX_OVL_STREAM=normal: the previous form, for A/B).
    const char* os = std::getenv("PSX_OVL_STREAM");
    if (os && os[0] == 'n') {
      hip_check(hipStreamCreateWithFlags(&ostream_, hipStreamNonBlocking), "hipStreamCreate(overlap)");
    } else {
      int prio_lo = 0, prio_hi = 0;
      hip_check(hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi), "hipDeviceGetStreamPriorityRange");
      hip_check(hipStreamCreateWithPriority(&ostream_, hipStreamNonBlocking, prio_lo), "hipStreamCreate(overlap)");
    }
    hip_check(hipEventCreateWithFlags(&ovl_in_, hipEventDisableTiming), "hipEventCreate");
    hip_check(hipEventCreateWithFlags(&ovl_out_, hipEventDisableTiming), "hipEventCreate");
    hip_check(hipEventCreateWithFlags(&ovl_last_, hipEventDisableTiming), "hipEventCreate");
  }
  if (side_eval_) {
    hip_check(hipStreamCreateWithFlags(&side_, hipStreamNonBlocking), "hipStreamCreate(side eval)");
    for (int p = 0; p < 2; ++p) {
      hip_check(hipEventCreateWithFlags(&ev_round_[p], hipEventDisableTiming), "hipEventCreate");
      hip_check(hipEventCreateWithFlags(&ev_eval_[p], hipEventDisableTiming), "hipEventCreate");
    }
  }
  if (cfg_.L > 0)
    hip_check(hipMemcpy(lanes_dev_, lanes_.data(), sizeof(LaneDev) * cfg_.L, hipMemcpyHostToDevice),
              "lanes table upload");
}

LanesLoop::~LanesLoop() {
  if (side_) {
    (void)hipStreamSynchronize(side_);
    (void)hipStreamDestroy(side_);
  }
  for (int p = 0; p < 2; ++p) {
    if (ev_round_[p]) (void)hipEventDestroy(ev_round_[p]);
    if (ev_eval_[p]) (void)hipEventDestroy(ev_eval_[p]);
  }
  if (ws_) (void)hipFree(ws_);
  if (aws_) (void)hipFree(aws_);
  if (rel_host_) (void)hipHostFree(rel_host_);
  for (hipEvent_t e : pull_ev_)
    if (e) (void)hipEventDestroy(e);
  if (astream_) {
    (void)hipStreamSynchronize(astream_);
    (void)hipStreamDestroy(astream_);
  }
  if (ostream_) {
    (void)hipStreamSynchronize(ostream_);
    (void)hipStreamDestroy(ostream_);
  }
  for (hipEvent_t e : {ovl_in_, ovl_out_, ovl_last_})
    if (e) (void)hipEventDestroy(e);
  if (aev_in_) (void)hipEventDestroy(aev_in_);
  if (aev_out_) (void)hipEventDestroy(aev_out_);
  if (tok_host_) (void)hipHostFree(tok_host_);
  if (err_host_) (void)hipHostFree(err_host_);
  if (tr_) (void)hipFree(tr_);
}

void LanesLoop::check(int64_t rc, const char* what) const {
  if (rc < 0) throw std::runtime_error(std::string("LanesLoop: ") + what + ": " + api().last_error());
}

bool LanesLoop::all_exhausted() const {
  for (int l = 0; l < cfg_.L; ++l)
    if (!exhausted(l)) return false;
  return true;
}

// Deliver lane `lane`'s due rows into its window (WorkerSamplingProcessor.java:
// 50-113 through the host runtime's SlidingWindow); the rows of the last
// contiguous run go to the round kernel (r->n, dst, first, step), earlier runs
// (a delivery that wraps the shard's epoch) to a ring-ingest launch.
int64_t LanesLoop::poll(int lane, double now_ms, LaneRound* r, hipStream_t stream) {
  if (exhausted(lane)) return 0;
  const int k = cfg_.k[lane];
  const int64_t lt = local_total_[lane];
  int64_t& nl = next_local_[lane];
  const int64_t limit = lt * cfg_.epochs - nl;
  int64_t n;
  if (cfg_.per_iter_rows > 0) {
    n = cfg_.per_iter_rows < limit ? cfg_.per_iter_rows : limit;
    times_.assign((size_t)n, now_ms);
  } else {
    const int64_t epoch = nl / lt, cur = nl - epoch * lt;
    int64_t mx = limit < lt - cur ? limit : lt - cur;
    if (mx > (int64_t(1) << 22)) mx = int64_t(1) << 22;
    times_.resize(mx > 0 ? (size_t)mx : 1);
    n = api().due_rows(k, cfg_.N, cfg_.p_ms, cfg_.ds_rows, cur, now_ms, mx, times_.data());
    check(n, "due_rows");
  }
  if (n <= 0) return 0;
  const int64_t first = api().window_insert_many(reinterpret_cast<void*>(cfg_.window[lane]), times_.data(), n);
  check(first, "window insert");
  const int64_t cap = cfg_.scfg.cap;
  // rows already pending for the kernel from an earlier delivery of this round: into
  // the ring now (the kernel carries at most the last two contiguous runs)
  flush_ingest(lane, r, stream);
  const int64_t keep = n < cap ? n : cap, skip = n - keep;
  int64_t slot = (first + skip) % cap, pos = nl + skip, remaining = keep;
  while (remaining > 0) {  // split at the shard's epoch boundaries
    const int64_t cur = pos % lt;
    const int64_t run = remaining < lt - cur ? remaining : lt - cur;
    const int64_t src_first = k + cur * (int64_t)cfg_.N;
    if (r->n2 > 0) {  // a third run: the oldest goes to a launch of its own
      ovl_wait_last(stream);
      launch_ring_ingest(cfg_.dsX, cfg_.dsy, r->first, r->step, r->n, reinterpret_cast<uint16_t*>(cfg_.X[lane]),
                         nullptr, reinterpret_cast<int32_t*>(cfg_.y[lane]), r->dst, cap, cfg_.scfg.Fp, stream);
      r->dst = (int)((r->dst + r->n) % cap);
      r->first = r->first2;
      r->n = r->n2;
      r->n2 = 0;
    }
    if (r->n == 0) {
      r->first = src_first;
      r->step = cfg_.N;
      r->n = (int)run;
      r->dst = (int)slot;
    } else {
      r->first2 = src_first;
      r->n2 = (int)run;
    }
    slot = (slot + run) % cap;
    pos += run;
    remaining -= run;
  }
  nl += n;
  return n;
}

void LanesLoop::ovl_wait_last(hipStream_t stream) {
  // (the previous round's launch runs on the other stream and reads the ring)
  if (ovl_ && ovl_n_ > 0) hip_check(hipStreamWaitEvent(stream, ovl_last_, 0), "ingest waits the last round");
}

void LanesLoop::flush_ingest(int lane, LaneRound* r, hipStream_t stream) {
  const int64_t cap = cfg_.scfg.cap;
  if (r->n > 0 || r->n2 > 0) ovl_wait_last(stream);
  if (r->n > 0)
    launch_ring_ingest(cfg_.dsX, cfg_.dsy, r->first, r->step, r->n, reinterpret_cast<uint16_t*>(cfg_.X[lane]), nullptr,
                       reinterpret_cast<int32_t*>(cfg_.y[lane]), r->dst, cap, cfg_.scfg.Fp, stream);
  if (r->n2 > 0)
    launch_ring_ingest(cfg_.dsX, cfg_.dsy, r->first2, r->step, r->n2, reinterpret_cast<uint16_t*>(cfg_.X[lane]),
                       nullptr, reinterpret_cast<int32_t*>(cfg_.y[lane]), (r->dst + r->n) % cap, cap, cfg_.scfg.Fp,
                       stream);
  r->n = r->n2 = 0;
}

int LanesLoop::rider_count(int nmodels, int L) const {
  // the riders of the launch: the CUs of the XCDs no lane uses, or (every XCD
  // solves) enough riders to run after the lanes; a launch has grid - L * 32
  int extra = 0;
  if (nmodels > 0 && L == 8 && !lane_riders_) {  // (lane riders: the lanes' own workgroups evaluate)
    const int np = (nmodels + 1) / 2, ppi = riders_ppi_ > 0 && riders_ppi_ < np ? riders_ppi_ : np;
    const int nT = (cfg_.T + 31) / 32, items = tile_riders_ ? nT * ((np + ppi - 1) / ppi) : np * nT;
    extra = items < 256 ? items : 256;
  }
  const int g = lanes_grid(L, extra);
  // (skipped XCDs: the grid is 8 x 32, one XCD's share each -- set_xcd_skip keeps extra at 0)
  return g - L * kLaneWg - (xcd_skip_ ? kLaneWg * __builtin_popcount(xcd_skip_) : 0);
}

void LanesLoop::set_xcd_skip(unsigned mask) {
  mask &= 0xffu;
  const unsigned lanes = ((1u << cfg_.L) - 1u) << cfg_.xcd0;
  if (mask & lanes) throw std::invalid_argument("LanesLoop::set_xcd_skip: a lane's XCD in the mask");
  if (mask && cfg_.L == 8) throw std::invalid_argument("LanesLoop::set_xcd_skip: 8 lanes use every XCD");
  if (mask && !lane_riders_ && cfg_.L == 8) throw std::invalid_argument("LanesLoop::set_xcd_skip: extra riders");
  xcd_skip_ = mask;
}

std::vector<unsigned> LanesLoop::peer_sum_tags() const {
  const int NS = cfg_.scfg.Fp / 32;
  std::vector<unsigned> h(2 * (size_t)NS, 0u);
  if (!psum_rx_) return h;
  hip_check(hipMemcpy(h.data(), psum_rx_tag_, (size_t)NS * 4, hipMemcpyDeviceToHost), "peer_sum rx tags");
  hip_check(hipMemcpy(h.data() + NS, psum_push_tag_, (size_t)NS * 4, hipMemcpyDeviceToHost), "peer_sum push tags");
  return h;
}

void LanesLoop::set_peer_sum(uintptr_t rx, uintptr_t rx_tag, uintptr_t push, uintptr_t push_tag, double wait_s) {
  if (!rx || !rx_tag || !push || !push_tag) throw std::invalid_argument("LanesLoop::set_peer_sum: null region");
  if (!ovl_ || comm_ || cfg_.L < 1)
    throw std::invalid_argument("LanesLoop::set_peer_sum: needs the overlapped launches (PSX_LANES_OVERLAP), lanes "
                                "and no communicator");
  psum_rx_ = reinterpret_cast<const float*>(rx);
  psum_rx_tag_ = reinterpret_cast<const unsigned*>(rx_tag);
  psum_push_ = reinterpret_cast<float*>(push);
  psum_push_tag_ = reinterpret_cast<unsigned*>(push_tag);
  psum_ticks_ = (long long)(std::min(std::max(wait_s, 1.0), 7200.0) * 1e8);
  // the riders flush their counts with atomics and a ticket (no publish launch behind each
  // round): on a GPU shared with the server kernel the publish launch waited 53 us behind
  // the next round's lanes every other round (rocprofv3, profiles/r06/README.md), 88 vs 132
  // us per round; in one process the two forms measure the same (90.1 / 89.8k updates/s)
  slab_on_ = false;
}

// The previous round's rows as models of one evaluation pass: the lanes' local
// models (worker rows, LogisticRegressionTaskSpark.java:186), then the global
// model (server row, ServerProcessor.java:154-165).
void LanesLoop::fill_eval(EvalMulti* ev, const Pending& p, std::vector<int>* slots, std::vector<uint64_t>* seqs,
                          std::vector<int>* kinds) {
  std::memset(ev, 0, sizeof(*ev));
  slots->clear();
  seqs->clear();
  kinds->clear();
  if (!p.valid || !cfg_.sink) return;
  ev->Xt = cfg_.Xt;
  ev->yt = cfg_.yt;
  ev->T = cfg_.T;
  ev->K = cfg_.scfg.K;
  ev->acc = acc_;
  ev->ticket = ticket_;
  const int nw = (cfg_.log_workers && p.workers) ? cfg_.L : 0, n = nw + (cfg_.log_server ? 1 : 0);
  if (n == 0) return;
  // the round's slots in one reservation (one lock of the sink)
  int sl[kMaxEvalModels];
  uint64_t sq[kMaxEvalModels];
  uintptr_t ad[kMaxEvalModels];
  check(api().sink_acquire_many(reinterpret_cast<void*>(cfg_.sink), n, sl, sq, ad), "metrics sink acquire");
  auto add = [&](int i, const uint16_t* hi, const uint16_t* lo, const float* bb, int coff, const float* loss,
                 int kind) {
    EvalModel& m = ev->m[ev->nmodels++];
    m.hi = hi;
    m.lo = lo;
    m.b = bb;
    m.coff = coff;
    m.loss = loss;
    m.slot = reinterpret_cast<char*>(ad[i]);
    m.seq = sq[i];
    slots->push_back(sl[i]);
    seqs->push_back(sq[i]);
    kinds->push_back(kind);
  };
  for (int l = 0; l < nw; ++l)
    add(l, lanes_[l].ohi[p.par], lanes_[l].olo[p.par], lanes_[l].ob[p.par], 0, lanes_[l].loss2 + p.par, 0);
  if (cfg_.log_server) add(nw, cfg_.shi[p.par], cfg_.slo[p.par], cfg_.sb[p.par], cfg_.scoff, nullptr, 1);
  ev->form = tile_riders_ ? 1 : 0;
  ev->ppi = riders_ppi_;
  ev->gq = riders_gq_ ? 1 : 0;
  // every rider of the launch arrives; lane riders: every lane workgroup as well
  ev->nticket = (unsigned)(rider_count(ev->nmodels, cfg_.L) + (lane_riders_ ? cfg_.L * kLaneWg : 0));
  ev->dbg = rider_dbg_;
}

int LanesLoop::fill_lane_eval(LanesArgs* a, int64_t r, int par, const std::vector<int64_t>& seen, SinkRecord* recs) {
  EvalMulti& ev = a->ev;
  std::memset(&ev, 0, sizeof(ev));
  a->lane_eval = 1;
  a->lacc = lacc_;
  a->lticket = lticket_;
  if (!cfg_.sink) return 0;
  ev.Xt = cfg_.Xt;
  ev.yt = cfg_.yt;
  ev.T = cfg_.T;
  ev.K = cfg_.scfg.K;
  const int L = cfg_.L;
  const bool wrows = cfg_.log_workers, srow = cfg_.log_server && pend_.valid;
  const int n = (wrows ? L : 0) + (srow ? 1 : 0);
  if (n == 0) return 0;
  int sl[kMaxEvalModels];
  uint64_t sq[kMaxEvalModels];
  uintptr_t ad[kMaxEvalModels];
  check(api().sink_acquire_many(reinterpret_cast<void*>(cfg_.sink), n, sl, sq, ad), "metrics sink acquire");
  int i = 0, nr = 0;
  if (srow) {  // the reference's order: the server row, then the worker rows
    EvalModel& m = ev.m[kMaxEvalModels - 1];
    m.hi = cfg_.shi[pend_.par];
    m.lo = cfg_.slo[pend_.par];
    m.b = cfg_.sb[pend_.par];
    m.coff = cfg_.scoff;
    m.slot = reinterpret_cast<char*>(ad[i]);
    m.seq = sq[i];
    recs[nr++] = SinkRecord{sl[i], 1 | kSinkTagged, sq[i], -1, -1, pend_.vc, 0};
    ++i;
  }
  if (wrows)
    for (int l = 0; l < L; ++l, ++i) {
      EvalModel& m = ev.m[l];
      m.hi = lanes_[l].ohi[par];
      m.lo = lanes_[l].olo[par];
      m.b = lanes_[l].ob[par];
      m.coff = 0;
      m.loss = lanes_[l].loss2 + par;
      m.slot = reinterpret_cast<char*>(ad[i]);
      m.seq = sq[i];
      recs[nr++] = SinkRecord{sl[i], kSinkTagged, sq[i], -1, cfg_.k[l], r, seen[l]};
    }
  return nr;
}

void LanesLoop::submit_rows(const Pending& p, const std::vector<int>& slots, const std::vector<uint64_t>& seqs,
                            const std::vector<int>& kinds) {
  // the reference's order: the server row, then the worker rows; timestamps are
  // taken by the sink when the evaluation lands (ts = -1); one hand-over
  SinkRecord rec[kMaxEvalModels];
  int n = 0;
  for (size_t i = 0; i < slots.size(); ++i)
    if (kinds[i] == 1) rec[n++] = SinkRecord{slots[i], 1 | kSinkTagged, seqs[i], -1, -1, p.vc, 0};
  int l = 0;
  for (size_t i = 0; i < slots.size(); ++i)
    if (kinds[i] == 0) {
      rec[n++] = SinkRecord{slots[i], kSinkTagged, seqs[i], -1, cfg_.k[l], p.vc, p.nseen[l]};
      ++l;
    }
  if (n) check(api().sink_submit_many(reinterpret_cast<void*>(cfg_.sink), n, rec), "metrics sink submit");
}

void LanesLoop::check_errors(int64_t round) {
  for (int l = 0; l < cfg_.L; ++l) {
    const unsigned long long e = __atomic_load_n(err_host_ + l, __ATOMIC_ACQUIRE);
    if (e) {
      __atomic_store_n(err_host_ + l, 0ull, __ATOMIC_RELAXED);
      throw std::runtime_error("LanesLoop: worker " + std::to_string(cfg_.k[l]) +
                               ": device solver: a cross-workgroup wait timed out (solve " +
                               std::to_string((long long)(e >> 8) - 1) + ", code " + std::to_string((int)(e & 0xff)) +
                               ", noticed at round " + std::to_string((long long)round) + ")");
    }
  }
}

int64_t LanesLoop::new_tuples_needed(int64_t size, int64_t updates) const {
  int64_t k = (int64_t)std::ceil(cfg_.new_frac * (double)size);  // as math.ceil in config.py
  if (k < 0) k = 0;
  if (cfg_.new_cap > 0 && k > cfg_.new_cap) k = cfg_.new_cap;
  if (cfg_.new_ramp > 0 && updates >= 0 && updates < 30) {  // the first solves come early
    const int64_t r = (int64_t)cfg_.new_ramp << updates;
    if (k > r) k = r;
  }
  return k > cfg_.new_rows ? k : cfg_.new_rows;
}

int64_t LanesLoop::run(int64_t rounds, int64_t r0, hipStream_t stream, double max_wait_s, double deadline_ms) {
  const int64_t t_begin = steady_ns();
  const int L = cfg_.L;
  const int KF = cfg_.scfg.K * cfg_.scfg.Fp;
  std::vector<int> slots, kinds;
  std::vector<uint64_t> seqs;
  SinkRecord lrec[kMaxEvalModels];
  int nlrec = 0;
  const bool is_server = !comm_ || comm_->rank() == cfg_.server_rank;
  if (ovl_) {  // the second stream after the caller's earlier work
    ovl_chain_ = false;
    hip_check(hipEventRecord(ovl_in_, stream), "overlap order in");
    hip_check(hipStreamWaitEvent(ostream_, ovl_in_, 0), "overlap order in");
  }
  bool joined = false;
  auto ovl_join = [&]() {  // the caller's later work after every round of this call
    if (!ovl_ || joined) return;
    joined = true;
    hip_check(hipEventRecord(ovl_out_, ostream_), "overlap order out");
    hip_check(hipStreamWaitEvent(stream, ovl_out_, 0), "overlap order out");
    if (psum_rx_ && ovl_n_ > 0) {  // peer_sum: the server's update of the last round into w
      launch_peer_pull(psum_rx_, psum_rx_tag_, (unsigned)ovl_n_, cfg_.w, cfg_.scfg.K, cfg_.scfg.Fp, psum_ticks_,
                       err_host_, stream);
      hip_check(hipGetLastError(), "peer pull launch");
    }
  };
  struct JoinOnThrow {  // an exception out of a round still orders the caller's stream
    bool* joined;
    bool ovl;
    hipEvent_t ev;
    hipStream_t from, to;
    ~JoinOnThrow() {
      if (ovl && !*joined && hipEventRecord(ev, from) == hipSuccess) (void)hipStreamWaitEvent(to, ev, 0);
    }
  } join_guard{&joined, ovl_, ovl_out_, ostream_, stream};
  int64_t done = 0;
  for (; done < rounds; ++done) {
    const int64_t r = r0 + done;
    const int par = ovl_ ? (int)(((r % 3) + 3) % 3) : (int)(r & 1);
    // this round's stream: the two alternate, the call's last round on the caller's --
    // what follows the call there (the last round's evaluation launch, the copies) then
    // needs no wait on the other queue (profiles/r04/s46: 31 us from the last round to
    // that launch when the last round ran on the other stream)
    hipStream_t rs = (ovl_ && ((rounds - 1 - done) & 1)) ? ostream_ : stream;
    int64_t tph = steady_ns();
    auto phase = [&](int i) {
      const int64_t t = steady_ns();
      host_ph_ns_[i] += (double)(t - tph);
      tph = t;
    };
    LanesArgs a;
    std::memset(&a, 0, sizeof(a));
    a.L = L;
    a.par = par;
    // ---- deliveries, then every lane's window (BSP: wait until all have rows, and
    // with a cadence until all saw enough new tuples, WorkerTrainingProcessor.java:63-98
    // runs on every new tuple; psx/runtime/roles.py:WorkerRole.ready) ----
    std::vector<int64_t> seen(L, 0);
    const double wait0 = epoch_ms();
    for (;;) {
      const double now = epoch_ms() - cfg_.t0_ms;
      for (int l = 0; l < L; ++l) poll(l, now, &a.r[l], rs);
      bool ready = true, rows = true;
      for (int l = 0; l < L; ++l) {
        int64_t size = 0, start = 0, sn = 0;
        check(api().window_state(reinterpret_cast<void*>(cfg_.window[l]), &size, &start, &sn), "window state");
        a.r[l].B = (int)size;
        a.r[l].start = (int)start;
        seen[l] = sn;
        rows &= size > 0;
        const int64_t need = new_tuples_needed(size, r);  // (BSP: every lane solved r times)
        ready &= size > 0 && (need <= 0 || sn - seen_at_solve_[l] >= need || exhausted(l));
      }
      if (ready) break;
      bool end = false;
      for (int l = 0; l < L; ++l)  // a lane with an empty window and nothing left to come: the run ends
        end |= a.r[l].B <= 0 && exhausted(l);
      if (deadline_ms > 0.0 && epoch_ms() >= deadline_ms) end = true;
      if (end) {
        for (int l = 0; l < L; ++l)  // rows delivered meanwhile: into the ring now
          if (a.r[l].n > 0 || a.r[l].n2 > 0) flush_ingest(l, &a.r[l], rs);
        ovl_join();
        rounds_run_ += done;
        host_ns_ += (double)(steady_ns() - t_begin);
        return done;
      }
      if (!rows && epoch_ms() - wait0 > max_wait_s * 1000.0) throw std::runtime_error("LanesLoop: no rows for a worker");
      std::this_thread::sleep_for(std::chrono::microseconds(500));
    }
    for (int l = 0; l < L; ++l) {
      seen_at_solve_[l] = seen[l];
      a.r[l].delay_us = l < (int)cfg_.delay_us.size() ? cfg_.delay_us[l] : 0;
    }
    phase(0);
    // ---- the round kernel: solves + update + riding evaluation of the last round ----
    if (side_eval_) {
      // this round rewrites the fragments the evaluation of round r - 2 reads
      if (eval_pending_[par]) {
        if (side_sync_ == 0)
          hip_check(hipStreamWaitEvent(stream, ev_eval_[par], 0), "wait evaluation");
        else if (side_sync_ == 1)
          hip_check(hipStreamWaitValue32(stream, sflags_ + 1, (uint32_t)(eval_round_[par] + 1), hipStreamWaitValueGte),
                    "wait evaluation");
      }
      eval_pending_[par] = false;
      slots.clear();
    } else if (lane_eval_) {
      slots.clear();
      nlrec = fill_lane_eval(&a, r, par, seen, lrec);
    } else {
      fill_eval(&a.ev, pend_, &slots, &seqs, &kinds);
    }
    phase(1);
    a.nride = rider_count(a.ev.nmodels, L);
    a.lane_riders = (lane_riders_ && a.ev.nmodels > 0 && !side_eval_ && !lane_eval_) ? 1 : 0;
    a.dsX = cfg_.dsX;
    a.dsy = cfg_.dsy;
    a.w = cfg_.w;
    a.lr = cfg_.lr;
    a.dsum = comm_ ? dsum_ : nullptr;
    a.shi = cfg_.shi[par];
    a.slo = cfg_.slo[par];
    a.sb = cfg_.sb[par];
    a.scoff = cfg_.scoff;
    a.arrive = arrive_;
    a.claim = claim_;
    a.cpar = (int)(launches_ & 1);
    a.xcd0 = cfg_.xcd0;
    // (the tile-resident riders pop their tiles from the first of these counters)
    a.ev.xq = ((xcd_riders_ || tile_riders_) && a.ev.nmodels > 0) ? (ovl_ ? ovlq_ : claim_ + 32 * a.cpar + 16)
                                                                     : nullptr;
    // (from the injected round on: a round whose workgroups happen to arrive together
    // polls nothing, so one round alone would not always time out)
    a.spin_max = (inject_round_ >= 0 && r >= inject_round_) ? inject_spin_ : 0;
    a.xcd_skip = xcd_skip_;
    if (psum_rx_) {  // the push into the server's inbox, the pull from this rank's receive slot
      a.push = psum_push_;
      a.push_tag = psum_push_tag_;
      a.rx = psum_rx_;
      a.rx_tag = psum_rx_tag_;
      a.peer_ticks = psum_ticks_;
    }
    if (tr_) {
      a.tr = tr_;
      a.tr_slot = (int)(tr_n_ % tr_cap_);
      tr_round_[a.tr_slot] = r;
      ++tr_n_;
    }
    if (L > 0 || a.ev.nmodels > 0) {
      if (a.nride == 0) a.nride = rider_count(0, L);
      if (rider_dbg_ && a.ev.nmodels > 0) {  // PSX_LANES_STAMPS: this launch's rider timeline
        hip_check(hipMemsetAsync(rider_dbg_, 0, 64 * sizeof(long long), rs), "rider stamps");
        hip_check(hipMemsetAsync(rider_dbg_ + 12, 0xff, sizeof(long long), rs), "rider stamps");
        hip_check(hipMemsetAsync(rider_dbg_ + 15, 0xff, sizeof(long long), rs), "rider stamps");
      }
      if (ovl_) {
        a.ovl = 1;
        a.round = (unsigned)ovl_n_;
        // (the call's last round publishes in its own launch: nothing follows it to co-run
        // with a publish launch, which would only lengthen the call's tail)
        if (slab_on_ && done + 1 < rounds && a.ev.nmodels > 0 && a.ev.form == 1 &&
            a.ev.nticket <= (unsigned)kSlabRiders)
          a.ev.slab = slab_;
        a.applied = applied_;
        a.evdone = evdone_;
        // dispatched once every workgroup of the previous round's launch holds its CU
        // (its lanes wait for nothing of this launch, so this one may take the CUs it frees)
        if (ovl_chain_)
          hip_check(hipStreamWaitValue32(rs, claim_ + 32 * ovl_prev_cpar_ + 9, (uint32_t)ovl_prev_grid_,
                                         hipStreamWaitValueGte),
                    "overlap: previous launch dispatched");
      }
      launch_lanes_round(cfg_.scfg, lanes_dev_, a, S_, rs);
      hip_check(hipGetLastError(), "lanes round launch");
      ++launches_;
      if (ovl_) {
        if (a.ev.slab) {  // the rows of this launch's evaluation, co-running with the next round
          launch_lanes_publish(a.ev, rs);
          hip_check(hipGetLastError(), "publish launch");
        }
        hip_check(hipStreamWriteValue32(rs, evdone_, (uint32_t)(ovl_n_ + 1), 0), "overlap: launch done");
        hip_check(hipEventRecord(ovl_last_, rs), "overlap: last launch");
        ovl_prev_grid_ = lanes_grid(L, a.nride) - (xcd_skip_ ? kLaneWg * __builtin_popcount(xcd_skip_) : 0);
        ovl_prev_cpar_ = a.cpar;
        ovl_chain_ = true;
        ++ovl_n_;
      }
    }
    phase(2);
    if (!slots.empty()) submit_rows(pend_, slots, seqs, kinds);
    if (nlrec) check(api().sink_submit_many(reinterpret_cast<void*>(cfg_.sink), nlrec, lrec), "metrics sink submit");
    nlrec = 0;
    // ---- multi-rank: lane sums -> server (reduce), update, weights -> every rank ----
    if (comm_) {
      hipStream_t cs = stream;
      if (L == 0) hip_check(hipMemsetAsync(dsum_, 0, (size_t)P_ * 4, stream), "zero contribution");
      if (cfg_.allreduce) {  // every replica applies the same summed update
        comm_->all_reduce(dsum_, dsum_, (size_t)P_, Comm::kF32, cs);
        launch_server_apply(cfg_.scfg.K, cfg_.scfg.F, cfg_.scfg.Fp, cfg_.w, dsum_, cfg_.lr,
                            cfg_.shi[par] ? cfg_.shi[par] : upd_hi_, cfg_.shi[par] ? cfg_.slo[par] : upd_lo_,
                            cfg_.shi[par] ? cfg_.sb[par] : upd_b_, cs, cfg_.scoff);
      } else {  // push: reduce to the server rank; update there; pull: broadcast
        comm_->reduce(dsum_, dsum_, (size_t)P_, Comm::kF32, cfg_.server_rank, cs);
        if (is_server)
          launch_server_apply(cfg_.scfg.K, cfg_.scfg.F, cfg_.scfg.Fp, cfg_.w, dsum_, cfg_.lr, cfg_.shi[par],
                              cfg_.slo[par], cfg_.sb[par], cs, cfg_.scoff);
        comm_->broadcast(cfg_.w, cfg_.w, (size_t)P_, Comm::kF32, cfg_.server_rank, cs);
      }
      hip_check(hipGetLastError(), "server update launch");
    }
    (void)KF;
    // ---- this round's rows: evaluated by the next launch, or side launch now ----
    last_par_ = par;
    pend_.valid = cfg_.sink != 0 && (!lane_eval_ || cfg_.log_server);
    pend_.workers = !lane_eval_;  // lane evaluation: this round's worker rows are already out
    pend_.vc = r;
    pend_.par = par;
    pend_.nseen = seen;
    if (side_eval_) {
      EvalMulti ev;
      fill_eval(&ev, pend_, &slots, &seqs, &kinds);
      if (ev.nmodels > 0) {
        ev.acc = acc2_;
        ev.ticket = ticket2_;
        ev.nticket = (unsigned)lanes_eval_grid();
        if (side_sync_ == 3) {  // stream order: the evaluation launch right behind the round
          launch_lanes_eval(cfg_.scfg, ev, stream);
          hip_check(hipGetLastError(), "evaluation launch");
          submit_rows(pend_, slots, seqs, kinds);
          pend_.valid = false;
          if (cfg_.tracker && is_server)
            check(api().tracker_bsp_round(reinterpret_cast<void*>(cfg_.tracker), r), "tracker");
          check_errors(r);
          continue;
        }
        if (side_sync_ == 1) {
          hip_check(hipStreamWriteValue32(stream, sflags_, (uint32_t)(r + 1), 0), "round done");
          hip_check(hipStreamWaitValue32(side_, sflags_, (uint32_t)(r + 1), hipStreamWaitValueGte), "side waits");
        } else {
          hip_check(hipEventRecord(ev_round_[par], stream), "record round");
          hip_check(hipStreamWaitEvent(side_, ev_round_[par], 0), "side waits round");
        }
        launch_lanes_eval(cfg_.scfg, ev, side_);
        hip_check(hipGetLastError(), "side evaluation launch");
        if (side_sync_ == 1)
          hip_check(hipStreamWriteValue32(side_, sflags_ + 1, (uint32_t)(r + 1), 0), "evaluation done");
        hip_check(hipEventRecord(ev_eval_[par], side_), "record evaluation");
        eval_pending_[par] = true;
        eval_round_[par] = r;
        submit_rows(pend_, slots, seqs, kinds);
      }
      pend_.valid = false;
    }
    if (cfg_.tracker && is_server) check(api().tracker_bsp_round(reinterpret_cast<void*>(cfg_.tracker), r), "tracker");
    check_errors(r);
    phase(3);
  }
  ovl_join();
  rounds_run_ += done;
  host_ns_ += (double)(steady_ns() - t_begin);
  return done;
}

void LanesLoop::flush(hipStream_t stream) {
  for (int p = 0; p < 2; ++p)  // side evaluations: ordered before the stream's later work
    if (eval_pending_[p]) {
      hip_check(hipStreamWaitEvent(stream, ev_eval_[p], 0), "wait evaluation");
      eval_pending_[p] = false;
    }
  if (!pend_.valid || !cfg_.sink) return;
  std::vector<int> slots, kinds;
  std::vector<uint64_t> seqs;
  LanesArgs a;
  std::memset(&a, 0, sizeof(a));
  a.L = 0;
  fill_eval(&a.ev, pend_, &slots, &seqs, &kinds);
  a.ev.nticket = (unsigned)rider_count(a.ev.nmodels, 0);
  a.nride = (int)a.ev.nticket;
  a.w = cfg_.w;
  a.arrive = arrive_;
  a.claim = claim_;
  a.cpar = (int)(launches_ & 1);
  a.xcd0 = cfg_.xcd0;
  a.xcd_skip = xcd_skip_;
  a.ev.xq = (xcd_riders_ || tile_riders_) ? claim_ + 32 * a.cpar + 16 : nullptr;
  if (a.ev.nmodels > 0) {
    launch_lanes_round(cfg_.scfg, lanes_dev_, a, S_, stream);
    hip_check(hipGetLastError(), "lanes evaluation launch");
    ++launches_;
  }
  submit_rows(pend_, slots, seqs, kinds);
  pend_ = Pending{};
}

std::vector<int> LanesLoop::stats(int lane, hipStream_t stream) const {
  std::vector<int> v(8, 0);
  hip_check(hipMemcpyAsync(v.data(), lanes_.at(lane).dv.stats, 8 * sizeof(int), hipMemcpyDeviceToHost, stream),
            "lane stats");
  hip_check(hipStreamSynchronize(stream), "sync");
  return v;
}

float LanesLoop::loss(int lane, hipStream_t stream) const {
  float v[kLaneBufs] = {0.f, 0.f, 0.f};
  hip_check(hipMemcpyAsync(v, lanes_.at(lane).loss2, kLaneBufs * sizeof(float), hipMemcpyDeviceToHost, stream),
            "lane loss");
  hip_check(hipStreamSynchronize(stream), "sync");
  return v[last_par_];
}

std::vector<long long> LanesLoop::read_stamps(int lane, hipStream_t stream) const {
  std::vector<long long> v;
  const long long* d = lanes_.at(lane).dv.dbg;
  if (!d) return v;
  v.resize(32 * 16);
  hip_check(hipMemcpyAsync(v.data(), d, v.size() * sizeof(long long), hipMemcpyDeviceToHost, stream), "stamps");
  hip_check(hipStreamSynchronize(stream), "sync");
  return v;
}

std::vector<long long> LanesLoop::read_rider_stamps(hipStream_t stream) const {
  std::vector<long long> v;
  if (!rider_dbg_) return v;
  v.resize(64);
  hip_check(hipMemcpyAsync(v.data(), rider_dbg_, v.size() * sizeof(long long), hipMemcpyDeviceToHost, stream),
            "rider stamps");
  hip_check(hipStreamSynchronize(stream), "sync");
  return v;
}

uintptr_t LanesLoop::delta_ptr(int lane) const { return reinterpret_cast<uintptr_t>(lanes_.at(lane).dv.delta); }

void LanesLoop::copy_out(int lane, uintptr_t loss_dst, uintptr_t delta_dst, hipStream_t stream) const {
  const LaneDev& ld = lanes_.at(lane);
  if (loss_dst)
    hip_check(hipMemcpyAsync(reinterpret_cast<void*>(loss_dst), ld.loss2 + last_par_, sizeof(float),
                             hipMemcpyDeviceToDevice, stream),
              "lane loss copy");
  if (delta_dst)
    hip_check(hipMemcpyAsync(reinterpret_cast<void*>(delta_dst), ld.dv.delta, (size_t)P_ * sizeof(float),
                             hipMemcpyDeviceToDevice, stream),
              "lane delta copy");
}

void LanesLoop::copy_out_all(const std::vector<uintptr_t>& loss_dst, const std::vector<uintptr_t>& delta_dst,
                             hipStream_t stream) const {
  const int L = cfg_.L;
  if ((int)loss_dst.size() != L || (int)delta_dst.size() != L)
    throw std::invalid_argument("LanesLoop::copy_out_all: one destination per lane");
  LanesCopyOut c;
  std::memset(&c, 0, sizeof(c));
  c.L = L;
  c.P = (int)P_;
  for (int l = 0; l < L; ++l) {
    const LaneDev& ld = lanes_.at(l);
    // (16-B pieces: the destinations are torch allocations, the sources workspace
    // slices; anything else takes the per-lane copies)
    if (delta_dst[l] % 16 != 0 || reinterpret_cast<uintptr_t>(ld.dv.delta) % 16 != 0) {
      for (int j = 0; j < L; ++j) copy_out(j, loss_dst[j], delta_dst[j], stream);
      return;
    }
    c.src_d[l] = ld.dv.delta;
    c.dst_d[l] = reinterpret_cast<float*>(delta_dst[l]);
    c.src_l[l] = ld.loss2 + last_par_;
    c.dst_l[l] = reinterpret_cast<float*>(loss_dst[l]);
  }
  launch_lanes_copy_out(c, stream);
  hip_check(hipGetLastError(), "lanes copy-out launch");
}

// ---------------------------------------------------------------------------
// Asynchronous consistency (SSP / ASP): see lanes_loop.h and lanes_kernels.h.

void LanesLoop::ensure_async() {
  if (aws_) return;
  const SolverCfg& s = cfg_.scfg;
  const int L = cfg_.L, FP = s.Fp, NS = FP / 32;
  if (L < 1) throw std::invalid_argument("LanesLoop::run_async: no lanes");
  for (int l = 0; l < L; ++l)
    if (local_total_[l] < s.cap)  // pending rows of one release span at most one epoch wrap
      throw std::invalid_argument("LanesLoop::run_async: a worker's shard is smaller than its ring");
  size_t off = 0;
  auto take = [&](size_t bytes) {
    const size_t o = off;
    off = align_up(off + bytes, 256);
    return o;
  };
  struct Offs {
    size_t wpull, shi, slo, sb, acc, etk, flags, rec, relc, eslab;
  };
  std::vector<Offs> o(L);
  for (int l = 0; l < L; ++l) {
    o[l].wpull = take((size_t)P_ * 4);
    o[l].shi = take((size_t)16 * FP * 2);
    o[l].slo = take((size_t)16 * FP * 2);
    o[l].sb = take(16 * 4);
    o[l].acc = take((size_t)2 * 256 * kAccStride * 4);
    o[l].etk = take(4);
    o[l].flags = take((size_t)kLaneWg * 32 * 8);
    o[l].rec = take(32 * 8);
    o[l].relc = take(8);
    o[l].eslab = take((size_t)kLaneWg * 128 * 4);
  }
  const size_t o_tab = take(sizeof(AsyncLaneDev) * L);
  const size_t o_snap = take((size_t)R_ * P_ * 4);
  const size_t o_stag = take((size_t)R_ * NS * 4);
  const size_t o_tick = take(8);
  const size_t o_turn = take((size_t)NS * 32 * 8);
  hip_check(hipMalloc(&aws_, off), "hipMalloc(async workspace)");
  hip_check(hipMemset(aws_, 0, off), "hipMemset(async workspace)");
  hip_check(hipHostMalloc((void**)&rel_host_, sizeof(AsyncRelease) * L, hipHostMallocCoherent | hipHostMallocMapped),
            "hipHostMalloc(release records)");
  hip_check(hipHostMalloc((void**)&tok_host_, sizeof(AsyncToken) * ring_, hipHostMallocCoherent | hipHostMallocMapped),
            "hipHostMalloc(token ring)");
  std::memset((void*)rel_host_, 0, sizeof(AsyncRelease) * L);
  std::memset((void*)tok_host_, 0, sizeof(AsyncToken) * ring_);
  hip_check(hipStreamCreateWithFlags(&astream_, hipStreamNonBlocking), "hipStreamCreate(async)");
  hip_check(hipEventCreateWithFlags(&aev_in_, hipEventDisableTiming), "hipEventCreate");
  hip_check(hipEventCreateWithFlags(&aev_out_, hipEventDisableTiming), "hipEventCreate");
  char* b = static_cast<char*>(aws_);
  al_.resize(L);
  for (int l = 0; l < L; ++l) {
    AsyncLaneDev& A = al_[l];
    std::memset(&A, 0, sizeof(A));
    A.wpull = reinterpret_cast<float*>(b + o[l].wpull);
    // the lane's solver as the asynchronous launch uses it: buffer 0 of the local
    // model / loss, the pulled weights from its private copy, no fused update
    A.dv = lanes_[l].dv;
    A.dv.out_hi = lanes_[l].ohi[0];
    A.dv.out_lo = lanes_[l].olo[0];
    A.dv.b_fin = lanes_[l].ob[0];
    A.dv.loss = lanes_[l].loss2;
    A.dv.w_old = A.wpull;
    A.dv.w_new = nullptr;
    A.dv.ap_w = nullptr;
    A.dv.spin_max = 0;
    A.spart = lanes_[l].spart;
    A.ctrl = lanes_[l].ctrl;
    A.shi = reinterpret_cast<uint16_t*>(b + o[l].shi);
    A.slo = reinterpret_cast<uint16_t*>(b + o[l].slo);
    A.sb = reinterpret_cast<float*>(b + o[l].sb);
    A.acc = reinterpret_cast<int*>(b + o[l].acc);
    A.eticket = reinterpret_cast<unsigned*>(b + o[l].etk);
    A.flags = reinterpret_cast<unsigned long long*>(b + o[l].flags);
    A.rec = reinterpret_cast<unsigned long long*>(b + o[l].rec);
    A.relc = reinterpret_cast<unsigned long long*>(b + o[l].relc);
    A.eslab = reinterpret_cast<int*>(b + o[l].eslab);
    A.rel = rel_host_ + l;
    if (peer_rx_) {
      A.inbox = reinterpret_cast<float*>(peer_inbox_[l]);
      A.inbox_tag = reinterpret_cast<unsigned*>(peer_inbox_tag_[l]);
    }
  }
  al_dev_ = reinterpret_cast<AsyncLaneDev*>(b + o_tab);
  hip_check(hipMemcpy(al_dev_, al_.data(), sizeof(AsyncLaneDev) * L, hipMemcpyHostToDevice), "async table upload");
  AsyncArgs& a = aargs_;
  std::memset(&a, 0, sizeof(a));
  a.L = L;
  a.dsX = cfg_.dsX;
  a.dsy = cfg_.dsy;
  a.w = cfg_.w;
  a.snap = reinterpret_cast<float*>(b + o_snap);
  a.snap_tag = reinterpret_cast<unsigned*>(b + o_stag);
  a.R = R_;
  a.sstride = P_;
  if (peer_rx_) {  // the receive slots are the peer region's (lane l = slot l)
    a.snap = peer_rx_;
    a.snap_tag = peer_rx_tag_;
    a.R = L;
    a.sstride = peer_stride_;
    a.peer_rx = 1;
  }
  a.ticket = reinterpret_cast<unsigned long long*>(b + o_tick);
  a.turn = reinterpret_cast<unsigned long long*>(b + o_turn);
  a.tok = tok_host_;
  a.ring = ring_;
  a.Xt = cfg_.Xt;
  a.yt = cfg_.yt;
  a.T = cfg_.T;
  a.Ti = cfg_.Ti;
  a.Tv = cfg_.Tv;
  a.tnz = (cfg_.Ti && cfg_.Tv && cfg_.tnz > 0 && cfg_.tnz % 8 == 0) ? cfg_.tnz : 0;
  a.claim = claim_;
  relc_.assign(L, 0);
  pend_r_.assign(L, LaneRound{});
  state_.assign(L, kIdle);
  want_vc_.assign(L, 0);
  runrec_.assign(L, RunRec{});
  lane_of_.assign(cfg_.N, -1);
  for (int l = 0; l < L; ++l) lane_of_.at(cfg_.k[l]) = l;
}

namespace {
// the pending new rows of a lane as <= 2 contiguous runs (LaneRound n / n2)
void drop_front(LaneRound& r, int64_t d, int64_t cap) {
  while (d > 0 && r.n > 0) {
    const int64_t k = d < r.n ? d : r.n;
    r.first += k * r.step;
    r.dst = (int)((r.dst + k) % cap);
    r.n -= (int)k;
    d -= k;
    if (r.n == 0 && r.n2 > 0) {
      r.first = r.first2;
      r.n = r.n2;
      r.n2 = 0;
    }
  }
}
void append_run(LaneRound& r, long long src_first, long long step, int64_t slot, int64_t run, int64_t cap) {
  if (r.n == 0) {
    r.first = src_first;
    r.step = step;
    r.n = (int)run;
    r.dst = (int)slot;
    r.n2 = 0;
    return;
  }
  if ((r.dst + r.n + r.n2) % cap != slot) throw std::logic_error("LanesLoop: ring slots of a delivery not contiguous");
  if (r.n2 == 0 && src_first == r.first + (long long)r.n * r.step)
    r.n += (int)run;
  else if (r.n2 > 0 && src_first == r.first2 + (long long)r.n2 * r.step)
    r.n2 += (int)run;
  else if (r.n2 == 0) {
    r.first2 = src_first;
    r.n2 = (int)run;
  } else {
    throw std::logic_error("LanesLoop: pending rows of a release span three runs");
  }
}
}  // namespace

int64_t LanesLoop::poll_async(int lane, double now_ms) {
  if (exhausted(lane)) return 0;
  const int k = cfg_.k[lane];
  const int64_t lt = local_total_[lane];
  int64_t& nl = next_local_[lane];
  const int64_t limit = lt * cfg_.epochs - nl;
  int64_t n;
  if (cfg_.per_iter_rows > 0) {
    n = cfg_.per_iter_rows < limit ? cfg_.per_iter_rows : limit;
    times_.assign((size_t)n, now_ms);
  } else {
    const int64_t epoch = nl / lt, cur = nl - epoch * lt;
    int64_t mx = limit < lt - cur ? limit : lt - cur;
    if (mx > (int64_t(1) << 22)) mx = int64_t(1) << 22;
    times_.resize(mx > 0 ? (size_t)mx : 1);
    n = api().due_rows(k, cfg_.N, cfg_.p_ms, cfg_.ds_rows, cur, now_ms, mx, times_.data());
    check(n, "due_rows");
  }
  if (n <= 0) return 0;
  const int64_t first = api().window_insert_many(reinterpret_cast<void*>(cfg_.window[lane]), times_.data(), n);
  check(first, "window insert");
  const int64_t cap = cfg_.scfg.cap;
  const int64_t keep = n < cap ? n : cap, skip = n - keep;
  LaneRound& r = pend_r_[lane];
  const int64_t tot = (int64_t)r.n + r.n2 + keep;
  if (tot > cap) drop_front(r, tot - cap, cap);  // rows the ring overwrites before the next solve
  int64_t slot = (first + skip) % cap, pos = nl + skip, remaining = keep;
  while (remaining > 0) {  // split at the shard's epoch boundaries
    const int64_t cur = pos % lt;
    const int64_t run = remaining < lt - cur ? remaining : lt - cur;
    append_run(r, k + cur * (int64_t)cfg_.N, cfg_.N, slot, run, cap);
    slot = (slot + run) % cap;
    pos += run;
    remaining -= run;
  }
  nl += n;
  return n;
}

void LanesLoop::write_release(int lane, const RelRec& q) {
  TagChunk ch[kRelChunks];
  pack_release(q, (unsigned)(++relc_[lane]), ch);
  volatile TagChunk* dst = rel_host_[lane].ch;
  for (int i = 0; i < kRelChunks; ++i) {
    __m128i v;
    std::memcpy(&v, &ch[i], 16);
    _mm_store_si128((__m128i*)(void*)&dst[i], v);  // one 16-B store per chunk
  }
  std::atomic_thread_fence(std::memory_order_release);
}

bool LanesLoop::try_release(int lane, int64_t vc, double now_ms, int64_t snap) {
  poll_async(lane, now_ms);
  int64_t size = 0, start = 0, sn = 0;
  check(api().window_state(reinterpret_cast<void*>(cfg_.window[lane]), &size, &start, &sn), "window state");
  const int64_t need = new_tuples_needed(size, vc);  // (vc: the worker's completed pushes)
  if (!(size > 0 && (need <= 0 || sn - seen_at_solve_[lane] >= need || exhausted(lane)))) return false;
  seen_at_solve_[lane] = sn;
  RelRec q;
  std::memset(&q, 0, sizeof(q));
  q.vc = vc;
  // the weights right after the latest applied update (remote: the lane's receive slot)
  q.snap = snap >= 0 ? (long long)snap : (long long)aticket_;
  q.r = pend_r_[lane];
  q.r.B = (int)size;
  q.r.start = (int)start;
  if (q.r.n == 0) q.r.step = cfg_.N;
  pend_r_[lane] = LaneRound{};
  RunRec& rr = runrec_[lane];
  rr = RunRec{};
  rr.vc = vc;
  rr.nseen = sn;
  rr.snap = q.snap;
  rr.r = q.r;
  if (cfg_.sink) {
    const bool w = cfg_.log_workers, sv = cfg_.log_server && lane == log_lane_;
    const int n = (w ? 1 : 0) + (sv ? 1 : 0);
    if (n) {
      int sl[2];
      uint64_t sq[2];
      uintptr_t ad[2];
      check(api().sink_acquire_many(reinterpret_cast<void*>(cfg_.sink), n, sl, sq, ad), "metrics sink acquire");
      int i = 0;
      if (w) {
        rr.slot_w = sl[i];
        rr.seq_w = sq[i];
        q.slot_w = ad[i];
        q.seq_w = (unsigned)sq[i];
        ++i;
      }
      if (sv) {
        rr.slot_s = sl[i];
        rr.seq_s = sq[i];
        q.slot_s = ad[i];
        q.seq_s = (unsigned)sq[i];
      }
    }
  }
  q.delay_us = lane < (int)cfg_.delay_us.size() ? cfg_.delay_us[lane] : 0;
  q.pull_tag = peer_rx_ ? pull_tag_[lane] : 0u;
  write_release(lane, q);
  return true;
}

void LanesLoop::set_trace(int cap) {
  if (tr_) {
    hip_check(hipDeviceSynchronize(), "trace ring free");
    (void)hipFree(tr_);
    tr_ = nullptr;
  }
  tr_cap_ = cap > 0 ? cap : 0;
  tr_n_ = tr_taken_ = 0;
  tr_tick_ = aticket_;
  if (!tr_cap_) return;
  const size_t bytes = ((size_t)tr_cap_ * kMaxLanes * 4 + 2 * kMaxLanes) * sizeof(long long);
  hip_check(hipMalloc((void**)&tr_, bytes), "trace ring");
  hip_check(hipMemset(tr_, 0, bytes), "trace ring");
  tr_round_.assign((size_t)tr_cap_, -1);
}

std::vector<std::vector<int64_t>> LanesLoop::trace_take(hipStream_t s) {
  std::vector<std::vector<int64_t>> out;
  if (!tr_) return out;
  hip_check(hipStreamSynchronize(s), "trace take");
  hip_check(hipDeviceSynchronize(), "trace take");  // (the round / asynchronous streams too)
  std::vector<long long> h((size_t)tr_cap_ * kMaxLanes * 4);
  hip_check(hipMemcpy(h.data(), tr_, h.size() * sizeof(long long), hipMemcpyDeviceToHost), "trace copy");
  const int L = cfg_.L;
  // BSP rounds
  const int64_t first = std::max(tr_taken_, tr_n_ - (int64_t)tr_cap_);
  for (int64_t n = first; n < tr_n_; ++n) {
    const int sl = (int)(n % tr_cap_);
    for (int l = 0; l < L; ++l) {
      const long long* e = h.data() + ((size_t)sl * kMaxLanes + l) * 4;
      out.push_back({0, tr_round_[sl], l, cfg_.k[l], e[0], e[1], e[2], e[3]});
    }
  }
  tr_taken_ = tr_n_;
  // asynchronous tickets (their entries are [t % cap][4] in the same ring)
  const uint64_t t0 = std::max<uint64_t>(tr_tick_, aticket_ > (uint64_t)tr_cap_ ? aticket_ - tr_cap_ : 0);
  for (uint64_t t = t0 + 1; t <= aticket_; ++t) {
    const long long* e = h.data() + (size_t)(t % (uint64_t)tr_cap_) * 4;
    const int l = (int)e[0];
    out.push_back({1, (int64_t)t, l, (l >= 0 && l < L) ? cfg_.k[l] : -1, e[1], e[2], e[3], 0});
  }
  tr_tick_ = aticket_;
  return out;
}

std::vector<int64_t> LanesLoop::clock_ref(hipStream_t s) {
  long long* h = nullptr;
  hip_check(hipHostMalloc((void**)&h, sizeof(long long), hipHostMallocDefault), "clock probe");
  *h = 0;
  timespec a{}, b{};
  clock_gettime(CLOCK_MONOTONIC, &a);
  launch_clock_probe(h, s);
  hip_check(hipStreamSynchronize(s), "clock probe");
  clock_gettime(CLOCK_MONOTONIC, &b);
  const int64_t ticks = *h;
  (void)hipHostFree(h);
  return {(int64_t)a.tv_sec * 1000000000ll + a.tv_nsec, ticks, (int64_t)b.tv_sec * 1000000000ll + b.tv_nsec};
}

std::string LanesLoop::launch_report() {
  // (failure reports) how far the current persistent launch got: its workgroups that
  // claimed a lane slot per XCD and all that started, read on a stream of its own
  // with a bounded wait
  std::string m = "launch " + std::to_string((long long)launches_) + ": ";
  const hipError_t q = hipStreamQuery(astream_);
  m += q == hipSuccess ? "drained" : (q == hipErrorNotReady ? "running" : hipGetErrorString(q));
  unsigned* h = nullptr;
  hipStream_t s = nullptr;
  if (hipHostMalloc((void**)&h, 32 * sizeof(unsigned), hipHostMallocDefault) != hipSuccess) return m;
  std::memset(h, 0xff, 32 * sizeof(unsigned));
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) == hipSuccess &&
      hipMemcpyAsync(h, claim_ + 32 * ((launches_ - 1) & 1), 32 * sizeof(unsigned), hipMemcpyDeviceToHost, s) ==
          hipSuccess) {
    const double t0 = epoch_ms();
    while (hipStreamQuery(s) == hipErrorNotReady && epoch_ms() - t0 < 2000.0)
      std::this_thread::sleep_for(std::chrono::microseconds(100));
    if (hipStreamQuery(s) == hipSuccess) {
      m += "; lane slots claimed per XCD:";
      for (int j = 0; j < 8; ++j) m += " " + std::to_string(h[j]);
      m += "; workgroups started " + std::to_string(h[9]) + " of " + std::to_string(8 * kLaneWg);
    } else {
      m += "; (claim counters unreadable: the copy did not complete in 2 s)";
    }
  }
  if (s) (void)hipStreamDestroy(s);
  (void)hipHostFree(h);
  return m;
}

void LanesLoop::prepare_async() {
  ensure_async();
  if (!peer_rx_) return;
  launch_async(astream_, true);
  stop_all(astream_);
  hip_check(hipStreamSynchronize(astream_), "warm-up launch");
  check_errors(-1);
}

void LanesLoop::set_injection(const std::vector<int64_t>& crash, const std::vector<int64_t>& stop, bool drop) {
  if ((!crash.empty() && (int)crash.size() != cfg_.L) || (!stop.empty() && (int)stop.size() != cfg_.L))
    throw std::invalid_argument("LanesLoop::set_injection: one entry per lane");
  inj_crash_ = crash;
  inj_stop_ = stop;
  inj_drop_ = drop;
}

void LanesLoop::stop_lane(int l) {
  if (lane_stopped_.size() != (size_t)cfg_.L) lane_stopped_.assign(cfg_.L, 0);
  if (lane_stopped_[l]) return;  // (an unread second stop record would end the lane's next launch at once)
  RelRec q;
  std::memset(&q, 0, sizeof(q));
  q.stop = 1;
  write_release(l, q);
  lane_stopped_[l] = 1;
}

void LanesLoop::stop_all(hipStream_t stream) {
  for (int l = 0; l < cfg_.L; ++l) stop_lane(l);
  // the launch drains once every workgroup has been dispatched and returned; a bounded
  // wait turns a launch that cannot drain into an error that says how far dispatch got
  const double t0 = epoch_ms();
  for (;;) {
    const hipError_t e = hipStreamQuery(astream_);
    if (e == hipSuccess) break;
    if (e != hipErrorNotReady) hip_check(e, "asynchronous launch drain");
    if (epoch_ms() - t0 > 30000.0) {
      unsigned c[32] = {0};
      (void)hipMemcpy(c, claim_ + 32 * ((launches_ - 1) & 1), sizeof(c), hipMemcpyDeviceToHost);
      std::string m = "LanesLoop: the asynchronous launch did not drain in 30 s; workgroups dispatched per XCD"
                      " (lane claims 0..7, others):";
      for (int j = 0; j < 9; ++j) m += " " + std::to_string(c[j]);
      throw std::runtime_error(m);
    }
    std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
  hip_check(hipEventRecord(aev_out_, astream_), "async order out");  // the caller's later work after it
  hip_check(hipStreamWaitEvent(stream, aev_out_, 0), "async order out");
}

void LanesLoop::launch_async(hipStream_t stream, bool remote) {
  // local: the snapshot of the current weights (aticket_) + the slices' turn words;
  // remote: the ticket (= this rank's push order) only
  AsyncArgs a = aargs_;
  a.lr = cfg_.lr;  // the server step (ServerProcessor.java:36): w += lr * delta
  a.log_lane = remote ? -1 : log_lane_;
  a.remote = remote ? 1 : 0;
  a.xcd0 = cfg_.xcd0;
  if (remote) a.w = nullptr;
  a.dbg_delta = remote ? nullptr : dbg_delta_;
  a.tr = tr_;
  a.tr_cap = tr_cap_;
  a.dbg_cap = dbg_cap_ > 0 ? dbg_cap_ : 1;
  a.launch = ++launch_no_;
  a.cpar = (int)(launches_ & 1);
  lane_stopped_.assign(cfg_.L, 0);
  // the lanes' release / pull waits outlast the host loop's own no-progress limit
  a.rel_ticks = (long long)((std::min(rel_wait_s_, 7200.0) + 10.0) * 1e8);
  hip_check(hipEventRecord(aev_in_, stream), "async order in");  // after the caller's work so far
  hip_check(hipStreamWaitEvent(astream_, aev_in_, 0), "async order in");
  if (remote) {
    // nothing to initialise: the device ticket counter only ever counts this loop's
    // pushes, so it equals aticket_ (every push is consumed before a run ends).  No copy
    // or fill before a remote launch: on a GPU shared with other ranks' persistent
    // launches the runtime's copy / fill work waits behind them (profiles/r05/README.md)
  } else {
    launch_async_init(cfg_.scfg, a, aticket_, astream_);
    hip_check(hipGetLastError(), "async init launch");
  }
  AsyncPack pk;
  pk.cfg = cfg_.scfg;
  pk.a = a;
  launch_lanes_async(cfg_.scfg, pk, al_dev_, S_, astream_);
  hip_check(hipGetLastError(), "async lanes launch");
  ++launches_;
}

int64_t LanesLoop::run_async(int64_t updates, hipStream_t stream, double max_wait_s, double deadline_ms,
                             int64_t per_lane) {
  std::vector<int64_t> b;
  if (per_lane > 0) b.assign((size_t)cfg_.L, per_lane);
  return run_async(updates, stream, max_wait_s, deadline_ms, b);
}

int64_t LanesLoop::run_async(int64_t updates, hipStream_t stream, double max_wait_s, double deadline_ms,
                             const std::vector<int64_t>& lane_budget) {
  const int64_t t_begin = steady_ns();
  if (!lane_budget.empty() && (int)lane_budget.size() != cfg_.L)
    throw std::invalid_argument("LanesLoop::run_async: one budget per lane");
  auto at_budget = [&](int l, int64_t started) { return !lane_budget.empty() && started >= lane_budget[l]; };
  if (!cfg_.tracker) throw std::invalid_argument("LanesLoop::run_async: needs the tracker");
  ensure_async();
  const int L = cfg_.L;
  void* trk = reinterpret_cast<void*>(cfg_.tracker);
  log_lane_ = (cfg_.log_worker >= 0 && cfg_.log_worker < cfg_.N) ? lane_of_[cfg_.log_worker] : -1;
  // where this run starts: the lanes the tracker has dispatched (bootstrap: all, vc
  // 0, MessageTracker.java:47-53), the others wait for a release
  for (int l = 0; l < L; ++l) {
    // a worker the tracker retired (it crashed or left in an earlier call: its `sent` bit
    // stays set) never starts again -- its lane stays gone and gets a stop record below
    const int live = api().tracker_is_live(trk, cfg_.k[l]);
    check(live, "tracker state");
    const int sent = api().tracker_is_sent(trk, cfg_.k[l]);
    check(sent, "tracker state");
    state_[l] = !live ? kGone : (sent ? kWant : kIdle);
    want_vc_[l] = api().tracker_clock(trk, cfg_.k[l]);
    check(want_vc_[l], "tracker clock");
  }
  // the lanes' release waits (the device) and the row-starved waits below are idle waits:
  // bounded by the idle limit, not by the in-flight watchdog max_wait_s
  rel_wait_s_ = std::max(max_wait_s, idle_wait_s_);
  // fault injection of this run (set_injection), consumed here
  const std::vector<int64_t> crash = std::move(inj_crash_), stop = std::move(inj_stop_);
  inj_crash_.clear();
  inj_stop_.clear();
  crashed_.clear();
  left_.clear();
  launch_async(stream, false);
  int64_t started = 0, done = 0;
  std::vector<int64_t> lane_started((size_t)L, 0);
  int running = 0;
  bool stopping = updates <= 0;
  std::vector<int> ks((size_t)cfg_.N);
  std::vector<int64_t> vs((size_t)cfg_.N);
  // a lane whose worker crashed / left: it gets its stop record now (its workgroups
  // leave the launch), the tracker retires the worker (the others are no longer held
  // back by its clock) and the lanes that releases are dispatched
  auto lane_leave = [&](int l, bool crashed) {
    const int k = cfg_.k[l];
    state_[l] = kGone;
    stop_lane(l);
    (crashed ? crashed_ : left_).push_back(k);
    if (crashed && !inj_drop_) {  // --on_worker_failure fail: the run ends here
      stopping = true;
      return;
    }
    if (l == log_lane_) {  // server rows follow the lowest surviving worker's deltas
      int nl = -1;
      for (int j = 0; j < L; ++j)
        if (state_[j] != kGone && (nl < 0 || cfg_.k[j] < cfg_.k[nl])) nl = j;
      log_lane_ = nl;
      if (nl >= 0) cfg_.log_worker = cfg_.k[nl];
    }
    const int n = api().tracker_retire(trk, k, ks.data(), vs.data(), cfg_.N);
    check(n, "tracker retire");
    for (int i = 0; i < n; ++i) {
      const int j = ks[i] >= 0 && ks[i] < cfg_.N ? lane_of_[ks[i]] : -1;
      if (j < 0) throw std::logic_error("LanesLoop: the tracker released a worker this loop does not host");
      if (state_[j] == kGone) continue;
      state_[j] = kWant;
      want_vc_[j] = vs[i];
    }
  };
  try {
    auto start_ready = [&](double now) {
      for (int l = 0; l < L; ++l) {
        if (state_[l] != kWant || stopping || started >= updates) continue;
        if (!crash.empty() && crash[l] >= 0 && lane_started[l] >= crash[l]) {
          lane_leave(l, true);  // released, and fails before its solve (roles.py WorkerRole.compute)
          l = -1;               // (a retirement may have released a lane already passed)
          continue;
        }
        if (at_budget(l, lane_started[l])) continue;
        if (try_release(l, want_vc_[l], now)) {
          state_[l] = kRunning;
          ++started;
          ++lane_started[l];
          ++running;
        }
      }
    };
    double wait0 = epoch_ms();
    start_ready(epoch_ms() - cfg_.t0_ms);
    uint64_t next = aticket_ + 1;
    int64_t idle_spins = 0;
    for (;;) {
      const volatile AsyncToken* slot = tok_host_ + (next % (uint64_t)ring_);
      __m128i v = _mm_load_si128((const __m128i*)(const void*)slot);
      AsyncToken tk;
      std::memcpy(&tk, &v, 16);
      if (tk.tag == (unsigned)next) {
        const int64_t tk0 = steady_ns();
        std::atomic_thread_fence(std::memory_order_acquire);
        const int l = (int)tk.a;
        const int64_t vc = (int64_t)(((uint64_t)tk.c << 32) | tk.b);
        if (l < 0 || l >= L || state_[l] != kRunning || runrec_[l].vc != vc)
          throw std::logic_error("LanesLoop: unexpected token (lane " + std::to_string(l) + ", vc " +
                                 std::to_string((long long)vc) + ")");
        aticket_ = next++;
        --running;
        ++done;
        // the rows of the iteration: server row first (ServerProcessor.java:154-165), then the worker row
        const RunRec& rr = runrec_[l];
        if (dbg_delta_)
          alog_.push_back({(int64_t)aticket_, l, cfg_.k[l], vc, rr.snap, rr.r.B, rr.r.start, rr.r.first, rr.r.step,
                           rr.r.n, rr.r.first2, rr.r.n2});
        SinkRecord rec[2];
        int nr = 0;
        if (rr.slot_s >= 0) rec[nr++] = SinkRecord{rr.slot_s, 1 | kSinkTagged, rr.seq_s, -1, -1, vc, 0};
        if (rr.slot_w >= 0) rec[nr++] = SinkRecord{rr.slot_w, kSinkTagged, rr.seq_w, -1, cfg_.k[l], vc, rr.nseen};
        if (nr) check(api().sink_submit_many(reinterpret_cast<void*>(cfg_.sink), nr, rec), "metrics sink submit");
        state_[l] = kIdle;
        const int n = api().tracker_on_delta(trk, cfg_.k[l], vc, ks.data(), vs.data(), cfg_.N);
        check(n, "tracker");
        for (int i = 0; i < n; ++i) {
          const int j = ks[i] >= 0 && ks[i] < cfg_.N ? lane_of_[ks[i]] : -1;
          if (j < 0) throw std::logic_error("LanesLoop: the tracker released a worker this loop does not host");
          if (state_[j] == kGone) continue;
          state_[j] = kWant;
          want_vc_[j] = vs[i];
        }
        if (!stop.empty() && stop[l] >= 0 && lane_started[l] >= stop[l]) lane_leave(l, false);
        if (deadline_ms > 0.0 && epoch_ms() >= deadline_ms) stopping = true;
        start_ready(epoch_ms() - cfg_.t0_ms);
        idle_spins = 0;
        wait0 = epoch_ms();
        ++tok_n_;
        tok_ns_ += (double)(steady_ns() - tk0);
        continue;
      }
      if (running > 0) {  // solves in flight: spin for their tokens
        if ((++idle_spins & 1023) == 0) {
          check_errors(-1);
          const double now = epoch_ms();
          if (deadline_ms > 0.0 && now >= deadline_ms) stopping = true;
          if (now - wait0 > max_wait_s * 1000.0)
            throw std::runtime_error("LanesLoop: no delta from the device for " + std::to_string(max_wait_s) + " s");
        } else {
          _mm_pause();
        }
        continue;
      }
      // nothing in flight: is the run over?
      if (stopping || started >= updates) break;
      bool any_want = false, end = false;
      for (int l = 0; l < L; ++l)
        if (state_[l] == kWant && !at_budget(l, lane_started[l])) {
          int64_t size = 0, start = 0, sn = 0;
          check(api().window_state(reinterpret_cast<void*>(cfg_.window[l]), &size, &start, &sn), "window state");
          if (size <= 0 && exhausted(l)) end = true;  // a worker with no rows left: the run ends
          any_want = true;
        }
      if (end || !any_want) break;
      const double now = epoch_ms();
      if (deadline_ms > 0.0 && now >= deadline_ms) break;
      start_ready(now - cfg_.t0_ms);  // every dispatched lane waits for rows (producer clock / cadence)
      if (running == 0) {
        if (now - wait0 > idle_wait_s_ * 1000.0) throw std::runtime_error("LanesLoop: no rows for a worker");
        std::this_thread::sleep_for(std::chrono::microseconds(200));
      } else {
        wait0 = epoch_ms();
      }
    }
    stop_all(stream);
  } catch (...) {
    // never leave the persistent launch running behind an exception
    try {
      stop_all(stream);
    } catch (...) {
    }
    throw;
  }
  check_errors(-1);
  last_par_ = 0;  // the lanes wrote loss / fragments of buffer 0
  async_updates_ += done;
  async_ns_ += (double)(steady_ns() - t_begin);
  return done;
}

void LanesLoop::set_peer(uintptr_t rx_data, uintptr_t rx_tags, int64_t rx_stride, const std::vector<uintptr_t>& inbox,
                         const std::vector<uintptr_t>& inbox_tag) {
  if (aws_) throw std::logic_error("LanesLoop::set_peer: before the first asynchronous run");
  const int L = cfg_.L;
  if (!rx_data || !rx_tags || rx_stride < P_ || (int)inbox.size() != L || (int)inbox_tag.size() != L)
    throw std::invalid_argument("LanesLoop::set_peer: receive region / one inbox slot per lane");
  for (int l = 0; l < L; ++l)
    if (!inbox[l] || !inbox_tag[l]) throw std::invalid_argument("LanesLoop::set_peer: null inbox slot");
  peer_rx_ = reinterpret_cast<float*>(rx_data);
  peer_rx_tag_ = reinterpret_cast<unsigned*>(rx_tags);
  peer_stride_ = rx_stride;
  peer_inbox_ = inbox;
  peer_inbox_tag_ = inbox_tag;
  pull_tag_.assign(L, 0u);
}

int64_t LanesLoop::run_async_remote(P2P* p2p, uintptr_t ctrl, uintptr_t reply, int64_t iters, hipStream_t stream,
                                    hipStream_t cs, double max_wait_s, double deadline_ms) {
  const int64_t t_begin = steady_ns();
  const bool peer = p2p == nullptr;
  if ((!p2p && !peer_rx_) || !ctrl || !reply)
    throw std::invalid_argument("LanesLoop::run_async_remote: transport (or set_peer) / queues");
  if (p2p && peer_rx_) throw std::invalid_argument("LanesLoop::run_async_remote: a transport AND the peer data plane");
  if (iters < 1) throw std::invalid_argument("LanesLoop::run_async_remote: iters >= 1");
  ensure_async();
  const int L = cfg_.L;
  if (R_ < L) throw std::invalid_argument("LanesLoop::run_async_remote: more lanes than receive slots");
  if (!peer && pull_ev_.empty()) {
    pull_ev_.assign(L, nullptr);
    for (auto& e : pull_ev_) hip_check(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
  }
  enum { kWaitPull = 3, kPulling = 4, kDone = 5 };
  for (int l = 0; l < L; ++l) state_[l] = kWaitPull;  // the server's begin() sends everybody its clock
  std::vector<int64_t> it(L, 0);
  rel_wait_s_ = std::max(max_wait_s, idle_wait_s_);
  launch_async(stream, true);
  int64_t done = 0;
  int running = 0, finished = 0;
  void* rq = reinterpret_cast<void*>(reply);
  void* cq = reinterpret_cast<void*>(ctrl);
  auto window_empty = [&](int l) {
    int64_t size = 0, start = 0, sn = 0;
    check(api().window_state(reinterpret_cast<void*>(cfg_.window[l]), &size, &start, &sn), "window state");
    return size <= 0;
  };
  try {
    double wait0 = epoch_ms();
    uint64_t next = aticket_ + 1;
    int64_t spins = 0;
    while (finished < L || running > 0) {
      bool progress = false;
      // the server's releases, in its send order to this rank
      CtrlToken rt{};
      while (api().ctrl_pop(rq, &rt, 0.0) == 1) {
        const int j = rt.worker >= 0 && rt.worker < cfg_.N ? lane_of_[rt.worker] : -1;
        if (j < 0 || state_[j] != kWaitPull)
          throw std::logic_error("LanesLoop: reply for worker " + std::to_string(rt.worker) + " not waiting");
        want_vc_[j] = rt.vc;
        progress = true;
        if (peer) {  // the server GPU writes the weights into slot j itself: the lane waits for tag aux
          pull_tag_[j] = (unsigned)rt.aux;
          state_[j] = kWant;
          continue;
        }
        p2p->recv(aargs_.snap + (size_t)j * P_, (size_t)P_, Comm::kF32, 0, cs);
        hip_check(hipEventRecord(pull_ev_[j], cs), "pull event");
        state_[j] = kPulling;
      }
      const double now = epoch_ms();
      for (int l = 0; l < L; ++l) {
        if (state_[l] == kPulling) {
          const hipError_t q = hipEventQuery(pull_ev_[l]);
          if (q == hipSuccess)
            state_[l] = kWant;
          else if (q != hipErrorNotReady)
            hip_check(q, "pull event query");
        }
        if (state_[l] == kWant && try_release(l, want_vc_[l], now - cfg_.t0_ms, l)) {
          state_[l] = kRunning;
          ++running;
          progress = true;
        }
      }
      // the lanes' pushes, in their push (ticket) order
      const volatile AsyncToken* slot = tok_host_ + (next % (uint64_t)ring_);
      __m128i v = _mm_load_si128((const __m128i*)(const void*)slot);
      AsyncToken tk;
      std::memcpy(&tk, &v, 16);
      if (tk.tag == (unsigned)next) {
        std::atomic_thread_fence(std::memory_order_acquire);
        const int l = (int)tk.a;
        const int64_t vc = (int64_t)(((uint64_t)tk.c << 32) | tk.b);
        if (l < 0 || l >= L || state_[l] != kRunning || runrec_[l].vc != vc)
          throw std::logic_error("LanesLoop: unexpected token (lane " + std::to_string(l) + ")");
        aticket_ = next++;
        --running;
        ++done;
        const bool fin = ++it[l] >= iters || (deadline_ms > 0.0 && now >= deadline_ms) ||
                         (exhausted(l) && window_empty(l));
        // push: the delta to the server, then its token (WorkerTrainingProcessor.java:95-97);
        // peer data plane: the lane already wrote it into the server's inbox (tagged)
        if (!peer) p2p->send(lanes_[l].dv.delta, (size_t)P_, Comm::kF32, 0, cs);
        CtrlToken ct{};
        ct.worker = cfg_.k[l];
        ct.kind = fin ? 1 : 0;
        ct.vc = vc;
        ct.aux = runrec_[l].nseen;
        if (api().ctrl_push(cq, &ct, max_wait_s) != 1) throw std::runtime_error("LanesLoop: control queue full");
        const RunRec& rr = runrec_[l];
        if (rr.slot_w >= 0) {
          SinkRecord rec{rr.slot_w, kSinkTagged, rr.seq_w, -1, cfg_.k[l], vc, rr.nseen};
          check(api().sink_submit_many(reinterpret_cast<void*>(cfg_.sink), 1, &rec), "metrics sink submit");
        }
        state_[l] = fin ? (int)kDone : (int)kWaitPull;
        finished += fin ? 1 : 0;
        progress = true;
      }
      if (progress) {
        wait0 = epoch_ms();
        spins = 0;
        continue;
      }
      if ((++spins & 1023) == 0) {
        check_errors(-1);
        if (epoch_ms() - wait0 > max_wait_s * 1000.0) {
          std::string m = "LanesLoop: no progress with the server for " + std::to_string(max_wait_s) +
                          " s; lanes (state 1 want / 2 running / 3 wait pull / 4 pulling / 5 done, vc, pull tag):";
          for (int l = 0; l < L; ++l)
            m += " [" + std::to_string(state_[l]) + " " + std::to_string((long long)want_vc_[l]) + " " +
                 std::to_string(peer ? pull_tag_[l] : 0u) + " it " + std::to_string((long long)it[l]) + "]";
          m += "; tokens pushed " + std::to_string((long long)done) + "; " + launch_report();
          throw std::runtime_error(m);
        }
        if (running == 0) std::this_thread::sleep_for(std::chrono::microseconds(100));
      } else {
        _mm_pause();
      }
    }
    stop_all(stream);
  } catch (...) {
    try {
      stop_all(stream);
    } catch (...) {
    }
    throw;
  }
  check_errors(-1);
  last_par_ = 0;
  async_updates_ += done;
  async_ns_ += (double)(steady_ns() - t_begin);
  return done;
}

}  // namespace psx
