#include "wide_solver.h"

#include <algorithm>
#include <cstdlib>
#include <stdexcept>
#include <string>
#include <vector>

#include "../kernels/common.h"  // kAccStride
#include "solver.h"            // hip_check

namespace psx {

static size_t align256(size_t v) { return (v + 255) / 256 * 256; }

WideSolver::WideSolver(const WideCfg& cfg, const WideBuffers& buf, bool use_graph) : cfg_(cfg), use_graph_(use_graph) {
  const int KP = cfg.KP;
  if (!(KP == 1 || KP == 2 || KP == 4 || KP == 8 || KP == 16)) throw std::invalid_argument("KP must be 1/2/4/8/16");
  if (cfg.K < 1 || cfg.K > KP) throw std::invalid_argument("K must be in [1, KP]");
  if (cfg.F < 1 || cfg.F > (int64_t)0x7fffffff) throw std::invalid_argument("F out of range");
  if (cfg.cap < 1 || cfg.NZ < 1 || cfg.NZ > 512) throw std::invalid_argument("ring must have cap >= 1 and 1 <= NZ <= 512");
  if (cfg.sc.hist < 1 || cfg.sc.hist > kMaxHist) throw std::invalid_argument("history must be in [1,16]");
  if (cfg.sc.nslots < 1) throw std::invalid_argument("nslots must be >= 1");
  if (cfg.dense_delta && !buf.delta_dense) throw std::invalid_argument("dense_delta needs a dense output buffer");
  if (!buf.uniq || !buf.dloc || !buf.wloc || !buf.loss || !buf.stats) throw std::invalid_argument("missing output buffer");
  if (cfg.pulled && (!buf.w_pull || !buf.w_pull_b)) throw std::invalid_argument("pull mode needs w_pull / w_pull_b");
  if (!cfg.pulled && !buf.w_old) throw std::invalid_argument("missing w_old");
  if (cfg.pulled && (cfg.own_W < 1 || cfg.own_W > kMaxOwners || (cfg.own_W > 1 && cfg.own_S < 1)))
    throw std::invalid_argument("owner split: 1 <= own_W <= 64 and own_S >= 1");
  if (cfg.pulled && cfg.dense_delta) throw std::invalid_argument("pull mode has no dense delta");
  const int64_t E = (int64_t)cfg.cap * cfg.NZ;
  const int64_t umax = cfg.F < E ? cfg.F : E;
  if (umax > 0x7fffffff / 2) throw std::invalid_argument("window too large");
  cfg_.umax = (int)umax;
  const int64_t PLmax = KP + umax * KP;
  const size_t H = cfg.sc.hist;
  nblk_dots_ = wide_dots_blocks(PLmax);

  size_t off = 0;
  auto take = [&](size_t bytes) {
    size_t o = off;
    off = align256(off + bytes);
    return o;
  };
  const size_t o_prm = take(sizeof(WideParams)), o_ctrl = take(sizeof(Ctrl)), o_cnt = take(16), o_gbar = take(8),
               o_pbar = take(8);
  unsigned HT = 1;
  while (HT < 2 * (unsigned)umax) HT <<= 1;
  const size_t o_tab = take((size_t)HT * 8), o_hslot = take(umax * 4), o_alt = take(umax * 4),
               o_own = take(2 * kMaxOwners * 4), o_lid = take((size_t)E * 4);
  const int RB = wide_rows_per_group(cfg.NZ, KP), EB = RB * cfg.NZ;
  int TS = 1;
  while (TS < 2 * EB) TS <<= 1;
  const int G = (cfg.cap + RB - 1) / RB;
  const size_t o_pslot = take((size_t)E * 2), o_bfeat = take((size_t)G * EB * 4), o_blid = take((size_t)G * EB * 4),
               o_bcount = take((size_t)G * 4);
  const size_t o_s1 = take(umax * 4), o_s2 = take(umax * 4), o_sc = take(umax * 4), o_gs = take(umax * 4);
  const size_t o_x = take(PLmax * 4), o_d = take(PLmax * 4), o_gt = take(PLmax * 4), o_gc = take(PLmax * 4),
               o_w0 = take(PLmax * 4);
  const size_t o_S = take(H * PLmax * 4), o_Y = take(H * PLmax * 4);
  // dot partials: one row per workgroup of the dots launches (nblk_dots_), of the
  // persistent tail (up to 64 workgroups) AND of the one-launch persistent solve
  // (wide_persist_grid() workgroups run its dots phase)
  int npart = nblk_dots_ > 64 ? nblk_dots_ : 64;
  if (npart < wide_persist_grid()) npart = wide_persist_grid();
  const size_t o_part = take((size_t)npart * kWideND * 8), o_loss = take((size_t)cfg.sc.nslots * 8);
  const bool stamps = std::getenv("PSX_WIDE_STAMPS") != nullptr;
  const size_t o_dbg = stamps ? take((size_t)cfg.sc.nslots * 8 * 8) : 0;
  ws_bytes_ = off;
  hip_check(hipMalloc(&ws_, ws_bytes_), "hipMalloc(wide solver workspace)");
  hip_check(hipMemset(ws_, 0, ws_bytes_), "hipMemset(wide solver workspace)");
  char* b = static_cast<char*>(ws_);
  hip_check(hipMemset(b + o_tab, 0xff, (size_t)HT * 8), "hipMemset(table)");  // all keys -1
  hip_check(hipHostMalloc((void**)&host_u_, 64, hipHostMallocCoherent | hipHostMallocMapped), "hipHostMalloc");
  *host_u_ = 0;

  dv_.ridx = buf.ridx;
  dv_.rval = buf.rval;
  dv_.rnnz = buf.rnnz;
  dv_.ry = buf.ry;
  dv_.w_old = buf.w_old;
  dv_.w_pull = buf.w_pull;
  dv_.w_pull_b = buf.w_pull_b;
  dv_.prm = reinterpret_cast<WideParams*>(b + o_prm);
  dv_.ctrl = reinterpret_cast<Ctrl*>(b + o_ctrl);
  dv_.cnt = reinterpret_cast<unsigned*>(b + o_cnt);
  dv_.gbar = reinterpret_cast<unsigned long long*>(b + o_gbar);
  dv_.pbar = reinterpret_cast<unsigned*>(b + o_pbar);
  dv_.htab = reinterpret_cast<int2*>(b + o_tab);
  dv_.hmask = HT - 1;
  dv_.hslot = reinterpret_cast<int32_t*>(b + o_hslot);
  dv_.uniq_alt = reinterpret_cast<int32_t*>(b + o_alt);
  dv_.own = reinterpret_cast<unsigned*>(b + o_own);
  dv_.uniq = buf.uniq;
  dv_.lid = reinterpret_cast<int32_t*>(b + o_lid);
  dv_.pslot = reinterpret_cast<uint16_t*>(b + o_pslot);
  dv_.bfeat = reinterpret_cast<int32_t*>(b + o_bfeat);
  dv_.blid = reinterpret_cast<int32_t*>(b + o_blid);
  dv_.bcount = reinterpret_cast<int32_t*>(b + o_bcount);
  dv_.RB = RB;
  dv_.EB = EB;
  dv_.TS = TS;
  dv_.s1 = reinterpret_cast<float*>(b + o_s1);
  dv_.s2 = reinterpret_cast<float*>(b + o_s2);
  dv_.scale = reinterpret_cast<float*>(b + o_sc);
  dv_.gscale = reinterpret_cast<float*>(b + o_gs);
  dv_.x = reinterpret_cast<float*>(b + o_x);
  dv_.d = reinterpret_cast<float*>(b + o_d);
  dv_.g_t = reinterpret_cast<float*>(b + o_gt);
  dv_.g_c = reinterpret_cast<float*>(b + o_gc);
  dv_.w0 = reinterpret_cast<float*>(b + o_w0);
  dv_.S = reinterpret_cast<float*>(b + o_S);
  dv_.Y = reinterpret_cast<float*>(b + o_Y);
  dv_.part = reinterpret_cast<double*>(b + o_part);
  dv_.loss_acc = reinterpret_cast<double*>(b + o_loss);
  dv_.dloc = buf.dloc;
  dv_.wloc = buf.wloc;
  dv_.loss = buf.loss;
  dv_.stats = buf.stats;
  dv_.delta_dense = buf.delta_dense;
  dv_.host_u = host_u_;
  dv_.dbg = stamps ? reinterpret_cast<long long*>(b + o_dbg) : nullptr;
  dv_.PLmax = PLmax;

  wide_prepare_kernels();  // before any capture
  hip_check(hipStreamCreateWithFlags(&cap_stream_, hipStreamNonBlocking), "hipStreamCreate");
  if (cfg_.persist) use_graph_ = false;  // one launch per phase: nothing to replay
  if (use_graph_) {
    hip_check(hipStreamBeginCapture(cap_stream_, hipStreamCaptureModeThreadLocal), "hipStreamBeginCapture");
    enqueue_plan(cap_stream_, 1, 0);
    if (!cfg_.pulled) enqueue_rest(cap_stream_);
    hip_check(hipStreamEndCapture(cap_stream_, &graph_), "hipStreamEndCapture");
    hip_check(hipGraphInstantiate(&exec_, graph_, nullptr, nullptr, 0), "hipGraphInstantiate");
    if (cfg_.pulled) {
      hip_check(hipStreamBeginCapture(cap_stream_, hipStreamCaptureModeThreadLocal), "hipStreamBeginCapture");
      enqueue_rest(cap_stream_);
      hip_check(hipStreamEndCapture(cap_stream_, &graph2_), "hipStreamEndCapture");
      hip_check(hipGraphInstantiate(&exec2_, graph2_, nullptr, nullptr, 0), "hipGraphInstantiate");
    }
    size_t n = 0;
    hip_check(hipGraphGetNodes(graph_, nullptr, &n), "hipGraphGetNodes");
    std::vector<hipGraphNode_t> nodes(n);
    hip_check(hipGraphGetNodes(graph_, nodes.data(), &n), "hipGraphGetNodes");
    for (auto nd : nodes) {
      hipGraphNodeType t;
      hip_check(hipGraphNodeGetType(nd, &t), "hipGraphNodeGetType");
      if (t != hipGraphNodeTypeKernel) continue;
      hipKernelNodeParams kp{};
      hip_check(hipGraphKernelNodeGetParams(nd, &kp), "hipGraphKernelNodeGetParams");
      if (kp.func == wide_begin_symbol()) {
        begin_node_ = nd;
        begin_params_ = kp;
      }
    }
    if (!begin_node_) throw std::runtime_error("wide solver graph: begin node not found");
    begin_args_ = BeginArgs{dv_, 1, 0};
    begin_kp_[0] = &begin_args_.d;
    begin_kp_[1] = &begin_args_.B;
    begin_kp_[2] = &begin_args_.start;
    begin_params_.kernelParams = begin_kp_;
    begin_params_.extra = nullptr;
  }
}

WideSolver::~WideSolver() {
  if (exec_) (void)hipGraphExecDestroy(exec_);
  if (graph_) (void)hipGraphDestroy(graph_);
  if (exec2_) (void)hipGraphExecDestroy(exec2_);
  if (graph2_) (void)hipGraphDestroy(graph2_);
  if (cap_stream_) (void)hipStreamDestroy(cap_stream_);
  if (ws_) (void)hipFree(ws_);
  if (host_u_) (void)hipHostFree(host_u_);
}

void WideSolver::enqueue_plan(hipStream_t s, int B, int start) {
  wide_launch_begin(cfg_, dv_, B, start, s);
  wide_launch_plan(cfg_, dv_, s);
  hip_check(hipGetLastError(), "wide solver launch");
}

void WideSolver::enqueue_rest(hipStream_t s) {
  wide_launch_prepare(cfg_, dv_, s);
  // slots launched one by one: the initial evaluation + one trial per iteration
  // (a solve whose line searches accept their first trial); the retry budget
  // runs in the persistent tail launch
  const int nfast = cfg_.sc.mode == 1 ? cfg_.sc.nslots
                                      : (1 + cfg_.sc.iters < cfg_.sc.nslots ? 1 + cfg_.sc.iters : cfg_.sc.nslots);
  for (int slot = 0; slot < nfast; ++slot) wide_launch_slot(cfg_, dv_, slot, nblk_dots_, s);
  if (cfg_.sc.nslots > nfast) wide_launch_tail(cfg_, dv_, nfast, cfg_.sc.nslots, s);
  if (cfg_.dense_delta)
    hip_check(hipMemsetAsync(dv_.delta_dense, 0, (size_t)(cfg_.F * cfg_.KP + cfg_.KP) * 4, s), "memset delta");
  wide_launch_finalize(cfg_, dv_, s);
  hip_check(hipGetLastError(), "wide solver launch");
}

void WideSolver::check_window(int B, int start) const {
  if (B <= 0) throw std::invalid_argument("local solve on an empty buffer");
  if (B > cfg_.cap || start < 0 || start >= cfg_.cap) throw std::invalid_argument("window out of ring bounds");
}

void WideSolver::run(int B, int start, hipStream_t stream) {
  if (cfg_.pulled) throw std::logic_error("pull mode: plan() + finish()");
  check_window(B, start);
  if (cfg_.persist) {
    if (cfg_.dense_delta)
      hip_check(hipMemsetAsync(dv_.delta_dense, 0, (size_t)(cfg_.F * cfg_.KP + cfg_.KP) * 4, stream), "memset delta");
    wide_launch_persist(cfg_, dv_, B, start, 3, stream);
    hip_check(hipGetLastError(), "wide persistent solve launch");
  } else if (use_graph_) {
    begin_args_.B = B;
    begin_args_.start = start;
    hip_check(hipGraphExecKernelNodeSetParams(exec_, begin_node_, &begin_params_), "hipGraphExecKernelNodeSetParams");
    hip_check(hipGraphLaunch(exec_, stream), "hipGraphLaunch");
  } else {
    enqueue_plan(stream, B, start);
    enqueue_rest(stream);
  }
}

void WideSolver::plan(int B, int start, hipStream_t stream) {
  if (!cfg_.pulled) throw std::logic_error("plan() is the pull mode's first phase");
  check_window(B, start);
  if (use_graph_) {
    begin_args_.B = B;
    begin_args_.start = start;
    hip_check(hipGraphExecKernelNodeSetParams(exec_, begin_node_, &begin_params_), "hipGraphExecKernelNodeSetParams");
    hip_check(hipGraphLaunch(exec_, stream), "hipGraphLaunch");
  } else {
    enqueue_plan(stream, B, start);
  }
}

void WideSolver::finish(hipStream_t stream) {
  if (!cfg_.pulled) throw std::logic_error("finish() is the pull mode's second phase");
  if (cfg_.persist) {
    wide_launch_persist(cfg_, dv_, 0, 0, 2, stream);
    hip_check(hipGetLastError(), "wide persistent solve launch");
  } else if (use_graph_)
    hip_check(hipGraphLaunch(exec2_, stream), "hipGraphLaunch");
  else
    enqueue_rest(stream);
}

std::vector<long long> WideSolver::read_stamps(hipStream_t stream) {
  std::vector<long long> v;
  if (!dv_.dbg) return v;
  v.resize((size_t)cfg_.sc.nslots * 8);
  hip_check(hipMemcpyAsync(v.data(), dv_.dbg, v.size() * sizeof(long long), hipMemcpyDeviceToHost, stream),
            "read stamps");
  hip_check(hipStreamSynchronize(stream), "sync");
  return v;
}

void WideSolver::read_ctrl(Ctrl* out, hipStream_t stream) {
  hip_check(hipMemcpyAsync(out, dv_.ctrl, sizeof(Ctrl), hipMemcpyDeviceToHost, stream), "read ctrl");
  hip_check(hipStreamSynchronize(stream), "sync");
}

// ---------------------------------------------------------------------------
WideLanes::WideLanes(const std::vector<WideSolver*>& solvers, int xcd0) : solvers_(solvers), xcd0_(xcd0) {
  const int L = (int)solvers_.size();
  if (L < 1 || L > kWideMaxLanes) throw std::invalid_argument("WideLanes: 1..8 solvers");
  if (!solvers_[0]) throw std::invalid_argument("WideLanes: null solver");
  if (xcd0 < 0 || xcd0 + L > 8) throw std::invalid_argument("WideLanes: lanes xcd0 .. xcd0 + L - 1 must be XCDs 0..7");
  cfg_ = solvers_[0]->cfg();
  std::vector<WideDev> devs(L);
  for (int l = 0; l < L; ++l) {
    const WideSolver* s = solvers_[l];
    if (!s) throw std::invalid_argument("WideLanes: null solver");
    const WideCfg& c = s->cfg();
    if (c.pulled) throw std::invalid_argument("WideLanes: pull-mode solvers have two phases");
    if (c.dense_delta) throw std::invalid_argument("WideLanes: sparse deltas only");
    if (c.K != cfg_.K || c.KP != cfg_.KP || c.F != cfg_.F || c.cap != cfg_.cap || c.NZ != cfg_.NZ ||
        c.sc.nslots != cfg_.sc.nslots || c.sc.iters != cfg_.sc.iters || c.sc.hist != cfg_.sc.hist)
      throw std::invalid_argument("WideLanes: every solver needs one configuration");
    if (s->dev().w_old != solvers_[0]->dev().w_old)
      throw std::invalid_argument("WideLanes: every lane pulls the same weights");
    devs[l] = s->dev();
    const size_t b = wide_persist_lds(c, devs[l]);
    if (b > lds_) lds_ = b;
  }
  if (lds_ > 96 * 1024) throw std::invalid_argument("WideLanes: ring rows too wide for the persistent solve's LDS");
  hip_check(hipMalloc(&devs_, sizeof(WideDev) * L), "hipMalloc(wide lanes table)");
  hip_check(hipMemcpy(devs_, devs.data(), sizeof(WideDev) * L, hipMemcpyHostToDevice), "wide lanes table");
  hip_check(hipMalloc(&claim_, 2 * 16 * sizeof(unsigned)), "hipMalloc(claim)");
  hip_check(hipMemset(claim_, 0, 2 * 16 * sizeof(unsigned)), "hipMemset(claim)");
  const size_t acc_bytes = (size_t)kWideEvalCopies * kWideMaxEval * 256 * kAccStride * sizeof(int);
  hip_check(hipMalloc(&acc_, acc_bytes), "hipMalloc(eval accumulators)");
  hip_check(hipMemset(acc_, 0, acc_bytes), "hipMemset(eval accumulators)");
  hip_check(hipMalloc(&ticket_, 64), "hipMalloc(ticket)");
  hip_check(hipMemset(ticket_, 0, 64), "hipMemset(ticket)");
  // two lane workgroups per CU when both fit (LDS, registers): twice the workgroups per
  // lane on the same XCD -- the solve's row groups and vector phases are latency-bound
  gpx_ = 32 * wide_lanes_per_cu(cfg_, lds_);
  if (const char* e = std::getenv("PSX_WIDE_LANE_PER_CU")) {
    const int v = std::atoi(e);
    if (v == 1 || v == 2) gpx_ = 32 * std::min(v, gpx_ / 32);
  }
  // the evaluation pass's overlay table: F presence words + F x 8 lanes' coefficient rows
  // (256 MB at 2^20 features and KP 8; up to 2 GB of the 288 GB HBM), else bitmaps + probes
  const size_t ov_bytes = (size_t)cfg_.F * kWideMaxLanes * cfg_.KP * 4;
  const char* eo = std::getenv("PSX_WIDE_EVAL_OVERLAY");
  if (ov_bytes <= ((size_t)2 << 30) && !(eo && std::atoi(eo) == 0)) {
    hip_check(hipMalloc(&ov_, ov_bytes), "hipMalloc(eval overlay rows)");
    hip_check(hipMalloc(&pres_, (size_t)cfg_.F * 4), "hipMalloc(eval overlay presence)");
    hip_check(hipMalloc(&lidt_, (size_t)cfg_.F * kWideMaxLanes * 4), "hipMalloc(eval overlay local ids)");
    hip_check(hipMemset(pres_, 0, (size_t)cfg_.F * 4), "hipMemset(eval overlay presence)");
  }
  // the evaluation pass's bitmaps of the lanes' window features (up to 64 MB)
  nw_ = (cfg_.F + 31) / 32;
  const size_t bm_bytes = (size_t)L * (size_t)nw_ * 4;
  const char* eb = std::getenv("PSX_WIDE_EVAL_BITMAP");
  if (!pres_ && bm_bytes <= ((size_t)64 << 20) && !(eb && std::atoi(eb) == 0))
    hip_check(hipMalloc(&bm_, bm_bytes), "hipMalloc(eval bitmaps)");
}

WideLanes::~WideLanes() {
  if (devs_) (void)hipFree(devs_);
  if (claim_) (void)hipFree(claim_);
  if (acc_) (void)hipFree(acc_);
  if (ticket_) (void)hipFree(ticket_);
  if (bm_) (void)hipFree(bm_);
  if (pres_) (void)hipFree(pres_);
  if (ov_) (void)hipFree(ov_);
  if (lidt_) (void)hipFree(lidt_);
}

void WideLanes::run(const std::vector<int>& B, const std::vector<int>& start, hipStream_t stream) {
  const int L = lanes();
  if ((int)B.size() != L || (int)start.size() != L) throw std::invalid_argument("WideLanes::run: one window per lane");
  WideLanesArgs a{};
  a.L = L;
  a.xcd0 = xcd0_;
  a.per = (8 - xcd0_) / L;  // every XCD from xcd0 on (an XCD's lane workgroups co-resident)
  if (a.per < 1) a.per = 1;
  if (const char* e = std::getenv("PSX_WIDE_LANE_XCDS")) {  // (measurements: XCDs per lane)
    const int v = std::atoi(e);
    if (v >= 1 && v * L <= 8 - xcd0_) a.per = v;
  }
  a.gpx = gpx_;
  a.claim = claim_;
  a.cpar = (int)(launches_ & 1);
  for (int l = 0; l < L; ++l) {
    if (B[l] <= 0) throw std::invalid_argument("local solve on an empty buffer");
    if (B[l] > cfg_.cap || start[l] < 0 || start[l] >= cfg_.cap) throw std::invalid_argument("window out of ring bounds");
    a.B[l] = B[l];
    a.start[l] = start[l];
  }
  if (pres_) {  // the lanes build this launch's overlay table (a table nobody applied: cleared first)
    if (ov_live_) wide_lanes_overlay(devs_, L, cfg_.KP, pres_, nullptr, nullptr, false, stream);
    a.pres = pres_;
    a.ov = ov_;
    a.lidt = lidt_;
  }
  wide_launch_lanes(cfg_, devs_, a, lds_, stream);
  hip_check(hipGetLastError(), "wide lanes launch");
  ++launches_;
  ov_live_ = pres_ != nullptr;  // this launch's table (eval reads it, apply clears it)
}

void WideLanes::apply(float* w, float lr, const std::vector<int>& order, hipStream_t stream) {
  if (ov_live_ && (int)order.size() == lanes()) {  // one launch over the overlay table of these solves
    WideLanesOrder o{};
    o.n = lanes();
    std::vector<int> seen(lanes(), 0);
    for (int q = 0; q < o.n; ++q) {
      const int l = order[q];
      if (l < 0 || l >= lanes() || seen[l]++) throw std::invalid_argument("WideLanes::apply: order must permute the lanes");
      o.ord[q] = l;
    }
    wide_lanes_apply(devs_, lanes(), o, cfg_.F, cfg_.KP, w, lr, pres_, lidt_, stream);
    hip_check(hipGetLastError(), "wide lanes apply launch");
    ov_live_ = false;
    return;
  }
  if (ov_live_) {  // a partial order: the per-push launches; the table is cleared
    wide_lanes_overlay(devs_, lanes(), cfg_.KP, pres_, nullptr, nullptr, false, stream);
    ov_live_ = false;
  }
  for (int l : order) {
    if (l < 0 || l >= lanes()) throw std::invalid_argument("WideLanes::apply: lane out of range");
    const WideSolver* s = solvers_[l];
    launch_wide_apply_sparse(w, cfg_.F, cfg_.KP, s->ucount_dev(), 0, s->uniq(), s->dev().dloc, lr, cfg_.umax, stream);
  }
  hip_check(hipGetLastError(), "wide lanes apply launch");
}

void WideLanes::eval(const int64_t* indptr, const int32_t* idx, const uint16_t* val, const int32_t* y, int T,
                     const float* w, int nov, const std::vector<uintptr_t>& slots,
                     const std::vector<unsigned long long>& seqs, uintptr_t server_slot,
                     unsigned long long server_seq, hipStream_t stream) {
  if (nov < 0 || nov > lanes() || (int)slots.size() != nov || (int)seqs.size() != nov)
    throw std::invalid_argument("WideLanes::eval: one slot per evaluated lane");
  WideEvalModels m{};
  m.nov = nov;
  m.plain = server_slot ? 1 : 0;
  for (int j = 0; j < nov; ++j) {
    const WideDev& d = solvers_[j]->dev();
    m.htab[j] = d.htab;
    m.hmask[j] = d.hmask;
    m.wloc[j] = d.wloc;
    m.loss[j] = d.loss;
    m.slot[j] = reinterpret_cast<char*>(slots[j]);
    m.seq[j] = seqs[j];
  }
  if (pres_ && nov > 0 && ov_live_) {  // the last launch built the table of its lanes' windows
    m.pres = pres_;
    m.ov = ov_;
  } else if (bm_ && nov > 0) {  // this pass's overlays: their window features' bitmaps
    hip_check(hipMemsetAsync(bm_, 0, (size_t)nov * (size_t)nw_ * 4, stream), "clear eval bitmaps");
    wide_lanes_bitmap(devs_, nov, bm_, nw_, stream);
    m.bm = bm_;
    m.nw = nw_;
  }
  if (server_slot) {
    m.loss[nov] = nullptr;
    m.slot[nov] = reinterpret_cast<char*>(server_slot);
    m.seq[nov] = server_seq;
  }
  launch_wide_eval_multi(cfg_.K, cfg_.KP, cfg_.F, indptr, idx, val, y, T, w, m, acc_, ticket_, stream);
  hip_check(hipGetLastError(), "wide lanes evaluation launch");

}

}  // namespace psx
