#include "solver.h"
#include <cstdlib>
#include <stdexcept>
#include <string>

namespace psx {

void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

static size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

LocalSolver::LocalSolver(const SolverCfg& cfg, const SolverBuffers& buf, int max_eval_wg, bool use_graph)
    : cfg_(cfg), use_graph_(use_graph) {
  if (!fp_supported(cfg.Fp)) throw std::invalid_argument("unsupported padded feature width " + std::to_string(cfg.Fp));
  if (cfg.K < 2 || cfg.K > 16) throw std::invalid_argument("num classes (incl. phantom) must be in [2,16]");
  if (cfg.P != cfg.K * cfg.Fp + cfg.K) throw std::invalid_argument("P mismatch");
  if (cfg.hist < 1 || cfg.hist > kMaxHist) throw std::invalid_argument("history must be in [1,16]");
  if (cfg.nslots < 1 || cfg.nslots >= kMaxSlots)
    throw std::invalid_argument("nslots must be in [1, " + std::to_string(kMaxSlots - 1) + "]");
  if (cfg.cap < 32 || cfg.cap % 32 != 0) throw std::invalid_argument("ring capacity must be a positive multiple of 32");
  rows_mode_ = cfg.xf32 || rows_mode_for(cfg.cap);  // fp32 rows: only the row-parallel solver reads them
  if (cfg.xf32 && (!buf.Xf || cfg.Fp > 1024))
    throw std::invalid_argument("fp32 rows: need the fp32 ring, at most 1024 padded features");
  if (!rows_mode_ && !buf.XT) throw std::invalid_argument("the solver needs the feature-major ring copy XT");
  const int tiles = cfg.cap / kTileRows + 1;  // window tiles (ring-aligned; a wrapped window may touch one twice)
  nwg_eval_ = tiles < max_eval_wg ? tiles : max_eval_wg;
  if (nwg_eval_ < 1) nwg_eval_ = 1;
  if (rows_mode_) {
    use_graph_ = false;  // eager: the rows chain has no per-run node to patch
    // two workgroups per CU keep >= 128 KB of each CU's window tiles in flight
    nwg_eval_ = tiles < 512 ? tiles : 512;
  }
  {  // persistent small-window solve (PSX_SOLVER_PERSIST=0 disables it)
    const char* e = std::getenv("PSX_SOLVER_PERSIST");
    const bool env_ok = !(e && *e && e[0] == '0');
    persist_ = cfg.persist && env_ok && !rows_mode_ && !use_graph_ && persist_supported(cfg.Fp, padded_classes(cfg.K)) &&
               cfg.cap <= 2048;
  }
  // slots launched one by one: the initial evaluation + one trial per iteration
  // (what a solve whose line searches accept their first trial uses); the
  // remaining budget runs in the persistent tail launch
  nfast_ = (cfg.mode == 1 || !cfg.tail) ? cfg.nslots : (1 + cfg.iters < cfg.nslots ? 1 + cfg.iters : cfg.nslots);

  // solver-private vectors use the padded layout of solve_kernels.hip
  dv_.KP = padded_classes(cfg.K);
  dv_.FPI = padded_stride(cfg.Fp);
  dv_.PI = dv_.KP * dv_.FPI + 16;
  const size_t PI = dv_.PI, FPI = dv_.FPI, FP = cfg.Fp, H = cfg.hist;
  size_t off = 0;
  auto take = [&](size_t bytes) {
    size_t o = off;
    off = align_up(off + bytes, 256);
    return o;
  };
  const size_t o_prm = take(sizeof(SolveParams));
  const size_t o_ctrl = take(sizeof(Ctrl));
  const size_t o_x = take(PI * 4), o_d = take(PI * 4), o_gc = take(PI * 4);
  const size_t o_S = take(H * PI * 4), o_Y = take(H * PI * 4);
  const size_t o_std = take(FPI * 4), o_istd = take(FPI * 4), o_wfix = take(PI * 4), o_beff = take(16 * 4);
  const size_t o_whi = take(16 * FP * 2), o_wlo = take(16 * FP * 2);
  const size_t o_R = take(rows_mode_ ? 256 : (size_t)tiles * 1024 * 2);  // rows mode keeps no residual tiles
  // PSX_SOLVER_GPF=1: the small-window chain's backward from the forward
  // workgroups' feature-major partials (gpf) instead of the feature-major ring
  // copy XT.  Measured equal on MI355X (profiles/r02_v3: the forward launch's
  // 1 MB of partials costs at the boundary what the backward saves on loads),
  // so the XT backward stays the default.
  {
    const char* e = std::getenv("PSX_SOLVER_GPF");
    gpf_ = !rows_mode_ && cfg.Fp <= 1024 && e && e[0] == '1';
  }
  const size_t Gp = persist_ ? (size_t)persist_grid(cfg.Fp, tiles) : 0;
  const size_t Gc = gpf_ ? (size_t)(nwg_eval_ > tail_grid(cfg.Fp, nwg_eval_) ? nwg_eval_ : tail_grid(cfg.Fp, nwg_eval_))
                         : 0;
  const size_t G = rows_mode_ ? (size_t)nwg_eval_ : (Gp > Gc ? Gp : Gc);
  const size_t o_gpart = (rows_mode_ || persist_ || gpf_) ? take(G * dv_.KP * FP * 4) : 0;
  const size_t o_spart = rows_mode_ ? take(G * 2 * FP * 8) : 0;
  const size_t o_gred = rows_mode_ ? take((size_t)dv_.KP * FPI * 4) : 0;
  const int npart = nwg_eval_ > tail_grid(cfg.Fp, nwg_eval_) ? nwg_eval_ : tail_grid(cfg.Fp, nwg_eval_);
  const size_t o_part = take((size_t)npart * 32 * 4);
  const size_t o_xch = take((size_t)xch_words() * 8);
  const bool stamps = std::getenv("PSX_SOLVER_STAMPS") != nullptr;
  const size_t o_dbg = stamps ? take(32 * 16 * sizeof(long long)) : 0;
  const size_t o_cnt = take(16);
  ws_bytes_ = off;
  hip_check(hipMalloc(&ws_, ws_bytes_), "hipMalloc(solver workspace)");
  hip_check(hipMemset(ws_, 0, ws_bytes_), "hipMemset(solver workspace)");
  char* b = static_cast<char*>(ws_);
  prm_ = reinterpret_cast<SolveParams*>(b + o_prm);
  ctrl_ = reinterpret_cast<Ctrl*>(b + o_ctrl);
  dv_.X = buf.X;
  dv_.Xf = buf.Xf;
  dv_.XT = buf.XT;
  dv_.y = buf.y;
  dv_.w_old = buf.w_old;
  dv_.x = reinterpret_cast<float*>(b + o_x);
  dv_.d = reinterpret_cast<float*>(b + o_d);
  dv_.g_c = reinterpret_cast<float*>(b + o_gc);
  dv_.S = reinterpret_cast<float*>(b + o_S);
  dv_.Y = reinterpret_cast<float*>(b + o_Y);
  dv_.std_ = reinterpret_cast<float*>(b + o_std);
  dv_.inv_std = reinterpret_cast<float*>(b + o_istd);
  dv_.wfix = reinterpret_cast<float*>(b + o_wfix);
  dv_.b_eff = reinterpret_cast<float*>(b + o_beff);
  dv_.whi = reinterpret_cast<uint16_t*>(b + o_whi);
  dv_.wlo = reinterpret_cast<uint16_t*>(b + o_wlo);
  dv_.R = reinterpret_cast<unsigned short*>(b + o_R);
  dv_.part = reinterpret_cast<float*>(b + o_part);
  dv_.xch = reinterpret_cast<unsigned long long*>(b + o_xch);
  dv_.delta = buf.delta;
  dv_.w_new = buf.w_new;
  dv_.out_hi = buf.wf_hi;
  dv_.out_lo = buf.wf_lo;
  dv_.b_fin = buf.b_fin;
  dv_.loss = buf.loss;
  dv_.stats = buf.stats;
  dv_.dbg = stamps ? reinterpret_cast<long long*>(b + o_dbg) : nullptr;
  dv_.prm_count = reinterpret_cast<unsigned*>(b + o_cnt);
  dv_.gpart = rows_mode_ ? reinterpret_cast<float*>(b + o_gpart) : nullptr;
  dv_.spart = rows_mode_ ? reinterpret_cast<double*>(b + o_spart) : nullptr;
  // small grids sum the partials inside bwd_update (one launch less per slot)
  dv_.gred = rows_mode_ && nwg_eval_ > kRowsReduceInBwd ? reinterpret_cast<float*>(b + o_gred) : nullptr;
  if (gpf_) dv_.gpf = reinterpret_cast<float*>(b + o_gpart);
  if (persist_) {  // the persistent launch reads the partials; the launch chain keeps XT / R
    dvp_ = dv_;
    dvp_.gpf = reinterpret_cast<float*>(b + o_gpart);
    dvp_.gred = nullptr;
  }

  // riding evaluation passes spread over this many slots' bwd_update launches
  if (const char* e = std::getenv("PSX_RIDE_SPLIT")) ride_split_ = std::atoi(e) > 0 ? std::atoi(e) : 1;
  if (const char* e = std::getenv("PSX_FIN_INPLACE")) fin_inplace_ = std::atoi(e) != 0;
  prepare_kernels();  // >64 KiB dynamic LDS for the wide tiles (gfx950: 160 KiB per CU)
  hip_check(hipStreamCreateWithFlags(&cap_stream_, hipStreamNonBlocking), "hipStreamCreate");
  if (use_graph_) {
    hip_check(hipStreamBeginCapture(cap_stream_, hipStreamCaptureModeThreadLocal), "hipStreamBeginCapture");
    enqueue_body(cap_stream_, cfg.cap, 0, RingIngest{}, /*capturing=*/true, nullptr);
    hip_check(hipStreamEndCapture(cap_stream_, &graph_), "hipStreamEndCapture");
    hip_check(hipGraphInstantiate(&exec_, graph_, nullptr, nullptr, 0), "hipGraphInstantiate");
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
      if (kp.func == stats_prep_symbol()) {
        stats_node_ = nd;
        stats_params_ = kp;
      }
    }
    if (!stats_node_) throw std::runtime_error("solver graph: stats_prep node not found");
    stats_args_ = StatsArgs{cfg_, prm_, dv_, ctrl_, cfg.cap, 0, RingIngest{}};
    stats_kp_[0] = &stats_args_.cfg;
    stats_kp_[1] = &stats_args_.prm;
    stats_kp_[2] = &stats_args_.dv;
    stats_kp_[3] = &stats_args_.ctrl;
    stats_kp_[4] = &stats_args_.B;
    stats_kp_[5] = &stats_args_.start;
    stats_kp_[6] = &stats_args_.ing;
    stats_params_.kernelParams = stats_kp_;
    stats_params_.extra = nullptr;
  }
}

LocalSolver::~LocalSolver() {
  if (exec_) (void)hipGraphExecDestroy(exec_);
  if (graph_) (void)hipGraphDestroy(graph_);
  if (cap_stream_) (void)hipStreamDestroy(cap_stream_);
  if (ws_) (void)hipFree(ws_);
}

void LocalSolver::enqueue_body(hipStream_t s, int B, int start, const RingIngest& ing, bool capturing,
                               const EvalRide* ride) {
  if (rows_mode_) {
    const int G = nwg_eval_;
    launch_stats_rows(cfg_, prm_, dv_, B, start, G, s);
    launch_prep_rows(cfg_, prm_, dv_, ctrl_, G, s);
    for (int slot = 0; slot < cfg_.nslots; ++slot) {  // slots after convergence exit at once
      launch_fwdbwd_rows(cfg_, prm_, ctrl_, slot, dv_, G, s);
      if (dv_.gred) launch_reduce_g(cfg_, prm_, ctrl_, dv_, G, s);
      launch_bwd(cfg_, prm_, ctrl_, slot, dv_, G, s, SolveParams{B, start, 0, 0});
    }
    launch_finalize(cfg_, ctrl_, dv_, s);
    hip_check(hipGetLastError(), "solver kernel launch (rows mode)");
    return;
  }
  launch_stats_prep(cfg_, prm_, dv_, ctrl_, B, start, ing, s);
  // eager launches carry the window as arguments; a captured graph reads prm
  const SolveParams win = capturing ? SolveParams{-1, 0, 0, 0} : SolveParams{B, start, 0, 0};
  // a riding evaluation pass: its test tiles are dealt over the bwd_update
  // launches of the first `nsplit` slots (extra workgroups beside the slices)
  const int rt = ride ? ride->ntiles() : 0;
  const int nsplit = ride ? (ride_split_ < nfast_ ? ride_split_ : nfast_) : 1;
  // the bwd_update launch that ends the solve finalises the features in place
  // (the tail / finalize launch then writes only the scalars), from the first
  // slot after the riding workgroups: none of them may read the model fragments
  // that finalisation rewrites
  const int fin_slot = fin_inplace_ ? (ride ? nsplit : 0) : kNoFinSlot;
  int t0 = 0;
  for (int slot = 0; slot < nfast_; ++slot) {
    const int n = slot < nsplit ? (rt - t0 + (nsplit - slot) - 1) / (nsplit - slot) : 0;
    if (n > 0)
      launch_slot_ride(cfg_, prm_, ctrl_, slot, dv_, nwg_eval_, s, win, *ride, t0, n, fin_slot);
    else
      launch_slot(cfg_, prm_, ctrl_, slot, dv_, nwg_eval_, s, win, fin_slot);
    t0 += n;
  }
  if (cfg_.nslots > nfast_)
    launch_tail(cfg_, prm_, ctrl_, nfast_, cfg_.nslots, dv_, nwg_eval_, s, /*with_finalize=*/1);
  else
    launch_finalize(cfg_, ctrl_, dv_, s);
  hip_check(hipGetLastError(), "solver kernel launch");
}

void LocalSolver::run(int B, int start, hipStream_t stream, const RingIngest& ing, const EvalRide* ride,
                      const FusedApply* ap) {
  if (B <= 0) throw std::invalid_argument("local solve on an empty buffer");
  if ((ride || ap) && use_graph_) throw std::invalid_argument("riding evaluation / fused update: eager solver only");
  if (ride) {
    if (rows_mode_) throw std::invalid_argument("riding evaluation: small-window solver only");
    if (!ride->Xt || !ride->yt || ride->T <= 0 || !ride->whi || !ride->wlo || !ride->wb || !ride->acc ||
        !ride->ticket || !ride->slot)
      throw std::invalid_argument("riding evaluation: incomplete descriptor");
    if (ride->K != cfg_.K || ride->coff1 < 0 || ride->coff1 + ride->K > 16 ||
        (ride->slot2 && (ride->coff2 < ride->coff1 + ride->K || ride->coff2 + ride->K > 16)))
      throw std::invalid_argument("riding evaluation: class columns out of range");
    if ((unsigned)ride->ntiles() != ride->nticket) throw std::invalid_argument("riding evaluation: ticket count");
    // (the pass may read the fragments this solve's finalisation -- and a fused
    // update -- rewrite: every riding workgroup belongs to a bwd_update launch,
    // and those all precede the finalisation in stream order)
  }
  if (ap) {
    if (!ap->w || !ap->hi || !ap->lo || !ap->b || ap->coff < 0 || ap->coff + cfg_.K > 16)
      throw std::invalid_argument("fused update: bad output buffers");
    dv_.ap_w = ap->w;
    dv_.ap_hi = ap->hi;
    dv_.ap_lo = ap->lo;
    dv_.ap_b = ap->b;
    dv_.ap_lr = ap->lr;
    dv_.ap_coff = ap->coff;
  }
  if (B > cfg_.cap || start < 0 || start >= cfg_.cap) throw std::invalid_argument("window out of ring bounds");
  if (ing.n < 0 || ing.n > kMaxFusedIngest || ing.n > cfg_.cap) throw std::invalid_argument("fused ingest: bad row count");
  if (ing.n > 0 && rows_mode_) throw std::invalid_argument("fused ingest is not available for large windows");
  if (ing.n > 0) {
    if (!ing.src || !ing.ysrc || ing.dst < 0 || ing.dst >= cfg_.cap || ing.first < 0 || ing.step < 1)
      throw std::invalid_argument("fused ingest: bad source / destination");
    if ((ing.dst + ing.n - 1) % cfg_.cap != (start + B - 1) % cfg_.cap)
      throw std::invalid_argument("fused ingest: the new rows must end the window");
  }
  if (persist_) {
    // stats_prep (fused ingest, window statistics, x0, the first trial point, the
    // controller), then ONE persistent launch for every slot and the finalisation
    const int nt = ((start & 31) + B + 31) >> 5;
    const int G = persist_grid(cfg_.Fp, nt);
    launch_stats_prep(cfg_, prm_, dv_, ctrl_, B, start, ing, stream);
    SolveDev d = dvp_;
    d.ap_w = dv_.ap_w;
    d.ap_hi = dv_.ap_hi;
    d.ap_lo = dv_.ap_lo;
    d.ap_b = dv_.ap_b;
    d.ap_lr = dv_.ap_lr;
    d.ap_coff = dv_.ap_coff;
    launch_persist(cfg_, d, ctrl_, SolveParams{B, start, 0, 0}, G, ride ? *ride : EvalRide{}, ride ? ride->ntiles() : 0,
                   stream);
    hip_check(hipGetLastError(), "persistent solve launch");
    dv_.ap_w = nullptr;
    return;
  }
  if (use_graph_) {
    stats_args_.B = B;
    stats_args_.start = start;
    stats_args_.ing = ing;
    hip_check(hipGraphExecKernelNodeSetParams(exec_, stats_node_, &stats_params_), "hipGraphExecKernelNodeSetParams");
    hip_check(hipGraphLaunch(exec_, stream), "hipGraphLaunch");
  } else {
    enqueue_body(stream, B, start, ing, false, ride);
  }
  dv_.ap_w = nullptr;  // the launches above took their copy of dv_
}

std::vector<long long> LocalSolver::read_stamps(hipStream_t stream) {
  std::vector<long long> v;
  if (!dv_.dbg) return v;
  v.resize(32 * 16);
  hip_check(hipMemcpyAsync(v.data(), dv_.dbg, v.size() * sizeof(long long), hipMemcpyDeviceToHost, stream),
            "read stamps");
  hip_check(hipStreamSynchronize(stream), "sync");
  return v;
}

void LocalSolver::read_ctrl(Ctrl* out, hipStream_t stream) {
  hip_check(hipMemcpyAsync(out, ctrl_, sizeof(Ctrl), hipMemcpyDeviceToHost, stream), "read ctrl");
  hip_check(hipStreamSynchronize(stream), "sync");
}

}  // namespace psx
