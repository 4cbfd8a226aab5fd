#include "solver.h"

#include <stdexcept>
#include <string>

namespace psx {

void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

static size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

LocalSolver::LocalSolver(const SolverCfg& cfg, const SolverBuffers& buf, int max_eval_wg, bool use_graph)
    : cfg_(cfg), buf_(buf), use_graph_(use_graph) {
  if (!fp_supported(cfg.Fp)) throw std::invalid_argument("unsupported padded feature width " + std::to_string(cfg.Fp));
  if (cfg.K < 2 || cfg.K > 16) throw std::invalid_argument("num classes (incl. phantom) must be in [2,16]");
  if (cfg.P != cfg.K * cfg.Fp + cfg.K) throw std::invalid_argument("P mismatch");
  if (cfg.hist < 1 || cfg.hist > kMaxHist) throw std::invalid_argument("history must be in [1,16]");
  if (cfg.nslots < 1) throw std::invalid_argument("nslots must be >= 1");
  const int tiles = (cfg.cap + kTileRows - 1) / kTileRows;
  nwg_eval_ = tiles < max_eval_wg ? tiles : max_eval_wg;
  if (nwg_eval_ < 1) nwg_eval_ = 1;
  stats_row_blocks_ = (cfg.cap + 127) / 128;
  if (stats_row_blocks_ > 64) stats_row_blocks_ = 64;
  if (stats_row_blocks_ < 1) stats_row_blocks_ = 1;

  const size_t P = cfg.P, FP = cfg.Fp, H = cfg.hist;
  const int nwg_red = (cfg.P + 255) / 256;
  size_t off = 0;
  auto take = [&](size_t bytes) {
    size_t o = off;
    off = align_up(off + bytes, 256);
    return o;
  };
  const size_t o_prm = take(sizeof(SolveParams));
  const size_t o_ctrl = take(sizeof(Ctrl));
  const size_t o_acc = take((size_t)stats_row_blocks_ * 2 * FP * sizeof(double));
  const size_t o_dot = take((size_t)nwg_red * num_dots(cfg.hist) * sizeof(double));
  const size_t o_x = take(P * 4), o_d = take(P * 4), o_gc = take(P * 4), o_gt = take(P * 4);
  const size_t o_S = take(H * P * 4), o_Y = take(H * P * 4);
  const size_t o_std = take(FP * 4), o_istd = take(FP * 4), o_wfix = take(P * 4), o_beff = take(16 * 4);
  const size_t o_whi = take(16 * FP * 2), o_wlo = take(16 * FP * 2);
  const size_t o_G = take((size_t)nwg_eval_ * cfg.K * FP * 4);
  const size_t o_R = take((size_t)nwg_eval_ * 16 * 4);
  const size_t o_L = take((size_t)nwg_eval_ * 4);
  ws_bytes_ = off;
  hip_check(hipMalloc(&ws_, ws_bytes_), "hipMalloc(solver workspace)");
  hip_check(hipMemset(ws_, 0, ws_bytes_), "hipMemset(solver workspace)");
  char* b = static_cast<char*>(ws_);
  prm_ = reinterpret_cast<SolveParams*>(b + o_prm);
  ctrl_ = reinterpret_cast<Ctrl*>(b + o_ctrl);
  acc_ = reinterpret_cast<double*>(b + o_acc);
  dotpart_ = reinterpret_cast<double*>(b + o_dot);
  x_ = reinterpret_cast<float*>(b + o_x);
  d_ = reinterpret_cast<float*>(b + o_d);
  gc_ = reinterpret_cast<float*>(b + o_gc);
  gt_ = reinterpret_cast<float*>(b + o_gt);
  S_ = reinterpret_cast<float*>(b + o_S);
  Y_ = reinterpret_cast<float*>(b + o_Y);
  std_ = reinterpret_cast<float*>(b + o_std);
  inv_std_ = reinterpret_cast<float*>(b + o_istd);
  wfix_ = reinterpret_cast<float*>(b + o_wfix);
  beff_ = reinterpret_cast<float*>(b + o_beff);
  whi_ = reinterpret_cast<uint16_t*>(b + o_whi);
  wlo_ = reinterpret_cast<uint16_t*>(b + o_wlo);
  Gpart_ = reinterpret_cast<float*>(b + o_G);
  Rpart_ = reinterpret_cast<float*>(b + o_R);
  Lpart_ = reinterpret_cast<float*>(b + o_L);

  // >64 KiB dynamic LDS for the wide tiles (gfx950 has 160 KiB per CU)
  prepare_kernels();
  hip_check(hipStreamCreateWithFlags(&cap_stream_, hipStreamNonBlocking), "hipStreamCreate");
  if (use_graph_) {
    hip_check(hipStreamBeginCapture(cap_stream_, hipStreamCaptureModeThreadLocal), "hipStreamBeginCapture");
    enqueue_body(cap_stream_);
    hip_check(hipStreamEndCapture(cap_stream_, &graph_), "hipStreamEndCapture");
    hip_check(hipGraphInstantiate(&exec_, graph_, nullptr, nullptr, 0), "hipGraphInstantiate");
  }
}

LocalSolver::~LocalSolver() {
  if (exec_) (void)hipGraphExecDestroy(exec_);
  if (graph_) (void)hipGraphDestroy(graph_);
  if (cap_stream_) (void)hipStreamDestroy(cap_stream_);
  if (ws_) (void)hipFree(ws_);
}

void LocalSolver::enqueue_body(hipStream_t s) {
  const SolverCfg& c = cfg_;
  launch_stats(buf_.X, prm_, c.cap, c.Fp, acc_, stats_row_blocks_, s);
  launch_prep(c, prm_, acc_, buf_.w_old, x_, d_, gc_, std_, inv_std_, wfix_, whi_, wlo_, beff_, ctrl_,
              stats_row_blocks_, s);
  for (int slot = 0; slot < c.nslots; ++slot) {
    launch_eval(c, prm_, ctrl_, slot, buf_.X, buf_.y, whi_, wlo_, beff_, Gpart_, Rpart_, Lpart_, nwg_eval_, s);
    launch_reduce(c, prm_, ctrl_, slot, Gpart_, Rpart_, Lpart_, nwg_eval_, inv_std_, d_, gc_, gt_, S_, Y_, dotpart_,
                  s);
    launch_update(c, ctrl_, slot, x_, d_, gc_, gt_, S_, Y_, inv_std_, wfix_, whi_, wlo_, beff_, s);
  }
  launch_finalize(c, ctrl_, x_, inv_std_, wfix_, buf_.w_old, buf_.delta, buf_.w_new, buf_.wf_hi, buf_.wf_lo,
                  buf_.b_fin, buf_.loss, buf_.stats, s);
  hip_check(hipGetLastError(), "solver kernel launch");
}

void LocalSolver::run(int B, int start, hipStream_t stream) {
  if (B <= 0) throw std::invalid_argument("local solve on an empty buffer");
  if (B > cfg_.cap || start < 0 || start >= cfg_.cap) throw std::invalid_argument("window out of ring bounds");
  launch_set_params(prm_, B, start, stream);
  if (use_graph_) {
    hip_check(hipGraphLaunch(exec_, stream), "hipGraphLaunch");
  } else {
    enqueue_body(stream);
  }
}

void LocalSolver::read_ctrl(Ctrl* out, hipStream_t stream) {
  hip_check(hipMemcpyAsync(out, ctrl_, sizeof(Ctrl), hipMemcpyDeviceToHost, stream), "read ctrl");
  hip_check(hipStreamSynchronize(stream), "sync");
}

}  // namespace psx
