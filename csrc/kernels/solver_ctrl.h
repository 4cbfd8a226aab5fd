// On-device control logic of the worker's local solver.
//
// The reference worker runs `new LogisticRegression().setMaxIter(2)
// .setInitialModel(..).fit(buffer)` (reference:
// src/main/java/de/hpi/datastreams/ml/LogisticRegressionTaskSpark.java:170-184),
// i.e. Spark's L-BFGS (history 10) with a strong-Wolfe line search on the
// standardised multinomial objective.  On MI355X the per-iteration vector work
// is done by multi-workgroup kernels; everything that is *scalar* -- the
// line-search bracket, the Wolfe tests, the L-BFGS curvature pairs -- lives in
// this struct and is advanced by ONE thread of the last-arriving workgroup of
// the reduction kernel.  No host round trip is needed between function
// evaluations, so a whole local solve is one hipGraph launch.
//
// L-BFGS uses the compact representation (Byrd, Nocedal & Schnabel 1994):
//   H g = gamma*g + S p - gamma*Y a,  a = R^-1 S^T g,
//   R^T p = (D + gamma Y^T Y) a - gamma Y^T g
// which needs only dot products of g with the stored pairs.  Those dots are
// produced by the same reduction pass that materialises the gradient, so a
// new search direction costs one elementwise pass instead of the 2m dependent
// reductions of the textbook two-loop recursion.
//
// The same code compiles for the host (unit tests, CPU reference checks).
#pragma once
#include <cmath>
#include <cstdint>

#if defined(__HIPCC__)
#define PSX_HD __host__ __device__
#else
#define PSX_HD
#endif

namespace psx {

constexpr int kMaxHist = 16;
// Evaluation slots per solve are < kMaxSlots: the persistent solve's all-gather
// tags (run * kMaxSlots + slot + 1) and barrier words (run << 16 | n) must not
// repeat between consecutive solves.
constexpr int kMaxSlots = 64;

// Workspace of the compact L-BFGS algebra.  On the device it lives in LDS (a
// stack array would be scratch memory: each access an L1/L2 round trip for
// the single controller thread).
struct CtrlScratch {
  int idx[kMaxHist];
  double u[kMaxHist], v[kMaxHist], a[kMaxHist], rhs[kMaxHist], p[kMaxHist], dy[kMaxHist];
};

enum SolverMode : int { kModeLBFGS = 0, kModeGD = 1 };
enum Phase : int { kPhInit = 0, kPhLS = 1, kPhDone = 2 };
enum Action : int {
  kActNone = 0,
  kActInit = 1,        // g_c <- g_t ; d <- coefs
  kActTrial = 2,       // only the trial step t changed
  kActAccept = 3,      // x += t_acc d ; push pair ; g_c <- g_t ; d <- coefs
  kActAcceptDone = 4,  // x += t_acc d ; finished
  kActDone = 5,        // finished without moving
};

struct SolverCfg {
  int K;       // logits (classes incl. phantom class 0)
  int F;       // real features
  int Fp;      // padded features (multiple of 128)
  int P;       // K*Fp + K
  int cap;     // ring capacity (rows)
  int iters;   // local solver iterations (reference: 2)
  int hist;    // L-BFGS history (reference/Spark: 10)
  int ls_max;  // line-search evaluations per iteration budget
  int mode;    // SolverMode
  int center;  // multinomial centering (Spark, regParam == 0)
  int zero_const;  // features with zero std get coefficient 0 (Spark behaviour)
  int nslots;  // evaluation slots in the graph
  float gd_lr; // step for mode GD
  float tol;   // convergence tolerance (Spark default 1e-6)
  int xf32 = 0;  // fp32 feature rows (--dtype fp32): row-parallel solver with hi+lo bf16 MFMA operands
  // the whole small-window solve as ONE persistent launch (solve_kernels.hip:
  // solve_persist_kernel); needs its G workgroups co-resident, so only for a
  // solver that has the device to itself (one worker per process)
  int persist = 0;
  // XCD (0..7) that hosts the persistent solve's workgroups and the chain's
  // bwd_update slices (their hand-offs through that XCD's L2); -1: the chain's
  // slices spread over the XCDs (sc1 hand-offs) -- a solver that shares the GPU
  // with other solvers' concurrent launches
  int xcd = 0;
  // 1: the line-search retry slots run in ONE tail launch with grid barriers (its
  // workgroups must be co-resident); 0: every budgeted slot is its own fwd /
  // bwd_update launch pair (no cross-launch co-residency: in-process workers that
  // solve concurrently)
  int tail = 1;
};

// New stream rows a solve ingests into its ring before reading the window
// (fused into the first kernel of the solve): rows src_first + i*src_step
// (i < n) of the resident dataset go to ring slots (dst + i) % cap, and must be
// the newest n rows of the window.  n == 0: nothing to ingest.
constexpr int kMaxFusedIngest = 1024;
// fin_slot of a launch chain that never finalises inside bwd_update
constexpr int kNoFinSlot = 1 << 30;
struct RingIngest {
  const uint16_t* src;   // dataset rows [*][Fp] bf16
  const int32_t* ysrc;   // dataset labels
  long long first, step;
  int n, dst;
};

struct SolveParams {
  int B;      // rows in the window
  int start;  // first ring slot of the window
  int pad0, pad1;
};

struct Ctrl {
  int phase, action, action_slot, iter;
  int ls_i, zoom, evals, m;
  int head, push_slot, nacc, ls_fail;
  int dir_reset, fin, pad1, pad2;  // fin: features finalised by the last bwd_update launch
  double t;      // next trial step (consumed by the update kernel)
  double t_acc;  // accepted step (consumed by the update kernel)
  double f_c, dg0, gg_c, f_init;
  double lo_t, lo_f, lo_d, hi_t, hi_f, hi_d;
  double gamma;
  double cg;
  double cs[kMaxHist], cy[kMaxHist];  // direction = cg*g_c + sum cs_i S_i + sum cy_i Y_i (physical slots)
  double SY[kMaxHist][kMaxHist];      // s_i . y_j  (physical slots)
  double YY[kMaxHist][kMaxHist];      // y_i . y_j
  double Sg[kMaxHist], Yg[kMaxHist];  // s_i . g_c, y_i . g_c
  unsigned ticket;
  unsigned pad3;
};

// Number of fp64 dot products the reduction kernel produces.
PSX_HD inline int num_dots(int hist) { return 3 + 2 * hist; }
// dots layout: [0]=g_t.g_t [1]=g_t.d [2]=g_t.g_c [3+i]=S_i.g_t [3+H+i]=Y_i.g_t

PSX_HD inline void ctrl_init(Ctrl& c) {
  c.phase = kPhInit;
  c.action = kActNone;
  c.action_slot = -1;
  c.iter = c.ls_i = c.zoom = c.evals = c.m = 0;
  c.head = -1;
  c.push_slot = -1;
  c.nacc = c.ls_fail = c.dir_reset = 0;
  c.fin = 0;
  c.t = 0.0;
  c.t_acc = 0.0;
  c.f_c = c.dg0 = c.gg_c = c.f_init = 0.0;
  c.lo_t = c.lo_f = c.lo_d = c.hi_t = c.hi_f = c.hi_d = 0.0;
  c.gamma = 1.0;
  c.cg = 0.0;
  for (int i = 0; i < kMaxHist; ++i) {
    c.cs[i] = c.cy[i] = c.Sg[i] = c.Yg[i] = 0.0;
  }
  // SY/YY entries are always written when a pair is pushed, before any read.
  c.ticket = 0;
}

// Cubic interpolation between two brackets (Nocedal & Wright eq. 3.59),
// safeguarded into the middle 80% of the interval; bisection when the cubic
// has no real minimiser.
PSX_HD inline double ls_interp(double lt, double lf, double ld, double rt, double rf, double rd) {
  if (lt > rt) {  // order the bracket
    double a = lt, b = lf, e = ld;
    lt = rt; lf = rf; ld = rd;
    rt = a; rf = b; rd = e;
  }
  double w = rt - lt;
  double lb = lt + 0.1 * w, ub = lt + 0.9 * w;
  double d1 = ld + rd - 3.0 * (lf - rf) / (lt - rt);
  double rad = d1 * d1 - ld * rd;
  double t;
  if (!(rad >= 0.0) || !(w > 0.0)) {
    t = lt + 0.5 * w;
  } else {
    double d2 = sqrt(rad);
    double den = rd - ld + 2.0 * d2;
    t = den != 0.0 ? rt - w * (rd + d2 - d1) / den : lt + 0.5 * w;
    if (!(t == t)) t = lt + 0.5 * w;
  }
  if (t < lb) t = lb;
  if (t > ub) t = ub;
  return t;
}

// Compact L-BFGS direction d = -H g for the current history.  Fills cg/cs/cy
// and returns d . g.
PSX_HD inline double ctrl_direction(Ctrl& __restrict__ c, int H, CtrlScratch& __restrict__ ws) {
  for (int i = 0; i < kMaxHist; ++i) c.cs[i] = c.cy[i] = 0.0;
  const int m = c.m;
  if (m == 0) {
    c.cg = -1.0;
    return -c.gg_c;
  }
  int* idx = ws.idx;  // logical (oldest..newest) -> physical
  for (int i = 0; i < m; ++i) {  // (head - (m - 1 - i)) mod H; the operand is > -H (no integer division)
    const int x = c.head - (m - 1 - i);
    idx[i] = x < 0 ? x + H : x;
  }
  const double gamma = c.gamma;
  double *u = ws.u, *v = ws.v, *a = ws.a, *rhs = ws.rhs, *p = ws.p;
  for (int i = 0; i < m; ++i) {
    u[i] = c.Sg[idx[i]];
    v[i] = c.Yg[idx[i]];
  }
  // R a = u   (R upper triangular, R_ij = s_i.y_j, i <= j): back substitution
  for (int i = m - 1; i >= 0; --i) {
    double s = u[i];
    for (int j = i + 1; j < m; ++j) s -= c.SY[idx[i]][idx[j]] * a[j];
    double r = c.SY[idx[i]][idx[i]];
    a[i] = r != 0.0 ? s / r : 0.0;
  }
  // rhs = (D + gamma YY) a - gamma v
  for (int i = 0; i < m; ++i) {
    double s = c.SY[idx[i]][idx[i]] * a[i];
    for (int j = 0; j < m; ++j) s += gamma * c.YY[idx[i]][idx[j]] * a[j];
    rhs[i] = s - gamma * v[i];
  }
  // R^T p = rhs   (R^T lower triangular): forward substitution
  for (int i = 0; i < m; ++i) {
    double s = rhs[i];
    for (int j = 0; j < i; ++j) s -= c.SY[idx[j]][idx[i]] * p[j];
    double r = c.SY[idx[i]][idx[i]];
    p[i] = r != 0.0 ? s / r : 0.0;
  }
  // H g = gamma g + S p - gamma Y a  ->  d = -H g
  c.cg = -gamma;
  double dg = -gamma * c.gg_c;
  for (int i = 0; i < m; ++i) {
    c.cs[idx[i]] = -p[i];
    c.cy[idx[i]] = gamma * a[i];
    dg += -p[i] * u[i] + gamma * a[i] * v[i];
  }
  return dg;
}

// Accept the evaluated trial point (step t_eval): bookkeeping of the new
// curvature pair and the next direction.  `dots` as produced by the reduction.
PSX_HD inline void ctrl_accept(Ctrl& __restrict__ c, const SolverCfg& cfg, double f_t,
                               const double* __restrict__ dots, int slot, CtrlScratch& __restrict__ ws) {
  const int H = cfg.hist;
  const double tt = dots[0], td = dots[1], tc = dots[2];
  const double t = c.t;
  c.t_acc = t;
  c.iter += 1;
  c.nacc += 1;
  const double f_prev = c.f_c;
  c.f_c = f_t;
  c.action_slot = slot;
  c.push_slot = -1;
  bool done = c.iter >= cfg.iters;
  double gnorm = sqrt(tt > 0 ? tt : 0.0);
  double fscale = fabs(f_t) > 1.0 ? fabs(f_t) : 1.0;
  if (cfg.mode == kModeLBFGS) {
    if (gnorm <= (double)cfg.tol * fscale) done = true;
    if (fabs(f_prev - f_t) <= (double)cfg.tol * fscale) done = true;
  }
  if (done) {
    c.action = kActAcceptDone;
    c.phase = kPhDone;
    return;
  }
  if (cfg.mode == kModeGD) {
    c.gg_c = tt;
    c.m = 0;
    c.cg = -1.0;
    for (int i = 0; i < kMaxHist; ++i) c.cs[i] = c.cy[i] = 0.0;
    c.dg0 = -tt;
    c.t = cfg.gd_lr;
    c.action = kActAccept;
    return;
  }
  // --- new curvature pair s = t d, y = g_t - g_c ---
  const int m = c.m;
  int* idx = ws.idx;
  for (int i = 0; i < m; ++i) {  // (head - (m - 1 - i)) mod H; the operand is > -H (no integer division)
    const int x = c.head - (m - 1 - i);
    idx[i] = x < 0 ? x + H : x;
  }
  // d . y_j for the stored pairs (d is known through its coefficients)
  double* dy = ws.dy;
  for (int jj = 0; jj < m; ++jj) {
    int j = idx[jj];
    double s = c.cg * c.Yg[j];
    for (int ii = 0; ii < m; ++ii) {
      int i = idx[ii];
      s += c.cs[i] * c.SY[i][j] + c.cy[i] * c.YY[i][j];
    }
    dy[jj] = s;
  }
  const double sy_new = t * (td - c.dg0);
  const double yy_new = tt - 2.0 * tc + c.gg_c;
  const bool keep = sy_new > 1e-10 * (yy_new > 0 ? yy_new : 1.0) && yy_new > 0.0;
  if (keep) {
    int slotp = c.head + 1 == H ? 0 : c.head + 1;  // (head + 1) mod H, head in [-1, H)
    // if the ring is full the oldest pair (physical slotp) is evicted
    int mm = m < H ? m : m - 1;  // surviving old pairs
    int first = m - mm;          // logical index of the first survivor
    for (int ii = first; ii < m; ++ii) {
      int i = idx[ii];
      double St = dots[3 + i], Yt = dots[3 + H + i];
      c.SY[i][slotp] = St - c.Sg[i];            // s_i . y_new
      c.SY[slotp][i] = t * dy[ii];              // s_new . y_i
      double yyi = Yt - c.Yg[i];                // y_i . y_new
      c.YY[i][slotp] = yyi;
      c.YY[slotp][i] = yyi;
      c.Sg[i] = St;  // dots with the new gradient
      c.Yg[i] = Yt;
    }
    c.SY[slotp][slotp] = sy_new;
    c.YY[slotp][slotp] = yy_new;
    c.Sg[slotp] = t * td;
    c.Yg[slotp] = tt - tc;
    c.head = slotp;
    c.m = mm + 1;
    c.push_slot = slotp;
    c.gamma = sy_new / yy_new;
  } else {
    for (int ii = 0; ii < m; ++ii) {
      int i = idx[ii];
      c.Sg[i] = dots[3 + i];
      c.Yg[i] = dots[3 + H + i];
    }
  }
  c.gg_c = tt;
  double dg = ctrl_direction(c, H, ws);
  if (!(dg < 0.0)) {  // not a descent direction: drop the history, steepest descent
    c.m = 0;
    c.head = -1;
    c.dir_reset += 1;
    dg = ctrl_direction(c, H, ws);
  }
  c.dg0 = dg;
  c.t = 1.0;
  c.lo_t = 0.0;
  c.lo_f = c.f_c;
  c.lo_d = dg;
  c.ls_i = 0;
  c.zoom = 0;
  c.action = kActAccept;
}

// Advance the state machine after the function evaluation of `slot`.
// f_t = objective at the trial point, dots as documented above.
// (__restrict__: the state, the dots and the scratch never alias -- on the device
// they are separate LDS blocks, so the single controller thread's loads need not
// wait behind its own stores)
PSX_HD inline void ctrl_step(Ctrl& __restrict__ c, const SolverCfg& cfg, double f_t, const double* __restrict__ dots,
                             int slot, CtrlScratch& __restrict__ ws) {
  c.evals += 1;
  const double tt = dots[0], td = dots[1];
  const bool finite = f_t == f_t && fabs(f_t) < 1e300;
  if (c.phase == kPhDone) return;
  if (c.phase == kPhInit) {
    c.f_c = f_t;
    c.f_init = f_t;
    c.gg_c = tt;
    c.m = 0;
    c.head = -1;
    c.action_slot = slot;
    double gnorm = sqrt(tt > 0 ? tt : 0.0);
    if (!finite || gnorm == 0.0 || cfg.iters <= 0) {
      c.action = kActDone;
      c.phase = kPhDone;
      return;
    }
    c.cg = -1.0;
    for (int i = 0; i < kMaxHist; ++i) c.cs[i] = c.cy[i] = 0.0;
    c.dg0 = -tt;
    c.t = cfg.mode == kModeGD ? (double)cfg.gd_lr : 1.0 / gnorm;  // first step 1/||d||
    c.lo_t = 0.0;
    c.lo_f = f_t;
    c.lo_d = c.dg0;
    c.ls_i = 0;
    c.zoom = 0;
    c.phase = kPhLS;
    c.action = kActInit;
    return;
  }
  // ---- line search on phi(t) = f(x + t d) ----
  c.action_slot = slot;
  if (cfg.mode == kModeGD) {
    ctrl_accept(c, cfg, f_t, dots, slot, ws);
    return;
  }
  const double c1 = 1e-4, c2 = 0.9;
  const double t = c.t;
  const double dd = td;
  c.ls_i += 1;
  const bool armijo = finite && f_t <= c.f_c + c1 * t * c.dg0;
  double tn = t;
  if (!c.zoom) {
    if (!finite) {
      tn = t * 0.5;
    } else if (!armijo || (f_t >= c.lo_f && c.ls_i > 1)) {
      c.hi_t = t; c.hi_f = f_t; c.hi_d = dd;
      c.zoom = 1;
      tn = ls_interp(c.lo_t, c.lo_f, c.lo_d, c.hi_t, c.hi_f, c.hi_d);
    } else if (fabs(dd) <= c2 * fabs(c.dg0)) {
      ctrl_accept(c, cfg, f_t, dots, slot, ws);
      return;
    } else if (dd >= 0.0) {
      c.hi_t = c.lo_t; c.hi_f = c.lo_f; c.hi_d = c.lo_d;
      c.lo_t = t; c.lo_f = f_t; c.lo_d = dd;
      c.zoom = 1;
      tn = ls_interp(c.lo_t, c.lo_f, c.lo_d, c.hi_t, c.hi_f, c.hi_d);
    } else {
      c.lo_t = t; c.lo_f = f_t; c.lo_d = dd;
      tn = t * 1.5;
    }
  } else {
    if (!armijo || f_t >= c.lo_f) {
      c.hi_t = t; c.hi_f = f_t; c.hi_d = dd;
    } else {
      if (fabs(dd) <= c2 * fabs(c.dg0)) {
        ctrl_accept(c, cfg, f_t, dots, slot, ws);
        return;
      }
      if (dd * (c.hi_t - c.lo_t) >= 0.0) {
        c.hi_t = c.lo_t; c.hi_f = c.lo_f; c.hi_d = c.lo_d;
      }
      c.lo_t = t; c.lo_f = f_t; c.lo_d = dd;
    }
    tn = ls_interp(c.lo_t, c.lo_f, c.lo_d, c.hi_t, c.hi_f, c.hi_d);
  }
  const bool out_of_slots = slot + 1 >= cfg.nslots;
  if (c.ls_i >= cfg.ls_max || out_of_slots) {
    c.ls_fail += 1;
    if (armijo && f_t < c.f_c) {  // settle for sufficient decrease
      ctrl_accept(c, cfg, f_t, dots, slot, ws);
      if (out_of_slots && c.phase != kPhDone) {
        c.action = kActAcceptDone;
        c.phase = kPhDone;
      }
      return;
    }
    c.action = kActDone;
    c.phase = kPhDone;
    return;
  }
  c.t = tn;
  c.action = kActTrial;
}

// Convenience overload with a stack workspace (host code, tests).
PSX_HD inline void ctrl_step(Ctrl& c, const SolverCfg& cfg, double f_t, const double* dots, int slot) {
  CtrlScratch ws;
  ctrl_step(c, cfg, f_t, dots, slot, ws);
}

}  // namespace psx
