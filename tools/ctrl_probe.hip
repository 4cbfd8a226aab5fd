// Standalone timing of the solver controller step (csrc/kernels/solver_ctrl.h) on one
// thread with its state in LDS, as inside the persistent solves: init, a trial, an accept.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I csrc/kernels -I csrc tools/ctrl_probe.hip -o tools/ctrl_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include "solver_ctrl.h"
constexpr int kND = 3 + 2 * psx::kMaxHist;
using namespace psx;
__global__ void kctrl(SolverCfg cfg, const double* dg, Ctrl* g, long long* t) {
  __shared__ Ctrl c, snap;
  __shared__ CtrlScratch ws;
  __shared__ double dots[3][64];
  if (threadIdx.x == 0) { c = *g; ctrl_init(c); for (int s = 0; s < 3; ++s) for (int i = 0; i < 64; ++i) dots[s][i] = dg[s * 64 + i]; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int s = 0; s < 3; ++s) {
      if (s == 1) snap = c;
      const long long t0 = __builtin_amdgcn_s_memrealtime();
      ctrl_step(c, cfg, dots[s][kND], dots[s], s, ws);
      __builtin_amdgcn_s_waitcnt(0);
      const long long t1 = __builtin_amdgcn_s_memrealtime();
      t[2 * s] = t1 - t0;
      t[2 * s + 1] = c.action;
    }
    // the accepting step again, its code now in the instruction cache
    c = snap;
    const long long t0 = __builtin_amdgcn_s_memrealtime();
    ctrl_step(c, cfg, dots[1][kND], dots[1], 1, ws);
    __builtin_amdgcn_s_waitcnt(0);
    t[6] = __builtin_amdgcn_s_memrealtime() - t0;
  }
  __syncthreads();
  if (threadIdx.x == 0) *g = c;
}
int main() {
  SolverCfg cfg{};
  cfg.K = 6; cfg.F = 1024; cfg.Fp = 1024; cfg.P = 6150; cfg.iters = 2; cfg.hist = 10; cfg.ls_max = 20; cfg.mode = 0;
  cfg.nslots = 16; cfg.tol = 1e-6f; cfg.gd_lr = 1.f;
  double h[3 * 64] = {0};
  // slot 0 (init): f=1.0, gg=4; slot 1: trial with sufficient decrease and curvature -> accept
  h[0] = 4.0; h[kND] = 1.0;
  h[64 + 0] = 1.0; h[64 + 1] = -0.1; h[64 + 2] = -1.0; h[64 + kND] = 0.5;
  h[128 + 0] = 0.5; h[128 + 1] = -0.05; h[128 + 2] = -0.5; h[128 + kND] = 0.4;
  double* dg; Ctrl* g; long long* t;
  hipMalloc(&dg, sizeof(h)); hipMalloc(&g, sizeof(Ctrl)); hipMalloc(&t, 64);
  hipMemcpy(dg, h, sizeof(h), hipMemcpyHostToDevice);
  hipMemset(g, 0, sizeof(Ctrl));
  for (int rep = 0; rep < 3; ++rep) {
    kctrl<<<1, 256>>>(cfg, dg, g, t);
    long long ht[7];
    hipMemcpy(ht, t, sizeof(ht), hipMemcpyDeviceToHost);
    printf("{\"rep\": %d, \"us\": [%.2f, %.2f, %.2f], \"action\": [%lld, %lld, %lld], \"accept_again_us\": %.2f}\n", rep,
           ht[0] / 100.0, ht[2] / 100.0, ht[4] / 100.0, ht[1], ht[3], ht[5], ht[6] / 100.0);
  }
  return 0;
}
