// pybind11 bindings for the HIP side (_psx_hip): the worker local solver, the
// server update, test-set evaluation and ring ingest.  Tensors are passed as
// raw device pointers (torch `data_ptr()`), streams as `cuda_stream` handles;
// the Python layer validates shapes/dtypes before calling in.
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <cstring>
#include <pybind11/stl.h>

#include <memory>
#include <stdexcept>

#include "../comm/ipc_comm.h"
#include "../comm/peer_bus.h"
#include "../comm/rccl_comm.h"
#include "../runtime/async_server.h"
#include "../runtime/bsp_loop.h"
#include "../runtime/lanes_loop.h"
#include "../runtime/peer_server.h"
#include "../runtime/keyrange_loop.h"
#include "../kernels/lr_kernels.h"
#include "../solver/solver.h"
#include "../solver/wide_solver.h"

namespace py = pybind11;
using namespace psx;

namespace {
template <typename T>
T* P(uintptr_t v) {
  return reinterpret_cast<T*>(v);
}
hipStream_t S(uintptr_t v) { return reinterpret_cast<hipStream_t>(v); }

py::dict ctrl_dict(const Ctrl& c, int H) {
  py::dict d;
  d["phase"] = c.phase;
  d["action"] = c.action;
  d["action_slot"] = c.action_slot;
  d["iter"] = c.iter;
  d["evals"] = c.evals;
  d["m"] = c.m;
  d["nacc"] = c.nacc;
  d["ls_fail"] = c.ls_fail;
  d["dir_reset"] = c.dir_reset;
  d["t"] = c.t;
  d["t_acc"] = c.t_acc;
  d["f_c"] = c.f_c;
  d["f_init"] = c.f_init;
  d["dg0"] = c.dg0;
  d["gg_c"] = c.gg_c;
  d["gamma"] = c.gamma;
  (void)H;
  return d;
}
}  // namespace

PYBIND11_MODULE(_psx_hip, m) {
  m.doc() = "psx HIP kernels (gfx950)";

  m.def("device_count", []() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
  });
  m.def("device_arch", [](int dev) {
    hipDeviceProp_t p;
    hip_check(hipGetDeviceProperties(&p, dev), "hipGetDeviceProperties");
    py::dict d;
    d["name"] = std::string(p.name);
    d["gcnArchName"] = std::string(p.gcnArchName);
    d["multiProcessorCount"] = p.multiProcessorCount;
    d["sharedMemPerBlock"] = (size_t)p.sharedMemPerBlock;
    d["maxSharedMemoryPerMultiProcessor"] = (size_t)p.maxSharedMemoryPerMultiProcessor;
    d["totalGlobalMem"] = (size_t)p.totalGlobalMem;
    return d;
  });
  m.def("fp_supported", &fp_supported);
  m.def("solver_rows_mode", &rows_mode_for, py::arg("cap"));
  m.def("eval_lds_bytes", &eval_lds_bytes);

  py::class_<SolverCfg>(m, "SolverCfg", py::module_local())
      .def(py::init<>())
      .def_readwrite("K", &SolverCfg::K)
      .def_readwrite("F", &SolverCfg::F)
      .def_readwrite("Fp", &SolverCfg::Fp)
      .def_readwrite("P", &SolverCfg::P)
      .def_readwrite("cap", &SolverCfg::cap)
      .def_readwrite("iters", &SolverCfg::iters)
      .def_readwrite("hist", &SolverCfg::hist)
      .def_readwrite("ls_max", &SolverCfg::ls_max)
      .def_readwrite("mode", &SolverCfg::mode)
      .def_readwrite("center", &SolverCfg::center)
      .def_readwrite("zero_const", &SolverCfg::zero_const)
      .def_readwrite("nslots", &SolverCfg::nslots)
      .def_readwrite("gd_lr", &SolverCfg::gd_lr)
      .def_readwrite("tol", &SolverCfg::tol)
      .def_readwrite("xf32", &SolverCfg::xf32)
      .def_readwrite("persist", &SolverCfg::persist)
      .def_readwrite("xcd", &SolverCfg::xcd)
      .def_readwrite("tail", &SolverCfg::tail);

  py::class_<LocalSolver>(m, "LocalSolver")
      .def(py::init([](const SolverCfg& cfg, uintptr_t X, uintptr_t XT, uintptr_t y, uintptr_t w_old,
                       uintptr_t delta, uintptr_t w_new, uintptr_t wf_hi, uintptr_t wf_lo, uintptr_t b_fin,
                       uintptr_t loss, uintptr_t stats, int max_eval_wg, bool use_graph) {
             SolverBuffers b;
             if (cfg.xf32)
               b.Xf = P<const float>(X);  // the ring holds fp32 rows
             else
               b.X = P<const uint16_t>(X);
             b.XT = P<const uint16_t>(XT);
             b.y = P<const int32_t>(y);
             b.w_old = P<const float>(w_old);
             b.delta = P<float>(delta);
             b.w_new = P<float>(w_new);
             b.wf_hi = P<uint16_t>(wf_hi);
             b.wf_lo = P<uint16_t>(wf_lo);
             b.b_fin = P<float>(b_fin);
             b.loss = P<float>(loss);
             b.stats = P<int>(stats);
             return std::make_unique<LocalSolver>(cfg, b, max_eval_wg, use_graph);
           }),
           py::arg("cfg"), py::arg("X"), py::arg("XT"), py::arg("y"), py::arg("w_old"), py::arg("delta"),
           py::arg("w_new"),
           py::arg("wf_hi"), py::arg("wf_lo"), py::arg("b_fin"), py::arg("loss"), py::arg("stats"),
           py::arg("max_eval_wg") = 512, py::arg("use_graph") = true)
      .def("run", [](LocalSolver& s, int B, int start, uintptr_t stream) { s.run(B, start, S(stream)); })
      .def("run_ingest",
           [](LocalSolver& s, int B, int start, uintptr_t stream, uintptr_t src, uintptr_t ysrc, int64_t first,
              int64_t step, int n, int dst) {
             RingIngest ing{reinterpret_cast<const uint16_t*>(src), reinterpret_cast<const int32_t*>(ysrc), first,
                            step, n, dst};
             s.run(B, start, S(stream), ing);
           })
      // One solve with the optional extras of LocalSolver::run: fused ingest
      // (n > 0), a riding evaluation pass (ride_Xt != 0) and a fused server
      // update (ap_w != 0).
      .def(
          "run_full",
          [](LocalSolver& s, int B, int start, uintptr_t stream, uintptr_t src, uintptr_t ysrc, int64_t first,
             int64_t step, int n, int dst, uintptr_t ride_Xt, uintptr_t ride_yt, int ride_T, uintptr_t whi,
             uintptr_t wlo, uintptr_t wb, int coff1, uintptr_t shi, uintptr_t slo, uintptr_t sb, int coff2,
             uintptr_t acc, uintptr_t ticket, uintptr_t slot, uintptr_t loss, unsigned long long seq, uintptr_t slot2,
             unsigned long long seq2, uintptr_t ap_w, float ap_lr, uintptr_t ap_hi, uintptr_t ap_lo, uintptr_t ap_b,
             int ap_coff) {
            RingIngest ing{};
            if (n > 0)
              ing = RingIngest{reinterpret_cast<const uint16_t*>(src), reinterpret_cast<const int32_t*>(ysrc), first,
                               step, n, dst};
            EvalRide r{};
            if (ride_Xt) {
              r.Xt = P<const uint16_t>(ride_Xt);
              r.yt = P<const int32_t>(ride_yt);
              r.T = ride_T;
              r.K = s.cfg().K;
              r.whi = P<const uint16_t>(whi);
              r.wlo = P<const uint16_t>(wlo);
              r.wb = P<const float>(wb);
              r.shi = P<const uint16_t>(shi);
              r.slo = P<const uint16_t>(slo);
              r.sb = P<const float>(sb);
              r.coff1 = coff1;
              r.coff2 = coff2;
              r.acc = P<int>(acc);
              r.ticket = P<unsigned>(ticket);
              r.slot = P<char>(slot);
              r.loss = P<const float>(loss);
              r.seq = seq;
              r.slot2 = P<char>(slot2);
              r.seq2 = seq2;
              r.nticket = (unsigned)r.ntiles();
              if (r.slot2 && (!r.shi || !r.slo || !r.sb))
                throw std::invalid_argument("run_full: the second model needs its own fragment buffer");
            }
            FusedApply ap{};
            if (ap_w) {
              ap.w = P<float>(ap_w);
              ap.lr = ap_lr;
              ap.hi = P<uint16_t>(ap_hi);
              ap.lo = P<uint16_t>(ap_lo);
              ap.b = P<float>(ap_b);
              ap.coff = ap_coff;
            }
            s.run(B, start, S(stream), ing, ride_Xt ? &r : nullptr, ap_w ? &ap : nullptr);
          },
          py::arg("B"), py::arg("start"), py::arg("stream"), py::arg("src") = 0, py::arg("ysrc") = 0,
          py::arg("first") = 0, py::arg("step") = 1, py::arg("n") = 0, py::arg("dst") = 0, py::arg("ride_Xt") = 0,
          py::arg("ride_yt") = 0, py::arg("ride_T") = 0, py::arg("whi") = 0, py::arg("wlo") = 0, py::arg("wb") = 0,
          py::arg("coff1") = 0, py::arg("shi") = 0, py::arg("slo") = 0, py::arg("sb") = 0, py::arg("coff2") = 0,
          py::arg("acc") = 0, py::arg("ticket") = 0, py::arg("slot") = 0, py::arg("loss") = 0, py::arg("seq") = 0,
          py::arg("slot2") = 0, py::arg("seq2") = 0, py::arg("ap_w") = 0, py::arg("ap_lr") = 1.f,
          py::arg("ap_hi") = 0, py::arg("ap_lo") = 0, py::arg("ap_b") = 0, py::arg("ap_coff") = 0)
      .def_property_readonly("eager", &LocalSolver::eager)
      .def_property_readonly("persistent", &LocalSolver::persistent)
      .def("read_ctrl",
           [](LocalSolver& s, uintptr_t stream) {
             Ctrl c;
             s.read_ctrl(&c, S(stream));
             return ctrl_dict(c, s.cfg().hist);
           })
      .def("read_stamps", [](LocalSolver& s, uintptr_t stream) { return s.read_stamps(S(stream)); })
      .def_property_readonly("eval_wg", &LocalSolver::eval_wg)
      .def_property_readonly("rows_mode", &LocalSolver::rows_mode)
      .def_property_readonly("kernels_per_solve", &LocalSolver::kernels_per_solve);

  m.def(
      "test_eval",
      [](int FP, int K, uintptr_t Xt, uintptr_t yt, int T, uintptr_t whi, uintptr_t wlo, uintptr_t b, uintptr_t conf,
         uintptr_t stream, uintptr_t ticket, uintptr_t slot, uintptr_t loss, unsigned long long seq, int coff1,
         int coff2, uintptr_t slot2, unsigned long long seq2) {
        prepare_kernels();
        if (coff1 < 0 || coff1 + K > 16 || (slot2 && (coff2 < 0 || coff2 + K > 16)))
          throw std::invalid_argument("test_eval: class offset out of range");
        launch_test_eval(FP, K, P<const uint16_t>(Xt), P<const int32_t>(yt), T, P<const uint16_t>(whi),
                         P<const uint16_t>(wlo), P<const float>(b), P<int>(conf), S(stream), P<unsigned>(ticket),
                         P<void>(slot), P<const float>(loss), seq, coff1, coff2, P<void>(slot2), seq2);
        hip_check(hipGetLastError(), "test_eval launch");
      },
      py::arg("FP"), py::arg("K"), py::arg("Xt"), py::arg("yt"), py::arg("T"), py::arg("whi"), py::arg("wlo"),
      py::arg("b"), py::arg("conf"), py::arg("stream"), py::arg("ticket") = 0, py::arg("slot") = 0,
      py::arg("loss") = 0, py::arg("seq") = 0, py::arg("coff1") = 0, py::arg("coff2") = 0, py::arg("slot2") = 0,
      py::arg("seq2") = 0);
  m.def(
      "eval_apply",
      [](int FP, int K, int F, uintptr_t Xt, uintptr_t yt, int T, uintptr_t whi, uintptr_t wlo, uintptr_t wb,
         uintptr_t shi, uintptr_t slo, uintptr_t sb, uintptr_t conf, uintptr_t stream, uintptr_t ticket,
         uintptr_t slot, uintptr_t loss, unsigned long long seq, int coff1, int coff2, uintptr_t slot2,
         unsigned long long seq2, uintptr_t w, std::vector<uintptr_t> deltas, float lr, uintptr_t ohi, uintptr_t olo,
         uintptr_t ob) {
        prepare_kernels();
        if (coff1 < 0 || coff1 + K > coff2 || coff2 + K > 16)
          throw std::invalid_argument("eval_apply: worker columns must precede the server's, within 16");
        if (deltas.size() > 16) throw std::invalid_argument("eval_apply: at most 16 deltas");
        if (!shi || !slo || !sb) throw std::invalid_argument("eval_apply: null server fragments");
        if (!deltas.empty()) {
          if (!w || !ohi || !olo || !ob) throw std::invalid_argument("eval_apply: null update buffer");
          if (shi == ohi || slo == olo || sb == ob || whi == ohi || wlo == olo || wb == ob)
            throw std::invalid_argument("eval_apply: the update would overwrite fragments this launch reads");
        }
        EvalApply ea{};
        ea.shi = P<const uint16_t>(shi);
        ea.slo = P<const uint16_t>(slo);
        ea.sb = P<const float>(sb);
        ea.w = P<float>(w);
        ea.dl.n = (int)deltas.size();
        for (size_t i = 0; i < deltas.size(); ++i) ea.dl.p[i] = P<const float>(deltas[i]);
        ea.lr = lr;
        ea.ohi = P<uint16_t>(ohi);
        ea.olo = P<uint16_t>(olo);
        ea.ob = P<float>(ob);
        ea.F = F;
        launch_eval_apply(FP, K, P<const uint16_t>(Xt), P<const int32_t>(yt), T, P<const uint16_t>(whi),
                          P<const uint16_t>(wlo), P<const float>(wb), P<int>(conf), S(stream), P<unsigned>(ticket),
                          P<void>(slot), P<const float>(loss), seq, coff1, coff2, P<void>(slot2), seq2, ea);
        hip_check(hipGetLastError(), "eval_apply launch");
      },
      py::arg("FP"), py::arg("K"), py::arg("F"), py::arg("Xt"), py::arg("yt"), py::arg("T"), py::arg("whi"),
      py::arg("wlo"), py::arg("wb"), py::arg("shi"), py::arg("slo"), py::arg("sb"), py::arg("conf"),
      py::arg("stream"), py::arg("ticket"), py::arg("slot"), py::arg("loss"), py::arg("seq"), py::arg("coff1"),
      py::arg("coff2"), py::arg("slot2"), py::arg("seq2"), py::arg("w"), py::arg("deltas"), py::arg("lr"),
      py::arg("ohi"), py::arg("olo"), py::arg("ob"));
  // Fine-grained (coherent) pinned host memory: device stores land in host
  // memory without a copy and device loads never see a stale cached line.
  m.def("pinned_alloc", [](size_t bytes) {
    void* p = nullptr;
    hip_check(hipHostMalloc(&p, bytes, hipHostMallocCoherent | hipHostMallocMapped), "hipHostMalloc");
    std::memset(p, 0, bytes);
    return reinterpret_cast<uintptr_t>(p);
  });
  m.def("pinned_free", [](uintptr_t p) {
    if (p) (void)hipHostFree(reinterpret_cast<void*>(p));
  });
  // stream-ordered device -> pinned host copy (the host polls the bytes later,
  // no synchronisation): the BSP stop vote's lagged read
  m.def("memcpy_d2h_async", [](uintptr_t dst, uintptr_t src, size_t bytes, uintptr_t stream) {
    hip_check(hipMemcpyAsync(reinterpret_cast<void*>(dst), reinterpret_cast<const void*>(src), bytes,
                             hipMemcpyDeviceToHost, S(stream)),
              "hipMemcpyAsync(d2h)");
  });
  m.def("logits", [](int FP, int K, uintptr_t X, int T, uintptr_t whi, uintptr_t wlo, uintptr_t b, uintptr_t out,
                     uintptr_t stream) {
    prepare_kernels();
    launch_logits(FP, K, P<const uint16_t>(X), T, P<const uint16_t>(whi), P<const uint16_t>(wlo), P<const float>(b),
                  P<float>(out), S(stream));
    hip_check(hipGetLastError(), "logits launch");
  });
  m.def(
      "server_apply",
      [](int K, int F, int FP, uintptr_t w, uintptr_t delta, float lr, uintptr_t whi, uintptr_t wlo, uintptr_t b,
         uintptr_t stream, int coff) {
        if (coff < 0 || coff + K > 16) throw std::invalid_argument("fragment class offset out of range");
        launch_server_apply(K, F, FP, P<float>(w), P<const float>(delta), lr, P<uint16_t>(whi), P<uint16_t>(wlo),
                            P<float>(b), S(stream), coff);
        hip_check(hipGetLastError(), "server_apply launch");
      },
      py::arg("K"), py::arg("F"), py::arg("FP"), py::arg("w"), py::arg("delta"), py::arg("lr"), py::arg("whi"),
      py::arg("wlo"), py::arg("b"), py::arg("stream"), py::arg("coff") = 0);
  m.def(
      "server_apply_n",
      [](int K, int F, int FP, uintptr_t w, std::vector<uintptr_t> deltas, float lr, uintptr_t whi, uintptr_t wlo,
         uintptr_t b, uintptr_t stream, int coff) {
        if (coff < 0 || coff + K > 16) throw std::invalid_argument("fragment class offset out of range");
        if (deltas.empty() || deltas.size() > 16) throw std::invalid_argument("1..16 deltas per call");
        DeltaList dl{};
        dl.n = (int)deltas.size();
        for (int i = 0; i < dl.n; ++i) dl.p[i] = P<const float>(deltas[i]);
        launch_server_apply_n(K, F, FP, P<float>(w), dl, lr, P<uint16_t>(whi), P<uint16_t>(wlo), P<float>(b),
                              S(stream), coff);
        hip_check(hipGetLastError(), "server_apply_n launch");
      },
      py::arg("K"), py::arg("F"), py::arg("FP"), py::arg("w"), py::arg("deltas"), py::arg("lr"), py::arg("whi"),
      py::arg("wlo"), py::arg("b"), py::arg("stream"), py::arg("coff") = 0);
  m.def(
      "make_fragments",
      [](int K, int F, int FP, uintptr_t w, uintptr_t whi, uintptr_t wlo, uintptr_t b, uintptr_t stream, int coff) {
        if (coff < 0 || coff + K > 16) throw std::invalid_argument("fragment class offset out of range");
        launch_make_fragments(K, F, FP, P<const float>(w), P<uint16_t>(whi), P<uint16_t>(wlo), P<float>(b), S(stream),
                              coff);
        hip_check(hipGetLastError(), "make_fragments launch");
      },
      py::arg("K"), py::arg("F"), py::arg("FP"), py::arg("w"), py::arg("whi"), py::arg("wlo"), py::arg("b"),
      py::arg("stream"), py::arg("coff") = 0);
  // ---- wide / sparse model (BASELINE.json configs 4, 5) ----
  py::class_<WideCfg>(m, "WideCfg", py::module_local())
      .def(py::init([]() {
        WideCfg c{};
        c.sc.iters = 2;
        c.sc.hist = 10;
        c.sc.ls_max = 4;
        c.sc.nslots = 9;
        c.sc.tol = 1e-6f;
        c.sc.gd_lr = 1.f;
        c.K = 2;
        c.KP = 2;
        c.F = 1;
        c.cap = 1;
        c.NZ = 1;
        c.standardize = 1;
        c.center = 1;
        return c;
      }))
      .def_property("iters", [](const WideCfg& c) { return c.sc.iters; }, [](WideCfg& c, int v) { c.sc.iters = v; })
      .def_property("hist", [](const WideCfg& c) { return c.sc.hist; }, [](WideCfg& c, int v) { c.sc.hist = v; })
      .def_property("ls_max", [](const WideCfg& c) { return c.sc.ls_max; }, [](WideCfg& c, int v) { c.sc.ls_max = v; })
      .def_property("mode", [](const WideCfg& c) { return c.sc.mode; }, [](WideCfg& c, int v) { c.sc.mode = v; })
      .def_property("nslots", [](const WideCfg& c) { return c.sc.nslots; }, [](WideCfg& c, int v) { c.sc.nslots = v; })
      .def_property("gd_lr", [](const WideCfg& c) { return c.sc.gd_lr; }, [](WideCfg& c, float v) { c.sc.gd_lr = v; })
      .def_property("tol", [](const WideCfg& c) { return c.sc.tol; }, [](WideCfg& c, float v) { c.sc.tol = v; })
      .def_readwrite("K", &WideCfg::K)
      .def_readwrite("KP", &WideCfg::KP)
      .def_readwrite("F", &WideCfg::F)
      .def_readwrite("cap", &WideCfg::cap)
      .def_readwrite("NZ", &WideCfg::NZ)
      .def_readwrite("standardize", &WideCfg::standardize)
      .def_readwrite("center", &WideCfg::center)
      .def_readwrite("zero_const", &WideCfg::zero_const)
      .def_readwrite("dense_delta", &WideCfg::dense_delta)
      .def_readwrite("pulled", &WideCfg::pulled)
      .def_readwrite("own_W", &WideCfg::own_W)
      .def_readwrite("own_S", &WideCfg::own_S)
      .def_readwrite("persist", &WideCfg::persist);

  // the collective transports (csrc/comm/comm.h): RCCL (one rank per GPU) and
  // IPC (ranks sharing one GPU); the lanes loop takes either
  py::class_<Comm>(m, "Comm")
      .def_property_readonly("rank", &Comm::rank)
      .def_property_readonly("size", &Comm::size)
      .def("all_reduce", [](Comm& c, uintptr_t send, uintptr_t recv, size_t n, int dt, uintptr_t s) {
        c.all_reduce(reinterpret_cast<const void*>(send), reinterpret_cast<void*>(recv), n, dt, S(s));
      })
      .def("reduce", [](Comm& c, uintptr_t send, uintptr_t recv, size_t n, int dt, int root, uintptr_t s) {
        c.reduce(reinterpret_cast<const void*>(send), reinterpret_cast<void*>(recv), n, dt, root, S(s));
      })
      .def("broadcast", [](Comm& c, uintptr_t send, uintptr_t recv, size_t n, int dt, int root, uintptr_t s) {
        c.broadcast(reinterpret_cast<const void*>(send), reinterpret_cast<void*>(recv), n, dt, root, S(s));
      });
  py::class_<IpcComm, Comm>(m, "IpcComm")
      .def(py::init<int, int, int, size_t>(), py::arg("nranks"), py::arg("rank"), py::arg("device"),
           py::arg("max_bytes"))
      .def("handle", [](const IpcComm& c) { return py::bytes(c.handle()); })
      .def("connect",
           [](IpcComm& c, const std::vector<py::bytes>& hs) {
             std::vector<std::string> v;
             for (const auto& h : hs) v.push_back(std::string(h));
             c.connect(v);
           })
      .def_property_readonly("collectives", &IpcComm::collectives)
      .def("close", [](IpcComm& c) {
        py::gil_scoped_release nogil;
        c.close();
      });
  py::class_<RcclComm, Comm>(m, "RcclComm")
      .def_static("unique_id", []() { return py::bytes(RcclComm::unique_id()); })
      .def_static("available", &RcclComm::available)
      .def(py::init([](py::bytes id, int nranks, int rank, int device) {
             std::string sid = id;
             py::gil_scoped_release nogil;  // blocks until every rank has joined
             return std::make_unique<RcclComm>(sid, nranks, rank, device);
           }),
           py::arg("id"), py::arg("nranks"), py::arg("rank"), py::arg("device"))
      .def_property_readonly("rank", &RcclComm::rank)
      .def_property_readonly("size", &RcclComm::size)
      .def("all_reduce", [](RcclComm& c, uintptr_t send, uintptr_t recv, size_t n, int dt, uintptr_t s) {
        c.all_reduce(reinterpret_cast<const void*>(send), reinterpret_cast<void*>(recv), n, dt, S(s));
      })
      .def("reduce", [](RcclComm& c, uintptr_t send, uintptr_t recv, size_t n, int dt, int root, uintptr_t s) {
        c.reduce(reinterpret_cast<const void*>(send), reinterpret_cast<void*>(recv), n, dt, root, S(s));
      })
      .def("broadcast", [](RcclComm& c, uintptr_t send, uintptr_t recv, size_t n, int dt, int root, uintptr_t s) {
        c.broadcast(reinterpret_cast<const void*>(send), reinterpret_cast<void*>(recv), n, dt, root, S(s));
      })
      .def("reduce_scatter", [](RcclComm& c, uintptr_t send, uintptr_t recv, size_t n, int dt, uintptr_t s) {
        c.reduce_scatter(reinterpret_cast<const void*>(send), reinterpret_cast<void*>(recv), n, dt, S(s));
      })
      .def("all_gather", [](RcclComm& c, uintptr_t send, uintptr_t recv, size_t n, int dt, uintptr_t s) {
        c.all_gather(reinterpret_cast<const void*>(send), reinterpret_cast<void*>(recv), n, dt, S(s));
      })
      .def("send", [](RcclComm& c, uintptr_t buf, size_t n, int dt, int peer, uintptr_t s) {
        c.send(reinterpret_cast<const void*>(buf), n, dt, peer, S(s));
      })
      .def("recv", [](RcclComm& c, uintptr_t buf, size_t n, int dt, int peer, uintptr_t s) {
        c.recv(reinterpret_cast<void*>(buf), n, dt, peer, S(s));
      })
      .def_property_readonly("side_stream", [](RcclComm& c) { return reinterpret_cast<uintptr_t>(c.side_stream()); })
      .def("fork", [](RcclComm& c, uintptr_t s) { c.fork(S(s)); })
      .def("join", [](RcclComm& c, uintptr_t s) { c.join(S(s)); })
      .def("group_start", &RcclComm::group_start)
      .def("group_end", &RcclComm::group_end)
      .def("close", [](RcclComm& c) {
        py::gil_scoped_release nogil;
        c.close();
      })
      .def("abort", &RcclComm::abort);

  py::class_<WideSolver>(m, "WideSolver")
      .def(py::init([](const WideCfg& cfg, uintptr_t ridx, uintptr_t rval, uintptr_t rnnz, uintptr_t ry,
                       uintptr_t w_old, uintptr_t dloc, uintptr_t wloc, uintptr_t loss, uintptr_t stats,
                       uintptr_t uniq, uintptr_t delta_dense, bool use_graph, uintptr_t w_pull, uintptr_t w_pull_b) {
             WideBuffers b;
             b.w_pull = P<const float>(w_pull);
             b.w_pull_b = P<const float>(w_pull_b);
             b.uniq = P<int32_t>(uniq);
             b.ridx = P<const int32_t>(ridx);
             b.rval = P<const uint16_t>(rval);
             b.rnnz = P<const int32_t>(rnnz);
             b.ry = P<const int32_t>(ry);
             b.w_old = P<const float>(w_old);
             b.dloc = P<float>(dloc);
             b.wloc = P<float>(wloc);
             b.loss = P<float>(loss);
             b.stats = P<int>(stats);
             b.delta_dense = P<float>(delta_dense);
             return std::make_unique<WideSolver>(cfg, b, use_graph);
           }),
           py::arg("cfg"), py::arg("ridx"), py::arg("rval"), py::arg("rnnz"), py::arg("ry"), py::arg("w_old"),
           py::arg("dloc"), py::arg("wloc"), py::arg("loss"), py::arg("stats"), py::arg("uniq"), py::arg("delta_dense") = 0,
           py::arg("use_graph") = true, py::arg("w_pull") = 0, py::arg("w_pull_b") = 0)
      .def("run", [](WideSolver& s, int B, int start, uintptr_t stream) { s.run(B, start, S(stream)); })
      .def("plan", [](WideSolver& s, int B, int start, uintptr_t stream) { s.plan(B, start, S(stream)); })
      .def("finish", [](WideSolver& s, uintptr_t stream) { s.finish(S(stream)); })
      .def_property_readonly("owner_counts_ptr",
                             [](const WideSolver& s) { return reinterpret_cast<uintptr_t>(s.owner_counts_dev()); })
      // (tests) U of the last plan and the per-owner counts, read after a sync
      .def("read_plan",
           [](const WideSolver& s, uintptr_t stream) {
             std::vector<unsigned> v(1 + kMaxOwners);
             hip_check(hipMemcpyAsync(v.data(), s.ucount_dev(), 4, hipMemcpyDeviceToHost, S(stream)), "read U");
             hip_check(hipMemcpyAsync(v.data() + 1, s.owner_counts_dev(), kMaxOwners * 4, hipMemcpyDeviceToHost,
                                      S(stream)),
                       "read owner counts");
             hip_check(hipStreamSynchronize(S(stream)), "sync");
             return v;
           })
      .def("read_ctrl",
           [](WideSolver& s, uintptr_t stream) {
             Ctrl c;
             s.read_ctrl(&c, S(stream));
             return ctrl_dict(c, s.cfg().sc.hist);
           })
      .def("read_stamps", [](WideSolver& s, uintptr_t stream) { return s.read_stamps(S(stream)); })
      .def_property_readonly("plmax", &WideSolver::plmax)
      .def_property_readonly("umax", [](const WideSolver& s) { return s.cfg().umax; })
      .def_property_readonly("table_ptr", [](const WideSolver& s) { return reinterpret_cast<uintptr_t>(s.table()); })
      .def_property_readonly("table_mask", &WideSolver::table_mask)
      .def_property_readonly("uniq_ptr", [](const WideSolver& s) { return reinterpret_cast<uintptr_t>(s.uniq()); })
      .def_property_readonly("ucount_ptr",
                             [](const WideSolver& s) { return reinterpret_cast<uintptr_t>(s.ucount_dev()); })
      .def_property_readonly("ucount_host", &WideSolver::ucount_host)
      .def_property_readonly("workspace_bytes", &WideSolver::workspace_bytes)
      .def_property_readonly("kernels_per_solve", &WideSolver::kernels_per_solve);

  py::class_<WideLanes>(m, "WideLanes")
      .def(py::init([](py::list solvers, int xcd0) {
             std::vector<WideSolver*> v;
             for (auto o : solvers) v.push_back(o.cast<WideSolver*>());
             return std::make_unique<WideLanes>(v, xcd0);
           }),
           py::arg("solvers"), py::arg("xcd0") = 0, py::keep_alive<1, 2>())
      .def("run",
           [](WideLanes& s, const std::vector<int>& B, const std::vector<int>& start, uintptr_t stream) {
             s.run(B, start, S(stream));
           })
      .def("eval",
           [](WideLanes& s, uintptr_t indptr, uintptr_t idx, uintptr_t val, uintptr_t y, int T, uintptr_t w, int nov,
              const std::vector<uintptr_t>& slots, const std::vector<unsigned long long>& seqs, uintptr_t server_slot,
              unsigned long long server_seq, uintptr_t stream) {
             s.eval(P<const int64_t>(indptr), P<const int32_t>(idx), P<const uint16_t>(val), P<const int32_t>(y), T,
                    P<const float>(w), nov, slots, seqs, server_slot, server_seq, S(stream));
           })
      .def("apply",
           [](WideLanes& s, uintptr_t w, float lr, const std::vector<int>& order, uintptr_t stream) {
             s.apply(P<float>(w), lr, order, S(stream));
           })
      .def_property_readonly("lanes", &WideLanes::lanes)
      .def_property_readonly("launches", &WideLanes::launches);

  // jobs: (src_first, src_step, n, dst_first, ridx, rval, rnnz, ry, trunc) per ring
  m.def("sparse_ring_ingest_many", [](uintptr_t indptr, uintptr_t idx, uintptr_t val, uintptr_t y,
                                      const std::vector<std::vector<int64_t>>& jobs, int cap, int NZ,
                                      uintptr_t stream) {
    SparseIngestJobs a{};
    if (jobs.size() > (size_t)kMaxIngestJobs) throw std::invalid_argument("sparse_ring_ingest_many: <= 16 jobs");
    a.njobs = (int)jobs.size();
    a.cap = cap;
    a.NZ = NZ;
    for (size_t q = 0; q < jobs.size(); ++q) {
      const auto& v = jobs[q];
      if (v.size() != 9) throw std::invalid_argument("sparse_ring_ingest_many: 9 fields per job");
      a.job[q] = SparseIngestJob{v[0], v[1], v[2], v[3], P<int32_t>((uintptr_t)v[4]), P<uint16_t>((uintptr_t)v[5]),
                                 P<int32_t>((uintptr_t)v[6]), P<int32_t>((uintptr_t)v[7]), P<int>((uintptr_t)v[8])};
    }
    launch_sparse_ring_ingest_many(P<const int64_t>(indptr), P<const int32_t>(idx), P<const uint16_t>(val),
                                   P<const int32_t>(y), a, S(stream));
    hip_check(hipGetLastError(), "sparse_ring_ingest_many launch");
  });
  m.def("sparse_ring_ingest", [](uintptr_t indptr, uintptr_t idx, uintptr_t val, uintptr_t y, int64_t src_first,
                                 int64_t src_step, int64_t n, uintptr_t ridx, uintptr_t rval, uintptr_t rnnz,
                                 uintptr_t ry, int64_t dst_first, int cap, int NZ, uintptr_t trunc, uintptr_t stream) {
    launch_sparse_ring_ingest(P<const int64_t>(indptr), P<const int32_t>(idx), P<const uint16_t>(val),
                              P<const int32_t>(y), src_first, src_step, n, P<int32_t>(ridx), P<uint16_t>(rval),
                              P<int32_t>(rnnz), P<int32_t>(ry), dst_first, cap, NZ, P<int>(trunc), S(stream));
    hip_check(hipGetLastError(), "sparse_ring_ingest launch");
  });
  m.def(
      "wide_eval",
      [](int K, int KP, int64_t F, uintptr_t indptr, uintptr_t idx, uintptr_t val, uintptr_t y, int T, uintptr_t w,
         uintptr_t table, unsigned mask, uintptr_t wloc, uintptr_t acc, uintptr_t ticket, uintptr_t slot,
         uintptr_t loss, unsigned long long seq, uintptr_t stream, uintptr_t slot2, unsigned long long seq2,
         uintptr_t zbase, uintptr_t bias) {
        if (slot2 && (!slot || !table || !wloc || !w))
          throw std::invalid_argument("wide_eval: the paired row needs a slot, the dense model and the overlay");
        if (!w && !zbase) throw std::invalid_argument("wide_eval: need the model or the margins base");
        if (!w && !bias && !table) throw std::invalid_argument("wide_eval: key-range form needs the intercepts");
        if (table && !wloc) throw std::invalid_argument("wide_eval: overlay table without values");
        launch_wide_eval(K, KP, F, P<const int64_t>(indptr), P<const int32_t>(idx), P<const uint16_t>(val),
                         P<const int32_t>(y), T, P<const float>(w), P<const int2>(table), mask, P<const float>(wloc),
                         P<int>(acc), P<unsigned>(ticket), P<void>(slot), P<const float>(loss), seq, S(stream),
                         P<void>(slot2), seq2, P<const float>(zbase), P<const float>(bias));
        hip_check(hipGetLastError(), "wide_eval launch");
      },
      py::arg("K"), py::arg("KP"), py::arg("F"), py::arg("indptr"), py::arg("idx"), py::arg("val"), py::arg("y"),
      py::arg("T"), py::arg("w"), py::arg("table"), py::arg("mask"), py::arg("wloc"), py::arg("acc"),
      py::arg("ticket") = 0, py::arg("slot") = 0, py::arg("loss") = 0, py::arg("seq") = 0, py::arg("stream") = 0,
      py::arg("slot2") = 0, py::arg("seq2") = 0, py::arg("zbase") = 0, py::arg("bias") = 0);
  m.def("wide_logits", [](int K, int KP, int64_t F, uintptr_t indptr, uintptr_t idx, uintptr_t val, int T,
                          uintptr_t w, uintptr_t out, uintptr_t stream) {
    launch_wide_logits(K, KP, F, P<const int64_t>(indptr), P<const int32_t>(idx), P<const uint16_t>(val), T,
                       P<const float>(w), P<float>(out), S(stream));
    hip_check(hipGetLastError(), "wide_logits launch");
  });
  m.def("wide_apply_sparse", [](uintptr_t w, int64_t F, int KP, uintptr_t U_dev, int U_host, uintptr_t uniq,
                                uintptr_t dloc, float lr, int umax, uintptr_t stream) {
    launch_wide_apply_sparse(P<float>(w), F, KP, P<const unsigned>(U_dev), U_host, P<const int32_t>(uniq),
                             P<const float>(dloc), lr, umax, S(stream));
    hip_check(hipGetLastError(), "wide_apply_sparse launch");
  });
  m.def("log_append", [](uintptr_t uniq, uintptr_t dloc, int U, int64_t F, int KP, uintptr_t lids, uintptr_t lvals,
                         int64_t pos, int64_t cap, uintptr_t stream) {
    launch_log_append(P<const int32_t>(uniq), P<const float>(dloc), U, F, KP, P<int32_t>(lids), P<float>(lvals), pos,
                      cap, S(stream));
    hip_check(hipGetLastError(), "log_append launch");
  });
  m.def("log_apply", [](uintptr_t w, uintptr_t ids, uintptr_t vals, int64_t n, int KP, float lr, uintptr_t stream) {
    launch_log_apply(P<float>(w), P<const int32_t>(ids), P<const float>(vals), n, KP, lr, S(stream));
    hip_check(hipGetLastError(), "log_apply launch");
  });
  m.def("axpy", [](uintptr_t w, uintptr_t x, float a, int64_t n, uintptr_t stream) {
    launch_axpy(P<float>(w), P<const float>(x), a, n, S(stream));
    hip_check(hipGetLastError(), "axpy launch");
  });

  // Native SSP/ASP server loop (csrc/runtime/async_server.h).  `cfg`: a dict of
  // ints / floats; pointers are device addresses (torch data_ptr) or host-runtime
  // handles (VectorClockTracker.handle, CtrlQueue.handle, MetricsSink.handle,
  // _psx_host.capi()).
  py::class_<P2P>(m, "P2P");
  py::class_<RcclP2P, P2P>(m, "RcclP2P").def(py::init<RcclComm*>(), py::arg("comm"), py::keep_alive<1, 2>());
  py::class_<LocalP2P, P2P>(m, "LocalP2P")
      .def(py::init<int, const std::vector<uintptr_t>&, const std::vector<uintptr_t>&, const std::vector<uintptr_t>&>(),
           py::arg("nworkers"), py::arg("out_f32"), py::arg("out_i32"), py::arg("inbox"))
      .def("released", &LocalP2P::released);
  py::class_<HostP2P, P2P>(m, "HostP2P")
      .def(py::init<const std::string&, int, int, bool, bool, size_t, double>(), py::arg("name"), py::arg("nworkers"),
           py::arg("rank"), py::arg("create"), py::arg("device") = false, py::arg("cap_bytes") = (size_t)8 << 20,
           py::arg("timeout_s") = 600.0)
      .def("send",
           [](HostP2P& p, uintptr_t buf, size_t n, int dt, int peer, uintptr_t s) {
             py::gil_scoped_release nogil;
             p.send(reinterpret_cast<const void*>(buf), n, dt, peer, S(s));
           })
      .def("recv",
           [](HostP2P& p, uintptr_t buf, size_t n, int dt, int peer, uintptr_t s) {
             py::gil_scoped_release nogil;
             p.recv(reinterpret_cast<void*>(buf), n, dt, peer, S(s));
           })
      .def("unlink", &HostP2P::unlink);
  py::class_<LocalFeeder>(m, "LocalFeeder")
      .def(py::init<uintptr_t, uintptr_t, LocalP2P*, int, int64_t, int64_t, double, const std::vector<int64_t>&,
                    const std::vector<uintptr_t>&>(),
           py::arg("api"), py::arg("ctrl"), py::arg("p2p"), py::arg("nworkers"), py::arg("iters"),
           py::arg("token_n") = 0, py::arg("timeout_s") = 60.0, py::arg("vc0") = std::vector<int64_t>{},
           py::arg("replies") = std::vector<uintptr_t>{}, py::keep_alive<1, 4>())
      .def_property_readonly("sparse_pulls", &LocalFeeder::sparse_pulls)
      .def("start", &LocalFeeder::start)
      .def("join", &LocalFeeder::join, py::call_guard<py::gil_scoped_release>());
  // Peer data plane (csrc/comm/peer_bus.h): IPC-exported fine-grained regions
  py::class_<PeerRegion>(m, "PeerRegion")
      .def(py::init([](int64_t P, int NS, int slots, int device) {
             PeerLayout lay;
             lay.P = P;
             lay.NS = NS;
             lay.slots = slots;
             return std::make_unique<PeerRegion>(lay, device);
           }),
           py::arg("P"), py::arg("NS"), py::arg("slots"), py::arg("device") = 0)
      .def("handle", [](const PeerRegion& r) { return py::bytes(r.handle()); })
      .def("fill_tags", &PeerRegion::fill_tags, py::arg("value"))
      .def_property_readonly("base", &PeerRegion::base)
      .def_property_readonly("stride", [](const PeerRegion& r) { return r.layout().stride(); })
      .def_property_readonly("nbytes", [](const PeerRegion& r) { return r.layout().bytes(); })
      .def("data", [](const PeerRegion& r, int slot) { return reinterpret_cast<uintptr_t>(r.data(slot)); })
      .def("tags", [](const PeerRegion& r, int slot) { return reinterpret_cast<uintptr_t>(r.tags(slot)); });
  py::class_<PeerMapping>(m, "PeerMapping")
      .def(py::init([](py::bytes h, int64_t P, int NS, int slots) {
             PeerLayout lay;
             lay.P = P;
             lay.NS = NS;
             lay.slots = slots;
             return std::make_unique<PeerMapping>(std::string(h), lay);
           }),
           py::arg("handle"), py::arg("P"), py::arg("NS"), py::arg("slots"))
      .def_property_readonly("base", &PeerMapping::base)
      .def("data", [](const PeerMapping& r, int slot) { return reinterpret_cast<uintptr_t>(r.data(slot)); })
      .def("tags", [](const PeerMapping& r, int slot) { return reinterpret_cast<uintptr_t>(r.tags(slot)); })
      .def("close", &PeerMapping::close);
  py::class_<PeerServer>(m, "PeerServer")
      .def(py::init([](py::dict d) {
             auto I = [&](const char* k, int64_t def) { return d.contains(k) ? d[k].cast<int64_t>() : def; };
             auto U = [&](const char* k) { return d.contains(k) ? d[k].cast<uintptr_t>() : (uintptr_t)0; };
             auto V = [&](const char* k) {
               return d.contains(k) ? d[k].cast<std::vector<uintptr_t>>() : std::vector<uintptr_t>{};
             };
             PeerServerCfg c;
             c.nworkers = (int)I("nworkers", 0);
             c.lr = d.contains("lr") ? d["lr"].cast<float>() : 1.f;
             c.K = (int)I("K", 0);
             c.F = (int)I("F", 0);
             c.FP = (int)I("FP", 0);
             c.P = I("P", 0);
             c.w = P<float>(U("w"));
             c.Xt = P<const uint16_t>(U("Xt"));
             c.yt = P<const int32_t>(U("yt"));
             c.T = (int)I("T", 0);
             c.inbox = U("inbox");
             c.lay.P = c.P;
             c.lay.NS = c.FP / 32;
             c.lay.slots = (int)I("inbox_slots", c.nworkers);
             c.rx = V("rx");
             c.rx_tag = V("rx_tag");
             c.api = U("api");
             c.tracker = U("tracker");
             c.ctrl = U("ctrl");
             c.sink = U("sink");
             c.replies = V("replies");
             c.worker_timeout_s = d.contains("worker_timeout_s") ? d["worker_timeout_s"].cast<double>() : 600.0;
             c.sxcd = (int)I("sxcd", 0);
             c.bsp = I("bsp", 0) != 0;
             c.nwg = (int)I("nwg", kSrvWg);
             c.batch = (int)I("batch", 64);
             c.standin = I("standin", 0) != 0;
             c.ahead = (int)I("ahead", 0);
             c.tag_wait_s = d.contains("tag_wait_s") ? d["tag_wait_s"].cast<double>() : 600.0;
             prepare_kernels();
             return std::make_unique<PeerServer>(c, nullptr);
           }),
           py::arg("cfg"))
      .def("begin", &PeerServer::begin, py::call_guard<py::gil_scoped_release>())
      .def(
          "run",
          [](PeerServer& s, int64_t checkpoint_every) {
            AsyncStatus st;
            {
              py::gil_scoped_release nogil;
              st = s.run(checkpoint_every);
            }
            return py::make_tuple(st.code, st.worker, st.updates);
          },
          py::arg("checkpoint_every") = 0)
      .def("run_bsp", &PeerServer::run_bsp, py::arg("rounds"), py::arg("r0"), py::call_guard<py::gil_scoped_release>())
      .def("run_bsp_async", &PeerServer::run_bsp_async, py::arg("rounds"), py::arg("r0"))
      .def("run_bsp_join", &PeerServer::run_bsp_join, py::call_guard<py::gil_scoped_release>())
      .def("seed_rx", &PeerServer::seed_rx, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("bsp_rounds", &PeerServer::bsp_rounds)
      .def("set_trace", &PeerServer::set_trace, py::arg("cap"))
      .def("bench_async", &PeerServer::bench_async, py::arg("deltas"), py::arg("log_every") = 0,
           py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("deltas_per_command", &PeerServer::deltas_per_command)
      .def("trace_take", &PeerServer::trace_take)
      .def_property_readonly("host_us_per_round", &PeerServer::host_us_per_round)
      .def("fail", &PeerServer::fail, py::call_guard<py::gil_scoped_release>())
      .def("stop", &PeerServer::stop, py::call_guard<py::gil_scoped_release>())
      .def("warm_up", &PeerServer::warm_up, py::call_guard<py::gil_scoped_release>())
      .def("set_stream", [](PeerServer&, uintptr_t) {})  // (own stream; AsyncServer's interface)
      .def_property("updates", &PeerServer::updates, &PeerServer::set_updates)
      .def_property_readonly("tokens", &PeerServer::tokens)
      .def_property_readonly("commands", &PeerServer::commands)
      .def_property_readonly("running", &PeerServer::running)
      .def_property_readonly("arrivals", &PeerServer::arrivals)
      .def_property_readonly("host_us_per_update", &PeerServer::host_us_per_update)
      .def_property_readonly("failed", &PeerServer::failed)
      .def_property_readonly("sparse_pulls", [](const PeerServer&) { return (int64_t)0; })
      .def_property_readonly("dense_pulls", &PeerServer::tokens);
  py::class_<AsyncServer>(m, "AsyncServer")
      .def(py::init([](P2P& comm, py::dict d, uintptr_t stream) {
             auto I = [&](const char* k, int64_t def) {
               return d.contains(k) ? d[k].cast<int64_t>() : def;
             };
             auto U = [&](const char* k) { return d.contains(k) ? d[k].cast<uintptr_t>() : (uintptr_t)0; };
             AsyncServerCfg c;
             c.nworkers = (int)I("nworkers", 0);
             c.model = (int)I("model", kAsyncDense);
             c.lr = d.contains("lr") ? d["lr"].cast<float>() : 1.f;
             c.P = I("P", 0);
             c.w = P<float>(U("w"));
             c.buf = P<float>(U("buf"));
             c.K = (int)I("K", 0);
             c.F = (int)I("F", 0);
             c.FP = (int)I("FP", 0);
             c.coff = (int)I("coff", 0);
             c.fhi = P<uint16_t>(U("fhi"));
             c.flo = P<uint16_t>(U("flo"));
             c.fb = P<float>(U("fb"));
             c.Xt = P<const uint16_t>(U("Xt"));
             c.yt = P<const int32_t>(U("yt"));
             c.T = (int)I("T", 0);
             c.KP = (int)I("KP", 0);
             c.Fw = I("Fw", 0);
             c.umax = (int)I("umax", 0);
             c.ubuf = P<int32_t>(U("ubuf"));
             c.dbuf = P<float>(U("dbuf"));
             c.t_indptr = P<const int64_t>(U("t_indptr"));
             c.t_idx = P<const int32_t>(U("t_idx"));
             c.t_val = P<const uint16_t>(U("t_val"));
             c.t_y = P<const int32_t>(U("t_y"));
             c.acc = P<int>(U("acc"));
             c.ticket = P<unsigned>(U("ticket"));
             c.api = U("api");
             c.tracker = U("tracker");
             c.ctrl = U("ctrl");
             c.sink = U("sink");
             c.worker_timeout_s = d.contains("worker_timeout_s") ? d["worker_timeout_s"].cast<double>() : 600.0;
             c.sparse_pull = (int)I("sparse_pull", 0);
             c.lids = P<int32_t>(U("lids"));
             c.lvals = P<float>(U("lvals"));
             c.logcap = I("logcap", 0);
             c.dense_every = (int)I("dense_every", 64);
             c.cpu = (int)I("cpu", 0);
             if (d.contains("replies")) c.replies = d["replies"].cast<std::vector<uintptr_t>>();
             if (d.contains("peer")) c.peer = d["peer"].cast<std::vector<int>>();
             if (!c.cpu && (c.model == kAsyncDense || c.sink)) prepare_kernels();
             return std::make_unique<AsyncServer>(&comm, c, S(stream));
           }),
           py::arg("p2p"), py::arg("cfg"), py::arg("stream"), py::keep_alive<1, 2>())
      .def("begin", &AsyncServer::begin)
      .def(
          "run",
          [](AsyncServer& s, int64_t checkpoint_every) {
            AsyncStatus st;
            {
              py::gil_scoped_release nogil;
              st = s.run(checkpoint_every);
            }
            return py::make_tuple(st.code, st.worker, st.updates);
          },
          py::arg("checkpoint_every") = 0)
      .def("fail", &AsyncServer::fail)
      .def("set_stream", [](AsyncServer& s, uintptr_t st) { s.set_stream(S(st)); })
      .def_property("updates", &AsyncServer::updates, &AsyncServer::set_updates)
      .def_property_readonly("tokens", &AsyncServer::tokens)
      .def_property_readonly("host_us_per_update", &AsyncServer::host_us_per_update)
      .def_property_readonly("failed", &AsyncServer::failed)
      .def_property_readonly("sparse_pulls", &AsyncServer::sparse_pulls)
      .def_property_readonly("dense_pulls", &AsyncServer::dense_pulls)
      .def_property_readonly("pull_floats", &AsyncServer::pull_floats);
  py::class_<BspLoop>(m, "BspLoop")
      .def(py::init([](LocalSolver& solver, RcclComm* comm, py::dict d) {
             auto I = [&](const char* k, int64_t def) { return d.contains(k) ? d[k].cast<int64_t>() : def; };
             auto U = [&](const char* k) { return d.contains(k) ? d[k].cast<uintptr_t>() : (uintptr_t)0; };
             auto D = [&](const char* k, double def) { return d.contains(k) ? d[k].cast<double>() : def; };
             BspLoopCfg c;
             c.dsX = P<const uint16_t>(U("dsX"));
             c.dsy = P<const int32_t>(U("dsy"));
             c.ds_rows = I("ds_rows", 0);
             c.k = (int)I("k", 0);
             c.N = (int)I("N", 1);
             c.per_iter_rows = (int)I("per_iter_rows", 0);
             c.p_ms = D("p_ms", 0.0);
             c.epochs = I("epochs", 1);
             c.t0_ms = D("t0_ms", 0.0);
             c.X = P<uint16_t>(U("X"));
             c.XT = P<uint16_t>(U("XT"));
             c.y = P<int32_t>(U("y"));
             c.cap = I("cap", 0);
             c.Fp = (int)I("Fp", 0);
             c.K = (int)I("K", 0);
             c.F = (int)I("F", 0);
             c.window = U("window");
             c.whi = P<const uint16_t>(U("whi"));
             c.wlo = P<const uint16_t>(U("wlo"));
             c.wb = P<const float>(U("wb"));
             c.loss = P<const float>(U("loss"));
             c.delta = P<float>(U("delta"));
             c.w = P<float>(U("w"));
             c.shi = P<uint16_t>(U("shi"));
             c.slo = P<uint16_t>(U("slo"));
             c.sb = P<float>(U("sb"));
             c.scoff = (int)I("scoff", 0);
             c.lr = (float)D("lr", 1.0);
             c.tracker = U("tracker");
             c.Xt = P<const uint16_t>(U("Xt"));
             c.yt = P<const int32_t>(U("yt"));
             c.T = (int)I("T", 0);
             c.acc = P<int>(U("acc"));
             c.ticket = P<unsigned>(U("ticket"));
             c.sink = U("sink");
             c.log_server = I("log_server", 1) != 0;
             c.api = U("api");
             prepare_kernels();
             return std::make_unique<BspLoop>(&solver, comm, c);
           }),
           py::arg("solver"), py::arg("comm"), py::arg("cfg"), py::keep_alive<1, 2>(), py::keep_alive<1, 3>())
      .def(
          "run",
          [](BspLoop& b, int64_t rounds, int64_t r0, uintptr_t stream) {
            py::gil_scoped_release nogil;
            return b.run(rounds, r0, S(stream));
          },
          py::arg("rounds"), py::arg("r0"), py::arg("stream"))
      .def("flush", [](BspLoop& b, uintptr_t stream) { b.flush(S(stream)); })
      .def_property("next_local", &BspLoop::next_local, &BspLoop::set_next_local)
      .def_property_readonly("exhausted", &BspLoop::exhausted)
      .def_property_readonly("host_us_per_round", &BspLoop::host_us_per_round);
  // Multi-lane BSP round loop (csrc/runtime/lanes_loop.h): `cfg` dict of ints /
  // floats / lists; pointers are device addresses or host-runtime handles.
  py::class_<LanesLoop>(m, "LanesLoop")
      .def(py::init([](py::dict d, Comm* comm) {
             auto I = [&](const char* k, int64_t def) { return d.contains(k) ? d[k].cast<int64_t>() : def; };
             auto U = [&](const char* k) { return d.contains(k) ? d[k].cast<uintptr_t>() : (uintptr_t)0; };
             auto D = [&](const char* k, double def) { return d.contains(k) ? d[k].cast<double>() : def; };
             auto V = [&](const char* k) {
               return d.contains(k) ? d[k].cast<std::vector<uintptr_t>>() : std::vector<uintptr_t>{};
             };
             LanesLoopCfg c;
             c.scfg = d["scfg"].cast<SolverCfg>();
             c.dsX = P<const uint16_t>(U("dsX"));
             c.dsy = P<const int32_t>(U("dsy"));
             c.ds_rows = I("ds_rows", 0);
             c.N = (int)I("N", 1);
             c.per_iter_rows = (int)I("per_iter_rows", 0);
             c.p_ms = D("p_ms", 0.0);
             c.epochs = I("epochs", 1);
             c.t0_ms = D("t0_ms", 0.0);
             c.k = d.contains("k") ? d["k"].cast<std::vector<int>>() : std::vector<int>{};
             c.L = (int)c.k.size();
             c.X = V("X");
             c.XT = V("XT");
             c.y = V("y");
             c.window = V("window");
             c.w = P<float>(U("w"));
             c.lr = (float)D("lr", 1.0);
             const auto shi = V("shi"), slo = V("slo"), sb = V("sb");
             for (int i = 0; i < kLaneBufs; ++i) {
               c.shi[i] = i < (int)shi.size() ? P<uint16_t>(shi[i]) : nullptr;
               c.slo[i] = i < (int)slo.size() ? P<uint16_t>(slo[i]) : nullptr;
               c.sb[i] = i < (int)sb.size() ? P<float>(sb[i]) : nullptr;
             }
             c.scoff = (int)I("scoff", 0);
             c.Xt = P<const uint16_t>(U("Xt"));
             c.yt = P<const int32_t>(U("yt"));
             c.T = (int)I("T", 0);
             c.Ti = P<const uint16_t>(U("Ti"));
             c.Tv = P<const uint16_t>(U("Tv"));
             c.tnz = (int)I("tnz", 0);
             c.sink = U("sink");
             c.log_server = I("log_server", 1) != 0;
             c.log_workers = I("log_workers", 1) != 0;
             c.tracker = U("tracker");
             c.api = U("api");
             c.server_rank = (int)I("server_rank", 0);
             c.allreduce = I("allreduce", 0) != 0;
             c.new_rows = (int)I("new_rows", 0);
             c.new_frac = D("new_frac", 0.0);
             c.new_cap = (int)I("new_cap", 0);
             c.new_ramp = (int)I("new_ramp", 0);
             c.log_worker = (int)I("log_worker", 0);
             c.delay_us = d.contains("delay_us") ? d["delay_us"].cast<std::vector<int>>() : std::vector<int>{};
             c.xcd0 = (int)I("xcd0", 0);
             return std::make_unique<LanesLoop>(c, comm);
           }),
           py::arg("cfg"), py::arg("comm") = nullptr, py::keep_alive<1, 3>())
      .def(
          "run",
          [](LanesLoop& l, int64_t rounds, int64_t r0, uintptr_t stream, double max_wait_s, double deadline_ms) {
            py::gil_scoped_release nogil;
            return l.run(rounds, r0, S(stream), max_wait_s, deadline_ms);
          },
          py::arg("rounds"), py::arg("r0"), py::arg("stream"), py::arg("max_wait_s") = 600.0,
          py::arg("deadline_ms") = 0.0)
      .def(
          "run_async",
          // per_lane: an int (the same bound for every lane, 0 = none) or one bound per lane
          [](LanesLoop& l, int64_t updates, uintptr_t stream, double max_wait_s, double deadline_ms,
             py::object per_lane) {
            std::vector<int64_t> b;
            if (py::isinstance<py::int_>(per_lane)) {
              const int64_t v = per_lane.cast<int64_t>();
              if (v > 0) b.assign((size_t)l.lanes(), v);
            } else if (!per_lane.is_none()) {
              b = per_lane.cast<std::vector<int64_t>>();
            }
            py::gil_scoped_release nogil;
            return l.run_async(updates, S(stream), max_wait_s, deadline_ms, b);
          },
          py::arg("updates"), py::arg("stream"), py::arg("max_wait_s") = 600.0, py::arg("deadline_ms") = 0.0,
          py::arg("per_lane") = 0)
      .def("set_peer", &LanesLoop::set_peer, py::arg("rx_data"), py::arg("rx_tags"), py::arg("rx_stride"),
           py::arg("inbox"), py::arg("inbox_tag"))
      .def("prepare_async", &LanesLoop::prepare_async)
      .def("set_peer_sum", &LanesLoop::set_peer_sum, py::arg("rx"), py::arg("rx_tag"), py::arg("push"),
           py::arg("push_tag"), py::arg("wait_s"))
      .def_property_readonly("peer_sum", &LanesLoop::peer_sum)
      .def("peer_sum_tags", &LanesLoop::peer_sum_tags)
      .def("set_xcd_skip", &LanesLoop::set_xcd_skip, py::arg("mask"))
      .def("set_async_debug", &LanesLoop::set_async_debug, py::arg("buf"), py::arg("cap"))
      .def("set_injection", &LanesLoop::set_injection, py::arg("crash"), py::arg("stop"), py::arg("drop"))
      .def("set_trace", &LanesLoop::set_trace, py::arg("cap"))
      .def("trace_take", [](LanesLoop& lp, uintptr_t s) { return lp.trace_take(reinterpret_cast<hipStream_t>(s)); },
           py::arg("stream"))
      .def("clock_ref", [](LanesLoop& lp, uintptr_t s) { return lp.clock_ref(reinterpret_cast<hipStream_t>(s)); },
           py::arg("stream"))
      .def_property_readonly("crashed", &LanesLoop::crashed)
      .def_property_readonly("left", &LanesLoop::left)
      .def_property_readonly("async_log", &LanesLoop::async_log)
      .def_property_readonly("peer", &LanesLoop::peer)
      .def(
          "run_async_remote",
          [](LanesLoop& l, P2P* p2p, uintptr_t ctrl, uintptr_t reply, int64_t iters, uintptr_t stream,
             uintptr_t comm_stream, double max_wait_s, double deadline_ms) {
            py::gil_scoped_release nogil;
            return l.run_async_remote(p2p, ctrl, reply, iters, S(stream), S(comm_stream), max_wait_s, deadline_ms);
          },
          py::arg("p2p"), py::arg("ctrl"), py::arg("reply"), py::arg("iters"), py::arg("stream"),
          py::arg("comm_stream"), py::arg("max_wait_s") = 600.0, py::arg("deadline_ms") = 0.0)
      .def_property_readonly("tickets", &LanesLoop::tickets)
      .def_property_readonly("host_us_per_update", &LanesLoop::host_us_per_update)
      .def_property_readonly("host_busy_us_per_token", &LanesLoop::host_busy_us_per_token)
      .def("seen_at_solve", &LanesLoop::seen_at_solve)
      .def("set_seen_at_solve", &LanesLoop::set_seen_at_solve)
      .def("new_tuples_needed", &LanesLoop::new_tuples_needed, py::arg("size"), py::arg("updates") = -1)
      .def("flush", [](LanesLoop& l, uintptr_t stream) { l.flush(S(stream)); })
      .def("set_sink", &LanesLoop::set_sink)
      .def("set_idle_wait", &LanesLoop::set_idle_wait)
      .def("set_lr", &LanesLoop::set_lr)
      .def("next_local", &LanesLoop::next_local)
      .def("set_next_local", &LanesLoop::set_next_local)
      .def("exhausted", &LanesLoop::exhausted)
      .def_property_readonly("all_exhausted", &LanesLoop::all_exhausted)
      .def_property_readonly("hand_off_scope", &LanesLoop::hand_off_scope)
      .def_property_readonly("side_eval", &LanesLoop::side_eval)
      .def_property_readonly("lane_eval", &LanesLoop::lane_eval)
      .def_property_readonly("overlap", &LanesLoop::overlap)
      .def_property_readonly("host_us_per_round", &LanesLoop::host_us_per_round)
      .def("host_phases_us", &LanesLoop::host_phases_us)
      .def_property_readonly("rounds_run", &LanesLoop::rounds_run)
      .def("stats", [](const LanesLoop& l, int lane, uintptr_t s) { return l.stats(lane, S(s)); })
      .def("loss", [](const LanesLoop& l, int lane, uintptr_t s) { return l.loss(lane, S(s)); })
      .def("delta_ptr", &LanesLoop::delta_ptr)
      .def("copy_out_all",
           [](const LanesLoop& l, const std::vector<uintptr_t>& loss, const std::vector<uintptr_t>& delta,
              uintptr_t s) { l.copy_out_all(loss, delta, S(s)); },
           py::arg("loss"), py::arg("delta"), py::arg("stream"))
      .def("copy_out", [](const LanesLoop& l, int lane, uintptr_t loss, uintptr_t delta,
                          uintptr_t s) { l.copy_out(lane, loss, delta, S(s)); },
           py::arg("lane"), py::arg("loss") = 0, py::arg("delta") = 0, py::arg("stream") = 0)
      .def("inject_spin_timeout", &LanesLoop::inject_spin_timeout)
      .def("poll_errors", &LanesLoop::poll_errors)
      .def("read_stamps", [](const LanesLoop& l, int lane, uintptr_t s) { return l.read_stamps(lane, S(s)); })
      .def("read_rider_stamps", [](const LanesLoop& l, uintptr_t s) { return l.read_rider_stamps(S(s)); })
      .def_static("probe_placement", [](uintptr_t s) { return LanesLoop::probe_placement(S(s)); });
  m.def("lanes_supported", &lanes_supported, py::arg("FP"), py::arg("K"), py::arg("cap"));

  py::class_<KeyRangeLoop>(m, "KeyRangeLoop")
      .def(py::init([](py::dict d, RcclComm* comm) {
             auto I = [&](const char* k, int64_t def) { return d.contains(k) ? d[k].cast<int64_t>() : def; };
             auto U = [&](const char* k) { return d.contains(k) ? d[k].cast<uintptr_t>() : (uintptr_t)0; };
             auto D = [&](const char* k, double def) { return d.contains(k) ? d[k].cast<double>() : def; };
             KeyRangeLoopCfg c;
             c.wcfg = d["wcfg"].cast<WideCfg>();
             c.use_graph = I("use_graph", 1) != 0;
             c.indptr = P<const int64_t>(U("indptr"));
             c.idx = P<const int32_t>(U("idx"));
             c.val = P<const uint16_t>(U("val"));
             c.y = P<const int32_t>(U("y"));
             c.ds_rows = I("ds_rows", 0);
             c.k = (int)I("k", 0);
             c.N = (int)I("N", 1);
             c.per_iter_rows = (int)I("per_iter_rows", 0);
             c.p_ms = D("p_ms", 0.0);
             c.epochs = I("epochs", 1);
             c.t0_ms = D("t0_ms", 0.0);
             c.ridx = P<int32_t>(U("ridx"));
             c.rval = P<uint16_t>(U("rval"));
             c.rnnz = P<int32_t>(U("rnnz"));
             c.ry = P<int32_t>(U("ry"));
             c.trunc = P<int>(U("trunc"));
             c.window = U("window");
             c.shard = P<float>(U("shard"));
             c.b = P<float>(U("b"));
             c.lr = (float)D("lr", 1.0);
             c.dloc = P<float>(U("dloc"));
             c.wloc = P<float>(U("wloc"));
             c.loss = P<float>(U("loss"));
             c.stats = P<int>(U("stats"));
             c.uniq = P<int32_t>(U("uniq"));
             c.t_indptr = P<const int64_t>(U("t_indptr"));
             c.t_idx = P<const int32_t>(U("t_idx"));
             c.t_val = P<const uint16_t>(U("t_val"));
             c.t_y = P<const int32_t>(U("t_y"));
             c.T = (int)I("T", 0);
             c.s_indptr = P<const int64_t>(U("s_indptr"));
             c.s_idx = P<const int32_t>(U("s_idx"));
             c.s_val = P<const uint16_t>(U("s_val"));
             c.sink = U("sink");
             c.log_server = I("log_server", 1) != 0;
             c.log_workers = I("log_workers", 1) != 0;
             c.tracker = U("tracker");
             c.api = U("api");
             c.margin_refresh = (int)I("margin_refresh", 256);
             return std::make_unique<KeyRangeLoop>(c, comm);
           }),
           py::arg("cfg"), py::arg("comm") = nullptr, py::keep_alive<1, 3>())
      .def(
          "run",
          [](KeyRangeLoop& l, int64_t rounds, int64_t r0, uintptr_t stream, double max_wait_s) {
            py::gil_scoped_release nogil;
            return l.run(rounds, r0, S(stream), max_wait_s);
          },
          py::arg("rounds"), py::arg("r0"), py::arg("stream"), py::arg("max_wait_s") = 600.0)
      .def_property_readonly("lo", &KeyRangeLoop::lo)
      .def_property_readonly("hi", &KeyRangeLoop::hi)
      .def_property_readonly("shard_size", &KeyRangeLoop::shard_size)
      .def_property_readonly("model_bytes", &KeyRangeLoop::model_bytes)
      .def_property_readonly("eval_bytes", &KeyRangeLoop::eval_bytes)
      .def_property_readonly("last_round_bytes", &KeyRangeLoop::last_round_bytes)
      .def_property_readonly("last_u", &KeyRangeLoop::last_u)
      .def_property_readonly("device_bytes", &KeyRangeLoop::device_bytes)
      .def_property_readonly("host_us_per_round", &KeyRangeLoop::host_us_per_round)
      .def_property_readonly("rounds_run", &KeyRangeLoop::rounds_run)
      .def("next_local", &KeyRangeLoop::next_local)
      .def("set_next_local", &KeyRangeLoop::set_next_local)
      .def_property_readonly("exhausted", &KeyRangeLoop::exhausted);
  // XCC_ID of every workgroup of an n-workgroup launch (placement diagnostics)
  m.def("xcc_map", [](int n, uintptr_t stream) {
    int* ids = nullptr;
    hip_check(hipMalloc(&ids, n * sizeof(int)), "hipMalloc");
    launch_xcc_probe(ids, n, S(stream));
    std::vector<int> h(n);
    hip_check(hipMemcpyAsync(h.data(), ids, n * sizeof(int), hipMemcpyDeviceToHost, S(stream)), "copy");
    hip_check(hipStreamSynchronize(S(stream)), "sync");
    (void)hipFree(ids);
    return h;
  });
  m.attr("ASYNC_DONE") = (int)kAsyncDone;
  m.attr("ASYNC_ERROR_TOKEN") = (int)kAsyncErrorToken;
  m.attr("ASYNC_WATCHDOG") = (int)kAsyncWatchdog;
  m.attr("ASYNC_CHECKPOINT") = (int)kAsyncCheckpoint;

  m.def("ring_ingest_f32", [](uintptr_t src, uintptr_t ysrc, int64_t src_first, int64_t src_step, int64_t n,
                              uintptr_t ring, uintptr_t yring, int64_t dst_first, int64_t cap, int FP, uintptr_t stream) {
    launch_ring_ingest_f32(P<const float>(src), P<const int32_t>(ysrc), src_first, src_step, n, P<float>(ring),
                           P<int32_t>(yring), dst_first, cap, FP, S(stream));
    hip_check(hipGetLastError(), "ring_ingest_f32 launch");
  });
  m.def("ring_ingest", [](uintptr_t src, uintptr_t ysrc, int64_t src_first, int64_t src_step, int64_t n,
                          uintptr_t ring, uintptr_t ringT, uintptr_t yring, int64_t dst_first, int64_t cap, int FP,
                          uintptr_t stream) {
    launch_ring_ingest(P<const uint16_t>(src), P<const int32_t>(ysrc), src_first, src_step, n, P<uint16_t>(ring),
                       P<uint16_t>(ringT), P<int32_t>(yring), dst_first, cap, FP, S(stream));
    hip_check(hipGetLastError(), "ring_ingest launch");
  });
}
