// pybind11 bindings for the native host runtime (_psx_host): tracker, sliding
// window, dataset ingest, producer schedule, control plane and CSV logger.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "../host/capi.h"
#include "../host/ctrl.h"
#include "../host/dataset.h"
#include "../host/libsvm.h"
#include "../host/logger.h"
#include "../host/metrics_sink.h"
#include "../host/sampling.h"
#include "../host/tracker.h"
#include "../kernels/solver_ctrl.h"

#include <cstring>
#include <memory>

namespace py = pybind11;
using namespace psx;

PYBIND11_MODULE(_psx_host, m) {
  // C ABI table for the GPU runtime's native server loop (capi.h)
  m.def("capi", []() { return reinterpret_cast<uintptr_t>(host_api()); });
  m.attr("CAPI_VERSION") = kHostApiVersion;

  m.doc() = "psx native host runtime";

  py::class_<VectorClockTracker>(m, "VectorClockTracker")
      .def(py::init<int, int>(), py::arg("num_workers"), py::arg("consistency_model"))
      .def("received", &VectorClockTracker::received)
      .def("sent", &VectorClockTracker::sent)
      .def("releasable", &VectorClockTracker::releasable)
      .def("on_delta", &VectorClockTracker::on_delta)
      .def("min_clock", &VectorClockTracker::min_clock)
      .def("max_clock", &VectorClockTracker::max_clock)
      .def("clock", &VectorClockTracker::clock)
      .def("is_sent", &VectorClockTracker::is_sent)
      .def("clocks", &VectorClockTracker::clocks)
      .def("sent_flags", &VectorClockTracker::sent_flags)
      .def("restore", &VectorClockTracker::restore)
      .def("retire", &VectorClockTracker::retire)
      .def("revive", &VectorClockTracker::revive)
      .def("bsp_round", &VectorClockTracker::bsp_round)
      .def("is_live", &VectorClockTracker::is_live)
      .def_property_readonly("num_live", &VectorClockTracker::num_live)
      .def_property_readonly("num_workers", &VectorClockTracker::num_workers)
      .def_property_readonly("consistency_model", &VectorClockTracker::consistency_model)
      .def_property_readonly("max_gap", &VectorClockTracker::max_gap)
      .def_property_readonly("handle", [](VectorClockTracker& t) { return reinterpret_cast<uintptr_t>(&t); });

  py::class_<RateEstimator>(m, "RateEstimator")
      .def(py::init<int>(), py::arg("window") = 500)
      .def("arrival", &RateEstimator::arrival)
      .def("mean_interarrival_ms", &RateEstimator::mean_interarrival_ms)
      .def_property_readonly("samples", &RateEstimator::samples);

  py::class_<SlotAssignment>(m, "SlotAssignment")
      .def_readonly("slot", &SlotAssignment::slot)
      .def_readonly("insertion_id", &SlotAssignment::insertion_id)
      .def_readonly("size", &SlotAssignment::size)
      .def_readonly("target", &SlotAssignment::target);

  py::class_<SlidingWindow>(m, "SlidingWindow")
      .def(py::init<int64_t, int64_t, double, int, int64_t>(), py::arg("min_size"), py::arg("max_size"),
           py::arg("buffer_coefficient"), py::arg("rate_window") = 500, py::arg("ring_capacity") = 0)
      .def("target_size", &SlidingWindow::target_size)
      .def("insert", &SlidingWindow::insert)
      .def("insert_many",
           [](SlidingWindow& w, py::array_t<double, py::array::c_style | py::array::forcecast> t) {
             auto n = t.size();
             py::array_t<int64_t> slots(n);
             w.insert_many(t.data(), n, slots.mutable_data());
             return slots;
           })
      // the round loops' form (no per-row slots: equal-stamp runs take the bulk path);
      // returns the slot of the first row
      .def("insert_bulk",
           [](SlidingWindow& w, py::array_t<double, py::array::c_style | py::array::forcecast> t) {
             return w.insert_many(t.data(), t.size(), nullptr);
           })
      .def("restore", &SlidingWindow::restore)
      .def_property_readonly("size", &SlidingWindow::size)
      .def_property_readonly("capacity", &SlidingWindow::capacity)
      .def_property_readonly("max_size", &SlidingWindow::max_size)
      .def_property_readonly("head", &SlidingWindow::head)
      .def_property_readonly("start", &SlidingWindow::start)
      .def_property_readonly("tuples_seen", &SlidingWindow::tuples_seen)
      .def_property_readonly("handle", [](SlidingWindow& w) { return reinterpret_cast<uintptr_t>(&w); })
      .def("mean_interarrival_ms", &SlidingWindow::mean_interarrival_ms);

  py::class_<CsvInfo>(m, "CsvInfo")
      .def_readonly("rows", &CsvInfo::rows)
      .def_readonly("cols", &CsvInfo::cols)
      .def_readonly("header", &CsvInfo::header)
      .def_readonly("names", &CsvInfo::names);

  m.def("csv_probe", &csv_probe, py::arg("path"), py::arg("header_mode") = 0);
  m.def(
      "csv_load",
      [](const std::string& path, const CsvInfo& info, int label_col, int64_t row_stride, bool want_f32,
         bool want_bf16, int threads) {
        int64_t rows = info.rows;
        py::array_t<float> xf;
        py::array_t<uint16_t> xb;
        py::array_t<int32_t> y(rows);
        if (want_f32) xf = py::array_t<float>({rows, row_stride});
        if (want_bf16) xb = py::array_t<uint16_t>({rows, row_stride});
        {
          py::gil_scoped_release rel;
          csv_load(path, info, label_col, row_stride, want_f32 ? xf.mutable_data() : nullptr,
                   want_bf16 ? xb.mutable_data() : nullptr, y.mutable_data(), threads);
        }
        return py::make_tuple(want_f32 ? py::object(xf) : py::none(), want_bf16 ? py::object(xb) : py::none(), y);
      },
      py::arg("path"), py::arg("info"), py::arg("label_col") = -1, py::arg("row_stride") = 0,
      py::arg("want_f32") = true, py::arg("want_bf16") = false, py::arg("threads") = 0);
  m.def("arrival_time_ms", &arrival_time_ms);
  m.def("due_rows", [](int k, int n, double p, int64_t total, int64_t next_local, double now, int64_t max_rows) {
    py::array_t<double> times(max_rows > 0 ? std::min<int64_t>(max_rows, 1 << 24) : 0);
    int64_t c = due_rows(k, n, p, total, next_local, now, times.size(), times.mutable_data());
    return py::make_tuple(c, times);
  });
  m.def("f32_to_bf16", &f32_to_bf16);
  m.def(
      "libsvm_load",
      [](const std::string& path, bool zero_based, int threads) {
        SparseRows r;
        {
          py::gil_scoped_release rel;
          r = libsvm_load(path, zero_based, threads);
        }
        auto mk = [](auto& v) {
          using T = typename std::decay_t<decltype(v)>::value_type;
          py::array_t<T> a(static_cast<py::ssize_t>(v.size()));
          if (!v.empty()) std::memcpy(a.mutable_data(), v.data(), v.size() * sizeof(T));
          return a;
        };
        return py::make_tuple(mk(r.indptr), mk(r.idx), mk(r.val), mk(r.y), r.max_feature);
      },
      py::arg("path"), py::arg("zero_based") = false, py::arg("threads") = 0);
  m.def(
      "libsvm_save",
      [](const std::string& path, py::array_t<int64_t, py::array::c_style | py::array::forcecast> indptr,
         py::array_t<int32_t, py::array::c_style | py::array::forcecast> idx,
         py::array_t<uint16_t, py::array::c_style | py::array::forcecast> val,
         py::array_t<int32_t, py::array::c_style | py::array::forcecast> y, bool zero_based) {
        const int64_t rows = static_cast<int64_t>(y.size());
        if (indptr.size() != rows + 1) throw std::invalid_argument("indptr must have rows + 1 entries");
        if (idx.size() != val.size() || (rows > 0 && indptr.data()[rows] != idx.size()))
          throw std::invalid_argument("idx / val / indptr sizes disagree");
        libsvm_save(path, indptr.data(), idx.data(), val.data(), y.data(), rows, zero_based);
      },
      py::arg("path"), py::arg("indptr"), py::arg("idx"), py::arg("val"), py::arg("y"), py::arg("zero_based") = false);

  py::class_<CtrlToken>(m, "CtrlToken")
      .def(py::init<>())
      .def_readwrite("worker", &CtrlToken::worker)
      .def_readwrite("kind", &CtrlToken::kind)
      .def_readwrite("vc", &CtrlToken::vc)
      .def_readwrite("aux", &CtrlToken::aux)
      .def_readwrite("ts_us", &CtrlToken::ts_us)
      .def_readwrite("n", &CtrlToken::n);

  py::class_<CtrlQueue>(m, "CtrlQueue")
      .def(py::init<const std::string&, uint32_t, bool>(), py::arg("name"), py::arg("capacity"), py::arg("create"))
      .def("try_push", &CtrlQueue::try_push)
      .def("push", &CtrlQueue::push, py::arg("token"), py::arg("timeout_s") = -1.0,
           py::call_guard<py::gil_scoped_release>())
      .def("try_pop",
           [](CtrlQueue& q) -> py::object {
             CtrlToken t;
             if (q.try_pop(&t)) return py::cast(t);
             return py::none();
           })
      .def(
          "pop",
          [](CtrlQueue& q, double timeout_s) -> py::object {
            CtrlToken t;
            bool ok;
            {
              py::gil_scoped_release rel;
              ok = q.pop(&t, timeout_s);
            }
            if (ok) return py::cast(t);
            return py::none();
          },
          py::arg("timeout_s") = -1.0)
      .def("unlink", &CtrlQueue::unlink)
      .def_property_readonly("capacity", &CtrlQueue::capacity)
      .def_property_readonly("name", &CtrlQueue::name)
      .def("state", [](const CtrlQueue& q) { return py::make_tuple(q.enqueued(), q.dequeued(), q.inode()); })
      .def_property_readonly("handle", [](CtrlQueue& q) { return reinterpret_cast<uintptr_t>(&q); });

  // Host build of the device solver state machine (csrc/kernels/solver_ctrl.h),
  // so the exact control logic the GPU runs can be unit-tested on the CPU.
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
      .def_readwrite("xf32", &SolverCfg::xf32);
  py::class_<Ctrl>(m, "SolverCtrl", py::module_local())
      .def(py::init([]() {
        auto c = std::make_unique<Ctrl>();
        std::memset(c.get(), 0, sizeof(Ctrl));
        ctrl_init(*c);
        return c;
      }))
      .def("step",
           [](Ctrl& c, const SolverCfg& cfg, double f_t, const std::vector<double>& dots, int slot) {
             if (static_cast<int>(dots.size()) < num_dots(cfg.hist)) throw std::invalid_argument("too few dots");
             ctrl_step(c, cfg, f_t, dots.data(), slot);
           })
      .def_readonly("phase", &Ctrl::phase)
      .def_readonly("action", &Ctrl::action)
      .def_readonly("action_slot", &Ctrl::action_slot)
      .def_readonly("iter", &Ctrl::iter)
      .def_readonly("m", &Ctrl::m)
      .def_readonly("head", &Ctrl::head)
      .def_readonly("push_slot", &Ctrl::push_slot)
      .def_readonly("nacc", &Ctrl::nacc)
      .def_readonly("ls_fail", &Ctrl::ls_fail)
      .def_readonly("evals", &Ctrl::evals)
      .def_readonly("t", &Ctrl::t)
      .def_readonly("t_acc", &Ctrl::t_acc)
      .def_readonly("f_c", &Ctrl::f_c)
      .def_readonly("cg", &Ctrl::cg)
      .def_property_readonly("cs", [](const Ctrl& c) { return std::vector<double>(c.cs, c.cs + kMaxHist); })
      .def_property_readonly("cy", [](const Ctrl& c) { return std::vector<double>(c.cy, c.cy + kMaxHist); });
  m.attr("kActNone") = static_cast<int>(kActNone);
  m.attr("kActInit") = static_cast<int>(kActInit);
  m.attr("kActTrial") = static_cast<int>(kActTrial);
  m.attr("kActAccept") = static_cast<int>(kActAccept);
  m.attr("kActAcceptDone") = static_cast<int>(kActAcceptDone);
  m.attr("kActDone") = static_cast<int>(kActDone);
  m.attr("kPhDone") = static_cast<int>(kPhDone);

  m.def("java_double", &java_double);
  py::class_<CsvLogger>(m, "CsvLogger")
      .def(py::init<const std::string&, bool, bool, bool>(), py::arg("path"), py::arg("worker_schema"),
           py::arg("write_header") = true, py::arg("append") = false)
      .def("log_worker", &CsvLogger::log_worker)
      .def("log_server", &CsvLogger::log_server)
      .def("log_line", &CsvLogger::log_line)
      .def("flush", &CsvLogger::flush, py::call_guard<py::gil_scoped_release>())
      .def("close", &CsvLogger::close, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("lines", &CsvLogger::lines);

  m.attr("EVAL_SLOT_BYTES") = (int)sizeof(EvalSlot);
  m.def(
      "weighted_f1_accuracy",
      [](py::array_t<int32_t, py::array::c_style | py::array::forcecast> conf16, int K) {
        if (conf16.size() != 256) throw std::invalid_argument("need a 16x16 confusion matrix");
        double f1 = 0.0, acc = 0.0;
        weighted_f1_accuracy(conf16.data(), K, &f1, &acc);
        return py::make_tuple(f1, acc);
      },
      py::arg("conf16"), py::arg("K"));
  py::class_<MetricsSink>(m, "MetricsSink")
      .def(py::init([](uintptr_t slots, int nslots, int K, CsvLogger* wlog, CsvLogger* slog, bool keep) {
             return std::make_unique<MetricsSink>(slots, nslots, K, wlog, slog, keep);
           }),
           py::arg("slots"), py::arg("nslots"), py::arg("K"), py::arg("wlog").none(true), py::arg("slog").none(true),
           py::arg("keep_records") = true, py::keep_alive<1, 5>(), py::keep_alive<1, 6>())
      .def(
          "acquire",
          [](MetricsSink& s) {
            uint64_t seq = 0;
            int slot;
            {
              py::gil_scoped_release nogil;
              slot = s.acquire(&seq);
            }
            return py::make_tuple(slot, seq, s.slot_address(slot));
          })
      .def("submit", &MetricsSink::submit, py::arg("slot"), py::arg("seq"), py::arg("kind"), py::arg("ts"),
           py::arg("partition"), py::arg("vc"), py::arg("nseen"))
      .def("flush", &MetricsSink::flush, py::arg("timeout_s") = 0.0, py::call_guard<py::gil_scoped_release>())
      .def("close", &MetricsSink::close, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("processed", &MetricsSink::processed)
      .def_property_readonly("handle", [](MetricsSink& s) { return reinterpret_cast<uintptr_t>(&s); })
      .def("worker_rows",
           [](MetricsSink& s) {
             py::list out;
             for (const auto& r : s.worker_rows())
               out.append(py::make_tuple(r.ts, r.partition, r.vc, r.loss, r.f1, r.acc, r.nseen));
             return out;
           })
      .def("server_rows", [](MetricsSink& s) {
        py::list out;
        for (const auto& r : s.server_rows()) out.append(py::make_tuple(r.ts, r.vc, r.f1, r.acc));
        return out;
      });
}
