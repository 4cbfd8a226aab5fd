// Host loop of the peer data plane's server rank (see peer_server.h).
#include "peer_server.h"

#include <emmintrin.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>

#include "../host/sink_record.h"
#include "../kernels/common.h"
#include "../solver/solver.h"

namespace psx {
namespace {
double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }
constexpr int kKindDelta = 0, kKindFinal = 1, kKindError = 2;
}  // namespace

PeerServer::PeerServer(const PeerServerCfg& cfg, hipStream_t stream) : cfg_(cfg), stream_(nullptr) {
  (void)stream;  // the persistent launch gets a stream of its own (nothing else is ordered behind it)
  const int N = cfg.nworkers;
  if (N < 1 || N > kSrvMaxWorkers) throw std::invalid_argument("PeerServer: 1 .. 64 workers");
  if (!cfg.api || (!cfg.bsp && (!cfg.tracker || (!cfg.ctrl && !cfg.standin))))
    throw std::invalid_argument("PeerServer: missing host runtime handles");
  api_ = reinterpret_cast<const HostApi*>(cfg.api);
  if (api_->version != kHostApiVersion) throw std::runtime_error("PeerServer: host runtime C ABI version mismatch");
  if (!cfg.w || cfg.P <= 0 || cfg.K < 1 || cfg.K > 8) throw std::invalid_argument("PeerServer: weights / classes");
  if (cfg.FP != 128 && cfg.FP != 256 && cfg.FP != 512 && cfg.FP != 1024)
    throw std::invalid_argument("PeerServer: FP in {128, 256, 512, 1024}");
  if (cfg.P != (int64_t)cfg.K * cfg.FP + cfg.K) throw std::invalid_argument("PeerServer: P != K * FP + K");
  NS_ = cfg.FP / 32;
  if (!cfg.inbox || cfg.lay.P != cfg.P || cfg.lay.NS != NS_ || cfg.lay.slots < N)
    throw std::invalid_argument("PeerServer: inbox region layout");
  if ((int)cfg.rx.size() != N || (int)cfg.rx_tag.size() != N ||
      (!cfg.bsp && !cfg.standin && (int)cfg.replies.size() != N))
    throw std::invalid_argument("PeerServer: one receive slot, tag array and reply queue per worker");
  const bool need_q = !cfg.bsp && !cfg.standin;  // (token / reply queues)
  for (int j = 0; j < N; ++j)
    if (!cfg.rx[j] || !cfg.rx_tag[j] || (need_q && !cfg.replies[j]))
      throw std::invalid_argument("PeerServer: null peer handle");
  if (cfg.batch < 1 || cfg.batch > kSrvMaxBatch) throw std::invalid_argument("PeerServer: batch 1 .. 64");
  if (cfg.sink && (!cfg.Xt || !cfg.yt || cfg.T < 1)) throw std::invalid_argument("PeerServer: server rows need the test set");
  if (cfg.sxcd < 0 || cfg.sxcd > 7) throw std::invalid_argument("PeerServer: sxcd in 0..7");
  // device workspace (ALL device memory and its zero-fill here, before any
  // persistent launch of another rank can hold the CUs a fill kernel would need)
  const int FP = cfg.FP;
  size_t off = 0;
  auto take = [&](size_t bytes) {
    const size_t o = off;
    off = align_up(off + bytes, 256);
    return o;
  };
  const size_t o_rx = take(sizeof(float*) * N);
  const size_t o_rxt = take(sizeof(unsigned*) * N);
  const size_t o_ptag = take((size_t)N * NS_ * 4);
  const size_t o_shi = take((size_t)16 * FP * 2);
  const size_t o_slo = take((size_t)16 * FP * 2);
  const size_t o_sb = take(16 * 4);
  const size_t o_acc = take((size_t)2 * 256 * kAccStride * 4);
  const size_t o_etk = take(4);
  const size_t o_flags = take((size_t)(kSrvWg + 1) * 32 * 8);
  const size_t o_rec = take(32 * 8);
  const size_t o_claim = take(64 * 4);
  const size_t o_erec = take((size_t)kSrvMaxBatch * kEntChunks * 16);
  // The persistent launch needs a hardware queue of its own: HIP multiplexes a process's
  // streams of one priority onto GPU_MAX_HW_QUEUES (4) queues, whose packets run in order --
  // a stream that shares the server kernel's queue would wait behind it for good (the
  // colocated peer_sum rank 0 launches its lanes beside it; every solver holds a capture
  // stream).  The greatest priority has a queue pool of its own, and nothing else here uses it
  // (tools/hwq_probe.hip, profiles/r06/s18_hwq: 2 of 12 normal streams wait behind a spinning
  // kernel on a normal stream, none behind one on this priority; the least priority -- the
  // lanes loop's overlap stream -- measured the same as this one for the server, s23).
  int prio_lo = 0, prio_hi = 0;
  hip_check(hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi), "hipDeviceGetStreamPriorityRange");
  hip_check(hipStreamCreateWithPriority(&stream_, hipStreamNonBlocking, prio_hi), "hipStreamCreate(peer server)");
  hip_check(hipMalloc(&ws_, off), "hipMalloc(peer server workspace)");
  hip_check(hipMemset(ws_, 0, off), "hipMemset(peer server workspace)");
  char* b = static_cast<char*>(ws_);
  hip_check(hipMemcpy(b + o_rx, cfg.rx.data(), sizeof(float*) * N, hipMemcpyHostToDevice), "rx table");
  hip_check(hipMemcpy(b + o_rxt, cfg.rx_tag.data(), sizeof(unsigned*) * N, hipMemcpyHostToDevice), "rx tag table");
  hip_check(hipHostMalloc((void**)&cmd_ring_, sizeof(TagChunk) * kCmdChunks * ring_,
                          hipHostMallocCoherent | hipHostMallocMapped),
            "hipHostMalloc(command ring)");
  hip_check(hipHostMalloc((void**)&err_host_, 2 * sizeof(unsigned long long), hipHostMallocCoherent | hipHostMallocMapped),
            "hipHostMalloc(error word)");
  std::memset((void*)cmd_ring_, 0, sizeof(TagChunk) * kCmdChunks * ring_);
  ent_cap_ = (ring_ + 1) * kSrvMaxBatch;  // (every command in flight holds <= kSrvMaxBatch entries)
  hip_check(hipHostMalloc((void**)&ent_ring_, sizeof(TagChunk) * kEntChunks * (size_t)ent_cap_,
                          hipHostMallocCoherent | hipHostMallocMapped),
            "hipHostMalloc(entry ring)");
  std::memset((void*)ent_ring_, 0, sizeof(TagChunk) * kEntChunks * (size_t)ent_cap_);
  err_host_[0] = err_host_[1] = 0;
  consumed_host_ = err_host_ + 1;
  hip_check(hipDeviceSynchronize(), "peer server setup");
  SrvArgs& a = args_;
  std::memset(&a, 0, sizeof(a));
  a.K = cfg.K;
  a.F = cfg.F;
  a.FP = FP;
  a.P = (int)cfg.P;
  a.N = N;
  a.lr = cfg.lr;
  a.w = cfg.w;
  a.shi = reinterpret_cast<uint16_t*>(b + o_shi);
  a.slo = reinterpret_cast<uint16_t*>(b + o_slo);
  a.sb = reinterpret_cast<float*>(b + o_sb);
  a.inbox = reinterpret_cast<const float*>(cfg.inbox);
  a.inbox_tag = reinterpret_cast<const unsigned*>(cfg.inbox + cfg.lay.tag_off());
  a.in_stride = cfg.lay.stride();
  a.rx = reinterpret_cast<float* const*>(b + o_rx);
  a.rx_tag = reinterpret_cast<unsigned* const*>(b + o_rxt);
  a.ptag = reinterpret_cast<unsigned*>(b + o_ptag);
  a.cmd = cmd_ring_;
  a.ring = ring_;
  a.ent = ent_ring_;
  a.ent_cap = ent_cap_;
  a.erec = reinterpret_cast<unsigned long long*>(b + o_erec);
  a.consumed_host = consumed_host_;
  a.err_host = err_host_;
  a.Xt = cfg.Xt;
  a.yt = cfg.yt;
  a.T = cfg.T;
  a.acc = reinterpret_cast<int*>(b + o_acc);
  a.eticket = reinterpret_cast<unsigned*>(b + o_etk);
  a.flags = reinterpret_cast<unsigned long long*>(b + o_flags);
  a.rec = reinterpret_cast<unsigned long long*>(b + o_rec);
  a.claim = reinterpret_cast<unsigned*>(b + o_claim);
  a.sxcd = cfg.sxcd;
  if (cfg.nwg < 1 || cfg.nwg > kSrvWg) throw std::invalid_argument("PeerServer: 1 .. 32 server workgroups");
  a.nwg = cfg.nwg;
  // wall-clock budgets: the command wait outlasts the host's own watchdog (the worker
  // timeout: a silent worker is failed and the commands resume); a delta's tag is
  // written before its token leaves the worker's GPU (a short wait at most)
  const double cmd_s = std::min(cfg.worker_timeout_s + 30.0, 7200.0);
  a.cmd_ticks = (long long)(cmd_s * 1e8);
  // (BSP rounds: the slowest rank's round, which may wait for its stream's rows)
  a.tag_ticks = cfg.bsp ? (long long)(std::min(std::max(cfg.tag_wait_s, 10.0), 7200.0) * 1e8) : 10ll * 100000000ll;
  if (cfg.bsp) a.cmd_ticks = std::max(a.cmd_ticks, a.tag_ticks + (long long)(30.0 * 1e8));
  a.spin = 1 << 22;
  ptag_.assign(N, 0u);
  finished_.assign(N, 0);
  failed_.assign(N, 0);
  dead_.assign(N, 0);
  busy_since_.assign(N, -1.0);
  rel_k_.resize(N + 1);
  rel_v_.resize(N + 1);
}

PeerServer::~PeerServer() {
  if (bsp_thr_.joinable()) bsp_thr_.join();  // (run_bsp_async's rounds end by themselves: drained or timed out)
  try {
    stop();
  } catch (...) {
  }
  if (stream_) {
    (void)hipStreamSynchronize(stream_);
    (void)hipStreamDestroy(stream_);
  }
  if (ws_) (void)hipFree(ws_);
  if (cmd_ring_) (void)hipHostFree(cmd_ring_);
  if (ent_ring_) (void)hipHostFree(ent_ring_);
  if (err_host_) (void)hipHostFree(err_host_);
  if (tr_) (void)hipFree(tr_);
}

void PeerServer::check_api(int rc, const char* what) const {
  if (rc < 0) throw std::runtime_error(std::string("PeerServer: ") + what + ": " + api_->last_error());
}

void PeerServer::check_device() const {
  const unsigned long long e = __atomic_load_n(err_host_, __ATOMIC_ACQUIRE);
  if (e) {
    // (the protocol state for the report: deltas applied per worker, commands written /
    // read by the kernel, the last arrivals)
    std::string m = "PeerServer: the server kernel's wait timed out (command " + std::to_string(e >> 8) + ", code " +
                    std::to_string((int)(e & 0xff)) +
                    (int(e & 0xff) == 11 ? ": a worker's delta never reached the inbox" : "") + "); commands " +
                    std::to_string(cmds_) + " written, " +
                    std::to_string(__atomic_load_n(consumed_host_, __ATOMIC_ACQUIRE)) + " read; deltas per worker:";
    std::vector<int> per(cfg_.nworkers, 0);
    for (const auto& a : arrivals_) ++per[a.first];
    for (int j = 0; j < cfg_.nworkers; ++j) m += " " + std::to_string(per[j]);
    m += "; last arrivals:";
    for (size_t i = arrivals_.size() > 12 ? arrivals_.size() - 12 : 0; i < arrivals_.size(); ++i)
      m += " (" + std::to_string(arrivals_[i].first) + "," + std::to_string((long long)arrivals_[i].second) + ")";
    if (cfg_.bsp) m += "; BSP rounds commanded " + std::to_string((long long)bsp_n_) + "; " + bsp_tags();
    throw std::runtime_error(m);
  }
}

int PeerServer::log_worker() const {
  // server rows follow worker 0's deltas (ServerProcessor.java:154-165), or the
  // lowest surviving worker's once 0 has failed
  for (int j = 0; j < cfg_.nworkers; ++j)
    if (!failed_[j]) return j;
  return -1;
}

std::vector<int> PeerServer::failed() const {
  std::vector<int> out;
  for (int j = 0; j < cfg_.nworkers; ++j)
    if (failed_[j]) out.push_back(j);
  return out;
}

void PeerServer::launch() {
  if (running_) return;
  SrvArgs a = args_;
  a.cmd0 = cmds_;
  a.cpar = (int)(launches_ & 1);
  a.launch = ++launches_;
  // (the arguments are the kernel argument: no copy in front of the launch -- on a GPU
  // shared with other ranks' persistent launches it could wait behind them)
  launch_server_persist(a, cfg_.FP, stream_);
  hip_check(hipGetLastError(), "server kernel launch");
  cmds_launch_ = cmds_;
  running_ = true;
}

void PeerServer::wait_ring() {
  // ring flow control: slot (n - 1) % ring is free once the kernel read command n - ring --
  // and with it every entry of that command (a command in flight holds <= kSrvMaxBatch
  // entries, the entry ring ring_ + 1 times that: the next command's entries never overwrite
  // those of a command the kernel has not read)
  const uint64_t n = cmds_ + 1;
  const uint64_t lim = (uint64_t)(cfg_.ahead > 0 && cfg_.ahead < ring_ ? cfg_.ahead : ring_);
  if (n > lim) {
    const double t0 = now_s();
    while (__atomic_load_n(consumed_host_, __ATOMIC_ACQUIRE) + lim < n) {
      check_device();
      if (now_s() - t0 > cfg_.worker_timeout_s) throw std::runtime_error("PeerServer: the server kernel stopped reading commands");
      _mm_pause();
    }
  }
}

void PeerServer::write_cmd(const SrvCmd& c) {
  wait_ring();
  const uint64_t n = cmds_ + 1;
  TagChunk ch[kCmdChunks];
  pack_cmd(c, (unsigned)n, ch);
  volatile TagChunk* dst = cmd_ring_ + (size_t)((n - 1) % (uint64_t)ring_) * kCmdChunks;
  for (int i = 0; i < kCmdChunks; ++i) {
    __m128i v;
    std::memcpy(&v, &ch[i], 16);
    _mm_store_si128((__m128i*)(void*)&dst[i], v);  // one 16-B store per chunk (a chunk is never torn)
  }
  std::atomic_thread_fence(std::memory_order_release);
  cmds_ = n;
}

void PeerServer::issue(int k, int64_t vc, const int* ks, const int64_t* vs, int n) {
  if (k < 0) flush_batch();  // (a release-only command: after the deltas before it)
  SrvEnt e{};
  e.k = k;
  e.dtag = k >= 0 ? (unsigned)(vc + 1) : 0u;
  const double t = now_s();
  for (int i = 0; i < n; ++i) {
    const int j = ks[i];
    if (j < 0 || j >= cfg_.nworkers) throw std::logic_error("PeerServer: release of an unknown worker");
    if (finished_[j]) continue;
    e.relmask |= 1ull << j;
    busy_since_[j] = t;
    // the replies: which worker the weights in flight are for, and their pull tag (the
    // kernel bumps a slot's tag once per release, in command / entry order)
    CtrlToken r{};
    r.worker = j;
    r.vc = vs[i];
    r.aux = (int64_t)++ptag_[j];
    bat_rep_.push_back(r);
  }
  const bool logs = k >= 0 && cfg_.sink && k == log_worker();
  if (k < 0) {  // releases only: a command of its own
    SrvCmd c{};
    c.k = -1;
    c.relmask = e.relmask;
    write_cmd(c);
    flush_batch();  // (the replies)
    return;
  }
  bat_.push_back(e);
  if (logs) {  // the global model's test metrics after this delta: one server row, ending the batch
    uintptr_t addr = 0;
    bat_slot_ = api().sink_acquire((void*)cfg_.sink, &bat_seq_, &addr);
    check_api(bat_slot_, "metrics sink acquire");
    bat_addr_ = addr;
    bat_vc_ = vc;
  }
  if (logs || (int)bat_.size() >= cfg_.batch) flush_batch();
}

void PeerServer::flush_batch() {
  const int m = (int)bat_.size();
  if (m == 1) {  // one delta: the classic command
    SrvCmd c{};
    c.k = bat_[0].k;
    c.dtag = bat_[0].dtag;
    c.relmask = bat_[0].relmask;
    if (bat_slot_ >= 0) {
      c.log = 1;
      c.slot_s = bat_addr_;
      c.seq_s = (unsigned)bat_seq_;
    }
    write_cmd(c);
  } else if (m > 1) {  // the entries first (the kernel reads them after the command's tag)
    wait_ring();  // (the command's slot free: so is every entry slot written below)
    const uint64_t e0 = ents_;
    for (int j = 0; j < m; ++j) {
      TagChunk ch[kEntChunks];
      pack_ent(bat_[j], (unsigned)(e0 + (uint64_t)j + 1), ch);
      volatile TagChunk* dst = ent_ring_ + (size_t)((e0 + (uint64_t)j) % (uint64_t)ent_cap_) * kEntChunks;
      for (int q = 0; q < kEntChunks; ++q) {
        __m128i v;
        std::memcpy(&v, &ch[q], 16);
        _mm_store_si128((__m128i*)(void*)&dst[q], v);
      }
    }
    ents_ = e0 + (uint64_t)m;
    std::atomic_thread_fence(std::memory_order_release);
    SrvCmd c{};
    c.k = kSrvBatch;
    c.dtag = (unsigned)m;
    c.relmask = e0;
    if (bat_slot_ >= 0) {
      c.log = 1;
      c.slot_s = bat_addr_;
      c.seq_s = (unsigned)bat_seq_;
    }
    write_cmd(c);
  }
  if (m > 0) {
    ++batches_;
    batched_deltas_ += m;
  }
  for (const CtrlToken& r : bat_rep_) {
    if (cfg_.standin) continue;
    if (api().ctrl_push((void*)cfg_.replies[r.worker], &r, cfg_.worker_timeout_s) != 1)
      throw std::runtime_error("PeerServer: reply queue of worker " + std::to_string(r.worker) + " full");
  }
  if (bat_slot_ >= 0) {
    SinkRecord rec{bat_slot_, 1 | kSinkTagged, bat_seq_, -1, -1, bat_vc_, 0};
    check_api(api().sink_submit_many((void*)cfg_.sink, 1, &rec), "metrics sink submit");
  }
  bat_.clear();
  bat_rep_.clear();
  bat_slot_ = -1;
}

void PeerServer::begin() {
  launch();
  std::fill(finished_.begin(), finished_.end(), 0);
  std::fill(failed_.begin(), failed_.end(), 0);
  std::fill(busy_since_.begin(), busy_since_.end(), -1.0);
  int n = 0;
  for (int j = 0; j < cfg_.nworkers; ++j) {
    int live = api().tracker_is_live((void*)cfg_.tracker, j);
    check_api(live, "tracker is_live");
    if (!live && !dead_[j]) {  // retired because it finished the previous run: rejoins
      check_api(api().tracker_revive((void*)cfg_.tracker, j), "tracker revive");
      live = 1;
    }
    if (!live) {
      failed_[j] = finished_[j] = dead_[j] = 1;
      continue;
    }
    const int64_t u = api().tracker_clock((void*)cfg_.tracker, j);
    if (u > 0) api().tracker_sent((void*)cfg_.tracker, j, u);
    rel_k_[n] = j;
    rel_v_[n] = u;
    ++n;
  }
  issue(-1, 0, rel_k_.data(), rel_v_.data(), n);  // the bootstrap (ServerProcessor.java:75-87)
}

void PeerServer::fail(int k) {
  if (k < 0 || k >= cfg_.nworkers) throw std::out_of_range("PeerServer::fail: worker id");
  launch();
  failed_[k] = finished_[k] = dead_[k] = 1;
  busy_since_[k] = -1.0;
  const int n = api().tracker_retire((void*)cfg_.tracker, k, rel_k_.data(), rel_v_.data(), (int)rel_k_.size());
  check_api(n, "tracker retire");
  if (n) issue(-1, 0, rel_k_.data(), rel_v_.data(), n);
}

void PeerServer::stop() {
  if (!running_) return;
  flush_batch();  // (deltas of an open batch before the stop command)
  SrvCmd c{};
  c.stop = 1;
  write_cmd(c);
  running_ = false;
  const double t0 = now_s();
  // (BSP: the commands ahead of the stop wait for the ranks' rounds)
  const double limit = cfg_.bsp ? std::max(60.0, cfg_.tag_wait_s + 30.0) : 60.0;
  for (;;) {
    const hipError_t e = hipStreamQuery(stream_);
    if (e == hipSuccess) break;
    if (e != hipErrorNotReady) hip_check(e, "server launch drain");
    if (now_s() - t0 > limit) {
      check_device();
      throw std::runtime_error("PeerServer: the server launch did not drain in " + std::to_string((int)limit) + " s");
    }
    std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
  check_device();
}

std::vector<double> PeerServer::bench_async(int64_t deltas, int log_every) {
  if (!cfg_.standin) throw std::logic_error("PeerServer::bench_async: needs stand-in workers (cfg standin)");
  const int N = cfg_.nworkers;
  // every stand-in worker holds the weights of its clock (the bootstrap), as after begin()
  std::fill(finished_.begin(), finished_.end(), 0);
  launch();
  std::vector<int64_t> vc(N, 0);
  for (int j = 0; j < N; ++j) vc[j] = api().tracker_clock((void*)cfg_.tracker, j);
  const double t0 = now_s();
  for (int64_t i = 0; i < deltas; ++i) {
    const int k = (int)(i % N);
    const int n = api().tracker_on_delta((void*)cfg_.tracker, k, vc[k], rel_k_.data(), rel_v_.data(), (int)rel_k_.size());
    check_api(n, "tracker on_delta");
    // (with a metrics sink, worker 0's deltas produce the server rows, as in run())
    issue(k, vc[k], rel_k_.data(), rel_v_.data(), n);
    ++vc[k];
    ++updates_;
  }
  flush_batch();
  (void)log_every;
  const double t1 = now_s();
  stop();
  const double t2 = now_s();
  return {t2 - t0, t1 - t0};
}

std::string PeerServer::bsp_tags() const {
  // (failure reports) the slice tags of every rank's inbox slot (its pushes) and receive
  // slot (the server's pulls), read on a stream of their own with a bounded wait
  const int N = cfg_.nworkers, NS = NS_;
  const size_t nt = (size_t)N * NS;
  std::vector<unsigned> h(2 * nt, 0xffffffffu);
  hipStream_t s = nullptr;
  std::string m = "tags (rank: inbox min..max / receive min..max):";
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return m + " (no stream)";
  bool ok = hipMemcpyAsync(h.data(), reinterpret_cast<const void*>(cfg_.inbox + cfg_.lay.tag_off()), nt * 4,
                           hipMemcpyDeviceToHost, s) == hipSuccess;
  for (int j = 0; j < N && ok; ++j)
    ok = hipMemcpyAsync(h.data() + nt + (size_t)j * NS, reinterpret_cast<const void*>(cfg_.rx_tag[j]), (size_t)NS * 4,
                        hipMemcpyDeviceToHost, s) == hipSuccess;
  const double t0 = now_s();
  while (ok && hipStreamQuery(s) == hipErrorNotReady && now_s() - t0 < 2.0)
    std::this_thread::sleep_for(std::chrono::microseconds(100));
  ok = ok && hipStreamQuery(s) == hipSuccess;
  (void)hipStreamDestroy(s);
  if (!ok) return m + " (unreadable)";
  for (int j = 0; j < N; ++j) {
    unsigned a0 = ~0u, a1 = 0, b0 = ~0u, b1 = 0;
    for (int q = 0; q < NS; ++q) {
      a0 = std::min(a0, h[(size_t)j * NS + q]);
      a1 = std::max(a1, h[(size_t)j * NS + q]);
      b0 = std::min(b0, h[nt + (size_t)j * NS + q]);
      b1 = std::max(b1, h[nt + (size_t)j * NS + q]);
    }
    m += " " + std::to_string(j) + ": " + std::to_string(a0) + ".." + std::to_string(a1) + " / " + std::to_string(b0) +
         ".." + std::to_string(b1);
  }
  return m;
}

void PeerServer::set_trace(int cap) {
  if (running_) throw std::logic_error("PeerServer::set_trace: the launch is running");
  if (tr_) (void)hipFree(tr_);
  tr_ = nullptr;
  tr_cap_ = cap > 0 ? cap : 0;
  if (tr_cap_) {
    hip_check(hipMalloc(&tr_, (size_t)tr_cap_ * 4 * sizeof(long long)), "hipMalloc(server trace)");
    hip_check(hipMemset(tr_, 0, (size_t)tr_cap_ * 4 * sizeof(long long)), "hipMemset(server trace)");
    hip_check(hipDeviceSynchronize(), "server trace");
  }
  args_.tr = tr_;
  args_.tr_cap = tr_cap_;
  tr_taken_ = cmds_;
}

std::vector<std::vector<long long>> PeerServer::trace_take() {
  std::vector<std::vector<long long>> out;
  if (!tr_ || running_) return out;
  std::vector<long long> h((size_t)tr_cap_ * 4);
  hip_check(hipMemcpy(h.data(), tr_, h.size() * sizeof(long long), hipMemcpyDeviceToHost), "server trace copy");
  const uint64_t first = std::max<uint64_t>(tr_taken_ + 1, cmds_ > (uint64_t)tr_cap_ ? cmds_ - tr_cap_ + 1 : 1);
  for (uint64_t n = first; n <= cmds_; ++n) {
    const long long* e = h.data() + (size_t)(n % (uint64_t)tr_cap_) * 4;
    if (e[3] == (long long)n) out.push_back({(long long)n, e[0], e[1], e[2]});
  }
  tr_taken_ = cmds_;
  return out;
}

void PeerServer::seed_rx() {
  if (running_) throw std::logic_error("PeerServer::seed_rx: the server launch is running");
  for (int j = 0; j < cfg_.nworkers; ++j)
    hip_check(hipMemcpy(reinterpret_cast<void*>(cfg_.rx[j]), cfg_.w, (size_t)cfg_.P * sizeof(float),
                        hipMemcpyDeviceToDevice),
              "peer_sum: weights into a rank's receive slot");
  hip_check(hipDeviceSynchronize(), "peer_sum seed");
}

int64_t PeerServer::run_bsp(int64_t rounds, int64_t r0) {
  if (!cfg_.bsp) throw std::logic_error("PeerServer::run_bsp: built for the asynchronous protocol");
  if (rounds <= 0) return 0;
  const auto h0 = std::chrono::steady_clock::now();
  launch();
  const unsigned long long all = cfg_.nworkers >= 64 ? ~0ull : ((1ull << cfg_.nworkers) - 1ull);
  for (int64_t i = 0; i < rounds; ++i) {
    SrvCmd c{};
    c.k = kSrvBspSum;
    c.dtag = (unsigned)(bsp_n_ + 1);
    c.relmask = all;
    int slot = -1;
    uint64_t seq = 0;
    if (cfg_.sink) {  // the global model after the round's update: its server row (ServerProcessor.java:154-165)
      uintptr_t addr = 0;
      slot = api().sink_acquire((void*)cfg_.sink, &seq, &addr);
      check_api(slot, "metrics sink acquire");
      c.log = 1;
      c.slot_s = addr;
      c.seq_s = (unsigned)seq;
    }
    write_cmd(c);
    ++bsp_n_;
    if (slot >= 0) {
      SinkRecord rec{slot, 1 | kSinkTagged, seq, -1, -1, r0 + i, 0};
      check_api(api().sink_submit_many((void*)cfg_.sink, 1, &rec), "metrics sink submit");
    }
    if (cfg_.tracker) check_api(api().tracker_bsp_round((void*)cfg_.tracker, r0 + i), "tracker");
    check_device();
  }
  bsp_ns_ += std::chrono::duration<double, std::nano>(std::chrono::steady_clock::now() - h0).count();
  stop();  // (the ranks' last sums applied: w is final)
  bsp_run_ += rounds;
  return rounds;
}

void PeerServer::run_bsp_async(int64_t rounds, int64_t r0) {
  if (bsp_thr_.joinable()) throw std::logic_error("PeerServer::run_bsp_async: the previous rounds not joined");
  bsp_err_ = nullptr;
  bsp_ret_ = 0;
  bsp_thr_ = std::thread([this, rounds, r0]() {
    try {
      bsp_ret_ = run_bsp(rounds, r0);
    } catch (...) {
      bsp_err_ = std::current_exception();
    }
  });
}

int64_t PeerServer::run_bsp_join() {
  if (!bsp_thr_.joinable()) return 0;
  bsp_thr_.join();
  if (bsp_err_) {
    std::exception_ptr e = bsp_err_;
    bsp_err_ = nullptr;
    std::rethrow_exception(e);
  }
  return bsp_ret_;
}

AsyncStatus PeerServer::run(int64_t checkpoint_every) {
  AsyncStatus st;
  launch();
  const double poll = cfg_.worker_timeout_s < 1.0 ? cfg_.worker_timeout_s : 1.0;
  for (;;) {
    int open = 0;
    for (int j = 0; j < cfg_.nworkers; ++j) open += !finished_[j];
    if (open == 0) break;
    CtrlToken t;
    int got = 0;
    if (!bat_.empty()) {  // an open batch takes the tokens already queued, then goes out
      got = api().ctrl_pop((void*)cfg_.ctrl, &t, 0.0);
      check_api(got, "token pop");
      if (!got) {
        flush_batch();
        continue;
      }
    } else {
      got = api().ctrl_pop((void*)cfg_.ctrl, &t, poll);
      check_api(got, "token pop");
    }
    check_device();
    if (!got) {  // watchdog: a worker holding weights that stays silent has failed
      const double now = now_s();
      for (int j = 0; j < cfg_.nworkers; ++j)
        if (!finished_[j] && busy_since_[j] >= 0.0 && now - busy_since_[j] > cfg_.worker_timeout_s) {
          st.code = kAsyncWatchdog;
          st.worker = j;
          st.updates = updates_;
          return st;
        }
      continue;
    }
    const auto h0 = std::chrono::steady_clock::now();
    ++tokens_;
    const int k = t.worker;
    if (k < 0 || k >= cfg_.nworkers) throw std::runtime_error("PeerServer: token from an unknown worker");
    if (t.kind == kKindError) {
      flush_batch();
      st.code = kAsyncErrorToken;
      st.worker = k;
      st.updates = updates_;
      return st;
    }
    if (finished_[k]) throw std::runtime_error("PeerServer: delta from a finished worker " + std::to_string(k));
    busy_since_[k] = -1.0;
    if (arrivals_.size() < kMaxArrivals) arrivals_.emplace_back(k, t.vc);
    int n = api().tracker_on_delta((void*)cfg_.tracker, k, t.vc, rel_k_.data(), rel_v_.data(), (int)rel_k_.size());
    check_api(n, "tracker on_delta");
    if (t.kind == kKindFinal) {  // a finished worker no longer holds the others back
      finished_[k] = 1;
      const int m = api().tracker_retire((void*)cfg_.tracker, k, rel_k_.data() + n, rel_v_.data() + n,
                                         (int)rel_k_.size() - n);
      check_api(m, "tracker retire");
      n += m;
    }
    issue(k, t.vc, rel_k_.data(), rel_v_.data(), n);
    ++updates_;
    ++updates_run_;
    host_ns_ += std::chrono::duration<double, std::nano>(std::chrono::steady_clock::now() - h0).count();
    if (checkpoint_every > 0 && updates_ % checkpoint_every == 0) {
      stop();  // (the caller reads w: the launch must have drained)
      st.code = kAsyncCheckpoint;
      st.updates = updates_;
      return st;
    }
  }
  stop();
  st.code = kAsyncDone;
  st.updates = updates_;
  return st;
}

}  // namespace psx
