#include "logger.h"

#include <charconv>
#include <cmath>
#include <cstring>
#include <stdexcept>

namespace psx {

std::string java_double(double v) {
  if (std::isnan(v)) return "NaN";
  if (std::isinf(v)) return v > 0 ? "Infinity" : "-Infinity";
  if (v == 0.0) return std::signbit(v) ? "-0.0" : "0.0";
  // shortest round-trip digits in scientific form: d.dddde[+-]XX
  char buf[64];
  auto r = std::to_chars(buf, buf + sizeof(buf), v, std::chars_format::scientific);
  std::string s(buf, r.ptr);
  bool neg = s[0] == '-';
  if (neg) s.erase(0, 1);
  size_t epos = s.find('e');
  int exp10 = std::stoi(s.substr(epos + 1));
  std::string mant = s.substr(0, epos);
  std::string digits;
  for (char c : mant)
    if (c != '.') digits.push_back(c);
  while (digits.size() > 1 && digits.back() == '0') digits.pop_back();
  std::string out;
  double a = std::fabs(v);
  if (a >= 1e-3 && a < 1e7) {
    int point = exp10 + 1;  // digits before the decimal point
    if (point <= 0) {
      out = "0." + std::string(static_cast<size_t>(-point), '0') + digits;
    } else if (static_cast<size_t>(point) >= digits.size()) {
      out = digits + std::string(static_cast<size_t>(point) - digits.size(), '0') + ".0";
    } else {
      out = digits.substr(0, static_cast<size_t>(point)) + "." + digits.substr(static_cast<size_t>(point));
    }
  } else {
    out = digits.substr(0, 1) + "." + (digits.size() > 1 ? digits.substr(1) : std::string("0")) + "E" +
          std::to_string(exp10);
  }
  return neg ? "-" + out : out;
}

static const char* header(bool worker_schema) {
  return worker_schema ? "timestamp;partition;vectorClock;loss;fMeasure;accuracy;numTuplesSeen\n"
                       : "timestamp;partition;vectorClock;loss;fMeasure;accuracy\n";
}

CsvLogger::CsvLogger(const std::string& path, bool worker_schema, bool write_header, bool append) {
  if (path.empty()) {
    f_ = stdout;
  } else {
    // append mode: several worker processes share one file; every write() is
    // a run of whole lines on an O_APPEND descriptor, so lines never interleave
    // A creating logger truncates, writes the header at once and continues on an
    // O_APPEND descriptor too: ranks that open the file later append after the
    // header, and nobody's lines overwrite another's.
    f_ = std::fopen(path.c_str(), append ? "a" : "w");
    if (!f_) throw std::runtime_error("cannot open log file " + path);
    own_ = true;
    if (!append) {
      if (write_header) std::fputs(header(worker_schema), f_);
      std::fclose(f_);
      f_ = std::fopen(path.c_str(), "a");
      if (!f_) throw std::runtime_error("cannot reopen log file " + path);
      write_header = false;
    }
  }
  if (write_header) pending_ = header(worker_schema);
  th_ = std::thread(&CsvLogger::run, this);
}

CsvLogger::~CsvLogger() { close(); }

void CsvLogger::log_line(const std::string& line) {
  std::lock_guard<std::mutex> g(mu_);
  pending_ += line;
  pending_.push_back('\n');
  ++lines_;
  if (pending_.size() > (1u << 16)) cv_.notify_one();
}

void CsvLogger::log_worker(int64_t ts, int64_t part, int64_t vc, double loss, double f1, double acc,
                           int64_t seen) {
  std::string l = std::to_string(ts) + ";" + std::to_string(part) + ";" + std::to_string(vc) + ";" +
                  java_double(loss) + ";" + java_double(f1) + ";" + java_double(acc) + ";" + std::to_string(seen);
  log_line(l);
}

void CsvLogger::log_server(int64_t ts, int64_t vc, double f1, double acc) {
  std::string l = std::to_string(ts) + ";-1;" + std::to_string(vc) + ";-1;" + java_double(f1) + ";" +
                  java_double(acc);
  log_line(l);
}

void CsvLogger::flush() {
  std::unique_lock<std::mutex> g(mu_);
  flush_req_ = true;
  cv_.notify_one();
  cv_.wait(g, [&] { return !flush_req_ || stop_; });
}

void CsvLogger::run() {
  std::unique_lock<std::mutex> g(mu_);
  for (;;) {
    // system_clock deadline: pthread_cond_timedwait (the steady_clock form maps
    // to pthread_cond_clockwait, which the toolchain's TSAN does not model)
    cv_.wait_until(g, std::chrono::system_clock::now() + std::chrono::milliseconds(200),
                   [&] { return stop_ || flush_req_ || pending_.size() > (1u << 16); });
    std::string out;
    out.swap(pending_);
    bool fl = flush_req_;
    bool st = stop_;
    g.unlock();
    if (!out.empty()) std::fwrite(out.data(), 1, out.size(), f_);
    if (fl || st || !out.empty()) std::fflush(f_);
    g.lock();
    if (fl) {
      flush_req_ = false;
      cv_.notify_all();
    }
    if (st && pending_.empty()) break;
  }
}

void CsvLogger::close() {
  {
    std::lock_guard<std::mutex> g(mu_);
    if (stop_) return;
    stop_ = true;
    cv_.notify_all();
  }
  if (th_.joinable()) th_.join();
  if (own_ && f_) std::fclose(f_);
  f_ = nullptr;
}

}  // namespace psx
