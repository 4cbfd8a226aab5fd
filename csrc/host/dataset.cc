#include "dataset.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <charconv>
#include <cmath>
#include <cstring>
#include <stdexcept>
#include <thread>

namespace psx {

namespace {

struct MappedFile {
  const char* data = nullptr;
  size_t size = 0;
  int fd = -1;
  explicit MappedFile(const std::string& path) {
    fd = ::open(path.c_str(), O_RDONLY);
    if (fd < 0) throw std::runtime_error("cannot open " + path);
    struct stat st;
    if (fstat(fd, &st) != 0) throw std::runtime_error("cannot stat " + path);
    size = static_cast<size_t>(st.st_size);
    if (size > 0) {
      void* p = mmap(nullptr, size, PROT_READ, MAP_PRIVATE, fd, 0);
      if (p == MAP_FAILED) throw std::runtime_error("cannot mmap " + path);
      madvise(p, size, MADV_SEQUENTIAL);
      data = static_cast<const char*>(p);
    }
  }
  ~MappedFile() {
    if (data) munmap(const_cast<char*>(data), size);
    if (fd >= 0) ::close(fd);
  }
};

inline const char* line_end(const char* p, const char* e) {
  const void* q = memchr(p, '\n', static_cast<size_t>(e - p));
  return q ? static_cast<const char*>(q) : e;
}

inline const char* trim_cr(const char* b, const char* e) {
  while (e > b && (e[-1] == '\r' || e[-1] == ' ')) --e;
  return e;
}

bool token_is_number(const char* b, const char* e) {
  while (b < e && *b == ' ') ++b;
  if (b == e) return false;
  double v;
  auto r = std::from_chars(b, e, v);
  return r.ec == std::errc() && r.ptr == e;
}

int64_t count_cols(const char* b, const char* e) {
  if (b == e) return 0;
  return 1 + std::count(b, e, ',');
}

}  // namespace

uint16_t f32_to_bf16(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return static_cast<uint16_t>((u >> 16) | 0x40);  // NaN
  u += 0x7fffu + ((u >> 16) & 1u);  // round to nearest even
  return static_cast<uint16_t>(u >> 16);
}

CsvInfo csv_probe(const std::string& path, int header_mode) {
  MappedFile f(path);
  CsvInfo info;
  const char* p = f.data;
  const char* e = f.data + f.size;
  if (f.size == 0) return info;
  const char* le = line_end(p, e);
  const char* te = trim_cr(p, le);
  info.cols = count_cols(p, te);
  bool hdr;
  if (header_mode == 1)
    hdr = true;
  else if (header_mode == 2)
    hdr = false;
  else {  // auto: a header has at least one non-numeric token
    hdr = false;
    const char* b = p;
    while (b <= te) {
      const char* c = static_cast<const char*>(memchr(b, ',', static_cast<size_t>(te - b)));
      const char* tend = c ? c : te;
      if (!token_is_number(b, tend)) {
        hdr = true;
        break;
      }
      if (!c) break;
      b = c + 1;
    }
  }
  info.header = hdr;
  if (hdr) {
    const char* b = p;
    while (true) {
      const char* c = static_cast<const char*>(memchr(b, ',', static_cast<size_t>(te - b)));
      const char* tend = c ? c : te;
      info.names.emplace_back(b, tend);
      if (!c) break;
      b = c + 1;
    }
    p = le < e ? le + 1 : e;
  }
  int64_t rows = 0;
  while (p < e) {
    const char* l = line_end(p, e);
    if (trim_cr(p, l) > p) ++rows;
    p = l < e ? l + 1 : e;
  }
  info.rows = rows;
  return info;
}

void csv_load(const std::string& path, const CsvInfo& info, int label_col, int64_t row_stride, float* x_f32,
              uint16_t* x_bf16, int32_t* labels, int num_threads) {
  MappedFile f(path);
  const char* e = f.data + f.size;
  const char* p = f.data;
  if (info.header) {
    const char* le = line_end(p, e);
    p = le < e ? le + 1 : e;
  }
  const int64_t cols = info.cols;
  const int64_t nfeat = cols - 1;
  const int64_t lab = label_col < 0 ? cols - 1 : label_col;
  if (lab >= cols) throw std::invalid_argument("label column out of range");
  if (row_stride < nfeat) throw std::invalid_argument("row_stride smaller than feature count");

  // Line index (single pass; memchr is memory-bound, parsing dominates).
  std::vector<const char*> starts;
  starts.reserve(static_cast<size_t>(info.rows) + 1);
  while (p < e) {
    const char* l = line_end(p, e);
    if (trim_cr(p, l) > p) starts.push_back(p);
    p = l < e ? l + 1 : e;
  }
  if (static_cast<int64_t>(starts.size()) != info.rows)
    throw std::runtime_error("csv changed between probe and load");

  if (num_threads <= 0) num_threads = static_cast<int>(std::max(1u, std::thread::hardware_concurrency()));
  num_threads = static_cast<int>(std::min<int64_t>(num_threads, std::max<int64_t>(1, info.rows / 64)));
  std::vector<std::string> errors(num_threads);

  auto work = [&](int t) {
    int64_t r0 = info.rows * t / num_threads, r1 = info.rows * (t + 1) / num_threads;
    for (int64_t r = r0; r < r1; ++r) {
      const char* b = starts[r];
      const char* le = trim_cr(b, line_end(b, e));
      float* xf = x_f32 ? x_f32 + r * row_stride : nullptr;
      uint16_t* xb = x_bf16 ? x_bf16 + r * row_stride : nullptr;
      int64_t col = 0, fi = 0;
      while (true) {
        const char* c = static_cast<const char*>(memchr(b, ',', static_cast<size_t>(le - b)));
        const char* tend = c ? c : le;
        const char* tb = b;
        while (tb < tend && *tb == ' ') ++tb;
        if (col == lab) {
          double v = 0;
          auto res = std::from_chars(tb, tend, v);
          if (res.ec != std::errc()) {
            errors[t] = "row " + std::to_string(r) + ": bad label";
            return;
          }
          labels[r] = static_cast<int32_t>(std::lround(v));
        } else {
          float v = 0.f;
          if (tb < tend) {
            auto res = std::from_chars(tb, tend, v);
            if (res.ec != std::errc()) {
              errors[t] = "row " + std::to_string(r) + " col " + std::to_string(col) + ": bad number";
              return;
            }
          }
          if (fi < nfeat) {
            if (xf) xf[fi] = v;
            if (xb) xb[fi] = f32_to_bf16(v);
          }
          ++fi;
        }
        ++col;
        if (!c) break;
        b = c + 1;
      }
      if (col != cols) {
        errors[t] = "row " + std::to_string(r) + " has " + std::to_string(col) + " columns, expected " +
                    std::to_string(cols);
        return;
      }
      for (int64_t j = nfeat; j < row_stride; ++j) {
        if (xf) xf[j] = 0.f;
        if (xb) xb[j] = 0;
      }
    }
  };
  std::vector<std::thread> th;
  for (int t = 1; t < num_threads; ++t) th.emplace_back(work, t);
  work(0);
  for (auto& x : th) x.join();
  for (auto& s : errors)
    if (!s.empty()) throw std::runtime_error(path + ": " + s);
}

double arrival_time_ms(int64_t r, int num_workers, double p_ms) {
  if (p_ms <= 0) return 0.0;
  const int64_t burst = static_cast<int64_t>(num_workers) * 128;
  if (p_ms > 1000.0) return r < burst ? 0.0 : static_cast<double>(r - burst + 1) * p_ms;
  const int64_t q = static_cast<int64_t>(std::floor(1000.0 / p_ms));
  // the producer sleeps 1 s after sending the m-th row whenever m >= burst and m % q == 0;
  // row r is sent after rows 0..r-1, i.e. after counts m = 1..r.
  const int64_t a = std::max<int64_t>(1, burst), b = r;
  if (b < a) return 0.0;
  const int64_t sleeps = b / q - (a - 1) / q;
  return 1000.0 * static_cast<double>(sleeps);
}

int64_t due_rows(int k, int num_workers, double p_ms, int64_t total_rows, int64_t next_local, double now_ms,
                 int64_t max_rows, double* times_out) {
  // local row j <-> global row k + j*N; count local rows total for this worker
  const int64_t N = num_workers;
  int64_t local_total = total_rows > k ? (total_rows - k + N - 1) / N : 0;
  int64_t hi = std::min(local_total, next_local + max_rows);
  if (next_local >= hi) return 0;
  // arrival time is monotone in the row index: binary search the last due row
  int64_t lo = next_local, up = hi;  // find first j in [lo, up) with t > now
  while (lo < up) {
    int64_t mid = lo + (up - lo) / 2;
    if (arrival_time_ms(k + mid * N, num_workers, p_ms) <= now_ms)
      lo = mid + 1;
    else
      up = mid;
  }
  int64_t n = lo - next_local;
  if (times_out)
    for (int64_t j = 0; j < n; ++j) times_out[j] = arrival_time_ms(k + (next_local + j) * N, num_workers, p_ms);
  return n;
}

}  // namespace psx
