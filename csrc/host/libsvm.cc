#include "libsvm.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <charconv>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <thread>

#include "dataset.h"  // f32_to_bf16

namespace psx {

namespace {

struct Mapped {
  const char* data = nullptr;
  size_t size = 0;
  int fd = -1;
  explicit Mapped(const std::string& path) {
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
  ~Mapped() {
    if (data) munmap(const_cast<char*>(data), size);
    if (fd >= 0) ::close(fd);
  }
};

inline const char* skip_ws(const char* p, const char* e) {
  while (p < e && (*p == ' ' || *p == '\t' || *p == '\r')) ++p;
  return p;
}

struct Part {
  std::vector<int64_t> rowlen;
  std::vector<int32_t> idx;
  std::vector<uint16_t> val;
  std::vector<int32_t> y;
  int64_t max_feature = -1;
  std::string error;
};

void parse_range(const char* b, const char* e, bool zero_based, Part& out) {
  const char* p = b;
  int64_t line = 0;
  while (p < e) {
    const char* le = static_cast<const char*>(memchr(p, '\n', static_cast<size_t>(e - p)));
    if (!le) le = e;
    ++line;
    const char* q = skip_ws(p, le);
    if (q == le || *q == '#') {  // blank / comment line
      p = le + 1;
      continue;
    }
    double lab = 0;
    auto r = std::from_chars(q, le, lab);
    if (r.ec != std::errc()) {
      out.error = "bad label";
      return;
    }
    q = r.ptr;
    int64_t n = 0;
    while (true) {
      q = skip_ws(q, le);
      if (q >= le || *q == '#') break;
      long long f = 0;
      auto rf = std::from_chars(q, le, f);
      if (rf.ec != std::errc() || rf.ptr >= le || *rf.ptr != ':') {
        out.error = "bad feature token";
        return;
      }
      float v = 0.f;
      auto rv = std::from_chars(rf.ptr + 1, le, v);
      if (rv.ec != std::errc()) {
        out.error = "bad feature value";
        return;
      }
      q = rv.ptr;
      const long long f0 = zero_based ? f : f - 1;
      if (f0 < 0 || f0 > 0x7ffffffeLL) {
        out.error = "feature index out of range";
        return;
      }
      if (v == 0.f) continue;
      out.idx.push_back(static_cast<int32_t>(f0));
      out.val.push_back(f32_to_bf16(v));
      if (f0 > out.max_feature) out.max_feature = f0;
      ++n;
    }
    out.rowlen.push_back(n);
    out.y.push_back(static_cast<int32_t>(lab));
    p = le + 1;
  }
}

}  // namespace

SparseRows libsvm_load(const std::string& path, bool zero_based, int num_threads) {
  Mapped m(path);
  SparseRows out;
  out.indptr.push_back(0);
  if (m.size == 0) return out;
  int T = num_threads > 0 ? num_threads : static_cast<int>(std::thread::hardware_concurrency());
  if (T < 1) T = 1;
  if (static_cast<size_t>(T) > m.size / 65536 + 1) T = static_cast<int>(m.size / 65536 + 1);
  // split on line boundaries
  std::vector<const char*> cut(T + 1);
  cut[0] = m.data;
  cut[T] = m.data + m.size;
  for (int t = 1; t < T; ++t) {
    const char* c = m.data + m.size * t / T;
    if (c < cut[t - 1]) c = cut[t - 1];
    const char* nl = static_cast<const char*>(memchr(c, '\n', static_cast<size_t>(cut[T] - c)));
    cut[t] = nl ? nl + 1 : cut[T];
  }
  std::vector<Part> parts(T);
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t) th.emplace_back([&, t] { parse_range(cut[t], cut[t + 1], zero_based, parts[t]); });
  for (auto& x : th) x.join();
  size_t rows = 0, nnz = 0;
  for (auto& pt : parts) {
    if (!pt.error.empty()) throw std::runtime_error(path + ": " + pt.error);
    rows += pt.rowlen.size();
    nnz += pt.idx.size();
    if (pt.max_feature > out.max_feature) out.max_feature = pt.max_feature;
  }
  out.indptr.reserve(rows + 1);
  out.idx.reserve(nnz);
  out.val.reserve(nnz);
  out.y.reserve(rows);
  for (auto& pt : parts) {
    for (int64_t n : pt.rowlen) out.indptr.push_back(out.indptr.back() + n);
    out.idx.insert(out.idx.end(), pt.idx.begin(), pt.idx.end());
    out.val.insert(out.val.end(), pt.val.begin(), pt.val.end());
    out.y.insert(out.y.end(), pt.y.begin(), pt.y.end());
  }
  return out;
}

void libsvm_save(const std::string& path, const int64_t* indptr, const int32_t* idx, const uint16_t* val,
                 const int32_t* y, int64_t rows, bool zero_based) {
  FILE* f = std::fopen(path.c_str(), "w");
  if (!f) throw std::runtime_error("cannot write " + path);
  const int off = zero_based ? 0 : 1;
  for (int64_t r = 0; r < rows; ++r) {
    std::fprintf(f, "%d", y[r]);
    for (int64_t e = indptr[r]; e < indptr[r + 1]; ++e) {
      uint32_t u = static_cast<uint32_t>(val[e]) << 16;
      float v;
      std::memcpy(&v, &u, 4);
      std::fprintf(f, " %d:%.9g", idx[e] + off, static_cast<double>(v));
    }
    std::fputc('\n', f);
  }
  std::fclose(f);
}

}  // namespace psx
