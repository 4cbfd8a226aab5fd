// Sparse dataset ingest: multithreaded mmap parser of the LIBSVM text format
//   <label> <feature>:<value> <feature>:<value> ...
// into CSR (indptr int64, idx int32, val bf16, labels int32).
//
// The reference's producer turns every CSV row into a sparse map of its
// non-zero columns before sending it (reference:
// src/main/java/de/hpi/datastreams/producer/CsvProducer.java:47-58); for the
// 10^6..10^8-feature configs the rows are stored sparse on disk as well.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace psx {

struct SparseRows {
  std::vector<int64_t> indptr;
  std::vector<int32_t> idx;
  std::vector<uint16_t> val;  // bf16 bit patterns
  std::vector<int32_t> y;
  int64_t max_feature = -1;   // largest (0-based) feature index seen
};

// zero_based: feature ids in the file start at 0 (else 1, LIBSVM's default).
// Entries of a row are kept in file order; explicit zeros are dropped.
SparseRows libsvm_load(const std::string& path, bool zero_based, int num_threads);

// Write CSR rows as LIBSVM text (tests, tools).  val is bf16.
void libsvm_save(const std::string& path, const int64_t* indptr, const int32_t* idx, const uint16_t* val,
                 const int32_t* y, int64_t rows, bool zero_based);

}  // namespace psx
