// Dataset ingest: multithreaded mmap CSV parser, binary row cache, and the
// producer arrival schedule.
//
// Reference behaviour being reproduced (reference:
// src/main/java/de/hpi/datastreams/producer/CsvProducer.java:36-87):
//   * optional header line skipped; the LAST column is the integer label,
//     all other columns are features (zeros are simply zeros in a dense row);
//   * rows are dealt round-robin: row r belongs to worker r % N;
//   * rate control: after a warm-up burst of N*128 rows the producer sleeps
//     1 s every floor(1000/p) rows, i.e. ~floor(1000/p) rows/s in total.
// Differences by design: the width is inferred from the file instead of being
// hard-coded to 1024 (quirk Q10), malformed rows are hard errors (Q11), p=0
// means unthrottled and p>1000 means one row every p ms (Q5).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace psx {

struct CsvInfo {
  int64_t rows = 0;        // data rows (header excluded)
  int64_t cols = 0;        // total columns including the label
  bool header = false;
  std::vector<std::string> names;  // header names when present
};

// header_mode: 0 = auto-detect, 1 = has header, 2 = no header.
CsvInfo csv_probe(const std::string& path, int header_mode);

// Parse every row. Features go to `X` (rows x num_features, row-major) as
// float32 (x_f32 != nullptr) and/or bf16 bit patterns (x_bf16 != nullptr), with
// rows padded to `row_stride` elements (zero-filled).  label_col < 0 means last.
void csv_load(const std::string& path, const CsvInfo& info, int label_col, int64_t row_stride,
              float* x_f32, uint16_t* x_bf16, int32_t* labels, int num_threads);

// Arrival time (ms since producer start) of global row r under `-p p_ms`.
double arrival_time_ms(int64_t r, int num_workers, double p_ms);

// Rows of worker `k` (r = k, k+N, ...) that have arrived by `now_ms`, starting
// from the worker-local cursor `next_local` (index into that worker's row list).
// Returns how many of them (capped at max_rows) are due; `times_out` receives
// their scheduled arrival times when non-null.
int64_t due_rows(int k, int num_workers, double p_ms, int64_t total_rows, int64_t next_local,
                 double now_ms, int64_t max_rows, double* times_out);

uint16_t f32_to_bf16(float f);

}  // namespace psx
