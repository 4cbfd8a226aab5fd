// CSV evaluation logger with the reference's exact schema.
//
// Reference: ServerAppRunner.java:78-82 / WorkerAppRunner.java:77-81 write
//   server: timestamp;partition;vectorClock;loss;fMeasure;accuracy
//   worker: timestamp;partition;vectorClock;loss;fMeasure;accuracy;numTuplesSeen
// with epoch-ms timestamps and java.lang.Double.toString values
// (ServerProcessor.java:154-165, WorkerTrainingProcessor.java:80-92).
// Records are appended under a short mutex and written by a background thread,
// so the training loop never blocks on file I/O.
#pragma once
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace psx {

// java.lang.Double.toString formatting (shortest round-trip digits).
std::string java_double(double v);

class CsvLogger {
 public:
  // path empty => stdout.  `worker_schema` selects the 7-column header.
  CsvLogger(const std::string& path, bool worker_schema, bool write_header, bool append = false);
  ~CsvLogger();
  void log_worker(int64_t ts_ms, int64_t partition, int64_t vc, double loss, double f1, double acc,
                  int64_t tuples_seen);
  // server rows carry partition -1 and loss -1 (reference ServerProcessor.java:159-164)
  void log_server(int64_t ts_ms, int64_t vc, double f1, double acc);
  void log_line(const std::string& line);
  void flush();
  void close();
  int64_t lines() const { return lines_; }

 private:
  void run();
  FILE* f_ = nullptr;
  bool own_ = false;
  std::mutex mu_;
  std::condition_variable cv_;
  std::string pending_;
  bool stop_ = false;
  bool flush_req_ = false;
  int64_t lines_ = 0;
  std::thread th_;
};

}  // namespace psx
