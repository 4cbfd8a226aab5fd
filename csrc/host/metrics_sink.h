// Native evaluation-record sink: device kernels deposit confusion counts (and
// the worker's training loss) straight into pinned host slots and publish a
// sequence number; a background thread waits for each slot's number, computes
// the reference's metrics (Spark MulticlassMetrics weighted F1 + accuracy,
// Metrics.java:15-24) and hands the row to the CsvLogger.  The training loop
// pays one slot reservation and one submit per record -- no copies, events or
// per-record Python work.
//
// Row semantics: worker rows carry (ts, partition, vectorClock, loss, f1,
// accuracy, numTuplesSeen) of the LOCALLY trained model
// (LogisticRegressionTaskSpark.java:186-211, WorkerAppRunner.java:77-81);
// server rows (ts, -1, vectorClock, -1, f1, accuracy) of the global model
// (ServerProcessor.java:154-165).
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>

#include "logger.h"
#include "sink_record.h"

namespace psx {

// One record's device-written payload (host memory, device-visible).
struct EvalSlot {
  int32_t conf[256];  // [true 16][pred 16]
  float loss;
  uint32_t pad0;
  uint64_t seq;       // written last (system-scope release) by the producer
  uint64_t pad1[6];
};
static_assert(sizeof(EvalSlot) == 1088, "EvalSlot layout is shared with the device");

// (weighted F1, accuracy) of a [K][K] block of a 16x16 confusion matrix.
void weighted_f1_accuracy(const int32_t* conf16, int K, double* f1, double* acc);

// Row timestamps: epoch milliseconds.  A record submitted with ts < 0 is stamped
// by the sink thread when it observes the record's evaluation complete (us
// resolution; the CSV keeps the reference's integer milliseconds).
struct WorkerRow {
  double ts;
  int64_t partition, vc;
  double loss, f1, acc;
  int64_t nseen;
};
struct ServerRow {
  double ts;
  int64_t vc;
  double f1, acc;
};


class MetricsSink {
 public:
  // slots: nslots EvalSlot records (host pointer).  Loggers may be null.
  MetricsSink(uintptr_t slots, int nslots, int K, CsvLogger* wlog, CsvLogger* slog, bool keep_records);
  ~MetricsSink();
  MetricsSink(const MetricsSink&) = delete;
  MetricsSink& operator=(const MetricsSink&) = delete;

  // Reserve a slot (blocks while every slot is in flight); returns its index
  // and the sequence number the producer must publish.
  int acquire(uint64_t* seq);
  uintptr_t slot_address(int slot) const;
  // n slots at once (one lock; blocks until n are free, n <= nslots).
  void acquire_many(int n, int* slots, uint64_t* seqs);
  // kind 0 = worker row, 1 = server row (| kSinkTagged: tagged-chunk payload).
  void submit(int slot, uint64_t seq, int kind, int64_t ts, int64_t partition, int64_t vc, int64_t nseen);
  // n records in order, one lock and one wake-up of the logger thread (a round of
  // the lanes loop hands over up to 9 rows)
  void submit_many(int n, const SinkRecord* recs);
  // Wait until every submitted record has been processed (timeout_s <= 0: forever).
  bool flush(double timeout_s = 0.0);
  void close();
  int64_t processed() const { return processed_.load(); }
  std::vector<WorkerRow> worker_rows();
  std::vector<ServerRow> server_rows();

 private:
  struct Pending {
    int slot;
    uint64_t seq;
    int kind;
    int64_t ts, partition, vc, nseen;
  };
  void run();
  // a kSinkTagged slot complete for `seq`: counts -> conf16 [16][16], loss
  bool read_tagged(const EvalSlot& s, uint64_t seq, int32_t* conf16, float* loss) const;
  EvalSlot* slots_;
  int nslots_, K_;
  CsvLogger *wlog_, *slog_;
  bool keep_;
  uint64_t next_seq_ = 1;
  std::mutex mu_;
  std::condition_variable cv_work_, cv_free_, cv_done_;
  std::deque<Pending> pending_;
  std::vector<int> free_;
  int64_t submitted_ = 0;
  std::atomic<int64_t> processed_{0};
  bool stop_ = false;
  std::vector<WorkerRow> wrows_;
  std::vector<ServerRow> srows_;
  std::thread th_;
};

}  // namespace psx
