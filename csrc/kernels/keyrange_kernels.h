// Key-range sharded parameter server kernels (BASELINE.json config 5).
//
// Reference: every message carries the KeyRange of the weights it holds
// (BaseMessage.java:24-27, KeyRange.java:11-49) so that a server can own a
// range of the key space.  Here rank j owns features [j*S, min(F, (j+1)*S)) of
// the wide model: its shard [(hi-lo)*KP] of coefficients lives only in its HBM;
// workers pull the coefficients of the features their next window touches and
// push deltas for exactly those features (csrc/runtime/keyrange_loop.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace psx {

// out[i*KP + c] = shard[(ids[i] - lo)*KP + c] for i < n (n = *n_dev, or n_host
// when n_dev is null).  The owner's answer to a pull request.
void launch_kr_gather(const float* shard, int64_t lo, int KP, const int32_t* ids, const unsigned* n_dev, int n_host,
                      float* out, int nmax, hipStream_t s);
// shard[(ids[i] - lo)*KP + c] += lr * vals[i*KP + c] for i < n; block 0 also
// does b[c] += lr * db[c] when db is given (the replicated intercepts).
void launch_kr_apply(float* shard, int64_t lo, int KP, const int32_t* ids, const unsigned* n_dev, int n_host,
                     const float* vals, float lr, float* b, const float* db, int nmax, hipStream_t s);

// The round's evaluation rows from maintained margins (no pass over the
// sharded model):
//  * worker row: zw = z[r] + sum over the row's window features of
//    v * dloc[KP + l*KP] (the solver's table maps f -> l) + wloc_b -> confusion
//    into `slot` with the solver's loss; dz[r] = that window sum (this worker's
//    share of the global margin update).  htab == nullptr: no worker row, dz = 0.
void launch_kr_worker_rows(int K, int KP, const int64_t* indptr, const int32_t* idx, const uint16_t* val,
                           const int32_t* y, int T, const float* z, const int2* htab, unsigned hmask,
                           const float* dloc, const float* wloc_b, float* dz, int* acc, unsigned* ticket, void* slot,
                           const float* loss, unsigned long long seq, hipStream_t s);
//  * server row: z += lr * dz (dz all-reduced over the ranks: every worker's
//    delta), then the confusion of z + b into `slot` (null: the update only).
void launch_kr_server_rows(int K, int KP, const int32_t* y, int T, float* z, const float* dz, float lr, const float* b,
                           int* acc, unsigned* ticket, void* slot, unsigned long long seq, hipStream_t s);

}  // namespace psx
