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

}  // namespace psx
