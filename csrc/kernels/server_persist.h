// Persistent server kernel of the peer data plane (SSP / ASP across GPUs).
//
// Reference: ServerProcessor.process (ServerProcessor.java:143-183) -- ONE
// GRADIENTS_TOPIC partition, so each delta is applied on arrival, strictly one
// after another (w += lr * delta, :148-151, :225-228); on worker-0 deltas the
// global model is evaluated (a server row, :154-165); the workers the
// MessageTracker releases (MessageTracker.java:69-87) are sent the weights
// right after that update (:172-182).
//
// MI355X mapping (server_persist.hip, csrc/runtime/peer_server.h):
//   * the server rank's GPU runs ONE persistent launch whose 32 workgroups sit
//     on one XCD (claimed from HW_REG_XCC_ID): workgroup s owns weight slice s
//     (32 features x K classes, + the intercepts on slice 0), so every update of
//     a slice happens on one CU, in command order;
//   * the host loop (PeerServer) pops the workers' tokens, runs the C++
//     VectorClockTracker and writes one COMMAND per token into a pinned ring:
//     {worker k, its delta's tag, release mask, server-row slot}; the kernel's
//     leader polls it (one PCIe round trip per poll) and broadcasts it to the
//     slices through the XCD's L2;
//   * the delta is already in the server GPU's memory: the worker's lane wrote it
//     over xGMI into k's inbox slot (fine-grained, IPC-exported) with a tag per
//     slice (lanes_async.hip peer_push_slice); a slice waits for its tag, applies
//     w += lr * delta, and writes the new slice straight into the receive slot of
//     every released worker on ITS GPU (an IPC mapping) followed by that slot's
//     slice tag (the pull count) -- no host synchronisation, no staging, no
//     collective kernel;
//   * a logging command (the log worker's delta) also writes the global model's
//     MFMA fragments and the 32 workgroups evaluate it on the test set (the
//     server row, tagged 16-B chunks into the pinned metrics slot).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lanes_kernels.h"

namespace psx {

constexpr int kSrvWg = 32;        // workgroups of the server launch (one XCD)
// SrvCmd::k of a peer_sum BSP round (LanesArgs::push): sum the N worker RANKS' inbox slots
// (each already the sum of that rank's lanes) once all carry tag dtag, apply
// w += lr * sum, and write the new weights into every rank of relmask's receive slot with
// tag dtag (ServerProcessor.java:111-120: every worker answered once the round is complete)
constexpr int kSrvBspSum = -2;
// SrvCmd::k of a BATCH of asynchronous deltas (the tokens the host had popped when it
// wrote the command): dtag = the entry count m <= kSrvMaxBatch, relmask = the index of the
// first entry (0-based) in the pinned entry ring; log / slot_s / seq_s belong to the last
// entry (the host ends a batch at a logging delta).  Each slice applies the m deltas in
// entry order -- the single GRADIENTS_TOPIC partition's order, ServerProcessor.java:143-183
// -- and writes each entry's releases right after ITS update.
constexpr int kSrvBatch = -3;
constexpr int kSrvMaxBatch = 64;
constexpr int kEntChunks = 2;  // 32-B entries {tag, k, dtag, 0} {tag, relmask lo, relmask hi, 0}
constexpr int kSrvMaxWorkers = 64;  // the release mask's width
constexpr int kCmdChunks = 4;     // 64-B command records

struct SrvCmd {
  int stop;                      // 1: leave the launch
  int k;                         // worker whose delta is applied (-1: releases only; kSrvBspSum: a BSP round)
  unsigned dtag;                 // the delta's inbox tag (its vc + 1)
  unsigned log;                  // 1: evaluate the global model after the update (server row)
  unsigned long long relmask;    // bit j: send the weights after this command to worker j
  unsigned long long slot_s;     // pinned EvalSlot of the server row
  unsigned seq_s;
};
PSX_HD inline void pack_cmd(const SrvCmd& c, unsigned tag, TagChunk* ch) {
  ch[0] = TagChunk{tag, (unsigned)c.stop, (unsigned)c.k, c.dtag};
  ch[1] = TagChunk{tag, c.log, (unsigned)c.relmask, (unsigned)(c.relmask >> 32)};
  ch[2] = TagChunk{tag, (unsigned)c.slot_s, (unsigned)(c.slot_s >> 32), c.seq_s};
  ch[3] = TagChunk{tag, 0u, 0u, 0u};
}
PSX_HD inline void unpack_cmd(const TagChunk* ch, SrvCmd& c) {
  c.stop = (int)ch[0].a;
  c.k = (int)ch[0].b;
  c.dtag = ch[0].c;
  c.log = ch[1].a;
  c.relmask = ((unsigned long long)ch[1].c << 32) | ch[1].b;
  c.slot_s = ((unsigned long long)ch[2].b << 32) | ch[2].a;
  c.seq_s = ch[2].c;
}

struct SrvEnt {
  int k;                        // worker whose delta is applied
  unsigned dtag;                // its inbox tag (vc + 1)
  unsigned long long relmask;   // workers released right after this delta's update
};
PSX_HD inline void pack_ent(const SrvEnt& e, unsigned tag, TagChunk* ch) {
  ch[0] = TagChunk{tag, (unsigned)e.k, e.dtag, 0u};
  ch[1] = TagChunk{tag, (unsigned)e.relmask, (unsigned)(e.relmask >> 32), 0u};
}
PSX_HD inline void unpack_ent(const TagChunk* ch, SrvEnt& e) {
  e.k = (int)ch[0].a;
  e.dtag = ch[0].b;
  e.relmask = ((unsigned long long)ch[1].b << 32) | ch[1].a;
}

struct SrvArgs {
  int K, F, FP, P;
  int N;                       // workers
  float lr;
  float* w;                    // fp32 master weights [P] (server GPU)
  uint16_t *shi, *slo;         // the global model's evaluation fragments (columns 0..K-1)
  float* sb;                   // [16]
  const float* inbox;          // [N][in_stride] deltas (fine-grained, written by the workers' GPUs)
  const unsigned* inbox_tag;   // [N][FP/32] slice tags
  long long in_stride;
  float* const* rx;            // [N] worker j's receive slot [P] on its GPU (IPC mappings)
  unsigned* const* rx_tag;     // [N] its slice tags [FP/32]
  unsigned* ptag;              // [N][FP/32] pulls sent per worker and slice (this GPU)
  TagChunk* cmd;               // pinned command ring [ring][kCmdChunks]
  int ring;
  TagChunk* ent;               // pinned entry ring [ent_cap][kEntChunks] of batch commands
  int ent_cap;
  unsigned long long* erec;    // [kSrvMaxBatch * kEntChunks * 2] the batch's entries broadcast (device)
  unsigned long long cmd0;     // commands consumed before this launch
  unsigned long long* consumed_host;  // pinned: the last command read (the host's ring flow control)
  unsigned long long* err_host;  // pinned: (command << 8) | code of a timed-out wait
  const uint16_t* Xt;          // test set
  const int32_t* yt;
  int T;
  int* acc;                    // [2][256][kAccStride] evaluation accumulators (zero between passes)
  unsigned* eticket;
  unsigned long long* flags;   // [kSrvWg][32] barrier lines
  unsigned long long* rec;     // [kCmdChunks * 2] the command broadcast
  unsigned* claim;             // [2][32] role claims
  int cpar;
  int sxcd;                    // the XCD the server workgroups claim
  int nwg;                     // server workgroups (<= kSrvWg; each owns slices wg, wg + nwg, ...)
  // (tools) per command n, workgroup 0's s_memrealtime stamps at tr[(n % tr_cap) * 4 + {0 command
  // read, 1 its slices applied, 2 evaluation done, 3 the command number}]; null: off
  long long* tr;
  int tr_cap;
  long long launch;
  long long cmd_ticks;         // command wait budget (s_memrealtime ticks, 100 MHz)
  long long tag_ticks;         // inbox tag wait budget (ticks)
  int spin;                    // the workgroups' barrier budget (polls)
};

size_t server_persist_lds_bytes();
// One persistent launch on `s` (8 x nwg workgroups; those not on XCD
// a.sxcd leave at once).  The arguments travel as the kernel argument: no copy
// before the launch (it could wait behind other processes' persistent launches).
void launch_server_persist(const SrvArgs& a, int FP, hipStream_t s);

}  // namespace psx
