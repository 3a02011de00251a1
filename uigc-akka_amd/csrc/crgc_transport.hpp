// crgc_transport.hpp — the data-movement layer between the shards of a
// hash-partitioned shadow graph.
//
// Two implementations behind one interface:
//   RcclTransport   one process per GPU, RCCL over xGMI (ncclAllGather and
//                   grouped ncclSend/ncclRecv), stream-ordered on the graph's
//                   stream.  This is the production transport.
//   LocalTransport  the G shards live in one process, each driven by its own
//                   host thread; the exchange is device-to-device copies
//                   through a shared rendezvous.  It lets G logical shards run
//                   on one GPU, which is how the sharded protocol is
//                   parity-tested on a single-GPU box.
// Every call is collective: all G shards make the same calls in the same
// order.  Buffers are device buffers; sizes are bytes.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <cstddef>
#include <cstdint>
#include <mutex>

#include "crgc_internal.hpp"

struct crgc_transport {
  uint32_t n_shards = 1;
  virtual ~crgc_transport() = default;
  // Whether `shard` may be driven through this transport (RCCL: its own rank).
  virtual bool accepts(uint32_t shard, int device) const = 0;
  // recv[r*bytes .. (r+1)*bytes) = shard r's send[0 .. bytes)
  virtual int allgather(uint32_t shard, const void *send, void *recv, size_t bytes, hipStream_t s) = 0;
  // shard me sends send[soff[r] .. +sbytes[r]) to r and receives r's block
  // for it into recv[roff[r] .. +rbytes[r]).  rbytes[r] must equal r's sbytes[me].
  virtual int alltoallv(uint32_t shard, const void *send, const size_t *soff, const size_t *sbytes,
                        void *recv, const size_t *roff, const size_t *rbytes, hipStream_t s) = 0;
  // Host wait for the graph's stream.  RCCL: bounded, and ended early by the
  // communicator's asynchronous error, so a failed or hung peer cannot block
  // this rank forever (crgc_xpost.hpp).
  virtual int wait(hipStream_t s) { return crgc::stream_wait(s) == hipSuccess ? 0 : -3; }
};

namespace crgc {

constexpr uint32_t TRANSPORT_MAX_SHARDS = 64;

struct Segs;  // a collective's copies (crgc_transport.hip)

// One process, one host thread per shard.
struct LocalTransport final : crgc_transport {
  struct Post {
    const void *ptr = nullptr;
    const size_t *soff = nullptr;
    // stream order across the shards' streams, without host waits: `ready`
    // recorded behind the send buffer's producers, `done` behind this shard's
    // copies out of its peers' buffers (created by the shard's own thread)
    hipEvent_t ready = nullptr, done = nullptr;
    int device = 0;  // the GPU of the shard's handle (read at every collective)
  };
  std::mutex m;
  std::condition_variable cv;
  uint32_t arrived = 0;
  uint64_t generation = 0;
  bool broken = false;
  // generation / broken for the waiters' spin phase (stored under m)
  std::atomic<uint64_t> gen_seen{0};
  std::atomic<bool> broken_seen{false};
  Post post[TRANSPORT_MAX_SHARDS];

  // A shard that never arrives (its caller failed before the collective)
  // breaks the transport after wait_s seconds (CRGC_LOCAL_BARRIER_S, default 60).
  long wait_s = 60;

  explicit LocalTransport(uint32_t g) {
    n_shards = g;
    if (const char *e = getenv("CRGC_LOCAL_BARRIER_S")) wait_s = std::max(1L, atol(e));
  }
  bool accepts(uint32_t shard, int) const override { return shard < n_shards; }
  int barrier();
  int events(uint32_t shard);  // the shard's two events, created on first use
  int collect(uint32_t shard, const Segs &sg, hipStream_t s);
  ~LocalTransport() override {
    for (uint32_t r = 0; r < TRANSPORT_MAX_SHARDS; ++r) {
      if (post[r].ready) hipEventDestroy(post[r].ready);
      if (post[r].done) hipEventDestroy(post[r].done);
    }
  }
  int allgather(uint32_t shard, const void *send, void *recv, size_t bytes, hipStream_t s) override;
  int alltoallv(uint32_t shard, const void *send, const size_t *soff, const size_t *sbytes, void *recv,
                const size_t *roff, const size_t *rbytes, hipStream_t s) override;
};

// One kernel gathering k <= 8 parts of u64 words (device or pinned-host views) into dst.
hipError_t gather_u64_parts(const uint64_t *const *src, const uint32_t *n, uint32_t k, uint64_t *dst,
                            hipStream_t s);

// Created by crgc_transport_rccl (crgc_transport.hip); RCCL types stay there.
crgc_transport *make_rccl_transport(const uint8_t id[128], uint32_t n_shards, uint32_t shard,
                                    int device, int *rc);
int rccl_unique_id(uint8_t id[128]);

}  // namespace crgc
