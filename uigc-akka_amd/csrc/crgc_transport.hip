// crgc_transport.hip — shard-to-shard exchange: RCCL over xGMI, or in-process
// device copies for G logical shards on one GPU (see crgc_transport.hpp).
#include <rccl/rccl.h>

#include <chrono>
#include <cstring>
#include <new>
#include <thread>

#include "../../include/crgc.h"
#include "crgc_internal.hpp"
#include "crgc_transport.hpp"
#include "crgc_xpost.hpp"

namespace crgc {

// ---- LocalTransport ----------------------------------------------------------
// A collective's G device copies in one launch (G hipMemcpyAsync calls were
// ~2.5 us of GPU time and a dispatch each: 2 000 copies per C4 wakeup over 8
// logical shards, profiles/r5n).  Segment j: bytes [0, n) of src[j] to dst[j];
// workgroups stride over 16-B units of every segment (byte tails apart).
struct Segs {
  const char *src[TRANSPORT_MAX_SHARDS];
  char *dst[TRANSPORT_MAX_SHARDS];
  uint64_t n[TRANSPORT_MAX_SHARDS];
  uint32_t from[TRANSPORT_MAX_SHARDS];  // the shard whose buffer src points into
  uint32_t count;
};

__global__ __launch_bounds__(256) void k_copy_segs(Segs sg) {
  const uint64_t t0 = (uint64_t)blockIdx.x * 256 + threadIdx.x, stride = (uint64_t)gridDim.x * 256;
  for (uint32_t j = 0; j < sg.count; ++j) {
    const char *src = sg.src[j];
    char *dst = sg.dst[j];
    const uint64_t n = sg.n[j];
    // the widest unit both ends are aligned to (segments are 8-B aligned at least)
    const uintptr_t al = ((uintptr_t)src | (uintptr_t)dst);
    uint64_t done = 0;
    if ((al & 15) == 0) {
      done = n / 16 * 16;
      for (uint64_t i = t0; i < n / 16; i += stride) ((uint4 *)dst)[i] = ((const uint4 *)src)[i];
    } else if ((al & 7) == 0) {
      done = n / 8 * 8;
      for (uint64_t i = t0; i < n / 8; i += stride) ((uint2 *)dst)[i] = ((const uint2 *)src)[i];
    } else if ((al & 3) == 0) {
      done = n / 4 * 4;
      for (uint64_t i = t0; i < n / 4; i += stride) ((uint32_t *)dst)[i] = ((const uint32_t *)src)[i];
    }
    for (uint64_t i = done + t0; i < n; i += stride) dst[i] = src[i];
  }
}

static hipError_t copy_segs(const Segs &sg, hipStream_t s) {
  uint64_t most = 0;
  for (uint32_t j = 0; j < sg.count; ++j) most = std::max(most, sg.n[j]);
  if (!most) return hipSuccess;
  const uint64_t grid = std::min<uint64_t>(std::max<uint64_t>((most / 16 + 255) / 256, 1), 2048);
  hipLaunchKernelGGL(k_copy_segs, dim3((uint32_t)grid), dim3(256), 0, s, sg);
  return hipGetLastError();
}

// Small all-gathers' send words (counters, flags, host words) gathered into
// one buffer by one kernel: a runtime copy per part was a ~3 us blit kernel
// each (~50 per shard and C2 wakeup over 8 logical shards in a round-6 kernel trace).
// Parts are device memory or pinned host memory's device view.
struct U64Parts {
  const uint64_t *p[8];
  uint32_t n[8];
  uint32_t k;
};

__global__ __launch_bounds__(256) void k_gather_u64(U64Parts a, uint64_t *dst) {
  uint32_t off = 0;
  for (uint32_t j = 0; j < a.k; ++j) {
    for (uint32_t i = threadIdx.x; i < a.n[j]; i += 256) dst[off + i] = a.p[j][i];
    off += a.n[j];
  }
}

hipError_t gather_u64_parts(const uint64_t *const *src, const uint32_t *n, uint32_t k, uint64_t *dst,
                            hipStream_t s) {
  if (k > 8) return hipErrorInvalidValue;
  U64Parts a{};
  for (uint32_t j = 0; j < k; ++j) {
    a.p[j] = src[j];
    a.n[j] = n[j];
  }
  a.k = k;
  hipLaunchKernelGGL(k_gather_u64, dim3(1), dim3(256), 0, s, a, dst);
  return hipGetLastError();
}

// A generation barrier with a bound: a shard that never arrives (its caller
// failed before the collective) breaks the transport instead of hanging the
// others forever.  The waiters first spin (yielding) for the host-wait bound
// (CRGC_SPIN_US) on the generation, then sleep on the condition variable: a
// sleeper's wake-up costs tens of microseconds, and a sharded wakeup passes
// ~50 rendezvous (two per collective).
int LocalTransport::barrier() {
  uint64_t gen;
  {
    std::unique_lock<std::mutex> lk(m);
    if (broken) return CRGC_E_TIMEOUT;
    gen = generation;
    if (++arrived == n_shards) {
      arrived = 0;
      ++generation;
      gen_seen.store(generation, std::memory_order_release);
      cv.notify_all();
      return CRGC_OK;
    }
  }
  const auto t0 = std::chrono::steady_clock::now();
  const auto spin = std::chrono::microseconds(spin_us_default());
  while (std::chrono::steady_clock::now() - t0 < spin) {
    if (gen_seen.load(std::memory_order_acquire) != gen) return CRGC_OK;
    if (broken_seen.load(std::memory_order_acquire)) return CRGC_E_TIMEOUT;
    std::this_thread::yield();
  }
  std::unique_lock<std::mutex> lk(m);
  if (!cv.wait_for(lk, std::chrono::seconds(wait_s), [&] { return generation != gen || broken; })) {
    broken = true;
    broken_seen.store(true, std::memory_order_release);
    cv.notify_all();
  }
  return broken ? CRGC_E_TIMEOUT : CRGC_OK;
}

// Every buffer the handles pass through a transport is device memory (their
// own scratch arrays), so a kernel copies it: no runtime copy, whose
// hipMemcpyDefault form looks both pointers up in the runtime's allocation map
// (under rocprofv3's API interception two such lookups from shard threads
// faulted inside the runtime, profiles/r5n/README.md).
int LocalTransport::events(uint32_t shard) {
  Post &p = post[shard];
  if (hipGetDevice(&p.device) != hipSuccess) return DEV_FAIL("transport");
  if (!p.ready && hipEventCreateWithFlags(&p.ready, hipEventDisableTiming) != hipSuccess) return DEV_FAIL("transport");
  if (!p.done && hipEventCreateWithFlags(&p.done, hipEventDisableTiming) != hipSuccess) return DEV_FAIL("transport");
  return CRGC_OK;
}

// A collective in stream order, with no host wait (round 4 waited for the
// stream before posting and after copying: two host round trips per collective
// and shard, most of the logical-shard runs' exchange time): the shard records
// `ready` behind its send buffer's producers, every shard's stream waits for
// every peer's `ready` before its copy kernel and records `done` after it, and
// after the second rendezvous every stream waits for every peer's `done`, so
// no later work of a shard's stream overwrites a buffer a peer still reads.
// (The host threads only rendezvous: an event is waited for by the peers only
// after its record was enqueued, and recorded again only after every peer has
// enqueued that wait.)
//
// Shards on other GPUs (one handle per GPU in one process):
// a kernel here cannot read a peer GPU's memory unless peer access is enabled,
// so their segments go through the runtime's peer copy instead; segments on
// this shard's own GPU stay in the copy kernel.
int LocalTransport::collect(uint32_t shard, const Segs &sg, hipStream_t s) {
  for (uint32_t r = 0; r < n_shards; ++r)
    if (r != shard && hipStreamWaitEvent(s, post[r].ready, 0) != hipSuccess) return DEV_FAIL("transport");
  (void)hipGetLastError();  // (a soft status of an earlier call is not this launch's)
  const int mine = post[shard].device;
  Segs same{};
  for (uint32_t j = 0; j < sg.count; ++j) {
    const int dev = post[sg.from[j]].device;
    if (dev == mine) {
      same.src[same.count] = sg.src[j];
      same.dst[same.count] = sg.dst[j];
      same.n[same.count] = sg.n[j];
      same.from[same.count++] = sg.from[j];
    } else if (sg.n[j] && hipMemcpyPeerAsync(sg.dst[j], mine, sg.src[j], dev, sg.n[j], s) != hipSuccess) {
      return DEV_FAIL("transport: peer copy");
    }
  }
  if (copy_segs(same, s) != hipSuccess) return DEV_FAIL("transport");
  if (hipEventRecord(post[shard].done, s) != hipSuccess) return DEV_FAIL("transport");
  if (int rc = barrier()) return rc;
  for (uint32_t r = 0; r < n_shards; ++r)
    if (r != shard && hipStreamWaitEvent(s, post[r].done, 0) != hipSuccess) return DEV_FAIL("transport");
  return CRGC_OK;
}

int LocalTransport::allgather(uint32_t shard, const void *send, void *recv, size_t bytes,
                              hipStream_t s) {
  if (int rc = events(shard)) return rc;
  if (hipEventRecord(post[shard].ready, s) != hipSuccess) return DEV_FAIL("transport");  // send's producers
  post[shard].ptr = send;
  if (int rc = barrier()) return rc;
  Segs sg{};
  for (uint32_t r = 0; r < n_shards && bytes; ++r) {
    sg.src[sg.count] = (const char *)post[r].ptr;
    sg.dst[sg.count] = (char *)recv + (size_t)r * bytes;
    sg.from[sg.count] = r;
    sg.n[sg.count++] = bytes;
  }
  return collect(shard, sg, s);
}

int LocalTransport::alltoallv(uint32_t shard, const void *send, const size_t *soff, const size_t *sbytes,
                              void *recv, const size_t *roff, const size_t *rbytes, hipStream_t s) {
  (void)sbytes;
  if (int rc = events(shard)) return rc;
  if (hipEventRecord(post[shard].ready, s) != hipSuccess) return DEV_FAIL("transport");
  post[shard].ptr = send;
  post[shard].soff = soff;
  if (int rc = barrier()) return rc;
  Segs sg{};
  for (uint32_t r = 0; r < n_shards; ++r) {
    if (!rbytes[r]) continue;
    sg.src[sg.count] = (const char *)post[r].ptr + post[r].soff[shard];
    sg.dst[sg.count] = (char *)recv + roff[r];
    sg.from[sg.count] = r;
    sg.n[sg.count++] = rbytes[r];
  }
  return collect(shard, sg, s);  // (peers read post[*].soff before the second rendezvous)
}

// ---- RcclTransport -------------------------------------------------------------
// Error discipline (crgc_xpost.hpp): every operation of an exchange is posted
// and the group closed even after a failure, any failure aborts the
// communicator (the peers' pending operations then fail instead of waiting),
// and host waits poll the stream and the communicator's asynchronous error
// under CRGC_RCCL_TIMEOUT_S (default 300 s).  An aborted transport refuses
// every later call; the graph handles using it are poisoned by their callers.
struct RcclTransport final : crgc_transport {
  ncclComm_t comm = nullptr;
  uint32_t rank = 0;
  int device = 0;
  long timeout_s = 300;
  ~RcclTransport() override {
    if (comm) ncclCommDestroy(comm);
  }
  void abort() {
    if (comm) ncclCommAbort(comm);
    comm = nullptr;
  }
  bool accepts(uint32_t shard, int dev) const override { return shard == rank && dev == device; }
  int allgather(uint32_t, const void *send, void *recv, size_t bytes, hipStream_t s) override {
    if (!comm) return DEV_FAIL("transport");
    if (!bytes) return CRGC_OK;
    if (ncclAllGather(send, recv, bytes, ncclUint8, comm, s) == ncclSuccess) return CRGC_OK;
    abort();
    return DEV_FAIL("transport");
  }
  int alltoallv(uint32_t, const void *send, const size_t *soff, const size_t *sbytes, void *recv,
                const size_t *roff, const size_t *rbytes, hipStream_t s) override {
    if (!comm) return DEV_FAIL("transport");
    // own block: a device copy; peers: one grouped send/recv per direction
    if (rbytes[rank] &&
        hipMemcpyAsync((char *)recv + roff[rank], (const char *)send + soff[rank], rbytes[rank],
                       hipMemcpyDeviceToDevice, s) != hipSuccess) {
      abort();  // the peers' exchange with this rank is never posted: fail it for them
      return DEV_FAIL("transport");
    }
    struct Ops {
      RcclTransport *t;
      const char *sbuf;
      const size_t *soff, *sbytes;
      char *rbuf;
      const size_t *roff, *rbytes;
      hipStream_t s;
      bool group_start() { return ncclGroupStart() == ncclSuccess; }
      bool send(uint32_t r) {
        return ncclSend(sbuf + soff[r], sbytes[r], ncclUint8, (int)r, t->comm, s) == ncclSuccess;
      }
      bool recv(uint32_t r) {
        return ncclRecv(rbuf + roff[r], rbytes[r], ncclUint8, (int)r, t->comm, s) == ncclSuccess;
      }
      bool group_end() { return ncclGroupEnd() == ncclSuccess; }
      void abort() { t->abort(); }
    } ops{this, (const char *)send, soff, sbytes, (char *)recv, roff, rbytes, s};
    return post_alltoallv(ops, n_shards, rank, sbytes, rbytes);
  }
  int wait(hipStream_t s) override {
    struct Q {
      RcclTransport *t;
      hipStream_t s;
      int query() {
        const hipError_t e = hipStreamQuery(s);
        if (e == hipErrorNotReady) (void)hipGetLastError();  // a soft status: not the caller's error
        return e == hipSuccess ? 0 : (e == hipErrorNotReady ? 1 : -1);
      }
      bool async_error() {
        if (!t->comm) return true;
        ncclResult_t ae = ncclSuccess;
        if (ncclCommGetAsyncError(t->comm, &ae) != ncclSuccess) return true;
        return ae != ncclSuccess && ae != ncclInProgress;
      }
      void abort() { t->abort(); }
    } q{this, s};
    return poll_wait(q, std::chrono::seconds(timeout_s), std::chrono::microseconds(spin_us_default()));
  }
};

// ---- HostTransport -------------------------------------------------------------
// One process per shard, the exchange done by the caller's host collectives:
// every collective copies this shard's bytes to pinned host memory, calls
// back, and copies what arrived to the device (stream waits on both sides, so
// the host buffers are free again when the call returns).
struct HostTransport final : crgc_transport {
  crgc_host_collectives cb{};
  uint32_t rank = 0;
  int device = 0;
  void *hs = nullptr, *hr = nullptr;
  size_t hs_bytes = 0, hr_bytes = 0;
  ~HostTransport() override {
    if (hs) hipHostFree(hs);
    if (hr) hipHostFree(hr);
  }
  bool accepts(uint32_t shard, int dev) const override { return shard == rank && dev == device; }
  static bool grow(void *&p, size_t &have, size_t need) {
    if (need <= have) return true;
    if (p) hipHostFree(p);
    p = nullptr;
    have = 0;
    const size_t sz = need + need / 4 + 4096;
    if (hipHostMalloc(&p, sz, hipHostMallocDefault) != hipSuccess) return false;
    have = sz;
    return true;
  }
  int allgather(uint32_t, const void *send, void *recv, size_t bytes, hipStream_t s) override {
    if (!bytes) return CRGC_OK;
    if (!grow(hs, hs_bytes, bytes) || !grow(hr, hr_bytes, bytes * n_shards)) return CRGC_E_NOMEM;
    if (hipMemcpyAsync(hs, send, bytes, hipMemcpyDeviceToHost, s) != hipSuccess || stream_wait(s) != hipSuccess)
      return DEV_FAIL("transport: staging");
    if (cb.allgather(cb.ctx, rank, hs, hr, bytes) != 0) return DEV_FAIL("transport: host all-gather");
    if (hipMemcpyAsync(recv, hr, bytes * n_shards, hipMemcpyHostToDevice, s) != hipSuccess ||
        stream_wait(s) != hipSuccess)
      return DEV_FAIL("transport: staging");
    return CRGC_OK;
  }
  int alltoallv(uint32_t, const void *send, const size_t *soff, const size_t *sbytes, void *recv,
                const size_t *roff, const size_t *rbytes, hipStream_t s) override {
    size_t sn = 0, rn = 0;
    for (uint32_t r = 0; r < n_shards; ++r) {
      if (sbytes[r]) sn = std::max(sn, soff[r] + sbytes[r]);
      if (rbytes[r]) rn = std::max(rn, roff[r] + rbytes[r]);
    }
    if (!grow(hs, hs_bytes, sn + 1) || !grow(hr, hr_bytes, rn + 1)) return CRGC_E_NOMEM;
    if (sn && (hipMemcpyAsync(hs, send, sn, hipMemcpyDeviceToHost, s) != hipSuccess || stream_wait(s) != hipSuccess))
      return DEV_FAIL("transport: staging");
    if (cb.alltoallv(cb.ctx, rank, hs, soff, sbytes, hr, roff, rbytes) != 0)
      return DEV_FAIL("transport: host all-to-all");
    if (rn && (hipMemcpyAsync(recv, hr, rn, hipMemcpyHostToDevice, s) != hipSuccess || stream_wait(s) != hipSuccess))
      return DEV_FAIL("transport: staging");
    return CRGC_OK;
  }
};

int rccl_unique_id(uint8_t id[128]) {
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId is 128 bytes");
  ncclUniqueId u;
  if (ncclGetUniqueId(&u) != ncclSuccess) return DEV_FAIL("transport");
  memcpy(id, &u, 128);
  return CRGC_OK;
}

crgc_transport *make_rccl_transport(const uint8_t id[128], uint32_t n_shards, uint32_t shard, int device,
                                    int *rc) {
  RcclTransport *t = new (std::nothrow) RcclTransport();
  if (!t) {
    *rc = CRGC_E_NOMEM;
    return nullptr;
  }
  t->n_shards = n_shards;
  t->rank = shard;
  t->device = device;
  if (const char *e = getenv("CRGC_RCCL_TIMEOUT_S")) t->timeout_s = std::max(1L, atol(e));
  int prev = 0;
  hipGetDevice(&prev);
  hipSetDevice(device);
  ncclUniqueId u;
  memcpy(&u, id, 128);
  const ncclResult_t r = ncclCommInitRank(&t->comm, (int)n_shards, u, (int)shard);
  hipSetDevice(prev);
  if (r != ncclSuccess) {
    t->comm = nullptr;
    delete t;
    *rc = DEV_FAIL("transport");
    return nullptr;
  }
  *rc = CRGC_OK;
  return t;
}

}  // namespace crgc

extern "C" {

int crgc_transport_local(uint32_t n_shards, crgc_transport **out) {
  if (!out || n_shards < 1 || n_shards > crgc::TRANSPORT_MAX_SHARDS) return CRGC_E_INVAL;
  *out = new (std::nothrow) crgc::LocalTransport(n_shards);
  return *out ? CRGC_OK : CRGC_E_NOMEM;
}

int crgc_transport_rccl_id(uint8_t id[128]) {
  if (!id) return CRGC_E_INVAL;
  return crgc::rccl_unique_id(id);
}

int crgc_transport_rccl(const uint8_t id[128], uint32_t n_shards, uint32_t shard, int32_t device,
                        crgc_transport **out) {
  if (!out || !id || n_shards < 1 || n_shards > crgc::TRANSPORT_MAX_SHARDS || shard >= n_shards)
    return CRGC_E_INVAL;
  int rc = CRGC_OK;
  *out = crgc::make_rccl_transport(id, n_shards, shard, device, &rc);
  return rc;
}

int crgc_transport_host(const crgc_host_collectives *c, uint32_t n_shards, uint32_t shard, int32_t device,
                        crgc_transport **out) {
  if (!out || !c || !c->allgather || !c->alltoallv || n_shards < 1 || n_shards > crgc::TRANSPORT_MAX_SHARDS ||
      shard >= n_shards)
    return CRGC_E_INVAL;
  crgc::HostTransport *t = new (std::nothrow) crgc::HostTransport();
  if (!t) return CRGC_E_NOMEM;
  t->cb = *c;
  t->n_shards = n_shards;
  t->rank = shard;
  t->device = device;
  *out = t;
  return CRGC_OK;
}

void crgc_transport_destroy(crgc_transport *t) { delete t; }

uint32_t crgc_shard_of(uint64_t id, uint32_t n_shards) {
  return n_shards <= 1 ? 0u : crgc::shard_of(id, n_shards);
}

}  // extern "C"
