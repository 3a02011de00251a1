// crgc_xpost.hpp — the error discipline of a shard exchange, independent of
// the library that moves the bytes (RCCL in crgc_transport.hip; a fake in
// tests/xpost_fake.cpp, which checks it on the CPU).
//
// A collective that fails on one rank must not leave its peers blocked:
//   * every send / recv of an exchange is posted even after one of them
//     failed, and the group is always closed, so no peer waits for an
//     operation this rank never issued;
//   * any failure aborts the communicator (ncclCommAbort), which makes the
//     peers' pending operations fail instead of waiting;
//   * a host wait polls the stream and the communicator's asynchronous error
//     under a wall-clock bound, so a peer that died or hung ends the wait
//     with an error (and an abort) rather than never returning.
// Host-only header: no HIP or RCCL types.
#pragma once

#include <chrono>
#include <cstddef>
#include <cstdint>
#include <thread>

#include "../../include/crgc.h"

namespace crgc {

// Ops: bool group_start(), bool send(uint32_t peer), bool recv(uint32_t peer),
// bool group_end(), void abort().  Returns CRGC_OK or CRGC_E_DEVICE.
template <class Ops>
int post_alltoallv(Ops &ops, uint32_t n_ranks, uint32_t rank, const size_t *sbytes, const size_t *rbytes) {
  if (!ops.group_start()) {
    ops.abort();
    return CRGC_E_DEVICE;
  }
  bool ok = true;
  for (uint32_t r = 0; r < n_ranks; ++r) {
    if (r == rank) continue;
    if (sbytes[r] && !ops.send(r)) ok = false;  // keep posting: the peer expects the rest
    if (rbytes[r] && !ops.recv(r)) ok = false;
  }
  const bool closed = ops.group_end();  // never leave a dangling group
  if (!ok || !closed) {
    ops.abort();
    return CRGC_E_DEVICE;
  }
  return CRGC_OK;
}

// Q: int query() (0 done, 1 pending, < 0 failed), bool async_error(),
// void abort().  Polls until the work is done, fails, or `timeout` passes;
// yields between polls for the first `spin`, then sleeps 20 us between them.
template <class Q, class Clock = std::chrono::steady_clock>
int poll_wait(Q &q, std::chrono::nanoseconds timeout,
              std::chrono::nanoseconds spin = std::chrono::microseconds(256)) {
  const auto t0 = Clock::now();
  for (uint64_t it = 0;; ++it) {
    const int st = q.query();
    if (st == 0) return CRGC_OK;
    if (st < 0) {
      q.abort();
      return CRGC_E_DEVICE;
    }
    // the communicator's error state is a host query: check it every few polls
    if ((it & 15) == 0) {
      if (q.async_error()) {
        q.abort();
        return CRGC_E_DEVICE;
      }
      if (Clock::now() - t0 > timeout) {
        q.abort();
        return CRGC_E_TIMEOUT;
      }
    }
    // a wakeup's exchange normally completes in microseconds: spin (the caller's
    // bound), then yield the pinned GC thread's core.  A sleep ends ~50-80 us
    // late: after 256 polls (round 5) the wait behind a sharded wakeup's level
    // run (~1 ms) left ~90 us of idle GPU (profiles/r6ad/c2rs_last_wakeup_timeline.txt)
    if (Clock::now() - t0 > spin) std::this_thread::sleep_for(std::chrono::microseconds(20));
    else std::this_thread::yield();
  }
}

}  // namespace crgc
