// CPU check of the shard exchange's error discipline (crgc_xpost.hpp), the
// code RcclTransport runs, driven by fake ranks instead of RCCL: a failing
// send / recv on one rank must still post every other operation, close the
// group and abort the communicator; a wait on a rank whose peer died must end
// (async error -> abort, or the wall-clock bound -> timeout).
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../uigc-akka_amd/csrc/crgc_xpost.hpp"

using namespace crgc;

static int failures = 0;
#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) {                                                    \
      std::fprintf(stderr, "%s:%d: CHECK(%s)\n", __FILE__, __LINE__, #c); \
      ++failures;                                                  \
    }                                                              \
  } while (0)

struct FakeOps {
  int fail_send_to = -1, fail_recv_from = -1;
  bool fail_start = false, fail_end = false;
  std::vector<int> sent, received;
  bool started = false, ended = false, aborted = false;
  bool group_start() { started = true; return !fail_start; }
  bool send(uint32_t r) { sent.push_back((int)r); return (int)r != fail_send_to; }
  bool recv(uint32_t r) { received.push_back((int)r); return (int)r != fail_recv_from; }
  bool group_end() { ended = true; return !fail_end; }
  void abort() { aborted = true; }
};

static void exchange_cases() {
  const uint32_t G = 8, me = 3;
  std::vector<size_t> sb(G, 16), rb(G, 16);
  sb[5] = 0;  // nothing for rank 5: no send posted
  {
    FakeOps ok;
    CHECK(post_alltoallv(ok, G, me, sb.data(), rb.data()) == CRGC_OK);
    CHECK(ok.sent.size() == G - 2 && ok.received.size() == G - 1);
    CHECK(ok.ended && !ok.aborted);
  }
  {
    FakeOps f;  // the first send fails: the other six peers still get theirs
    f.fail_send_to = 0;
    CHECK(post_alltoallv(f, G, me, sb.data(), rb.data()) == CRGC_E_DEVICE);
    CHECK(f.sent.size() == G - 2 && f.received.size() == G - 1);
    CHECK(f.ended && f.aborted);
  }
  {
    FakeOps f;  // a receive in the middle fails
    f.fail_recv_from = 4;
    CHECK(post_alltoallv(f, G, me, sb.data(), rb.data()) == CRGC_E_DEVICE);
    CHECK(f.sent.size() == G - 2 && f.received.size() == G - 1);
    CHECK(f.ended && f.aborted);
  }
  {
    FakeOps f;  // closing the group fails
    f.fail_end = true;
    CHECK(post_alltoallv(f, G, me, sb.data(), rb.data()) == CRGC_E_DEVICE);
    CHECK(f.aborted);
  }
  {
    FakeOps f;  // opening the group fails: nothing posted, aborted
    f.fail_start = true;
    CHECK(post_alltoallv(f, G, me, sb.data(), rb.data()) == CRGC_E_DEVICE);
    CHECK(f.sent.empty() && f.received.empty() && f.aborted);
  }
}

struct FakeStream {
  int done_after = -1;      // polls until the stream drains; -1 never
  int error_after = -1;     // polls until the communicator reports an async error
  int fault_after = -1;     // polls until the stream itself reports a fault
  int polls = 0;
  bool aborted = false;
  int query() {
    ++polls;
    if (fault_after >= 0 && polls > fault_after) return -1;
    return (done_after >= 0 && polls > done_after) ? 0 : 1;
  }
  bool async_error() { return error_after >= 0 && polls > error_after; }
  void abort() { aborted = true; }
};

static void wait_cases() {
  using namespace std::chrono;
  {
    FakeStream s;
    s.done_after = 100;
    CHECK(poll_wait(s, seconds(5)) == CRGC_OK && !s.aborted);
  }
  {
    FakeStream s;  // a dead peer: the stream never drains, the communicator errors
    s.error_after = 40;
    CHECK(poll_wait(s, seconds(5)) == CRGC_E_DEVICE && s.aborted);
  }
  {
    FakeStream s;  // a hung peer, no error ever reported: the bound ends the wait
    const auto t0 = steady_clock::now();
    CHECK(poll_wait(s, milliseconds(50)) == CRGC_E_TIMEOUT && s.aborted);
    CHECK(steady_clock::now() - t0 < seconds(5));
  }
  {
    FakeStream s;  // the stream faults
    s.fault_after = 3;
    CHECK(poll_wait(s, seconds(5)) == CRGC_E_DEVICE && s.aborted);
  }
  {
    FakeStream s;  // drains after many polls, all inside a long spin window: no 20-us sleeps
    s.done_after = 20000;
    const auto t0 = steady_clock::now();
    CHECK(poll_wait(s, seconds(5), seconds(2)) == CRGC_OK && !s.aborted);
    CHECK(steady_clock::now() - t0 < milliseconds(400));  // 20 000 sleeps would take >= 0.4 s
  }
  {
    FakeStream s;  // no spin window: sleeps between polls, still completes
    s.done_after = 30;
    CHECK(poll_wait(s, seconds(5), nanoseconds(0)) == CRGC_OK && !s.aborted);
  }
  {
    FakeStream s;  // a spin window longer than the bound: the bound still ends the wait
    const auto t0 = steady_clock::now();
    CHECK(poll_wait(s, milliseconds(50), seconds(10)) == CRGC_E_TIMEOUT && s.aborted);
    CHECK(steady_clock::now() - t0 < seconds(5));
  }
}

int main() {
  exchange_cases();
  wait_cases();
  if (failures) {
    std::fprintf(stderr, "%d checks failed\n", failures);
    return 1;
  }
  std::printf("xpost ok\n");
  return 0;
}
