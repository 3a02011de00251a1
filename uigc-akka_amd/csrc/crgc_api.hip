// crgc_api.hip — the C ABI of include/crgc.h: host orchestration of the HBM
// shadow graph.  One handle = one ShadowGraph (ShadowGraph.java:9-21).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <functional>
#include <cstdio>
#include <cstring>
#include <new>
#include <vector>

#include "crgc_host.hpp"
#include "crgc_transport.hpp"

using namespace crgc;

namespace {

uint64_t pow2ceil(uint64_t x) {
  uint64_t p = 1;
  while (p < x) p <<= 1;
  return p;
}
uint64_t round_up(uint64_t x, uint64_t m) { return (x + m - 1) / m * m; }

struct Caps {
  uint64_t scap, hcap, pcap, ecap;
  uint64_t pbase;  // first proxy slot; == scap without a proxy region (unsharded graphs)
};

// Device arrays of one graph generation.
struct Arrays {
  DevGraph d{};
  Caps caps{};
  bool allocated = false;
};

template <class T>
hipError_t dmalloc(T **p, uint64_t n) {
  return hipMalloc((void **)p, std::max<uint64_t>(n, 1) * sizeof(T));
}

void free_arrays(Arrays &a) {
  if (!a.allocated) return;
  DevGraph &d = a.d;
  void *ps[] = {d.htab, d.vid, d.recv, d.flags, d.sup, d.adj, d.vseq, d.sseq,
                d.pool, d.etab, d.vis, d.front[0], d.front[1],
                d.dirty[0], d.dirty[1], d.out_a, d.out_b, d.qn_buf, d.qh_buf, d.qn_tag, d.blkstat, d.xbytes,
                d.sweep_cnt, d.sweep_off, d.out_ids, d.out_kill,
                d.nzdeg, d.radj, d.rnew, d.rpool, d.par, d.fx, d.cb, d.cb2, d.tq, d.tl_buf, d.tl_tag, d.cm, d.pb[0], d.pb[1],
                d.xsent, d.xkey, d.wpc, d.rq_buf, d.rq_cnt, d.phs, d.psh, d.freel, d.freel2, d.gslot};
  for (void *p : ps)
    if (p) hipFree(p);
  a.allocated = false;
  a.d = DevGraph{};
}

hipError_t alloc_arrays(Arrays &a, const Caps &c, Counters *ctr, hipStream_t s, uint32_t n_shards,
                        uint32_t shard, bool sharded, bool reuse) {
  a.caps = c;
  DevGraph &d = a.d;
  d = DevGraph{};
  d.n_shards = n_shards;
  d.shard = shard;
  // slots are u32 below SLOT_DEAD, and reverse candidates keep bit 31 (RC_POS)
  if (c.scap >= (1ull << 31)) return hipErrorOutOfMemory;
  d.hcap = c.hcap;
  d.hmask = c.hcap - 1;
  d.scap = c.scap;
  d.pbase = c.pbase;
  d.pcap = c.pcap;
  d.ecap_tab = c.ecap;
  d.emask = c.ecap - 1;
  d.ctr = ctr;
  hipError_t e = hipSuccess;
#define A(call)                         \
  do {                                  \
    if ((e = (call)) != hipSuccess) {   \
      a.allocated = true;               \
      free_arrays(a);                   \
      return e;                         \
    }                                   \
  } while (0)
  A(dmalloc(&d.htab, c.hcap));
  A(dmalloc(&d.vid, c.scap));
  A(dmalloc(&d.recv, c.scap));
  A(dmalloc(&d.flags, c.scap));
  A(dmalloc(&d.sup, c.scap));
  A(dmalloc(&d.adj, c.scap));
  A(dmalloc(&d.vseq, c.scap));
  A(dmalloc(&d.sseq, c.scap));
  A(dmalloc(&d.pool, c.pcap));
  A(dmalloc(&d.etab, c.ecap));
  A(dmalloc(&d.vis, c.scap / 32));
  A(dmalloc(&d.front[0], c.scap));
  A(dmalloc(&d.front[1], c.scap));
  A(dmalloc(&d.dirty[0], c.scap / BLK_SLOTS));
  A(dmalloc(&d.dirty[1], c.scap / BLK_SLOTS));
  A(dmalloc(&d.out_a, c.scap));
  A(dmalloc(&d.out_b, c.scap));
  d.qn_cap = c.scap;
  d.qh_cap = c.pcap / 128 + 1024;
  A(dmalloc(&d.qn_buf, d.qn_cap));
  A(dmalloc(&d.qh_buf, d.qh_cap));
  A(dmalloc(&d.qn_tag, c.scap / BLK_SLOTS));
  A(dmalloc(&d.blkstat, (uint64_t)STAT_WG * 4));
  A(dmalloc(&d.xbytes, (uint64_t)STAT_WG));
  A(dmalloc(&d.sweep_cnt, 2 * (c.scap / BLK_SLOTS)));
  A(dmalloc(&d.sweep_off, 2 * (c.scap / BLK_SLOTS)));
  A(dmalloc(&d.out_ids, c.scap));
  A(dmalloc(&d.out_kill, c.scap));
  d.rpcap = c.pcap;
  A(dmalloc(&d.nzdeg, c.scap));
  A(dmalloc(&d.radj, c.scap));
  A(dmalloc(&d.rnew, c.scap));
  A(dmalloc(&d.rpool, d.rpcap));
  A(dmalloc(&d.par, c.scap));
  A(dmalloc(&d.fx, c.scap / 32));
  A(dmalloc(&d.cb, c.scap / 32));
  A(dmalloc(&d.cb2, c.scap / 32));
  A(dmalloc(&d.tq, 2 * (uint64_t)TAIL_QCAP));
  d.wpc_cap = (uint64_t)TAIL_QCAP + c.pcap / 256 + 1;  // (WALK_PIECE = 256 edges)
  A(dmalloc(&d.wpc, d.wpc_cap));
  A(dmalloc(&d.tl_buf, c.scap));
  A(dmalloc(&d.tl_tag, c.scap / BLK_SLOTS));
  A(dmalloc(&d.cm, c.scap / 32));
  A(dmalloc(&d.pb[0], c.scap / 32));
  A(dmalloc(&d.pb[1], c.scap / 32));
  if (reuse && !sharded) {  // slot reuse (crgc_reuse.hip): the free list, its successor, garbage slots
    A(dmalloc(&d.freel, c.scap));
    A(dmalloc(&d.freel2, c.scap));
    A(dmalloc(&d.gslot, c.scap));
  }
  if (sharded) {
    A(dmalloc(&d.xsent, c.scap / 32));
    A(dmalloc(&d.xkey, c.scap));
    A(dmalloc(&d.rq_buf, c.scap));
    A(dmalloc(&d.rq_cnt, c.scap / BLK_SLOTS));
    A(dmalloc(&d.phs, c.scap));
    A(dmalloc(&d.psh, c.scap));
  }
#undef A
  a.allocated = true;
  // Default state of every unused slot / bucket (each memset's own status:
  // hipGetLastError would also report a soft failure of an earlier call).
  hipError_t ms = hipSuccess;
#define M(p, v, n)                                  \
  do {                                              \
    const hipError_t r = hipMemsetAsync(p, v, n, s); \
    if (ms == hipSuccess) ms = r;                   \
  } while (0)
  M(d.htab, 0xFF, c.hcap * sizeof(IdBucket));
  M(d.recv, 0, c.scap * 4);
  M(d.flags, 0, c.scap);
  M(d.sup, 0xFF, c.scap * 4);
  M(d.adj, 0, c.scap * 8);
  M(d.vseq, 0, c.scap * 8);
  M(d.sseq, 0, c.scap * 8);
  M(d.etab, 0xFF, c.ecap * sizeof(EdgeBucket));
  M(d.vis, 0, c.scap / 8);
  M(d.front[0], 0, c.scap);
  M(d.front[1], 0, c.scap);
  M(d.dirty[0], 0, c.scap / BLK_SLOTS);
  M(d.dirty[1], 0, c.scap / BLK_SLOTS);
  M(d.nzdeg, 0, c.scap * 4);
  M(d.radj, 0, c.scap * 8);
  M(d.rnew, 0, c.scap * 4);
  M(d.par, 0xFF, c.scap * 4);  // no hints in a new generation
  M(d.fx, 0, c.scap / 8);
  M(d.cb, 0, c.scap / 8);
  M(d.cb2, 0, c.scap / 8);
  M(d.cm, 0, c.scap / 8);
  M(d.pb[0], 0, c.scap / 8);
  M(d.pb[1], 0, c.scap / 8);
  if (sharded) {
    M(d.phs, 0xFF, c.scap * 4);  // PHS_NONE: a new generation resolves again
    M(d.xsent, 0, c.scap / 8);
    M(d.rq_cnt, 0, c.scap / BLK_SLOTS * 4);
  }
#undef M
  if (ms != hipSuccess) free_arrays(a);
  return ms;
}

// Slots of one region for `live` kept shadows and `ids` that a pending merge may add.
uint64_t region_cap(uint64_t live, uint64_t ids) {
  return round_up(std::max<uint64_t>(2 * live + ids, live + 2 * ids) + 8192, BLK_SLOTS);
}

// Sharded graphs (G > 1) keep their proxies in a region of their own above
// pbase (DevGraph::pbase), sized like the shadows' region from the live
// proxies; the id table and the pools serve both.
// idtab_x2: id-table buckets per slot, times 2 (3: load <= 1/3 of the slots'
// worth at 1.5 buckets per slot; CRGC_IDTAB_X2, an A/B of the table's cache
// footprint)
Caps caps_regions(uint64_t H, uint64_t P, uint64_t edges, uint64_t atoms_pending, uint32_t idtab_x2 = 3) {
  Caps c;
  c.pbase = H;
  c.scap = H + P;
  c.hcap = pow2ceil(c.scap * idtab_x2 / 2 + 1024);
  uint64_t pc = 4 * edges + 8 * atoms_pending + 4 * c.scap + 65536;
  c.pcap = std::min<uint64_t>(pc, 0xFFFFFFF0ull);
  c.ecap = pow2ceil((edges + 2 * atoms_pending) * 3 / 2 + 65536);
  return c;
}

Caps caps_for(uint64_t live, uint64_t live_proxies, bool proxies, uint64_t edges, uint64_t ids_pending,
              uint64_t atoms_pending, uint32_t idtab_x2 = 3) {
  return caps_regions(region_cap(live, ids_pending), proxies ? region_cap(live_proxies, ids_pending) : 0, edges,
                      atoms_pending, idtab_x2);
}

// A new graph's capacities from the caller's hints (expected live shadows v0,
// proxies p0 of a sharded graph, and live (owner, target) pairs e0): slots for
// twice the live shadows (a trace compacts once dead slots outnumber live
// ones), the id table at load <= 1/3, the edge table at load <= 2/3 of e0, the
// pools for power-of-two segments with room to move.  (caps_for sizes a
// rebuild, which also reserves for the pending merge.)  At C4 on one GPU
// (1.1e8 / 1.1e9 hints) this is ~130 GB of the 288 GB: caps_for(v0, e0, v0, e0)
// asked for ~250 GB there.
Caps caps_create(uint64_t v0, uint64_t p0, bool proxies, uint64_t e0, uint32_t idtab_x2 = 3) {
  auto reg = [](uint64_t v) { return round_up(2 * v + v / 4 + 8192, BLK_SLOTS); };
  Caps c = caps_regions(reg(v0), proxies ? reg(p0) : 0, 0, 0, idtab_x2);
  c.pcap = std::min<uint64_t>(4 * e0 + 4 * c.scap + 65536, 0xFFFFFFF0ull);
  c.ecap = pow2ceil(e0 * 3 / 2 + 65536);
  return c;
}

#define CTR_OFF(f) offsetof(Counters, f)

}  // namespace

// Switches, read once when the handle is created (not per call).
//
// Production reads only the documented keys:
//   CRGC_LEVEL_TIMEOUT_S  wall bound of one trace's level loop (default 300 s)
//   CRGC_KERNEL_TIMING    0: chunk events only, 1: k_expand's dispatch events too,
//                         2: every level kernel, 3 (default): the expand of the wide
//                         levels 0 and 1 (the roofline's live timing)
//   CRGC_TIMING_EVERY     k: only every k-th trace carries timing events (default 1)
//   CRGC_LEVEL_LOG        per-level device times on stderr (diagnostics)
//   CRGC_SPIN_US          host waits poll the stream this long before blocking
//                         (default 20000; 0 blocks at once; crgc_internal.hpp)
// (and, in the transports, CRGC_RCCL_TIMEOUT_S / CRGC_LOCAL_BARRIER_S).
// Everything else — the A/B variants of DESIGN.md §4 and the test hooks of
// tests/ — is read only when CRGC_TEST_HOOKS=1, so a JVM host that inherits a
// stray environment variable cannot change the kernels it runs.
struct Knobs {
  bool pull = true;              // CRGC_PULL=0: push only
  uint64_t pull_div = 16;        // CRGC_PULL_DIV: pull after a frontier of >= slots / div
  // (4 until round 5: on the C2 graph grown to 2.2e7 shadows level 1's
  // frontier fell under a quarter of the slots and pushed its 6e7 edges in
  // 0.83 ms where the pull took 0.24 ms; at 8, 2.65 -> 2.08 ms per wakeup there,
  // profiles/r5r)
  uint32_t pull_cur_div = 8;     // CRGC_PULL_CUR_DIV
  uint32_t alpha = 0;            // CRGC_ALPHA: Beamer's rule (off by default)
  bool has_pull_thresh = false;  // CRGC_PULL_THRESH: absolute threshold (test hook)
  uint64_t pull_thresh = 0;
  bool has_sparse = false;       // CRGC_SPARSE_THRESH (test hook)
  uint32_t sparse_thresh = 0;
  bool tail = true;              // CRGC_TAIL=0: no narrow-frontier takeover
  uint32_t tail_start = 8192;    // CRGC_TAIL_START
  uint32_t tail_max = 32768;     // CRGC_TAIL_MAX
  // Sharded graphs: one workgroup walks a shard's narrow levels with its marked
  // bitmap in HBM (no LDS copy past 2^20 slots) and lists most targets as
  // proxies, ~1 G edges/s: the level kernels are faster from a few thousand
  // shadows up (C2 over 8 logical shards: 18.4 -> 17.1 ms per wakeup at
  // 2048 / 4096 against 8192 / 32768, profiles/r5h).  CRGC_TAIL_START /
  // CRGC_TAIL_MAX set both forms.
  uint32_t tail_start_sharded = 2048;
  uint32_t tail_max_sharded = 4096;
  // k_tail walks frontiers of at most this many out-edges per round (0: no
  // bound).  A shard's hubs are mostly edges to proxies, each a global claim
  // by the one workgroup: C2 over 8 logical shards spent 2.1 of its 3.4 ms of
  // k_tail per wakeup in ~11 walks of 230-275 us in an early round-6 run (its
  // record was lost); with the bound k_tail averages 14.5 us per launch there
  // (profiles/r6i/c2l8s_kernels_per_wakeup.txt).  CRGC_TAIL_EDGES
  uint32_t tail_edges = 0;
  uint32_t tail_edges_sharded = 32768;
  // k_walk (WALK_WG workgroups with grid barriers) in place of k_tail for a
  // sharded graph's narrow levels: correct, and slower as measured (C4 at half
  // size over 8 logical shards 33.0 -> 36.4 ms per wakeup, GPU work 38.4 ->
  // 39.3 ms: as the level controller it runs on every level, and a narrow
  // level's hub leaves the other workgroups waiting at the barrier,
  // profiles/r5r), so off by default (CRGC_WALK=1).
  bool walk = false;             // CRGC_WALK
  bool walk_unsharded = false;   // CRGC_WALK_UNSHARDED=1: k_walk for unsharded graphs too (no chain mode then)
  uint32_t walk_start = 16384;   // CRGC_WALK_START
  uint32_t walk_max = 32768;     // CRGC_WALK_MAX
  // CRGC_CHAIN_AFTER: a k_tail walk of this many links hands the rest of the
  // mark to chain mode.  16 (64 until round 6): C3 1.112 / 1.086 -> 0.968 /
  // 1.059 ms per trace, C2 and C1 unchanged (profiles/r6u)
  uint32_t chain_after = 16;
  // CRGC_KERNEL_TIMING: 0 chunks only, 1 every level's expand, 2 all level
  // kernels, 3 (default) the expand of the wide levels 0 and 1 only.  A timing
  // event carried by a dispatch costs ~5 us of idle GPU around it
  // (tools/event_probe.hip, profiles/r6g/event_probe.txt): ~60 us per C2 wakeup with every
  // expand timed, most of it on narrow levels that carry ~20 % of the
  // expand's device time.
  int kernel_timing = 3;
  // CRGC_TIMING_EVERY=k: only every k-th trace carries timing events (its
  // level chunks, timed expands and sweep; the others report 0 ms and 0 timed
  // launches).  Each event costs ~5 us of idle GPU (r6g), ~45 us per C2 wakeup
  // in all (profiles/r6d/c2_last_wakeup_timeline.txt); a sample of the traces
  // is enough for the device-time figures.
  uint32_t timing_every = 1;
  bool level_log = false;        // CRGC_LEVEL_LOG
  uint64_t level_timeout_s = 300;  // CRGC_LEVEL_TIMEOUT_S
  int xbits = 1;                 // CRGC_XBITS: sharded mark form (0 ids, 1 cheaper, 2 bitmaps)
  int buckets_log2 = 0;          // CRGC_BUCKETS_LOG2: edge-pipeline buckets (test hook; 0 = by size)
  // Sharded deep marks switch to the replicated chain closure (crgc_xchain.hip)
  // after this many rounds (0: never), once a round's marks are at most
  // 1 / xclosure_narrow of the graph's slots (0: at any width; a test hook).
  uint32_t xclosure_after = 8;   // CRGC_XCLOSURE_AFTER
  uint32_t xclosure_narrow = 1024;  // CRGC_XCLOSURE_NARROW
  // A mark round's fixed cost in link bytes (two host round trips, the
  // all-gathered counts and ~4 near-empty level launches: ~0.1 ms ≈ 4 MB at
  // ~50 GB/s per xGMI link direction), against which the closure's all-gathers
  // are priced.  CRGC_XROUND_BYTES
  uint64_t xround_bytes = 4ull << 20;
  uint32_t xslices = 1;          // CRGC_XSLICES: push-level target slices (1, 2, 4, 8)
  // Sharded marks: a round runs at most this many level launches before its
  // exchange (0: to the shard's local fixpoint).  Pending candidates carry
  // over into the next round.
  uint32_t xlevels = 0;          // CRGC_XLEVELS
  uint32_t idtab_x2 = 3;         // CRGC_IDTAB_X2: id-table buckets per slot x 2 (caps_regions)
  bool xfilter = true;           // CRGC_XFILTER=0: send every newly marked proxy (mark_all)
  // CRGC_ROUND_CHUNK (test hook): levels a sharded mark round launches before
  // its first host check when it starts from more than tail_start_sharded marks
  // (0: as many as the previous round needed, 1 .. 4)
  uint32_t round_chunk = 4;
  // CRGC_XSCAN_Q (test hook): k_xscan's units (waves) per proxy block, 1, 2, 4 or 8; 0 (default):
  // 4 while the grid stays within its 8192-workgroup cap, fewer above (C2 over 8 logical shards:
  // 66 -> 38 us per shard and round; C4 at half size 148.6 -> 135.9 us, profiles/r6ac, r6ad)
  uint32_t xscan_q = 0;
  uint64_t xbitmap_ratio = 32;   // CRGC_XBITMAP_RATIO: a mark round's home slots as a bitmap above
                                 // this many list bytes per bitmap byte (mark_all; 32: never)
  bool bin = true;               // CRGC_BIN=0: the pseudo-root level pushes candidate bytes directly
  uint64_t bin_min = 1ull << 22; // CRGC_BIN_MIN_SLOTS: binned only above this many slots (a smaller
                                 // candidate byte map stays in the L2: C1 mark +10 us binned)
  bool route = true;             // CRGC_ROUTE=0: sharded entry merges all-gather every batch
  bool side_stream = false;      // CRGC_SIDE_STREAM=1: edge pipeline beside the vertex updates
  bool side_prio = false;        // CRGC_SIDE_PRIO=1: that side stream at the highest priority
  bool chunk_host = true;        // CRGC_CHUNK_HOST=0: large pageable host batches in one piece
  uint32_t chunk_max = 4;        // CRGC_CHUNK_MAX: at most this many chunks (2 .. 8)
  uint32_t chunk_reg = 1;        // CRGC_CHUNK_REG: at most this many chunks of a registered batch (1 .. 8)
  uint64_t dev_chunk = 0;        // CRGC_DEV_CHUNK: sub-merge size of large device batches (test hook; 0 = 2^20)
  uint32_t spin_us = spin_us_default();  // CRGC_SPIN_US (production): host waits poll this long before blocking (0: block at once)
  bool repack_each = false;      // CRGC_REPACK_EACH_MERGE=1: repack the pools before every merge (test hook)
  bool pull_pred = false;        // CRGC_PULL_PRED=1: the previous trace's pull levels pull again
  bool supbin = true;            // CRGC_SUPBIN=0: the binned level 0 stores supervisor candidate bytes at once
  // CRGC_BIN512=1: up to 512 bins of 2^16 slots (u16 offsets) past 2^24 slots; measured slower on
  // the C2 graph (level 0 expand 162 against 135 us: the per-window bin tables, profiles/r5ae)
  bool bin512 = false;
  bool cbits = true;             // CRGC_CBITS=0: a pull level's finds go out as candidate bytes
  bool roots_co = true;          // CRGC_ROOTS_CO=0: the pseudo-root pass reads 128 B of counts per lane
  // A registered batch's chunk is copied by the DMA engines (one
  // hipMemcpyAsync of the span its arrays occupy in the caller's arena) rather
  // than read over PCIe by k_copy_ranges, which shares the memory pipeline with
  // the merge kernels beside it (profiles/r4ab): registered C2 wakeup 2.13 /
  // 2.19 against 2.32 / 2.31 ms, merge call 0.82 / 0.85 against 0.95 / 0.99 ms,
  // interleaved on one box (profiles/r6e/ab_pcie).  CRGC_REG_SDMA=0: the kernel copy.
  bool reg_sdma = true;
  // CRGC_SLOT_REUSE=0: collected shadows' slots are reclaimed only by a rebuild
  // (round 5); by default the sweep's garbage slots are purged of their edges
  // and taken by the next merges' new shadows (crgc_reuse.hip)
  bool slot_reuse = true;
  // The listed garbage slots are purged and freed in one batch once they make up
  // 1 / reuse_div of the slot range (0: after every committed sweep, the test
  // suite's setting).  CRGC_SLOT_REUSE_DIV
  uint32_t reuse_div = 16;
  void read() {
    auto env = [](const char *k) { return getenv(k); };
    if (const char *m = env("CRGC_KERNEL_TIMING")) kernel_timing = atoi(m);
    if (const char *m = env("CRGC_TIMING_EVERY")) timing_every = std::max<uint32_t>(1, (uint32_t)strtoul(m, nullptr, 10));
    level_log = env("CRGC_LEVEL_LOG") != nullptr;
    if (const char *m = env("CRGC_LEVEL_TIMEOUT_S")) level_timeout_s = std::max<uint64_t>(1, strtoull(m, nullptr, 10));
    const char *hooks = env("CRGC_TEST_HOOKS");
    if (!hooks || atoi(hooks) != 1) return;
    if (const char *m = env("CRGC_PULL")) pull = atoi(m) != 0;
    if (const char *m = env("CRGC_PULL_DIV")) pull_div = std::max<uint64_t>(1, strtoull(m, nullptr, 10));
    if (const char *m = env("CRGC_PULL_CUR_DIV")) pull_cur_div = (uint32_t)strtoul(m, nullptr, 10);
    if (const char *m = env("CRGC_ALPHA")) alpha = (uint32_t)strtoul(m, nullptr, 10);
    if (const char *m = env("CRGC_PULL_THRESH")) {
      has_pull_thresh = true;
      pull_thresh = strtoull(m, nullptr, 10);
    }
    if (const char *m = env("CRGC_SPARSE_THRESH")) {
      has_sparse = true;
      sparse_thresh = (uint32_t)strtoul(m, nullptr, 10);
    }
    if (const char *m = env("CRGC_TAIL")) tail = atoi(m) != 0;
    if (const char *m = env("CRGC_TAIL_START")) tail_start = tail_start_sharded = (uint32_t)strtoul(m, nullptr, 10);
    if (const char *m = env("CRGC_TAIL_MAX")) tail_max = tail_max_sharded = (uint32_t)strtoul(m, nullptr, 10);
    if (const char *m = env("CRGC_TAIL_EDGES")) tail_edges = tail_edges_sharded = (uint32_t)strtoul(m, nullptr, 10);
    if (const char *m = env("CRGC_WALK")) walk = atoi(m) != 0;
    if (const char *m = env("CRGC_WALK_UNSHARDED")) walk_unsharded = atoi(m) != 0;
    if (const char *m = env("CRGC_WALK_START")) walk_start = (uint32_t)strtoul(m, nullptr, 10);
    if (const char *m = env("CRGC_WALK_MAX")) walk_max = (uint32_t)strtoul(m, nullptr, 10);
    if (const char *m = env("CRGC_CHAIN_AFTER")) chain_after = (uint32_t)strtoul(m, nullptr, 10);
    if (const char *m = env("CRGC_XBITS")) xbits = atoi(m);
    if (const char *m = env("CRGC_BUCKETS_LOG2"))
      buckets_log2 = std::min(10, std::max(1, atoi(m)));
    if (const char *m = env("CRGC_XCLOSURE_AFTER")) xclosure_after = (uint32_t)strtoul(m, nullptr, 10);
    if (const char *m = env("CRGC_XCLOSURE_NARROW")) xclosure_narrow = (uint32_t)strtoul(m, nullptr, 10);
    if (const char *m = env("CRGC_XROUND_BYTES")) xround_bytes = strtoull(m, nullptr, 10);
    if (const char *m = env("CRGC_BIN")) bin = atoi(m) != 0;
    if (const char *m = env("CRGC_BIN_MIN_SLOTS")) bin_min = strtoull(m, nullptr, 10);
    if (const char *m = env("CRGC_XLEVELS")) xlevels = (uint32_t)strtoul(m, nullptr, 10);
    if (const char *m = env("CRGC_XFILTER")) xfilter = atoi(m) != 0;
    if (const char *m = env("CRGC_XBITMAP_RATIO")) xbitmap_ratio = std::max<uint64_t>(1, strtoull(m, nullptr, 10));
    if (const char *m = env("CRGC_ROUND_CHUNK")) round_chunk = std::min<uint32_t>((uint32_t)strtoul(m, nullptr, 10), 64);
    if (const char *m = env("CRGC_XSCAN_Q")) {
      const uint32_t v = (uint32_t)strtoul(m, nullptr, 10);
      if (v == 1 || v == 2 || v == 4 || v == 8) xscan_q = v;
    }
    if (const char *m = env("CRGC_IDTAB_X2")) idtab_x2 = std::max<uint32_t>(1, (uint32_t)strtoul(m, nullptr, 10));
    if (const char *m = env("CRGC_XSLICES")) {
      const uint32_t v = (uint32_t)strtoul(m, nullptr, 10);
      xslices = v >= 8 ? 8 : v >= 4 ? 4 : v >= 2 ? 2 : 1;
    }
    if (const char *m = env("CRGC_ROUTE")) route = atoi(m) != 0;
    if (const char *m = env("CRGC_CBITS")) cbits = atoi(m) != 0;
    if (const char *m = env("CRGC_BIN512")) bin512 = atoi(m) != 0;
    if (const char *m = env("CRGC_SUPBIN")) supbin = atoi(m) != 0;
    if (const char *m = env("CRGC_PULL_PRED")) pull_pred = atoi(m) != 0;
    if (const char *m = env("CRGC_ROOTS_CO")) roots_co = atoi(m) != 0;
    if (const char *m = env("CRGC_SIDE_STREAM")) side_stream = atoi(m) != 0;
    if (const char *m = env("CRGC_SIDE_PRIO")) side_prio = atoi(m) != 0;
    if (const char *m = env("CRGC_CHUNK_HOST")) chunk_host = atoi(m) != 0;
    if (const char *m = env("CRGC_CHUNK_MAX")) chunk_max = std::min<uint32_t>(8, std::max(2, atoi(m)));
    if (const char *m = env("CRGC_CHUNK_REG")) chunk_reg = std::min<uint32_t>(8, std::max(1, atoi(m)));
    if (const char *m = env("CRGC_REG_SDMA")) reg_sdma = atoi(m) != 0;
    if (const char *m = env("CRGC_SLOT_REUSE")) slot_reuse = atoi(m) != 0;
    if (const char *m = env("CRGC_SLOT_REUSE_DIV")) reuse_div = (uint32_t)strtoul(m, nullptr, 10);
    if (const char *m = env("CRGC_DEV_CHUNK")) {  // 0: the default
      dev_chunk = strtoull(m, nullptr, 10);
      if (dev_chunk) dev_chunk = std::max<uint64_t>(64, dev_chunk);
    }
    if (const char *m = env("CRGC_REPACK_EACH_MERGE")) repack_each = atoi(m) != 0;
  }
};

struct crgc_graph {
  int device = 0;
  Knobs knobs;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  uint32_t F = 4, DGS = 64;
  Arrays g;
  Counters *ctr = nullptr;   // device
  Counters *hctr = nullptr;  // pinned host mirror
  Counters *hctr_dev = nullptr;  // its device view (k_publish stores the level loop's counters there)
  unsigned long long epoch = 0;
  bool poisoned = false;
  // exact values as of the last synchronisation + upper-bound increments since
  uint64_t slot_top = 0, pool_top = 0, rpool_top = 0, etab_used = 0, live = 0;
  uint64_t proxy_top = 0;  // proxy region slots in use (sharded graphs), as of the last synchronisation
  uint64_t n_rebuild = 0, n_grow = 0, n_repack = 0;  // crgc_usage_of
  uint64_t pend_n = 0;        // slot reuse: committed garbage slots listed in gslot, not purged yet
  uint64_t n_traces = 0;      // crgc_trace calls (timing_every)
  bool free_avail = false;    // slot reuse: the free list may hold untaken slots (ids_view)
  bool timed = true;          // the current mark carries timing events
  bool halted_seen = false;   // an undo log was merged: live shadows may be halted (k_sup_fix)
  bool walk_ok = false;  // CRGC_WALK: k_walk's workgroups fit the device at once (walk_fits)
  std::vector<uint8_t> lvl_timed;  // per level launch of the current run_levels: timed (events)
  uint64_t ids_since = 0, atoms_since = 0;
  uint64_t inserted_at_trace = 0;  // Counters::inserted when `live` was exact
  Scratch stage, work;
  hipEvent_t ev[4] = {};
  // The edge pipeline of a merge runs on `side` beside the vertex updates on
  // `stream` (they touch disjoint arrays); fork / join events order them.
  hipStream_t side = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  // Large host batches are copied in chunks on `cpy` while the chunks before
  // them merge on `stream` (merge_entries_chunked).
  hipStream_t cpy = nullptr;
  hipEvent_t ev_cstart = nullptr, ev_chunk[8] = {};
  // Host-batch chunk merges stage into two areas in turn: a call's copy waits
  // only for the merges that last read its area (ev_cfree), so a drain loop's
  // next chunk is copied while the previous one merges
  Scratch cstage[2];
  hipEvent_t ev_cfree[2] = {};
  bool cfree_rec[2] = {false, false};
  int cstage_k = 0;
  // CRGC_SIDE_STREAM=1 (read at create): the edge pipeline beside the vertex
  // updates.  Off: both halves are bound by random memory operations, so the
  // overlap bought nothing (merge 0.578-0.587 ms alone vs 0.588-0.598 ms with
  // it on C2, profiles/r3f/ab_merge.txt)
  bool use_side = false;
  bool chunk_host = true;  // CRGC_CHUNK_HOST=0: large host batches in one piece
  uint32_t chunk_max = 4;  // CRGC_CHUNK_MAX: at most this many chunks (2 .. 8)
  uint32_t chunk_reg = 1;  // CRGC_CHUNK_REG: the same for registered batches (kernel copies; 1: one piece)
  // last trace
  uint64_t last_garbage = 0, last_kill = 0, last_live = 0;
  crgc_trace_stats last_stats{};
  bool have_last = false;
  uint64_t last_levels = 0;  // level launches (after level 0) the previous trace needed
  uint64_t pull_pred = 0;    // levels (bit L) whose k_expand pulled in the previous trace
  std::vector<hipEvent_t> lvl_ev;  // 6 per level launch: start / stop of its 3 kernels
  std::vector<hipEvent_t> chunk_ev;  // start / stop of every chunk of level launches
  uint64_t *roots_buf = nullptr;
  uint64_t roots_cap = 0;
  // sharded graphs (G > 1): transport and exchange buffers
  crgc_transport *tp = nullptr;
  uint32_t G = 1, shard = 0;
  uint64_t n_proxy = 0;              // alive proxy slots after the last trace
  Scratch x_send, x_slot, x_recv, x_ans, x_ans_back, x_small, x_pack, x_pack_recv;
  Scratch x_route, x_route_send, x_cat;  // routed entry merges
  Scratch x_dg, x_dg_out;    // DeltaGraph production
  Scratch x_chain;           // chain mode (crgc_chain.hip)
  Scratch x_chunk;           // rebased offsets of a large device batch's sub-merges
  Scratch x_bin;             // the pseudo-root level's binned push: counters, then bin regions
  Scratch x_gc, x_gc_list;   // replicated chain closure of sharded marks (crgc_xchain.hip)
  Scratch x_gvis;            // every shard's marked bitmap of its shadows (mark_all's send filter)
  Scratch x_wgc;             // k_xscan's per-workgroup counts
  uint64_t *h_small = nullptr;       // pinned host staging for small all-gathers
  uint64_t *h_small_dev = nullptr;   // its device view (ag_u64 reads host words from it)
  uint64_t *h_bounce = nullptr;      // pinned bounce for id lists into partly pinned caller buffers
  uint64_t h_bounce_bytes = 0;
  char *h_route = nullptr;           // pinned RoutePart / ConcatPart tables
  bool route = true;                 // CRGC_ROUTE=0: all-gather every batch instead
  // mark rounds in home-slot form: this shard's slot numbering generation
  // (bumped by every rebuild), and each home's generation / slot count as of
  // this shard's last resolution
  uint64_t slot_gen = 0;
  std::vector<uint64_t> peer_gen, peer_top;
  // host buffers pinned by crgc_host_register: (base, bytes, device view of base)
  struct Pinned {
    char *first;
    uint64_t second;
    char *dev;
  };
  std::vector<Pinned> pinned;
};

// Slot reuse (crgc_reuse.hip): unsharded graphs (a sharded graph's proxies
// cache their homes' slots), unless CRGC_SLOT_REUSE=0.
static bool reuse_on(const crgc_graph *h) { return h->G <= 1 && !h->tp && h->knobs.slot_reuse; }

// The graph as k_ids sees it: without the free list while the host knows it is
// empty (k_ids then takes every new slot from slot_top with no free-list step;
// a per-round check on the device cost ~14 us per C2 merge, profiles/r6g).
static DevGraph ids_view(const crgc_graph *h) {
  DevGraph d = h->g.d;
  if (!h->free_avail) d.freel = nullptr;
  return d;
}

namespace {
thread_local int api_depth = 0;
thread_local char err_detail[256];
}  // namespace

void crgc::note_error(const char *file, int line, const char *what) {
  if (err_detail[0]) return;  // the first failure of the call is the cause
  const char *base = strrchr(file, '/');
  snprintf(err_detail, sizeof err_detail, "%s:%d: %s", base ? base + 1 : file, line,
           what && *what ? what : "failed");
}

namespace {

int map_hip_at(hipError_t e, int line) {
  if (e == hipSuccess) return CRGC_OK;
  note_error(__FILE__, line, hipGetErrorName(e));
  if (e == hipErrorOutOfMemory) return CRGC_E_NOMEM;
  if (e == hipErrorLaunchTimeOut) return CRGC_E_TIMEOUT;
  return CRGC_E_DEVICE;
}
#define map_hip(e) map_hip_at((e), __LINE__)

#define HIP_TRY(x)                                  \
  do {                                              \
    hipError_t _e = (x);                            \
    if (_e != hipSuccess) return map_hip(_e);       \
  } while (0)

// Every API entry point takes one.  It also drops a stale "last error" of this
// thread: the launch helpers report hipGetLastError(), which must not pick up
// an error an earlier call left behind (each call checks its own results).
struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (api_depth++ == 0) err_detail[0] = 0;  // a new call: forget the last one's failure
    (void)hipGetLastError();
    hipGetDevice(&prev);
    if (prev != dev) hipSetDevice(dev);
  }
  ~DeviceGuard() {
    --api_depth;
    int cur;
    hipGetDevice(&cur);
    if (prev >= 0 && cur != prev) hipSetDevice(prev);
  }
};

// Host wait for the graph's stream.  Sharded graphs wait through their
// transport: over RCCL that wait is bounded and ends early when the
// communicator reports an asynchronous error (a failed peer), and the handle
// is poisoned, instead of blocking forever in a collective.
hipError_t hsync(crgc_graph *h) {
  if (!h->tp) return stream_wait(h->stream, h->knobs.spin_us);
  const int rc = h->tp->wait(h->stream);
  if (rc == CRGC_OK) return hipSuccess;
  h->poisoned = true;
  return rc == CRGC_E_TIMEOUT ? hipErrorLaunchTimeOut : hipErrorLaunchFailure;
}

void absorb_counters(crgc_graph *h);

// Read back the small counters (blocking).
hipError_t sync_counters(crgc_graph *h) {
  hipError_t e = hipMemcpyAsync(h->hctr, h->ctr, offsetof(Counters, ring), hipMemcpyDeviceToHost,
                                h->stream);
  if (e != hipSuccess) return e;
  e = hsync(h);
  if (e != hipSuccess) return e;
  absorb_counters(h);
  return hipSuccess;
}

// Bookkeeping from a fresh host copy of the counters.
void absorb_counters(crgc_graph *h) {
  h->slot_top = h->hctr->slot_top;
  h->proxy_top = h->hctr->proxy_top;
  h->pool_top = h->hctr->pool_top;
  h->rpool_top = h->hctr->rpool_top;
  h->etab_used = h->hctr->etab_used;
  h->ids_since = h->atoms_since = 0;
}

int device_error(crgc_graph *h) {
  const uint64_t err = h->hctr->err;
  if (!err) return CRGC_OK;
  h->poisoned = true;
  char what[48];
  snprintf(what, sizeof what, "device error flags 0x%llx", (unsigned long long)err);
  note_error(__FILE__, __LINE__, what);
  if (err & (ERR_RESERVED_ID | ERR_TOO_MANY | ERR_BAD_OFFSETS)) return CRGC_E_INVAL;
  if (err & (ERR_SPIN | ERR_WALK_STUCK)) return CRGC_E_TIMEOUT;
  if (err & ERR_QUEUE_FULL) return DEV_FAIL("");
  return CRGC_E_NOMEM;
}

// The last trace's garbage / kill lists outlive a generation: crgc_last_trace
// may still copy them (two-phase trace, or a trace whose buffers were short).
// They can hold more ids than the new generation has slots.
hipError_t carry_lists(crgc_graph *h, Arrays &dst) {
  if (!h->have_last) return hipSuccess;
  auto carry = [&](uint64_t *&dptr, const uint64_t *src, uint64_t n) -> hipError_t {
    if (n > dst.caps.scap) {
      hipFree(dptr);
      dptr = nullptr;
      if (hipError_t r = dmalloc(&dptr, n)) return r;
    }
    return n ? hipMemcpyAsync(dptr, src, n * 8, hipMemcpyDeviceToDevice, h->stream) : hipSuccess;
  };
  hipError_t e = carry(dst.d.out_ids, h->g.d.out_ids, h->last_garbage);
  if (e == hipSuccess) e = carry(dst.d.out_kill, h->g.d.out_kill, h->last_kill);
  return e;
}

// Larger arrays for the same slots (crgc_rebuild.hip, grow): an unsharded graph
// that outgrew its capacities with few dead slots keeps its numbering — the
// per-slot arrays and the pools are copied as they are, the hash tables are
// re-hashed — instead of a rebuild (the C2 long run: 129 ms per rebuild,
// profiles/r5a; nothing of the trace's pull hints or candidate order is lost).
int grow(crgc_graph *h, uint64_t ids, uint64_t atoms) {
  const uint64_t top = h->slot_top;
  Caps c = caps_for(std::max<uint64_t>(top, 1), 0, false, h->etab_used, ids, atoms, h->knobs.idtab_x2);
  // never smaller than before (a grow may be for the tables, not the slots)
  const Caps &oc = h->g.caps;
  c.scap = c.pbase = std::max(c.scap, oc.scap);
  c.hcap = std::max(c.hcap, oc.hcap);
  c.ecap = std::max(c.ecap, oc.ecap);
  c.pcap = std::min<uint64_t>(std::max(c.pcap, oc.pcap + oc.pcap / 2), 0xFFFFFFF0ull);
  if (h->knobs.level_log)
    fprintf(stderr, "[crgc] grow: slots %llu -> %llu, id table %llu -> %llu, edge table %llu -> %llu, pools %llu -> %llu\n",
            (unsigned long long)h->g.caps.scap, (unsigned long long)c.scap, (unsigned long long)h->g.caps.hcap,
            (unsigned long long)c.hcap, (unsigned long long)h->g.caps.ecap, (unsigned long long)c.ecap,
            (unsigned long long)h->g.caps.pcap, (unsigned long long)c.pcap);
  Arrays dst;
  HIP_TRY(alloc_arrays(dst, c, h->ctr, h->stream, h->G, h->shard, h->tp != nullptr, reuse_on(h)));
  const DevGraph &o = h->g.d;
  DevGraph &d = dst.d;
  hipError_t e = hipSuccess;
  auto cp = [&](void *to, const void *from, size_t bytes) {
    if (e == hipSuccess && bytes) e = hipMemcpyAsync(to, from, bytes, hipMemcpyDeviceToDevice, h->stream);
  };
  cp(d.vid, o.vid, top * 8);
  cp(d.recv, o.recv, top * 4);
  cp(d.flags, o.flags, top);
  cp(d.sup, o.sup, top * 4);
  cp(d.adj, o.adj, top * 8);
  cp(d.vseq, o.vseq, top * 8);
  cp(d.sseq, o.sseq, top * 8);
  cp(d.nzdeg, o.nzdeg, top * 4);
  cp(d.radj, o.radj, top * 8);
  cp(d.par, o.par, top * 4);
  if (d.freel && o.freel) cp(d.freel, o.freel, top * 4);  // (the lists hold slots below slot_top)
  if (d.gslot && o.gslot) cp(d.gslot, o.gslot, h->pend_n * 4);
  cp(d.pool, o.pool, h->pool_top * 8);
  cp(d.rpool, o.rpool, h->rpool_top * 4);
  if (e == hipSuccess) e = launch_grow_tables(o, d, h->stream);
  // (the re-hashed id table has no tombstones left: reused slots' ids no longer load it)
  if (e == hipSuccess) e = hipMemsetAsync((char *)h->ctr + CTR_OFF(reused), 0, 8, h->stream);
  if (e == hipSuccess) e = carry_lists(h, dst);
  if (e == hipSuccess) e = sync_counters(h);
  if (e != hipSuccess) {
    free_arrays(dst);
    h->poisoned = true;
    return map_hip(e);
  }
  free_arrays(h->g);
  h->g = dst;
  ++h->n_grow;
  if (int rc = device_error(h)) return rc;
  return CRGC_OK;
}

// Rebuild into fresh arrays with room for `ids`/`atoms` more, then swap.
// may_grow: an unsharded graph with few dead slots (at most a quarter) grows
// instead (same slots, larger arrays).
int rebuild(crgc_graph *h, uint64_t ids, uint64_t atoms, bool may_grow = false) {
  HIP_TRY(sync_counters(h));
  if (int rc = device_error(h)) return rc;
  const uint64_t src_top = h->slot_top, src_ptop = h->proxy_top;
  // The slots the rebuild keeps, counted exactly: every alive slot, the
  // shadows' and (sharded graphs) the proxies'.  (Round 4 sized the new arrays
  // from the live count at the last trace plus the *home* shadows created
  // since — Counters::inserted is totalActorsSeen — which left out the proxies
  // a sharded load creates: 68 M alive slots went into 27 M at C4 over 8
  // logical shards, and the rebuild's passes wrote past the new arrays.)
  HIP_TRY(hipMemsetAsync((char *)h->ctr + CTR_OFF(alive_cnt), 0, 16, h->stream));
  HIP_TRY(launch_count_alive(h->g.d, src_top, src_ptop, h->ctr->alive_cnt, h->stream));
  HIP_TRY(sync_counters(h));
  const uint64_t live_ub = std::min<uint64_t>(src_top, h->hctr->alive_cnt[0]);
  const uint64_t live_p = std::min<uint64_t>(src_ptop, h->hctr->alive_cnt[1]);
  if (may_grow && h->G <= 1 && live_ub * 4 >= src_top * 3) return grow(h, ids, atoms);
  Caps c = caps_for(std::max<uint64_t>(live_ub, 1), live_p, h->G > 1, h->etab_used, ids, atoms, h->knobs.idtab_x2);
  if (h->knobs.level_log)
    fprintf(stderr, "[crgc] rebuild: slots %llu (alive %llu) proxies %llu (alive %llu) pool %llu / %llu rpool %llu "
                    "edge keys %llu / %llu -> slots %llu pool %llu edge table %llu\n",
            (unsigned long long)src_top, (unsigned long long)live_ub, (unsigned long long)src_ptop,
            (unsigned long long)live_p, (unsigned long long)h->pool_top,
            (unsigned long long)h->g.caps.pcap, (unsigned long long)h->rpool_top,
            (unsigned long long)h->etab_used, (unsigned long long)h->g.caps.ecap, (unsigned long long)c.scap,
            (unsigned long long)c.pcap, (unsigned long long)c.ecap);
  Arrays dst;
  HIP_TRY(alloc_arrays(dst, c, h->ctr, h->stream, h->G, h->shard, h->tp != nullptr, reuse_on(h)));
  Scratch tmp;
  const size_t need = Carver::need({h->g.caps.scap * 4 + 4, c.scap * 8, rebuild_scan_tmp_bytes(c.scap)});
  if (tmp.ensure(need) != hipSuccess) {
    free_arrays(dst);
    return CRGC_E_NOMEM;
  }
  Carver cv(tmp.ptr);
  uint32_t *map = cv.take<uint32_t>(h->g.caps.scap + 1);  // by source slot (both regions)
  uint64_t *offs = cv.take<uint64_t>(c.scap);
  void *scan_tmp = cv.take<uint64_t>(rebuild_scan_tmp_bytes(c.scap) / 8);
  hipError_t e = hipMemsetAsync(offs, 0, c.scap * 8, h->stream);
  // new generation counters: slot_top, pool_top, etab_used, the proxy region's restart
  for (size_t off : {CTR_OFF(slot_top), CTR_OFF(pool_top), CTR_OFF(rpool_top), CTR_OFF(etab_used),
                     CTR_OFF(proxy_top), CTR_OFF(proxy_dead), CTR_OFF(res_top), CTR_OFF(free_n),
                     CTR_OFF(free_used), CTR_OFF(reused)})
    if (e == hipSuccess) e = hipMemsetAsync((char *)h->ctr + off, 0, 8, h->stream);
  // src keeps a view of the old counters' bounds via src_top / src_ptop (passed by value)
  if (e == hipSuccess) e = launch_rebuild(h->g.d, src_top, src_ptop, dst.d, map, offs, scan_tmp, h->stream);
  if (e == hipSuccess) e = carry_lists(h, dst);
  if (e == hipSuccess) e = sync_counters(h);
  tmp.release();
  if (e != hipSuccess) {
    free_arrays(dst);
    h->poisoned = true;
    return map_hip(e);
  }
  free_arrays(h->g);
  h->g = dst;
  h->pend_n = 0;  // (the rebuild dropped every collected slot)
  h->free_avail = false;
  ++h->n_rebuild;
  ++h->slot_gen;  // other shards' cached home slots of this shard are stale now
  h->live = h->slot_top;
  h->inserted_at_trace = h->hctr->inserted;
  if (int rc = device_error(h)) return rc;
  return CRGC_OK;
}

// The two pools packed afresh (launch_repack): dead space of relocated
// segments reclaimed, slots and tables unchanged.  If the new pools cannot be
// allocated the graph is as before (CRGC_E_NOMEM), so the caller may rebuild.
int repack(crgc_graph *h) {
  HIP_TRY(sync_counters(h));
  if (int rc = device_error(h)) return rc;
  const Caps &c = h->g.caps;
  uint64_t *pool2 = nullptr;
  uint32_t *rpool2 = nullptr;
  Scratch tmp;
  const size_t scan = rebuild_scan_tmp_bytes(c.scap);
  if (dmalloc(&pool2, c.pcap) != hipSuccess || dmalloc(&rpool2, h->g.d.rpcap) != hipSuccess ||
      tmp.ensure(Carver::need({c.scap * 8, c.scap * 8, 2 * scan})) != hipSuccess) {
    (void)hipGetLastError();
    if (pool2) hipFree(pool2);
    if (rpool2) hipFree(rpool2);
    return CRGC_E_NOMEM;
  }
  Carver cv(tmp.ptr);
  uint64_t *pp = cv.take<uint64_t>(c.scap), *rp = cv.take<uint64_t>(c.scap);
  void *st = cv.take<uint64_t>(2 * scan / 8);
  const uint64_t old_p = h->pool_top, old_r = h->rpool_top;
  hipError_t e = launch_repack(h->g.d, h->slot_top, h->proxy_top, pp, rp, st, pool2, rpool2, h->stream);
  if (e == hipSuccess) e = sync_counters(h);
  tmp.release();
  if (e != hipSuccess) {  // the device may have moved part of adj / radj: unusable
    hipFree(pool2);
    hipFree(rpool2);
    h->poisoned = true;
    return map_hip(e);
  }
  hipFree(h->g.d.pool);
  hipFree(h->g.d.rpool);
  h->g.d.pool = pool2;
  h->g.d.rpool = rpool2;
  ++h->n_repack;
  if (h->knobs.level_log)
    fprintf(stderr, "[crgc] repack: pool %llu -> %llu, candidate pool %llu -> %llu (of %llu)\n",
            (unsigned long long)old_p, (unsigned long long)h->pool_top, (unsigned long long)old_r,
            (unsigned long long)h->rpool_top, (unsigned long long)c.pcap);
  return CRGC_OK;
}

// Make sure `ids` more vertices and `atoms` more edge updates fit.
int ensure_capacity(crgc_graph *h, uint64_t ids, uint64_t atoms) {
  // A merge's relocations need at most 2*(stored + new) + 4*touched pool
  // entries in either direction (power-of-two segments).
  auto pools_fit = [&](uint64_t pt, uint64_t rt, uint64_t eu) {
    const Caps &c = h->g.caps;
    return pt + 2 * eu + 6 * atoms <= c.pcap && rt + 2 * eu + 6 * atoms + 4 * ids <= c.pcap;
  };
  // (new shadows fill the shadows' region, new proxies the proxy region; `ids`
  // bounds either)
  // (slot reuse: the id table also holds the tombstones of the collected ids
  // whose slots new shadows took since its last rehash — reused, plus the
  // merges' takes since the last reclaim — which slot_top no longer bounds)
  const uint64_t tomb = h->g.d.freel ? h->hctr->reused + h->hctr->free_used : 0;
  auto rest_fits = [&](uint64_t st, uint64_t pt, uint64_t eu) {
    const Caps &c = h->g.caps;
    return st + ids <= c.pbase && (h->G <= 1 || pt + ids <= c.scap - c.pbase) &&
           (st + pt + ids + tomb) * 10 <= c.hcap * 7 && (eu + atoms) * 10 <= c.ecap * 7;
  };
  // upper bounds since the last sync (an unsharded graph has no proxies: its
  // pending ids are counted once, in st)
  const uint64_t st = h->slot_top + h->ids_since, pt = h->G > 1 ? h->proxy_top + h->ids_since : 0;
  const uint64_t eu = h->etab_used + h->atoms_since;
  const uint64_t grow = 2 * (h->etab_used + h->atoms_since) + 6 * h->atoms_since;
  // (+ 4 reverse-candidate entries per new shadow: k_ids' first segments)
  if (rest_fits(st, pt, eu) && pools_fit(h->pool_top + grow, h->rpool_top + grow + 4 * h->ids_since, eu))
    return CRGC_OK;
  HIP_TRY(sync_counters(h));
  if (int rc = device_error(h)) return rc;
  const bool rest = rest_fits(h->slot_top, h->proxy_top, h->etab_used);
  if (rest && pools_fit(h->pool_top, h->rpool_top, h->etab_used)) return CRGC_OK;
  // only the pools are short: reclaim their dead space before rebuilding the
  // whole graph (a rebuild allocates a second graph; a repack, two pools)
  if (rest) {
    const int rc = repack(h);
    if (rc == CRGC_OK && pools_fit(h->pool_top, h->rpool_top, h->etab_used)) return CRGC_OK;
    if (rc != CRGC_OK && rc != CRGC_E_NOMEM) return rc;
    return rebuild(h, ids, atoms);
  }
  // slots or tables are short: a graph with few dead slots grows (same slots),
  // whose pools may then want a repack; else a rebuild
  if (int rc = rebuild(h, ids, atoms, /*may_grow=*/true)) return rc;
  if (rest_fits(h->slot_top, h->proxy_top, h->etab_used) && pools_fit(h->pool_top, h->rpool_top, h->etab_used))
    return CRGC_OK;
  if (rest_fits(h->slot_top, h->proxy_top, h->etab_used)) {
    const int rc = repack(h);
    if (rc == CRGC_OK && pools_fit(h->pool_top, h->rpool_top, h->etab_used)) return CRGC_OK;
    if (rc != CRGC_OK && rc != CRGC_E_NOMEM) return rc;
  }
  return rebuild(h, ids, atoms);
}

// Upper bounds, without a synchronisation, of the slots in use: the shadows'
// (slot_top) and the proxy region's (sharded graphs), and their blocks.
uint64_t home_top_ub(const crgc_graph *h) {
  return std::min<uint64_t>(h->slot_top + h->ids_since, h->g.caps.pbase);
}
uint64_t proxy_top_ub(const crgc_graph *h) {
  return h->G > 1 ? std::min<uint64_t>(h->proxy_top + h->ids_since, h->g.caps.scap - h->g.caps.pbase) : 0;
}
uint64_t blocks_of(uint64_t slots) { return (slots + BLK_SLOTS - 1) / BLK_SLOTS; }

void note_merge(crgc_graph *h, uint64_t ids, uint64_t atoms) {
  h->ids_since += ids;
  h->atoms_since += atoms;
}

// Copy `bytes` from a host or device pointer into the staging area.
template <class T>
const T *stage(crgc_graph *h, Carver &cv, const T *src, uint64_t n, uint32_t memory) {
  if (memory == CRGC_MEM_DEVICE) return src;
  if (n == 0) return nullptr;
  T *dst = cv.take<T>(n);
  hipMemcpyAsync(dst, src, n * sizeof(T), hipMemcpyHostToDevice, h->stream);
  return dst;
}

// Host batches are read by stream-ordered copies; the ABI promises that the
// caller's buffers are free again when the call returns (crgc.h), so a merge
// that staged host memory waits for those copies (only: ev[3] is recorded
// right after them, the kernels behind it keep running).  The guard is armed
// before the first copy and waits on every return path, errors included.
struct Staged {
  crgc_graph *h;
  bool armed, recorded = false;
  Staged(crgc_graph *g, uint32_t memory) : h(g), armed(memory == CRGC_MEM_HOST) {}
  hipError_t mark() {
    if (!armed) return hipSuccess;
    const hipError_t e = hipEventRecord(h->ev[3], h->stream);
    recorded = e == hipSuccess;
    return e;
  }
  hipError_t wait() {
    if (!armed) return hipSuccess;
    armed = false;
    return recorded ? event_wait(h->ev[3], h->knobs.spin_us) : stream_wait(h->stream, h->knobs.spin_us);
  }
  ~Staged() { wait(); }
  Staged(const Staged &) = delete;
  Staged &operator=(const Staged &) = delete;
};

int check_graph(crgc_graph *h) {
  if (!h) return CRGC_E_INVAL;
  if (h->poisoned) return CRGC_E_POISONED;
  return CRGC_OK;
}

}  // namespace

extern "C" {

const char *crgc_strerror(int code) {
  switch (code) {
    case CRGC_OK: return "ok";
    case CRGC_E_INVAL: return "invalid argument";
    case CRGC_E_NOMEM: return "out of memory";
    case CRGC_E_DEVICE: return "device error";
    case CRGC_E2BIG: return "output buffer too small";
    case CRGC_E_NULL_SUPERVISOR: return "local garbage shadow without supervisor (reference NPE)";
    case CRGC_E_UNDO_NEW_SHADOW: return "undo log names an unknown actor (reference CME)";
    case CRGC_E_POISONED: return "graph unusable after an earlier error";
    case CRGC_E_TIMEOUT: return "device wait bound exceeded";
    default: return "unknown error";
  }
}

const char *crgc_last_error_detail(void) { return err_detail; }

int crgc_create(const crgc_config *cfg, crgc_graph **out) {
  if (!out) return CRGC_E_INVAL;
  *out = nullptr;
  if (cfg && cfg->abi_version != CRGC_ABI_VERSION) return CRGC_E_INVAL;
  crgc_graph *h = new (std::nothrow) crgc_graph();
  if (!h) return CRGC_E_NOMEM;
  h->device = cfg ? cfg->device : 0;
  h->F = (cfg && cfg->entry_field_size) ? cfg->entry_field_size : 4;
  h->DGS = (cfg && cfg->delta_graph_size) ? cfg->delta_graph_size : 64;
  h->knobs.read();
  if (h->knobs.walk) h->walk_ok = walk_fits(h->device);
  // A transport makes the handle a shard (a transport with n_shards == 1 runs
  // the sharded protocol on one shard: a self-check of the transport).
  if (cfg && (cfg->n_shards > 1 || cfg->transport)) {
    if (cfg->n_shards < 1 || cfg->n_shards > MAX_SHARDS || cfg->shard >= cfg->n_shards || !cfg->transport ||
        cfg->transport->n_shards != cfg->n_shards ||
        !cfg->transport->accepts(cfg->shard, cfg->device)) {
      delete h;
      return CRGC_E_INVAL;
    }
    h->G = cfg->n_shards;
    h->shard = cfg->shard;
    h->tp = cfg->transport;
    h->route = h->knobs.route;
  }
  DeviceGuard dg(h->device);
  int rc = CRGC_OK;
  do {
    if (cfg && cfg->stream) {
      h->stream = (hipStream_t)cfg->stream;
    } else {
      if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess) {
        rc = DEV_FAIL("");
        break;
      }
      h->own_stream = true;
    }
    for (auto &e : h->ev)
      if (hipEventCreate(&e) != hipSuccess) rc = DEV_FAIL("");
    h->use_side = h->knobs.side_stream;  // A/B switch
    h->chunk_host = h->knobs.chunk_host;
    h->chunk_max = h->knobs.chunk_max;
    h->chunk_reg = h->knobs.chunk_reg;
    // (The copy stream at the highest priority, with registered batches in up
    // to 6 chunks, made the registered merge call slower, 1.19 -> 1.47 ms:
    // profiles/r4j.  Each chunk is a whole merge with its fixed costs.)
    int prio_lo = 0, prio_hi = 0;
    hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi);
    if (hipStreamCreateWithFlags(&h->cpy, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&h->ev_cstart, hipEventDisableTiming) != hipSuccess)
      rc = DEV_FAIL("");
    for (auto &e : h->ev_chunk)
      if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) rc = DEV_FAIL("");
    for (auto &e : h->ev_cfree)
      if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) rc = DEV_FAIL("");
    // CRGC_SIDE_PRIO=1: the side stream (the merge's critical path) at the
    // device's highest priority, so its workgroups dispatch first
    const int side_prio = h->knobs.side_prio ? prio_hi : 0;
    if (hipStreamCreateWithPriority(&h->side, hipStreamNonBlocking, side_prio) != hipSuccess ||
        hipEventCreateWithFlags(&h->ev_fork, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&h->ev_join, hipEventDisableTiming) != hipSuccess)
      rc = DEV_FAIL("");
    if (rc) break;
    if (hipMalloc(&h->ctr, sizeof(Counters)) != hipSuccess ||
        hipHostMalloc(&h->hctr, sizeof(Counters), hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc(&h->h_small, 8 * (size_t)MAX_SHARDS * (MAX_SHARDS + 8), hipHostMallocDefault) !=
            hipSuccess ||
        hipHostMalloc(&h->h_route, ROUTE_TABLE_BYTES, hipHostMallocDefault) != hipSuccess) {
      rc = CRGC_E_NOMEM;
      break;
    }
    hipMemsetAsync(h->ctr, 0, sizeof(Counters), h->stream);
    memset(h->hctr, 0, sizeof(Counters));
    if (hipHostGetDevicePointer((void **)&h->hctr_dev, h->hctr, 0) != hipSuccess || !h->hctr_dev) {
      rc = DEV_FAIL("");
      break;
    }
    if (hipHostGetDevicePointer((void **)&h->h_small_dev, h->h_small, 0) != hipSuccess) {
      (void)hipGetLastError();  // (ag_u64 then copies host words by the runtime)
      h->h_small_dev = nullptr;
    }
    const uint64_t v0 = cfg && cfg->vertex_capacity ? cfg->vertex_capacity : (1u << 16);
    const uint64_t e0 = cfg && cfg->edge_capacity ? cfg->edge_capacity : 8 * v0;
    // a shard's proxy region from its own hint (ABI 5); without one it is sized
    // like the shadows' region
    const uint64_t p0 = cfg && cfg->proxy_capacity ? cfg->proxy_capacity : v0;
    Caps c = caps_create(v0, p0, h->G > 1, e0, h->knobs.idtab_x2);
    if (hipError_t e = alloc_arrays(h->g, c, h->ctr, h->stream, h->G, h->shard, h->tp != nullptr, reuse_on(h))) {
      rc = map_hip(e);
      break;
    }
    if (hipStreamSynchronize(h->stream) != hipSuccess) rc = DEV_FAIL("");
  } while (0);
  if (rc) {
    crgc_destroy(h);
    return rc;
  }
  *out = h;
  return CRGC_OK;
}

void crgc_destroy(crgc_graph *h) {
  if (!h) return;
  DeviceGuard dg(h->device);
  if (h->stream) hipStreamSynchronize(h->stream);
  free_arrays(h->g);
  h->stage.release();
  for (Scratch &x : h->cstage) x.release();
  h->work.release();
  for (Scratch *x : {&h->x_send, &h->x_slot, &h->x_recv, &h->x_ans, &h->x_ans_back, &h->x_small,
                     &h->x_pack, &h->x_pack_recv, &h->x_route, &h->x_route_send, &h->x_cat,
                     &h->x_dg, &h->x_dg_out, &h->x_chain, &h->x_gc, &h->x_gc_list, &h->x_bin, &h->x_chunk,
                     &h->x_gvis, &h->x_wgc})
    x->release();
  if (h->ctr) hipFree(h->ctr);
  if (h->hctr) hipHostFree(h->hctr);
  if (h->h_small) hipHostFree(h->h_small);
  if (h->h_bounce) hipHostFree(h->h_bounce);
  if (h->h_route) hipHostFree(h->h_route);
  if (h->roots_buf) hipFree(h->roots_buf);
  if (h->side) {
    hipStreamSynchronize(h->side);
    hipStreamDestroy(h->side);
  }
  for (auto &p : h->pinned) hipHostUnregister(p.first);
  if (h->cpy) {
    hipStreamSynchronize(h->cpy);
    hipStreamDestroy(h->cpy);
  }
  if (h->ev_cstart) hipEventDestroy(h->ev_cstart);
  for (auto &e : h->ev_chunk)
    if (e) hipEventDestroy(e);
  for (auto &e : h->ev_cfree)
    if (e) hipEventDestroy(e);
  if (h->ev_fork) hipEventDestroy(h->ev_fork);
  if (h->ev_join) hipEventDestroy(h->ev_join);
  for (auto &e : h->ev)
    if (e) hipEventDestroy(e);
  for (auto &e : h->lvl_ev) hipEventDestroy(e);
  for (auto &e : h->chunk_ev) hipEventDestroy(e);
  if (h->own_stream && h->stream) hipStreamDestroy(h->stream);
  delete h;
}

// Shared tail of every merge: the edge pipeline over the staged atoms
// (crgc_edges.hip).  Partition geometry: 2..1024 hash buckets of slots (about
// 256 slots each below that); <= 512 blocks of >= 1024 atoms.
static void edge_geometry(const crgc_graph *h, uint64_t max_atoms, uint32_t &bshift, uint32_t &nbk,
                          uint64_t &nblk) {
  uint32_t lg = 0;
  while ((1ull << lg) < h->g.d.scap) ++lg;
  // 512 owner buckets at scale: one 1024-thread workgroup per bucket, two per CU,
  // so every bucket is resident at once (1024 left a second, partial wave of
  // workgroups: the C2 merge 20-30 us slower, profiles/r2p/ab_buckets.txt)
  uint32_t lk = lg > 18 ? 9u : (lg > 9 ? lg - 8 : 1u);
  // test hook: fewer buckets, so buckets take several rounds of atoms
  if (h->knobs.buckets_log2) lk = (uint32_t)h->knobs.buckets_log2;
  bshift = 32 - lk;
  nbk = 1u << lk;
  nblk = std::min<uint64_t>((max_atoms + 1023) / 1024, 512);
}

// Work scratch of a merge's atoms and its edge pipeline.
static size_t edge_scratch(const crgc_graph *h, uint64_t max_atoms) {
  uint32_t bshift, nbk;
  uint64_t nblk;
  edge_geometry(h, max_atoms, bshift, nbk, nblk);
  const uint64_t nh = (uint64_t)nbk * nblk;
  // the callers' atom arrays (o, t, d, exact count), then the pipeline's own
  return Carver::need({max_atoms * 4, max_atoms * 4, max_atoms * 4, 8, nh * 4, nh * 8,
                       ((nh + 1023) / 1024) * 4 * 8 + 64, 16, max_atoms * 8, max_atoms * 4, max_atoms * 4,
                       max_atoms * 4, max_atoms * 4, max_atoms * 4, 8});
}

static int run_edges(crgc_graph *h, uint32_t *ao, uint32_t *at, int32_t *ad, uint64_t max_atoms,
                     Carver &cv, const uint64_t *n_atoms_dev = nullptr, hipStream_t s = nullptr) {
  if (max_atoms == 0) return CRGC_OK;
  EdgeArgs ea{};
  ea.err = &h->g.d.ctr->err;
  ea.max_atoms = max_atoms;
  ea.n_atoms_dev = n_atoms_dev;
  ea.atom_o = ao;
  ea.atom_t = at;
  ea.atom_d = ad;
  edge_geometry(h, max_atoms, ea.bshift, ea.nbk, ea.nblk);
  const uint64_t nh = (uint64_t)ea.nbk * ea.nblk;
  ea.hist = cv.take<uint32_t>(nh);
  ea.hoff = cv.take<uint64_t>(nh);
  ea.bsum = cv.take<uint64_t>(((nh + 1023) / 1024) * 4 + 8);
  ea.tot = cv.take<unsigned long long>(2);
  ea.pk = cv.take<uint64_t>(max_atoms);
  ea.pv = cv.take<uint32_t>(max_atoms);
  ea.rv_t = cv.take<uint32_t>(max_atoms);
  ea.rv_i = cv.take<uint32_t>(max_atoms);
  ea.rv_o = cv.take<uint32_t>(max_atoms);
  ea.rv_b = cv.take<uint32_t>(max_atoms);
  ea.n_ov = cv.take<unsigned long long>(1);
  HIP_TRY(launch_edges(h->g.d, ea, s ? s : h->stream));
  return CRGC_OK;
}

// The edge pipeline on the side stream, forked from the graph's stream after
// the atoms are written and joined before the merge returns (on every path).
struct SideFork {
  crgc_graph *h;
  bool forked = false;
  explicit SideFork(crgc_graph *g) : h(g) {}
  hipError_t fork() {
    if (!h->use_side) return hipSuccess;
    hipError_t e = hipEventRecord(h->ev_fork, h->stream);
    if (e == hipSuccess) e = hipStreamWaitEvent(h->side, h->ev_fork, 0);
    forked = e == hipSuccess;
    return e;
  }
  hipStream_t stream() const { return forked ? h->side : h->stream; }
  hipError_t join() {
    if (!forked) return hipSuccess;
    forked = false;
    hipError_t e = hipEventRecord(h->ev_join, h->side);
    if (e == hipSuccess) e = hipStreamWaitEvent(h->stream, h->ev_join, 0);
    if (e != hipSuccess) hipStreamSynchronize(h->side);  // never leave the side stream unordered
    return e;
  }
  ~SideFork() { join(); }
};

}  // extern "C"

namespace {
// ---- sharded graphs: collective helpers ---------------------------------------
// All-gather K u64 per shard: `parts` device sources concatenated -> out[G*K] (host).
constexpr size_t SMALL_BYTES = 8 * (size_t)MAX_SHARDS * (MAX_SHARDS + 8);  // h_small

static int ag_u64(crgc_graph *h, std::initializer_list<std::pair<const void *, uint32_t>> parts,
                  uint64_t *out) {
  uint32_t K = 0;
  for (auto &p : parts) K += p.second;
  const size_t bytes = (size_t)K * 8;
  if (h->x_small.ensure(bytes * (h->G + 1)) != hipSuccess) return CRGC_E_NOMEM;
  char *snd = (char *)h->x_small.ptr, *rcv = snd + bytes;
  // one gather kernel (device words, or host words through h_small's device view)
  const uint64_t *src[8];
  uint32_t cnt[8], k = 0;
  bool kern = parts.size() <= 8 && h->h_small_dev;
  for (auto &p : parts) {
    if (!kern) break;
    const char *c = (const char *)p.first, *hs = (const char *)h->h_small;
    if (c >= hs && c < hs + SMALL_BYTES) c = (const char *)h->h_small_dev + (c - hs);
    src[k] = (const uint64_t *)c;
    cnt[k++] = p.second;
  }
  if (kern) {
    HIP_TRY(gather_u64_parts(src, cnt, k, (uint64_t *)snd, h->stream));
  } else {
    size_t at = 0;
    for (auto &p : parts) {
      HIP_TRY(hipMemcpyAsync(snd + at, p.first, (size_t)p.second * 8, hipMemcpyDefault, h->stream));
      at += (size_t)p.second * 8;
    }
  }
  if (int rc = h->tp->allgather(h->shard, snd, rcv, bytes, h->stream)) {
    h->poisoned = true;
    return rc;
  }
  // the pinned staging words hold 8 * MAX_SHARDS * (MAX_SHARDS + 8) bytes; a
  // larger gather (K = 2 + 4G at G > 47) lands in `out` directly
  const bool staged = bytes * h->G <= 8 * (size_t)MAX_SHARDS * (MAX_SHARDS + 8);
  HIP_TRY(hipMemcpyAsync(staged ? (void *)h->h_small : (void *)out, rcv, bytes * h->G, hipMemcpyDeviceToHost,
                         h->stream));
  HIP_TRY(hsync(h));
  if (staged) memcpy(out, h->h_small, bytes * h->G);
  return CRGC_OK;
}

// All-gather K host u64 per shard -> out[G*K] (host).
static int ag_host(crgc_graph *h, const uint64_t *vals, uint32_t K, uint64_t *out) {
  memcpy(h->h_small, vals, (size_t)K * 8);
  if (h->h_small_dev && (size_t)K * 8 <= SMALL_BYTES) return ag_u64(h, {{h->h_small, K}}, out);
  if (h->x_small.ensure((size_t)K * 8 * (h->G + 2)) != hipSuccess) return CRGC_E_NOMEM;
  char *tmp = (char *)h->x_small.ptr + (size_t)K * 8 * (h->G + 1);
  HIP_TRY(hipMemcpyAsync(tmp, h->h_small, (size_t)K * 8, hipMemcpyHostToDevice, h->stream));
  return ag_u64(h, {{tmp, K}}, out);
}

// Exchange by a count matrix M (M[r*G + d] = items r sends d, `elem` bytes
// each): send holds this shard's items grouped by destination in shard order;
// recv gets every source's items for this shard, in source order.
// transpose = true runs the reverse direction (answers back to the askers).
static int a2a(crgc_graph *h, const void *send, const uint64_t *M, size_t elem, Scratch &recv,
               bool transpose, uint64_t *n_recv) {
  const uint32_t G = h->G, me = h->shard;
  auto cnt = [&](uint32_t from, uint32_t to) { return transpose ? M[to * G + from] : M[from * G + to]; };
  size_t soff[MAX_SHARDS], sb[MAX_SHARDS], roff[MAX_SHARDS], rb[MAX_SHARDS];
  size_t so = 0, ro = 0;
  for (uint32_t r = 0; r < G; ++r) {
    soff[r] = so;
    sb[r] = cnt(me, r) * elem;
    so += sb[r];
    roff[r] = ro;
    rb[r] = cnt(r, me) * elem;
    ro += rb[r];
  }
  if (recv.ensure(ro + 8) != hipSuccess) return CRGC_E_NOMEM;
  if (int rc = h->tp->alltoallv(h->shard, send, soff, sb, recv.ptr, roff, rb, h->stream)) {
    h->poisoned = true;
    return rc;
  }
  *n_recv = ro / elem;
  return CRGC_OK;
}

// ---- batch packing (sharded merges all-gather the shards' batches) ----------
struct Layout {
  size_t off[11];
  size_t size[11];
  size_t total;
};

static Layout make_layout(std::initializer_list<size_t> sizes) {
  Layout l{};
  size_t o = 0;
  int i = 0;
  for (size_t s : sizes) {
    o = (o + 255) & ~(size_t)255;
    l.off[i] = o;
    l.size[i] = s;
    o += s;
    ++i;
  }
  l.total = (o + 255) & ~(size_t)255;  // shards' blocks sit back to back: keep them aligned
  return l;
}

static Layout entry_layout(uint64_t n, uint64_t C, uint64_t S, uint64_t U) {
  return make_layout({n * 8, n * 2, n, (n + 1) * 4, C * 8, C * 8, (n + 1) * 4, S * 8, (n + 1) * 4,
                      U * 8, U * 2});
}

static Layout delta_layout(uint64_t n, uint64_t nout) {
  return make_layout({n * 8, n * 4, n * 8, n, (n + 1) * 4, nout * 8, nout * 4});
}

static int pack(crgc_graph *h, const Layout &l, const void *const *src, int narr, uint32_t memory,
                char *dst) {
  const hipMemcpyKind k = memory == CRGC_MEM_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
  for (int i = 0; i < narr; ++i)
    if (l.size[i]) HIP_TRY(hipMemcpyAsync(dst + l.off[i], src[i], l.size[i], k, h->stream));
  return CRGC_OK;
}

// All-gather the shards' packed batches: vals = per-shard header (status
// first), returns the G headers and the packed bytes of every shard, in shard
// order, in x_pack_recv (offsets in roff).
template <class LayoutOf>
static int gather_batches(crgc_graph *h, const uint64_t *hdr, uint32_t K, const void *const *src,
                          int narr, uint32_t memory, LayoutOf layout_of, std::vector<uint64_t> &H,
                          std::vector<size_t> &roff) {
  const uint32_t G = h->G;
  H.assign((size_t)G * K, 0);
  if (int rc = ag_host(h, hdr, K, H.data())) return rc;
  // every shard learns every shard's validation verdict: all fail together
  const int mine_rc = (int)(int64_t)H[(size_t)h->shard * K];
  for (uint32_t r = 0; r < G; ++r)
    if ((int64_t)H[(size_t)r * K] != 0) return mine_rc ? mine_rc : CRGC_E_INVAL;
  const Layout mine = layout_of(&H[(size_t)h->shard * K]);
  size_t soff[MAX_SHARDS], sb[MAX_SHARDS], rb[MAX_SHARDS];
  roff.assign(G, 0);
  size_t tot = 0;
  for (uint32_t r = 0; r < G; ++r) {
    soff[r] = 0;
    sb[r] = mine.total;
    roff[r] = tot;
    rb[r] = layout_of(&H[(size_t)r * K]).total;
    tot += rb[r];
  }
  if (h->x_pack.ensure(mine.total) != hipSuccess || h->x_pack_recv.ensure(tot) != hipSuccess)
    return CRGC_E_NOMEM;
  if (int rc = pack(h, mine, src, narr, memory, (char *)h->x_pack.ptr)) return rc;
  if (memory == CRGC_MEM_HOST && narr) HIP_TRY(hsync(h));  // caller's buffers free on return
  if (int rc = h->tp->alltoallv(h->shard, h->x_pack.ptr, soff, sb, h->x_pack_recv.ptr, roff.data(), rb,
                                h->stream)) {
    h->poisoned = true;
    return rc;
  }
  return CRGC_OK;
}

}  // namespace

extern "C" {

// Validates an entry batch and learns its record counts (exact for host
// batches; for device batches too when `exact`, by reading the last offsets).
// Small device-to-host reads go through the handle's pinned staging words when
// they fit: a copy into pageable memory is staged and waited for inside the
// runtime, on its blocking wait (not our polling one, crgc_internal.hpp).
// `off` keeps a read clear of the words an all-gather in flight uses.
constexpr size_t SMALL_XFLAG_OFF = SMALL_BYTES / 2;
constexpr size_t SMALL_PEND_OFF = SMALL_BYTES - 64;  // a mark round's pending word (mark_all)
static hipError_t d2h_small(crgc_graph *h, void *dst, const void *src, size_t bytes, size_t off = 0) {
  void *to = off + bytes <= SMALL_BYTES ? (void *)((char *)h->h_small + off) : dst;
  return hipMemcpyAsync(to, src, bytes, hipMemcpyDeviceToHost, h->stream);
}
static void d2h_small_done(crgc_graph *h, void *dst, size_t bytes, size_t off = 0) {
  if (off + bytes <= SMALL_BYTES) memcpy(dst, (char *)h->h_small + off, bytes);
}

static int entry_counts(crgc_graph *h, const crgc_entry_batch *b, bool exact, uint64_t *C, uint64_t *S,
                        uint64_t *U) {
  if (!b || b->memory > CRGC_MEM_DEVICE) return CRGC_E_INVAL;
  const uint64_t n = b->n_entries;
  *C = *S = *U = 0;
  if (n == 0) return CRGC_OK;
  if (n >= (1ull << 31) / (h->F + 1)) return CRGC_E_INVAL;
  if (!b->self || !b->recv_count || !b->flags || !b->created_off || !b->spawned_off || !b->updated_off)
    return CRGC_E_INVAL;
  if (b->memory == CRGC_MEM_HOST) {
    *C = b->created_off[n];
    *S = b->spawned_off[n];
    *U = b->updated_off[n];
    if (b->created_off[0] || b->spawned_off[0] || b->updated_off[0]) return CRGC_E_INVAL;
  } else if (exact) {
    uint32_t v[3] = {0, 0, 0};
    HIP_TRY(hipMemcpyAsync(&v[0], b->created_off + n, 4, hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hipMemcpyAsync(&v[1], b->spawned_off + n, 4, hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hipMemcpyAsync(&v[2], b->updated_off + n, 4, hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hsync(h));
    *C = v[0];
    *S = v[1];
    *U = v[2];
  } else if (b->created_owner && b->created_target && b->spawned && b->updated_ref && b->updated_info) {
    *C = *S = *U = n * h->F;  // bounds; kernels read the exact offsets
    return CRGC_OK;
  } else {
    // a null record array is legal only when its count is zero: learn the
    // counts (one round trip) so the checks below refuse the batch otherwise
    return entry_counts(h, b, true, C, S, U);
  }
  if (*C > n * h->F || *S > n * h->F || *U > n * h->F) return CRGC_E_INVAL;
  if ((*C && (!b->created_owner || !b->created_target)) || (*S && !b->spawned) ||
      (*U && (!b->updated_ref || !b->updated_info)))
    return CRGC_E_INVAL;
  return CRGC_OK;
}

// One batch into this shard (every record applied by its home shard).
static int merge_entries_one(crgc_graph *h, const crgc_entry_batch *b, uint64_t C, uint64_t S,
                             uint64_t U) {
  const uint64_t n = b->n_entries;
  if (n == 0) return CRGC_OK;
  const uint64_t ids = n + 2 * C + S + U;
  const uint64_t max_atoms = n * 2 * (uint64_t)h->F;
  if (h->knobs.repack_each)
    if (int rc = repack(h)) return rc;
  if (int rc = ensure_capacity(h, ids, C + U)) return rc;

  const size_t host_bytes =
      b->memory == CRGC_MEM_HOST
          ? Carver::need({n * 8, n * 2, n, (n + 1) * 4, C * 8, C * 8, (n + 1) * 4, S * 8, (n + 1) * 4,
                          U * 8, U * 2})
          : 0;
  const bool sh = h->tp;
  const uint64_t nb256 = (n + 255) / 256;
  const size_t work_bytes =
      Carver::need({n * 4, n * h->F * 4, n * h->F * 4, n * h->F * 4, n * h->F * 4, sh ? n : 0,
                    sh ? n * h->F * 8 : 0, 8, nb256 * 256 * 4, nb256 * 256 * h->F * 4, nb256 * 8}) +
      edge_scratch(h, max_atoms);
  if (h->stage.ensure(host_bytes + 256) != hipSuccess || h->work.ensure(work_bytes) != hipSuccess)
    return CRGC_E_NOMEM;
  Carver sc(h->stage.ptr), wc(h->work.ptr);
  Staged staged(h, b->memory);
  EntryArgs a{};
  a.n = n;
  a.F = h->F;
  a.epoch = ++h->epoch;
  a.self = stage(h, sc, b->self, n, b->memory);
  a.recv = stage(h, sc, b->recv_count, n, b->memory);
  a.flags = stage(h, sc, b->flags, n, b->memory);
  a.c_off = stage(h, sc, b->created_off, n + 1, b->memory);
  a.c_owner = stage(h, sc, b->created_owner, C, b->memory);
  a.c_target = stage(h, sc, b->created_target, C, b->memory);
  a.s_off = stage(h, sc, b->spawned_off, n + 1, b->memory);
  a.spawned = stage(h, sc, b->spawned, S, b->memory);
  a.u_off = stage(h, sc, b->updated_off, n + 1, b->memory);
  a.u_ref = stage(h, sc, b->updated_ref, U, b->memory);
  a.u_info = stage(h, sc, b->updated_info, U, b->memory);
  HIP_TRY(staged.mark());
  a.self_slot = wc.take<uint32_t>(n);
  a.spawn_slot = wc.take<uint32_t>(n * h->F);
  a.ct_slot = wc.take<uint32_t>(n * h->F);
  a.co_slot = wc.take<uint32_t>(n * h->F);
  a.u_slot = wc.take<uint32_t>(n * h->F);
  if (sh) {
    a.self_need = wc.take<uint8_t>(n);
    a.u_partner = wc.take<uint64_t>(n * h->F);
  }
  a.atom_o = wc.take<uint32_t>(max_atoms);
  a.atom_t = wc.take<uint32_t>(max_atoms);
  a.atom_d = wc.take<int32_t>(max_atoms);
  a.n_atoms = wc.take<uint64_t>(1);
  a.conf_v = wc.take<uint32_t>(nb256 * 256);
  a.conf_s = wc.take<uint32_t>(nb256 * 256 * h->F);
  a.conf_n = wc.take<uint32_t>(2 * nb256);
  // a batch refused for its offsets writes no atoms and the edge pipeline
  // skips it (EdgeArgs::err), so the atom arrays need no clearing
  HIP_TRY(launch_entries(ids_view(h), a, h->stream, 0));
  {
    SideFork sf(h);
    HIP_TRY(sf.fork());
    if (int rc = run_edges(h, a.atom_o, a.atom_t, a.atom_d, max_atoms, wc, a.n_atoms, sf.stream())) return rc;
    HIP_TRY(launch_entries(h->g.d, a, h->stream, 1));
    HIP_TRY(sf.join());
  }
  note_merge(h, ids, C + U);
  HIP_TRY(staged.wait());
  return CRGC_OK;
}

static size_t part_bytes(uint64_t n, uint64_t C, uint64_t S, uint64_t U) {
  return n ? entry_layout(n, C, S, U).total : 0;
}

static RoutePart part_at(char *base, uint64_t n, uint64_t C, uint64_t S, uint64_t U) {
  const Layout l = entry_layout(n, C, S, U);
  RoutePart p;
  p.self = (uint64_t *)(base + l.off[0]);
  p.recv = (int16_t *)(base + l.off[1]);
  p.flags = (uint8_t *)(base + l.off[2]);
  p.c_off = (uint32_t *)(base + l.off[3]);
  p.c_owner = (uint64_t *)(base + l.off[4]);
  p.c_target = (uint64_t *)(base + l.off[5]);
  p.s_off = (uint32_t *)(base + l.off[6]);
  p.spawned = (uint64_t *)(base + l.off[7]);
  p.u_off = (uint32_t *)(base + l.off[8]);
  p.u_ref = (uint64_t *)(base + l.off[9]);
  p.u_info = (int16_t *)(base + l.off[10]);
  return p;
}

static crgc_entry_batch batch_of(const RoutePart &p, uint64_t n) {
  crgc_entry_batch v{};
  v.n_entries = n;
  v.self = p.self;
  v.recv_count = p.recv;
  v.flags = p.flags;
  v.created_off = p.c_off;
  v.created_owner = p.c_owner;
  v.created_target = p.c_target;
  v.spawned_off = p.s_off;
  v.spawned = p.spawned;
  v.updated_off = p.u_off;
  v.updated_ref = p.u_ref;
  v.updated_info = p.u_info;
  v.memory = CRGC_MEM_DEVICE;
  return v;
}

// Sharded, routed (crgc_route.hip): every shard cuts its batch into one part
// per destination shard, one all-to-all moves the parts, and every shard
// merges what it received, concatenated in shard order, as one batch.
static int merge_entries_routed(crgc_graph *h, const crgc_entry_batch *b, int vrc, uint64_t C, uint64_t S,
                                uint64_t U) {
  const uint32_t G = h->G, me = h->shard;
  const uint64_t n = vrc ? 0 : b->n_entries;
  const uint64_t nblk = (n + RT_THREADS - 1) / RT_THREADS;
  const size_t need = Carver::need({8, (size_t)G * 32, (size_t)G * nblk * 8, (size_t)G * nblk * 32,
                                    sizeof(RoutePart) * ROUTE_MAX_SHARDS, sizeof(ConcatPart) * ROUTE_MAX_SHARDS});
  if (h->x_route.ensure(need) != hipSuccess) return CRGC_E_NOMEM;
  Carver rv(h->x_route.ptr);
  RouteArgs a{};
  a.err = rv.take<unsigned long long>(1);
  a.totals = rv.take<uint64_t>((size_t)G * 4);
  a.blk_tot = rv.take<uint64_t>((size_t)G * nblk);
  a.blk_pre = rv.take<uint64_t>((size_t)G * nblk * 4);
  RoutePart *d_parts = rv.take<RoutePart>(ROUTE_MAX_SHARDS);
  ConcatPart *d_cat = rv.take<ConcatPart>(ROUTE_MAX_SHARDS);
  // err and totals (carved 256 B apart, from the region's start) zeroed by one dispatch
  HIP_TRY(launch_zero_u64(a.err, (uint32_t)((char *)(a.totals + (size_t)G * 4) - (char *)a.err) / 8, h->stream));
  if (n) {
    const void *src[11] = {b->self,    b->recv_count, b->flags,       b->created_off, b->created_owner,
                           b->created_target, b->spawned_off, b->spawned, b->updated_off, b->updated_ref,
                           b->updated_info};
    const void *p[11];
    if (b->memory == CRGC_MEM_HOST) {  // one staging copy per array, then every part from HBM
      const Layout l = entry_layout(n, C, S, U);
      if (h->x_pack.ensure(l.total) != hipSuccess) return CRGC_E_NOMEM;
      if (int rc = pack(h, l, src, 11, CRGC_MEM_HOST, (char *)h->x_pack.ptr)) return rc;
      for (int i = 0; i < 11; ++i) p[i] = (char *)h->x_pack.ptr + l.off[i];
    } else {
      for (int i = 0; i < 11; ++i) p[i] = src[i];
    }
    a.n = n;
    a.nblk = nblk;
    a.G = G;
    a.F = h->F;
    a.C = C;
    a.S = S;
    a.U = U;
    a.self = (const uint64_t *)p[0];
    a.recv = (const int16_t *)p[1];
    a.flags = (const uint8_t *)p[2];
    a.c_off = (const uint32_t *)p[3];
    a.c_owner = (const uint64_t *)p[4];
    a.c_target = (const uint64_t *)p[5];
    a.s_off = (const uint32_t *)p[6];
    a.spawned = (const uint64_t *)p[7];
    a.u_off = (const uint32_t *)p[8];
    a.u_ref = (const uint64_t *)p[9];
    a.u_info = (const int16_t *)p[10];
    HIP_TRY(launch_route(a, 0, nullptr, h->stream));
  }
  // every shard's validation status, malformed-offset word and per-destination counts
  const uint32_t K = 2 + 4 * G;
  std::vector<uint64_t> H((size_t)G * K);
  h->h_small[0] = (uint64_t)(int64_t)vrc;
  if (int rc = ag_u64(h, {{h->h_small, 1}, {a.err, 1}, {a.totals, 4 * G}}, H.data())) return rc;
  bool bad = false;
  for (uint32_t r = 0; r < G; ++r) bad |= H[(size_t)r * K] != 0 || H[(size_t)r * K + 1] != 0;
  if (bad) {  // all fail together; malformed offsets would have poisoned every shard
    if (vrc) return vrc;
    for (uint32_t r = 0; r < G; ++r)
      if (H[(size_t)r * K + 1]) h->poisoned = true;
    return CRGC_E_INVAL;
  }
  auto tot = [&](uint32_t from, uint32_t to, int q) { return H[(size_t)from * K + 2 + to * 4 + q]; };
  size_t soff[MAX_SHARDS], sb[MAX_SHARDS], roff[MAX_SHARDS], rb[MAX_SHARDS];
  size_t so = 0, ro = 0;
  for (uint32_t r = 0; r < G; ++r) {
    soff[r] = so;
    sb[r] = part_bytes(tot(me, r, 0), tot(me, r, 1), tot(me, r, 2), tot(me, r, 3));
    so += sb[r];
    roff[r] = ro;
    rb[r] = part_bytes(tot(r, me, 0), tot(r, me, 1), tot(r, me, 2), tot(r, me, 3));
    ro += rb[r];
  }
  if (h->x_route_send.ensure(so + 256) != hipSuccess || h->x_pack_recv.ensure(ro + 256) != hipSuccess)
    return CRGC_E_NOMEM;
  if (n) {
    RoutePart *tab = (RoutePart *)h->h_route;
    for (uint32_t d = 0; d < G; ++d)
      tab[d] = part_at((char *)h->x_route_send.ptr + soff[d], tot(me, d, 0), tot(me, d, 1), tot(me, d, 2),
                       tot(me, d, 3));
    HIP_TRY(hipMemcpyAsync(d_parts, tab, sizeof(RoutePart) * G, hipMemcpyHostToDevice, h->stream));
    HIP_TRY(launch_route(a, 1, d_parts, h->stream));
  }
  if (int rc = h->tp->alltoallv(me, h->x_route_send.ptr, soff, sb, h->x_pack_recv.ptr, roff, rb, h->stream)) {
    h->poisoned = true;
    return rc;
  }
  // the received parts, in shard order, as one batch
  uint64_t N = 0, Ct = 0, St = 0, Ut = 0;
  uint32_t sources = 0, last = 0;
  ConcatPart *cat = (ConcatPart *)(h->h_route + 4096);
  for (uint32_t r = 0; r < G; ++r) {
    const uint64_t rn = tot(r, me, 0);
    const Layout l = entry_layout(rn, tot(r, me, 1), tot(r, me, 2), tot(r, me, 3));
    cat[r].base = (const char *)h->x_pack_recv.ptr + roff[r];
    for (int i = 0; i < 11; ++i) cat[r].off[i] = l.off[i];
    cat[r].pn = N;
    cat[r].pC = Ct;
    cat[r].pS = St;
    cat[r].pU = Ut;
    N += rn;
    Ct += tot(r, me, 1);
    St += tot(r, me, 2);
    Ut += tot(r, me, 3);
    if (rn) {
      ++sources;
      last = r;
    }
  }
  if (N == 0) return CRGC_OK;
  crgc_entry_batch v;
  if (sources == 1) {  // one sender: its part is the batch
    v = batch_of(part_at((char *)h->x_pack_recv.ptr + roff[last], N, Ct, St, Ut), N);
  } else {
    if (h->x_cat.ensure(part_bytes(N, Ct, St, Ut) + 256) != hipSuccess) return CRGC_E_NOMEM;
    const RoutePart dst = part_at((char *)h->x_cat.ptr, N, Ct, St, Ut);
    HIP_TRY(hipMemcpyAsync(d_cat, cat, sizeof(ConcatPart) * G, hipMemcpyHostToDevice, h->stream));
    HIP_TRY(launch_concat(d_cat, G, dst, N, Ct, St, Ut, h->stream));
    v = batch_of(dst, N);
  }
  return merge_entries_one(h, &v, Ct, St, Ut);
}

// A large pageable host batch in K chunks of whole entries: chunk j's arrays
// are copied on the copy stream while chunks < j merge on the graph's stream,
// so the hand-off's PCIe time overlaps the merge (C2: 3.4 ms per wakeup
// against 4.9 ms in one piece; batches in buffers registered with
// crgc_host_register are copied whole, host_registered below).  Every chunk is a merge of
// its own (its own epoch): merges commute, and the last-write-wins fields
// follow chunk order, then record order — the batch's order.
// Offsets are rebased on the device (k_rebase).  The caller's buffers are
// free when this returns (the last copy is waited for).
// The device view of a pointer into a crgc_host_register range (nullptr if none).
static const char *registered_view(const crgc_graph *h, const void *p) {
  const char *c = (const char *)p;
  for (const auto &r : h->pinned)
    if (c >= r.first && c < r.first + r.second) return r.dev + (c - r.first);
  return nullptr;
}

constexpr uint64_t CHUNK_MIN = 1u << 18;      // entries per chunk at least (runtime copies)
constexpr uint64_t CHUNK_MIN_REG = 1u << 18;  // (kernel copies of a registered batch)
constexpr uint32_t CHUNK_MAX = 8;

// async (crgc_merge_entries_async, registered batches): return without waiting
// for the copies; the caller keeps the buffers until a trace or sync.
static int merge_entries_chunked(crgc_graph *h, const crgc_entry_batch *b, uint32_t K, bool registered,
                                 bool async = false) {
  const uint64_t n = b->n_entries;
  struct Part {
    uint64_t lo, hi, c0, c1, s0, s1, u0, u1;
    size_t off[11];
  };
  Part p[CHUNK_MAX];
  size_t total = 0;
  // (CRGC_REG_SDMA: a chunk's arrays as one span of the caller's arena, copied
  // by one DMA; its staging region keeps the host addresses' offsets mod 256)
  const bool sdma = registered && h->knobs.reg_sdma;
  const char *span_lo[CHUNK_MAX] = {};
  size_t span_at[CHUNK_MAX] = {}, span_len[CHUNK_MAX] = {};
  for (uint32_t j = 0; j < K; ++j) {
    Part &q = p[j];
    q.lo = (n * j / K) & ~63ull;  // 64-entry boundaries: every per-entry array's chunk is 64-B aligned
    q.hi = j + 1 == K ? n : (n * (j + 1) / K) & ~63ull;
    q.c0 = b->created_off[q.lo], q.c1 = b->created_off[q.hi];
    q.s0 = b->spawned_off[q.lo], q.s1 = b->spawned_off[q.hi];
    q.u0 = b->updated_off[q.lo], q.u1 = b->updated_off[q.hi];
    if (q.c1 < q.c0 || q.s1 < q.s0 || q.u1 < q.u0) return CRGC_E_INVAL;  // offsets run backwards
    const uint64_t m = q.hi - q.lo, C = q.c1 - q.c0, S = q.s1 - q.s0, U = q.u1 - q.u0;
    const size_t sz[11] = {m * 8, m * 2, m, (m + 1) * 4, C * 8, C * 8, (m + 1) * 4, S * 8, (m + 1) * 4, U * 8, U * 2};
    const void *src[11] = {b->self + q.lo, b->recv_count + q.lo, b->flags + q.lo, b->created_off + q.lo,
                           b->created_owner + q.c0, b->created_target + q.c0, b->spawned_off + q.lo,
                           b->spawned + q.s0, b->updated_off + q.lo, b->updated_ref + q.u0,
                           b->updated_info + q.u0};
    if (sdma) {
      const char *lo = nullptr, *hi = nullptr;
      size_t sum = 0;
      for (int i = 0; i < 11; ++i)
        if (sz[i]) {
          const char *c = (const char *)src[i];
          if (!lo || c < lo) lo = c;
          if (!hi || c + sz[i] > hi) hi = c + sz[i];
          sum += sz[i];
        }
      if (lo && (size_t)(hi - lo) <= 2 * sum + (1u << 20)) {  // a packed arena: one span
        total = (total + 255) & ~(size_t)255;
        span_lo[j] = lo;
        span_at[j] = total + ((uintptr_t)lo & 255);
        span_len[j] = (size_t)(hi - lo);
        for (int i = 0; i < 11; ++i)
          q.off[i] = sz[i] ? span_at[j] + (size_t)((const char *)src[i] - lo) : span_at[j];
        total = span_at[j] + span_len[j];
        continue;
      }
    }
    for (int i = 0; i < 11; ++i) {
      total = (total + 255) & ~(size_t)255;
      // a kernel copy wants the source's alignment mod 16 (the body in 16-B groups)
      if (registered) total += (uintptr_t)src[i] & 15;
      q.off[i] = total;
      total += sz[i];
    }
  }
  // This call's staging area (two in turn): free once the merges of the call
  // that last used it are done (ev_cfree, recorded behind them on the graph's
  // stream), so its copy can run beside the previous call's merge.  (A larger
  // area frees the old one: let the work queued on it finish first — an async
  // merge's copies and merges may still read it.)
  const int sk = h->cstage_k;
  h->cstage_k ^= 1;
  Scratch &stg = h->cstage[sk];
  if (total + 256 > stg.bytes) HIP_TRY(hsync(h));
  if (stg.ensure(total + 256) != hipSuccess) return CRGC_E_NOMEM;
  char *base = (char *)stg.ptr;
  if (h->cfree_rec[sk]) HIP_TRY(hipStreamWaitEvent(h->cpy, h->ev_cfree[sk], 0));
  auto copy_chunk = [&](uint32_t j) -> hipError_t {
    const Part &q = p[j];
    const uint64_t m = q.hi - q.lo;
    const void *src[11] = {b->self + q.lo, b->recv_count + q.lo, b->flags + q.lo, b->created_off + q.lo,
                           b->created_owner + q.c0, b->created_target + q.c0, b->spawned_off + q.lo,
                           b->spawned + q.s0, b->updated_off + q.lo, b->updated_ref + q.u0,
                           b->updated_info + q.u0};
    const size_t sz[11] = {m * 8, m * 2, m, (m + 1) * 4, (q.c1 - q.c0) * 8, (q.c1 - q.c0) * 8, (m + 1) * 4,
                           (q.s1 - q.s0) * 8, (m + 1) * 4, (q.u1 - q.u0) * 8, (q.u1 - q.u0) * 2};
    if (span_lo[j]) {  // CRGC_REG_SDMA: the chunk's span in one DMA from the registered arena
      hipError_t e = hipMemcpyAsync(base + span_at[j], span_lo[j], span_len[j], hipMemcpyHostToDevice, h->cpy);
      if (e != hipSuccess) return e;
    } else if (registered && !sdma) {  // read over PCIe by a kernel (k_copy_ranges): no per-copy runtime overhead
      HostCopy hc{};
      for (int i = 0; i < 11; ++i)
        if (sz[i]) {
          hc.src[hc.n] = registered_view(h, src[i]);
          hc.dst[hc.n] = base + q.off[i];
          hc.bytes[hc.n] = sz[i];
          ++hc.n;
        }
      if (hipError_t e = launch_copy_ranges(hc, h->cpy)) return e;
    } else {
      for (int i = 0; i < 11; ++i)
        if (sz[i]) {
          hipError_t e = hipMemcpyAsync(base + q.off[i], src[i], sz[i], hipMemcpyHostToDevice, h->cpy);
          if (e != hipSuccess) return e;
        }
    }
    return hipEventRecord(h->ev_chunk[j], h->cpy);
  };
  int rc = CRGC_OK;
  uint32_t copied = 0;
  for (uint32_t j = 0; j < K && rc == CRGC_OK; ++j) {
    // keep one chunk's copy ahead of the merges
    while (copied < K && copied <= j + 1) {
      if (hipError_t e = copy_chunk(copied)) {
        rc = map_hip(e);
        break;
      }
      ++copied;
    }
    if (rc) break;
    const Part &q = p[j];
    const uint64_t m = q.hi - q.lo;
    if (hipError_t e = hipStreamWaitEvent(h->stream, h->ev_chunk[j], 0)) {
      rc = map_hip(e);
      break;
    }
    uint32_t *co = (uint32_t *)(base + q.off[3]), *so = (uint32_t *)(base + q.off[6]),
             *uo = (uint32_t *)(base + q.off[8]);
    if (hipError_t e = launch_rebase(co, so, uo, m + 1, (uint32_t)q.c0, (uint32_t)q.s0, (uint32_t)q.u0,
                                     h->stream)) {
      rc = map_hip(e);
      break;
    }
    crgc_entry_batch v{};
    v.n_entries = m;
    v.self = (const uint64_t *)(base + q.off[0]);
    v.recv_count = (const int16_t *)(base + q.off[1]);
    v.flags = (const uint8_t *)(base + q.off[2]);
    v.created_off = co;
    v.created_owner = (const uint64_t *)(base + q.off[4]);
    v.created_target = (const uint64_t *)(base + q.off[5]);
    v.spawned_off = so;
    v.spawned = (const uint64_t *)(base + q.off[7]);
    v.updated_off = uo;
    v.updated_ref = (const uint64_t *)(base + q.off[9]);
    v.updated_info = (const int16_t *)(base + q.off[10]);
    v.memory = CRGC_MEM_DEVICE;
    rc = merge_entries_one(h, &v, q.c1 - q.c0, q.s1 - q.s0, q.u1 - q.u0);
  }
  // the area is free again once these merges are done
  if (hipError_t e = hipEventRecord(h->ev_cfree[sk], h->stream)) {
    if (rc == CRGC_OK) rc = map_hip(e);
  } else {
    h->cfree_rec[sk] = true;
  }
  // the caller's buffers are read only during the call (async: until the
  // next trace or sync, which wait for the graph's stream and so for these
  // copies, its merges' dependencies)
  if (async && registered && rc == CRGC_OK) return CRGC_OK;
  const hipError_t e = stream_wait(h->cpy, h->knobs.spin_us);
  if (rc == CRGC_OK && e != hipSuccess) rc = map_hip(e);
  return rc;
}

// Whether every record array of a host batch lies in buffers registered with
// crgc_host_register.  Such batches are chunked too, but their chunks are read
// over PCIe by a kernel (k_copy_ranges) rather than copied by the runtime: from
// registered memory one large runtime copy per array runs at ~57 GB/s but ~1 MB
// copies at 4.4 GB/s (profiles/r3g/pcie_probe.txt; round 3 therefore copied them
// whole, 0.9 ms in the merge call, with nothing overlapped).
static bool host_registered(const crgc_graph *h, const crgc_entry_batch *b, uint64_t C, uint64_t S,
                            uint64_t U);

static bool host_registered(const crgc_graph *h, const crgc_entry_batch *b, uint64_t C, uint64_t S,
                            uint64_t U) {
  if (h->pinned.empty()) return false;
  const uint64_t n = b->n_entries;
  const std::pair<const void *, uint64_t> arr[11] = {
      {b->self, n * 8},          {b->recv_count, n * 2},     {b->flags, n},
      {b->created_off, (n + 1) * 4}, {b->created_owner, C * 8}, {b->created_target, C * 8},
      {b->spawned_off, (n + 1) * 4}, {b->spawned, S * 8},      {b->updated_off, (n + 1) * 4},
      {b->updated_ref, U * 8},   {b->updated_info, U * 2}};
  for (const auto &a : arr) {
    if (!a.second) continue;
    const char *p = (const char *)a.first;
    bool in = false;
    for (const auto &r : h->pinned)
      if (p >= r.first && p + a.second <= r.first + r.second) in = true;
    if (!in) return false;
  }
  return true;
}

// A large device batch in sub-merges of DEV_CHUNK entries (offsets rebased on
// the device): each sub-merge checks capacity with its own exact record counts,
// so the upper bounds of one 1e7-entry wakeup (C4 on one GPU: n + 2C + S + U =
// 1.7e8 possible new shadows) never force a rebuild the real growth does not
// need.  Chunks merge in order, each its own epoch: the same result.
constexpr uint64_t DEV_CHUNK = 1u << 20;

static int merge_entries_dev_chunked(crgc_graph *h, const crgc_entry_batch *b) {
  const uint64_t n = b->n_entries;
  const uint64_t CH = h->knobs.dev_chunk ? h->knobs.dev_chunk : DEV_CHUNK;
  const uint64_t K = (n + CH - 1) / CH;
  std::vector<uint32_t> bo(3 * (K + 1));
  if (h->x_chunk.ensure(Carver::need({(CH + 1) * 4, (CH + 1) * 4, (CH + 1) * 4, 3 * (K + 1) * 4})) != hipSuccess)
    return CRGC_E_NOMEM;
  Carver cv(h->x_chunk.ptr);
  uint32_t *co = cv.take<uint32_t>(CH + 1), *so = cv.take<uint32_t>(CH + 1), *uo = cv.take<uint32_t>(CH + 1);
  uint32_t *dbo = cv.take<uint32_t>(3 * (K + 1));
  // the boundaries' offsets in one gather and one copy
  HIP_TRY(launch_bounds(b->created_off, b->spawned_off, b->updated_off, n, CH, K, dbo, h->stream));
  // into the pinned staging words when they fit (a copy into pageable memory is
  // staged and waited for inside the runtime, where our polling cannot reach)
  HIP_TRY(d2h_small(h, bo.data(), dbo, bo.size() * 4));
  HIP_TRY(hsync(h));
  d2h_small_done(h, bo.data(), bo.size() * 4);
  if (bo[0] || bo[1] || bo[2]) return CRGC_E_INVAL;
  // Every chunk's boundaries are checked before the first sub-merge, so a batch
  // refused for them is refused whole (a later chunk's bad boundary
  // used to surface after the chunks before it had merged).  Offsets that run
  // backwards inside a chunk are the device's ERR_BAD_OFFSETS, which poisons
  // the handle (device_error), as a single merge does.
  for (uint64_t j = 0; j < K; ++j) {
    const uint64_t lo = j * CH, hi = std::min(n, lo + CH), m = hi - lo;
    const uint32_t c0 = bo[3 * j], s0 = bo[3 * j + 1], u0 = bo[3 * j + 2];
    const uint32_t c1 = bo[3 * j + 3], s1 = bo[3 * j + 4], u1 = bo[3 * j + 5];
    if (c1 < c0 || s1 < s0 || u1 < u0 || c1 - c0 > m * h->F || s1 - s0 > m * h->F || u1 - u0 > m * h->F)
      return CRGC_E_INVAL;  // offsets run backwards or past F per entry: refused, nothing merged
  }
  for (uint64_t j = 0; j < K; ++j) {
    const uint64_t lo = j * CH, hi = std::min(n, lo + CH), m = hi - lo;
    const uint32_t c0 = bo[3 * j], s0 = bo[3 * j + 1], u0 = bo[3 * j + 2];
    const uint32_t c1 = bo[3 * j + 3], s1 = bo[3 * j + 4], u1 = bo[3 * j + 5];
    // (stream order: the previous chunk's kernels have read these buffers)
    HIP_TRY(launch_rebase_copy(b->created_off + lo, b->spawned_off + lo, b->updated_off + lo, co, so, uo, m + 1, c0,
                               s0, u0, h->stream));
    crgc_entry_batch v{};
    v.n_entries = m;
    v.self = b->self + lo;
    v.recv_count = b->recv_count + lo;
    v.flags = b->flags + lo;
    v.created_off = co;
    v.created_owner = b->created_owner + c0;
    v.created_target = b->created_target + c0;
    v.spawned_off = so;
    v.spawned = b->spawned + s0;
    v.updated_off = uo;
    v.updated_ref = b->updated_ref + u0;
    v.updated_info = b->updated_info + u0;
    v.memory = CRGC_MEM_DEVICE;
    if (int rc = merge_entries_one(h, &v, c1 - c0, s1 - s0, u1 - u0)) return rc;
  }
  return CRGC_OK;
}

static int merge_entries(crgc_graph *h, const crgc_entry_batch *b, bool async);

int crgc_merge_entries(crgc_graph *h, const crgc_entry_batch *b) { return merge_entries(h, b, false); }
int crgc_merge_entries_async(crgc_graph *h, const crgc_entry_batch *b) { return merge_entries(h, b, true); }

static int merge_entries(crgc_graph *h, const crgc_entry_batch *b, bool async) {
  if (int rc = check_graph(h)) return rc;
  DeviceGuard dg(h->device);
  uint64_t C = 0, S = 0, U = 0;
  // A routed sharded merge needs no exact record counts of a device batch (the
  // route kernels read the offsets and check them against n*F, as an unsharded
  // merge does): one host round trip less per merge.  The all-gather form
  // sizes its copies by them.
  const bool routed = h->tp && h->route && h->G <= ROUTE_MAX_SHARDS && h->F <= ROUTE_MAX_F;
  const int vrc = entry_counts(h, b, h->tp && !routed, &C, &S, &U);
  if (!h->tp) {
    if (vrc) return vrc;
    if (b->memory == CRGC_MEM_DEVICE && b->n_entries > (h->knobs.dev_chunk ? h->knobs.dev_chunk : DEV_CHUNK) &&
        b->created_owner && b->created_target &&
        b->spawned && b->updated_ref && b->updated_info)
      return merge_entries_dev_chunked(h, b);
    if (b->memory == CRGC_MEM_HOST && h->chunk_host) {
      const bool reg = host_registered(h, b, C, S, U);
      const uint64_t k = reg ? std::min<uint64_t>(h->chunk_reg, b->n_entries / CHUNK_MIN_REG)
                             : std::min<uint64_t>(h->chunk_max, b->n_entries / CHUNK_MIN);
      // A registered batch of >= CHUNK_MIN_REG entries is read over PCIe by
      // k_copy_ranges in one piece and merged once: merge kernels running beside
      // a PCIe-reading copy slow down 5-25x (profiles/r4ab), so overlapping
      // chunks bought nothing (C2 registered wakeup 2.20 ms in one piece, 2.30
      // in 3 chunks, interleaved on one box, profiles/r4ae)
      if (reg && (b->n_entries >= CHUNK_MIN_REG || async))
        return merge_entries_chunked(h, b, (uint32_t)std::max<uint64_t>(k, 1), true, async);
      if (k >= 2) return merge_entries_chunked(h, b, (uint32_t)k, reg);
    }
    return merge_entries_one(h, b, C, S, U);
  }
  if (routed) return merge_entries_routed(h, b, vrc, C, S, U);
  // Sharded: every shard applies its part of every shard's batch, in shard order.
  const uint64_t n = vrc ? 0 : b->n_entries;
  const uint64_t hdr[5] = {(uint64_t)(int64_t)vrc, n, C, S, U};
  const void *arr[11] = {b ? b->self : nullptr,        b ? b->recv_count : nullptr,
                         b ? b->flags : nullptr,       b ? b->created_off : nullptr,
                         b ? b->created_owner : nullptr, b ? b->created_target : nullptr,
                         b ? b->spawned_off : nullptr, b ? b->spawned : nullptr,
                         b ? b->updated_off : nullptr, b ? b->updated_ref : nullptr,
                         b ? b->updated_info : nullptr};
  std::vector<uint64_t> H;
  std::vector<size_t> roff;
  auto lay = [](const uint64_t *x) { return entry_layout(x[1], x[2], x[3], x[4]); };
  if (int rc = gather_batches(h, hdr, 5, arr, n ? 11 : 0, b ? b->memory : CRGC_MEM_HOST, lay, H, roff))
    return rc;
  for (uint32_t r = 0; r < h->G; ++r) {
    const uint64_t *x = &H[(size_t)r * 5];
    if (!x[1]) continue;
    const Layout l = lay(x);
    char *base = (char *)h->x_pack_recv.ptr + roff[r];
    crgc_entry_batch v{};
    v.n_entries = x[1];
    v.self = (const uint64_t *)(base + l.off[0]);
    v.recv_count = (const int16_t *)(base + l.off[1]);
    v.flags = (const uint8_t *)(base + l.off[2]);
    v.created_off = (const uint32_t *)(base + l.off[3]);
    v.created_owner = (const uint64_t *)(base + l.off[4]);
    v.created_target = (const uint64_t *)(base + l.off[5]);
    v.spawned_off = (const uint32_t *)(base + l.off[6]);
    v.spawned = (const uint64_t *)(base + l.off[7]);
    v.updated_off = (const uint32_t *)(base + l.off[8]);
    v.updated_ref = (const uint64_t *)(base + l.off[9]);
    v.updated_info = (const int16_t *)(base + l.off[10]);
    v.memory = CRGC_MEM_DEVICE;
    if (int rc = merge_entries_one(h, &v, x[2], x[3], x[4])) return rc;
  }
  return CRGC_OK;
}

static int delta_counts(crgc_graph *h, const crgc_delta_batch *b, uint64_t *nout) {
  if (!b || b->memory > CRGC_MEM_DEVICE) return CRGC_E_INVAL;
  const uint64_t n = b->n_shadows;
  *nout = 0;
  if (n == 0) return CRGC_OK;
  if (!b->id || !b->recv_count || !b->supervisor || !b->flags || !b->out_off) return CRGC_E_INVAL;
  if (b->memory == CRGC_MEM_HOST) {
    if (b->out_off[0]) return CRGC_E_INVAL;
    *nout = b->out_off[n];
  } else {
    uint32_t v = 0;  // ordered behind whatever produced the batch on this stream
    HIP_TRY(hipMemcpyAsync(&v, b->out_off + n, 4, hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hsync(h));
    *nout = v;
  }
  if (*nout && (!b->out_target || !b->out_count)) return CRGC_E_INVAL;
  return CRGC_OK;
}

static int merge_deltas_one(crgc_graph *h, const crgc_delta_batch *b, uint64_t nout) {
  const uint64_t n = b->n_shadows;
  if (n == 0) return CRGC_OK;
  const uint64_t ids = 2 * n + nout;
  if (int rc = ensure_capacity(h, ids, nout)) return rc;
  const size_t host_bytes =
      b->memory == CRGC_MEM_HOST ? Carver::need({n * 8, n * 4, n * 8, n, (n + 1) * 4, nout * 8, nout * 4})
                                 : 0;
  const bool sh = h->tp;
  const size_t work_bytes =
      Carver::need({n * 4, n * 4, std::max<uint64_t>(nout, 1) * 4, sh ? std::max<uint64_t>(nout, 1) * 8 : 0}) +
      edge_scratch(h, nout);
  if (h->stage.ensure(host_bytes + 256) != hipSuccess || h->work.ensure(work_bytes) != hipSuccess)
    return CRGC_E_NOMEM;
  Carver sc(h->stage.ptr), wc(h->work.ptr);
  Staged staged(h, b->memory);
  DeltaArgs a{};
  a.n = n;
  a.nout = nout;
  a.epoch = ++h->epoch;
  a.id = stage(h, sc, b->id, n, b->memory);
  a.recv = stage(h, sc, b->recv_count, n, b->memory);
  a.sup = stage(h, sc, b->supervisor, n, b->memory);
  a.flags = stage(h, sc, b->flags, n, b->memory);
  a.out_off = stage(h, sc, b->out_off, n + 1, b->memory);
  a.out_target = stage(h, sc, b->out_target, nout, b->memory);
  a.out_count = stage(h, sc, b->out_count, nout, b->memory);
  HIP_TRY(staged.mark());
  a.self_slot = wc.take<uint32_t>(n);
  a.sup_slot = wc.take<uint32_t>(n);
  a.ot_slot = wc.take<uint32_t>(std::max<uint64_t>(nout, 1));
  if (sh) a.o_partner = wc.take<uint64_t>(std::max<uint64_t>(nout, 1));
  a.atom_o = wc.take<uint32_t>(std::max<uint64_t>(nout, 1));
  a.atom_t = wc.take<uint32_t>(std::max<uint64_t>(nout, 1));
  a.atom_d = wc.take<int32_t>(std::max<uint64_t>(nout, 1));
  HIP_TRY(launch_deltas(ids_view(h), a, nout, h->stream, 0));
  {
    SideFork sf(h);
    HIP_TRY(sf.fork());
    if (int rc = run_edges(h, a.atom_o, a.atom_t, a.atom_d, nout, wc, nullptr, sf.stream())) return rc;
    HIP_TRY(launch_deltas(h->g.d, a, nout, h->stream, 1));
    HIP_TRY(sf.join());
  }
  note_merge(h, ids, nout);
  HIP_TRY(staged.wait());
  return CRGC_OK;
}

int crgc_merge_deltas(crgc_graph *h, const crgc_delta_batch *b) {
  if (int rc = check_graph(h)) return rc;
  DeviceGuard dg(h->device);
  uint64_t nout = 0;
  const int vrc = delta_counts(h, b, &nout);
  if (!h->tp) return vrc ? vrc : merge_deltas_one(h, b, nout);
  const uint64_t n = vrc ? 0 : b->n_shadows;
  const uint64_t hdr[3] = {(uint64_t)(int64_t)vrc, n, nout};
  const void *arr[7] = {b ? b->id : nullptr,      b ? b->recv_count : nullptr, b ? b->supervisor : nullptr,
                        b ? b->flags : nullptr,   b ? b->out_off : nullptr,    b ? b->out_target : nullptr,
                        b ? b->out_count : nullptr};
  std::vector<uint64_t> H;
  std::vector<size_t> roff;
  auto lay = [](const uint64_t *x) { return delta_layout(x[1], x[2]); };
  if (int rc = gather_batches(h, hdr, 3, arr, n ? 7 : 0, b ? b->memory : CRGC_MEM_HOST, lay, H, roff))
    return rc;
  for (uint32_t r = 0; r < h->G; ++r) {
    const uint64_t *x = &H[(size_t)r * 3];
    if (!x[1]) continue;
    const Layout l = lay(x);
    char *base = (char *)h->x_pack_recv.ptr + roff[r];
    crgc_delta_batch v{};
    v.n_shadows = x[1];
    v.id = (const uint64_t *)(base + l.off[0]);
    v.recv_count = (const int32_t *)(base + l.off[1]);
    v.supervisor = (const uint64_t *)(base + l.off[2]);
    v.flags = (const uint8_t *)(base + l.off[3]);
    v.out_off = (const uint32_t *)(base + l.off[4]);
    v.out_target = (const uint64_t *)(base + l.off[5]);
    v.out_count = (const int32_t *)(base + l.off[6]);
    v.memory = CRGC_MEM_DEVICE;
    if (int rc = merge_deltas_one(h, &v, x[2])) return rc;
  }
  return CRGC_OK;
}

// mergeUndoLog.  Sharded graphs: collective, every shard passes the same log.
int crgc_merge_undo(crgc_graph *h, const crgc_undo_log *log) {
  if (int rc = check_graph(h)) return rc;
  DeviceGuard dg(h->device);
  int vrc = CRGC_OK;
  uint64_t n = 0, nc = 0;
  if (!log || log->memory != CRGC_MEM_HOST) {
    vrc = CRGC_E_INVAL;
  } else {
    n = log->n_fields;
    if (n && (!log->actor || !log->message_count || !log->created_off)) vrc = CRGC_E_INVAL;
    else if (n && log->created_off[0]) vrc = CRGC_E_INVAL;
    else {
      nc = n ? log->created_off[n] : 0;
      if (nc && (!log->created_target || !log->created_count)) vrc = CRGC_E_INVAL;
      // UndoLog.admitted is a map: one field per actor.
      std::vector<uint64_t> ids(log->actor, log->actor + n);
      std::sort(ids.begin(), ids.end());
      if (std::adjacent_find(ids.begin(), ids.end()) != ids.end()) vrc = CRGC_E_INVAL;
    }
  }
  if (h->tp) {  // agree on validity before any collective work
    const uint64_t st = (uint64_t)(int64_t)vrc;
    std::vector<uint64_t> all(h->G);
    if (int rc = ag_host(h, &st, 1, all.data())) return rc;
    for (uint64_t v : all)
      if (v) return vrc ? vrc : CRGC_E_INVAL;
  } else if (vrc) {
    return vrc;
  }
  if (int rc = ensure_capacity(h, nc, nc)) return rc;
  std::vector<uint64_t> c_actor(nc);
  for (uint64_t i = 0; i < n; ++i)
    for (uint32_t k = log->created_off[i]; k < log->created_off[i + 1]; ++k) c_actor[k] = log->actor[i];
  const size_t host_bytes = Carver::need({n * 8, n * 4, (n + 1) * 4, nc * 8, nc * 4, nc * 8});
  const size_t work_bytes = edge_scratch(h, nc) + Carver::need({n + nc + 8});
  if (h->stage.ensure(host_bytes + 256) != hipSuccess || h->work.ensure(work_bytes) != hipSuccess)
    return CRGC_E_NOMEM;
  Carver sc(h->stage.ptr), wc(h->work.ptr);
  UndoArgs a{};
  a.n = n;
  a.nc = nc;
  a.location = log->node_location;
  a.actor = stage(h, sc, log->actor, n, CRGC_MEM_HOST);
  a.msg = stage(h, sc, log->message_count, n, CRGC_MEM_HOST);
  a.c_off = stage(h, sc, log->created_off, n + 1, CRGC_MEM_HOST);
  a.c_target = stage(h, sc, log->created_target, nc, CRGC_MEM_HOST);
  a.c_count = stage(h, sc, log->created_count, nc, CRGC_MEM_HOST);
  a.c_actor = stage(h, sc, c_actor.data(), nc, CRGC_MEM_HOST);
  a.exists = wc.take<uint8_t>(n + nc + 8);
  a.atom_o = wc.take<uint32_t>(std::max<uint64_t>(nc, 1));
  a.atom_t = wc.take<uint32_t>(std::max<uint64_t>(nc, 1));
  a.atom_d = wc.take<int32_t>(std::max<uint64_t>(nc, 1));
  // The reference's ConcurrentModificationException, detected
  // before any mutation: an admitted actor in the graph names a target that is not.
  std::vector<uint8_t> ex(n + nc, 0);
  if (n + nc) {
    HIP_TRY(launch_undo_check(h->g.d, a, h->stream));
    if (h->tp) {
      const size_t words = (n + nc + 7) / 8;
      std::vector<uint64_t> all(words * h->G);
      if (h->x_ans.ensure(words * 8) != hipSuccess) return CRGC_E_NOMEM;
      HIP_TRY(hipMemsetAsync(h->x_ans.ptr, 0, words * 8, h->stream));
      HIP_TRY(hipMemcpyAsync(h->x_ans.ptr, a.exists, n + nc, hipMemcpyDeviceToDevice, h->stream));
      if (words > MAX_SHARDS + 8) {  // beyond the small-gather staging: a direct exchange
        if (h->x_ans_back.ensure(words * 8 * h->G) != hipSuccess) return CRGC_E_NOMEM;
        if (int rc = h->tp->allgather(h->shard, h->x_ans.ptr, h->x_ans_back.ptr, words * 8, h->stream)) {
          h->poisoned = true;
          return rc;
        }
        HIP_TRY(hipMemcpy(all.data(), h->x_ans_back.ptr, words * 8 * h->G, hipMemcpyDeviceToHost));
      } else if (int rc = ag_u64(h, {{h->x_ans.ptr, (uint32_t)words}}, all.data())) {
        return rc;
      }
      for (uint32_t r = 0; r < h->G; ++r) {
        const uint8_t *p = (const uint8_t *)&all[(size_t)r * words];
        for (uint64_t i = 0; i < n + nc; ++i) ex[i] |= p[i];
      }
    } else {
      HIP_TRY(hipMemcpyAsync(ex.data(), a.exists, n + nc, hipMemcpyDeviceToHost, h->stream));
      HIP_TRY(hsync(h));
    }
  }
  for (uint64_t i = 0; i < n; ++i) {
    if (!ex[i]) continue;  // field ignored (:166-167)
    for (uint32_t k = log->created_off[i]; k < log->created_off[i + 1]; ++k)
      if (!ex[n + k]) return CRGC_E_UNDO_NEW_SHADOW;
  }
  HIP_TRY(sync_counters(h));
  if (int rc = device_error(h)) return rc;
  h->halted_seen = true;  // (k_undo_halt: the downed location's shadows)
  HIP_TRY(launch_undo_apply(h->g.d, a, h->slot_top, h->stream));
  if (int rc = run_edges(h, a.atom_o, a.atom_t, a.atom_d, nc, wc)) return rc;
  note_merge(h, nc, nc);
  return CRGC_OK;
}

// ---- mark ---------------------------------------------------------------------
// Chain mode (crgc_chain.hip): close the marked set by pointer jumping along
// each shadow's unique out-target and its supervisor, expanding shadows with
// several out-targets edge by edge, until an iteration marks nothing.  One
// host synchronisation per iteration; each doubling sequence is enqueued in
// full (ceil(log2 slots) + 1 rounds) and its rounds exit at once after a
// round that marked nothing.
static int run_chains(crgc_graph *h, bool investigate, uint64_t top) {
  const uint64_t words = (top + 31) / 32 + 2;
  uint32_t R = 1;
  while ((1ull << (R - 1)) < top) ++R;
  const size_t need = Carver::need({top * 4, top * 4, top * 4, top * 4, words * 4, (2 * (size_t)R + 8) * 4, 8});
  if (h->x_chain.ensure(need) != hipSuccess) return CRGC_E_NOMEM;
  Carver cv(h->x_chain.ptr);
  ChainArgs ca{};
  ca.nx0 = cv.take<uint32_t>(top);
  ca.sp0 = cv.take<uint32_t>(top);
  uint32_t *ja = cv.take<uint32_t>(top), *jb = cv.take<uint32_t>(top);
  ca.cx = cv.take<uint32_t>(words);
  ca.flag = cv.take<uint32_t>(2 * R + 8);
  ca.n_new = cv.take<unsigned long long>(1);
  ca.investigate = investigate ? 1 : 0;
  const DevGraph &g = h->g.d;
  HIP_TRY(hipMemsetAsync(ca.n_new, 0, 8, h->stream));
  HIP_TRY(launch_chain(g, ca, 0, nullptr, nullptr, top, 0, 0, 0, h->stream));
  std::vector<uint32_t> fl(2 * R + 1);
  uint32_t marked_rounds = 0;
  int pcur = 0;
  for (uint64_t it = 0;; ++it) {
    if (it > top) return CRGC_E_TIMEOUT;  // every iteration but the last marks a shadow
    ca.pb_in = g.pb[pcur];
    ca.pb_out = g.pb[pcur ^ 1];
    HIP_TRY(hipMemsetAsync(ca.flag, 0, (2 * R + 1) * 4, h->stream));
    for (uint32_t seq = 0; seq < 2; ++seq) {
      const uint32_t *src = seq ? ca.sp0 : ca.nx0;
      uint32_t *dst = ja;
      for (uint32_t r = 0; r < R; ++r) {
        HIP_TRY(launch_chain(g, ca, 1, src, dst, top, seq * R + r, r == 0, 0, h->stream));
        src = dst;
        dst = dst == ja ? jb : ja;
      }
    }
    HIP_TRY(launch_chain(g, ca, 2, nullptr, nullptr, top, 2 * R, 0, 0, h->stream));
    HIP_TRY(d2h_small(h, fl.data(), ca.flag, fl.size() * 4));
    HIP_TRY(hsync(h));
    d2h_small_done(h, fl.data(), fl.size() * 4);
    bool any = false;
    for (uint32_t f : fl)
      if (f) {
        any = true;
        ++marked_rounds;
      }
    if (!any) break;
    pcur ^= 1;
  }
  HIP_TRY(launch_chain(g, ca, 3, nullptr, nullptr, top, 0, 0, 0, h->stream));
  HIP_TRY(launch_chain(g, ca, 4, nullptr, nullptr, top, 0, 0, marked_rounds, h->stream));
  return CRGC_OK;
}

struct LevelRun {
  uint64_t levels = 0, roots = 0, launches = 0, depth = 0;
  uint64_t timed = 0;  // level launches whose expand carried timing events (crgc_trace_stats.expand_launches)
  uint64_t first_chunk = 0;  // level launches after level 0 that this trace needed
  double ms = 0, ms_f = 0, ms_t = 0, ms_e = 0;
  uint64_t time_fail = 0;              // event pairs the runtime could not time
  bool defer = false;                  // leave the event queries to the caller (pending)
  std::function<void()> pending;
};

static void collect_times(crgc_graph *h, LevelRun &lr, size_t nl, size_t nc, int timing, bool log,
                          size_t first_level, size_t last, const std::vector<unsigned long long> &ring);

// Level-synchronous BFS from the pseudo-roots (roots = true, start = 0) or
// from candidates of level `start` (sharded rounds), until a level is empty.
// Every level is bracketed by events between its three kernels, so the
// timings are device time of each level kernel.  Levels are enqueued in
// chunks; the first chunk of a trace is as long as the previous trace needed
// (through the level at which k_tail finished the mark, or one level past the
// first empty one), so a steady-state wakeup needs one host synchronisation
// and launches no idle levels.  *end = the first empty
// level (levels start .. *end-1 were non-empty).
// max_levels > 0 (sharded rounds): at most that many level launches after
// level 0; a round that reaches it with work left returns *capped = true and
// *end = the next level, whose candidates are pending.
static int run_levels(crgc_graph *h, bool investigate, uint16_t location, uint64_t top, bool roots,
                      int start, LevelRun &lr, int *end,
                      const std::function<hipError_t()> &after_chunk = nullptr, int max_levels = 0,
                      bool *capped = nullptr, int first_chunk = 4) {
  if (capped) *capped = false;
  LevelArgs la{};
  la.location = location;
  // Losing A/B variants of round 1 (atomicOr candidate bitmap, 8 edges per lane,
  // sequential pull walk, plain candidate stores, default-policy edge stream,
  // always-on marked-word filter) were removed; their records stay in
  // profiles/r1h, r1n, r1r.
  const Knobs &kn = h->knobs;
  // sharded graphs: the level kernels visit the proxy region too (grids from
  // vtop), and level 0's bins cover it (imax: one past the largest slot)
  const uint64_t ptop = proxy_top_ub(h);
  const uint64_t vtop = top + ptop;
  const uint64_t imax = ptop ? h->g.caps.pbase + ptop : top;
  la.flags = 0;
  la.sparse_thresh = (uint32_t)std::max<uint64_t>(64, (top / BLK_SLOTS) / 4);
  // Direction optimisation: dense levels after a frontier of >= top/div shadows pull.
  if (kn.pull) la.flags |= LV_PULL;
  la.pull_div = (uint32_t)kn.pull_div;  // against the exact slot count, on the device
  la.pull_cur_div = kn.pull_cur_div;
  // Beamer's direction rule (CRGC_ALPHA=a: pull when a * m_f > m_u, level 0
  // included; m_u from the edge keys the graph holds, an upper bound).  Off by
  // default: on the C2 wakeup (10 % pseudo-roots) alpha = 14 pulls at level 0
  // and the mark takes 1.27 ms against 0.89 ms with the frontier-size rule
  // (k_expand level 0: 670 us pull vs 306 us push; profiles/r2b/ab.json) — a
  // pull over a 7.6 % frontier walks long in-candidate lists before a hit.
  la.alpha = kn.alpha;
  la.e_total = h->etab_used + h->atoms_since;
  la.pull_thresh = 0;
  // unsharded pseudo-root traces: the previous trace's pull levels pull again
  la.pull_pred = (kn.pull_pred && roots && !investigate && !h->tp) ? h->pull_pred : 0;
  // Test hooks: absolute thresholds (0 disables sparse levels entirely).
  if (kn.has_pull_thresh) {
    la.pull_thresh = kn.pull_thresh;
    la.pull_div = 0;
  }
  if (kn.has_sparse) la.sparse_thresh = kn.sparse_thresh;
  // Narrow frontiers: one workgroup finishes the mark (k_tail), or in a
  // sharded graph WALK_WG of them (k_walk, to larger frontiers).
  if (kn.tail) la.flags |= LV_TAIL;
  const bool walk = (h->tp || kn.walk_unsharded) && kn.tail && kn.walk && h->walk_ok;
  if (walk) la.flags |= LV_WALK;
  if (kn.cbits) la.flags |= LV_CBITS;
  if (kn.roots_co) la.flags |= LV_ROOTS_CO;
  if (kn.supbin) la.flags |= LV_SUPBIN;
  // Deep marks: a k_tail walk of chain_after links hands the rest to chain mode
  // (pointer jumping, crgc_chain.hip).  Unsharded graphs only.
  la.chain_after = h->tp ? 0 : kn.chain_after;
  la.xslices = kn.xslices;
  la.tail_start = std::min<uint32_t>(walk ? kn.walk_start : h->tp ? kn.tail_start_sharded : kn.tail_start, TAIL_QCAP);
  la.tail_edge_max = walk ? 0u : h->tp ? kn.tail_edges_sharded : kn.tail_edges;
  la.tail_max = std::min<uint32_t>(std::max(walk ? kn.walk_max : h->tp ? kn.tail_max_sharded : kn.tail_max, 1u),
                                   TAIL_QCAP);
  // The pseudo-root level's binned push (crgc_trace.hip k_bin_place / k_bin_apply):
  // up to 256 bins of >= 65536 slots (an LDS bitmap of <= 128 KiB each), BIN_WG
  // place workgroups with a fixed-capacity slice of every bin each; the slices
  // together hold half the graph's edge keys (targets past a slice are stored
  // at once).  The place pass writes the mode word k_bin_apply reads.
  if (roots && kn.bin && !kn.alpha && top > 0 && top >= kn.bin_min) {
    uint32_t lg = 0;
    while (lg < 63 && (1ull << lg) < imax) ++lg;
    // Bins of 2^16 slots (u16 offsets: the place pass writes 2 B per target)
    // up to 512 of them (2^25 slots: the C2 bench graph's range passes 2^24),
    // else up to 256 wider bins of u32 slots.
    const bool b16 = kn.bin512 && ((imax + 0xFFFFull) >> 16) <= BIN_MAX;
    const uint32_t shift = b16 ? 16u : std::max<uint32_t>(16, lg > 8 ? lg - 8 : 0);
    const uint64_t nb = (imax + (1ull << shift) - 1) >> shift;
    if (shift <= 20 && nb <= (b16 ? BIN_MAX : BIN_MAX_WIDE)) {
      const uint64_t nc = nb * BIN_WG;
      const uint64_t want = std::max<uint64_t>(1u << 16, (h->etab_used + h->atoms_since) / 2);
      // (a multiple of 8: the apply pass reads a slice of u16 offsets in 16-B groups)
      // (below 2^23: the place pass packs a clamped reservation into 23 bits)
      const uint64_t sc = std::min<uint64_t>(std::max<uint64_t>(round_up(want / nc, 8), 16), (1u << 23) - 8);
      const size_t need = Carver::need({16, nc * 4, nc * sc * 4});
      HIP_TRY(h->x_bin.ensure(need));
      Carver cv(h->x_bin.ptr);
      la.bin_mode_w = cv.take<uint32_t>(4);
      la.bin_cnt = cv.take<uint32_t>(nc);
      la.bins = cv.take<uint32_t>(nc * sc);
      la.bin_slice = (uint32_t)sc;
      la.bin_shift = shift;
      la.nbins = (uint32_t)nb;
      la.bin_grid = BIN_WG;
    }
  }
  // Device times, from timing-only events (no system-scope fence):
  //   every chunk of levels: an event pair around it (ms_mark, dispatch gaps included);
  //   CRGC_KERNEL_TIMING=1 (default): k_expand's start / stop carried by its dispatch;
  //   CRGC_KERNEL_TIMING=2: all three level kernels (each timed dispatch costs a few us);
  //   CRGC_KERNEL_TIMING=0: chunks only.
  const int timing = h->timed ? kn.kernel_timing : 0;
  auto new_event = [&](std::vector<hipEvent_t> &v, size_t n) -> hipError_t {
    while (v.size() < n) {
      hipEvent_t e;
      hipError_t r = hipEventCreateWithFlags(&e, hipEventDisableSystemFence);
      if (r != hipSuccess) return r;
      v.push_back(e);
    }
    return hipSuccess;
  };
  size_t nl = 0, nc = 0;
  h->lvl_timed.clear();
  auto launch = [&](int level, bool rootk) -> hipError_t {
    hipEvent_t ev[6] = {};
    // (mode 3: levels 0 and 1 of a trace from the pseudo-roots; a sharded
    // round's levels after its first are narrow)
    const bool timed = timing == 1 || timing == 2 || (timing == 3 && level <= 1);
    h->lvl_timed.push_back(timed ? 1 : 0);
    if (timed) {
      if (hipError_t r = new_event(h->lvl_ev, 6 * (nl + 1))) return r;
      for (int k = timing == 2 ? 0 : 4; k < 6; ++k) ev[k] = h->lvl_ev[6 * nl + k];
    }
    la.level = level;
    if (!timed) la.flags |= LV_NOBYTES;
    else la.flags &= ~LV_NOBYTES;
    hipError_t r = launch_level(h->g.d, la, rootk, investigate, vtop, h->stream, ev);
    if (timed) ++lr.timed;
    ++nl;
    return r;
  };
  auto chunk_event = [&]() -> hipError_t {
    if (!h->timed) return hipSuccess;
    if (hipError_t r = new_event(h->chunk_ev, nc + 1)) return r;
    return hipEventRecord(h->chunk_ev[nc++], h->stream);
  };
  HIP_TRY(chunk_event());
  int L = start;
  if (roots) {
    HIP_TRY(launch(0, true));
    L = 1;
  }
  int chunk = roots && h->last_levels ? (int)std::min<uint64_t>(h->last_levels, 512) : std::max(first_chunk, 1);
  std::vector<unsigned long long> ring(LEVEL_RING);
  unsigned long long tail[3] = {0, 0, 0};
  const bool log = kn.level_log;
  // Bounds on the host loop: every pass either reaches an
  // empty level, finishes in k_tail / chain mode, or moves L forward (a bail
  // must resume past the level it bailed from before); levels are bounded by
  // the (level + 1) << 12 tag width, passes by a count and a wall clock.
  const auto loop_t0 = std::chrono::steady_clock::now();
  int last_bail = -1;
  int launched = 0;  // level launches of this call after level 0
  for (uint64_t pass = 0;; ++pass) {
    if (pass > 4096 || std::chrono::steady_clock::now() - loop_t0 > std::chrono::seconds(kn.level_timeout_s)) {
      h->poisoned = true;
      return CRGC_E_TIMEOUT;
    }
    if (max_levels) chunk = std::max(1, std::min(chunk, max_levels - launched));
    if (nc % 2 == 0) HIP_TRY(chunk_event());
    for (int k = 0; k < chunk; ++k) HIP_TRY(launch(L + k, false));
    HIP_TRY(chunk_event());
    // work that runs only if this chunk finished the mark (its kernels check mark_done)
    if (after_chunk) HIP_TRY(after_chunk());
    // counts of levels L-1 .. L+chunk-1
    const int first = L - 1, last = L + chunk - 1;
    const uint32_t nring = (uint32_t)std::min(last - first + 1, LEVEL_RING);
    HIP_TRY(launch_publish(h->ctr, h->hctr_dev, (uint32_t)first, nring, h->stream));
    HIP_TRY(hsync(h));
    for (uint32_t i = 0; i < nring; ++i) {
      const int k = (first + (int)i) % LEVEL_RING;
      ring[k] = h->hctr->ring[k];
    }
    tail[0] = h->hctr->tail_state;
    tail[1] = h->hctr->tail_level;
    tail[2] = h->hctr->tail_from;
    if (roots && first == 0) lr.roots = ring[0];
    if (tail[0] == TAIL_CHAINS) {  // k_tail handed a deep mark to chain mode, which finishes it
      HIP_TRY(chunk_event());  // chain mode's device time counts as mark time
      if (int rc = run_chains(h, investigate, top)) return rc;
      HIP_TRY(chunk_event());
      if (after_chunk) HIP_TRY(after_chunk());
      HIP_TRY(launch_publish(h->ctr, h->hctr_dev, 0, 0, h->stream));
      HIP_TRY(hsync(h));
      tail[0] = h->hctr->tail_state;
      tail[1] = h->hctr->tail_level;
      tail[2] = h->hctr->tail_from;
    }
    if (tail[0] == TAIL_BAILED) {  // k_tail handed a wide frontier back: resume there
      if ((int)tail[1] <= last_bail || (uint64_t)tail[1] > (1ull << 19)) {
        h->poisoned = true;  // no progress since the last bail
        return CRGC_E_TIMEOUT;
      }
      last_bail = (int)tail[1];
      HIP_TRY(hipMemsetAsync((char *)h->ctr + CTR_OFF(tail_state), 0, 8, h->stream));
      L = (int)tail[1];
      continue;
    }
    for (int lv = first; lv <= last; ++lv) {
      if (tail[0] == TAIL_DONE || ring[lv % LEVEL_RING] == 0) {
        const int e = tail[0] == TAIL_DONE ? (int)tail[1] : lv;
        *end = e;
        lr.levels += (uint64_t)std::max(0, e - (roots ? 0 : start));
        // level launches that did work: the first chunk of the next trace
        if (roots) {
          lr.depth = tail[0] == TAIL_DONE ? (uint64_t)tail[2] + 1 : (uint64_t)lv;
          lr.first_chunk = tail[0] == TAIL_DONE ? std::max<uint64_t>(1, tail[2]) : (uint64_t)lv + 1;
        }
        lr.launches += nl;
        lr.pending = [h, nl, nc, timing, log, roots, start, last, ring, &lr]() {
          collect_times(h, lr, nl, nc, timing, log, roots ? 0 : (size_t)start, (size_t)last, ring);
        };
        if (!lr.defer) {
          lr.pending();
          lr.pending = nullptr;
        }
        return CRGC_OK;
      }
    }
    L += chunk;
    launched += chunk;
    if (max_levels && launched >= max_levels) {  // the round's exchange comes first; level L is pending
      *end = L;
      if (capped) *capped = true;
      lr.levels += (uint64_t)launched;
      lr.launches += nl;
      lr.pending = [h, nl, nc, timing, log, roots, start, last, ring, &lr]() {
        collect_times(h, lr, nl, nc, timing, log, roots ? 0 : (size_t)start, (size_t)last, ring);
      };
      if (!lr.defer) {
        lr.pending();
        lr.pending = nullptr;
      }
      return CRGC_OK;
    }
    chunk = std::min(chunk * 2, 512);
    if ((uint64_t)L > (1ull << 19)) return CRGC_E_TIMEOUT;  // (level + 1) << 12 tags are 32-bit
  }
}

// Event-pair time in ms.  A pair the runtime cannot time counts as 0 ms and is
// counted in *fails (crgc_trace_stats.time_query_failures: the ms_* fields are
// then short, and bench.py refuses to print a roofline from them); the failed
// query's status is read here so that no later call reports it.
static float elapsed_ms(hipEvent_t a, hipEvent_t b, uint64_t *fails) {
  float t = 0;
  if (hipEventElapsedTime(&t, a, b) != hipSuccess) {
    (void)hipGetLastError();
    ++*fails;
    return 0.f;
  }
  return t;
}

// Device times of one run_levels call, from its events (host-side queries,
// deferred by crgc_trace until the result copies are in flight).
static void collect_times(crgc_graph *h, LevelRun &lr, size_t nl, size_t nc, int timing, bool log,
                          size_t first_level, size_t last, const std::vector<unsigned long long> &ring) {
  for (size_t i = 0; i + 1 < nc; i += 2) {
    lr.ms += elapsed_ms(h->chunk_ev[i], h->chunk_ev[i + 1], &lr.time_fail);
  }
  for (size_t i = 0; i < (timing ? nl : 0); ++i) {
    float t[3] = {0, 0, 0};
    if (i >= h->lvl_timed.size() || !h->lvl_timed[i]) continue;
    for (int k = timing == 2 ? 0 : 2; k < 3; ++k)
      t[k] = elapsed_ms(h->lvl_ev[6 * i + 2 * k], h->lvl_ev[6 * i + 2 * k + 1], &lr.time_fail);
    lr.ms_f += t[0];
    lr.ms_t += t[1];
    lr.ms_e += t[2];
    char who[24] = "";
    if (log && h->G > 1) snprintf(who, sizeof who, " s%u", h->shard);
    if (log)
      fprintf(stderr, "[crgc%s] level %zu frontier %llu  %.1f us (frontier %.1f tail %.1f expand %.1f)\n",
              who, first_level + i, first_level + i <= last ? ring[(first_level + i) % LEVEL_RING] : 0ull,
              (t[0] + t[1] + t[2]) * 1e3, t[0] * 1e3, t[1] * 1e3, t[2] * 1e3);
  }
}

static void reset_trace_counters(crgc_graph *h) {
  // marked .. the level ring, and the per-block state of the blocks this trace can touch
  const size_t a = CTR_OFF(marked), b = sizeof(Counters);
  launch_trace_reset(h->g.d, blocks_of(home_top_ub(h)), blocks_of(proxy_top_ub(h)), (uint32_t)(a / 8),
                     (uint32_t)((b - a) / 8), h->stream);
}

// Mark to the global fixpoint: local levels, then (sharded graphs) rounds of
// exporting newly marked proxies to their home shards and continuing from
// what arrives, until no shard has anything to send.
// Home-slot resolution before a sharded mark: every shard learns the others'
// slot generations and counts; proxies of a home whose generation changed
// forget their cached slots; proxies without one ask their home (one id
// exchange, one answer exchange — in steady state only the proxies created
// since the last trace).
static int resolve_home_slots(crgc_graph *h, uint64_t top, int xmode, uint64_t *bytes) {
  const uint32_t G = h->G, me = h->shard;
  const uint64_t mine[2] = {h->slot_gen, top};
  std::vector<uint64_t> T((size_t)G * 2);
  if (int rc = ag_host(h, mine, 2, T.data())) return rc;
  if (h->peer_gen.size() != G) {
    h->peer_gen.assign(G, ~0ull);
    h->peer_top.assign(G, 0);
  }
  uint64_t mask = 0;  // one bit per home: MAX_SHARDS = 64
  for (uint32_t d = 0; d < G; ++d) {
    if (h->peer_gen[d] != T[2 * d]) mask |= 1ull << d;
    h->peer_gen[d] = T[2 * d];
    h->peer_top[d] = T[2 * d + 1];
  }
  if (xmode == 0) return CRGC_OK;  // ids only: nothing to resolve
  const uint64_t ptop = proxy_top_ub(h);  // (grids over the proxy region)
  if (mask) HIP_TRY(launch_resolve(h->g.d, 0, mask, nullptr, nullptr, nullptr, 0, nullptr, ptop, h->stream));
  HIP_TRY(launch_zero_u64((char *)h->ctr + CTR_OFF(xcnt), 2 * MAX_SHARDS, h->stream));
  HIP_TRY(launch_resolve(h->g.d, 1, 0, nullptr, nullptr, nullptr, 0, nullptr, ptop, h->stream));
  std::vector<uint64_t> M((size_t)G * G);
  if (int rc = ag_u64(h, {{(char *)h->ctr + CTR_OFF(xcnt), G}}, M.data())) return rc;
  uint64_t total = 0, nsend = 0;
  for (uint64_t v : M) total += v;
  for (uint32_t d = 0; d < G; ++d) nsend += M[(size_t)me * G + d];
  if (total == 0) {
    HIP_TRY(launch_resolve(h->g.d, 5, 0, nullptr, nullptr, nullptr, 0, nullptr, 0, h->stream));
    return CRGC_OK;
  }
  if (h->x_send.ensure(nsend * 8 + 8) != hipSuccess || h->x_slot.ensure(nsend * 4 + 8) != hipSuccess)
    return CRGC_E_NOMEM;
  HIP_TRY(launch_resolve(h->g.d, 2, 0, (uint64_t *)h->x_send.ptr, (uint32_t *)h->x_slot.ptr, nullptr, 0,
                         nullptr, ptop, h->stream));
  HIP_TRY(launch_resolve(h->g.d, 5, 0, nullptr, nullptr, nullptr, 0, nullptr, 0, h->stream));
  uint64_t nin = 0, nback = 0;
  if (int rc = a2a(h, h->x_send.ptr, M.data(), 8, h->x_recv, false, &nin)) return rc;
  if (h->x_ans.ensure(nin * 4 + 8) != hipSuccess) return CRGC_E_NOMEM;
  HIP_TRY(launch_resolve(h->g.d, 3, 0, nullptr, nullptr, (const uint64_t *)h->x_recv.ptr, nin,
                         (uint32_t *)h->x_ans.ptr, ptop, h->stream));
  if (int rc = a2a(h, h->x_ans.ptr, M.data(), 4, h->x_ans_back, true, &nback)) return rc;
  HIP_TRY(launch_resolve(h->g.d, 4, 0, nullptr, (uint32_t *)h->x_slot.ptr, nullptr, nsend,
                         (uint32_t *)h->x_ans_back.ptr, ptop, h->stream));
  *bytes += nsend * 8 + nin * 4;
  return CRGC_OK;
}

// The replicated chain closure (crgc_xchain.hip) from this round's received
// marks: every shard all-gathers the successor structure of its home shadows,
// closes the marked set by pointer doubling (the same work on every shard, so
// the same result), expands branching shadows at their homes and all-gathers
// what that marks, until an iteration marks nothing; then keeps its own range.
// Decided identically on every shard (from all-gathered counts), so every
// shard takes this path or none does.
static int xclosure(crgc_graph *h, bool investigate, const XRecv &xr, uint64_t *rounds, uint64_t *x_bytes) {
  const uint32_t G = h->G, me = h->shard;
  XcArgs x{};
  x.G = G;
  x.me = me;
  x.investigate = investigate ? 1 : 0;
  uint64_t P[MAX_SHARDS], N = 0;
  for (uint32_t d = 0; d < G; ++d) {
    P[d] = round_up(std::max<uint64_t>(h->peer_top[d], 1), 64);
    x.off[d] = N;
    N += P[d];
  }
  x.off[G] = N;
  x.N = N;
  x.P_me = P[me];
  uint32_t R = 1;
  while ((1ull << (R - 1)) < N) ++R;
  const uint32_t nflag = 2 * R + 4, fi_apply = 2 * R + 1;
  const size_t need = Carver::need({x.P_me * 4, x.P_me * 4, x.P_me / 8, x.P_me / 8, x.P_me / 8, x.P_me / 8,
                                    N * 4, N * 4, N * 4, N * 4, N / 8, N / 8, N / 8, N / 8, (size_t)nflag * 4,
                                    N * 4, 8});
  if (h->x_gc.ensure(need) != hipSuccess) return CRGC_E_NOMEM;
  Carver cv(h->x_gc.ptr);
  x.lnx = cv.take<uint32_t>(x.P_me);
  x.lsp = cv.take<uint32_t>(x.P_me);
  x.lvis = cv.take<uint32_t>(x.P_me / 32);
  x.lcx = cv.take<uint32_t>(x.P_me / 32);
  x.lpb = cv.take<uint32_t>(x.P_me / 32);
  x.seed = cv.take<uint32_t>(x.P_me / 32);
  x.gnx = cv.take<uint32_t>(N);
  x.gsp = cv.take<uint32_t>(N);
  uint32_t *ja = cv.take<uint32_t>(N), *jb = cv.take<uint32_t>(N);
  x.gvis = cv.take<uint32_t>(N / 32);
  x.gcx = cv.take<uint32_t>(N / 32);
  x.gpb_in = cv.take<uint32_t>(N / 32);
  x.gpb_out = cv.take<uint32_t>(N / 32);
  x.flag = cv.take<uint32_t>(nflag);
  x.xl = cv.take<uint32_t>(N);
  x.xl_n = cv.take<unsigned long long>(1);
  const DevGraph &g = h->g.d;
  HIP_TRY(hipMemsetAsync(x.seed, 0, x.P_me / 8, h->stream));
  HIP_TRY(hipMemsetAsync(x.flag, 0, (size_t)nflag * 4, h->stream));
  HIP_TRY(hipMemsetAsync(x.gpb_out, 0, N / 8, h->stream));
  HIP_TRY(launch_xclosure(g, x, 0, h->x_recv.ptr, (uint32_t *)&xr, 0, 0, 0, h->stream));
  HIP_TRY(launch_xclosure(g, x, 1, nullptr, nullptr, 0, 0, 0, h->stream));
  // the blocks to every shard: five all-gathers of variable-size blocks
  auto gather = [&](const void *send, void *recv, uint64_t unit_num, uint64_t unit_den) -> int {
    size_t soff[MAX_SHARDS], sb[MAX_SHARDS], roff[MAX_SHARDS], rb[MAX_SHARDS];
    for (uint32_t d = 0; d < G; ++d) {
      soff[d] = 0;
      sb[d] = P[me] * unit_num / unit_den;
      roff[d] = x.off[d] * unit_num / unit_den;
      rb[d] = P[d] * unit_num / unit_den;
    }
    if (int rc = h->tp->alltoallv(me, send, soff, sb, recv, roff, rb, h->stream)) {
      h->poisoned = true;
      return rc;
    }
    *x_bytes += sb[0] * (G - 1);
    return CRGC_OK;
  };
  if (int rc = gather(x.lnx, x.gnx, 4, 1)) return rc;
  if (int rc = gather(x.lsp, x.gsp, 4, 1)) return rc;
  if (int rc = gather(x.lvis, x.gvis, 1, 8)) return rc;
  if (int rc = gather(x.lcx, x.gcx, 1, 8)) return rc;
  if (int rc = gather(x.lpb, x.gpb_in, 1, 8)) return rc;
  std::vector<uint32_t> fl(nflag);
  std::vector<uint64_t> cnt(G);
  for (uint64_t it = 0;; ++it) {
    if (it > N) {
      h->poisoned = true;
      return CRGC_E_TIMEOUT;  // every iteration but the last marks a shadow
    }
    if (it) HIP_TRY(hipMemsetAsync(x.flag + 1, 0, (size_t)(nflag - 1) * 4, h->stream));
    HIP_TRY(hipMemsetAsync(x.xl_n, 0, 8, h->stream));
    for (uint32_t seq = 0; seq < 2; ++seq) {
      const uint32_t *src = seq ? x.gsp : x.gnx;
      uint32_t *dst = ja;
      for (uint32_t r = 0; r < R; ++r) {
        HIP_TRY(launch_xclosure(g, x, 2, src, dst, 0, 1 + seq * R + r, r == 0, h->stream));
        src = dst;
        dst = dst == ja ? jb : ja;
      }
    }
    HIP_TRY(launch_xclosure(g, x, 3, nullptr, nullptr, 0, 0, 0, h->stream));
    HIP_TRY(d2h_small(h, fl.data(), x.flag, (size_t)nflag * 4, SMALL_XFLAG_OFF));
    if (int rc = ag_u64(h, {{x.xl_n, 1}}, cnt.data())) return rc;  // synchronises
    d2h_small_done(h, fl.data(), (size_t)nflag * 4, SMALL_XFLAG_OFF);
    if (fl[0]) {
      h->poisoned = true;
      return DEV_FAIL("");  // a proxy without a resolved home slot: the resolution step failed
    }
    ++*rounds;
    bool jumped = false;
    for (uint32_t k = 1; k <= 2 * R; ++k) jumped |= fl[k] != 0;
    uint64_t total = 0;
    for (uint32_t d = 0; d < G; ++d) {
      cnt[d] = std::min<uint64_t>(cnt[d], N);
      total += cnt[d];
    }
    if (!jumped && total == 0) break;
    if (total) {
      size_t soff[MAX_SHARDS], sb[MAX_SHARDS], roff[MAX_SHARDS], rb[MAX_SHARDS];
      size_t ro = 0;
      for (uint32_t d = 0; d < G; ++d) {
        soff[d] = 0;
        sb[d] = cnt[me] * 4;
        roff[d] = ro;
        rb[d] = cnt[d] * 4;
        ro += rb[d];
      }
      if (h->x_gc_list.ensure(ro + 8) != hipSuccess) return CRGC_E_NOMEM;
      if (int rc = h->tp->alltoallv(me, x.xl, soff, sb, h->x_gc_list.ptr, roff, rb, h->stream)) {
        h->poisoned = true;
        return rc;
      }
      *x_bytes += cnt[me] * 4 * (G - 1);
      HIP_TRY(launch_xclosure(g, x, 4, h->x_gc_list.ptr, nullptr, total, fi_apply, 0, h->stream));
    }
    std::swap(x.gpb_in, x.gpb_out);
  }
  HIP_TRY(launch_xclosure(g, x, 5, nullptr, nullptr, 0, 0, 0, h->stream));
  return CRGC_OK;
}

// Sharded marks run in rounds: a local fixpoint, then every shard sends the
// proxies it marked to their homes, which continue from them.  A marked proxy
// travels as its home slot when the proxy has one cached — as a u32 list, or
// as a bitmap over the home's slots once the list would be longer (a dense
// round) — and as its id otherwise.  CRGC_XBITS: 0 ids only, 1 (default) the
// cheaper form per destination, 2 bitmaps whenever slots are sent.
//
// CRGC_XLEVELS = k > 0 caps a round at k level launches (after level 0): the
// exchange then follows the BFS level by level rather than each shard's local
// fixpoint, and a capped shard's pending candidates carry into its next round.
// The mark ends when no shard sends anything and none has pending work.
static int mark_all(crgc_graph *h, bool investigate, uint16_t location, uint64_t top, LevelRun &lr,
                    uint64_t *rounds, uint64_t *ids_sent, double *ms_x, uint64_t *x_bytes) {
  int end = 0;
  bool capped = false;
  const int cap = h->tp ? (int)h->knobs.xlevels : 0;
  if (int rc = run_levels(h, investigate, location, top, true, 0, lr, &end, nullptr, cap, &capped)) return rc;
  *rounds = 1;
  if (!h->tp) return CRGC_OK;
  const uint32_t G = h->G, me = h->shard;
  const int xmode = h->knobs.xbits;
  {
    const auto t0 = std::chrono::steady_clock::now();
    if (int rc = resolve_home_slots(h, top, xmode, x_bytes)) return rc;
    *ms_x += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  }
  // (the export scans the proxy region's blocks: k_xscan)
  const uint64_t npb = blocks_of(proxy_top_ub(h));
  std::vector<uint64_t> M((size_t)G * (2 * G + 1));  // per shard: ids, slots per destination; pending
  auto n_id = [&](uint32_t r, uint32_t d) { return M[(size_t)r * (2 * G + 1) + d]; };
  auto n_sl = [&](uint32_t r, uint32_t d) { return M[(size_t)r * (2 * G + 1) + G + d]; };
  auto words = [&](uint32_t d) { return (h->peer_top[d] + 31) / 32; };
  // A destination's home slots travel as a bitmap only once the list would be
  // xbitmap_ratio times its bytes: a bitmap costs the sender one global atomicOr
  // per mark (~20 G/s on gfx950), a list an LDS atomic and a coalesced store,
  // and the receiver imports either mark by mark.
  const uint64_t ratio = h->knobs.xbitmap_ratio;
  auto bitmap = [&](uint32_t r, uint32_t d) {
    return n_sl(r, d) > 0 && (xmode == 2 || n_sl(r, d) > ratio * words(d));
  };
  auto seg_bytes = [&](uint32_t r, uint32_t d) {
    const uint64_t b = 8 * n_id(r, d) + 4 * (bitmap(r, d) ? words(d) : n_sl(r, d));
    return (b + 7) & ~7ull;
  };
  // Most marks a round would send find their home already marked (C4 over 8
  // shards: ~29 M sent per shard and wakeup, ~3.5 M of them new at home), so
  // while rounds are wide every shard first all-gathers the homes' marked
  // bitmaps (4 B per 32 shadows of the graph) and sends only the marks whose
  // homes lack them.  On when the previous round sent at least as many marks
  // as the bitmaps have words (the first round always), the same decision on
  // every shard (all-gathered counts).
  uint64_t gwords = 0, prev_total = ~0ull;
  for (uint32_t d = 0; d < G; ++d) gwords += words(d);
  std::vector<uint64_t> hist;  // marks sent per round (the closure's shape test)
  int prev_used = 4;           // level launches the previous round needed (CRGC_ROUND_CHUNK=0)
  for (;;) {
    const auto t0 = std::chrono::steady_clock::now();
    // xcnt / xcnt2: k_xscan_sum writes every destination's totals; zeroed
    // only when there is no proxy block to scan
    if (npb == 0) HIP_TRY(launch_zero_u64((char *)h->ctr + CTR_OFF(xcnt), 3 * MAX_SHARDS, h->stream));
    XSend xs{};
    xs.use_slots = xmode != 0;
    xs.xq = h->knobs.xscan_q;
    if (xs.xq == 0) {
      xs.xq = 4;
      while (xs.xq > 1 && npb * xs.xq > 32768) xs.xq /= 2;
    }
    if (xmode != 0 && h->knobs.xfilter && prev_total >= gwords && gwords) {
      if (h->x_gvis.ensure(gwords * 4 + 8) != hipSuccess) return CRGC_E_NOMEM;
      size_t soff[MAX_SHARDS], sb[MAX_SHARDS], roff[MAX_SHARDS], rb[MAX_SHARDS];
      uint64_t o = 0;
      for (uint32_t d = 0; d < G; ++d) {
        xs.gvis_off[d] = o;
        soff[d] = 0;
        sb[d] = words(me) * 4;
        roff[d] = o * 4;
        rb[d] = words(d) * 4;
        o += words(d);
      }
      xs.gvis_off[G] = o;
      if (int rc = h->tp->alltoallv(me, h->g.d.vis, soff, sb, h->x_gvis.ptr, roff, rb, h->stream)) {
        h->poisoned = true;
        return rc;
      }
      *x_bytes += words(me) * 4 * (G - 1);
      xs.gvis = (const uint32_t *)h->x_gvis.ptr;
    }
    if (h->x_wgc.ensure((size_t)xscan_grid(npb, xs.xq) * 2 * G * 4 + 8) != hipSuccess) return CRGC_E_NOMEM;
    HIP_TRY(launch_xlist(h->g.d, false, npb, nullptr, xs, (uint32_t *)h->x_wgc.ptr, h->stream));
    // (with the counts, whether each shard's round was capped with work pending)
    h->h_small[SMALL_PEND_OFF / 8] = capped ? 1 : 0;
    if (int rc = ag_u64(h, {{(char *)h->ctr + CTR_OFF(xcnt), G}, {(char *)h->ctr + CTR_OFF(xcnt2), G},
                            {h->h_small + SMALL_PEND_OFF / 8, 1}}, M.data()))
      return rc;
    uint64_t total = 0, nsend = 0, pending = 0;
    for (uint32_t r = 0; r < G; ++r) {
      for (uint32_t k = 0; k < 2 * G; ++k) total += M[(size_t)r * (2 * G + 1) + k];
      pending += M[(size_t)r * (2 * G + 1) + 2 * G];
    }
    prev_total = total;
    hist.push_back(total);
    if (total == 0 && pending == 0) {
      *ms_x += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      return CRGC_OK;
    }
    // this shard's segments: ids, then slots or a bitmap, per destination
    std::vector<uint64_t> B((size_t)G * G);
    for (uint32_t r = 0; r < G; ++r)
      for (uint32_t d = 0; d < G; ++d) B[(size_t)r * G + d] = seg_bytes(r, d);
    uint64_t so = 0;
    for (uint32_t d = 0; d < G; ++d) {
      xs.id_off[d] = so;
      xs.sl_off[d] = so + 8 * n_id(me, d);
      xs.bitmap[d] = bitmap(me, d) ? 1 : 0;
      so += B[(size_t)me * G + d];
      nsend += n_id(me, d) + n_sl(me, d);
    }
    if (h->x_send.ensure(so + 8) != hipSuccess) return CRGC_E_NOMEM;
    bool any_bitmap = false;  // (the bitmap segments zeroed by one memset of the send buffer)
    for (uint32_t d = 0; d < G; ++d) any_bitmap |= xs.bitmap[d] != 0;
    if (any_bitmap) HIP_TRY(hipMemsetAsync(h->x_send.ptr, 0, so, h->stream));
    HIP_TRY(launch_xlist(h->g.d, true, npb, (char *)h->x_send.ptr, xs, (uint32_t *)h->x_wgc.ptr, h->stream));
    uint64_t nrecv = 0;
    if (int rc = a2a(h, h->x_send.ptr, B.data(), 1, h->x_recv, false, &nrecv)) return rc;
    *ids_sent += nsend;
    *x_bytes += so;
    XRecv xr{};
    xr.G = G;
    uint64_t ro = 0, items = 0;
    for (uint32_t r = 0; r < G; ++r) {
      xr.off[r] = ro;
      xr.n_id[r] = n_id(r, me);
      xr.bitmap[r] = bitmap(r, me) ? 1 : 0;
      xr.start[r] = items;
      items += n_id(r, me) + (xr.bitmap[r] ? words(me) : n_sl(r, me));
      ro += B[(size_t)r * G + me];
    }
    xr.start[G] = items;
    // A deep, narrow mark (chains across shards: about one round per link)
    // finishes in the replicated chain closure.  Every shard decides from the
    // same all-gathered counts.
    {
      const Knobs &kn = h->knobs;
      uint64_t n_all = 0, marks = total;
      for (uint32_t d = 0; d < G; ++d) n_all += h->peer_top[d];
      // (never with candidates pending: the closure starts from marks only)
      bool closure = xmode != 0 && pending == 0 && kn.xclosure_after && *rounds >= kn.xclosure_after &&
                     (kn.xclosure_narrow == 0 || marks * kn.xclosure_narrow <= n_all) && n_all < 0xF0000000ull;
      // ... and only for a chain-shaped mark, when the rounds it saves would cost
      // more than it does.  Its five all-gathers bring every shard ~8.4 B per
      // slot of the rest of the graph; a further round costs a fixed exchange
      // and level floor (xround_bytes, in link bytes) plus its marks.  A
      // chain's marks per round stay level: over the last XC_WINDOW rounds no
      // round sent less than half the round before (rounds left: from their
      // mean ratio, unbounded when level).  A shallow graph's last rounds fall
      // off faster: on C2 over 8 logical shards a closure at round 8 (the
      // round-5 rule, and a one-ratio test this round) moved 1.05 GB per
      // wakeup and still ended at round 9, 15.6 / 17.0 against 13.5 / 13.5 ms
      // without it (profiles/r6j).  The test hook xclosure_narrow = 0 forces it.
      if (closure && kn.xclosure_narrow != 0) {
        constexpr size_t XC_WINDOW = 3;
        const double cbytes = 8.375 * (double)n_all * (double)(G - 1) / (double)G;
        bool chain = hist.size() > XC_WINDOW;
        double lr = 0;  // mean log ratio of the window's rounds
        for (size_t k = hist.size() - std::min(hist.size(), XC_WINDOW); chain && k < hist.size(); ++k) {
          if (k == 0 || hist[k - 1] == 0 || 2 * hist[k] < hist[k - 1]) chain = false;
          else lr += std::log((double)hist[k] / (double)hist[k - 1]) / (double)XC_WINDOW;
        }
        double left = 1e30;
        if (marks == 0) left = 1;
        else if (chain && lr < -0.05) left = std::log((double)marks) / -lr + 1.0;
        closure = chain && left * ((double)kn.xround_bytes + 4.0 * (double)marks) >= cbytes;
        if (kn.level_log)
          fprintf(stderr, "[crgc] shard %u round %llu: marks %llu, closure %.1f MB, chain-shaped %d, %.1f rounds left: %s\n",
                  me, (unsigned long long)*rounds, (unsigned long long)marks, cbytes / 1e6, chain ? 1 : 0,
                  left > 1e29 ? -1.0 : left, closure ? "closure" : "rounds");
      }
      if (closure) {
        *ms_x += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        const auto t1 = std::chrono::steady_clock::now();
        const int rc = xclosure(h, investigate, xr, rounds, x_bytes);
        *ms_x += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t1).count();
        return rc;
      }
    }
    // received marks are candidates of level L: a sparse level after an empty
    // one, or — the round was capped — the pending level itself, whose
    // candidates (and the counts of the levels before it) are already there
    const int L = capped ? end : end + 2;
    HIP_TRY(launch_round_start(h->ctr, L, !capped, h->stream));
    HIP_TRY(launch_ximport(h->g.d, (const char *)h->x_recv.ptr, xr, L, h->stream));
    *ms_x += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    // A round from a few received marks is usually finished by k_tail in its
    // first level: launch one level first, not four (the rest would only check
    // that the mark is done: ~13 us each)
    const int wide = h->knobs.round_chunk ? (int)h->knobs.round_chunk : std::max(1, std::min(4, prev_used));
    const int first = !capped && items <= (h->knobs.walk ? h->knobs.walk_start : h->knobs.tail_start_sharded) ? 1 : wide;
    if (int rc = run_levels(h, investigate, location, top, false, L, lr, &end, nullptr, cap, &capped, first))
      return rc;
    prev_used = std::max(1, end - L + 1);  // (its levels with marks and the empty one that ended it)
    ++*rounds;
  }
}

// How the device can reach a caller's host buffer of `bytes` bytes
// (tools/hip_probe.hip, profiles/r4a/README.md):
//   HOST_PAGEABLE  unknown to the runtime: stream copies stage it
//   HOST_PINNED    wholly inside one page-locked allocation — a range of this
//                  handle's crgc_host_register, or a hipHostMalloc block (whose
//                  extent hipMemGetAddressRange reports; for registered memory it
//                  reports no base): device stores or copies; *dview = device view
//   HOST_PARTIAL   page-locked at its start but running past that allocation: the
//                  runtime refuses a copy into it and a device store past the
//                  range would fault, so its ids go through a bounce buffer
enum HostKind { HOST_PAGEABLE, HOST_PINNED, HOST_PARTIAL };

static HostKind host_kind(crgc_graph *h, const void *p, uint64_t bytes, uint64_t **dview) {
  *dview = nullptr;
  if (!p || !bytes) return HOST_PAGEABLE;
  hipPointerAttribute_t at{};
  if (hipPointerGetAttributes(&at, p) != hipSuccess) {
    (void)hipGetLastError();  // a soft status: not the caller's error
    return HOST_PAGEABLE;
  }
  if (at.type != hipMemoryTypeHost || !at.devicePointer) return HOST_PAGEABLE;
  const char *c = (const char *)p;
  for (const auto &r : h->pinned)
    if (c >= r.first && c < r.first + r.second) {
      if (c + bytes > r.first + r.second) return HOST_PARTIAL;
      *dview = (uint64_t *)at.devicePointer;
      return HOST_PINNED;
    }
  void *base = nullptr;
  size_t size = 0;
  if (hipMemGetAddressRange((hipDeviceptr_t *)&base, &size, (hipDeviceptr_t)p) != hipSuccess) {
    (void)hipGetLastError();  // sticky otherwise (hipErrorNotFound)
    return HOST_PARTIAL;
  }
  const char *bs = (const char *)base;
  const char *dv = (const char *)at.devicePointer;
  // the runtime reports the allocation in host or device addresses (one VA on gfx950)
  const bool in_host = bs && c >= bs && c + bytes <= bs + size;
  const bool in_dev = bs && dv >= bs && dv + bytes <= bs + size;
  if (!(in_host || in_dev)) return HOST_PARTIAL;
  *dview = (uint64_t *)at.devicePointer;
  return HOST_PINNED;
}

// The garbage / kill lists of the last trace into the caller's buffers by
// stream copies (or, for HOST_PARTIAL buffers, through a pinned bounce buffer).
static int copy_lists(crgc_graph *h, crgc_trace_out *out, bool sync = true) {
  bool big = false;
  out->n_garbage = h->last_garbage;
  out->n_kill = h->last_kill;
  out->n_live = h->last_live;
  out->stats = h->last_stats;
  struct Job {
    uint64_t *dst;
    const uint64_t *src;
    uint64_t n;
    bool bounce;
  } jobs[2] = {{out->garbage_ids, h->g.d.out_ids, h->last_garbage, false},
               {out->kill_ids, h->g.d.out_kill, h->last_kill, false}};
  const uint64_t caps[2] = {out->garbage_cap, out->kill_cap};
  uint64_t bounce_bytes = 0;
  for (int j = 0; j < 2; ++j) {
    Job &q = jobs[j];
    if (!q.dst) continue;
    if (caps[j] < q.n) {
      big = true;
      q.n = 0;
      continue;
    }
    uint64_t *dv;
    q.bounce = q.n && host_kind(h, q.dst, caps[j] * 8, &dv) == HOST_PARTIAL;
    if (q.bounce) bounce_bytes += q.n * 8;
  }
  if (bounce_bytes > h->h_bounce_bytes) {
    if (h->h_bounce) hipHostFree(h->h_bounce);
    h->h_bounce = nullptr;
    h->h_bounce_bytes = 0;
    HIP_TRY(hipHostMalloc((void **)&h->h_bounce, bounce_bytes, hipHostMallocDefault));
    h->h_bounce_bytes = bounce_bytes;
  }
  uint64_t at = 0;
  for (Job &q : jobs) {
    if (!q.dst || !q.n) continue;
    uint64_t *to = q.bounce ? h->h_bounce + at / 8 : q.dst;
    HIP_TRY(hipMemcpyAsync(to, q.src, q.n * 8, hipMemcpyDeviceToHost, h->stream));
    if (q.bounce) at += q.n * 8;
  }
  if (sync || bounce_bytes) HIP_TRY(hsync(h));
  at = 0;
  for (Job &q : jobs)
    if (q.dst && q.n && q.bounce) {
      memcpy(q.dst, h->h_bounce + at / 8, q.n * 8);
      at += q.n * 8;
    }
  return big ? CRGC_E2BIG : CRGC_OK;
}

// Sharded sweep: garbage whose supervisor is a proxy asks the supervisor's
// home for its mark; every shard learns the NPE verdict before committing;
// committed garbage invalidates the other shards' proxies of it.
static int sweep_sharded(crgc_graph *h, int should_kill, uint64_t top, double *ms_x) {
  const uint32_t G = h->G, me = h->shard;
  const uint64_t nblk = round_up(std::min<uint64_t>(top, h->g.caps.scap), BLK_SLOTS) / BLK_SLOTS;
  HIP_TRY(launch_sweep(h->g.d, should_kill, top, h->stream, 1));
  HIP_TRY(launch_zero_u64((char *)h->ctr + CTR_OFF(xcnt), 2 * MAX_SHARDS, h->stream));
  HIP_TRY(launch_list(h->g.d, 1, false, h->g.d.rq_buf, h->g.d.rq_cnt, nblk, nullptr, nullptr, h->stream));
  const auto t0 = std::chrono::steady_clock::now();
  // one all-gather: every shard's NPE count, garbage count (k_sweep_scan has it)
  // and kill requests per destination
  const uint32_t K = G + 2;
  std::vector<uint64_t> V((size_t)G * K);
  if (int rc = ag_u64(h, {{(char *)h->ctr + CTR_OFF(npe), 1}, {(char *)h->ctr + CTR_OFF(n_garbage), 1},
                          {(char *)h->ctr + CTR_OFF(xcnt), G}}, V.data()))
    return rc;
  uint64_t npe = 0;
  std::vector<uint64_t> R((size_t)G * G), NG(G);
  for (uint32_t r = 0; r < G; ++r) {
    npe += V[(size_t)r * K];
    NG[r] = V[(size_t)r * K + 1];
    for (uint32_t d = 0; d < G; ++d) R[(size_t)r * G + d] = V[(size_t)r * K + 2 + d];
  }
  if (npe) {  // the reference's NullPointerException on some shard: nobody commits
    HIP_TRY(hipMemcpyAsync((char *)h->ctr + CTR_OFF(npe), &npe, 8, hipMemcpyHostToDevice, h->stream));
    HIP_TRY(launch_sweep(h->g.d, should_kill, top, h->stream, 2));
    HIP_TRY(hsync(h));
    *ms_x += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return CRGC_OK;
  }
  uint64_t nreq = 0;
  for (uint32_t d = 0; d < G; ++d) nreq += R[(size_t)me * G + d];
  uint64_t total_req = 0;
  for (uint64_t v : R) total_req += v;
  if (total_req) {
    if (h->x_send.ensure(nreq * 8 + 8) != hipSuccess || h->x_slot.ensure(nreq * 4 + 8) != hipSuccess)
      return CRGC_E_NOMEM;
    HIP_TRY(launch_list(h->g.d, 1, true, h->g.d.rq_buf, h->g.d.rq_cnt, nblk, (uint64_t *)h->x_send.ptr,
                        (uint32_t *)h->x_slot.ptr, h->stream));
    uint64_t nin = 0, nback = 0;
    if (int rc = a2a(h, h->x_send.ptr, R.data(), 8, h->x_recv, false, &nin)) return rc;
    if (h->x_ans.ensure(nin + 8) != hipSuccess) return CRGC_E_NOMEM;
    HIP_TRY(launch_requests(h->g.d, 0, (const uint64_t *)h->x_recv.ptr, nin, (uint8_t *)h->x_ans.ptr,
                            nullptr, h->stream));
    if (int rc = a2a(h, h->x_ans.ptr, R.data(), 1, h->x_ans_back, true, &nback)) return rc;
  }
  HIP_TRY(launch_sweep(h->g.d, should_kill, top, h->stream, 2));  // ids + commit
  if (nreq)
    HIP_TRY(launch_requests(h->g.d, 1, nullptr, nreq, (uint8_t *)h->x_ans_back.ptr,
                            (const uint32_t *)h->x_slot.ptr, h->stream));
  // the other shards' proxies of this shard's garbage die with it (a shard
  // holds no proxy of an actor it homes: nothing goes to itself, so a one-shard
  // graph exchanges nothing here; the condition is the same on every shard)
  uint64_t tg = 0, tin = 0;
  for (uint32_t r = 0; r < G; ++r) {
    tg += NG[r];
    if (r != me) tin += NG[r];
  }
  if (G > 1 && tg) {
    size_t soff[MAX_SHARDS], sb[MAX_SHARDS], roff[MAX_SHARDS], rb[MAX_SHARDS];
    size_t ro = 0;
    for (uint32_t r = 0; r < G; ++r) {
      soff[r] = 0;
      sb[r] = r == me ? 0 : NG[me] * 8;
      roff[r] = ro;
      rb[r] = r == me ? 0 : NG[r] * 8;
      ro += rb[r];
    }
    if (h->x_recv.ensure(ro + 8) != hipSuccess) return CRGC_E_NOMEM;
    if (int rc = h->tp->alltoallv(me, h->g.d.out_ids, soff, sb, h->x_recv.ptr, roff, rb, h->stream)) {
      h->poisoned = true;
      return rc;
    }
    HIP_TRY(launch_invalidate(h->g.d, (const uint64_t *)h->x_recv.ptr, tin, h->stream));
  }
  *ms_x += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return CRGC_OK;
}

int crgc_trace(crgc_graph *h, int should_kill, crgc_trace_out *out) {
  if (int rc = check_graph(h)) return rc;
  if (!out) return CRGC_E_INVAL;
  DeviceGuard dg(h->device);
  const auto t0 = std::chrono::steady_clock::now();
  // Grids are sized from an upper bound of slot_top; the kernels read the
  // exact value from the device counters, so no synchronisation is needed here.
  const uint64_t top = h->slot_top + h->ids_since;
  reset_trace_counters(h);
  h->timed = h->n_traces++ % h->knobs.timing_every == 0;
  h->g.d.gslot_at = h->pend_n;  // this sweep's garbage slots are listed after the pending ones
  LevelRun lr;
  uint64_t rounds = 0, ids_sent = 0, x_bytes = 0;
  double ms_x = 0;
  bool direct = false;  // the lists are in the caller's buffers already
  if (!h->tp) {
    // The sweep is enqueued behind every level chunk and runs only once the
    // mark is done (mark_done), together with the counter read-back, so a
    // steady-state wakeup has one host synchronisation for mark + sweep.
    // caller buffers the device can write (page-locked / registered): the
    // lists go there behind the sweep, and the trace needs one host round trip
    uint64_t *dg = nullptr, *dk = nullptr;
    if (out->garbage_ids) (void)host_kind(h, out->garbage_ids, out->garbage_cap * 8, &dg);
    if (out->kill_ids) (void)host_kind(h, out->kill_ids, out->kill_cap * 8, &dk);
    auto sweep = [&]() -> hipError_t {
      hipError_t e = h->timed ? hipEventRecord(h->ev[1], h->stream) : hipSuccess;
      HostLists hl;
      hl.g = dg;
      hl.gcap = dg ? out->garbage_cap : 0;
      hl.k = dk;
      hl.kcap = dk ? out->kill_cap : 0;
      if (e == hipSuccess) e = launch_sweep(h->g.d, should_kill ? 1 : 0, top, h->stream, 3, hl);
      if (e == hipSuccess && h->timed) e = hipEventRecord(h->ev[2], h->stream);
      return e;  // the counters come back with the chunk's k_publish
    };
    int end = 0;
    rounds = 1;
    lr.defer = true;
    if (int rc = run_levels(h, false, 0, top, true, 0, lr, &end, sweep)) return rc;
    absorb_counters(h);  // read back with the last chunk's level counts
    const Counters &cc = *h->hctr;
    direct = (dg || dk) && (!out->garbage_ids || (dg && cc.n_garbage <= out->garbage_cap)) &&
             (!out->kill_ids || (dk && cc.n_kill <= out->kill_cap));
  } else {
    if (int rc = mark_all(h, false, 0, top, lr, &rounds, &ids_sent, &ms_x, &x_bytes)) return rc;
    if (h->timed) HIP_TRY(hipEventRecord(h->ev[1], h->stream));
    if (int rc = sweep_sharded(h, should_kill ? 1 : 0, top, &ms_x)) return rc;
    if (h->timed) HIP_TRY(hipEventRecord(h->ev[2], h->stream));
    HIP_TRY(sync_counters(h));
  }
  const Counters &c = *h->hctr;
  if (c.npe) return CRGC_E_NULL_SUPERVISOR;  // commit skipped: graph unchanged
  if (int rc = device_error(h)) return rc;
  h->last_garbage = c.n_garbage;
  h->last_kill = c.n_kill;
  h->last_live = c.n_live;
  // result copies first; the event queries overlap them
  int rc = CRGC_OK;
  if (direct) {
    out->n_garbage = h->last_garbage;
    out->n_kill = h->last_kill;
    out->n_live = h->last_live;
  } else {
    rc = copy_lists(h, out, /*sync=*/false);
  }
  if (lr.pending) {
    lr.pending();
    lr.pending = nullptr;
  }
  if (!direct) HIP_TRY(hsync(h));
  crgc_trace_stats st{};
  st.edges_scanned = c.edges_scanned;
  st.sup_edges = c.sup_edges;
  st.expand_launches = lr.timed;  // (the launches whose expand was timed: ms_expand, expand_bytes)
  st.expand_bytes = c.expand_bytes;
  st.levels = lr.levels;
  st.launches = lr.launches;
  st.ms_mark = lr.ms;
  st.ms_frontier = lr.ms_f;
  st.ms_tail = lr.ms_t;
  st.ms_expand = lr.ms_e;
  st.rounds = rounds;
  st.ids_sent = ids_sent;
  st.exchange_bytes = x_bytes;
  st.ms_exchange = ms_x;
  st.ms_sweep = h->timed ? elapsed_ms(h->ev[1], h->ev[2], &lr.time_fail) : 0.f;
  st.time_query_failures = lr.time_fail;
  st.direct_lists = direct ? 1 : 0;
  st.pseudo_roots = lr.roots;
  h->live = c.n_live;
  h->n_proxy = c.proxy_top - std::min(c.proxy_top, c.proxy_dead);
  h->inserted_at_trace = c.inserted;
  h->have_last = true;
  h->last_levels = lr.first_chunk;
  h->pull_pred = c.pulled;
  st.ms_total =
      std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  h->last_stats = st;
  out->stats = st;
  // Reclaim the listed garbage slots for the next merges' new shadows
  // (crgc_reuse.hip) once they are 1 / reuse_div of the range: queued behind
  // the trace, so it runs while the caller takes the results, and the next
  // merge on this stream starts after it.
  bool reclaimed = false;
  if (rc == CRGC_OK && h->g.d.freel && c.n_garbage) {
    h->pend_n += c.n_garbage;
    const uint32_t div = h->knobs.reuse_div;
    if (div == 0 || h->pend_n * div >= h->slot_top) {
      HIP_TRY(launch_reclaim(h->g.d, h->slot_top, h->pend_n, c.free_n, h->halted_seen, h->stream));
      std::swap(h->g.d.freel, h->g.d.freel2);
      h->pend_n = 0;
      h->free_avail = true;
      reclaimed = true;
    }
  }
  // Whether the merges since the last purge used the free list up: read only
  // while it may still hold slots (the traces after a batch purge).
  if (rc == CRGC_OK && h->free_avail && !reclaimed && h->g.d.freel) {
    HIP_TRY(sync_counters(h));
    h->free_avail = h->hctr->free_used < h->hctr->free_n;
  }
  // Keep the slot space dense: rebuild once dead slots outnumber live ones in
  // the shadows' region, or (sharded graphs) in the proxy region.
  const uint64_t ptop = c.proxy_top;
  if (rc == CRGC_OK && ((h->slot_top > 65536 && h->slot_top > 2 * h->live) ||
                        (ptop > 65536 && ptop > 2 * h->n_proxy))) {
    if (int r2 = rebuild(h, 0, 0)) return r2;
  }
  return rc;
}

int crgc_last_trace(crgc_graph *h, crgc_trace_out *out) {
  if (int rc = check_graph(h)) return rc;
  if (!out || !h->have_last) return CRGC_E_INVAL;
  DeviceGuard dg(h->device);
  return copy_lists(h, out);
}

// DeltaGraphs of one wakeup (crgc_delta.hip): the chain of graph starts,
// then a count pass, scans, and a write pass over the graphs.
int crgc_build_delta_graphs(crgc_graph *h, const crgc_entry_batch *b, crgc_delta_graphs *out) {
  if (int rc = check_graph(h)) return rc;
  if (!out || out->memory > CRGC_MEM_DEVICE) return CRGC_E_INVAL;
  if (h->DGS > DG_MAX || h->DGS <= 4 * h->F + 1) return CRGC_E_INVAL;
  DeviceGuard dg(h->device);
  uint64_t C = 0, S = 0, U = 0;
  // device batches: bounds only (the kernels read the exact totals), no round trip
  if (int rc = entry_counts(h, b, false, &C, &S, &U)) return rc;
  const uint64_t n = b->n_entries;
  if (n >= (1ull << 31)) return CRGC_E_INVAL;
  const size_t nh_bytes =
      b->memory == CRGC_MEM_HOST
          ? Carver::need({n * 8, n * 2, n, (n + 1) * 4, C * 8, C * 8, (n + 1) * 4, S * 8, (n + 1) * 4, U * 8,
                          U * 2})
          : 0;
  const uint32_t levels = 2;  // J and J^64
  const uint64_t N = n + 1, nblk = (n + 1023) / 1024, nbs = 4 * ((N + 1023) / 1024) + 8;
  // the write pass's slots: every shadow of a graph is an id occurrence of its
  // entries, every outgoing entry a created or updated ref
  const uint64_t TR = n + 2 * C + S + U, TO = C + U, TW = 2 * N + 13 * TR + 6 * TO;
  const size_t need = Carver::need({sizeof(DgCounters), (size_t)levels * N * 4, N, N, nblk * 4 + 4,
                                    nblk * 8 + 8, nbs * 8, N * 4, N * 4, N * 4, N * 4, N * 8, N * 8, N * 8,
                                    N * 4, N * 4, N * 4, N * 8, N * 8, N * 8, TR * 8, TR * 4, TR * 8, TR,
                                    TR * 4, TO * 8, TO * 4, TW});
  if (h->stage.ensure(nh_bytes + 256) != hipSuccess || h->x_dg.ensure(need) != hipSuccess)
    return CRGC_E_NOMEM;
  Carver sc(h->stage.ptr), dc(h->x_dg.ptr);
  DgArgs a{};
  a.n = n;
  a.F = h->F;
  a.DGS = h->DGS;
  a.T = h->DGS - 4 * h->F - 1;
  a.C = C;
  a.S = S;
  a.U = U;
  if (n) {
    a.self = stage(h, sc, b->self, n, b->memory);
    a.recv = stage(h, sc, b->recv_count, n, b->memory);
    a.flags = stage(h, sc, b->flags, n, b->memory);
    a.c_off = stage(h, sc, b->created_off, n + 1, b->memory);
    a.c_owner = stage(h, sc, b->created_owner, C, b->memory);
    a.c_target = stage(h, sc, b->created_target, C, b->memory);
    a.s_off = stage(h, sc, b->spawned_off, n + 1, b->memory);
    a.spawned = stage(h, sc, b->spawned, S, b->memory);
    a.u_off = stage(h, sc, b->updated_off, n + 1, b->memory);
    a.u_ref = stage(h, sc, b->updated_ref, U, b->memory);
    a.u_info = stage(h, sc, b->updated_info, U, b->memory);
  }
  a.ctr = dc.take<DgCounters>(1);
  a.J = dc.take<uint32_t>((size_t)levels * N);
  a.mark = dc.take<uint8_t>(N);
  a.lng = dc.take<uint8_t>(N);
  a.blk = dc.take<uint32_t>(nblk + 1);
  a.blk_off = dc.take<uint64_t>(nblk + 1);
  a.bsum = dc.take<uint64_t>(nbs);
  a.starts = dc.take<uint32_t>(N);
  a.g_size = dc.take<uint32_t>(N);
  a.g_nout = dc.take<uint32_t>(N);
  a.g_bytes = dc.take<uint32_t>(N);
  a.g_shadow = dc.take<uint64_t>(N);
  a.g_out = dc.take<uint64_t>(N);
  a.g_wire = dc.take<uint64_t>(N);
  a.b_size = dc.take<uint32_t>(N);
  a.b_out = dc.take<uint32_t>(N);
  a.b_bytes = dc.take<uint32_t>(N);
  a.t_shadow = dc.take<uint64_t>(N);
  a.t_out = dc.take<uint64_t>(N);
  a.t_wire = dc.take<uint64_t>(N);
  DgOut t{};
  t.id = dc.take<uint64_t>(TR);
  t.recv = dc.take<int32_t>(TR);
  t.sup = dc.take<uint64_t>(TR);
  t.flags = dc.take<uint8_t>(TR);
  t.out_off = dc.take<uint32_t>(TR);
  t.out_target = dc.take<uint64_t>(TO);
  t.out_count = dc.take<int32_t>(TO);
  t.wire = dc.take<uint8_t>(TW);
  t.shadow_cap = TR;
  t.out_cap = TO;
  t.wire_cap = TW;
  HIP_TRY(hipMemsetAsync(a.ctr, 0, sizeof(DgCounters), h->stream));
  DgCounters hc{};
  auto fetch = [&]() -> int {
    HIP_TRY(hipMemcpyAsync(&hc, a.ctr, sizeof(DgCounters), hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hsync(h));
    return CRGC_OK;
  };
  // Device outputs of the right shape: the write pass can run on the device's
  // counts before the host has seen them (capacities checked on the device).
  const bool dev = out->memory == CRGC_MEM_DEVICE;
  const bool any = out->graph_off || out->wire_off || out->id || out->recv_count || out->supervisor ||
                   out->flags || out->out_off || out->out_target || out->out_count || out->wire;
  const bool complete = out->graph_off && out->wire_off && out->id && out->recv_count && out->supervisor &&
                        out->flags && out->out_off && out->out_target && out->out_count && out->wire;
  DgOut o{};
  if (dev) {
    o = DgOut{out->graph_off, out->wire_off, out->id, out->recv_count, out->supervisor, out->flags,
              out->out_off, out->out_target, out->out_count, out->wire,
              out->graph_cap, out->shadow_cap, out->out_cap, out->wire_cap};
  }
  const bool speculate = dev && complete;
  uint64_t G = 0;
  bool written = false;
  if (n) {
    // The chain, then the write pass into bounded slots and the scans of the
    // exact sizes, on the device's graph count without a host round trip; with
    // device outputs the compaction and offsets follow the same way.
    HIP_TRY(launch_dg_chain(a, 0, h->stream));
    HIP_TRY(launch_dg_write(a, DG_NG_DEVICE, t, h->stream));
    if (speculate) {
      HIP_TRY(launch_dg_compact(a, DG_NG_DEVICE, t, o, h->stream));
      HIP_TRY(launch_dg_offsets(a, DG_NG_DEVICE, o, h->stream));
    }
    if (int rc = fetch()) return rc;
    if (hc.err) return CRGC_E_INVAL;  // malformed offsets or reserved ids: nothing was built
    written = speculate && hc.first_long == ~0u && !hc.overflow;
    if (hc.first_long != ~0u) {  // a chain start whose graph runs past the span window
      while (hc.first_long != ~0u) {
        HIP_TRY(launch_dg_chain(a, 1, h->stream));
        if (int rc = fetch()) return rc;
      }
      HIP_TRY(launch_dg_write(a, hc.n_graphs, t, h->stream));
      if (int rc = fetch()) return rc;
      if (hc.err) return CRGC_E_INVAL;
    }
    G = hc.n_graphs;
  }
  const uint64_t NS = n ? hc.n_shadows : 0, NO = n ? hc.n_out : 0, NW = n ? hc.wire : 0;
  out->n_graphs = G;
  out->n_shadows = NS;
  out->n_out = NO;
  out->wire_bytes = NW;
  if (!any) return CRGC_OK;  // sizes only
  if (!out->graph_off || !out->wire_off || !out->id || !out->recv_count || !out->supervisor || !out->flags ||
      !out->out_off || (NO && (!out->out_target || !out->out_count)) || !out->wire)
    return CRGC_E_INVAL;
  if (out->graph_cap < G || out->shadow_cap < NS || out->out_cap < NO || out->wire_cap < NW) return CRGC_E2BIG;
  if (!dev) {
    const size_t ob = Carver::need({(G + 1) * 4, (G + 1) * 8, NS * 8, NS * 4, NS * 8, NS, (NS + 1) * 4, NO * 8,
                                    NO * 4, NW});
    if (h->x_dg_out.ensure(ob) != hipSuccess) return CRGC_E_NOMEM;
    Carver oc(h->x_dg_out.ptr);
    o.graph_off = oc.take<uint32_t>(G + 1);
    o.wire_off = oc.take<uint64_t>(G + 1);
    o.id = oc.take<uint64_t>(NS);
    o.recv = oc.take<int32_t>(NS);
    o.sup = oc.take<uint64_t>(NS);
    o.flags = oc.take<uint8_t>(NS);
    o.out_off = oc.take<uint32_t>(NS + 1);
    o.out_target = oc.take<uint64_t>(NO);
    o.out_count = oc.take<int32_t>(NO);
    o.wire = oc.take<uint8_t>(NW);
  }
  if (G && !written) {
    HIP_TRY(launch_dg_compact(a, G, t, o, h->stream));
    HIP_TRY(launch_dg_offsets(a, G, o, h->stream));
  } else if (!G) {  // no graphs: the closing offsets only
    HIP_TRY(hipMemsetAsync(o.graph_off, 0, 4, h->stream));
    HIP_TRY(hipMemsetAsync(o.wire_off, 0, 8, h->stream));
    HIP_TRY(hipMemsetAsync(o.out_off, 0, 4, h->stream));
  }
  if (!dev) {
    auto d2h = [&](void *dst, const void *src, size_t bytes) -> hipError_t {
      return bytes ? hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, h->stream) : hipSuccess;
    };
    HIP_TRY(d2h(out->graph_off, o.graph_off, (G + 1) * 4));
    HIP_TRY(d2h(out->wire_off, o.wire_off, (G + 1) * 8));
    HIP_TRY(d2h(out->id, o.id, NS * 8));
    HIP_TRY(d2h(out->recv_count, o.recv, NS * 4));
    HIP_TRY(d2h(out->supervisor, o.sup, NS * 8));
    HIP_TRY(d2h(out->flags, o.flags, NS));
    HIP_TRY(d2h(out->out_off, o.out_off, (NS + 1) * 4));
    HIP_TRY(d2h(out->out_target, o.out_target, NO * 8));
    HIP_TRY(d2h(out->out_count, o.out_count, NO * 4));
    HIP_TRY(d2h(out->wire, o.wire, NW));
    HIP_TRY(hsync(h));
  }
  return CRGC_OK;  // device outputs: stream-ordered (crgc_sync waits for them)
}

int crgc_sync(crgc_graph *h) {
  if (int rc = check_graph(h)) return rc;
  DeviceGuard dg(h->device);
  HIP_TRY(hsync(h));
  return CRGC_OK;
}

}  // extern "C"

// ---- UndoLog folding on the device (crgc_undo.hip) ---------------------------
struct crgc_undo_acc {
  crgc_graph *h = nullptr;
  uint16_t location = 0;
  UndoAccDev d{};
  void *mem = nullptr;                 // the tables
  unsigned long long *ctr = nullptr;   // n_ids, n_pairs
  uint64_t ids_ub = 0, pairs_ub = 0;   // upper bounds of the inserted keys
  Scratch stage, exp;
};

namespace {

static uint64_t pow2_at_least(uint64_t v) {
  uint64_t p = 1024;
  while (p < v) p <<= 1;
  return p;
}

static hipError_t ua_alloc(UndoAccDev &d, void **mem, uint64_t cap, uint64_t pcap, unsigned long long *ctr,
                           hipStream_t s) {
  const size_t bytes = Carver::need({cap * 8, cap, cap * 4, pcap * 8, pcap * 4});
  if (hipError_t e = hipMalloc(mem, bytes)) return e;
  Carver c(*mem);
  d.keys = c.take<uint64_t>(cap);
  d.adm = c.take<uint8_t>(cap);
  d.msg = c.take<int32_t>(cap);
  d.pkeys = c.take<uint64_t>(pcap);
  d.pcnt = c.take<int32_t>(pcap);
  d.cap = cap;
  d.pcap = pcap;
  d.n_ids = ctr;
  d.n_pairs = ctr + 1;
  return launch_ua_init(d, s);
}

// Room for `ids` / `pairs` more keys at load <= 1/2, rehashing into larger tables.
static int ua_reserve(crgc_undo_acc *u, uint64_t ids, uint64_t pairs) {
  crgc_graph *h = u->h;
  if (u->ids_ub + ids <= u->d.cap / 2 && u->pairs_ub + pairs <= u->d.pcap / 2) return CRGC_OK;
  unsigned long long c[2];
  HIP_TRY(hipMemcpyAsync(c, u->ctr, 16, hipMemcpyDeviceToHost, h->stream));
  HIP_TRY(hsync(h));
  u->ids_ub = c[0];
  u->pairs_ub = c[1];
  const bool grow_ids = u->ids_ub + ids > u->d.cap / 2;
  const bool grow_pairs = grow_ids || u->pairs_ub + pairs > u->d.pcap / 2;
  if (!grow_pairs) return CRGC_OK;
  const uint64_t cap = grow_ids ? pow2_at_least(4 * (u->ids_ub + ids)) : u->d.cap;
  const uint64_t pcap = u->pairs_ub + pairs > u->d.pcap / 2 ? pow2_at_least(4 * (u->pairs_ub + pairs)) : u->d.pcap;
  UndoAccDev n{};
  void *mem = nullptr;
  HIP_TRY(ua_alloc(n, &mem, cap, pcap, u->ctr, h->stream));
  uint32_t *map = nullptr;  // the new tables are one allocation: ids move too
  if (hipMalloc(&map, u->d.cap * 4) != hipSuccess) {
    hipFree(mem);
    return CRGC_E_NOMEM;
  }
  hipError_t e = launch_ua_rehash(u->d, n, map, true, h->stream);
  if (e == hipSuccess) e = hsync(h);
  if (map) hipFree(map);
  if (e != hipSuccess) {
    hipFree(mem);
    return map_hip(e);
  }
  hipFree(u->mem);
  u->mem = mem;
  u->d = n;
  return CRGC_OK;
}

}  // namespace

extern "C" {

int crgc_undo_acc_create(crgc_graph *h, uint16_t node_location, crgc_undo_acc **out) {
  if (!out) return CRGC_E_INVAL;
  *out = nullptr;
  if (int rc = check_graph(h)) return rc;
  DeviceGuard dg(h->device);
  crgc_undo_acc *u = new (std::nothrow) crgc_undo_acc();
  if (!u) return CRGC_E_NOMEM;
  u->h = h;
  u->location = node_location;
  if (hipMalloc(&u->ctr, 16) != hipSuccess) {
    delete u;
    return CRGC_E_NOMEM;
  }
  hipError_t e = hipMemsetAsync(u->ctr, 0, 16, h->stream);
  // Initial size from the graph's: a node's log names at most the actors the
  // graph has seen from it, so a quarter of the slots avoids the rehashes of a
  // log that grows from nothing (HBM is plentiful; an export scans the table).
  const uint64_t hint = pow2_at_least(std::max<uint64_t>(1 << 12, (h->slot_top + h->ids_since) / 4));
  if (e == hipSuccess) e = ua_alloc(u->d, &u->mem, hint, 2 * hint, u->ctr, h->stream);
  if (e != hipSuccess) {
    crgc_undo_acc_destroy(u);
    return map_hip(e);
  }
  *out = u;
  return CRGC_OK;
}

void crgc_undo_acc_destroy(crgc_undo_acc *u) {
  if (!u) return;
  DeviceGuard dg(u->h->device);
  hipStreamSynchronize(u->h->stream);
  if (u->mem) hipFree(u->mem);
  if (u->ctr) hipFree(u->ctr);
  u->stage.release();
  u->exp.release();
  delete u;
}

int crgc_undo_acc_fold_deltas(crgc_undo_acc *u, const crgc_delta_batch *b) {
  if (!u) return CRGC_E_INVAL;
  crgc_graph *h = u->h;
  if (int rc = check_graph(h)) return rc;
  DeviceGuard dg(h->device);
  uint64_t nout = 0;
  if (int rc = delta_counts(h, b, &nout)) return rc;
  const uint64_t n = b->n_shadows;
  if (n == 0) return CRGC_OK;
  if (int rc = ua_reserve(u, n + nout, nout)) return rc;
  const size_t host_bytes =
      b->memory == CRGC_MEM_HOST ? Carver::need({n * 8, n * 4, n, (n + 1) * 4, nout * 8, nout * 4}) : 0;
  if (u->stage.ensure(host_bytes + 256) != hipSuccess) return CRGC_E_NOMEM;
  Carver sc(u->stage.ptr);
  Staged staged(h, b->memory);
  UaDeltaArgs a{};
  a.n = n;
  a.nout = nout;
  a.id = stage(h, sc, b->id, n, b->memory);
  a.recv = stage(h, sc, b->recv_count, n, b->memory);
  a.flags = stage(h, sc, b->flags, n, b->memory);
  a.out_off = stage(h, sc, b->out_off, n + 1, b->memory);
  a.out_target = stage(h, sc, b->out_target, nout, b->memory);
  a.out_count = stage(h, sc, b->out_count, nout, b->memory);
  HIP_TRY(staged.mark());
  HIP_TRY(launch_ua_fold_deltas(u->d, a, h->stream));
  HIP_TRY(staged.wait());
  u->ids_ub += n + nout;
  u->pairs_ub += nout;
  return CRGC_OK;
}

int crgc_undo_acc_fold_ingress(crgc_undo_acc *u, const crgc_undo_log *f) {
  if (!u || !f || f->memory > CRGC_MEM_DEVICE) return CRGC_E_INVAL;
  crgc_graph *h = u->h;
  if (int rc = check_graph(h)) return rc;
  DeviceGuard dg(h->device);
  const uint64_t n = f->n_fields;
  if (n == 0) return CRGC_OK;
  if (!f->actor || !f->message_count || !f->created_off) return CRGC_E_INVAL;
  uint32_t nc32 = 0;
  if (f->memory == CRGC_MEM_HOST) {
    if (f->created_off[0]) return CRGC_E_INVAL;
    nc32 = f->created_off[n];
  } else {
    HIP_TRY(hipMemcpyAsync(&nc32, f->created_off + n, 4, hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hsync(h));
  }
  const uint64_t nc = nc32;
  if (nc && (!f->created_target || !f->created_count)) return CRGC_E_INVAL;
  if (int rc = ua_reserve(u, n + nc, nc)) return rc;
  const size_t host_bytes =
      f->memory == CRGC_MEM_HOST ? Carver::need({n * 8, n * 4, (n + 1) * 4, nc * 8, nc * 4}) : 0;
  if (u->stage.ensure(host_bytes + 256) != hipSuccess) return CRGC_E_NOMEM;
  Carver sc(u->stage.ptr);
  Staged staged(h, f->memory);
  UaFieldArgs a{};
  a.n = n;
  a.nc = nc;
  a.sign = 1;
  a.actor = stage(h, sc, f->actor, n, f->memory);
  a.msg = stage(h, sc, f->message_count, n, f->memory);
  a.c_off = stage(h, sc, f->created_off, n + 1, f->memory);
  a.c_target = stage(h, sc, f->created_target, nc, f->memory);
  a.c_count = stage(h, sc, f->created_count, nc, f->memory);
  HIP_TRY(staged.mark());
  HIP_TRY(launch_ua_fold_fields(u->d, a, h->stream));
  HIP_TRY(staged.wait());
  u->ids_ub += n + nc;
  u->pairs_ub += nc;
  return CRGC_OK;
}

int crgc_undo_acc_export(crgc_undo_acc *u, crgc_undo_log_out *out) {
  if (!u || !out) return CRGC_E_INVAL;
  crgc_graph *h = u->h;
  if (int rc = check_graph(h)) return rc;
  DeviceGuard dg(h->device);
  const uint64_t cap = u->d.cap, nbs = 4 * ((cap + 1023) / 1024) + 8;
  const size_t need = Carver::need({16, cap * 4, cap * 4, cap * 8, cap * 8, nbs * 8});
  if (u->exp.ensure(need) != hipSuccess) return CRGC_E_NOMEM;
  Carver c(u->exp.ptr);
  UaExportArgs x{};
  x.n_fields = c.take<unsigned long long>(2);
  x.n_created = x.n_fields + 1;
  x.admf = c.take<uint32_t>(cap);
  x.deg = c.take<uint32_t>(cap);
  x.aidx = c.take<uint64_t>(cap);
  x.roff = c.take<uint64_t>(cap);
  x.bsum = c.take<uint64_t>(nbs);
  HIP_TRY(launch_ua_export(u->d, x, 0, h->stream));
  unsigned long long nn[2];
  HIP_TRY(hipMemcpyAsync(nn, x.n_fields, 16, hipMemcpyDeviceToHost, h->stream));
  HIP_TRY(hsync(h));
  const uint64_t NF = nn[0], NC = nn[1];
  out->n_fields = NF;
  out->n_created = NC;
  if (!out->actor && !out->message_count && !out->created_off && !out->created_target && !out->created_count)
    return CRGC_OK;
  if (!out->actor || !out->message_count || !out->created_off || (NC && (!out->created_target || !out->created_count)))
    return CRGC_E_INVAL;
  if (out->field_cap < NF || out->created_cap < NC) return CRGC_E2BIG;
  Scratch o;
  if (o.ensure(Carver::need({NF * 8, NF * 4, (NF + 1) * 4, NC * 8, NC * 4})) != hipSuccess) return CRGC_E_NOMEM;
  Carver oc(o.ptr);
  x.actor = oc.take<uint64_t>(NF);
  x.msg = oc.take<int32_t>(NF);
  x.c_off = oc.take<uint32_t>(NF + 1);
  x.c_target = oc.take<uint64_t>(NC);
  x.c_count = oc.take<int32_t>(NC);
  hipError_t e = launch_ua_export(u->d, x, 1, h->stream);
  auto d2h = [&](void *dst, const void *src, size_t bytes) {
    if (e == hipSuccess && bytes) e = hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, h->stream);
  };
  d2h(out->actor, x.actor, NF * 8);
  d2h(out->message_count, x.msg, NF * 4);
  d2h(out->created_off, x.c_off, (NF + 1) * 4);
  d2h(out->created_target, x.c_target, NC * 8);
  d2h(out->created_count, x.c_count, NC * 4);
  if (e == hipSuccess) e = hsync(h);
  o.release();
  return map_hip(e);
}

int crgc_merge_undo_acc(crgc_graph *h, crgc_undo_acc *u) {
  if (!u || u->h != h) return CRGC_E_INVAL;
  crgc_undo_log_out q{};
  if (int rc = crgc_undo_acc_export(u, &q)) return rc;
  std::vector<uint64_t> actor(q.n_fields + 1), target(q.n_created + 1);
  std::vector<int32_t> msg(q.n_fields + 1), count(q.n_created + 1);
  std::vector<uint32_t> off(q.n_fields + 1);
  q.field_cap = q.n_fields;
  q.created_cap = q.n_created;
  q.actor = actor.data();
  q.message_count = msg.data();
  q.created_off = off.data();
  q.created_target = target.data();
  q.created_count = count.data();
  if (int rc = crgc_undo_acc_export(u, &q)) return rc;
  crgc_undo_log log{};
  log.node_location = u->location;
  log.n_fields = q.n_fields;
  log.actor = actor.data();
  log.message_count = msg.data();
  log.created_off = off.data();
  log.created_target = target.data();
  log.created_count = count.data();
  log.memory = CRGC_MEM_HOST;
  return crgc_merge_undo(h, &log);
}

int crgc_local_roots(crgc_graph *h, uint64_t *out, uint64_t cap, uint64_t *n) {
  if (int rc = check_graph(h)) return rc;
  if (!n) return CRGC_E_INVAL;
  DeviceGuard dg(h->device);
  HIP_TRY(sync_counters(h));
  if (h->roots_cap < h->g.caps.scap) {
    if (h->roots_buf) hipFree(h->roots_buf);
    h->roots_buf = nullptr;
    h->roots_cap = 0;
    HIP_TRY(hipMalloc(&h->roots_buf, h->g.caps.scap * 8));
    h->roots_cap = h->g.caps.scap;
  }
  hipMemsetAsync((char *)h->ctr + CTR_OFF(n_out), 0, 8, h->stream);
  DevGraph d = h->g.d;
  d.out_a = h->roots_buf;
  HIP_TRY(launch_local_roots(d, h->slot_top, h->stream));
  unsigned long long k = 0;
  HIP_TRY(hipMemcpyAsync(&k, (char *)h->ctr + CTR_OFF(n_out), 8, hipMemcpyDeviceToHost,
                         h->stream));
  HIP_TRY(hsync(h));
  *n = k;
  if (!out) return CRGC_OK;
  if (cap < k) return CRGC_E2BIG;
  if (k) HIP_TRY(hipMemcpy(out, h->roots_buf, k * 8, hipMemcpyDeviceToHost));
  return CRGC_OK;
}

int crgc_count_reachable_from(crgc_graph *h, uint16_t location, int64_t *out) {
  if (int rc = check_graph(h)) return rc;
  if (!out) return CRGC_E_INVAL;
  DeviceGuard dg(h->device);
  HIP_TRY(sync_counters(h));
  if (int rc = device_error(h)) return rc;
  reset_trace_counters(h);
  h->timed = true;
  LevelRun lr;
  uint64_t rounds = 0, sent = 0, x_bytes = 0;
  double ms_x = 0;
  const uint64_t saved = h->last_levels;
  const int rl = mark_all(h, true, location, h->slot_top, lr, &rounds, &sent, &ms_x, &x_bytes);
  h->last_levels = saved;
  if (rl) return rl;
  if (!h->tp) {
    HIP_TRY(sync_counters(h));
    *out = (int64_t)h->hctr->marked;
    return CRGC_OK;
  }
  HIP_TRY(hipMemsetAsync((char *)h->ctr + CTR_OFF(n_out), 0, 8, h->stream));
  HIP_TRY(launch_count_marked(h->g.d, h->slot_top, h->stream));
  std::vector<uint64_t> all(h->G);
  if (int rc = ag_u64(h, {{(char *)h->ctr + CTR_OFF(n_out), 1}}, all.data())) return rc;
  int64_t sum = 0;
  for (uint64_t v : all) sum += (int64_t)v;
  *out = sum;
  return CRGC_OK;
}


int crgc_total_actors_seen(crgc_graph *h, uint64_t *out) {
  if (!h || !out) return CRGC_E_INVAL;
  DeviceGuard dg(h->device);
  HIP_TRY(sync_counters(h));
  *out = h->hctr->inserted;
  return CRGC_OK;
}

int crgc_host_register(crgc_graph *h, void *ptr, uint64_t bytes) {
  if (int rc = check_graph(h)) return rc;
  if (!ptr || !bytes) return CRGC_E_INVAL;
  char *b = (char *)ptr;
  for (auto &p : h->pinned)
    if (b < p.first + p.second && p.first < b + bytes) return CRGC_E_INVAL;
  DeviceGuard dg(h->device);
  const hipError_t e = hipHostRegister(ptr, bytes, hipHostRegisterDefault);
  if (e != hipSuccess) return e == hipErrorOutOfMemory ? CRGC_E_NOMEM : CRGC_E_INVAL;
  void *dev = nullptr;  // the device's view, for the chunk copies of registered batches
  if (hipHostGetDevicePointer(&dev, ptr, 0) != hipSuccess || !dev) {
    (void)hipGetLastError();
    hipHostUnregister(ptr);
    return DEV_FAIL("");
  }
  h->pinned.push_back({b, bytes, (char *)dev});
  return CRGC_OK;
}

int crgc_host_unregister(crgc_graph *h, void *ptr) {
  if (!h || !ptr) return CRGC_E_INVAL;
  for (size_t i = 0; i < h->pinned.size(); ++i)
    if (h->pinned[i].first == (char *)ptr) {
      DeviceGuard dg(h->device);
      // An async merge (crgc_merge_entries_async) returns while k_copy_ranges on
      // the copy stream may still read this range over PCIe, and its merges on
      // the graph's stream read the staged copy: wait for both before the pages
      // are unpinned (a queued kernel reading unpinned pages faults the GPU).
      const hipError_t ec = stream_wait(h->cpy, h->knobs.spin_us);
      const hipError_t es = h->poisoned ? hipSuccess : hsync(h);
      hipHostUnregister(ptr);
      h->pinned.erase(h->pinned.begin() + (long)i);
      if (ec != hipSuccess) return map_hip(ec);
      if (es != hipSuccess) return map_hip(es);
      return CRGC_OK;
    }
  return CRGC_E_INVAL;
}

int crgc_usage_of(crgc_graph *h, crgc_usage *out) {
  if (int rc = check_graph(h)) return rc;
  if (!out) return CRGC_E_INVAL;
  DeviceGuard dg(h->device);
  HIP_TRY(sync_counters(h));
  const Caps &c = h->g.caps;
  *out = crgc_usage{};
  out->slot_top = h->slot_top;
  out->slot_cap = c.pbase;
  out->proxy_top = h->proxy_top;
  out->proxy_cap = c.scap - c.pbase;
  out->free_slots = h->hctr->free_n - std::min(h->hctr->free_used, h->hctr->free_n);
  out->pool_top = h->pool_top;
  out->pool_cap = c.pcap;
  out->etab_used = h->etab_used;
  out->etab_cap = c.ecap;
  out->rebuilds = h->n_rebuild;
  out->grows = h->n_grow;
  out->repacks = h->n_repack;
  return CRGC_OK;
}

int crgc_compact(crgc_graph *h) {
  if (int rc = check_graph(h)) return rc;
  DeviceGuard dg(h->device);
  return rebuild(h, 0, 0);
}

int crgc_live_count(crgc_graph *h, uint64_t *out) {
  if (int rc = check_graph(h)) return rc;
  if (!out) return CRGC_E_INVAL;
  DeviceGuard dg(h->device);
  HIP_TRY(sync_counters(h));
  // alive slots = slot_top minus dead slots: count on the host copy of flags
  std::vector<uint8_t> fl(h->slot_top);
  if (h->slot_top)
    HIP_TRY(hipMemcpy(fl.data(), h->g.d.flags, h->slot_top, hipMemcpyDeviceToHost));
  uint64_t k = 0;  // proxies stand for other shards' shadows
  for (uint8_t f : fl) k += (f & (FL_ALIVE | FL_PROXY)) == FL_ALIVE ? 1 : 0;
  *out = k;
  return CRGC_OK;
}

int crgc_export(crgc_graph *h, crgc_graph_export *out) {
  if (int rc = check_graph(h)) return rc;
  if (!out) return CRGC_E_INVAL;
  DeviceGuard dg(h->device);
  HIP_TRY(sync_counters(h));
  if (int rc = device_error(h)) return rc;
  const uint64_t top = h->slot_top;
  std::vector<uint64_t> vid(top);
  std::vector<int32_t> recv(top);
  std::vector<uint8_t> fl(top);
  std::vector<uint32_t> sup(top);
  std::vector<uint2> adj(top);
  std::vector<uint64_t> pool(h->pool_top);
  if (top) {
    HIP_TRY(hipMemcpy(vid.data(), h->g.d.vid, top * 8, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(recv.data(), h->g.d.recv, top * 4, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(fl.data(), h->g.d.flags, top, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(sup.data(), h->g.d.sup, top * 4, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(adj.data(), h->g.d.adj, top * 8, hipMemcpyDeviceToHost));
  }
  if (h->pool_top)
    HIP_TRY(hipMemcpy(pool.data(), h->g.d.pool, h->pool_top * 8, hipMemcpyDeviceToHost));
  // far ends in the proxy region (sharded graphs)
  const uint64_t pb = h->g.caps.pbase, ptop = h->proxy_top;
  std::vector<uint64_t> pvid(ptop);
  std::vector<uint8_t> pfl(ptop);
  if (ptop) {
    HIP_TRY(hipMemcpy(pvid.data(), h->g.d.vid + pb, ptop * 8, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(pfl.data(), h->g.d.flags + pb, ptop, hipMemcpyDeviceToHost));
  }
  // the actor id of an alive slot (a shadow or a proxy), or false
  auto alive_id = [&](uint32_t t, uint64_t *id) {
    if (t < top && (fl[t] & FL_ALIVE)) {
      *id = vid[t];
      return true;
    }
    if (t >= pb && t - pb < ptop && (pfl[t - pb] & FL_ALIVE)) {
      *id = pvid[t - pb];
      return true;
    }
    return false;
  };
  uint64_t nv = 0, ne = 0;
  bool big = false;
  for (uint64_t v = 0; v < top; ++v) {
    if ((fl[v] & (FL_ALIVE | FL_PROXY)) != FL_ALIVE) continue;  // this shard's shadows only
    if (out->id) {
      if (nv < out->vertex_cap) {
        out->id[nv] = vid[v];
        out->recv_count[nv] = recv[v];
        out->flags[nv] = fl[v] & (uint8_t)~FL_ALIVE;
        const uint32_t s = sup[v];
        uint64_t sid = CRGC_DEAD_ACTOR;
        if (s == SLOT_NONE) sid = CRGC_NO_ACTOR;
        else if (!alive_id(s, &sid)) sid = CRGC_DEAD_ACTOR;
        out->supervisor[nv] = sid;
      } else {
        big = true;
      }
    }
    ++nv;
    for (uint32_t e = 0; e < adj[v].y; ++e) {
      const uint64_t ed = pool[(uint64_t)adj[v].x + e];
      const uint32_t t = (uint32_t)ed;
      const int32_t cnt = (int32_t)(uint32_t)(ed >> 32);
      uint64_t tid;
      if (cnt == 0 || !alive_id(t, &tid)) continue;
      if (out->edge_owner) {
        if (ne < out->edge_cap) {
          out->edge_owner[ne] = vid[v];
          out->edge_target[ne] = tid;
          out->edge_count[ne] = cnt;
        } else {
          big = true;
        }
      }
      ++ne;
    }
  }
  out->n_vertices = nv;
  out->n_edges = ne;
  return big ? CRGC_E2BIG : CRGC_OK;
}

}  // extern "C"
