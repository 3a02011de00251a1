// crgc_internal.hpp — HBM layout of the shadow graph and the device helpers
// shared by the merge, trace and rebuild kernels (gfx950 / CDNA4 only).
//
// Layout (DESIGN.md "Data layout in HBM"):
//   id table   htab[{key u64, slot u32}] 16-B buckets, linear probing:
//                                      actor id -> dense vertex slot
//   vertex SoA, indexed by slot         (ShadowGraph.shadowMap + Shadow fields)
//     vid[u64]    actor id of the slot
//     recv[i32]   Shadow.recvCount
//     flags[u8]   ALIVE|INTERNED|LOCAL|BUSY|ROOT|HALTED
//     sup[u32]    Shadow.supervisor as a slot (NONE = null, DEAD = collected)
//     adj[uint2]  {offset, degree} of the slot's out-edge segment in the pool
//                 (capacity seg_cap(degree))
//   edge pool   pool[u64] = target slot (lo 32) | count (hi 32): Shadow.outgoing
//   edge table  etab[{key u64 = owner<<32|target, val u32 = index inside the
//               segment, rev u32 = index of its reverse candidate}] 16-B buckets
//   trace state vis bitmap + two frontier byte maps + two block-dirty maps
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <chrono>
#include <cstdlib>

namespace crgc {

// Host waits poll the stream (event) for up to `spin_us` before blocking in
// the runtime's synchronize: a blocking wait sleeps on the completion
// interrupt, and its wake-up cost ~1 ms per wait at C4 scale, where a
// 1e7-entry merge waits once per 2^20-entry sub-merge (profiles/r4o: the merge
// 15.8 ms against 5.8 ms of kernels).  A not-ready query leaves no sticky
// error (tools/hip_probe.hip).
// CRGC_SPIN_US (a production switch; read once per process)
// sets the bound: 0 blocks at once, which frees the waiting core (a JVM host with
// one thread per shard may prefer that over the ~1 ms later wake-up).
constexpr uint32_t SPIN_US_DEFAULT = 20000;
inline uint32_t spin_us_default() {
  static const uint32_t v = [] {
    const char *m = getenv("CRGC_SPIN_US");
    return m ? (uint32_t)strtoul(m, nullptr, 10) : SPIN_US_DEFAULT;
  }();
  return v;
}
inline hipError_t stream_wait(hipStream_t s, uint32_t spin_us = spin_us_default()) {
  if (spin_us) {
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
      const hipError_t e = hipStreamQuery(s);
      if (e != hipErrorNotReady) return e;
      if (std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(spin_us)) break;
    }
  }
  return hipStreamSynchronize(s);
}
inline hipError_t event_wait(hipEvent_t ev, uint32_t spin_us = spin_us_default()) {
  if (spin_us) {
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
      const hipError_t e = hipEventQuery(ev);
      if (e != hipErrorNotReady) return e;
      if (std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(spin_us)) break;
    }
  }
  return hipEventSynchronize(ev);
}

// Every launch_* helper reports hipGetLastError() after its launches.  The
// runtime keeps the last failing status of ANY call on the thread until it is
// read — soft failures included (a stream query's hipErrorNotReady, an event
// query, a pointer query on pageable memory; tools/hip_probe.hip,
// profiles/r4a/README.md) — so each helper first drops whatever an earlier
// call left behind and reports only its own launches.
inline void launch_begin() { (void)hipGetLastError(); }

// Where this thread's last failing API call went wrong: file:line and what
// failed (the HIP status name, device error flags, a transport step).  The
// first failure of a call wins; crgc_last_error_detail() returns it.
void note_error(const char *file, int line, const char *what);
#define DEV_FAIL(what) (note_error(__FILE__, __LINE__, (what)), CRGC_E_DEVICE)

constexpr uint64_t KEY_EMPTY = 0xFFFFFFFFFFFFFFFFull;
constexpr uint32_t PHS_NONE = 0xFFFFFFFFu;    // proxy's home slot not resolved yet
constexpr uint32_t PHS_ABSENT = 0xFFFFFFFEu;  // the home shard has no live shadow of the id
constexpr uint64_t KEY_TOMB = 0xFFFFFFFFFFFFFFFEull;
constexpr uint32_t SLOT_NONE = 0xFFFFFFFFu;  // Java null supervisor
constexpr uint32_t SLOT_DEAD = 0xFFFFFFFEu;  // supervisor collected (post-rebuild)
constexpr uint32_t VAL_PENDING = 0xFFFFFFFFu;
constexpr uint32_t RC_POS = 0x80000000u;     // reverse candidate: the edge's count is > 0

// flags bits: ALIVE is internal; the rest equal CRGC_F_* of include/crgc.h
constexpr uint8_t FL_ALIVE = 0x01, FL_INTERNED = 0x02, FL_LOCAL = 0x04, FL_BUSY = 0x08,
                  FL_ROOT = 0x10, FL_HALTED = 0x20;
// Sharded graphs only: a proxy slot stands for an actor whose home is another
// shard.  It carries the id (the edge / supervisor endpoint of a local owner)
// and nothing else: never a pseudo-root, never live or garbage, no out-edges.
constexpr uint8_t FL_PROXY = 0x40;
constexpr uint32_t MAX_SHARDS = 64;

// device error bits (Counters::err)
constexpr uint32_t ERR_RESERVED_ID = 1u << 0;
constexpr uint32_t ERR_TOO_MANY = 1u << 1;   // more than F records in an entry
constexpr uint32_t ERR_IDTAB_FULL = 1u << 2;
constexpr uint32_t ERR_SLOTS_FULL = 1u << 3;
constexpr uint32_t ERR_POOL_FULL = 1u << 4;
constexpr uint32_t ERR_ETAB_FULL = 1u << 5;
constexpr uint32_t ERR_UNDO_NEW = 1u << 6;
constexpr uint32_t ERR_SPIN = 1u << 7;
constexpr uint32_t ERR_BAD_OFFSETS = 1u << 8;
constexpr uint32_t ERR_QUEUE_FULL = 1u << 9;
constexpr uint32_t ERR_WALK_STUCK = 1u << 10;  // k_walk: a grid barrier wait ran out

constexpr int WAVE = 64;
constexpr int BLK_SLOTS = 2048;          // slots per wave-block (64 lanes x 32)
constexpr int LEVEL_RING = 4096;         // ring of per-level frontier counts
constexpr int STAT_WG = 2048;            // max workgroups of the level / sweep kernels
constexpr int TAIL_QCAP = 1 << 16;       // narrow-frontier queue capacity (per buffer)
constexpr unsigned long long TAIL_DONE = 1, TAIL_BAILED = 2, TAIL_CHAINS = 3;

struct Counters {
  unsigned long long inserted;       // vertices created (totalActorsSeen)
  unsigned long long slot_top;       // next dense slot
  unsigned long long pool_top;       // next free edge in pool
  unsigned long long rpool_top;      // next free reverse-candidate entry
  unsigned long long etab_used;      // edge-table keys ever inserted
  // Sharded graphs: proxy slots live in their own region, [pbase, pbase + proxy_top)
  // (DevGraph::pbase), so the per-slot passes over the shard's own shadows
  // (pseudo-roots, sweep, dense frontier scans) never read them.
  unsigned long long proxy_top;      // proxy slots allocated in this generation
  unsigned long long proxy_dead;     // ... of which invalidated (their home collected the actor)
  unsigned long long res_top;        // proxies below pbase + res_top have asked their homes (resolution)
  unsigned long long alive_cnt[2];   // a rebuild's kept shadows / proxies (k_rb_count_alive)
  // Slot reuse (unsharded graphs, crgc_reuse.hip): slots of collected shadows,
  // purged of their edges after the sweep, wait in DevGraph::freel[0 .. free_n)
  // for the next merges' new shadows, which take them in order (free_used).
  unsigned long long free_n;
  unsigned long long free_used;
  unsigned long long reused;         // slots taken from the list since the id table's last rehash
                                     // (their collected ids' tombstones load the table)
  // per-merge lists (reset together before every edge pipeline)
  unsigned long long err;
  unsigned long long spin_max;
  // trace
  unsigned long long marked;
  unsigned long long edges_scanned;
  unsigned long long sup_edges;
  unsigned long long expand_bytes;   // bytes k_expand read / wrote over the trace (summed by k_sweep_scan)
  unsigned long long mf_level;       // nonzero out-edges of the current level's expandable frontier
  unsigned long long mf_sum;         // ... summed over the levels so far (Beamer's explored edges)
  unsigned long long chain_marked;   // shadows marked by chain mode (crgc_chain.hip)
  unsigned long long chain_rounds;   // pointer-jumping rounds that marked something
  unsigned long long n_garbage;
  unsigned long long n_kill;
  unsigned long long n_live;
  unsigned long long npe;
  unsigned long long n_out;          // generic output counter (local roots)
  unsigned long long mark_done;      // set by k_tail at the first empty level (or its own finish):
                                     // the sweep kernels enqueued behind the level chunk run
  unsigned long long tail_state;     // narrow-frontier kernel: 0 idle, TAIL_DONE, TAIL_BAILED
  unsigned long long tail_level;     // DONE: levels traced; BAILED: level to resume at
  unsigned long long tail_from;      // level at which k_tail took over
  unsigned long long cb_level;       // a pull k_expand wrote level cb_level's candidates as bits (cb)
  unsigned long long cb_two;         // ... and the second half of k_bin_apply's bits is in cb2 (level 1)
  unsigned long long bin_ovf;        // k_bin_place stored a candidate byte at once (a full slice)
  unsigned long long pulled;         // bit L (L < 64): level L's k_expand pulled (the next trace's prediction)
  unsigned long long qn[2], qh[2];   // per-level edge-range queue lengths
  // sharded graphs
  unsigned long long n_req;          // kill requests (garbage with a remote supervisor)
  unsigned long long xcnt[MAX_SHARDS];  // ids to send per destination shard
  unsigned long long xpos[MAX_SHARDS];  // scatter cursors
  unsigned long long xcnt2[MAX_SHARDS]; // mark rounds: home slots to send per destination
  // k_walk (the multi-workgroup narrow-frontier walk): queue lengths by level
  // mod 3, claims and supervisor edges, and its grid barrier
  unsigned long long walk_n[3];
  unsigned long long walk_np[2];     // heavy shadows' edge pieces by level parity
  unsigned long long walk_claims, walk_sup;
  unsigned int walk_bar, walk_gen, walk_fail, walk_pad;
  unsigned long long ring[LEVEL_RING];
};

// Hash buckets: key and value share one 16-B line, so a probe is one load.
struct alignas(16) IdBucket {
  uint64_t key;  // actor id, KEY_EMPTY or KEY_TOMB
  uint32_t val;  // dense slot, VAL_PENDING while the inserting wave allocates it
  uint32_t pad;
};
struct alignas(16) EdgeBucket {
  uint64_t key;  // owner << 32 | target
  uint32_t val;  // entry index in the owner's segment
  uint32_t rev;  // entry index in the target's reverse-candidate segment (during a merge,
                 // 0x80000000 | reverse-atom position until it is appended)
};

__device__ inline uint64_t bucket_key(const uint4 &b) { return (uint64_t)b.x | ((uint64_t)b.y << 32); }
template <class B>
__device__ inline uint4 load_bucket(const B *p) { return *reinterpret_cast<const uint4 *>(p); }

// Everything a kernel needs, passed by value.
struct DevGraph {
  // id table
  uint64_t hcap, hmask;
  IdBucket *htab;
  // vertex SoA
  uint64_t scap;   // slot capacity (multiple of BLK_SLOTS)
  uint64_t pbase;  // first proxy slot (multiple of BLK_SLOTS): homes in [0, pbase), proxies in
                   // [pbase, scap); == scap for an unsharded graph (no proxy region)
  uint64_t *vid;
  int32_t *recv;
  uint8_t *flags;
  uint32_t *sup;
  uint2 *adj;                // {segment offset, degree}; the segment's capacity is seg_cap(degree)
  unsigned long long *vseq;  // last-write-wins tag for busy/root
  unsigned long long *sseq;  // last-write-wins tag for supervisor
  uint32_t *nzdeg;           // out-edges with count != 0 (reference `outgoing.size()`)
  // slot reuse (unsharded; nullptr when off): the free list, the next one being
  // built (ping-pong), and the committed sweeps' garbage slots not purged yet
  // (dense; a sweep appends its own from gslot_at)
  uint32_t *freel, *freel2, *gslot;
  uint64_t gslot_at;
  // reverse candidates (pull BFS): owners that ever created an edge key to the
  // slot; a candidate is verified against the forward count when used
  uint2 *radj;               // {offset, rlen | log2(capacity) << RLEN_BITS} into rpool (rseg_*)
  uint32_t *rnew;            // rebuild scratch: in-degree per target
  uint32_t *rpool;           // owner slot | RC_POS while count(owner -> slot) > 0
  uint32_t *par;             // pull hint per slot: an owner whose edge to it has a positive count
                             // (the candidate a pull level last found; cleared when that count
                             // stops being positive), or SLOT_NONE
  uint64_t rpcap;
  uint32_t *fx;              // expandable frontier bitmap (frontier & !halted)
  uint32_t *cb;              // candidates of the level after a pull level, 1 bit / slot (LV_CBITS)
  uint32_t *cb2;             // level 1: the second k_bin_apply workgroup of each bin's bits
  uint32_t *tq;              // narrow-frontier queues, 2 x TAIL_QCAP slots
  uint32_t *tl_buf;          // per-block regions: a listed level's frontier slots
  uint32_t *tl_tag;          // per block: (level+1) << 12 | listed slots
  // chain mode (crgc_chain.hip): zero outside it
  uint32_t *cm;              // bitmap: marked by chain mode, or handed to it unexpanded by k_tail
  uint32_t *pb[2];           // bitmaps: marked, not yet expanded, more than one traceable out-edge
  // edges
  uint64_t pcap;
  uint64_t *pool;
  uint64_t ecap_tab, emask;
  EdgeBucket *etab;
  // trace
  uint32_t *vis;
  uint8_t *front[2];
  uint8_t *dirty[2];
  uint2 *qn_buf;     // per-block regions of light edge ranges {offset, degree}
  uint32_t *qn_tag;   // per block: (level+1) << 12 | number of light ranges
  uint2 *qh_buf;      // RANGE_MAX-edge pieces of hub segments
  uint64_t qn_cap, qh_cap;
  uint64_t *blkstat;  // STAT_WG x 4 per-workgroup statistics partials
  uint64_t *xbytes;   // STAT_WG per-workgroup k_expand byte counts
  uint32_t *sweep_cnt;  // per block: garbage, kill counts
  uint64_t *sweep_off;  // per block: exclusive offsets of the above
  uint64_t *out_a;    // per-block regions: garbage slots (u32) / generic ids
  uint64_t *out_b;    // per-block regions: kill slots (u32)
  uint64_t *out_ids;  // dense garbage ids
  uint64_t *out_kill; // dense kill ids
  // sharded graphs (n_shards > 1)
  uint32_t n_shards, shard;
  uint32_t *xsent;    // 1 bit / slot (the proxy region's words): a marked proxy already exported
  uint8_t *xkey;      // 1 B / slot (proxies): the export key of a new mark (k_xscan)
  uint2 *wpc;         // k_walk: a level's heavy-shadow edge pieces {offset, length}
  uint64_t wpc_cap;   // TAIL_QCAP + pcap / WALK_PIECE: room for any level's pieces
  uint32_t *rq_buf;   // per-block regions: garbage slots whose kill waits on a remote mark
  uint32_t *rq_cnt;   // per block: listed requests
  uint32_t *phs;      // per proxy slot: its slot at the home shard (PHS_NONE / PHS_ABSENT)
  uint8_t *psh;       // per proxy slot: its home shard (the exchange lists read it, not the id)
  Counters *ctr;
};

// Segment capacities are powers of two >= 4 (0: no segment).  An owner's
// out-edge segment always has capacity seg_cap(degree): it grows to that when
// its degree passes the old capacity, a rebuild sizes it the same way, and the
// degree only grows in between — so no capacity array is read (one random line
// less per new edge in k_ep_owner).
__host__ __device__ inline uint32_t seg_cap(uint32_t deg) {
  if (deg == 0) return 0;
  uint32_t c = 4;
  while (c < deg) c <<= 1;
  return c;
}
// A reverse-candidate segment's length and capacity share radj[t].y, so the one
// returning 64-bit atomic that appends a candidate also tells whether it fits:
// length in the low RLEN_BITS bits (at most 2^27 - 1 candidates per shadow;
// more sets ERR_POOL_FULL), log2(capacity) above them (0: no segment).
constexpr uint32_t RLEN_BITS = 27;
constexpr uint32_t RLEN_MASK = (1u << RLEN_BITS) - 1;
__host__ __device__ inline uint32_t rseg_len(uint32_t y) { return y & RLEN_MASK; }
__host__ __device__ inline uint32_t rseg_cap(uint32_t y) {
  const uint32_t lc = y >> RLEN_BITS;
  return lc ? (1u << lc) : 0u;
}
__host__ __device__ inline uint32_t rseg_pack(uint32_t len, uint32_t cap) {
  return len | ((cap ? (uint32_t)__builtin_ctz(cap) : 0u) << RLEN_BITS);
}

// splitmix64 finaliser
__host__ __device__ inline uint64_t mix64(uint64_t x) {
  x ^= x >> 30;
  x *= 0xbf58476d1ce4e5b9ull;
  x ^= x >> 27;
  x *= 0x94d049bb133111ebull;
  x ^= x >> 31;
  return x;
}

// Home shard of an actor id.  Independent of the id-table hash (mix64(id) &
// mask): with a power-of-two shard count a shared hash would leave each
// shard's table using 1/G of its buckets.
__host__ __device__ inline uint32_t shard_of(uint64_t id, uint32_t n_shards) {
  const uint64_t h = mix64(id ^ 0x6a09e667f3bcc909ull);
  return (uint32_t)(((h >> 32) * (uint64_t)n_shards) >> 32);
}

__device__ inline bool is_home(const DevGraph &g, uint64_t id) {
  return g.n_shards <= 1 || shard_of(id, g.n_shards) == g.shard;
}

// Blocks of the slot space a per-block pass visits: the shadows' own blocks
// [0, nh) and, when `proxies`, the proxy region's [p0, p0 + np), as one run of
// virtual block numbers vb < n (at(vb) is the real block).
struct VBlocks {
  uint32_t nh, n, p0;
  __device__ uint32_t at(uint32_t vb) const { return vb < nh ? vb : p0 + (vb - nh); }
  __device__ bool proxy(uint32_t vb) const { return vb >= nh; }
};
__device__ inline VBlocks vblocks(const DevGraph &g, bool proxies) {
  const Counters *c = g.ctr;
  VBlocks b;
  b.nh = (uint32_t)((c->slot_top + BLK_SLOTS - 1) / BLK_SLOTS);
  const uint32_t np = proxies ? (uint32_t)((c->proxy_top + BLK_SLOTS - 1) / BLK_SLOTS) : 0u;
  b.n = b.nh + np;
  b.p0 = (uint32_t)(g.pbase / BLK_SLOTS);
  return b;
}
// One past the largest slot in use (homes, and the proxy region when it has any).
__device__ inline uint64_t slot_end(const DevGraph &g) {
  const Counters *c = g.ctr;
  return c->proxy_top ? g.pbase + c->proxy_top : c->slot_top;
}
// Virtual slot u of [0, slot_top + proxy_top) -> real slot.
__device__ inline uint64_t vslot(const DevGraph &g, uint64_t u, uint64_t nh) {
  return u < nh ? u : g.pbase + (u - nh);
}

__host__ __device__ inline bool reserved_id(uint64_t id) {
  return id >= KEY_TOMB || (id >> 48) == 0xFFFFull;
}

__device__ inline void set_err(Counters *c, uint32_t bit) {
  atomicOr(&c->err, (unsigned long long)bit);
}

__device__ inline int lane_id() { return threadIdx.x & 63; }
// Orders one wave's LDS writes before its later LDS reads.
__device__ inline void wave_lds_fence() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ inline uint64_t lanemask_lt() { return (1ull << lane_id()) - 1ull; }

// Full-wave inclusive scan (all 64 lanes must be active).
__device__ inline uint32_t wave_incl_scan(uint32_t x) {
  const int lane = lane_id();
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint32_t y = __shfl_up(x, d);
    if (lane >= d) x += y;
  }
  return x;
}

__device__ inline uint32_t wave_sum(uint32_t x) { return __shfl(wave_incl_scan(x), 63); }

__device__ inline uint32_t wave_max(uint32_t x) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) x = max(x, (uint32_t)__shfl_xor(x, d));
  return x;
}

// Wave-aggregated atomic add: one atomic per wave.  ALL 64 lanes must call
// (v = 0 to abstain).  Returns this lane's exclusive base.
__device__ inline unsigned long long wave_atomic_add(unsigned long long *p, uint32_t v) {
  const uint32_t incl = wave_incl_scan(v);
  const uint32_t total = __shfl(incl, 63);
  unsigned long long base = 0;
  if (lane_id() == 0 && total) base = atomicAdd(p, (unsigned long long)total);
  base = __shfl(base, 0);
  return base + (incl - v);
}

// Workgroup-aggregated appends to K counters: one atomic per counter per
// workgroup (a counter that every wave bumps saturates near 88 atomics/us).
// Every thread of the block must call it; v[k] is this thread's count for
// ctr[k], out[k] its exclusive base.  Up to 1024 threads.
template <int K>
__device__ inline void block_append(unsigned long long *const (&ctr)[K], const uint32_t (&v)[K],
                                    unsigned long long (&out)[K]) {
  __shared__ uint32_t s_wave[16][K];
  __shared__ unsigned long long s_base[K];
  const int w = threadIdx.x >> 6, nw = (int)(blockDim.x >> 6);
  uint32_t incl[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    incl[k] = wave_incl_scan(v[k]);
    if ((threadIdx.x & 63) == 63) s_wave[w][k] = incl[k];
  }
  __syncthreads();
  if (threadIdx.x < (unsigned)K) {
    const int k = threadIdx.x;
    uint32_t run = 0;
    for (int j = 0; j < nw; ++j) {
      const uint32_t t = s_wave[j][k];
      s_wave[j][k] = run;
      run += t;
    }
    s_base[k] = run ? atomicAdd(ctr[k], (unsigned long long)run) : 0ull;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < K; ++k) out[k] = s_base[k] + s_wave[w][k] + incl[k] - v[k];
  __syncthreads();
}

// Wave-aggregated 1-bit append: lanes with `pred` get consecutive indices.
__device__ inline unsigned long long wave_append(unsigned long long *p, bool pred) {
  const uint64_t ball = __ballot(pred);
  unsigned long long base = 0;
  if (lane_id() == 0 && ball) base = atomicAdd(p, (unsigned long long)__popcll(ball));
  base = __shfl(base, 0);
  return base + __popcll(ball & lanemask_lt());
}

// ---- id table --------------------------------------------------------------
// Resolving an id to its dense slot, inserting it if absent, is split in two
// so that slot allocation is one atomic per wave and no wave can deadlock:
//   id_probe   (divergent)  claims the key with a CAS or finds it;
//   id_settle  (ALL lanes)  the wave allocates slots for the keys it claimed,
//                           publishes them with memory-side atomic exchanges,
//                           and only then waits (memory-side atomic reads, so
//                           no stale per-XCD L2 line can satisfy the wait) for
//                           keys another wave claimed but has not published.
// Every wave publishes before it waits, so a wait always ends.
constexpr uint32_t SLOT_INVALID = 0xFFFFFFFDu;  // published on overflow
enum : int { RS_NONE = 0, RS_FOUND = 1, RS_INSERTED = 2, RS_PENDING = 3 };

__device__ inline int id_probe(const DevGraph &g, uint64_t id, uint64_t &bucket,
                               uint32_t &slot) {
  uint64_t h = mix64(id) & g.hmask;
  for (uint64_t probe = 0; probe < g.hcap; ++probe) {
    const uint4 b = load_bucket(&g.htab[h]);
    uint64_t k = bucket_key(b);
    uint32_t v = b.z;
    if (k == KEY_EMPTY) {
      k = atomicCAS((unsigned long long *)&g.htab[h].key, (unsigned long long)KEY_EMPTY,
                    (unsigned long long)id);
      if (k == KEY_EMPTY) {
        bucket = h;
        return RS_INSERTED;
      }
      v = g.htab[h].val;  // someone else's fresh key: its slot may still be pending
    }
    if (k == id) {
      bucket = h;
      if (v != VAL_PENDING) {
        slot = v;
        return RS_FOUND;
      }
      return RS_PENDING;
    }
    h = (h + 1) & g.hmask;
  }
  set_err(g.ctr, ERR_IDTAB_FULL);
  slot = SLOT_INVALID;
  return RS_FOUND;
}

// A new shadow's slot: homes from slot_top (below pbase), proxies from
// proxy_top (at pbase and above).  SLOT_INVALID (and ERR_SLOTS_FULL) past a region.
__device__ inline uint64_t region_slot(const DevGraph &g, bool home, unsigned long long k) {
  const uint64_t s = home ? k : g.pbase + k;
  return (home ? s < g.pbase : s < g.scap) ? s : ~0ull;
}

__device__ inline uint32_t id_settle(const DevGraph &g, uint64_t id, uint64_t bucket,
                                     uint32_t slot, int state) {
  const bool ins = state == RS_INSERTED;
  const bool home = ins && is_home(g, id);
  const unsigned long long kh = wave_append(&g.ctr->slot_top, home);
  const unsigned long long kp = wave_append(&g.ctr->proxy_top, ins && !home);
  const uint64_t s = ins ? region_slot(g, home, home ? kh : kp) : ~0ull;
  const uint64_t ball = __ballot(home);
  if (lane_id() == 0 && ball) atomicAdd(&g.ctr->inserted, (unsigned long long)__popcll(ball));
  if (ins) {
    if (s == ~0ull) {
      set_err(g.ctr, ERR_SLOTS_FULL);
      slot = SLOT_INVALID;
    } else {
      slot = (uint32_t)s;
      g.vid[s] = id;
      g.flags[s] = home ? FL_ALIVE : (FL_ALIVE | FL_PROXY);
      if (!home) g.psh[s] = (uint8_t)shard_of(id, g.n_shards);
    }
    atomicExch(&g.htab[bucket].val, slot);
  }
  if (state == RS_PENDING) {
    slot = SLOT_INVALID;
    for (uint32_t spin = 0; spin < (1u << 24); ++spin) {
      uint32_t v = atomicOr(&g.htab[bucket].val, 0u);
      if (v != VAL_PENDING) {
        slot = v;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    if (slot == SLOT_INVALID) set_err(g.ctr, ERR_SPIN);
  }
  return state == RS_NONE ? SLOT_INVALID : slot;
}

// Workgroup form of id_settle: one slot_top / inserted atomic per workgroup.
// Every thread of the block must call it; every thread publishes its claims
// before any waits, so the protocol above still cannot deadlock.
__device__ inline uint32_t id_settle_block(const DevGraph &g, uint64_t id, uint64_t bucket,
                                           uint32_t slot, int state) {
  const bool ins = state == RS_INSERTED;
  const bool home = ins && is_home(g, id);
  unsigned long long *const ctrs[3] = {&g.ctr->slot_top, &g.ctr->proxy_top, &g.ctr->inserted};
  const uint32_t v[3] = {home ? 1u : 0u, ins && !home ? 1u : 0u, home ? 1u : 0u};
  unsigned long long base[3];
  block_append<3>(ctrs, v, base);
  if (ins) {
    const uint64_t s = region_slot(g, home, home ? base[0] : base[1]);
    if (s == ~0ull) {
      set_err(g.ctr, ERR_SLOTS_FULL);
      slot = SLOT_INVALID;
    } else {
      slot = (uint32_t)s;
      g.vid[s] = id;
      g.flags[s] = home ? FL_ALIVE : (FL_ALIVE | FL_PROXY);
      if (!home) g.psh[s] = (uint8_t)shard_of(id, g.n_shards);
    }
    atomicExch(&g.htab[bucket].val, slot);
  }
  if (state == RS_PENDING) {
    slot = SLOT_INVALID;
    for (uint32_t spin = 0; spin < (1u << 24); ++spin) {
      uint32_t v2 = atomicOr(&g.htab[bucket].val, 0u);
      if (v2 != VAL_PENDING) {
        slot = v2;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    if (slot == SLOT_INVALID) set_err(g.ctr, ERR_SPIN);
  }
  return state == RS_NONE ? SLOT_INVALID : slot;
}

// Uniform helper: every lane calls; lanes with !has get SLOT_INVALID.
__device__ inline uint32_t id_resolve(const DevGraph &g, bool has, uint64_t id) {
  uint64_t bucket = 0;
  uint32_t slot = SLOT_INVALID;
  int st = RS_NONE;
  if (has) st = id_probe(g, id, bucket, slot);
  return id_settle(g, id, bucket, slot, st);
}

// Lookup without insertion (tombstones are skipped, EMPTY ends the chain).
__device__ inline uint32_t id_find(const DevGraph &g, uint64_t id, uint64_t *bucket = nullptr) {
  uint64_t h = mix64(id) & g.hmask;
  for (uint64_t probe = 0; probe < g.hcap; ++probe) {
    const uint4 b = load_bucket(&g.htab[h]);
    const uint64_t k = bucket_key(b);
    if (k == id) {
      if (bucket) *bucket = h;
      return b.z;
    }
    if (k == KEY_EMPTY) return SLOT_NONE;
    h = (h + 1) & g.hmask;
  }
  return SLOT_NONE;
}

// ---- edge table ------------------------------------------------------------
__device__ inline uint64_t edge_key(uint32_t owner, uint32_t target) {
  return ((uint64_t)owner << 32) | target;
}

// Returns the bucket of `key`; *inserted tells whether this thread created it,
// *val / *rev are the bucket's value and reverse index as loaded.
__device__ inline uint64_t edge_find_or_insert(const DevGraph &g, uint64_t key, bool *inserted,
                                               uint32_t *val, uint32_t *rev = nullptr) {
  uint64_t h = mix64(key) & g.emask;
  *inserted = false;
  for (uint64_t probe = 0; probe < g.ecap_tab; ++probe) {
    const uint4 b = load_bucket(&g.etab[h]);
    uint64_t k = bucket_key(b);
    *val = b.z;
    if (rev) *rev = b.w;
    if (k == KEY_EMPTY) {
      k = atomicCAS((unsigned long long *)&g.etab[h].key, (unsigned long long)KEY_EMPTY,
                    (unsigned long long)key);
      if (k == KEY_EMPTY) {
        *inserted = true;
        return h;
      }
      *val = g.etab[h].val;
      if (rev) *rev = g.etab[h].rev;
    }
    if (k == key) return h;
    h = (h + 1) & g.emask;
  }
  set_err(g.ctr, ERR_ETAB_FULL);
  return KEY_EMPTY;
}

// Lookup only: the entry offset of edge (owner -> target) in owner's segment,
// or SLOT_NONE when the key was never created.
__device__ inline uint32_t edge_find(const DevGraph &g, uint32_t owner, uint32_t target) {
  const uint64_t key = edge_key(owner, target);
  uint64_t h = mix64(key) & g.emask;
  for (uint64_t probe = 0; probe < g.ecap_tab; ++probe) {
    const uint4 b = load_bucket(&g.etab[h]);
    const uint64_t k = bucket_key(b);
    if (k == key) return b.z;
    if (k == KEY_EMPTY) break;
    h = (h + 1) & g.emask;
  }
  return SLOT_NONE;
}

__device__ inline uint64_t pack_edge(uint32_t target, int32_t count) {
  return ((uint64_t)(uint32_t)count << 32) | target;
}
__device__ inline uint32_t edge_target(uint64_t e) { return (uint32_t)e; }
__device__ inline int32_t edge_count(uint64_t e) { return (int32_t)(uint32_t)(e >> 32); }
__device__ inline int32_t *edge_count_ptr(uint64_t *pool, uint64_t i) {
  return reinterpret_cast<int32_t *>(pool + i) + 1;
}

// RefobInfo.count / isActive (RefobInfo.java:23-29)
__device__ inline int32_t refob_count(int16_t info) { return (int16_t)(((int32_t)info) >> 1); }
__device__ inline bool refob_deactivated(int16_t info) { return (info & 1) != 0; }

}  // namespace crgc
