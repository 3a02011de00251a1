// crgc_host.hpp — host-side state of one shadow-graph handle and the kernel
// launchers each .hip translation unit provides.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#include "../../include/crgc.h"
#include "crgc_internal.hpp"

namespace crgc {

// A grow-only device scratch buffer.
struct Scratch {
  void *ptr = nullptr;
  size_t bytes = 0;
  hipError_t ensure(size_t need) {
    if (need <= bytes) return hipSuccess;
    if (ptr) hipFree(ptr);
    ptr = nullptr;
    bytes = 0;
    size_t sz = need + need / 4 + 4096;
    hipError_t e = hipMalloc(&ptr, sz);
    if (e == hipSuccess) bytes = sz;
    return e;
  }
  void release() {
    if (ptr) hipFree(ptr);
    ptr = nullptr;
    bytes = 0;
  }
};

// Carves aligned sub-buffers out of a Scratch.
struct Carver {
  char *base;
  size_t off = 0;
  explicit Carver(void *p) : base((char *)p) {}
  template <class T>
  T *take(size_t n) {
    off = (off + 255) & ~(size_t)255;
    T *p = (T *)(base + off);
    off += n * sizeof(T);
    return p;
  }
  static size_t need(std::initializer_list<size_t> sizes) {
    size_t o = 0;
    for (size_t s : sizes) o = ((o + 255) & ~(size_t)255) + s;
    return o + 256;
  }
};

// Flattened id resolution (k_ids): up to 5 segments of ids, one slot each.
struct IdSeg {
  const uint64_t *ids;
  uint32_t *slots;
  uint64_t n;              // bound (grid sizing)
  const uint32_t *n_dev;   // exact count on the device (an offsets array's last entry), or null
  bool none_ok;            // CRGC_NO_ACTOR means "none" here (SLOT_INVALID, no error)
  // Sharded graphs: an id is resolved on this shard when it is home here, or
  // when partner[r] (an aligned id, CRGC_NO_ACTOR = none) is home here (the
  // id is then the far end of a local edge / supervisor: a proxy), or when
  // need[r] is set.  Both null: home only.
  const uint64_t *partner;
  const uint8_t *need;
};
struct IdArgs {
  IdSeg seg[5];
  int nseg;
};
hipError_t launch_ids(const DevGraph &g, const IdArgs &a, hipStream_t s);

struct EntryArgs {
  uint64_t n;
  uint32_t F;
  unsigned long long epoch;
  const uint64_t *self;
  const int16_t *recv;
  const uint8_t *flags;
  const uint32_t *c_off;
  const uint64_t *c_owner;
  const uint64_t *c_target;
  const uint32_t *s_off;
  const uint64_t *spawned;
  const uint32_t *u_off;
  const uint64_t *u_ref;
  const int16_t *u_info;
  uint32_t *self_slot;   // [n]
  uint32_t *spawn_slot;  // [n*F]
  uint32_t *ct_slot;     // [n*F] created targets, resolved by k_ids
  uint32_t *co_slot;     // [n*F] created owners
  uint32_t *u_slot;      // [n*F] updated refs
  uint64_t *n_atoms;     // out: C + U, the atoms k_entries_apply wrote (exact edge-pipeline count)
  // last-write-wins conflicts, per block of 256 entries (k_entries_vertex -> k_entries_lww)
  uint32_t *conf_v;      // [n rounded to 256] slots whose busy/root several entries tagged
  uint32_t *conf_s;      // [same * F] children whose supervisor several entries tagged
  uint32_t *conf_n;      // [2 * blocks] counts: self slots, spawned children
  uint32_t *atom_o;      // [2*n*F]: created atoms, then updated atoms
  uint32_t *atom_t;
  int32_t *atom_d;
  // sharded graphs: filled by k_entries_shard_prep
  uint8_t *self_need;    // [n]   self is home here or supervises a child homed here
  uint64_t *u_partner;   // [n*F] self for a deactivating update, else CRGC_NO_ACTOR
};

struct DeltaArgs {
  uint64_t n, nout;
  unsigned long long epoch;
  const uint64_t *id;
  const int32_t *recv;
  const uint64_t *sup;
  const uint8_t *flags;
  const uint32_t *out_off;
  const uint64_t *out_target;
  const int32_t *out_count;
  uint32_t *self_slot;
  uint32_t *sup_slot;
  uint32_t *ot_slot;     // [nout] outgoing targets, resolved by k_ids
  uint32_t *atom_o;
  uint32_t *atom_t;
  int32_t *atom_d;
  uint64_t *o_partner;   // sharded graphs: [nout] owning delta shadow of each outgoing entry
};

struct UndoArgs {
  uint64_t n, nc;
  uint16_t location;
  const uint64_t *actor;
  const int32_t *msg;
  const uint32_t *c_off;
  const uint64_t *c_target;
  const int32_t *c_count;
  const uint64_t *c_actor;  // [nc] the admitted actor each created-ref entry belongs to
  uint8_t *exists;          // [n + nc] existence of each actor / target at its home shard
  uint32_t *atom_o;
  uint32_t *atom_t;
  int32_t *atom_d;
};

struct EdgeArgs {
  const unsigned long long *err;  // the graph's error word: a batch refused for its offsets has no atoms
  uint64_t max_atoms;          // grid bound
  const uint64_t *n_atoms_dev; // exact count on device (or null: use max_atoms)
  const uint32_t *atom_o;
  const uint32_t *atom_t;
  const int32_t *atom_d;
  // partition (crgc_edges.hip): nbk = 2^(32 - bshift) buckets, nblk blocks of atoms
  uint32_t bshift, nbk;
  uint64_t nblk;
  uint32_t *hist;            // [nbk * nblk] bucket-major block counts
  uint64_t *hoff;            // [nbk * nblk] their exclusive scan
  uint64_t *bsum;            // scan scratch
  unsigned long long *tot;   // [2] atoms in the forward / reverse partition
  uint64_t *pk;              // [max_atoms] partitioned keys
  uint32_t *pv;              // [max_atoms] partitioned deltas / edge-table buckets
  // [max_atoms] reverse candidates past their target segment's capacity:
  // target, index, owner | RC_POS, edge-table bucket; *n_ov of them
  uint32_t *rv_t, *rv_i, *rv_o, *rv_b;
  unsigned long long *n_ov;
};

constexpr uint32_t LV_PULL = 4;                // dense levels scan in-candidates (pull)
constexpr uint32_t LV_TAIL = 8;                // narrow frontiers go to one workgroup (k_tail)
constexpr uint32_t LV_INVESTIGATE = 16;        // set by launch_level: no supervisor edges
constexpr uint32_t LV_ROOTS = 32;              // set by launch_level: the pseudo-root level
constexpr uint32_t LV_WALK = 64;               // narrow frontiers go to WALK_WG workgroups (k_walk)
constexpr uint32_t LV_CBITS = 128;             // a pull level hands the next level its candidates as bits (cb)
constexpr uint32_t LV_SUPBIN = 512;            // the binned pseudo-root level's supervisor pushes go through the bins
constexpr uint32_t LV_ROOTS_CO = 256;          // the pseudo-root pass reads receive counts lane-interleaved
constexpr uint32_t LV_NOBYTES = 1024;          // an untimed level expand: its bytes stay out of the roofline

struct LevelArgs {
  int level;
  uint32_t sparse_thresh;
  uint64_t pull_thresh;    // pull_div == 0: a level pulls after a frontier of >= this many shadows
  uint32_t pull_div;       // else: after a frontier of >= slot_top / pull_div shadows
  uint32_t tail_start;     // k_tail takes over after a level of <= this many shadows
  uint32_t tail_max;       // ... whose candidates number <= this, and bails above it
  uint32_t tail_edge_max;  // ... and whose frontier has <= this many out-edges; a later round of the
                           // walk with more bails too (one workgroup's global claims: ~1 G edges/s); 0: no bound
  uint32_t frontier_grid;  // workgroups of k_frontier (set by launch_level)
  uint32_t flags;          // LV_*
  uint32_t pull_cur_div;   // alpha == 0: k_expand also pulls once the current frontier is >= slot_top / div
  uint32_t alpha;          // Beamer: pull when alpha * m_f > m_u (0: the pull_cur_div rule)
  uint64_t e_total;        // edge keys in the graph (m_u = e_total - explored edges)
  uint32_t chain_after;    // k_tail hands a deep mark to chain mode after this many rounds (0: never)
  uint32_t xslices;        // push levels: 1, 2, 4 or 8 target slices (k_expand: XCD-local candidate stores)
  uint16_t location;
  // the pseudo-root level's binned push (k_bin_place, k_bin_apply), nbins == 0: off
  uint32_t *bins;          // the targets: slice (bin b, workgroup w) at [(b * bin_grid + w) * bin_slice, + bin_slice)
  uint32_t *bin_cnt;       // [nbins x bin_grid] targets in each slice, bin-major (place pass)
  uint32_t *bin_mode_w;    // [1] the binned-mode word (written by the place pass, read by k_bin_apply)
  uint32_t bin_slice;      // entries of a slice (a multiple of 4; targets past it are stored as bytes at once)
  uint32_t bin_shift;      // a bin covers slots [b << bin_shift, (b + 1) << bin_shift)
  uint32_t nbins;
  uint32_t bin_grid;       // workgroups of the place pass
  uint64_t pull_pred;      // bit L: level L pulled in the previous trace, so it pulls again (lists skipped)
};
constexpr uint32_t BIN_WG = 512;     // k_bin_place workgroups (16 waves each)
constexpr uint32_t BIN_MAX = 512;    // bins at most (one LDS counter and table word each)
constexpr uint32_t BIN_MAX_WIDE = 256;  // ... when a bin spans more than 2^16 slots

// Chain mode (crgc_chain.hip).
struct ChainArgs {
  uint32_t *nx0, *sp0;        // per slot: unique out-target / supervisor (CH_NONE, CH_COMPLEX)
  uint32_t *cx;               // bitmap: more than one out-target
  uint32_t *pb_in, *pb_out;   // pending complex shadows: this iteration's / the next one's
  uint32_t *flag;             // per round / expansion: marked something
  unsigned long long *n_new;  // shadows marked by chain mode
  int investigate;
};
// step 0 init, 1 jump round (src -> dst, flag fi, first of its sequence), 2 expand
// (flag fi), 3 statistics, 4 done (rounds that marked something)
hipError_t launch_chain(const DevGraph &g, const ChainArgs &ca, int step, const uint32_t *src, uint32_t *dst,
                        uint64_t top, uint32_t fi, int first, uint32_t rounds, hipStream_t s);

// ---- launchers (return hipError_t of the launch) ---------------------------
// phase 0: ids and edge atoms (the edge pipeline may start behind it); 1: vertex updates
hipError_t launch_entries(const DevGraph &g, const EntryArgs &a, hipStream_t s, int phase);
hipError_t launch_deltas(const DevGraph &g, const DeltaArgs &a, uint64_t n_out, hipStream_t s, int phase);
// the offsets of a chunk of a host batch, rebased to its first entry
// byte ranges from device-visible host memory into HBM (k_copy_ranges)
struct HostCopy {
  const char *src[11];
  char *dst[11];
  uint64_t bytes[11];
  int n;
};
hipError_t launch_copy_ranges(const HostCopy &c, hipStream_t s);
hipError_t launch_bounds(const uint32_t *c_off, const uint32_t *s_off, const uint32_t *u_off, uint64_t n,
                         uint64_t ch, uint64_t k, uint32_t *out, hipStream_t s);
hipError_t launch_rebase_copy(const uint32_t *c_src, const uint32_t *s_src, const uint32_t *u_src, uint32_t *c_off,
                              uint32_t *s_off, uint32_t *u_off, uint64_t n, uint32_t c0, uint32_t s0, uint32_t u0,
                              hipStream_t s);
hipError_t launch_rebase(uint32_t *c_off, uint32_t *s_off, uint32_t *u_off, uint64_t n, uint32_t c0, uint32_t s0,
                         uint32_t u0, hipStream_t s);
hipError_t launch_undo_check(const DevGraph &g, const UndoArgs &a, hipStream_t s);
hipError_t launch_undo_apply(const DevGraph &g, const UndoArgs &a, uint64_t slot_top,
                             hipStream_t s);
hipError_t launch_edges(const DevGraph &g, const EdgeArgs &a, hipStream_t s);

// ev: null, or 6 events: start / stop of k_frontier, k_tail, k_expand
hipError_t launch_level(const DevGraph &g, const LevelArgs &a, bool roots, bool investigate,
                        uint64_t slot_top, hipStream_t s, hipEvent_t *ev = nullptr);
// nh blocks of the shadows' own slots and np of the proxy region
hipError_t launch_trace_reset(const DevGraph &g, uint64_t nh, uint64_t np, uint32_t ctr_from, uint32_t ctr_words,
                              hipStream_t s);
// The caller's device-writable host buffers for the garbage / kill ids (page-
// locked or registered; null: none), filled by k_sweep_gather beside out_ids /
// out_kill when the lists fit and no NPE was seen.
struct HostLists {
  uint64_t *g = nullptr, *k = nullptr;
  uint64_t gcap = 0, kcap = 0;
};
// sweep + id compaction + removal of the garbage (skipped on a reference NPE)
// phase 1: classify + counts (k_sweep, k_sweep_scan); phase 2: ids + commit
// (k_sweep_gather); 3: both
hipError_t launch_sweep(const DevGraph &g, int should_kill, uint64_t slot_top, hipStream_t s,
                        int phase = 3, const HostLists &hl = HostLists{});
int level_grid(uint64_t slot_top);
bool walk_fits(int device);
hipError_t launch_publish(const Counters *c, Counters *hdst, uint32_t r0, uint32_t rn, hipStream_t s);
hipError_t launch_copy_lists(const DevGraph &g, uint64_t *gdst, uint64_t gcap, uint64_t *kdst, uint64_t kcap,
                             hipStream_t s);
// sharded graphs
hipError_t launch_list(const DevGraph &g, int mode, bool scatter, uint32_t *buf, uint32_t *cnt,
                       uint64_t nblk, uint64_t *send, uint32_t *send_slot, hipStream_t s);
// mark rounds in home-slot form: what this shard sends each destination
// (byte offsets into the send buffer; bitmap[d]: a bitmap over d's slots in
// place of a slot list) and what it received from each source
struct XSend {
  uint64_t id_off[MAX_SHARDS], sl_off[MAX_SHARDS];
  uint8_t bitmap[MAX_SHARDS];
  int use_slots;
  uint32_t xq;  // k_xscan's units per 2048-proxy block (1, 2, 4 or 8; a wave each)
  // every shard's marked bitmap of its own shadows, as of this round's
  // exchange (word offsets per shard, G + 1 of them; null: none): a proxy
  // whose home slot is marked there is not sent
  const uint32_t *gvis;
  uint64_t gvis_off[MAX_SHARDS + 1];
};
struct XRecv {
  uint32_t G;
  uint64_t off[MAX_SHARDS];        // the source's segment in the receive buffer
  uint64_t n_id[MAX_SHARDS];       // its ids, then u32 slots or bitmap words
  uint64_t start[MAX_SHARDS + 1];  // work items before each source (ids + slots / words)
  uint8_t bitmap[MAX_SHARDS];
};
// (nblk: a bound of the proxy region's blocks, for the grid)
hipError_t launch_xlist(const DevGraph &g, bool scatter, uint64_t nblk, char *send, const XSend &x,
                        uint32_t *wgc, hipStream_t s);
int xscan_grid(uint64_t nblk, uint32_t xq);  // k_xscan's workgroups (the counts `wgc` holds: 2 G u32 each)
// The replicated chain closure of deep sharded marks (crgc_xchain.hip).
struct XcArgs {
  uint32_t G, me;
  int investigate;
  uint64_t off[MAX_SHARDS + 1];  // first global index of each shard's slots (multiples of 64)
  uint64_t N, P_me;              // global indices; this shard's (padded) slot range
  uint32_t *lnx, *lsp;           // [P_me] this shard's block: successor, supervisor (global)
  uint32_t *lvis, *lcx, *lpb;    // [P_me / 32] marked / branching / pending bits of the block
  uint32_t *seed;                // [P_me / 32] marks imported this round (not yet expanded)
  uint32_t *gnx, *gsp;           // [N] all shards' blocks
  uint32_t *gvis, *gcx, *gpb_in, *gpb_out;  // [N / 32]
  uint32_t *flag;                // [0] a proxy without a home slot; jump / apply flags after it
  uint32_t *xl;                  // [N] shadows this shard's expansions marked
  unsigned long long *xl_n;
};
// step 0 import (p0 = receive buffer, p1 = XRecv*), 1 local block, 2 jump
// (p0 -> p1, flag fi, first of its sequence), 3 expand, 4 apply (p0 = list of
// n), 5 finish
hipError_t launch_xclosure(const DevGraph &g, const XcArgs &x, int step, const void *p0, uint32_t *p1, uint64_t n,
                           uint32_t fi, int first, hipStream_t s);
hipError_t launch_ximport(const DevGraph &g, const char *recv, const XRecv &x, int level, hipStream_t s);
hipError_t launch_round_start(Counters *c, int level, bool fresh, hipStream_t s);
// n words from p zeroed by one dispatch (a small hipMemsetAsync is up to three
// fill kernels, ~3.6 us each, several per sharded mark round: profiles/r6y)
hipError_t launch_zero_u64(void *p, uint32_t n, hipStream_t s);
// home-slot resolution: 0 reset(mask), 1 count unresolved, 2 list them (ids, slots),
// 3 answer asked ids (at the home), 4 store the answers, 5 every proxy so far has asked
// (n_proxy: a bound of the proxy slots, for the grids)
hipError_t launch_resolve(const DevGraph &g, int step, uint64_t mask, uint64_t *send, uint32_t *slots,
                          const uint64_t *ids, uint64_t n, uint32_t *ans, uint64_t n_proxy, hipStream_t s);
hipError_t launch_requests(const DevGraph &g, int phase, const uint64_t *ids, uint64_t n, uint8_t *ans,
                           const uint32_t *slots, hipStream_t s);
hipError_t launch_invalidate(const DevGraph &g, const uint64_t *ids, uint64_t n, hipStream_t s);
hipError_t launch_count_marked(const DevGraph &g, uint64_t slot_top, hipStream_t s);
hipError_t launch_local_roots(const DevGraph &g, uint64_t slot_top, hipStream_t s);

// rebuild: compact `src` (live vertices only, purged edges) into `dst`,
// whose arrays are freshly allocated and initialised by init_graph_arrays.
hipError_t launch_init_arrays(const DevGraph &g, hipStream_t s);
// (src_top / src_ptop: the source's shadow and proxy slot counts; out[0] / out[1]
// the alive ones of each; map: src.scap + 1 entries, by source slot)
hipError_t launch_count_alive(const DevGraph &src, uint64_t src_top, uint64_t src_ptop, unsigned long long *out,
                              hipStream_t s);
hipError_t launch_rebuild(const DevGraph &src, uint64_t src_top, uint64_t src_ptop, const DevGraph &dst, uint32_t *map,
                          uint64_t *offs, void *scan_tmp, hipStream_t s);
size_t rebuild_scan_tmp_bytes(uint64_t n);
// grow: both hash tables of `src` re-hashed into `dst`'s (larger) ones; the
// caller copies the per-slot arrays and the pools (same slots, same offsets)
hipError_t launch_grow_tables(const DevGraph &src, const DevGraph &dst, hipStream_t s);
// crgc_reuse.hip: after a committed sweep, purge the listed garbage slots
// gslot[0, n_purge) and list them free for the next merges (unsharded graphs;
// no-op without a free list); sup_fix: some live shadow may be halted
hipError_t launch_reclaim(const DevGraph &g, uint64_t slot_top, uint64_t n_purge, uint64_t n_free,
                          bool sup_fix, hipStream_t s);
// the pools alone, packed into pool2 / rpool2 (pp / rp: scap u64 each; scan_tmp:
// 2 x rebuild_scan_tmp_bytes(scap)); slots and tables unchanged
hipError_t launch_repack(const DevGraph &g, uint64_t top, uint64_t ptop, uint64_t *pp, uint64_t *rp, void *scan_tmp,
                         uint64_t *pool2, uint32_t *rpool2, hipStream_t s);

// routed sharded entry merges (crgc_route.hip)
constexpr int RT_THREADS = 256;
constexpr uint32_t ROUTE_MAX_SHARDS = 16;  // above: the all-gather form
constexpr uint32_t ROUTE_MAX_F = 255;      // per-block counts packed in 16 bits
constexpr size_t ROUTE_TABLE_BYTES = 8192; // pinned RoutePart[16] at 0, ConcatPart[16] at 4096

struct RouteArgs {
  uint64_t n, nblk;
  uint32_t G, F;
  uint64_t C, S, U;  // record counts of the batch (offset bounds)
  const uint64_t *self;
  const int16_t *recv;
  const uint8_t *flags;
  const uint32_t *c_off;
  const uint64_t *c_owner;
  const uint64_t *c_target;
  const uint32_t *s_off;
  const uint64_t *spawned;
  const uint32_t *u_off;
  const uint64_t *u_ref;
  const int16_t *u_info;
  unsigned long long *err;  // malformed offsets (set by k_route_count)
  uint64_t *blk_tot;        // [G * nblk] packed per-block counts
  uint64_t *blk_pre;        // [G * nblk * 4] exclusive block prefixes
  uint64_t *totals;         // [G * 4] entries, created, spawned, updated per destination
};

// One destination's part: an entry batch in device memory.
struct RoutePart {
  uint64_t *self;
  int16_t *recv;
  uint8_t *flags;
  uint32_t *c_off;
  uint64_t *c_owner;
  uint64_t *c_target;
  uint32_t *s_off;
  uint64_t *spawned;
  uint32_t *u_off;
  uint64_t *u_ref;
  int16_t *u_info;
};

// One received part (entry_layout offsets from base) and where it lands in
// the concatenated batch.
struct ConcatPart {
  const char *base;
  uint64_t off[11];
  uint64_t pn, pC, pS, pU;
};

// phase 0: k_route_count + k_route_scan; phase 1: k_route_scatter (parts on the device)
hipError_t launch_route(const RouteArgs &a, int phase, const RoutePart *parts, hipStream_t s);
hipError_t launch_concat(const ConcatPart *parts, uint32_t G, const RoutePart &dst, uint64_t N, uint64_t C,
                         uint64_t S, uint64_t U, hipStream_t s);

// Exclusive scans of up to 4 u32 arrays of n elements (two levels of 1024,
// crgc_delta.hip): out[j][i] = sum of in[j][0..i), *total[j] = the sum.
struct ScanSet {
  const uint32_t *in[4];
  uint64_t *out[4];
  unsigned long long *total[4];
  int k;
  uint64_t n, nb;
  uint64_t *bsum;  // [4 * ceil(n / 1024)] scratch
};
hipError_t run_scan(ScanSet q, hipStream_t s);

// device DeltaGraph production (crgc_delta.hip)
constexpr uint32_t DG_MAX = 64;         // delta_graph_size bound: per-thread state in LDS

struct DgCounters {
  unsigned long long err;       // malformed offsets / reserved ids
  unsigned int first_long;      // first graph start whose span was deferred (~0: none)
  unsigned int n_long;
  unsigned int walk_from;       // where the chain walk (re)starts: 0, then past a resolved deferred start
  unsigned int pad;
  unsigned long long n_graphs;  // graph starts (exclusive-scan total)
  unsigned long long n_shadows, n_out, wire;  // totals of the per-graph scans
  unsigned long long overflow;  // a write pass on the device's count found the outputs too small
  unsigned long long t_shadows, t_out, t_wire;  // totals of the per-graph slot bounds
};

struct DgArgs {
  uint64_t n;
  uint32_t F, DGS, T;  // T: a graph is full once it holds T shadows (isFull, :174-180)
  uint64_t C, S, U;
  const uint64_t *self;
  const int16_t *recv;
  const uint8_t *flags;
  const uint32_t *c_off;
  const uint64_t *c_owner;
  const uint64_t *c_target;
  const uint32_t *s_off;
  const uint64_t *spawned;
  const uint32_t *u_off;
  const uint64_t *u_ref;
  const int16_t *u_info;
  DgCounters *ctr;
  uint32_t *J;         // [2][n+1] successor graph start J, then J^64 (k_dg_jump)
  uint8_t *mark;       // [n+1] graph starts
  uint8_t *lng;        // [n+1] span deferred to k_dg_long
  uint32_t *blk;       // [nblk] marked starts per 1024 entries
  uint64_t *blk_off;   // [nblk]
  uint64_t *bsum;      // [4 * ceil(n / 1024)] block sums of the scans
  uint32_t *starts;    // [n_graphs+1]
  // per graph: sizes from the count pass, exclusive scans for the write pass
  uint32_t *g_size, *g_nout, *g_bytes;
  uint64_t *g_shadow, *g_out, *g_wire;
  // per graph: slot bounds of the write pass and their exclusive scans
  uint32_t *b_size, *b_out, *b_bytes;
  uint64_t *t_shadow, *t_out, *t_wire;
};

struct DgOut {
  uint32_t *graph_off;
  uint64_t *wire_off;
  uint64_t *id;
  int32_t *recv;
  uint64_t *sup;
  uint8_t *flags;
  uint32_t *out_off;
  uint64_t *out_target;
  int32_t *out_count;
  uint8_t *wire;
  // capacities, checked on the device when the pass runs on the device's count
  uint64_t graph_cap, shadow_cap, out_cap, wire_cap;
};

// phase 0: spans + doubling + chain from entry 0; 1: chain from a resolved
// deferred start (k_dg_long, then marking); 2: compaction of the starts.
hipError_t launch_dg_chain(const DgArgs &a, int phase, hipStream_t s);
// The write pass (one wave per graph) into bounded per-graph slots of t,
// recording each graph's exact sizes, and their exclusive scans (n_graphs ==
// DG_NG_DEVICE: the count on the device, bounded by n + 1)
constexpr uint64_t DG_NG_DEVICE = ~0ull;
hipError_t launch_dg_write(const DgArgs &a, uint64_t n_graphs, const DgOut &t, hipStream_t s);
// exclusive scans of the per-graph sizes
hipError_t launch_dg_scans(const DgArgs &a, uint64_t n_graphs, hipStream_t s);
// the slots of t packed into o at the exact offsets; then the offset arrays
// (n_graphs == DG_NG_DEVICE: the device's count, and the capacities in o are
// checked on the device)
hipError_t launch_dg_compact(const DgArgs &a, uint64_t n_graphs, const DgOut &t, const DgOut &o, hipStream_t s);
hipError_t launch_dg_offsets(const DgArgs &a, uint64_t n_graphs, const DgOut &o, hipStream_t s);

// UndoLog folding on the device (crgc_undo.hip)
struct UndoAccDev {
  uint64_t *keys;   // [cap] ids (~0: empty); the bucket index is the id's slot
  uint8_t *adm;     // [cap] UndoLog.admitted holds a Field for this id
  int32_t *msg;     // [cap] Field.messageCount
  uint64_t cap;
  uint64_t *pkeys;  // [pcap] actor bucket << 32 | target bucket
  int32_t *pcnt;    // [pcap] Field.createdRefs[target]
  uint64_t pcap;
  unsigned long long *n_ids, *n_pairs;  // keys inserted so far
};
struct UaDeltaArgs {
  uint64_t n, nout;
  const uint64_t *id;
  const int32_t *recv;
  const uint8_t *flags;
  const uint32_t *out_off;
  const uint64_t *out_target;
  const int32_t *out_count;
};
struct UaFieldArgs {
  uint64_t n, nc;
  int32_t sign;
  const uint64_t *actor;
  const int32_t *msg;
  const uint32_t *c_off;
  const uint64_t *c_target;
  const int32_t *c_count;
};
struct UaExportArgs {
  uint32_t *admf, *deg;  // [cap]
  uint64_t *aidx, *roff; // [cap] exclusive scans
  uint64_t *bsum;
  unsigned long long *n_fields, *n_created;
  uint64_t *actor;
  int32_t *msg;
  uint32_t *c_off;
  uint64_t *c_target;
  int32_t *c_count;
};
hipError_t launch_ua_fold_deltas(const UndoAccDev &u, const UaDeltaArgs &a, hipStream_t s);
hipError_t launch_ua_fold_fields(const UndoAccDev &u, const UaFieldArgs &a, hipStream_t s);
hipError_t launch_ua_init(const UndoAccDev &u, hipStream_t s);
hipError_t launch_ua_rehash(const UndoAccDev &o, const UndoAccDev &n, uint32_t *map, bool ids, hipStream_t s);
// phase 0: counts and scans; 1: the arrays
hipError_t launch_ua_export(const UndoAccDev &u, const UaExportArgs &x, int phase, hipStream_t s);

int grid_for(uint64_t threads, int block = 256, int cap = 4096);

}  // namespace crgc
