// crgc_delta.hip — DeltaGraph production on the device.
//
// With num-nodes > 1, LocalGC folds every drained Entry into a DeltaGraph
// and finalizes the graph whenever isFull() holds after an entry, and once
// more at the end of the wakeup (LocalGC.scala:159-177; DeltaGraph.java:73-180).
// Where one graph ends depends on where it started — a graph is full once it
// holds T = DGS - 4F - 1 distinct actors — so the cut is a chain:
//   k_dg_span     for every entry s, the end of a graph that would start at
//                 s (one wave streams the entries past 64 starts through a
//                 last-seen table; graphs longer than its window are deferred)
//   k_dg_jump / k_dg_walk / k_dg_fill   the starts reachable from entry 0:
//                 64-step jumps, one walk over them, the starts in between
//   k_dg_long     one workgroup resolves the first deferred start on the
//                 chain, 64 entries per step
//   k_dg_count / k_dg_scatter   the starts, compacted
// Then one wave per graph replays DeltaGraph.mergeEntry over its entries
// (k_dg_write, state in LDS) into slots bounded by the graph's entries: the
// decoded shadows and the DataOutput bytes of DeltaShadow.serialize, the
// outgoing map in java.util.HashMap iteration order; k_dg_compact packs the
// slots at the exact offsets.
#include "crgc_host.hpp"

namespace crgc {

constexpr uint32_t DG_LONG_P = 8192;  // k_dg_long: the set plus one step's new ids
constexpr uint32_t SCAN_B = 1024;
constexpr uint8_t NONE8 = 0xFF;

__device__ inline uint32_t dg_hash(uint64_t id, uint32_t bits) {
  return (uint32_t)((id * 0x9E3779B97F4A7C15ull) >> (64 - bits));
}
__device__ inline bool dg_reserved(uint64_t id) { return id >= CRGC_DEAD_ACTOR; }

// Lane j's value with j wave-uniform: v_readlane (scalar), not an LDS permute,
// for the loops that walk a batch lane by lane.
__device__ inline uint32_t rl32(uint32_t v, uint32_t j) { return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)j); }
__device__ inline uint64_t rl64(uint64_t v, uint32_t j) {
  return ((uint64_t)rl32((uint32_t)(v >> 32), j) << 32) | rl32((uint32_t)v, j);
}

struct DgRange {
  uint32_t c0, c1, s0, s1, u0, u1;
  bool bad;
};

// Record ranges of entry e clamped to the batch and to F records; `bad`
// reports offsets the merges would reject.
__device__ inline DgRange dg_range(const DgArgs &a, uint64_t e) {
  DgRange r;
  // record totals: the offsets' last entries (a.C / a.S / a.U bound them: for a
  // device batch the host has not read them)
  const uint64_t Ct = min(a.C, (uint64_t)a.c_off[a.n]), St = min(a.S, (uint64_t)a.s_off[a.n]),
                 Ut = min(a.U, (uint64_t)a.u_off[a.n]);
  const uint32_t c0 = a.c_off[e], c1 = a.c_off[e + 1], s0 = a.s_off[e], s1 = a.s_off[e + 1];
  const uint32_t u0 = a.u_off[e], u1 = a.u_off[e + 1];
  r.bad = c1 < c0 || s1 < s0 || u1 < u0 || c1 > Ct || s1 > St || u1 > Ut || c1 - c0 > a.F ||
          s1 - s0 > a.F || u1 - u0 > a.F || a.c_off[a.n] > a.C || a.s_off[a.n] > a.S || a.u_off[a.n] > a.U ||
          a.c_off[0] || a.s_off[0] || a.u_off[0];
  r.c1 = (uint32_t)min((uint64_t)c1, Ct);
  r.c0 = min(c0, r.c1);
  r.c1 = min(r.c1, r.c0 + a.F);
  r.s1 = (uint32_t)min((uint64_t)s1, St);
  r.s0 = min(s0, r.s1);
  r.s1 = min(r.s1, r.s0 + a.F);
  r.u1 = (uint32_t)min((uint64_t)u1, Ut);
  r.u0 = min(u0, r.u1);
  r.u1 = min(r.u1, r.u0 + a.F);
  return r;
}

// Visits the ids of entry e in DeltaGraph.encode order (:75, 86-89, 100, 111).
template <class Fn>
__device__ inline void dg_ids(const DgArgs &a, uint64_t e, const DgRange &r, Fn &&fn) {
  fn(a.self[e]);
  for (uint32_t k = r.c0; k < r.c1; ++k) {
    fn(a.c_target[k]);
    fn(a.c_owner[k]);
  }
  for (uint32_t k = r.s0; k < r.s1; ++k) fn(a.spawned[k]);
  for (uint32_t k = r.u0; k < r.u1; ++k) fn(a.u_ref[k]);
}

// The ranges of 64 consecutive entries from cb (lane l: entry cb + l), read
// once and consumed by several batches.
struct DgCursor {
  uint64_t cb;
  DgRange r;
  uint32_t m, incl;     // ids of the entry, inclusive scan over the chunk
  uint8_t eflags;       // Entry.isBusy / isRoot
  int16_t erecv;        // receive count
  bool bad;             // offsets the merges reject
};

__device__ inline void dg_load(const DgArgs &a, DgCursor &C, uint64_t cb, uint64_t e1) {
  const uint64_t el = cb + lane_id();
  C.cb = cb;
  C.r = DgRange{};
  C.m = 0;
  C.eflags = 0;
  C.erecv = 0;
  C.bad = false;
  if (el < e1) {
    C.r = dg_range(a, el);
    C.m = 1 + 2 * (C.r.c1 - C.r.c0) + (C.r.s1 - C.r.s0) + (C.r.u1 - C.r.u0);
    C.bad = C.r.bad;
    C.eflags = a.flags[el];
    C.erecv = a.recv[el];
  }
  C.incl = wave_incl_scan(C.m);
}

// One batch of whole entries from eb: lane l holds the l-th id, in encode
// order (:75, 86-89, 100, 111).
struct DgBatch {
  uint32_t ne, mt;      // entries, ids
  uint64_t id;          // lane < mt: its id
  int16_t info;         // updated refs: the RefobInfo
  uint32_t e, k;        // the id's entry (batch-local) and position in it
  uint32_t elane;       // the cursor lane holding that entry
  uint32_t nc, ns;      // that entry's created / spawned record counts
  uint32_t base;        // lane of that entry's first id
  bool bad;             // a reserved id
};

__device__ inline DgBatch dg_batch(const DgArgs &a, DgCursor &C, uint64_t eb, uint64_t e1) {
  const int lane = lane_id();
  if (eb < C.cb || eb - C.cb >= 48) dg_load(a, C, eb, e1);
  DgBatch B{};
  const uint32_t off = (uint32_t)(eb - C.cb);  // first cursor lane of the batch
  const uint32_t before = off ? rl32(C.incl, off - 1) : 0u;
  const uint64_t fits = __ballot((uint32_t)lane >= off && C.cb + lane < e1 && C.incl - before <= 64);
  B.ne = fits ? (uint32_t)__popcll(fits) : 1;  // (m <= 1 + 4F <= 64)
  B.mt = rl32(C.incl, off + B.ne - 1) - before;
  uint32_t my_e = 0;  // the number of entries ending at or before this lane's id
  for (uint32_t q = 0; q < B.ne; ++q)
    if (rl32(C.incl, off + q) - before <= (uint32_t)lane) my_e = q + 1;
  if (my_e >= B.ne) my_e = B.ne - 1;
  B.e = my_e;
  B.elane = off + my_e;
  const uint32_t c0 = __shfl(C.r.c0, B.elane), c1 = __shfl(C.r.c1, B.elane);
  const uint32_t s0 = __shfl(C.r.s0, B.elane), s1 = __shfl(C.r.s1, B.elane), u0 = __shfl(C.r.u0, B.elane);
  B.base = __shfl(C.incl - C.m, B.elane) - before;
  B.nc = c1 - c0;
  B.ns = s1 - s0;
  B.k = lane - B.base;
  if ((uint32_t)lane < B.mt) {
    const uint32_t k = B.k, nc = B.nc, ns = B.ns;
    if (k == 0) B.id = a.self[eb + my_e];
    else if (k < 1 + 2 * nc) B.id = ((k - 1) & 1) ? a.c_owner[c0 + (k - 1) / 2] : a.c_target[c0 + (k - 1) / 2];
    else if (k < 1 + 2 * nc + ns) B.id = a.spawned[s0 + (k - 1 - 2 * nc)];
    else {
      B.id = a.u_ref[u0 + (k - 1 - 2 * nc - ns)];
      B.info = a.u_info[u0 + (k - 1 - 2 * nc - ns)];
    }
    B.bad = dg_reserved(B.id);
  }
  return B;
}

// ---- the chain of graph starts ----------------------------------------------
// One wave per SPAN_S consecutive starts (lane l: start s0 + l).  The wave streams
// entries from s0, a batch of whole entries (<= 64 ids, one per lane) at a
// time, through one table of the ids seen so far with the last entry each was
// seen in.  An occurrence is new to lane l's graph iff the id's previous
// entry is before s0 + l: every lane finds its id's previous entry in the
// table or among the batch's earlier lanes, then every lane walks the batch's
// (entry, previous entry) pairs in order, counting its graph's actors and
// stopping after the entry that fills it.  Lanes still short of T after
// SPAN_WIN entries (or when the table is 3/4 full) are deferred.
constexpr uint32_t SPAN_P = 1024;    // ids per wave table
constexpr uint32_t SPAN_WIN = 192;   // entries a wave streams past s0
constexpr uint32_t SPAN_S = 64;      // graph starts per wave (32 measured no faster: profiles/r2j)

__global__ __launch_bounds__(256) void k_dg_span(DgArgs a) {
  __shared__ uint64_t key[4][SPAN_P];
  __shared__ uint16_t last[4][SPAN_P];  // entry relative to s0 (< SPAN_WIN + 64): 40 KB per workgroup, 4 per CU
  const int w = threadIdx.x >> 6, lane = lane_id();
  const uint64_t s0 = ((uint64_t)blockIdx.x * 4 + w) * SPAN_S;
  if (s0 > a.n) return;
  uint64_t *K = key[w];
  uint16_t *Ls = last[w];
  for (uint32_t k = lane; k < SPAN_P; k += 64) K[k] = CRGC_NO_ACTOR;
  wave_lds_fence();
  const bool mine = (uint32_t)lane < SPAN_S;  // lanes past SPAN_S only carry ids
  const uint64_t s = s0 + lane;
  uint32_t cnt = 0;
  bool done = !mine || s >= a.n, bad = false;
  uint64_t end = s >= a.n ? a.n : s;
  uint32_t used = 0;
  uint64_t e = s0;
  const uint64_t stop = min(a.n, s0 + SPAN_WIN);
  DgCursor C;
  dg_load(a, C, e, a.n);
  while (e < stop) {
    if (__ballot(!done) == 0) break;
    if (used > SPAN_P - SPAN_P / 4) break;
    const DgBatch B = dg_batch(a, C, e, a.n);
    bad |= B.bad || C.bad;
    const bool has = (uint32_t)lane < B.mt;
    const uint64_t x = has ? B.id : CRGC_NO_ACTOR;
    const uint32_t my_e = (uint32_t)(e - s0) + B.e;  // entry, relative to s0
    // the previous entry of this occurrence: in the table, or an earlier lane
    int32_t prev = -1;
    uint32_t h = dg_hash(x, 10);
    if (has) {
      for (;;) {
        const uint64_t y = K[h];
        if (y == x) {
          prev = (int32_t)Ls[h];
          break;
        }
        if (y == CRGC_NO_ACTOR) break;
        h = (h + 1) & (SPAN_P - 1);
      }
    }
    bool later = false;
    for (uint32_t j = 0; j < B.mt; ++j) {
      const uint64_t xj = rl64(x, j);
      const uint32_t ej = rl32(my_e, j);
      if (xj == x) {
        if (j < (uint32_t)lane) prev = (int32_t)ej;
        else if (j > (uint32_t)lane) later = true;
      }
    }
    // the last occurrence of each id in the batch updates the table
    bool fresh = false;
    if (has && !later) {
      for (;;) {
        const uint64_t y = atomicCAS((unsigned long long *)&K[h], (unsigned long long)CRGC_NO_ACTOR,
                                     (unsigned long long)x);
        if (y == CRGC_NO_ACTOR) fresh = true;
        if (y == CRGC_NO_ACTOR || y == x) break;
        h = (h + 1) & (SPAN_P - 1);
      }
      Ls[h] = (uint16_t)my_e;
    }
    used += (uint32_t)__popcll(__ballot(fresh));
    wave_lds_fence();
    // each lane's graph: new actors, entry by entry; isFull after an entry (:174-180)
    const uint32_t me_rel = (uint32_t)lane;  // this lane's start, relative to s0
    const uint32_t next_e = __shfl(B.e, (lane + 1) & 63);
    const bool last_of_entry = has && (lane + 1 == (int)B.mt || next_e != B.e);
    const uint64_t lasts = __ballot(last_of_entry);
    for (uint32_t j = 0; j < B.mt; ++j) {
      const uint32_t ej = rl32(my_e, j);
      const int32_t pj = (int32_t)rl32((uint32_t)prev, j);
      if (!done && ej >= me_rel) {
        if (pj < (int32_t)me_rel) ++cnt;
        if (((lasts >> j) & 1) && cnt >= a.T) {
          done = true;
          end = s0 + ej + 1;
        }
      }
    }
    e += B.ne;
  }
  if (!done && e >= a.n) {  // the last graph of the wakeup (LocalGC.scala:174-177)
    done = true;
    end = a.n;
  }
  if (__ballot(bad) && lane == 0) atomicOr(&a.ctr->err, 1ull);
  const uint64_t dl = __ballot(mine && s < a.n && !done);
  if (lane == 0 && dl) atomicAdd(&a.ctr->n_long, (unsigned)__popcll(dl));
  if (!mine || s > a.n) return;
  a.mark[s] = 0;  // the chain walks mark after this launch
  if (s == a.n) {
    a.J[s] = (uint32_t)a.n;
    a.lng[s] = 0;
    return;
  }
  a.J[s] = (uint32_t)(done ? end : s);  // a deferred start points at itself until k_dg_long
  a.lng[s] = !done;
}

// The chain from entry 0 in three launches (round 2 used 2 log4(n) + 1
// pointer-jumping launches, ~95 us at C5's 125 000 entries):
//   k_dg_jump    J64[s] = J^64(s), 64 dependent L2-resident loads per start
//   k_dg_walk    one thread walks J64 from the chain's start, marking every
//                64th graph start (a milestone, mark 2)
//   k_dg_fill    from each milestone, the next 63 starts along J (mark 1)
// A start whose span was deferred points at itself (J[s] = s), and so does the
// batch end n, so every walk stops there; k_dg_long resolves a deferred start,
// and the chain is walked again from the start after it.
constexpr uint32_t DG_STRIDE = 64;

__global__ __launch_bounds__(256) void k_dg_jump(DgArgs a) {
  const uint64_t N = a.n + 1;
  const uint32_t *J = a.J;
  uint32_t *J64 = a.J + N;
  for (uint64_t s = (uint64_t)blockIdx.x * 256 + threadIdx.x; s < N; s += (uint64_t)gridDim.x * 256) {
    uint32_t t = (uint32_t)s;
    for (uint32_t i = 0; i < DG_STRIDE; ++i) t = J[t];
    J64[s] = t;
  }
}

__global__ __launch_bounds__(64) void k_dg_walk(DgArgs a) {
  if (threadIdx.x != 0) return;
  const uint32_t *J64 = a.J + (a.n + 1);
  a.ctr->first_long = ~0u;  // k_dg_first_long looks again after k_dg_fill
  uint32_t t = a.ctr->walk_from;
  for (;;) {
    a.mark[t] = 2;
    const uint32_t nt = J64[t];
    if (nt == t) break;
    t = nt;
  }
}

__global__ __launch_bounds__(256) void k_dg_fill(DgArgs a) {
  const uint64_t N = a.n + 1;
  for (uint64_t s = (uint64_t)blockIdx.x * 256 + threadIdx.x; s < N; s += (uint64_t)gridDim.x * 256) {
    if (a.mark[s] != 2) continue;
    uint32_t t = (uint32_t)s;
    for (uint32_t i = 1; i < DG_STRIDE; ++i) {  // never reaches the next milestone (64 steps on)
      const uint32_t nt = a.J[t];
      if (nt == t) break;
      t = nt;
      a.mark[t] = 1;
    }
  }
}

__global__ __launch_bounds__(256) void k_dg_first_long(DgArgs a) {
  for (uint64_t s = (uint64_t)blockIdx.x * 256 + threadIdx.x; s < a.n; s += (uint64_t)gridDim.x * 256)
    if (a.mark[s] && a.lng[s]) atomicMin(&a.ctr->first_long, (unsigned int)s);
}

// One workgroup: the graph starting at the first deferred chain start, 64
// entries per step.  Ids already in the graph are "old" (first = 0); every
// new id keeps the first entry of the step it appears in (atomicMin), and a
// histogram + scan of those firsts tells where the graph fills.
__global__ __launch_bounds__(256) void k_dg_long(DgArgs a) {
  __shared__ uint64_t key[DG_LONG_P];
  __shared__ uint32_t first[DG_LONG_P];
  __shared__ uint32_t cnt[64];
  __shared__ uint64_t s_end;
  __shared__ uint32_t s_size;
  const uint64_t s = a.ctr->first_long;
  if (s >= a.n) return;
  for (uint32_t k = threadIdx.x; k < DG_LONG_P; k += 256) {
    key[k] = CRGC_NO_ACTOR;
    first[k] = ~0u;
  }
  if (threadIdx.x == 0) {
    s_end = a.n;  // no fill before the batch ends: the last graph
    s_size = 0;
  }
  __syncthreads();
  for (uint64_t e0 = s; e0 < a.n; e0 += 64) {
    if (threadIdx.x < 64) cnt[threadIdx.x] = 0;
    const uint64_t e = e0 + threadIdx.x;
    if (threadIdx.x < 64 && e < a.n) {
      const DgRange r = dg_range(a, e);
      const uint32_t tag = threadIdx.x + 1;
      dg_ids(a, e, r, [&](uint64_t id) {
        uint32_t h = dg_hash(id, 13);
        for (;;) {
          const uint64_t prev = atomicCAS((unsigned long long *)&key[h], (unsigned long long)CRGC_NO_ACTOR,
                                          (unsigned long long)id);
          if (prev == CRGC_NO_ACTOR || prev == id) {
            atomicMin(&first[h], tag);
            return;
          }
          h = (h + 1) & (DG_LONG_P - 1);
        }
      });
    }
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < DG_LONG_P; k += 256) {
      const uint32_t f = first[k];
      if (f >= 1 && f <= 64) atomicAdd(&cnt[f - 1], 1u);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t size = s_size;
      for (uint32_t j = 0; j < 64 && e0 + j < a.n; ++j) {
        size += cnt[j];
        if (size >= a.T) {
          s_end = e0 + j + 1;
          break;
        }
      }
      s_size = size;
    }
    __syncthreads();
    if (s_end != a.n) break;
    for (uint32_t k = threadIdx.x; k < DG_LONG_P; k += 256)  // this step's ids join the graph
      if (first[k] != ~0u) first[k] = 0;
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    a.J[s] = (uint32_t)s_end;
    a.lng[s] = 0;
    a.ctr->walk_from = (uint32_t)s_end;
  }
}

__device__ inline uint32_t block_excl_1024(uint32_t v, uint32_t *total) {
  __shared__ uint32_t w[16];
  const uint32_t incl = wave_incl_scan(v);
  const int wv = threadIdx.x >> 6;
  if (lane_id() == 63) w[wv] = incl;
  __syncthreads();
  uint32_t pre = 0, tot = 0;
  for (int k = 0; k < (int)(blockDim.x >> 6); ++k) {
    if (k < wv) pre += w[k];
    tot += w[k];
  }
  __syncthreads();
  *total = tot;
  return pre + incl - v;
}

// Marked starts per 1024 entries.
__global__ __launch_bounds__(256) void k_dg_count(DgArgs a) {
  const uint64_t base = (uint64_t)blockIdx.x * 1024 + threadIdx.x * 4;
  uint32_t c = 0;
  for (int j = 0; j < 4; ++j) c += (base + j < a.n && a.mark[base + j]) ? 1u : 0u;
  uint32_t tot;
  block_excl_1024(c, &tot);
  if (threadIdx.x == 0) a.blk[blockIdx.x] = tot;
}

__global__ __launch_bounds__(256) void k_dg_scatter(DgArgs a) {
  const uint64_t base = (uint64_t)blockIdx.x * 1024 + threadIdx.x * 4;
  uint32_t c = 0;
  for (int j = 0; j < 4; ++j) c += (base + j < a.n && a.mark[base + j]) ? 1u : 0u;
  uint32_t tot;
  uint64_t pos = a.blk_off[blockIdx.x] + block_excl_1024(c, &tot);
  for (int j = 0; j < 4; ++j)
    if (base + j < a.n && a.mark[base + j]) a.starts[pos++] = (uint32_t)(base + j);
  if (blockIdx.x == 0 && threadIdx.x == 0) a.starts[a.ctr->n_graphs] = (uint32_t)a.n;
}

// ---- exclusive scans of up to 4 u32 arrays (two levels of 1024) -------------

__global__ __launch_bounds__(SCAN_B) void k_scan_sums(ScanSet q) {
  const uint64_t i = (uint64_t)blockIdx.x * SCAN_B + threadIdx.x;
  for (int j = 0; j < q.k; ++j) {
    uint32_t tot;
    block_excl_1024(i < q.n ? q.in[j][i] : 0u, &tot);
    if (threadIdx.x == 0) q.bsum[(uint64_t)j * q.nb + blockIdx.x] = tot;
  }
}

__global__ __launch_bounds__(SCAN_B) void k_scan_top(ScanSet q) {
  __shared__ uint64_t w[16];
  const int wv = threadIdx.x >> 6;
  for (int j = 0; j < q.k; ++j) {
    uint64_t carry = 0;
    uint64_t *b = q.bsum + (uint64_t)j * q.nb;
    for (uint64_t c0 = 0; c0 < q.nb; c0 += SCAN_B) {
      const uint64_t i = c0 + threadIdx.x;
      const uint64_t v = i < q.nb ? b[i] : 0;
      uint64_t incl = v;  // 64-bit wave scan
      for (int d = 1; d < 64; d <<= 1) {
        const uint64_t o = __shfl_up(incl, d);
        if (lane_id() >= d) incl += o;
      }
      if (lane_id() == 63) w[wv] = incl;
      __syncthreads();
      uint64_t pre = carry, tot = 0;
      for (int k = 0; k < 16; ++k) {
        if (k < wv) pre += w[k];
        tot += w[k];
      }
      if (i < q.nb) b[i] = pre + incl - v;
      carry += tot;
      __syncthreads();
    }
    if (threadIdx.x == 0) *q.total[j] = carry;
  }
}

__global__ __launch_bounds__(SCAN_B) void k_scan_apply(ScanSet q) {
  const uint64_t i = (uint64_t)blockIdx.x * SCAN_B + threadIdx.x;
  for (int j = 0; j < q.k; ++j) {
    uint32_t tot;
    const uint32_t x = block_excl_1024(i < q.n ? q.in[j][i] : 0u, &tot);
    if (i < q.n) q.out[j][i] = q.bsum[(uint64_t)j * q.nb + blockIdx.x] + x;
  }
}

// Up to SCAN_B block sums: each workgroup adds up the sums before its own (at
// most SCAN_B loads, one per thread), so no k_scan_top launch; the last block
// writes the totals.
__global__ __launch_bounds__(SCAN_B) void k_scan_apply_top(ScanSet q) {
  __shared__ uint64_t w[4][SCAN_B / 64];
  const uint64_t i = (uint64_t)blockIdx.x * SCAN_B + threadIdx.x;
  const int lane = lane_id(), wv = threadIdx.x >> 6;
  uint64_t pre[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    uint64_t p = j < q.k && threadIdx.x < blockIdx.x ? q.bsum[(uint64_t)j * q.nb + threadIdx.x] : 0;
    for (int d = 32; d > 0; d >>= 1) p += __shfl_xor(p, d);
    if (lane == 0) w[j][wv] = p;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    pre[j] = 0;
    for (int k = 0; k < (int)(SCAN_B / 64); ++k) pre[j] += w[j][k];
  }
  for (int j = 0; j < q.k; ++j) {
    uint32_t tot;
    const uint32_t x = block_excl_1024(i < q.n ? q.in[j][i] : 0u, &tot);
    if (i < q.n) q.out[j][i] = pre[j] + x;
    if (blockIdx.x == q.nb - 1 && threadIdx.x == 0) *q.total[j] = pre[j] + tot;
  }
}

// Small scans in one workgroup (one launch instead of three).  n_dev: the
// element count on the device (null: q.n); a set *skip (a deferred DeltaGraph
// chain start, nothing was counted) scans nothing.
constexpr uint64_t SCAN_ONE_MAX = 1 << 16;  // elements x arrays

__global__ __launch_bounds__(SCAN_B) void k_scan_one(ScanSet q, const unsigned long long *n_dev,
                                                   const unsigned int *skip) {
  constexpr uint32_t E = 4;  // consecutive elements per thread per chunk
  __shared__ uint64_t s_w[4][16];
  __shared__ uint64_t carry[4];
  uint64_t n = n_dev ? *n_dev : q.n;
  if (skip && *skip != ~0u) n = 0;
  const int lane = lane_id(), wv = threadIdx.x >> 6;
  if (threadIdx.x < 4) carry[threadIdx.x] = 0;
  __syncthreads();
  for (uint64_t c0 = 0; c0 < n; c0 += (uint64_t)SCAN_B * E) {
    const uint64_t i0 = c0 + (uint64_t)threadIdx.x * E;
    uint32_t v[4][E], sum[4], incl[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {  // every array's wave scans, then one barrier
      sum[j] = 0;
      incl[j] = 0;
      if (j >= q.k) continue;
#pragma unroll
      for (uint32_t e = 0; e < E; ++e) {
        v[j][e] = i0 + e < n ? q.in[j][i0 + e] : 0u;
        sum[j] += v[j][e];
      }
      incl[j] = wave_incl_scan(sum[j]);
      if (lane == 63) s_w[j][wv] = incl[j];
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (j >= q.k) continue;
      uint64_t pre = carry[j], tot = 0;
      for (int w = 0; w < (int)(SCAN_B / 64); ++w) {
        if (w < wv) pre += s_w[j][w];
        tot += s_w[j][w];
      }
      uint64_t run = pre + incl[j] - sum[j];
#pragma unroll
      for (uint32_t e = 0; e < E; ++e) {
        if (i0 + e < n) q.out[j][i0 + e] = run;
        run += v[j][e];
      }
      __syncthreads();  // every thread has read carry[j] and s_w[j]
      if (threadIdx.x == 0) carry[j] += tot;
    }
    __syncthreads();
  }
  if (threadIdx.x < (unsigned)q.k) *q.total[threadIdx.x] = carry[threadIdx.x];
}

hipError_t run_scan(ScanSet q, hipStream_t s) {
  if (q.n == 0) {
    for (int j = 0; j < q.k; ++j) hipMemsetAsync(q.total[j], 0, 8, s);
    return hipGetLastError();
  }
  if (q.n * q.k <= SCAN_ONE_MAX) {
    hipLaunchKernelGGL(k_scan_one, dim3(1), dim3(SCAN_B), 0, s, q, nullptr, nullptr);
    return hipGetLastError();
  }
  q.nb = (q.n + SCAN_B - 1) / SCAN_B;
  hipLaunchKernelGGL(k_scan_sums, dim3(q.nb), dim3(SCAN_B), 0, s, q);
  if (q.nb <= SCAN_B) {
    hipLaunchKernelGGL(k_scan_apply_top, dim3(q.nb), dim3(SCAN_B), 0, s, q);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(SCAN_B), 0, s, q);
  hipLaunchKernelGGL(k_scan_apply, dim3(q.nb), dim3(SCAN_B), 0, s, q);
  return hipGetLastError();
}

static int dg_grid(uint64_t n) { return (int)std::min<uint64_t>((n + 255) / 256, 8192); }

hipError_t launch_dg_chain(const DgArgs &a, int phase, hipStream_t s) {
  launch_begin();
  const uint64_t N = a.n + 1;
  if (phase == 0) {
    hipLaunchKernelGGL(k_dg_span, dim3((N + 4 * SPAN_S - 1) / (4 * SPAN_S)), dim3(256), 0, s, a);
  } else if (phase == 1) {
    hipLaunchKernelGGL(k_dg_long, dim3(1), dim3(256), 0, s, a);
  }
  if (phase <= 1) {
    hipLaunchKernelGGL(k_dg_jump, dim3(dg_grid(N)), dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_dg_walk, dim3(1), dim3(64), 0, s, a);
    hipLaunchKernelGGL(k_dg_fill, dim3(dg_grid(N)), dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_dg_first_long, dim3(dg_grid(a.n)), dim3(256), 0, s, a);
  }
  const uint64_t nblk = (a.n + 1023) / 1024;
  hipLaunchKernelGGL(k_dg_count, dim3(nblk), dim3(256), 0, s, a);
  ScanSet q{};
  q.in[0] = a.blk;
  q.out[0] = a.blk_off;
  q.total[0] = &a.ctr->n_graphs;
  q.k = 1;
  q.n = nblk;
  q.bsum = a.bsum;
  if (hipError_t e = run_scan(q, s)) return e;
  hipLaunchKernelGGL(k_dg_scatter, dim3(nblk), dim3(256), 0, s, a);
  return hipGetLastError();
}

// ---- one graph: DeltaGraph.mergeEntry replayed by one wave ------------------
// The wave reads the graph's entries a batch at a time (whole entries, at most
// 64 ids: one id per lane) in two passes, neither serialised per id:
//   1. every lane inserts its id into an LDS hash table (64-bit LDS CAS) and
//      records its position with an LDS atomicMin; receive counts add up per
//      slot (LDS atomics), and isBusy/isRoot/interned and the supervisor are
//      last-write-wins tags (LDS atomicMax of entry index << 8 | value).
//      DeltaGraph.encode (:148-156) numbers actors by first appearance, so a
//      slot's compressed id is the rank of its first position.
//   2. updateOutgoing (:127-136) in op order, one owner per lane: each batch's
//      ops are broadcast and the owner's lane applies them to its row of a
//      64 x 64 count matrix (count and time of the key's last insertion) and
//      its map's size and largest size — all that java.util.HashMap iteration
//      order depends on.
constexpr uint32_t DGW_P = 128;  // id -> cid hash slots
constexpr uint32_t DG_OPCAP = 512;  // updateOutgoing ops kept in LDS by pass 1 (more: pass 2 re-reads the ids)

struct DgWave {
  uint64_t key[DGW_P];       // id per hash slot (KEY_EMPTY: free)
  uint64_t hfl[DGW_P];       // per slot: (entry + 1) << 8 | CRGC_DELTA_* of the last entry of the actor
  uint64_t hsup[DGW_P];      // per slot: (entry + 1) << 8 | slot of the last spawner
  uint32_t first[DGW_P];     // per slot: position of the id's first appearance
  int32_t hrecv[DGW_P];      // per slot: receive count
  uint64_t dec[DG_MAX];      // decoder: id per cid (DeltaGraph.java:162-169)
  int32_t cnt[DG_MAX * DG_MAX];   // outgoing[o][t] (0: absent)
  uint32_t ins[DG_MAX * DG_MAX];  // op time of the key's last insertion
  int32_t recv[DG_MAX];
  uint8_t tabc[DGW_P];       // cid per hash slot
  uint8_t sup[DG_MAX];       // supervisor cid, NONE8: -1
  uint8_t fl[DG_MAX];        // CRGC_DELTA_*
  uint8_t osz[DG_MAX];       // outgoing.size()
  uint8_t omax[DG_MAX];      // largest outgoing.size(): the HashMap's capacity
  uint32_t ops[DG_OPCAP];    // pass 1's ops in order: owner slot | target slot << 8 | (+1) << 16
};

// Replays DeltaGraph.mergeEntry (DeltaGraph.java:73-125) over entries
// [starts[g], starts[g+1]); returns the number of shadows.
__device__ uint32_t dg_replay(const DgArgs &a, uint64_t g, DgWave &W) {
  const int lane = lane_id();
  for (uint32_t k = lane; k < DGW_P; k += 64) {
    W.key[k] = KEY_EMPTY;
    W.first[k] = 0xFFFFFFFFu;
    W.hrecv[k] = 0;
    W.hfl[k] = 0;
    W.hsup[k] = 0;
  }
  wave_lds_fence();
  const uint64_t e0 = a.starts[g], e1 = a.starts[g + 1];
  // pass 1: the ids, receive counts and last-write-wins fields, per hash slot
  uint32_t pos = 0, ei = 0, nops = 0;
  DgCursor C;
  dg_load(a, C, e0, e1);
  for (uint64_t eb = e0; eb < e1;) {
    const DgBatch B = dg_batch(a, C, eb, e1);
    uint32_t h = 0;
    if ((uint32_t)lane < B.mt) {
      const uint64_t x = B.id == KEY_EMPTY ? KEY_EMPTY - 1 : B.id;  // reserved ids are errors already
      h = dg_hash(x, 7);
      for (;;) {
        const uint64_t k = atomicCAS((unsigned long long *)&W.key[h], (unsigned long long)KEY_EMPTY,
                                     (unsigned long long)x);
        if (k == KEY_EMPTY || k == x) break;
        h = (h + 1) & (DGW_P - 1);
      }
      atomicMin(&W.first[h], pos + lane);
    }
    const uint32_t me = __shfl(h, B.base);
    {  // the batch's updateOutgoing ops, in order, by hash slot (pass 2 maps them to cids)
      const uint32_t prev_h = __shfl(h, (lane + 63) & 63);  // a created owner's target is the lane before
      const uint32_t k = B.k;
      bool emit = false;
      uint32_t opv = 0;
      if ((uint32_t)lane < B.mt && k >= 1) {
        if (k < 1 + 2 * B.nc) {
          if ((k - 1) & 1) {
            emit = true;
            opv = h | (prev_h << 8) | (1u << 16);
          }
        } else if (k >= 1 + 2 * B.nc + B.ns && refob_deactivated(B.info)) {
          emit = true;
          opv = me | (h << 8);
        }
      }
      const uint64_t eball = __ballot(emit);
      const uint32_t at = nops + (uint32_t)__popcll(eball & lanemask_lt());
      if (emit && at < DG_OPCAP) W.ops[at] = opv;
      nops += (uint32_t)__popcll(eball);
    }
    const uint8_t ef = (uint8_t)__shfl((uint32_t)C.eflags, B.elane);
    const int32_t er = __shfl((int32_t)C.erecv, B.elane);
    if ((uint32_t)lane < B.mt) {
      const uint64_t tag = (uint64_t)(ei + B.e + 1) << 8;
      const uint32_t k = B.k;
      if (k == 0) {  // local information (:75-80)
        atomicAdd(&W.hrecv[h], er);
        atomicMax((unsigned long long *)&W.hfl[h],
                  (unsigned long long)(tag | CRGC_DELTA_INTERNED | ((ef & CRGC_ENTRY_ROOT) ? CRGC_DELTA_ROOT : 0) |
                                       ((ef & CRGC_ENTRY_BUSY) ? CRGC_DELTA_BUSY : 0)));
      } else if (k >= 1 + 2 * B.nc && k < 1 + 2 * B.nc + B.ns) {  // spawned actors (:95-104)
        atomicMax((unsigned long long *)&W.hsup[h], (unsigned long long)(tag | me));
      } else if (k >= 1 + 2 * B.nc) {  // updated refs (:107-124)
        const int32_t sc = refob_count(B.info);
        if (sc > 0) atomicAdd(&W.hrecv[h], -sc);
      }
    }
    pos += B.mt;
    ei += B.ne;
    eb += B.ne;
  }
  wave_lds_fence();
  // compressed ids: rank of the first appearance
  uint32_t size = 0;
  for (uint32_t s = lane; s < DGW_P; s += 64) {
    const uint32_t f = W.first[s];
    size += (uint32_t)__popcll(__ballot(f != 0xFFFFFFFFu));
    if (f == 0xFFFFFFFFu) continue;
    uint32_t r = 0;
    for (uint32_t j = 0; j < DGW_P; ++j) r += W.first[j] < f ? 1u : 0u;
    W.tabc[s] = (uint8_t)r;
    W.dec[r] = W.key[s];
    W.recv[r] = W.hrecv[s];
    W.fl[r] = (uint8_t)W.hfl[s];
  }
  wave_lds_fence();
  for (uint32_t s = lane; s < DGW_P; s += 64) {
    if (W.first[s] == 0xFFFFFFFFu) continue;
    const uint64_t sp = W.hsup[s];
    W.sup[W.tabc[s]] = sp ? W.tabc[sp & 0xFF] : NONE8;
  }
  for (uint32_t k = lane; k < size * DG_MAX; k += 64) W.cnt[k] = 0;
  wave_lds_fence();
  // pass 2: updateOutgoing in op order; lane o owns row o
  uint32_t clock = 0, osz = 0, omax = 0;
  auto apply = [&](uint32_t v) {  // v = owner cid | target cid << 8 | (+1) << 16
    if ((v & 0xFF) == (uint32_t)lane) {
      const uint32_t kk = (uint32_t)lane * DG_MAX + ((v >> 8) & 0xFF);
      const int32_t c0 = W.cnt[kk];
      const int32_t nc = (int32_t)((uint32_t)c0 + ((v >> 16) ? 1u : 0xFFFFFFFFu));
      W.cnt[kk] = nc;
      if (c0 == 0) {  // put of an absent key: appended to its bin
        W.ins[kk] = clock;
        ++osz;
        omax = max(omax, osz);
      } else if (nc == 0) {  // remove
        --osz;
      }
    }
    ++clock;
  };
  if (nops <= DG_OPCAP) {  // the ops pass 1 kept: no global reads
    for (uint32_t c0 = 0; c0 < nops; c0 += 64) {
      const uint32_t n = min(64u, nops - c0);
      uint32_t op = 0;
      if ((uint32_t)lane < n) {
        const uint32_t v = W.ops[c0 + lane];
        op = W.tabc[v & 0xFF] | ((uint32_t)W.tabc[(v >> 8) & 0xFF] << 8) | (v & (1u << 16));
      }
      for (uint32_t j = 0; j < n; ++j) apply(rl32(op, j));
    }
    W.osz[lane] = (uint8_t)osz;
    W.omax[lane] = (uint8_t)omax;
    wave_lds_fence();
    return size;
  }
  dg_load(a, C, e0, e1);
  for (uint64_t eb = e0; eb < e1;) {
    const DgBatch B = dg_batch(a, C, eb, e1);
    uint32_t c = 0;
    if ((uint32_t)lane < B.mt) {
      const uint64_t x = B.id == KEY_EMPTY ? KEY_EMPTY - 1 : B.id;
      uint32_t h = dg_hash(x, 7);
      while (W.key[h] != x) h = (h + 1) & (DGW_P - 1);
      c = W.tabc[h];
    }
    const uint32_t me = __shfl(c, B.base);
    const uint32_t prev = __shfl(c, (lane + 63) & 63);  // a created owner's target is the lane before
    const uint32_t k = B.k;
    bool emit = false;
    uint32_t op = 0;
    if ((uint32_t)lane < B.mt && k >= 1) {
      if (k < 1 + 2 * B.nc) {
        if ((k - 1) & 1) {  // created ref (:83-92): outgoing[owner][target] += 1
          emit = true;
          op = c | (prev << 8) | (1u << 16);
        }
      } else if (k >= 1 + 2 * B.nc + B.ns && refob_deactivated(B.info)) {  // :120-123
        emit = true;
        op = me | (c << 8);
      }
    }
    uint64_t bits = __ballot(emit);
    while (bits) {
      const int j = __ffsll((unsigned long long)bits) - 1;
      bits &= bits - 1;
      apply(rl32(op, j));
    }
    eb += B.ne;
  }
  W.osz[lane] = (uint8_t)osz;
  W.omax[lane] = (uint8_t)omax;
  wave_lds_fence();
  return size;
}

__device__ inline void put_be(uint8_t *p, uint32_t v, int bytes) {
  for (int i = 0; i < bytes; ++i) p[i] = (uint8_t)(v >> (8 * (bytes - 1 - i)));
}

// The graph's shadows in compressed-id order, lane c = shadow c: decoded rows,
// and the bytes of writeShort(size) + DeltaShadow.serialize each
// (DeltaShadow.java:57-69).  A DeltaShadow.outgoing is a HashMap<Short,
// Integer> built by the default constructor: 16 bins, doubling whenever its
// size passes 3/4 of them, so its capacity follows from the largest size it
// ever had; iteration walks bins in order (bin = key & (capacity - 1):
// Short.hashCode is the value) and each bin in insertion order (a removed key
// re-put goes to the tail; resizes keep the order).  Keys < DGS <= 64 never
// fill a bin to the treeify threshold.
// Writes go to graph g's bounded slots (k_dg_bounds): rows [row0, row0 +
// rcap), outgoing entries [ob0, ob0 + ocap), bytes [wb0, wb0 + wcap); a valid
// batch never reaches the caps, a malformed one (reported by the span kernel)
// is kept inside them.
__device__ void dg_emit(const DgWave &W, uint32_t size, const DgOut &o, uint64_t row0, uint64_t ob0,
                        uint64_t wb0, uint32_t rcap, uint32_t ocap, uint32_t wcap) {
  const uint32_t c = lane_id();
  const bool on = c < size;
  const uint32_t nk = on ? W.osz[c] : 0;
  const uint32_t nb = on ? 13 + 6 * nk : 0;
  const uint32_t oi = wave_incl_scan(nk), bi = wave_incl_scan(nb);
  if (!on || c >= rcap || oi > ocap || 2 + bi > wcap) return;
  const uint64_t row = row0 + c;
  uint64_t ob = ob0 + oi - nk;
  uint8_t *w = o.wire + wb0 + 2 + bi - nb;
  if (c == 0) put_be(o.wire + wb0, size, 2);
  const uint8_t sp = W.sup[c], f = W.fl[c];
  const int32_t rc = W.recv[c];
  o.id[row] = W.dec[c];
  o.recv[row] = rc;
  o.sup[row] = sp == NONE8 ? CRGC_NO_ACTOR : W.dec[sp];
  o.flags[row] = f;
  o.out_off[row] = (uint32_t)(ob - ob0);  // graph-relative until k_dg_compact
  put_be(w, (uint32_t)rc, 4);
  put_be(w + 4, sp == NONE8 ? 0xFFFFu : sp, 2);
  w[6] = (f & CRGC_DELTA_INTERNED) ? 1 : 0;
  w[7] = (f & CRGC_DELTA_ROOT) ? 1 : 0;
  w[8] = (f & CRGC_DELTA_BUSY) ? 1 : 0;
  put_be(w + 9, nk, 4);
  w += 13;
  uint32_t cap = 16;
  while (W.omax[c] > cap - cap / 4) cap <<= 1;
  const int32_t *row_cnt = W.cnt + c * DG_MAX;
  const uint32_t *row_ins = W.ins + c * DG_MAX;
  for (uint32_t bin = 0; bin < cap && bin < DG_MAX; ++bin) {
    // the bin's keys (bin, bin + cap, ...) in insertion order: at most 4 (cap >= 16, keys < 64)
    uint32_t ks[4], n = 0;
    for (uint32_t t = bin; t < DG_MAX; t += cap) {
      if (row_cnt[t] == 0) continue;
      uint32_t i = n++;
      while (i > 0 && row_ins[ks[i - 1]] > row_ins[t]) {
        ks[i] = ks[i - 1];
        --i;
      }
      ks[i] = t;
    }
    for (uint32_t i = 0; i < n; ++i) {
      const uint32_t t = ks[i];
      o.out_target[ob] = W.dec[t];
      o.out_count[ob] = row_cnt[t];
      ++ob;
      put_be(w, t, 2);
      put_be(w + 2, (uint32_t)row_cnt[t], 4);
      w += 6;
    }
  }
}

// ng == DG_NG_DEVICE: the graph count is the device's (n_graphs), and nothing
// is built while a deferred chain start is unresolved (first_long set): the
// host then resolves it and runs the passes again.
__device__ inline bool dg_count(const DgArgs &a, uint64_t &ng) {
  if (ng != DG_NG_DEVICE) return true;
  if (a.ctr->first_long != ~0u) return false;
  ng = a.ctr->n_graphs;
  return true;
}

// One pass instead of a count pass and a write pass: every graph gets slots
// bounded by its entries (shadows <= its ids and < DGS, outgoing entries <= its
// created refs + updated refs), the write pass fills them and records the exact
// sizes, and k_dg_compact packs the slots once the exact offsets are scanned.
__global__ __launch_bounds__(256) void k_dg_bounds(DgArgs a, uint64_t ng) {
  if (!dg_count(a, ng)) return;
  for (uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x; g < ng; g += (uint64_t)gridDim.x * 256) {
    const uint64_t e0 = a.starts[g], e1 = a.starts[g + 1];
    auto d = [](uint32_t x0, uint32_t x1) { return x1 >= x0 ? (uint64_t)(x1 - x0) : ~0ull >> 8; };
    const uint64_t cc = d(a.c_off[e0], a.c_off[e1]), uu = d(a.u_off[e0], a.u_off[e1]);
    const uint64_t ids = (e1 - e0) + 2 * cc + d(a.s_off[e0], a.s_off[e1]) + uu;
    const uint32_t sh = (uint32_t)min<uint64_t>(ids, DG_MAX);
    const uint32_t ou = (uint32_t)min<uint64_t>(cc + uu, (uint64_t)DG_MAX * DG_MAX);
    a.b_size[g] = sh;
    a.b_out[g] = ou;
    a.b_bytes[g] = 2 + 13 * sh + 6 * ou;
  }
}

__global__ __launch_bounds__(64) void k_dg_write(DgArgs a, uint64_t ng, DgOut t) {
  __shared__ DgWave W;
  if (!dg_count(a, ng)) return;
  for (uint64_t g = blockIdx.x; g < ng; g += gridDim.x) {
    const uint32_t size = dg_replay(a, g, W);
    const uint32_t c = lane_id();
    const uint32_t nk = c < size ? W.osz[c] : 0;
    const uint32_t nout = __shfl(wave_incl_scan(nk), 63);
    const uint64_t row0 = a.t_shadow[g], ob0 = a.t_out[g], wb0 = a.t_wire[g];
    const uint32_t rcap = a.b_size[g], ocap = a.b_out[g], wcap = a.b_bytes[g];
    const bool fits = row0 + rcap <= t.shadow_cap && ob0 + ocap <= t.out_cap && wb0 + wcap <= t.wire_cap;
    if (c == 0) {
      a.g_size[g] = size;
      a.g_nout[g] = nout;
      a.g_bytes[g] = 2 + 13 * size + 6 * nout;
      if (!fits || size > rcap || nout > ocap) atomicOr(&a.ctr->err, 2ull);  // only a malformed batch
    }
    if (fits) dg_emit(W, size, t, row0, ob0, wb0, rcap, ocap, wcap);
    wave_lds_fence();
  }
}

// The outputs hold the graphs the device counted (passes that run before the
// host has seen the totals).
__device__ inline bool dg_fits(const DgArgs &a, uint64_t ng, const DgOut &o) {
  return ng <= o.graph_cap && a.ctr->n_shadows <= o.shadow_cap && a.ctr->n_out <= o.out_cap &&
         a.ctr->wire <= o.wire_cap;
}

// One wave per graph: its slots, packed at the exact offsets.
__global__ __launch_bounds__(256) void k_dg_compact(DgArgs a, uint64_t ng, DgOut t, DgOut o) {
  const bool dev = ng == DG_NG_DEVICE;
  if (!dg_count(a, ng)) return;
  if (dev && !dg_fits(a, ng, o)) {
    if (blockIdx.x == 0 && threadIdx.x == 0) a.ctr->overflow = 1;
    return;
  }
  const int lane = lane_id();
  const uint64_t nw = (uint64_t)gridDim.x * 4;
  for (uint64_t g = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); g < ng; g += nw) {
    const uint64_t r0 = a.t_shadow[g], o0 = a.t_out[g], w0 = a.t_wire[g];
    const uint64_t R0 = a.g_shadow[g], O0 = a.g_out[g], W0 = a.g_wire[g];
    const uint32_t size = a.g_size[g], nout = a.g_nout[g], nb = a.g_bytes[g];
    for (uint32_t i = lane; i < size; i += 64) {
      o.id[R0 + i] = t.id[r0 + i];
      o.recv[R0 + i] = t.recv[r0 + i];
      o.sup[R0 + i] = t.sup[r0 + i];
      o.flags[R0 + i] = t.flags[r0 + i];
      o.out_off[R0 + i] = (uint32_t)O0 + t.out_off[r0 + i];
    }
    for (uint32_t i = lane; i < nout; i += 64) {
      o.out_target[O0 + i] = t.out_target[o0 + i];
      o.out_count[O0 + i] = t.out_count[o0 + i];
    }
    for (uint32_t i = lane; i < nb; i += 64) o.wire[W0 + i] = t.wire[w0 + i];
  }
}

hipError_t launch_dg_write(const DgArgs &a, uint64_t ng, const DgOut &t, hipStream_t s) {
  launch_begin();
  if (ng == 0) return hipSuccess;
  const uint64_t bound = ng == DG_NG_DEVICE ? a.n + 1 : ng;
  hipLaunchKernelGGL(k_dg_bounds, dim3(dg_grid(bound)), dim3(256), 0, s, a, ng);
  ScanSet q{};
  q.n = ng;
  q.bsum = a.bsum;
  q.in[0] = a.b_size;
  q.out[0] = a.t_shadow;
  q.total[0] = &a.ctr->t_shadows;
  q.in[1] = a.b_out;
  q.out[1] = a.t_out;
  q.total[1] = &a.ctr->t_out;
  q.in[2] = a.b_bytes;
  q.out[2] = a.t_wire;
  q.total[2] = &a.ctr->t_wire;
  q.k = 3;
  if (ng != DG_NG_DEVICE) {
    if (hipError_t e = run_scan(q, s)) return e;
  } else {
    hipLaunchKernelGGL(k_scan_one, dim3(1), dim3(SCAN_B), 0, s, q, &a.ctr->n_graphs, &a.ctr->first_long);
  }
  hipLaunchKernelGGL(k_dg_write, dim3((unsigned)std::min<uint64_t>(bound, 4096)), dim3(64), 0, s, a, ng, t);
  if (hipError_t e = hipGetLastError()) return e;  // before the nested helper drops it
  return launch_dg_scans(a, ng, s);
}

hipError_t launch_dg_compact(const DgArgs &a, uint64_t ng, const DgOut &t, const DgOut &o, hipStream_t s) {
  launch_begin();
  if (ng == 0) return hipSuccess;
  const uint64_t bound = ng == DG_NG_DEVICE ? a.n + 1 : ng;
  hipLaunchKernelGGL(k_dg_compact, dim3((unsigned)std::min<uint64_t>((bound + 3) / 4, 4096)), dim3(256), 0, s, a,
                     ng, t, o);
  return hipGetLastError();
}

hipError_t launch_dg_scans(const DgArgs &a, uint64_t ng, hipStream_t s) {
  launch_begin();
  ScanSet q{};
  q.n = ng;
  q.bsum = a.bsum;
  q.in[0] = a.g_size;
  q.out[0] = a.g_shadow;
  q.total[0] = &a.ctr->n_shadows;
  q.in[1] = a.g_nout;
  q.out[1] = a.g_out;
  q.total[1] = &a.ctr->n_out;
  q.in[2] = a.g_bytes;
  q.out[2] = a.g_wire;
  q.total[2] = &a.ctr->wire;
  q.k = 3;
  if (ng != DG_NG_DEVICE) return run_scan(q, s);
  // over the graphs the device counted, so the counts past them need no zeroing
  hipLaunchKernelGGL(k_scan_one, dim3(1), dim3(SCAN_B), 0, s, q, &a.ctr->n_graphs, &a.ctr->first_long);
  return hipGetLastError();
}

__global__ __launch_bounds__(256) void k_dg_offsets(DgArgs a, uint64_t ng, DgOut o) {
  if (ng == DG_NG_DEVICE) {
    if (a.ctr->first_long != ~0u) return;
    ng = a.ctr->n_graphs;
    if (!dg_fits(a, ng, o)) return;
  }
  for (uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x; g <= ng; g += (uint64_t)gridDim.x * 256) {
    if (g < ng) {
      o.graph_off[g] = (uint32_t)a.g_shadow[g];
      o.wire_off[g] = a.g_wire[g];
    } else {
      o.graph_off[g] = (uint32_t)a.ctr->n_shadows;
      o.wire_off[g] = a.ctr->wire;
      o.out_off[a.ctr->n_shadows] = (uint32_t)a.ctr->n_out;
    }
  }
}

hipError_t launch_dg_offsets(const DgArgs &a, uint64_t ng, const DgOut &o, hipStream_t s) {
  launch_begin();
  hipLaunchKernelGGL(k_dg_offsets, dim3(dg_grid((ng == DG_NG_DEVICE ? a.n + 1 : ng) + 1)), dim3(256), 0, s, a, ng,
                     o);
  return hipGetLastError();
}

}  // namespace crgc
