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
//   k_dg_double   J_{k+1} = J_k o J_k (pointer doubling)
//   k_dg_mark     starts reachable from entry 0, top level down
//   k_dg_long     one workgroup resolves the first deferred start on the
//                 chain, 64 entries per step
//   k_dg_count / k_dg_scatter   the starts, compacted
// Then one wave per graph replays DeltaGraph.mergeEntry over its entries
// (k_dg_build, state in LDS) — once to size the outputs, once to write them:
// the decoded shadows and the DataOutput bytes of DeltaShadow.serialize, the
// outgoing map in java.util.HashMap iteration order.
#include "crgc_host.hpp"

namespace crgc {

constexpr uint32_t DG_LONG_P = 8192;  // k_dg_long: the set plus one step's new ids
constexpr uint32_t SCAN_B = 1024;
constexpr uint8_t NONE8 = 0xFF;

__device__ inline uint32_t dg_hash(uint64_t id, uint32_t bits) {
  return (uint32_t)((id * 0x9E3779B97F4A7C15ull) >> (64 - bits));
}
__device__ inline bool dg_reserved(uint64_t id) { return id >= CRGC_DEAD_ACTOR; }

struct DgRange {
  uint32_t c0, c1, s0, s1, u0, u1;
  bool bad;
};

// Record ranges of entry e clamped to the batch and to F records; `bad`
// reports offsets the merges would reject.
__device__ inline DgRange dg_range(const DgArgs &a, uint64_t e) {
  DgRange r;
  const uint32_t c0 = a.c_off[e], c1 = a.c_off[e + 1], s0 = a.s_off[e], s1 = a.s_off[e + 1];
  const uint32_t u0 = a.u_off[e], u1 = a.u_off[e + 1];
  r.bad = c1 < c0 || s1 < s0 || u1 < u0 || c1 > a.C || s1 > a.S || u1 > a.U || c1 - c0 > a.F ||
          s1 - s0 > a.F || u1 - u0 > a.F;
  r.c1 = (uint32_t)min((uint64_t)c1, a.C);
  r.c0 = min(c0, r.c1);
  r.c1 = min(r.c1, r.c0 + a.F);
  r.s1 = (uint32_t)min((uint64_t)s1, a.S);
  r.s0 = min(s0, r.s1);
  r.s1 = min(r.s1, r.s0 + a.F);
  r.u1 = (uint32_t)min((uint64_t)u1, a.U);
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

// ---- the chain of graph starts ----------------------------------------------
// One wave per 64 consecutive starts (lane l: start s0 + l).  The wave streams
// entries from s0 through one table of the ids seen so far, each with the last
// entry it was seen in; an occurrence is new to lane l's graph iff that entry
// is before s0 + l.  So every entry is read once per wave and no lane keeps a
// set of its own.  Lanes still short of T after SPAN_WIN entries (or when the
// table is 3/4 full) are deferred.
constexpr uint32_t SPAN_P = 1024;    // ids per wave table
constexpr uint32_t SPAN_WIN = 192;   // entries a wave streams past s0

__global__ __launch_bounds__(256) void k_dg_span(DgArgs a) {
  __shared__ uint64_t key[4][SPAN_P];
  __shared__ uint32_t last[4][SPAN_P];
  const int w = threadIdx.x >> 6, lane = lane_id();
  const uint64_t s0 = ((uint64_t)blockIdx.x * 4 + w) * 64;
  if (s0 > a.n) return;
  uint64_t *K = key[w];
  uint32_t *Ls = last[w];
  for (uint32_t k = lane; k < SPAN_P; k += 64) K[k] = CRGC_NO_ACTOR;
  wave_lds_fence();
  const uint64_t s = s0 + lane;
  uint32_t cnt = 0;
  bool done = s >= a.n, bad = false;
  uint64_t end = s >= a.n ? a.n : s;
  uint32_t used = 0;
  uint64_t e = s0;
  const uint64_t stop = min(a.n, s0 + SPAN_WIN);
  for (; e < stop; ++e) {
    if (__ballot(!done) == 0) break;
    if (used > SPAN_P - SPAN_P / 4) break;
    const DgRange r = dg_range(a, e);
    bad |= r.bad;
    const uint32_t nc = r.c1 - r.c0, ns = r.s1 - r.s0, nu = r.u1 - r.u0;
    const uint32_t m = 1 + 2 * nc + ns + nu;  // <= 1 + 4F <= 64 ids, in encode order
    uint64_t myid = 0;
    if ((uint32_t)lane < m) {
      const uint32_t k = lane;
      if (k == 0) myid = a.self[e];
      else if (k < 1 + 2 * nc) myid = ((k - 1) & 1) ? a.c_owner[r.c0 + (k - 1) / 2] : a.c_target[r.c0 + (k - 1) / 2];
      else if (k < 1 + 2 * nc + ns) myid = a.spawned[r.s0 + (k - 1 - 2 * nc)];
      else myid = a.u_ref[r.u0 + (k - 1 - 2 * nc - ns)];
      bad |= dg_reserved(myid);
    }
    const bool in = !done && e >= s;
    for (uint32_t k = 0; k < m; ++k) {
      const uint64_t x = __shfl(myid, k);
      uint32_t h = dg_hash(x, 10);
      int64_t prev = -1;
      for (;;) {  // every lane walks the same probe sequence (broadcast reads)
        const uint64_t y = K[h];
        if (y == x) {
          prev = Ls[h];
          break;
        }
        if (y == CRGC_NO_ACTOR) {
          if (lane == 0) K[h] = x;
          ++used;
          break;
        }
        h = (h + 1) & (SPAN_P - 1);
      }
      if (lane == 0) Ls[h] = (uint32_t)e;
      wave_lds_fence();
      if (in && prev < (int64_t)s) ++cnt;
    }
    if (in && cnt >= a.T) {  // isFull after entry e (:174-180)
      done = true;
      end = e + 1;
    }
  }
  if (!done && e == a.n) {  // the last graph of the wakeup (LocalGC.scala:174-177)
    done = true;
    end = a.n;
  }
  if (__ballot(bad) && lane == 0) atomicOr(&a.ctr->err, 1ull);
  if (s > a.n) return;
  if (s == a.n) {
    a.J[s] = (uint32_t)a.n;
    a.lng[s] = 0;
    return;
  }
  a.J[s] = (uint32_t)(done ? end : s);  // a deferred start points at itself until k_dg_long
  a.lng[s] = !done;
  const uint64_t dl = __ballot(!done);
  if (lane == 0 && dl) atomicAdd(&a.ctr->n_long, (unsigned)__popcll(dl));
}

__global__ __launch_bounds__(256) void k_dg_double(DgArgs a, uint32_t k) {
  const uint64_t N = a.n + 1;
  const uint32_t *Jk = a.J + (uint64_t)k * N;
  uint32_t *Jn = a.J + (uint64_t)(k + 1) * N;
  for (uint64_t s = (uint64_t)blockIdx.x * 256 + threadIdx.x; s < N; s += (uint64_t)gridDim.x * 256)
    Jn[s] = Jk[Jk[s]];
}

// Marked after levels L-1 .. k: the chain's starts at multiples of 2^k steps
// (a start marked early by a racing thread is a chain start too).
__global__ __launch_bounds__(256) void k_dg_mark(DgArgs a, uint32_t k) {
  const uint64_t N = a.n + 1;
  const uint32_t *Jk = a.J + (uint64_t)k * N;
  for (uint64_t s = (uint64_t)blockIdx.x * 256 + threadIdx.x; s < N; s += (uint64_t)gridDim.x * 256)
    if (a.mark[s]) a.mark[Jk[s]] = 1;
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
    a.mark[s_end] = 1;
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

hipError_t run_scan(ScanSet q, hipStream_t s) {
  if (q.n == 0) {
    for (int j = 0; j < q.k; ++j) hipMemsetAsync(q.total[j], 0, 8, s);
    return hipGetLastError();
  }
  q.nb = (q.n + SCAN_B - 1) / SCAN_B;
  hipLaunchKernelGGL(k_scan_sums, dim3(q.nb), dim3(SCAN_B), 0, s, q);
  hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(SCAN_B), 0, s, q);
  hipLaunchKernelGGL(k_scan_apply, dim3(q.nb), dim3(SCAN_B), 0, s, q);
  return hipGetLastError();
}

static int dg_grid(uint64_t n) { return (int)std::min<uint64_t>((n + 255) / 256, 8192); }

hipError_t launch_dg_chain(const DgArgs &a, int phase, hipStream_t s) {
  const uint64_t N = a.n + 1;
  if (phase == 0) {
    hipLaunchKernelGGL(k_dg_span, dim3((N + 255) / 256), dim3(256), 0, s, a);
    for (uint32_t k = 0; k + 1 < a.levels; ++k)
      hipLaunchKernelGGL(k_dg_double, dim3(dg_grid(N)), dim3(256), 0, s, a, k);
    hipMemsetAsync(a.mark, 0, N, s);
    hipMemsetAsync(a.mark, 1, 1, s);
  } else if (phase == 1) {
    hipLaunchKernelGGL(k_dg_long, dim3(1), dim3(256), 0, s, a);
  }
  if (phase <= 1) {
    for (uint32_t k = a.levels; k-- > 0;)
      hipLaunchKernelGGL(k_dg_mark, dim3(dg_grid(N)), dim3(256), 0, s, a, k);
    hipMemsetAsync(&a.ctr->first_long, 0xFF, 4, s);
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
// The wave loads the graph's entries a batch at a time (whole entries, at most
// 64 ids: one id per lane), encodes the ids in order against an LDS table
// (DeltaGraph.encode, :148-156) and applies each entry's effects in order.
// Outgoing maps are one 64 x 64 count matrix: cnt[o][t] and the time of the
// key's last insertion, plus each owner's size and largest size — all that
// java.util.HashMap iteration order depends on.
constexpr uint32_t DGW_P = 128;  // id -> cid hash slots

struct DgWave {
  uint64_t key[DGW_P];
  uint64_t dec[DG_MAX];      // decoder: id per cid (DeltaGraph.java:162-169)
  int32_t cnt[DG_MAX * DG_MAX];   // outgoing[o][t] (0: absent)
  uint32_t ins[DG_MAX * DG_MAX];  // op time of the key's last insertion
  int32_t recv[DG_MAX];
  uint8_t tabc[DGW_P];       // cid per hash slot
  uint8_t sup[DG_MAX];       // supervisor cid, NONE8: -1
  uint8_t fl[DG_MAX];        // CRGC_DELTA_*
  uint8_t osz[DG_MAX];       // outgoing.size()
  uint8_t omax[DG_MAX];      // largest outgoing.size(): the HashMap's capacity
};

// Replays DeltaGraph.mergeEntry (DeltaGraph.java:73-125) over entries
// [starts[g], starts[g+1]); returns the number of shadows.  Lane-uniform
// control flow; lane 0 performs the LDS writes of the serial steps.
__device__ uint32_t dg_replay(const DgArgs &a, uint64_t g, DgWave &W) {
  const int lane = lane_id();
  for (uint32_t k = lane; k < DGW_P; k += 64) W.tabc[k] = NONE8;
  for (uint32_t k = lane; k < DG_MAX * DG_MAX; k += 64) W.cnt[k] = 0;
  wave_lds_fence();
  uint32_t size = 0, clock = 0;
  const uint64_t e0 = a.starts[g], e1 = a.starts[g + 1];
  auto op = [&](uint32_t o, uint32_t t, int32_t d) {  // updateOutgoing (:127-136)
    const uint32_t k = o * DG_MAX + t;
    const int32_t c = W.cnt[k];
    const int32_t nc = (int32_t)((uint32_t)c + (uint32_t)d);
    if (lane == 0) {
      W.cnt[k] = nc;
      if (c == 0) {  // put of an absent key: appended to its bin
        W.ins[k] = clock;
        const uint32_t sz = W.osz[o] + 1u;
        W.osz[o] = (uint8_t)sz;
        if (sz > W.omax[o]) W.omax[o] = (uint8_t)sz;
      } else if (nc == 0) {  // remove
        W.osz[o] = (uint8_t)(W.osz[o] - 1u);
      }
    }
    ++clock;
    wave_lds_fence();
  };
  for (uint64_t eb = e0; eb < e1;) {
    // a batch of whole entries with at most 64 ids: lane l holds entry eb+l's ranges
    const uint64_t el = eb + lane;
    DgRange r{};
    uint32_t m = 0;
    if (el < e1) {
      r = dg_range(a, el);
      m = 1 + 2 * (r.c1 - r.c0) + (r.s1 - r.s0) + (r.u1 - r.u0);
    }
    const uint32_t incl = wave_incl_scan(m);
    const uint64_t fits = __ballot(el < e1 && incl <= 64);
    const uint32_t ne = fits ? (uint32_t)__popcll(fits) : 1;  // entries of this batch (m <= 63)
    const uint32_t mt = __shfl(incl, ne - 1);
    // lane k: the k-th id of the batch, in encode order
    uint64_t myid = 0;
    int16_t myinfo = 0;
    uint32_t my_e = 0;  // entry of id `lane`: the number of entries ending at or before it
    for (uint32_t q = 0; q < ne; ++q)
      if (__shfl(incl, q) <= (uint32_t)lane) my_e = q + 1;
    if (my_e >= ne) my_e = ne - 1;
    const uint8_t myflags = el < e1 ? a.flags[el] : 0;
    const int16_t myrecv = el < e1 ? a.recv[el] : 0;
    {
      // every lane needs the ranges of the entry its id belongs to
      const uint32_t c0 = __shfl(r.c0, my_e), c1 = __shfl(r.c1, my_e);
      const uint32_t s0 = __shfl(r.s0, my_e), s1 = __shfl(r.s1, my_e), u0 = __shfl(r.u0, my_e);
      const uint32_t base = __shfl(incl - m, my_e);
      if ((uint32_t)lane < mt) {
        const uint32_t k = lane - base, nc = c1 - c0, ns = s1 - s0;
        if (k == 0) myid = a.self[eb + my_e];
        else if (k < 1 + 2 * nc) myid = ((k - 1) & 1) ? a.c_owner[c0 + (k - 1) / 2] : a.c_target[c0 + (k - 1) / 2];
        else if (k < 1 + 2 * nc + ns) myid = a.spawned[s0 + (k - 1 - 2 * nc)];
        else {
          myid = a.u_ref[u0 + (k - 1 - 2 * nc - ns)];
          myinfo = a.u_info[u0 + (k - 1 - 2 * nc - ns)];
        }
      }
    }
    // encode, in order (:148-156)
    uint32_t mycid = 0;
    for (uint32_t k = 0; k < mt; ++k) {
      const uint64_t x = __shfl(myid, k);
      uint32_t h = dg_hash(x, 7);
      uint32_t c;
      for (;;) {
        c = W.tabc[h];
        if (c == NONE8) {
          c = size++;
          if (lane == 0) {
            W.tabc[h] = (uint8_t)c;
            W.key[h] = x;
            W.dec[c] = x;
            W.recv[c] = 0;
            W.sup[c] = NONE8;
            W.fl[c] = 0;
            W.osz[c] = 0;
            W.omax[c] = 0;
          }
          wave_lds_fence();
          break;
        }
        if (W.key[h] == x) break;
        h = (h + 1) & (DGW_P - 1);
      }
      if ((uint32_t)lane == k) mycid = c;
    }
    // effects, entry by entry
    for (uint32_t q = 0; q < ne; ++q) {
      const uint32_t base = __shfl(incl - m, q);
      const uint32_t c0 = __shfl(r.c0, q), c1 = __shfl(r.c1, q), s0 = __shfl(r.s0, q),
                     s1 = __shfl(r.s1, q), u0 = __shfl(r.u0, q), u1 = __shfl(r.u1, q);
      (void)c0;
      (void)s0;
      (void)u0;
      const uint32_t nc = c1 - c0, ns = s1 - s0, nu = u1 - u0;
      const uint32_t me = __shfl(mycid, base);
      const uint8_t ef = (uint8_t)__shfl((uint32_t)myflags, q);
      const int32_t erecv = __shfl((int32_t)myrecv, q);
      if (lane == 0) {  // local information (:75-80)
        W.fl[me] = (uint8_t)(CRGC_DELTA_INTERNED | ((ef & CRGC_ENTRY_ROOT) ? CRGC_DELTA_ROOT : 0) |
                             ((ef & CRGC_ENTRY_BUSY) ? CRGC_DELTA_BUSY : 0));
        W.recv[me] = (int32_t)((uint32_t)W.recv[me] + (uint32_t)erecv);
      }
      wave_lds_fence();
      for (uint32_t j = 0; j < nc; ++j)  // created refs (:83-92)
        op(__shfl(mycid, base + 2 + 2 * j), __shfl(mycid, base + 1 + 2 * j), 1);
      for (uint32_t j = 0; j < ns; ++j) {  // spawned actors (:95-104)
        const uint32_t ch = __shfl(mycid, base + 1 + 2 * nc + j);
        if (lane == 0) W.sup[ch] = (uint8_t)me;
      }
      for (uint32_t j = 0; j < nu; ++j) {  // updated refs (:107-124)
        const uint32_t t = __shfl(mycid, base + 1 + 2 * nc + ns + j);
        const int16_t info = (int16_t)__shfl((int32_t)myinfo, base + 1 + 2 * nc + ns + j);
        const int32_t sc = refob_count(info);
        if (sc > 0 && lane == 0) W.recv[t] = (int32_t)((uint32_t)W.recv[t] - (uint32_t)sc);
        wave_lds_fence();
        if (refob_deactivated(info)) op(me, t, -1);
      }
      wave_lds_fence();
    }
    eb += ne;
  }
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
__device__ void dg_emit(const DgArgs &a, uint64_t g, const DgWave &W, uint32_t size, const DgOut &o) {
  const uint32_t c = lane_id();
  const bool on = c < size;
  const uint32_t nk = on ? W.osz[c] : 0;
  const uint32_t nb = on ? 13 + 6 * nk : 0;
  const uint32_t oi = wave_incl_scan(nk), bi = wave_incl_scan(nb);
  if (!on) return;
  const uint64_t row = a.g_shadow[g] + c;
  uint64_t ob = a.g_out[g] + oi - nk;
  uint8_t *w = o.wire + a.g_wire[g] + 2 + bi - nb;
  if (c == 0) put_be(o.wire + a.g_wire[g], size, 2);
  const uint8_t sp = W.sup[c], f = W.fl[c];
  const int32_t rc = W.recv[c];
  o.id[row] = W.dec[c];
  o.recv[row] = rc;
  o.sup[row] = sp == NONE8 ? CRGC_NO_ACTOR : W.dec[sp];
  o.flags[row] = f;
  o.out_off[row] = (uint32_t)ob;
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

template <bool WRITE>
__global__ __launch_bounds__(64) void k_dg_build(DgArgs a, uint64_t ng, DgOut o) {
  __shared__ DgWave W;
  for (uint64_t g = blockIdx.x; g < ng; g += gridDim.x) {
    const uint32_t size = dg_replay(a, g, W);
    if (WRITE) {
      dg_emit(a, g, W, size, o);
    } else {
      const uint32_t c = lane_id();
      const uint32_t nk = c < size ? W.osz[c] : 0;
      const uint32_t nout = __shfl(wave_incl_scan(nk), 63);
      if (c == 0) {
        a.g_size[g] = size;
        a.g_nout[g] = nout;
        a.g_bytes[g] = 2 + 13 * size + 6 * nout;
      }
    }
    wave_lds_fence();
  }
}

hipError_t launch_dg_build(const DgArgs &a, uint64_t ng, bool write, const DgOut &o, hipStream_t s) {
  if (ng == 0) return hipSuccess;
  const dim3 grid((unsigned)std::min<uint64_t>(ng, 4096));
  if (write) hipLaunchKernelGGL(k_dg_build<true>, grid, dim3(64), 0, s, a, ng, o);
  else hipLaunchKernelGGL(k_dg_build<false>, grid, dim3(64), 0, s, a, ng, o);
  return hipGetLastError();
}

hipError_t launch_dg_scans(const DgArgs &a, uint64_t ng, hipStream_t s) {
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
  return run_scan(q, s);
}

__global__ __launch_bounds__(256) void k_dg_offsets(DgArgs a, uint64_t ng, DgOut o) {
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
  hipLaunchKernelGGL(k_dg_offsets, dim3(dg_grid(ng + 1)), dim3(256), 0, s, a, ng, o);
  return hipGetLastError();
}

}  // namespace crgc
