// crgc_delta.hip — DeltaGraph production on the device.
//
// With num-nodes > 1, LocalGC folds every drained Entry into a DeltaGraph
// and finalizes the graph whenever isFull() holds after an entry, and once
// more at the end of the wakeup (LocalGC.scala:159-177; DeltaGraph.java:73-180).
// Where one graph ends depends on where it started — a graph is full once it
// holds T = DGS - 4F - 1 distinct actors — so the cut is a chain:
//   k_dg_span     thread per entry s: the end of a graph that would start at
//                 s (per-thread id set in LDS, at most DG_SPAN_CAP entries;
//                 longer ones are deferred)
//   k_dg_double   J_{k+1} = J_k o J_k (pointer doubling)
//   k_dg_mark     starts reachable from entry 0, top level down
//   k_dg_long     one workgroup resolves the first deferred start on the
//                 chain, 64 entries per step
//   k_dg_count / k_dg_scatter   the starts, compacted
// Then one thread per graph replays DeltaGraph.mergeEntry over its entries
// (k_dg_build: state in LDS, or in a global store for graphs with more than
// DG_RCAP outgoing records) — once to size the outputs, once to write them:
// the decoded shadows and the DataOutput bytes of DeltaShadow.serialize, the
// outgoing map in java.util.HashMap iteration order.
#include "crgc_host.hpp"

namespace crgc {

constexpr uint32_t DG_P = 128;     // per-thread hash slots (2 x DG_MAX)
constexpr uint32_t DG_T = 64;      // threads per workgroup of the per-thread kernels
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
__global__ __launch_bounds__(DG_T) void k_dg_span(DgArgs a) {
  __shared__ uint64_t tab[DG_P * DG_T];
  const uint32_t t = threadIdx.x;
  const uint64_t s = (uint64_t)blockIdx.x * DG_T + t;
  if (s > a.n) return;
  if (s == a.n) {
    a.J[s] = (uint32_t)a.n;
    a.lng[s] = 0;
    return;
  }
  uint64_t *tb = tab + t;
  for (uint32_t k = 0; k < DG_P; ++k) tb[k * DG_T] = CRGC_NO_ACTOR;
  uint32_t size = 0;
  bool bad = false;
  auto ins = [&](uint64_t id) {
    bad |= dg_reserved(id);
    uint32_t h = dg_hash(id, 7);
    for (;;) {  // never full: at most DGS - 1 < DG_P ids
      const uint64_t k = tb[h * DG_T];
      if (k == id) return;
      if (k == CRGC_NO_ACTOR) {
        tb[h * DG_T] = id;
        ++size;
        return;
      }
      h = (h + 1) & (DG_P - 1);
    }
  };
  uint64_t end = s;
  bool deferred = true;
  uint64_t e = s;
  for (; e < a.n && e < s + DG_SPAN_CAP; ++e) {
    const DgRange r = dg_range(a, e);
    bad |= r.bad;
    dg_ids(a, e, r, ins);
    if (size >= a.T) {  // isFull after this entry (:174-180)
      end = e + 1;
      deferred = false;
      break;
    }
  }
  if (deferred && e == a.n) {  // the last graph of the wakeup (LocalGC.scala:174-177)
    end = a.n;
    deferred = false;
  }
  if (bad) atomicOr(&a.ctr->err, 1ull);
  a.J[s] = (uint32_t)end;  // a deferred start points at itself until k_dg_long resolves it
  a.lng[s] = deferred;
  if (deferred) atomicAdd(&a.ctr->n_long, 1u);
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
struct ScanSet {
  const uint32_t *in[4];
  uint64_t *out[4];
  unsigned long long *total[4];
  int k;
  uint64_t n, nb;
  uint64_t *bsum;  // [4][nb]
};

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

static hipError_t run_scan(ScanSet q, hipStream_t s) {
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
    hipLaunchKernelGGL(k_dg_span, dim3((N + DG_T - 1) / DG_T), dim3(DG_T), 0, s, a);
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

// ---- one graph: DeltaGraph.mergeEntry replayed by one thread -----------------
// Element i of a per-thread array X is X[i * st] (st = DG_T in LDS, 1 in a
// global store).
struct DgStore {
  uint8_t *tab;    // [DG_P] cid per hash slot (NONE8: empty)
  uint64_t *dec;   // [DGS] decoder: id per cid (DeltaGraph.java:162-169)
  int32_t *recv;   // [DGS] DeltaShadow.recvCount
  uint8_t *sup;    // [DGS] supervisor cid (NONE8: -1)
  uint8_t *fl;     // [DGS] CRGC_DELTA_*
  uint8_t *osz;    // [DGS] outgoing.size()
  uint8_t *omax;   // [DGS] largest outgoing.size() so far: the HashMap's capacity
  uint64_t *rec;   // [rcap] owner | target << 8 | (u32)count << 32; count 0: key absent
  uint32_t *rins;  // [rcap] time of the key's last insertion (HashMap bin order)
  uint32_t st, rcap;
};

__device__ inline DgStore dg_global_store(uint64_t *base, uint32_t dgs) {
  DgStore S;
  char *p = (char *)base;
  S.dec = (uint64_t *)p;
  p += DG_MAX * 8;
  S.rec = (uint64_t *)p;
  p += (size_t)dgs * dgs * 8;
  S.rins = (uint32_t *)p;
  p += (size_t)dgs * dgs * 4;
  S.recv = (int32_t *)p;
  p += DG_MAX * 4;
  S.tab = (uint8_t *)p;
  p += DG_P;
  S.sup = (uint8_t *)p;
  p += DG_MAX;
  S.fl = (uint8_t *)p;
  p += DG_MAX;
  S.osz = (uint8_t *)p;
  p += DG_MAX;
  S.omax = (uint8_t *)p;
  S.st = 1;
  S.rcap = dgs * dgs;  // distinct (owner, target) pairs never exceed DGS^2
  return S;
}

uint64_t dg_store_words(uint32_t dgs) {
  const uint64_t bytes = DG_MAX * 8 + (uint64_t)dgs * dgs * 12 + DG_MAX * 4 + DG_P + 4 * DG_MAX;
  return (bytes + 63) / 64 * 8;
}

struct DgGraph {
  uint32_t size, nrec;
  bool ok;
};

// Replays DeltaGraph.mergeEntry (DeltaGraph.java:73-125) over entries
// [starts[g], starts[g+1]).  ok = false: more than rcap outgoing records.
__device__ DgGraph dg_replay(const DgArgs &a, uint64_t g, const DgStore &S) {
  const uint32_t st = S.st;
  for (uint32_t k = 0; k < DG_P; ++k) S.tab[k * st] = NONE8;
  DgGraph G{0, 0, true};
  uint32_t clock = 0;
  auto enc = [&](uint64_t id) -> uint32_t {  // encode (:148-156)
    uint32_t h = dg_hash(id, 7);
    for (;;) {
      const uint32_t c = S.tab[h * st];
      if (c == NONE8) {
        const uint32_t n = G.size++;
        S.tab[h * st] = (uint8_t)n;
        S.dec[n * st] = id;
        S.recv[n * st] = 0;
        S.sup[n * st] = NONE8;
        S.fl[n * st] = 0;
        S.osz[n * st] = 0;
        S.omax[n * st] = 0;
        return n;
      }
      if (S.dec[c * st] == id) return c;
      h = (h + 1) & (DG_P - 1);
    }
  };
  auto upd = [&](uint32_t o, uint32_t t, int32_t d) {  // updateOutgoing (:127-136)
    const uint64_t key = (uint64_t)o | ((uint64_t)t << 8);
    uint32_t k = 0;
    for (; k < G.nrec; ++k)
      if ((S.rec[k * st] & 0xFFFFull) == key) break;
    int32_t cnt;
    if (k == G.nrec) {
      if (G.nrec == S.rcap) {
        G.ok = false;
        return;
      }
      ++G.nrec;
      cnt = 0;
    } else {
      cnt = (int32_t)(uint32_t)(S.rec[k * st] >> 32);
    }
    const int32_t nc = (int32_t)((uint32_t)cnt + (uint32_t)d);
    if (cnt == 0) {  // put of an absent key: appended to its bin
      S.rins[k * st] = clock;
      const uint32_t sz = S.osz[o * st] + 1u;
      S.osz[o * st] = (uint8_t)sz;
      if (sz > S.omax[o * st]) S.omax[o * st] = (uint8_t)sz;
    } else if (nc == 0) {  // remove
      S.osz[o * st] = (uint8_t)(S.osz[o * st] - 1u);
    }
    S.rec[k * st] = key | ((uint64_t)(uint32_t)nc << 32);
    ++clock;
  };
  const uint64_t e0 = a.starts[g], e1 = a.starts[g + 1];
  for (uint64_t e = e0; e < e1 && G.ok; ++e) {
    const DgRange r = dg_range(a, e);
    const uint32_t me = enc(a.self[e]);  // local information (:75-80)
    const uint8_t ef = a.flags[e];
    S.fl[me * st] = (uint8_t)(CRGC_DELTA_INTERNED | ((ef & CRGC_ENTRY_ROOT) ? CRGC_DELTA_ROOT : 0) |
                              ((ef & CRGC_ENTRY_BUSY) ? CRGC_DELTA_BUSY : 0));
    S.recv[me * st] = (int32_t)((uint32_t)S.recv[me * st] + (uint32_t)(int32_t)a.recv[e]);
    for (uint32_t k = r.c0; k < r.c1; ++k) {  // created refs (:83-92): target, then owner
      const uint32_t t = enc(a.c_target[k]);
      const uint32_t o = enc(a.c_owner[k]);
      upd(o, t, 1);
    }
    for (uint32_t k = r.s0; k < r.s1; ++k) S.sup[enc(a.spawned[k]) * st] = (uint8_t)me;  // (:95-104)
    for (uint32_t k = r.u0; k < r.u1; ++k) {  // updated refs (:107-124)
      const uint32_t t = enc(a.u_ref[k]);
      const int16_t info = a.u_info[k];
      const int32_t sc = refob_count(info);
      if (sc > 0) S.recv[t * st] = (int32_t)((uint32_t)S.recv[t * st] - (uint32_t)sc);
      if (refob_deactivated(info)) upd(me, t, -1);
    }
  }
  return G;
}

__device__ inline uint32_t dg_nout(const DgStore &S, const DgGraph &G) {
  uint32_t n = 0;
  for (uint32_t k = 0; k < G.nrec; ++k) n += (S.rec[k * S.st] >> 32) ? 1u : 0u;
  return n;
}

__device__ inline void put_be(uint8_t *p, uint32_t v, int bytes) {
  for (int i = 0; i < bytes; ++i) p[i] = (uint8_t)(v >> (8 * (bytes - 1 - i)));
}

// The graph's shadows in compressed-id order: decoded rows, and the bytes of
// writeShort(size) + DeltaShadow.serialize each (DeltaShadow.java:57-69).  A
// DeltaShadow.outgoing is a HashMap<Short,Integer> built by the default
// constructor: 16 bins, doubling whenever its size passes 3/4 of them, so its
// capacity follows from the largest size it ever had; iteration walks bins in
// order (bin = key & (capacity - 1): Short.hashCode is the value) and each bin
// in insertion order (a removed key re-put goes to the tail; resizes keep the
// order).  Keys < DGS <= 64 never fill a bin to the treeify threshold.
__device__ void dg_emit(const DgArgs &a, uint64_t g, const DgStore &S, const DgGraph &G, const DgOut &o) {
  const uint32_t st = S.st;
  const uint64_t sb = a.g_shadow[g];
  uint64_t ob = a.g_out[g];
  uint8_t *w = o.wire + a.g_wire[g];
  put_be(w, G.size, 2);
  w += 2;
  for (uint32_t c = 0; c < G.size; ++c) {
    const uint64_t row = sb + c;
    const uint8_t sp = S.sup[c * st], f = S.fl[c * st];
    const int32_t rc = S.recv[c * st];
    const uint32_t nk = S.osz[c * st];
    o.id[row] = S.dec[c * st];
    o.recv[row] = rc;
    o.sup[row] = sp == NONE8 ? CRGC_NO_ACTOR : S.dec[sp * st];
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
    while (S.omax[c * st] > cap - cap / 4) cap <<= 1;
    uint64_t last = 0;
    for (uint32_t j = 0; j < nk; ++j) {  // next key in iteration order
      uint64_t best = ~0ull;
      uint32_t bk = 0;
      for (uint32_t k = 0; k < G.nrec; ++k) {
        const uint64_t r = S.rec[k * st];
        if ((r & 0xFF) != c || !(r >> 32)) continue;
        const uint32_t t = (uint32_t)(r >> 8) & 0xFF;
        const uint64_t ord = ((uint64_t)(t & (cap - 1)) << 32 | S.rins[k * st]) + 1;  // > 0
        if (ord > last && ord < best) {
          best = ord;
          bk = k;
        }
      }
      last = best;
      const uint64_t r = S.rec[bk * st];
      const uint32_t t = (uint32_t)(r >> 8) & 0xFF;
      const int32_t cnt = (int32_t)(uint32_t)(r >> 32);
      o.out_target[ob] = S.dec[t * st];
      o.out_count[ob] = cnt;
      ++ob;
      put_be(w, t, 2);
      put_be(w + 2, (uint32_t)cnt, 4);
      w += 6;
    }
  }
}

__device__ inline void dg_sizes(const DgArgs &a, uint64_t g, const DgStore &S, const DgGraph &G) {
  const uint32_t nout = dg_nout(S, G);
  a.g_size[g] = G.size;
  a.g_nout[g] = nout;
  a.g_bytes[g] = 2 + 13 * G.size + 6 * nout;
}

template <bool WRITE>
__global__ __launch_bounds__(DG_T) void k_dg_build(DgArgs a, uint64_t ng, DgOut o) {
  __shared__ uint64_t l_dec[DG_MAX * DG_T];
  __shared__ uint64_t l_rec[DG_RCAP * DG_T];
  __shared__ uint32_t l_rins[DG_RCAP * DG_T];
  __shared__ int32_t l_recv[DG_MAX * DG_T];
  __shared__ uint8_t l_tab[DG_P * DG_T];
  __shared__ uint8_t l_sup[DG_MAX * DG_T], l_fl[DG_MAX * DG_T], l_osz[DG_MAX * DG_T], l_omax[DG_MAX * DG_T];
  const uint32_t t = threadIdx.x;
  const uint64_t g = (uint64_t)blockIdx.x * DG_T + t;
  if (g >= ng) return;
  if (WRITE && a.g_big[g]) return;
  DgStore S{l_tab + t, l_dec + t, l_recv + t, l_sup + t, l_fl + t, l_osz + t, l_omax + t, l_rec + t,
            l_rins + t, DG_T, DG_RCAP};
  const DgGraph G = dg_replay(a, g, S);
  if (WRITE) {
    dg_emit(a, g, S, G, o);
  } else if (G.ok) {
    a.g_big[g] = 0;
    dg_sizes(a, g, S, G);
  } else {  // sized by the global-store pass
    a.g_big[g] = 1;
    a.g_size[g] = a.g_nout[g] = a.g_bytes[g] = 0;
  }
}

// Graphs with more than DG_RCAP outgoing records: big ranks [r0, r0 + DG_BIG_WINDOW).
template <bool WRITE>
__global__ __launch_bounds__(64) void k_dg_build_big(DgArgs a, uint64_t ng, uint64_t r0, DgOut o) {
  for (uint64_t g = (uint64_t)blockIdx.x * 64 + threadIdx.x; g < ng; g += (uint64_t)gridDim.x * 64) {
    if (!a.g_big[g]) continue;
    const uint64_t r = a.g_bigrank[g];
    if (r < r0 || r >= r0 + DG_BIG_WINDOW) continue;
    const DgStore S = dg_global_store(a.store + (r - r0) * a.store_words, a.DGS);
    const DgGraph G = dg_replay(a, g, S);
    if (WRITE) dg_emit(a, g, S, G, o);
    else dg_sizes(a, g, S, G);
  }
}

hipError_t launch_dg_build(const DgArgs &a, uint64_t ng, bool write, bool big, uint64_t r0, const DgOut &o,
                           hipStream_t s) {
  if (ng == 0) return hipSuccess;
  if (big) {
    const int grid = (int)std::min<uint64_t>((ng + 63) / 64, 4096);
    if (write) hipLaunchKernelGGL(k_dg_build_big<true>, dim3(grid), dim3(64), 0, s, a, ng, r0, o);
    else hipLaunchKernelGGL(k_dg_build_big<false>, dim3(grid), dim3(64), 0, s, a, ng, r0, o);
  } else {
    const dim3 grid((unsigned)((ng + DG_T - 1) / DG_T));
    if (write) hipLaunchKernelGGL(k_dg_build<true>, grid, dim3(DG_T), 0, s, a, ng, o);
    else hipLaunchKernelGGL(k_dg_build<false>, grid, dim3(DG_T), 0, s, a, ng, o);
  }
  return hipGetLastError();
}

hipError_t launch_dg_scans(const DgArgs &a, uint64_t ng, bool big_only, hipStream_t s) {
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
  if (!big_only) {
    q.in[3] = a.g_big;
    q.out[3] = a.g_bigrank;
    q.total[3] = &a.ctr->n_big;
    q.k = 4;
  }
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
