// crgc_edges.hip — the edge pipeline: outgoing[o][t] += d for a merge's edge
// atoms (ShadowGraph.updateOutgoing, ShadowGraph.java:64-73), as a partition by
// owner, then a segmented reduce with LDS-staged atomics per owner range.
//
// Absent == 0: a pair whose deltas sum to 0 changes nothing; zero counts that
// result from a merge are kept in their segment (never traced, never counted:
// nzdeg tracks the reference's outgoing.size(), :231) until a rebuild drops them.
//
//   1. k_ep_count / run_scan / k_ep_scatter: the atoms, partitioned by owner
//      (a hash of the slot to one of <= 1024 buckets; an LDS histogram per
//      block of atoms, a bucket-major scan of the block x bucket counts, a
//      scatter; <= 512 blocks split the exact atom count between them).
//   2. k_ep_owner: one workgroup per owner bucket — every atom of an owner is
//      in its workgroup, so the owner's segment, degree and nonzero count are
//      written without atomics.  1024 atoms at a time: the pairs are reduced in
//      an LDS hash table (LDS atomics); each distinct pair finds or inserts its
//      edge-table key; existing edges take the summed delta (a count that
//      changes sign updates its reverse candidate in place); new edges get a
//      rank among their owner's new edges (LDS atomics on an LDS owner table),
//      each owner's segment grows once (one pool allocation per workgroup per
//      round) and the new edges are written after its old degree.  Every new
//      edge appends its reverse candidate (owner | RC_POS) to its target's
//      candidate segment with one 64-bit atomic on radj[target] = {offset,
//      length}: the old length is the candidate's index, written at once when
//      it is below the segment's capacity.
//   3. The candidates past a capacity (a target whose segment fills up this
//      merge) go to an overflow list; k_rv_grow moves each such target's
//      segment to a power-of-two segment for its final length (one pool
//      allocation per workgroup) and k_rv_place writes them there.  Round 2
//      partitioned every new edge by target for this (two partition passes and
//      a target-bucket kernel); now only the overflow is handled apart.
// Pool, candidate pool and edge-table sizes follow the same bounds as before
// (ensure_capacity in crgc_api.hip).
#include "crgc_host.hpp"

namespace crgc {

constexpr int EP_THREADS = 256;     // partition kernels
constexpr int EP_WG = 1024;         // owner / target bucket kernels (2 workgroups per CU)
constexpr uint32_t EP_CH = 1024;    // atoms per round in a bucket workgroup (one per thread)
constexpr uint32_t EP_TAB = 2048;   // LDS pair / owner tables (load <= 1/2)
constexpr uint32_t EP_EXIST = 0xFFFFFFFFu;
constexpr uint32_t EP_SKIP = 0xFFFFFFFEu;
constexpr uint32_t EP_PENDING = 0x80000000u;  // etab rev: reverse atom (position) not yet appended
constexpr uint32_t EP_SMALL_COPY = 8;

__device__ inline bool ep_valid(uint32_t s) { return s < 0xFFFFFFF0u; }

__device__ inline uint32_t seg_cap_ep(uint32_t need) {
  uint32_t c = 4;
  while (c < need) c <<= 1;
  return c;
}

// ---- 1. partition ------------------------------------------------------------
// Slots go to buckets by a multiplicative hash: fresh slots are contiguous and
// take most of a wakeup's atoms, so ranges of slots would load a few buckets.
__device__ inline uint32_t ep_bucket(const EdgeArgs &a, uint32_t slot) {
  return (slot * 0x9E3779B1u) >> a.bshift;
}

// An atom (ao, at, ad) as (bucket of the owner, key o << 32 | t, delta).
__device__ inline bool ep_atom(const EdgeArgs &a, uint64_t i, uint64_t n, uint32_t &bucket, uint64_t &key,
                               uint32_t &val) {
  if (i >= n) return false;
  const int32_t d = a.atom_d[i];
  const uint32_t o = a.atom_o[i], t = a.atom_t[i];
  if (d == 0 || !ep_valid(o) || !ep_valid(t)) return false;
  bucket = ep_bucket(a, o);
  key = ((uint64_t)o << 32) | t;
  val = (uint32_t)d;
  return true;
}

// Atoms to partition: the merge's (exact count when the device has it).
__device__ inline uint64_t ep_count(const EdgeArgs &a) {
  // a batch refused for its offsets (or > F records) left unwritten atoms:
  // nothing of it is applied (the handle is poisoned by that error anyway)
  if (a.err && (*a.err & (ERR_BAD_OFFSETS | ERR_TOO_MANY))) return 0;
  return a.n_atoms_dev ? *a.n_atoms_dev : a.max_atoms;
}

// [begin, end) of bucket b in the partition (its total ends the last bucket)
__device__ inline uint64_t ep_end(const EdgeArgs &a, uint32_t b, int which) {
  return b + 1 == a.nbk ? a.tot[which] : a.hoff[(uint64_t)(b + 1) * a.nblk];
}

__global__ __launch_bounds__(EP_THREADS) void k_ep_count(EdgeArgs a) {
  extern __shared__ uint32_t hist[];  // [nbk]
  const uint64_t n = ep_count(a);
  if (blockIdx.x == 0 && threadIdx.x == 0) *a.n_ov = 0;  // k_ep_owner's overflow list
  for (uint32_t k = threadIdx.x; k < a.nbk; k += EP_THREADS) hist[k] = 0;
  __syncthreads();
  const uint64_t per = (n + a.nblk - 1) / a.nblk;
  const uint64_t i0 = (uint64_t)blockIdx.x * per, i1 = min(n, i0 + per);
  for (uint64_t i = i0 + threadIdx.x; i < i1; i += EP_THREADS) {
    uint32_t b;
    uint64_t key;
    uint32_t val;
    if (ep_atom(a, i, n, b, key, val)) atomicAdd(&hist[b], 1u);
  }
  __syncthreads();
  for (uint32_t k = threadIdx.x; k < a.nbk; k += EP_THREADS) a.hist[(uint64_t)k * a.nblk + blockIdx.x] = hist[k];
}

__global__ __launch_bounds__(EP_THREADS) void k_ep_scatter(EdgeArgs a) {
  extern __shared__ uint32_t cur[];  // [nbk]
  const uint64_t n = ep_count(a);
  for (uint32_t k = threadIdx.x; k < a.nbk; k += EP_THREADS) cur[k] = 0;
  __syncthreads();
  const uint64_t per = (n + a.nblk - 1) / a.nblk;
  const uint64_t i0 = (uint64_t)blockIdx.x * per, i1 = min(n, i0 + per);
  for (uint64_t i = i0 + threadIdx.x; i < i1; i += EP_THREADS) {
    uint32_t b;
    uint64_t key;
    uint32_t val;
    if (!ep_atom(a, i, n, b, key, val)) continue;
    const uint64_t at = a.hoff[(uint64_t)b * a.nblk + blockIdx.x] + atomicAdd(&cur[b], 1u);
    a.pk[at] = key;
    a.pv[at] = val;
  }
}

// ---- 2. owner buckets --------------------------------------------------------
// A segment that outgrows its capacity moves to a new power-of-two segment:
// a short one is copied by its own lane, longer ones by the whole wave.  Every
// lane of the wave calls (r = ~0: nothing to move).
template <typename T>
__device__ inline void ep_move(T *pool, uint32_t from, uint32_t len, uint32_t r) {
  const bool mv = r != 0xFFFFFFFFu;
  const bool small = mv && len <= EP_SMALL_COPY;
  if (small) {
    T x[EP_SMALL_COPY];
#pragma unroll
    for (uint32_t e = 0; e < EP_SMALL_COPY; ++e)
      if (e < len) x[e] = pool[(uint64_t)from + e];
#pragma unroll
    for (uint32_t e = 0; e < EP_SMALL_COPY; ++e)
      if (e < len) pool[(uint64_t)r + e] = x[e];
  }
  uint64_t big = __ballot(mv && !small);
  while (big) {
    const int k = __ffsll((unsigned long long)big) - 1;
    big &= big - 1;
    const uint32_t rk = __shfl(r, k), xk = __shfl(from, k), yk = __shfl(len, k);
    for (uint32_t e = lane_id(); e < yk; e += 64) pool[(uint64_t)rk + e] = pool[(uint64_t)xk + e];
  }
}

// A distinct pair is handled by the same thread before and after the owners'
// growth (thread i: plist[i]), so its sum, edge-table bucket and rank stay in
// that thread's registers; LDS holds the reduction and the owner table.
struct EpOwnerLds {
  uint64_t key[EP_TAB];   // pair o << 32 | t
  int32_t sum[EP_TAB];
  uint32_t okey[EP_TAB];  // owner table: owner slot (~0: free)
  uint32_t ocnt[EP_TAB];  // new edges of the owner in this round; after the growth, its
                          // segment offset + 1 (0: its new edges were dropped, pool full)
  int32_t onz[EP_TAB];    // change of the owner's nonzero count; after the growth,
                          // the owner's degree before its new edges
  uint32_t oseg[EP_TAB];  // owners with new edges: segment offset, and degree | log2(capacity)
  uint32_t oinf[EP_TAB];  // << 27 (ep_pack_inf), loaded by their new pairs' threads beside the
                          // existing pairs' count updates
  uint32_t plist[EP_CH];  // pair table entries in use
  uint32_t olist[EP_CH];  // owner table entries in use
  uint32_t np, nol, nnew;
};

// Degree and segment capacity (0 or a power of two >= 4) in one word; a degree
// of 2^27 or more (never seen) is marked for a reload from the arrays.
constexpr uint32_t EP_INF_RELOAD = 0xFFFFFFFFu;
__device__ inline uint32_t ep_pack_inf(uint32_t deg, uint32_t cap) {
  if (deg >= (1u << 27)) return EP_INF_RELOAD;
  return deg | ((cap ? (uint32_t)__builtin_ctz(cap) : 31u) << 27);
}

__device__ inline uint32_t ep_owner_slot(EpOwnerLds &L, uint32_t o) {
  uint32_t h = (uint32_t)mix64(o) & (EP_TAB - 1);
  for (;;) {
    const uint32_t k = atomicCAS(&L.okey[h], 0xFFFFFFFFu, o);
    if (k == 0xFFFFFFFFu) {
      L.olist[atomicAdd(&L.nol, 1u)] = h;
      return h;
    }
    if (k == o) return h;
    h = (h + 1) & (EP_TAB - 1);
  }
}

// All of a bucket's atoms are in one workgroup, hence every edge of its owners:
// the owners' segments, degrees and nonzero counts are written without atomics.
// Workgroup-scope visibility of earlier rounds' global writes (edge-table
// values, degrees) is the barrier's (one CU, one L1).
__global__ __launch_bounds__(EP_WG) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_ep_owner(DevGraph g, EdgeArgs a) {
  __shared__ EpOwnerLds L;
  const uint32_t b = blockIdx.x;
  const uint64_t a0 = a.hoff[(uint64_t)b * a.nblk], a1 = ep_end(a, b, 0);
  if (a0 == a1) return;
  for (uint32_t k = threadIdx.x; k < EP_TAB; k += EP_WG) {
    L.key[k] = KEY_EMPTY;
    L.sum[k] = 0;
    L.okey[k] = 0xFFFFFFFFu;
    L.ocnt[k] = 0;
    L.onz[k] = 0;
  }
  Counters *c = g.ctr;
  unsigned long long *const tops[1] = {&c->pool_top};
  const uint32_t tid = threadIdx.x;
  // this round's atom (one per thread), loaded during the previous round
  uint64_t nkey = 0;
  uint32_t nval = 0;
  if (a0 + tid < a1) {
    nkey = a.pk[a0 + tid];
    nval = a.pv[a0 + tid];
  }
  for (uint64_t c0 = a0; c0 < a1; c0 += EP_CH) {
    const uint32_t m = (uint32_t)min((uint64_t)EP_CH, a1 - c0);
    if (tid == 0) L.np = L.nol = L.nnew = 0;
    __syncthreads();
    // reduce the round's atoms (one per thread) per pair
    if (tid < m) {
      const uint64_t key = nkey;
      uint32_t h = (uint32_t)mix64(key) & (EP_TAB - 1);
      for (;;) {
        const uint64_t k = atomicCAS((unsigned long long *)&L.key[h], (unsigned long long)KEY_EMPTY,
                                     (unsigned long long)key);
        if (k == KEY_EMPTY) L.plist[atomicAdd(&L.np, 1u)] = h;
        if (k == KEY_EMPTY || k == key) break;
        h = (h + 1) & (EP_TAB - 1);
      }
      atomicAdd(&L.sum[h], (int32_t)nval);
    }
    __syncthreads();
    // the next round's atom, in flight with this round's probes
    if (c0 + EP_CH + tid < a1) {
      nkey = a.pk[c0 + EP_CH + tid];
      nval = a.pv[c0 + EP_CH + tid];
    }
    // each distinct pair (one per thread): its edge-table key; existing edges take the sum
    const uint32_t np = L.np;
    const uint32_t ph = tid < np ? L.plist[tid] : 0;
    const uint64_t pkey = tid < np ? L.key[ph] : 0;
    const int32_t psum = tid < np ? L.sum[ph] : 0;
    uint32_t rk = EP_SKIP, pbk = 0;
    if (tid < np && psum != 0) {  // absent == 0: a zero sum changes nothing
      const int32_t d = psum;
      const uint32_t o = (uint32_t)(pkey >> 32), t = (uint32_t)pkey;
      bool ins = false;
      uint32_t v = 0, rv = 0;
      // the owner's segment, loaded beside the probe (an existing edge needs it)
      const uint32_t seg = g.adj[o].x;
      const uint64_t bk = edge_find_or_insert(g, pkey, &ins, &v, &rv);
      if (bk != KEY_EMPTY) {  // else the table is full: ERR_ETAB_FULL is set
        pbk = (uint32_t)bk;
        const uint32_t oh = ep_owner_slot(L, o);
        if (!ins) {
          int32_t *p = edge_count_ptr(g.pool, (uint64_t)seg + v);
          const int32_t old = *p;
          const int32_t now = (int32_t)((uint32_t)old + (uint32_t)d);
          *p = now;
          if ((old != 0) != (now != 0)) atomicAdd(&L.onz[oh], now != 0 ? 1 : -1);
          if ((old > 0) != (now > 0)) {  // the reverse candidate follows the count's sign
            const uint32_t r = rv;  // loaded with the key: this workgroup owns the pair
            const uint32_t cand = o | (now > 0 ? RC_POS : 0u);
            if (r != 0xFFFFFFFFu && (r & EP_PENDING)) {
              a.rv_o[r & ~EP_PENDING] = cand;  // still in the overflow list
            } else {
              const uint2 rd = g.radj[t];  // offset and capacity in one load
              if (r < rseg_cap(rd.y)) g.rpool[(uint64_t)rd.x + r] = cand;
            }
            if (now <= 0 && g.par[t] == o) g.par[t] = SLOT_NONE;  // the pull hint dies with the count
          }
          rk = EP_EXIST;
        } else {
          // a new edge: its owner's segment and degree (for the growth; the
          // capacity follows from the degree), beside the existing pairs' updates
          const uint2 oad = g.adj[o];
          L.oseg[oh] = oad.x;  // every new pair of the owner stores the same values
          L.oinf[oh] = ep_pack_inf(oad.y, seg_cap(oad.y));
          rk = atomicAdd(&L.ocnt[oh], 1u);
          atomicAdd(&L.nnew, 1u);
        }
      }
    }
    __syncthreads();
    // owners with new edges (one per thread): one growth each, one pool
    // allocation per workgroup
    {
      const uint32_t nol = L.nol;
      const uint32_t oh = tid < nol ? L.olist[tid] : 0;
      const uint32_t o = tid < nol ? L.okey[oh] : 0;
      const uint32_t nn = tid < nol ? L.ocnt[oh] : 0;
      uint2 ad = make_uint2(0, 0);
      uint32_t want = 0;
      if (nn) {
        const uint32_t inf = L.oinf[oh];
        uint32_t cap;
        if (inf == EP_INF_RELOAD) {
          ad = g.adj[o];
          cap = seg_cap(ad.y);
        } else {
          ad = make_uint2(L.oseg[oh], inf & ((1u << 27) - 1));
          cap = (inf >> 27) == 31 ? 0u : (1u << (inf >> 27));
        }
        if (ad.y + nn > cap) want = seg_cap_ep(ad.y + nn);
      }
      const uint32_t v1[1] = {want};
      unsigned long long offs[1];
      block_append<1>(tops, v1, offs);
      uint32_t r = 0xFFFFFFFFu, add = nn;
      if (want) {
        if (offs[0] + want > g.pcap) {
          set_err(c, ERR_POOL_FULL);  // the owner's new edges are dropped
          add = 0;
        } else {
          r = (uint32_t)offs[0];
        }
      }
      ep_move(g.pool, ad.x, ad.y, r);
      if (tid < nol) {
        if (r != 0xFFFFFFFFu) ad.x = r;  // capacity: seg_cap of the new degree (= want)
        L.ocnt[oh] = add ? ad.x + 1 : 0u;  // (LDS: two 1024-thread workgroups per CU need <= 80 KiB each)
        if (add) g.adj[o] = make_uint2(ad.x, ad.y + add);
        const int32_t dz = L.onz[oh] + (int32_t)add;  // new edges have nonzero counts
        if (dz) atomicAdd(&g.nzdeg[o], (uint32_t)dz);  // no return: nothing waits for it
        L.onz[oh] = (int32_t)ad.y;
      }
    }
    __syncthreads();
    // the new edges, after their owner's old degree; each appends its reverse
    // candidate to its target's segment (or to the overflow list)
    uint32_t ovf = 0, nt = 0, ridx = 0, cand = 0, nbk = 0, nidx = 0;
    if (tid < np && rk < EP_SKIP) {  // not EP_SKIP / EP_EXIST
      const uint32_t o = (uint32_t)(pkey >> 32);
      nt = (uint32_t)pkey;
      const uint32_t oh = ep_owner_slot(L, o);
      if (L.ocnt[oh]) {  // else the pool is full (error set)
        nidx = (uint32_t)L.onz[oh] + rk;
        const int32_t d = psum;
        nbk = pbk;
        g.pool[(uint64_t)(L.ocnt[oh] - 1) + nidx] = pack_edge(nt, d);
        cand = o | (d > 0 ? RC_POS : 0u);
        // the append returns the segment's offset, length and capacity at once
        const unsigned long long old = atomicAdd((unsigned long long *)&g.radj[nt], 1ull << 32);
        const uint32_t ry = (uint32_t)(old >> 32);
        ridx = rseg_len(ry);
        if (ridx >= RLEN_MASK) set_err(c, ERR_POOL_FULL);  // 2^27 candidates on one shadow: unsupported
        if (ridx < rseg_cap(ry)) {
          g.rpool[(uint64_t)(uint32_t)old + ridx] = cand;
          g.etab[nbk].val = nidx;
          g.etab[nbk].rev = ridx;
        } else {
          ovf = 1;
        }
      }
    }
    {
      unsigned long long *const otop[1] = {a.n_ov};
      const uint32_t vo[1] = {ovf};
      unsigned long long ob[1];
      block_append<1>(otop, vo, ob);
      if (ovf) {
        const uint64_t q = ob[0];
        a.rv_t[q] = nt;
        a.rv_i[q] = ridx;
        a.rv_o[q] = cand;
        a.rv_b[q] = nbk;
        g.etab[nbk].val = nidx;
        g.etab[nbk].rev = EP_PENDING | (uint32_t)q;
      }
    }
    __syncthreads();
    if (tid == 0 && L.nnew) atomicAdd(&c->etab_used, (unsigned long long)L.nnew);
    if (tid < np) {
      L.key[ph] = KEY_EMPTY;
      L.sum[ph] = 0;
    }
    if (tid < L.nol) {
      const uint32_t oh = L.olist[tid];
      L.okey[oh] = 0xFFFFFFFFu;
      L.ocnt[oh] = 0;
      L.onz[oh] = 0;
    }
    __syncthreads();
  }
}

// ---- 3. overflow candidates ---------------------------------------------------
// A target whose candidate segment filled up during k_ep_owner: the candidate
// with index == the old capacity (exactly one per such target: indices come
// from one counter) moves the segment to a power-of-two segment for the final
// length; k_rv_place then writes every overflow candidate at its index.
constexpr int RV_THREADS = 256;

__global__ __launch_bounds__(RV_THREADS) void k_rv_grow(DevGraph g, EdgeArgs a) {
  const uint64_t n = *a.n_ov;
  Counters *c = g.ctr;
  unsigned long long *const tops[1] = {&c->rpool_top};
  const uint64_t stride = (uint64_t)gridDim.x * RV_THREADS;
  for (uint64_t b0 = (uint64_t)blockIdx.x * RV_THREADS; b0 < n; b0 += stride) {  // uniform per block
    const uint64_t q = b0 + threadIdx.x;
    uint32_t t = 0, cap = 0, want = 0, len = 0;
    uint2 rd = make_uint2(0, 0);
    if (q < n) {
      t = a.rv_t[q];
      rd = g.radj[t];  // final length: every append of the merge is done
      cap = rseg_cap(rd.y);
      len = rseg_len(rd.y);
      if (a.rv_i[q] == cap) want = seg_cap_ep(len);  // the first overflow of t
    }
    const uint32_t v1[1] = {want};
    unsigned long long offs[1];
    block_append<1>(tops, v1, offs);
    uint32_t r = 0xFFFFFFFFu;
    if (want) {
      if (offs[0] + want > g.rpcap) set_err(c, ERR_POOL_FULL);  // candidates dropped: the handle is poisoned
      else r = (uint32_t)offs[0];
    }
    ep_move(g.rpool, rd.x, cap, r);  // the candidates that fitted
    if (r != 0xFFFFFFFFu) g.radj[t] = make_uint2(r, rseg_pack(len, want));
  }
}

__global__ __launch_bounds__(RV_THREADS) void k_rv_place(DevGraph g, EdgeArgs a) {
  const uint64_t n = *a.n_ov;
  const uint64_t stride = (uint64_t)gridDim.x * RV_THREADS;
  for (uint64_t q = (uint64_t)blockIdx.x * RV_THREADS + threadIdx.x; q < n; q += stride) {
    const uint32_t t = a.rv_t[q], i = a.rv_i[q];
    const uint2 rd = g.radj[t];
    if (i >= rseg_cap(rd.y)) continue;  // its growth failed (ERR_POOL_FULL)
    g.rpool[(uint64_t)rd.x + i] = a.rv_o[q];
    g.etab[a.rv_b[q]].rev = i;
  }
}

// ---- driver --------------------------------------------------------------------
hipError_t launch_edges(const DevGraph &g, const EdgeArgs &a, hipStream_t s) {
  launch_begin();
  if (a.max_atoms == 0) return hipSuccess;
  const size_t lds_hist = (size_t)a.nbk * 4;
  const dim3 pgrid((unsigned)a.nblk);
  ScanSet q{};
  q.k = 1;
  q.n = (uint64_t)a.nbk * a.nblk;
  q.nb = (q.n + 1023) / 1024;
  q.in[0] = a.hist;
  q.out[0] = a.hoff;
  q.total[0] = a.tot;
  q.bsum = a.bsum;
  // forward: partition by owner, then the owner ranges
  hipLaunchKernelGGL(k_ep_count, pgrid, dim3(EP_THREADS), lds_hist, s, a);
  if (hipError_t e = run_scan(q, s)) return e;
  hipLaunchKernelGGL(k_ep_scatter, pgrid, dim3(EP_THREADS), lds_hist, s, a);
  hipLaunchKernelGGL(k_ep_owner, dim3(a.nbk), dim3(EP_WG), 0, s, g, a);
  // the reverse candidates that did not fit their targets' segments
  const int og = grid_for(a.max_atoms, RV_THREADS, 512);
  hipLaunchKernelGGL(k_rv_grow, dim3(og), dim3(RV_THREADS), 0, s, g, a);
  hipLaunchKernelGGL(k_rv_place, dim3(og), dim3(RV_THREADS), 0, s, g, a);
  return hipGetLastError();
}

}  // namespace crgc
