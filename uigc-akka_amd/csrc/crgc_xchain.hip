// crgc_xchain.hip — deep marks on a sharded graph: the replicated chain closure.
//
// A sharded mark runs in rounds (crgc_api.hip mark_all): a local fixpoint of
// the level kernels, then every shard sends the proxies it marked to their
// homes.  Along a chain whose links are hash-partitioned over G shards about
// (G-1)/G of the links cross shards, so a chain of L links costs about L
// rounds — two host synchronisations and an exchange each.  Once a mark has
// run `xclosure_after` rounds and its rounds have become narrow, the shards
// switch to this closure, which needs O(log L) local doubling rounds and one
// exchange per alternation between chains and branching shadows:
//
//   1. every shard describes its home shadows in one global index space
//      (shard r's slots at off[r] .. off[r] + P[r]): the unique traceable
//      out-target nx (ShadowGraph.java:231-241, count > 0, a proxy resolved to
//      its home slot), the supervisor sp (:258-267), whether it has several
//      out-targets (cx), whether it is marked, and which of its marks just
//      arrived unexpanded (the round's imported marks: pending);
//   2. one all-gather of those arrays: every shard now holds the successor
//      structure of the whole graph;
//   3. every shard closes the marked set along nx and sp by pointer doubling
//      (crgc_chain.hip's algorithm over global indices) — identical work on
//      every shard, so identical results, with no exchange; shadows with several
//      out-targets that become marked are expanded edge by edge by their home
//      shard only, which broadcasts the shadows that marks (all-gather of a
//      list), and the closure repeats until an iteration marks nothing;
//   4. every shard keeps the marks of its own range.
// Halted shadows are marked, never expanded (:226-229); investigate mode
// (:302-330) follows no supervisor edges.  The marked set is the least set
// closed under the traceable edges that contains the marks the closure started
// from, so it equals what the rounds would have reached.
#include "crgc_host.hpp"

namespace crgc {

constexpr uint32_t GC_NONE = 0xFFFFFFFFu;
constexpr uint32_t GC_COMPLEX = 0xFFFFFFFEu;
constexpr int GC_STAT_SUP = 1;  // crgc_trace.hip STAT_SUP of block 0's partials

__device__ inline bool gbit(const uint32_t *bm, uint64_t v) { return (bm[v >> 5] >> (v & 31)) & 1u; }

// A local slot as a global index: a home slot of this shard, or a proxy's
// home slot (PHS_ABSENT: its home holds no live shadow — nothing to mark).
__device__ inline uint32_t gc_global(const DevGraph &g, const XcArgs &x, uint32_t t, bool *unresolved) {
  if (!(g.flags[t] & FL_PROXY)) return (uint32_t)(x.off[x.me] + t);
  const uint32_t p = g.phs[t];
  if (p == PHS_NONE) {
    *unresolved = true;
    return GC_NONE;
  }
  if (p == PHS_ABSENT) return GC_NONE;
  const uint32_t home = g.psh[t];
  return (uint32_t)(x.off[home] + p);
}

// Received marks of this round (the payload k_ximport would import as
// candidates): marked now, and remembered as pending (not yet expanded).
// Returns whether v is newly marked with a supervisor edge to follow (:258,
// counted like the level kernels count a frontier shadow's).
__device__ inline uint32_t gc_import(const DevGraph &g, const XcArgs &x, uint32_t v, uint64_t top) {
  if (v >= top) return 0;
  const uint8_t f = g.flags[v];
  if ((f & (FL_ALIVE | FL_PROXY)) != FL_ALIVE) return 0;
  const uint32_t bit = 1u << (v & 31);
  if (atomicOr(&g.vis[v >> 5], bit) & bit) return 0;
  atomicOr(&x.seed[v >> 5], bit);
  return (!(f & FL_HALTED) && !x.investigate && g.sup[v] < 0xFFFFFFF0u) ? 1u : 0u;
}

__global__ __launch_bounds__(256) void k_xc_import(DevGraph g, XcArgs x, const char *recv, XRecv r) {
  const uint64_t top = g.ctr->slot_top;
  const uint64_t total = r.start[r.G], stride = (uint64_t)gridDim.x * 256;
  uint32_t su = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += stride) {
    uint32_t s = 0;
    while (s + 1 < r.G && r.start[s + 1] <= i) ++s;
    const uint64_t k = i - r.start[s];
    const char *seg = recv + r.off[s];
    if (k < r.n_id[s]) {
      const uint32_t v = id_find(g, ((const uint64_t *)seg)[k]);
      if (v < 0xFFFFFFF0u) su += gc_import(g, x, v, top);
      continue;
    }
    const uint64_t j = k - r.n_id[s];
    const uint32_t w = ((const uint32_t *)(seg + 8 * r.n_id[s]))[j];
    if (!r.bitmap[s]) su += gc_import(g, x, w, top);
    else
      for (uint32_t m = w; m; m &= m - 1) su += gc_import(g, x, (uint32_t)(j * 32) + __ffs(m) - 1, top);
  }
  const uint32_t t = wave_sum(su);
  if (lane_id() == 0 && t) atomicAdd((unsigned long long *)&g.blkstat[GC_STAT_SUP], (unsigned long long)t);
}

// Step 1: this shard's block of the global arrays (one wave per 64 slots, so
// bitmap words are written whole).  `x.lnx` / `x.lsp` / the three bitmaps are
// the send buffers of the all-gathers.
__global__ __launch_bounds__(256) void k_xc_local(DevGraph g, XcArgs x, uint64_t P) {
  const uint64_t top = g.ctr->slot_top;
  const uint64_t nwv = (uint64_t)gridDim.x * 4;
  bool unresolved = false;
  for (uint64_t c0 = ((uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 64; c0 < P; c0 += nwv * 64) {
    const uint64_t v = c0 + lane_id();
    uint32_t nx = GC_NONE, sp = GC_NONE;
    bool cplx = false, marked = false, home = false;
    if (v < top) {
      const uint8_t f = g.flags[v];
      home = (f & (FL_ALIVE | FL_PROXY)) == FL_ALIVE;
      marked = home && gbit(g.vis, v);
      if (home && !(f & FL_HALTED)) {
        const uint2 ad = g.adj[v];
        uint32_t first = GC_NONE;  // local slot of the first traceable target
        for (uint32_t e = 0; e < ad.y && !cplx; ++e) {
          const uint64_t ed = g.pool[(uint64_t)ad.x + e];
          const uint32_t t = edge_target(ed);
          if (edge_count(ed) <= 0 || t == (uint32_t)v) continue;
          if (first == GC_NONE) first = t;
          else if (t != first) cplx = true;
        }
        if (!cplx && first != GC_NONE) nx = gc_global(g, x, first, &unresolved);
        const uint32_t s = g.sup[v];
        if (!x.investigate && s < 0xFFFFFFF0u) sp = gc_global(g, x, s, &unresolved);
      }
    }
    if (v < P) {
      x.lnx[v] = cplx ? GC_COMPLEX : nx;
      x.lsp[v] = sp;
    }
    const uint64_t bm = __ballot(marked), bc = __ballot(cplx);
    const uint64_t bs = __ballot(home && v < top && gbit(x.seed, v));
    if (lane_id() == 0) {
      const uint64_t w = c0 >> 5;
      x.lvis[w] = (uint32_t)bm;
      x.lvis[w + 1] = (uint32_t)(bm >> 32);
      x.lcx[w] = (uint32_t)bc;
      x.lcx[w + 1] = (uint32_t)(bc >> 32);
      x.lpb[w] = (uint32_t)(bs & bc);
      x.lpb[w + 1] = (uint32_t)((bs & bc) >> 32);
    }
  }
  if (__ballot(unresolved) && lane_id() == 0) x.flag[0] = 1;  // a proxy without a home slot: no closure
}

// Marks global index t; a newly marked branching shadow becomes pending.
__device__ inline bool gc_mark(const XcArgs &x, uint32_t *pb, uint32_t t) {
  const uint32_t bit = 1u << (t & 31);
  if (x.gvis[t >> 5] & bit) return false;
  if (atomicOr(&x.gvis[t >> 5], bit) & bit) return false;
  if (gbit(x.gcx, t)) atomicOr(&pb[t >> 5], bit);
  return true;
}

// One doubling round over the global arrays (crgc_chain.hip k_chain_jump):
// marked u marks src[u]; dst[u] = src[src[u]].  Exits at once after a round of
// its sequence that marked nothing.
__global__ __launch_bounds__(256) void k_xc_jump(XcArgs x, const uint32_t *src, uint32_t *dst, uint32_t fi,
                                                 int first) {
  if (!first && x.flag[fi - 1] == 0) return;
  uint32_t mine = 0;
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t u = (uint64_t)blockIdx.x * 256 + threadIdx.x; u < x.N; u += stride) {
    const uint32_t j = src[u];
    uint32_t jj = j;
    if (j < GC_COMPLEX) {
      if (gbit(x.gvis, u)) mine += gc_mark(x, x.gpb_in, j) ? 1u : 0u;
      jj = src[j];
    }
    dst[u] = jj;
  }
  if (wave_sum(mine) && lane_id() == 0) x.flag[fi] = 1;
}

// Pending branching shadows of this shard's range (the other shards expand
// theirs): every positive out-edge; the shadows it marks are listed for the
// other shards, the branching ones among them pending for the next iteration.
// All pending bits are cleared (every shard clears the whole map).
__global__ __launch_bounds__(256) void k_xc_expand(DevGraph g, XcArgs x) {
  const uint64_t words = x.N / 32, lo = x.off[x.me] / 32, hi = (x.off[x.me] + x.P_me) / 32;
  const int lane = lane_id();
  const uint64_t nwv = (uint64_t)gridDim.x * 4;
  bool unresolved = false;
  for (uint64_t w0 = ((uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 64; w0 < words; w0 += nwv * 64) {
    const uint64_t w = w0 + lane;
    uint32_t bits = w < words ? x.gpb_in[w] : 0u;
    if (bits) x.gpb_in[w] = 0;
    if (w < lo || w >= hi) bits = 0;
    uint64_t busy = __ballot(bits != 0);
    while (busy) {
      const int k = __ffsll((unsigned long long)busy) - 1;
      busy &= busy - 1;
      uint32_t kb = __shfl(bits, k);
      while (kb) {
        const uint64_t gi = (w0 + k) * 32 + (__ffs(kb) - 1);
        kb &= kb - 1;
        const uint32_t v = (uint32_t)(gi - x.off[x.me]);
        if ((g.flags[v] & (FL_ALIVE | FL_PROXY | FL_HALTED)) != FL_ALIVE) continue;
        const uint2 ad = g.adj[v];
        for (uint32_t e = lane; e < ad.y; e += 64) {
          const uint64_t ed = g.pool[(uint64_t)ad.x + e];
          if (edge_count(ed) <= 0) continue;
          const uint32_t t = gc_global(g, x, edge_target(ed), &unresolved);
          if (t < GC_COMPLEX && gc_mark(x, x.gpb_out, t)) {
            const unsigned long long at = atomicAdd(x.xl_n, 1ull);
            if (at < x.N) x.xl[at] = t;
          }
        }
      }
    }
  }
  if (__ballot(unresolved) && lane_id() == 0) x.flag[0] = 1;
}

// The other shards' expansion marks (every shard applies every list, its own
// included: idempotent).
__global__ __launch_bounds__(256) void k_xc_apply(XcArgs x, const uint32_t *list, uint64_t n, uint32_t fi) {
  uint32_t mine = 0;
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
    const uint32_t t = list[i];
    if (t < x.N) mine += gc_mark(x, x.gpb_out, t) ? 1u : 0u;
  }
  if (wave_sum(mine) && lane_id() == 0) x.flag[fi] = 1;
}

// Step 4: this shard's range back into its marked bitmap; the supervisor edges
// of the shadows the closure marked (:258) into the level statistics.
__global__ __launch_bounds__(256) void k_xc_finish(DevGraph g, XcArgs x) {
  const uint64_t top = g.ctr->slot_top;
  const uint64_t words = (x.P_me + 31) / 32, base = x.off[x.me] / 32;
  uint64_t su = 0;
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t w = (uint64_t)blockIdx.x * 256 + threadIdx.x; w < words; w += stride) {
    const uint32_t gv = x.gvis[base + w];
    const uint32_t old = g.vis[w];
    uint32_t add = gv & ~old;
    if (!add) continue;
    uint32_t keep = 0;
    for (uint32_t m = add; m; m &= m - 1) {
      const uint32_t j = __ffs(m) - 1;
      const uint64_t v = w * 32 + j;
      if (v >= top) continue;
      const uint8_t f = g.flags[v];
      if ((f & (FL_ALIVE | FL_PROXY)) != FL_ALIVE) continue;
      keep |= 1u << j;
      if (!(f & FL_HALTED) && !x.investigate && g.sup[v] < 0xFFFFFFF0u) ++su;
    }
    if (keep) g.vis[w] = old | keep;
  }
  __shared__ unsigned long long s_su;
  if (threadIdx.x == 0) s_su = 0;
  __syncthreads();
  if (su) atomicAdd(&s_su, (unsigned long long)su);
  __syncthreads();
  if (threadIdx.x == 0 && s_su) atomicAdd((unsigned long long *)&g.blkstat[GC_STAT_SUP], s_su);
}

hipError_t launch_xclosure(const DevGraph &g, const XcArgs &x, int step, const void *p0, uint32_t *p1, uint64_t n,
                           uint32_t fi, int first, hipStream_t s) {
  launch_begin();
  switch (step) {
    case 0: {  // import this round's received marks
      const XRecv *r = (const XRecv *)p1;
      const uint64_t total = r->start[r->G];
      if (total)
        hipLaunchKernelGGL(k_xc_import, dim3(grid_for(total, 256, 4096)), dim3(256), 0, s, g, x, (const char *)p0,
                           *r);
      break;
    }
    case 1:
      hipLaunchKernelGGL(k_xc_local, dim3(grid_for((x.P_me + 63) / 64, 4, 4096)), dim3(256), 0, s, g, x, x.P_me);
      break;
    case 2:
      hipLaunchKernelGGL(k_xc_jump, dim3(grid_for(x.N, 256, 4096)), dim3(256), 0, s, x, (const uint32_t *)p0, p1,
                         fi, first);
      break;
    case 3:
      hipLaunchKernelGGL(k_xc_expand, dim3(grid_for((x.N / 32 + 63) / 64, 4, 4096)), dim3(256), 0, s, g, x);
      break;
    case 4:
      if (n)
        hipLaunchKernelGGL(k_xc_apply, dim3(grid_for(n, 256, 4096)), dim3(256), 0, s, x, (const uint32_t *)p0, n,
                           fi);
      break;
    default:
      hipLaunchKernelGGL(k_xc_finish, dim3(grid_for((x.P_me + 31) / 32, 256, 4096)), dim3(256), 0, s, g, x);
      break;
  }
  return hipGetLastError();
}

}  // namespace crgc
