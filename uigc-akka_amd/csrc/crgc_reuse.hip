// crgc_reuse.hip — reclaiming the slots of collected shadows (gfx950).
//
// The reference drops a collected shadow from shadowMap at the sweep
// (ShadowGraph.java:276) and keeps its per-trace scans O(live).  Here slots are
// dense and every per-slot pass of a trace (pseudo-roots, dense frontier
// scans, sweep) covers [0, slot_top): without reuse a collected shadow's slot
// is reclaimed only by a rebuild, and a long run's slot range outgrows its live
// set (C2 over 200 wakeups: 4.17e7 slots for 3.15e7 live shadows, profiles/r5ao).
// So the committed sweeps' garbage slots (no NPE, the mark done) are listed
// (gslot), and once they make up 1/reuse_div of the slot range they are purged
// in one batch and listed free; the next merges' new shadows take them first
// (k_ids).  Purging at every sweep cost more than the dead slots it saves the
// per-slot passes on a short run (a purged slot ~1 ns once, a dead slot
// ~10 ps per trace: C2 1.249 / 1.273 against 1.177 / 1.216 ms per wakeup
// with reuse off, profiles/r6e); a dead slot waiting for its batch is exactly
// round 5's collected slot.  Unsharded graphs only: a sharded graph's proxies
// cache their homes' slots.
//
// What a reused slot must not inherit (the incarnation rule):
//   * its out-edges: their edge-table keys (slot << 32 | target) are
//     tombstoned, their reverse candidates in the targets' lists lose RC_POS
//     (the pull then never takes them), and pull hints naming the slot die;
//   * its in-edges (owner -> slot, from the slot's candidate list): the owners'
//     pool entries keep their place with count 0 (never traced, exported or
//     counted), their keys are tombstoned.  The owners' nonzero counts are left
//     as they are: the reference's `outgoing` keeps an entry for the removed
//     Shadow object, and `outgoing.size()` is what the traced-edge count sums
//     (a rebuild keeps nzdeg the same way);
//   * its per-slot state (counts, flags, supervisor, segments, LWW tags, hint);
//   * supervisor pointers to it: only halted live shadows (never expanded) can
//     point at a collected supervisor; they get SLOT_DEAD, as a rebuild gives.
// Collected ids stay tombstoned in the id table until its next rehash, so a
// reappearing id is a new incarnation (a new shadow), exactly as before.
//
//   k_purge        one wave per listed garbage slot: out-edges, then in-edges
//   k_sup_fix      halted live shadows whose supervisor was collected (only
//                  once an undo log has halted shadows)
//   k_free_list    the untaken rest of the free list, then the garbage slots
//                  (reset), into the next list; k_free_commit its counts
#include "crgc_host.hpp"

namespace crgc {

// The bucket of edge key (owner, target), or KEY_EMPTY.
__device__ inline uint64_t etab_find(const DevGraph &g, uint32_t owner, uint32_t target) {
  const uint64_t key = edge_key(owner, target);
  uint64_t h = mix64(key) & g.emask;
  for (uint64_t probe = 0; probe < g.ecap_tab; ++probe) {
    const uint4 b = load_bucket(&g.etab[h]);
    const uint64_t k = bucket_key(b);
    if (k == key) return h;
    if (k == KEY_EMPTY) break;
    h = (h + 1) & g.emask;
  }
  return KEY_EMPTY;
}

__device__ inline bool reclaim_commit(const Counters *c) { return c->mark_done && c->npe == 0; }

__global__ __launch_bounds__(256) void k_purge(DevGraph g, uint64_t ng) {
  const Counters *c = g.ctr;
  if (!reclaim_commit(c)) return;
  const uint32_t lane = lane_id();
  const uint64_t nw = (uint64_t)gridDim.x * 4;
  for (uint64_t i = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); i < ng; i += nw) {
    const uint32_t t = g.gslot[i];
    const uint2 ad = g.adj[t];
    // out-edges t -> u: key gone, u's candidate for t inert, u's hint to t gone
    for (uint32_t e = lane; e < ad.y; e += 64) {
      const uint32_t u = edge_target(g.pool[(uint64_t)ad.x + e]);
      if (u >= g.scap) continue;
      const uint64_t b = etab_find(g, t, u);
      if (b != KEY_EMPTY) {
        const uint32_t rev = g.etab[b].rev;
        g.etab[b].key = KEY_TOMB;
        const uint2 rd = g.radj[u];
        if (rev < rseg_cap(rd.y)) g.rpool[(uint64_t)rd.x + rev] = t;  // (without RC_POS)
      }
      if (g.par[u] == t) g.par[u] = SLOT_NONE;
    }
    // in-edges o -> t from t's candidates: the owner's entry stays with count 0
    const uint2 rd = g.radj[t];
    const uint32_t rl = min(rseg_len(rd.y), rseg_cap(rd.y));
    for (uint32_t e = lane; e < rl; e += 64) {
      const uint32_t o = g.rpool[(uint64_t)rd.x + e] & ~RC_POS;
      if (o == t || o >= g.pbase) continue;  // (a self-edge is an out-edge, above)
      const uint64_t b = etab_find(g, o, t);
      if (b == KEY_EMPTY) continue;  // an inert candidate of an earlier purge
      const uint32_t val = g.etab[b].val;
      g.etab[b].key = KEY_TOMB;
      const uint2 oad = g.adj[o];
      if (val < oad.y) *edge_count_ptr(g.pool, (uint64_t)oad.x + val) = 0;
    }
  }
}

// Halted live shadows are marked but never expanded (ShadowGraph.java:226-229),
// so theirs are the only supervisor pointers a sweep can leave dangling.
__global__ __launch_bounds__(256) void k_sup_fix(DevGraph g) {
  const Counters *c = g.ctr;
  if (!reclaim_commit(c)) return;
  const uint64_t top = c->slot_top;
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t v = (uint64_t)blockIdx.x * 256 + threadIdx.x; v < top; v += stride) {
    if ((g.flags[v] & (FL_ALIVE | FL_HALTED)) != (FL_ALIVE | FL_HALTED)) continue;
    const uint32_t s = g.sup[v];
    if (s < g.scap && !(g.flags[s] & FL_ALIVE)) g.sup[v] = SLOT_DEAD;
  }
}

// The next free list: the entries the merges since the last sweep did not take,
// then this sweep's garbage slots, each reset to a fresh slot's state
// (alloc_arrays' defaults).
__global__ __launch_bounds__(256) void k_free_list(DevGraph g, uint64_t n_purged) {
  const Counters *c = g.ctr;
  const uint64_t fn = c->free_n, fu = min((uint64_t)c->free_used, fn), rem = fn - fu;
  const uint64_t ng = reclaim_commit(c) ? n_purged : 0;
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < rem + ng; i += stride) {
    if (i < rem) {
      g.freel2[i] = g.freel[fu + i];
      continue;
    }
    const uint32_t t = g.gslot[i - rem];
    g.recv[t] = 0;
    g.sup[t] = SLOT_NONE;
    g.adj[t] = make_uint2(0, 0);
    g.vseq[t] = 0;
    g.sseq[t] = 0;
    g.nzdeg[t] = 0;
    g.radj[t] = make_uint2(0, 0);
    g.par[t] = SLOT_NONE;
    g.freel2[i] = t;
  }
}

__global__ void k_free_commit(Counters *c, uint64_t n_purged) {
  const uint64_t fn = c->free_n, fu = min((uint64_t)c->free_used, fn);
  const uint64_t ng = reclaim_commit(c) ? n_purged : 0;
  c->reused += fu;  // taken slots: their collected ids' tombstones stay in the id table
  c->free_n = fn - fu + ng;
  c->free_used = 0;
}

hipError_t launch_reclaim(const DevGraph &g, uint64_t slot_top, uint64_t n_purge, uint64_t n_free,
                          bool sup_fix, hipStream_t s) {
  launch_begin();
  if (!g.freel) return hipSuccess;
  if (n_purge) {
    hipLaunchKernelGGL(k_purge, dim3(grid_for(n_purge, 4, 4096)), dim3(256), 0, s, g, n_purge);
    if (sup_fix) hipLaunchKernelGGL(k_sup_fix, dim3(grid_for(slot_top, 256, 4096)), dim3(256), 0, s, g);
  }
  hipLaunchKernelGGL(k_free_list, dim3(grid_for(n_purge + n_free, 256, 4096)), dim3(256), 0, s, g, n_purge);
  hipLaunchKernelGGL(k_free_commit, dim3(1), dim3(1), 0, s, g.ctr, n_purge);
  return hipGetLastError();
}

}  // namespace crgc
