// crgc_trace.hip — ShadowGraph.trace on gfx950 (ShadowGraph.java:205-289).
//
// Mark = level-synchronous reachability over
//   { (o -> t) : outgoing[o][t] > 0 }  U  { (c -> supervisor(c)) }
// from the pseudo-roots, never expanding halted shadows (:226-229).
// Reachability does not depend on visiting order, so a level-synchronous
// sweep marks exactly the reference's `to` set.
//
// Frontier representation, no atomics on the per-edge path:
//   vis     1 bit / slot   marked set as of the start of the level
//   front   1 byte / slot  candidates for the next level; discovered targets
//                          get a plain byte store (idempotent, so concurrent
//                          stores from any XCD merge correctly at write-back)
//   dirty   1 byte / 2048 slots, only in sparse levels: which blocks to scan
// A wave owns 2048 consecutive slots (32 per lane = one vis word per lane).
// It turns its candidate bytes into new frontier bits (cand & ~vis), sets
// them in vis (it is the only writer of those words), compacts the frontier
// slots into LDS with a wave scan of popcounts, and expands them with a
// load-balanced merge over the concatenated edge segments (degree scan +
// binary search in LDS), 64 edges per step.
#include "crgc_host.hpp"

namespace crgc {

__device__ inline bool sparse_level(const Counters *c, int L, uint32_t thr) {
  if (L <= 1) return false;
  return c->ring[(L - 2) % LEVEL_RING] < thr;
}

__device__ inline void wave_lds_fence() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ inline void mark_target(const DevGraph &g, uint8_t *Fn, uint8_t *Dn, bool sp_next,
                                   uint32_t t) {
  const uint32_t w = g.vis[t >> 5];
  if (!((w >> (t & 31)) & 1u)) {
    Fn[t] = 1;
    if (sp_next) Dn[t >> 11] = 1;
  }
}

template <bool ROOTS, bool INVESTIGATE>
__global__ __launch_bounds__(256) void k_level(DevGraph g, LevelArgs a) {
  __shared__ uint32_t s_front[4][BLK_SLOTS];
  __shared__ uint32_t s_start[4][64];
  __shared__ uint32_t s_off[4][64];
  Counters *c = g.ctr;
  const int L = a.level;
  if (blockIdx.x == 0 && threadIdx.x == 0) c->ring[(L + 1) % LEVEL_RING] = 0;
  if (!ROOTS && c->ring[(L - 1) % LEVEL_RING] == 0) return;  // previous level was empty
  const bool sp_cur = !ROOTS && sparse_level(c, L, a.sparse_thresh);
  const bool sp_next = sparse_level(c, L + 1, a.sparse_thresh);
  const uint64_t slot_top = c->slot_top;
  const uint32_t nblk = (uint32_t)((slot_top + BLK_SLOTS - 1) / BLK_SLOTS);
  const int wv = threadIdx.x >> 6;
  const int lane = lane_id();
  const uint32_t gw = blockIdx.x * 4 + wv;
  const uint32_t nw = gridDim.x * 4;
  uint8_t *Fc = g.front[L & 1];
  uint8_t *Fn = g.front[(L + 1) & 1];
  uint8_t *Dc = g.dirty[L & 1];
  uint8_t *Dn = g.dirty[(L + 1) & 1];
  uint32_t n_front = 0, n_edges = 0, n_sup = 0;

  for (uint32_t blk = gw; blk < nblk; blk += nw) {
    if (sp_cur && Dc[blk] == 0) continue;
    const uint64_t base = (uint64_t)blk * BLK_SLOTS + (uint64_t)lane * 32;
    const uint32_t word = g.vis[(uint64_t)blk * 64 + lane];
    uint32_t m = 0;
    if (ROOTS) {
      const uint4 f4[2] = {*(const uint4 *)(g.flags + base), *(const uint4 *)(g.flags + base + 16)};
      const uint8_t *fb = (const uint8_t *)f4;
#pragma unroll
      for (int j = 0; j < 32; ++j) {
        const uint8_t f = fb[j];
        if (!(f & FL_ALIVE)) continue;
        bool root;
        if (INVESTIGATE) {
          // investigateRemotelyHeldActors: every shadow at `location` (:305-310)
          root = (uint16_t)(g.vid[base + j] >> 48) == a.location;
        } else {
          // isPseudoRoot (:201-203)
          root = ((f & (FL_ROOT | FL_BUSY)) || !(f & FL_INTERNED) || g.recv[base + j] != 0) &&
                 !(f & FL_HALTED);
        }
        if (root) m |= 1u << j;
      }
    } else {
      uint4 *fp = (uint4 *)(Fc + base);
      const uint4 x0 = fp[0], x1 = fp[1];
      const uint32_t xs[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
      uint32_t bits = 0;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const uint32_t v = xs[q];
        bits |= ((v & 0xFFu) ? 1u : 0u) << (4 * q);
        bits |= ((v & 0xFF00u) ? 1u : 0u) << (4 * q + 1);
        bits |= ((v & 0xFF0000u) ? 1u : 0u) << (4 * q + 2);
        bits |= ((v & 0xFF000000u) ? 1u : 0u) << (4 * q + 3);
      }
      if (bits) {
        fp[0] = make_uint4(0, 0, 0, 0);
        fp[1] = make_uint4(0, 0, 0, 0);
      }
      m = bits & ~word;
    }
    if (m) g.vis[(uint64_t)blk * 64 + lane] = word | m;
    if (sp_cur && lane == 0) Dc[blk] = 0;

    // Compact this block's frontier slots into LDS (ballot/popc scan).
    const uint32_t cnt = __popc(m);
    const uint32_t incl = wave_incl_scan(cnt);
    const uint32_t total = __shfl(incl, 63);
    uint32_t pos = incl - cnt;
    while (m) {
      const int j = __ffs(m) - 1;
      m &= m - 1;
      s_front[wv][pos++] = (uint32_t)(base + j);
    }
    n_front += cnt;  // per lane; summed over the wave below
    wave_lds_fence();

    // Expand, 64 frontier shadows at a time.
    for (uint32_t c0 = 0; c0 < total; c0 += 64) {
      const uint32_t idx = c0 + lane;
      const bool valid = idx < total;
      const uint32_t v = valid ? s_front[wv][idx] : 0;
      const uint8_t f = valid ? g.flags[v] : 0;
      const bool expand = valid && !(f & FL_HALTED);
      const uint2 ad = expand ? g.adj[v] : make_uint2(0, 0);
      if (!INVESTIGATE && expand) {
        const uint32_t s = g.sup[v];  // supervisor edge (:258-267)
        if (s < 0xFFFFFFF0u) {  // not null, not collected
          n_sup++;
          mark_target(g, Fn, Dn, sp_next, s);
        }
      }
      const uint32_t deg = ad.y;
      const uint32_t dincl = wave_incl_scan(deg);
      const uint32_t dtot = __shfl(dincl, 63);
      wave_lds_fence();
      s_start[wv][lane] = dincl - deg;
      s_off[wv][lane] = ad.x;
      wave_lds_fence();
      for (uint32_t e = lane; e < dtot; e += 64) {
        int lo = 0, hi = 63;
        while (lo < hi) {
          const int mid = (lo + hi + 1) >> 1;
          if (s_start[wv][mid] <= e) lo = mid;
          else hi = mid - 1;
        }
        const uint64_t ptr = (uint64_t)s_off[wv][lo] + (e - s_start[wv][lo]);
        const uint64_t ed = g.pool[ptr];
        const int32_t cntv = edge_count(ed);
        n_edges += cntv != 0;
        if (cntv > 0) mark_target(g, Fn, Dn, sp_next, edge_target(ed));  // (:231-241)
      }
      wave_lds_fence();
    }
  }
  const uint32_t tf = wave_sum(n_front), te = wave_sum(n_edges), ts = wave_sum(n_sup);
  if (lane == 0) {
    if (tf) {
      atomicAdd(&c->ring[L % LEVEL_RING], (unsigned long long)tf);
      atomicAdd(&c->marked, (unsigned long long)tf);
    }
    if (te) atomicAdd(&c->edges_scanned, (unsigned long long)te);
    if (ts) atomicAdd(&c->sup_edges, (unsigned long long)ts);
  }
}

static int level_grid(uint64_t slot_top) {
  const uint64_t blocks = (slot_top + BLK_SLOTS - 1) / BLK_SLOTS;  // wave-blocks
  uint64_t wg = (blocks + 3) / 4;
  if (wg < 1) wg = 1;
  if (wg > 2048) wg = 2048;  // 8 workgroups of 4 waves per CU
  return (int)wg;
}

hipError_t launch_level(const DevGraph &g, const LevelArgs &a, bool roots, bool investigate,
                        uint64_t slot_top, hipStream_t s) {
  const int grid = level_grid(slot_top);
  if (roots && investigate)
    hipLaunchKernelGGL((k_level<true, true>), dim3(grid), dim3(256), 0, s, g, a);
  else if (roots)
    hipLaunchKernelGGL((k_level<true, false>), dim3(grid), dim3(256), 0, s, g, a);
  else if (investigate)
    hipLaunchKernelGGL((k_level<false, true>), dim3(grid), dim3(256), 0, s, g, a);
  else
    hipLaunchKernelGGL((k_level<false, false>), dim3(grid), dim3(256), 0, s, g, a);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Sweep (:270-284): unmarked shadows are garbage; a local one is told StopMsg
// when its supervisor is marked and it is not halted.  A local garbage shadow
// without a supervisor is the reference's NullPointerException: counted here,
// and the commit pass below then leaves the graph untouched.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_sweep(DevGraph g, int should_kill) {
  Counters *c = g.ctr;
  const uint64_t slot_top = c->slot_top;
  const uint32_t nblk = (uint32_t)((slot_top + BLK_SLOTS - 1) / BLK_SLOTS);
  const int lane = lane_id();
  const uint32_t gw = blockIdx.x * 4 + (threadIdx.x >> 6);
  const uint32_t nw = gridDim.x * 4;
  uint32_t n_live = 0, n_npe = 0;
  for (uint32_t blk = gw; blk < nblk; blk += nw) {
    const uint64_t base = (uint64_t)blk * BLK_SLOTS + (uint64_t)lane * 32;
    const uint32_t word = g.vis[(uint64_t)blk * 64 + lane];
    const uint4 f4[2] = {*(const uint4 *)(g.flags + base), *(const uint4 *)(g.flags + base + 16)};
    const uint8_t *fb = (const uint8_t *)f4;
    uint32_t alive = 0, kill = 0;
#pragma unroll
    for (int j = 0; j < 32; ++j) alive |= (fb[j] & FL_ALIVE) ? (1u << j) : 0u;
    const uint32_t garbage = alive & ~word;
    n_live += __popc(alive & word);
    uint32_t gm = garbage;
    while (gm) {
      const int j = __ffs(gm) - 1;
      gm &= gm - 1;
      const uint8_t f = fb[j];
      if (f & FL_LOCAL) {
        const uint32_t s = g.sup[base + j];
        if (s == SLOT_NONE) {
          n_npe++;
        } else if (should_kill && !(f & FL_HALTED) && s < 0xFFFFFFF0u &&
                   ((g.vis[s >> 5] >> (s & 31)) & 1u)) {
          kill |= 1u << j;
        }
      }
    }
    const unsigned long long gbase = wave_atomic_add(&c->n_garbage, __popc(garbage));
    const unsigned long long kbase = wave_atomic_add(&c->n_kill, __popc(kill));
    uint32_t k = 0;
    gm = garbage;
    while (gm) {
      const int j = __ffs(gm) - 1;
      gm &= gm - 1;
      g.out_a[gbase + k++] = g.vid[base + j];
    }
    k = 0;
    uint32_t km = kill;
    while (km) {
      const int j = __ffs(km) - 1;
      km &= km - 1;
      g.out_b[kbase + k++] = g.vid[base + j];
    }
  }
  const uint32_t tl = wave_sum(n_live), tn = wave_sum(n_npe);
  if (lane == 0) {
    if (tl) atomicAdd(&c->n_live, (unsigned long long)tl);
    if (tn) atomicAdd(&c->npe, (unsigned long long)tn);
  }
}

// Remove the garbage from shadowMap (:276): tombstone its id-table bucket and
// clear its slot.  Slots and pool segments are reclaimed by the next rebuild,
// which also purges edges pointing at them.
__global__ __launch_bounds__(256) void k_commit(DevGraph g) {
  Counters *c = g.ctr;
  if (c->npe) return;
  const uint64_t slot_top = c->slot_top;
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t v = (uint64_t)blockIdx.x * 256 + threadIdx.x; v < slot_top; v += stride) {
    const uint8_t f = g.flags[v];
    if (!(f & FL_ALIVE)) continue;
    if ((g.vis[v >> 5] >> (v & 31)) & 1u) continue;
    uint64_t bucket = KEY_EMPTY;
    id_find(g, g.vid[v], &bucket);
    if (bucket != KEY_EMPTY) g.hkey[bucket] = KEY_TOMB;
    g.flags[v] = 0;
  }
}

hipError_t launch_sweep(const DevGraph &g, int should_kill, uint64_t slot_top, hipStream_t s) {
  hipLaunchKernelGGL(k_sweep, dim3(level_grid(slot_top)), dim3(256), 0, s, g, should_kill);
  return hipGetLastError();
}

hipError_t launch_commit(const DevGraph &g, uint64_t slot_top, hipStream_t s) {
  hipLaunchKernelGGL(k_commit, dim3(grid_for(slot_top, 256, 8192)), dim3(256), 0, s, g);
  return hipGetLastError();
}

// startWave (:291-299): local roots.
__global__ __launch_bounds__(256) void k_local_roots(DevGraph g) {
  Counters *c = g.ctr;
  const uint64_t slot_top = c->slot_top;
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t base = (uint64_t)blockIdx.x * 256 + (threadIdx.x & ~63u); base < slot_top;
       base += stride) {
    const uint64_t v = base + lane_id();
    bool hit = false;
    if (v < slot_top) {
      const uint8_t f = g.flags[v];
      hit = (f & FL_ALIVE) && (f & FL_ROOT) && (f & FL_LOCAL);
    }
    const unsigned long long k = wave_append(&c->n_out, hit);
    if (hit) g.out_a[k] = g.vid[v];
  }
}

hipError_t launch_local_roots(const DevGraph &g, uint64_t slot_top, hipStream_t s) {
  hipLaunchKernelGGL(k_local_roots, dim3(grid_for(slot_top, 256, 8192)), dim3(256), 0, s, g);
  return hipGetLastError();
}

}  // namespace crgc
