// crgc_rebuild.hip — compaction of the HBM shadow graph.
//
// Collected shadows leave a tombstone in the id table and a dead slot whose
// pool segment and incoming edges linger; slots are never reused before a
// rebuild, which makes the lingering edges harmless (they point at a slot no
// live id maps to, exactly like the reference's outgoing keys that still name
// a collected Shadow object — SURVEY E9).  A rebuild renumbers the live slots
// densely, drops zero-count edges and edges to dead slots, re-packs every
// segment at power-of-two capacity and rebuilds both hash tables.  It runs
// when a capacity would be exceeded, never on the per-wakeup path unless the
// graph has grown.
#include "crgc_host.hpp"

namespace crgc {

__device__ inline uint32_t rb_cap(uint32_t k) {
  if (k == 0) return 0;
  uint32_t c = 4;
  while (c < k) c <<= 1;
  return c;
}

// 1. live vertices -> dense new slots, id table rebuilt.  The source's slots
//    are visited as one virtual run: its shadows [0, src_top), then its proxy
//    region [src.pbase, + src_ptop); homes go to the new graph's low slots,
//    proxies to its proxy region.  `map` is indexed by source slot.
__global__ __launch_bounds__(256) void k_rb_vertices(DevGraph src, uint64_t src_top, uint64_t src_ptop, DevGraph dst,
                                                     uint32_t *map) {
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  const uint64_t vtop = src_top + src_ptop;
  for (uint64_t base = (uint64_t)blockIdx.x * 256 + (threadIdx.x & ~63u); base < vtop; base += stride) {
    const uint64_t u = base + lane_id();
    const uint64_t v = vslot(src, u, src_top);
    const uint8_t f = u < vtop ? src.flags[v] : 0;
    const bool alive = f & FL_ALIVE, home = alive && !(f & FL_PROXY);
    const unsigned long long kh = wave_append(&dst.ctr->slot_top, home);
    const unsigned long long kp = wave_append(&dst.ctr->proxy_top, alive && !home);
    // past the new arrays (the host sized them too small): dropped, so no later
    // pass indexes a new array with it; the error poisons the handle
    const uint64_t ns = alive ? region_slot(dst, home, home ? kh : kp) : ~0ull;
    const bool fits = ns != ~0ull;
    if (u < vtop) map[v] = fits ? (uint32_t)ns : SLOT_NONE;
    if (!alive) continue;
    if (!fits) {
      set_err(dst.ctr, ERR_SLOTS_FULL);
      continue;
    }
    const uint64_t id = src.vid[v];
    dst.vid[ns] = id;
    dst.recv[ns] = src.recv[v];
    dst.flags[ns] = f;
    if (!home) dst.psh[ns] = src.psh[v];
    uint64_t h = mix64(id) & dst.hmask;
    for (uint64_t p = 0; p < dst.hcap; ++p) {
      if (atomicCAS((unsigned long long *)&dst.htab[h].key, (unsigned long long)KEY_EMPTY,
                    (unsigned long long)id) == KEY_EMPTY) {
        dst.htab[h].val = (uint32_t)ns;
        break;
      }
      h = (h + 1) & dst.hmask;
    }
  }
}

// 2. kept out-degree of every live vertex: nonzero count, live target.
__global__ __launch_bounds__(256) void k_rb_count(DevGraph src, uint64_t src_top, const uint32_t *map,
                                                  uint64_t *caps) {
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t v = (uint64_t)blockIdx.x * 256 + threadIdx.x; v < src_top; v += stride) {
    const uint32_t ns = map[v];
    if (ns == SLOT_NONE) continue;
    const uint2 ad = src.adj[v];
    uint32_t k = 0;
    for (uint32_t e = 0; e < ad.y; ++e) {
      const uint64_t ed = src.pool[(uint64_t)ad.x + e];
      if (edge_count(ed) != 0 && (src.flags[edge_target(ed)] & FL_ALIVE)) ++k;
    }
    caps[ns] = rb_cap(k);
  }
}

// 4. copy kept edges (targets remapped), rebuild the edge table, remap the
//    supervisor (a collected supervisor becomes SLOT_DEAD: non-null, unmarked).
__global__ __launch_bounds__(256) void k_rb_edges(DevGraph src, uint64_t src_top, DevGraph dst,
                                                  const uint32_t *map, const uint64_t *offs) {
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t base = (uint64_t)blockIdx.x * 256 + (threadIdx.x & ~63u); base < src_top;
       base += stride) {
    const uint64_t v = base + lane_id();
    uint32_t kept = 0;
    if (v < src_top) {
      const uint32_t ns = map[v];
      if (ns != SLOT_NONE && ns < dst.scap) {
        const uint2 ad = src.adj[v];
        const uint64_t off = offs[ns];
        for (uint32_t e = 0; e < ad.y; ++e) {
          const uint64_t ed = src.pool[(uint64_t)ad.x + e];
          const uint32_t t = edge_target(ed);
          if (edge_count(ed) == 0 || !(src.flags[t] & FL_ALIVE)) continue;
          const uint32_t nt = map[t];
          if (nt == SLOT_NONE) continue;  // a target dropped by an overflow (ERR_SLOTS_FULL is set)
          dst.pool[off + kept] = pack_edge(nt, edge_count(ed));
          atomicAdd(&dst.rnew[nt], 1u);  // in-degree, for the candidate lists
          const uint64_t key = edge_key(ns, nt);
          uint64_t h = mix64(key) & dst.emask;
          for (uint64_t p = 0; p < dst.ecap_tab; ++p) {
            if (atomicCAS((unsigned long long *)&dst.etab[h].key, (unsigned long long)KEY_EMPTY,
                          (unsigned long long)key) == KEY_EMPTY) {
              dst.etab[h].val = kept;
              break;
            }
            h = (h + 1) & dst.emask;
          }
          ++kept;
        }
        dst.adj[ns] = make_uint2((uint32_t)off, kept);
        // The reference keeps nonzero counts toward collected shadows in
        // `outgoing` (their Shadow objects stay keys there), so they still
        // count in outgoing.size(): carry the owner's count over unchanged.
        // The purged entries can never change again (their ids now map to
        // fresh shadows).
        dst.nzdeg[ns] = src.nzdeg[v];
        const uint32_t s = src.sup[v];
        uint32_t nsup = SLOT_NONE;
        if (s == SLOT_DEAD) nsup = SLOT_DEAD;
        else if (s != SLOT_NONE) nsup = (src.flags[s] & FL_ALIVE) ? map[s] : SLOT_DEAD;  // (NONE: overflow)
        dst.sup[ns] = nsup;
      }
    }
    wave_atomic_add(&dst.ctr->etab_used, kept);
  }
}

// ---- exclusive scan of uint64 (in place), 2048 elements per block ----------
constexpr int SCAN_ITEMS = 8;
constexpr int SCAN_TILE = 256 * SCAN_ITEMS;

__device__ inline uint64_t block_excl_scan_u64(uint64_t x, uint64_t *total) {
  __shared__ uint64_t warp_tot[4];
  const int lane = lane_id(), wv = threadIdx.x >> 6;
  uint64_t incl = x;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint64_t y = __shfl_up(incl, d);
    if (lane >= d) incl += y;
  }
  if (lane == 63) warp_tot[wv] = incl;
  __syncthreads();
  uint64_t pre = 0, tot = 0;
  for (int w = 0; w < 4; ++w) {
    if (w < wv) pre += warp_tot[w];
    tot += warp_tot[w];
  }
  __syncthreads();
  *total = tot;
  return pre + incl - x;
}

__global__ __launch_bounds__(256) void k_scan_tiles(uint64_t *data, uint64_t n, uint64_t *partials) {
  const uint64_t t0 = (uint64_t)blockIdx.x * SCAN_TILE + (uint64_t)threadIdx.x * SCAN_ITEMS;
  uint64_t v[SCAN_ITEMS];
  uint64_t sum = 0;
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; ++k) {
    v[k] = (t0 + k < n) ? data[t0 + k] : 0;
    sum += v[k];
  }
  uint64_t tot;
  uint64_t run = block_excl_scan_u64(sum, &tot);
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; ++k) {
    if (t0 + k < n) data[t0 + k] = run;
    run += v[k];
  }
  if (threadIdx.x == 0) partials[blockIdx.x] = tot;
}

__global__ __launch_bounds__(256) void k_scan_partials(uint64_t *partials, uint64_t nb, uint64_t *grand) {
  uint64_t carry = 0;
  for (uint64_t b0 = 0; b0 < nb; b0 += 256) {
    const uint64_t i = b0 + threadIdx.x;
    const uint64_t x = i < nb ? partials[i] : 0;
    uint64_t tot;
    const uint64_t ex = block_excl_scan_u64(x, &tot);
    if (i < nb) partials[i] = carry + ex;
    carry += tot;
  }
  if (threadIdx.x == 0) *grand = carry;
}

__global__ __launch_bounds__(256) void k_scan_add(uint64_t *data, uint64_t n, const uint64_t *partials) {
  const uint64_t t0 = (uint64_t)blockIdx.x * SCAN_TILE;
  const uint64_t add = partials[blockIdx.x];
  for (int k = threadIdx.x; k < SCAN_TILE; k += 256)
    if (t0 + k < n) data[t0 + k] += add;
}

size_t rebuild_scan_tmp_bytes(uint64_t n) { return ((n + SCAN_TILE - 1) / SCAN_TILE + 2) * 8; }

// scan_tmp layout: [partials (nb)] [grand total]
static void exclusive_scan(uint64_t *data, uint64_t n, uint64_t *tmp, hipStream_t s) {
  const uint64_t nb = (n + SCAN_TILE - 1) / SCAN_TILE;
  if (nb == 0) return;
  hipLaunchKernelGGL(k_scan_tiles, dim3(nb), dim3(256), 0, s, data, n, tmp);
  hipLaunchKernelGGL(k_scan_partials, dim3(1), dim3(256), 0, s, tmp, nb, tmp + nb);
  hipLaunchKernelGGL(k_scan_add, dim3(nb), dim3(256), 0, s, data, n, tmp);
}

__global__ void k_rb_pool_top(Counters *c, const uint64_t *grand) { c->pool_top = *grand; }
__global__ void k_rb_rpool_top(Counters *c, const uint64_t *grand) { c->rpool_top = *grand; }

// 5. reverse candidate lists from the kept edges: capacities from the
//    in-degrees counted in k_rb_edges, offsets by scan, then a fill pass.
// Whether slot v of a (new) graph is in use: its shadows [0, slot_top), its
// proxies [pbase, pbase + proxy_top) — both clamped to the arrays (k_rb_vertices
// maps slots past a region to SLOT_NONE, but the counters still count them —
// ADVICE r4).
__device__ inline bool rb_used(const DevGraph &d, uint64_t v) {
  const Counters *c = d.ctr;
  return v < min((uint64_t)c->slot_top, d.pbase) || (v >= d.pbase && v < min(d.pbase + c->proxy_top, d.scap));
}

__global__ __launch_bounds__(256) void k_rb_rcaps(DevGraph dst, uint64_t *caps) {
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t v = (uint64_t)blockIdx.x * 256 + threadIdx.x; v < dst.scap; v += stride)
    caps[v] = rb_used(dst, v) ? rb_cap(dst.rnew[v]) : 0;
}

__global__ __launch_bounds__(256) void k_rb_rsetup(DevGraph dst, const uint64_t *offs) {
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t v = (uint64_t)blockIdx.x * 256 + threadIdx.x; v < dst.scap; v += stride) {
    if (!rb_used(dst, v)) continue;
    dst.radj[v] = make_uint2((uint32_t)offs[v], rseg_pack(0, rb_cap(dst.rnew[v])));
    dst.rnew[v] = 0;
  }
}

// (owners: the shadows' own slots; proxies have no out-edges)
__global__ __launch_bounds__(256) void k_rb_rfill(DevGraph dst) {
  const uint64_t n = min((uint64_t)dst.ctr->slot_top, dst.pbase);
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t o = (uint64_t)blockIdx.x * 256 + threadIdx.x; o < n; o += stride) {
    const uint2 ad = dst.adj[o];
    for (uint32_t e = 0; e < ad.y; ++e) {
      const uint64_t ed = dst.pool[(uint64_t)ad.x + e];
      const uint32_t t = edge_target(ed);
      const uint32_t pos = rseg_len(atomicAdd(&dst.radj[t].y, 1u));
      dst.rpool[(uint64_t)dst.radj[t].x + pos] = (uint32_t)o | (edge_count(ed) > 0 ? RC_POS : 0u);
      // the edge's bucket, for its candidate index
      const uint64_t key = edge_key((uint32_t)o, t);
      uint64_t hb = mix64(key) & dst.emask;
      for (uint64_t p = 0; p < dst.ecap_tab && dst.etab[hb].key != key; ++p) hb = (hb + 1) & dst.emask;
      if (dst.etab[hb].key == key) dst.etab[hb].rev = pos;
    }
  }
}

// ---- repack: the two pools alone ---------------------------------------------
// Relocated segments leave dead space in the pools (a segment that outgrows its
// capacity moves to a fresh one).  A repack moves every owner's out-edge segment
// and every target's candidate segment into new pools, packed in slot order at
// their current capacities.  Slots, both hash tables and every index inside a
// segment (edge-table val / rev) stay as they are: only adj.x and radj.x
// change.  So a merge whose pools would overflow repacks instead of rebuilding
// the graph — no slot renumbering, and about a third of a rebuild's memory
// (the C4 graph on one GPU: 51 GB of new pools against a second 130-GB graph).
// (top / ptop: the graph's shadow and proxy slot counts)
__global__ __launch_bounds__(256) void k_rp_sizes(DevGraph g, uint64_t top, uint64_t ptop, uint64_t *pp,
                                                  uint64_t *rp) {
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t v = (uint64_t)blockIdx.x * 256 + threadIdx.x; v < g.scap; v += stride) {
    const bool used = v < top || (v >= g.pbase && v < g.pbase + ptop);
    pp[v] = used ? seg_cap(g.adj[v].y) : 0;
    rp[v] = used ? rseg_cap(g.radj[v].y) : 0;
  }
}

// One slot per lane: its segments' live entries to their new offsets (short
// ones by the lane, longer ones by the whole wave).
template <typename T>
__device__ inline void rp_copy(const T *from, T *to, uint32_t len) {
  const bool small = len <= 8;
  if (small)
    for (uint32_t e = 0; e < len; ++e) to[e] = from[e];
  uint64_t big = __ballot(!small);
  while (big) {
    const int k = __ffsll((unsigned long long)big) - 1;
    big &= big - 1;
    const T *fk = (const T *)__shfl((unsigned long long)(uintptr_t)from, k);
    T *tk = (T *)__shfl((unsigned long long)(uintptr_t)to, k);
    const uint32_t lk = __shfl(len, k);
    for (uint32_t e = lane_id(); e < lk; e += 64) tk[e] = fk[e];
  }
}

__global__ __launch_bounds__(256) void k_rp_move(DevGraph g, uint64_t top, uint64_t ptop, const uint64_t *pp,
                                                 const uint64_t *rp, uint64_t *pool2, uint32_t *rpool2) {
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  const uint64_t vtop = top + ptop;
  for (uint64_t base = (uint64_t)blockIdx.x * 256 + (threadIdx.x & ~63u); base < vtop; base += stride) {
    const uint64_t u = base + lane_id();
    const bool in = u < vtop;
    const uint64_t v = vslot(g, u, top);
    const uint2 ad = in ? g.adj[v] : make_uint2(0, 0);
    const uint2 rd = in ? g.radj[v] : make_uint2(0, 0);
    const uint64_t po = in ? pp[v] : 0, ro = in ? rp[v] : 0;
    rp_copy(g.pool + ad.x, pool2 + po, ad.y);
    rp_copy(g.rpool + rd.x, rpool2 + ro, rseg_len(rd.y));
    if (in) {
      g.adj[v].x = (uint32_t)po;
      g.radj[v].x = (uint32_t)ro;
    }
  }
}

hipError_t launch_repack(const DevGraph &g, uint64_t top, uint64_t ptop, uint64_t *pp, uint64_t *rp, void *scan_tmp,
                         uint64_t *pool2, uint32_t *rpool2, hipStream_t s) {
  launch_begin();
  const int grid = grid_for(g.scap, 256, 8192);
  const uint64_t nb = (g.scap + SCAN_TILE - 1) / SCAN_TILE;
  uint64_t *tp = (uint64_t *)scan_tmp, *tr = tp + nb + 2;
  hipLaunchKernelGGL(k_rp_sizes, dim3(grid), dim3(256), 0, s, g, top, ptop, pp, rp);
  exclusive_scan(pp, g.scap, tp, s);
  exclusive_scan(rp, g.scap, tr, s);
  hipLaunchKernelGGL(k_rb_pool_top, dim3(1), dim3(1), 0, s, g.ctr, tp + nb);
  hipLaunchKernelGGL(k_rb_rpool_top, dim3(1), dim3(1), 0, s, g.ctr, tr + nb);
  hipLaunchKernelGGL(k_rp_move, dim3(grid_for(top + ptop, 256, 8192)), dim3(256), 0, s, g, top, ptop, pp, rp, pool2,
                     rpool2);
  return hipGetLastError();
}

// 0. the alive slots a rebuild keeps, counted exactly (out[0] shadows, out[1]
//    proxies): the host sizes the new arrays from them.
__global__ __launch_bounds__(256) void k_rb_count_alive(DevGraph src, uint64_t src_top, uint64_t src_ptop,
                                                        unsigned long long *out) {
  const uint64_t stride = (uint64_t)gridDim.x * 256 * 16;
  uint32_t k[2] = {0, 0};
  for (int r = 0; r < 2; ++r) {
    const uint64_t lo = r ? src.pbase : 0, n = r ? src_ptop : src_top;
    for (uint64_t i = ((uint64_t)blockIdx.x * 256 + threadIdx.x) * 16; i < n; i += stride) {
      const uint64_t v = lo + i;
      if (i + 16 <= n) {
        const uint4 f = *(const uint4 *)(src.flags + v);
        const uint32_t w[4] = {f.x, f.y, f.z, f.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) k[r] += __popc(w[j] & 0x01010101u * FL_ALIVE);
      } else {
        for (uint64_t u = v; u < lo + n; ++u) k[r] += (src.flags[u] & FL_ALIVE) ? 1u : 0u;
      }
    }
  }
  for (int r = 0; r < 2; ++r) {
    const uint32_t ws = wave_sum(k[r]);
    if (lane_id() == 0 && ws) atomicAdd(&out[r], (unsigned long long)ws);
  }
}

hipError_t launch_count_alive(const DevGraph &src, uint64_t src_top, uint64_t src_ptop, unsigned long long *out,
                              hipStream_t s) {
  launch_begin();
  if (src_top + src_ptop == 0) return hipSuccess;
  hipLaunchKernelGGL(k_rb_count_alive, dim3(grid_for((std::max(src_top, src_ptop) + 15) / 16, 256, 4096)), dim3(256),
                     0, s, src, src_top, src_ptop, out);
  return hipGetLastError();
}

// ---- grow: larger arrays, the same slots -------------------------------------
// A graph that outgrows its capacities with few dead slots keeps its slot
// numbering: the per-slot arrays and the pools are copied as they are and the
// two hash tables are re-hashed into larger ones (collected ids' tombstones
// dropped).  About a tenth of a rebuild's work: no renumbering, no CSR or
// candidate-list rebuild.
__global__ __launch_bounds__(256) void k_gr_ids(DevGraph src, DevGraph dst) {
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t b = (uint64_t)blockIdx.x * 256 + threadIdx.x; b < src.hcap; b += stride) {
    const uint4 k4 = load_bucket(&src.htab[b]);
    const uint64_t key = bucket_key(k4);
    if (key == KEY_EMPTY || key == KEY_TOMB) continue;
    uint64_t h = mix64(key) & dst.hmask;
    for (uint64_t p = 0; p < dst.hcap; ++p) {
      if (atomicCAS((unsigned long long *)&dst.htab[h].key, (unsigned long long)KEY_EMPTY,
                    (unsigned long long)key) == KEY_EMPTY) {
        dst.htab[h].val = k4.z;
        break;
      }
      h = (h + 1) & dst.hmask;
    }
  }
}

__global__ __launch_bounds__(256) void k_gr_edges(DevGraph src, DevGraph dst) {
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t b = (uint64_t)blockIdx.x * 256 + threadIdx.x; b < src.ecap_tab; b += stride) {
    const uint4 k4 = load_bucket(&src.etab[b]);
    const uint64_t key = bucket_key(k4);
    if (key == KEY_EMPTY || key == KEY_TOMB) continue;  // (TOMB: an edge of a reused slot, purged)
    uint64_t h = mix64(key) & dst.emask;
    for (uint64_t p = 0; p < dst.ecap_tab; ++p) {
      if (atomicCAS((unsigned long long *)&dst.etab[h].key, (unsigned long long)KEY_EMPTY,
                    (unsigned long long)key) == KEY_EMPTY) {
        dst.etab[h].val = k4.z;
        dst.etab[h].rev = k4.w;
        break;
      }
      h = (h + 1) & dst.emask;
    }
  }
}

hipError_t launch_grow_tables(const DevGraph &src, const DevGraph &dst, hipStream_t s) {
  launch_begin();
  hipLaunchKernelGGL(k_gr_ids, dim3(grid_for(src.hcap, 256, 8192)), dim3(256), 0, s, src, dst);
  hipLaunchKernelGGL(k_gr_edges, dim3(grid_for(src.ecap_tab, 256, 8192)), dim3(256), 0, s, src, dst);
  return hipGetLastError();
}

hipError_t launch_rebuild(const DevGraph &src, uint64_t src_top, uint64_t src_ptop, const DevGraph &dst, uint32_t *map,
                          uint64_t *offs, void *scan_tmp, hipStream_t s) {
  launch_begin();
  const int grid = grid_for(src_top, 256, 8192);
  hipLaunchKernelGGL(k_rb_vertices, dim3(grid_for(src_top + src_ptop, 256, 8192)), dim3(256), 0, s, src, src_top,
                     src_ptop, dst, map);
  hipLaunchKernelGGL(k_rb_count, dim3(grid), dim3(256), 0, s, src, src_top, map, offs);
  exclusive_scan(offs, dst.scap, (uint64_t *)scan_tmp, s);
  const uint64_t nb = (dst.scap + SCAN_TILE - 1) / SCAN_TILE;
  hipLaunchKernelGGL(k_rb_pool_top, dim3(1), dim3(1), 0, s, dst.ctr, (uint64_t *)scan_tmp + nb);
  hipLaunchKernelGGL(k_rb_edges, dim3(grid), dim3(256), 0, s, src, src_top, dst, map, offs);
  const int dgrid = grid_for(dst.scap, 256, 8192);
  hipLaunchKernelGGL(k_rb_rcaps, dim3(dgrid), dim3(256), 0, s, dst, offs);
  exclusive_scan(offs, dst.scap, (uint64_t *)scan_tmp, s);
  hipLaunchKernelGGL(k_rb_rpool_top, dim3(1), dim3(1), 0, s, dst.ctr, (uint64_t *)scan_tmp + nb);
  hipLaunchKernelGGL(k_rb_rsetup, dim3(dgrid), dim3(256), 0, s, dst, offs);
  hipLaunchKernelGGL(k_rb_rfill, dim3(dgrid), dim3(256), 0, s, dst);
  return hipGetLastError();
}

}  // namespace crgc
