// crgc_merge.hip — entry / delta / undo-log merge kernels (gfx950).
//
// A merge call replaces N sequential ShadowGraph.mergeEntry / mergeDelta calls
// (ShadowGraph.java:75-156) by one data-parallel pass, exact because the merge
// is commutative except for last-write-wins fields:
//   * recvCount        += deltas          -> wrapping int32 atomics
//   * outgoing[o][t]   += deltas          -> edge pipeline (k_edge_* below)
//   * interned/isLocal |= ...             -> written by the LWW winner (every
//                                            record that sets busy/root sets them)
//   * isBusy/isRoot     last write wins   -> atomicMax of (epoch<<32 | seq) tags,
//   * supervisor        last write wins      then the winner writes the field.
// `epoch` counts merge calls, `seq` is the record's position inside the call,
// so "last" is exactly the reference's order (LocalGC.scala:152-172).
#include "crgc_host.hpp"

namespace crgc {

__device__ inline bool vs(uint32_t s) { return s < 0xFFFFFFF0u; }

// ---------------------------------------------------------------------------
// Id resolution, flattened: one thread per id reference of the batch (every
// self / created target and owner / spawned / updated ref of the entries, or
// every delta id / supervisor / outgoing target), no per-entry loops.  Slot
// allocation for new shadows is one atomic per 1024-thread workgroup.  Which
// thread creates a shadow does not matter: creation order only affects the
// reference's `from` order.
// ---------------------------------------------------------------------------
constexpr int IDS_THREADS = 1024;
#ifndef CRGC_IDS_K
#define CRGC_IDS_K 1
#endif
constexpr uint32_t IDS_RCAP = 4;  // reverse-candidate entries a new shadow starts with
constexpr int IDS_K = CRGC_IDS_K;  // ids per thread per round (4: merge +20 us on C2, profiles/r3f/ab_merge.txt)

// Continues a probe whose first bucket `b` (at h) was already loaded.
__device__ inline int id_probe_from(const DevGraph &g, uint64_t id, uint64_t h, uint4 b, uint64_t &bucket,
                                    uint32_t &slot) {
  const uint64_t k = bucket_key(b);
  if (k == id && b.z != VAL_PENDING) {  // the common case: an existing shadow, one load
    bucket = h;
    slot = b.z;
    return RS_FOUND;
  }
  return id_probe(g, id, bucket, slot);
}

__global__ __launch_bounds__(IDS_THREADS) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_ids(DevGraph g, IdArgs a) {
  uint64_t cnt[5], total = 0;
  for (int k = 0; k < 5; ++k) {
    cnt[k] = k < a.nseg ? (a.seg[k].n_dev ? (uint64_t)*a.seg[k].n_dev : a.seg[k].n) : 0;
    if (cnt[k] > a.seg[k].n) cnt[k] = a.seg[k].n;  // bad offsets: flagged by the apply kernel
    total += cnt[k];
  }
  const uint64_t per = (uint64_t)IDS_THREADS * IDS_K;
  const uint64_t stride = (uint64_t)gridDim.x * per;
  for (uint64_t base = (uint64_t)blockIdx.x * per; base < total; base += stride) {
    uint64_t id[IDS_K], h[IDS_K], bucket[IDS_K], r[IDS_K];
    uint32_t slot[IDS_K];
    int kseg[IDS_K], st[IDS_K];
    bool has[IDS_K], in[IDS_K];
    uint4 b0[IDS_K];
#pragma unroll
    for (int j = 0; j < IDS_K; ++j) {
      r[j] = base + (uint64_t)j * IDS_THREADS + threadIdx.x;
      in[j] = r[j] < total;
      int k = 0;
      if (in[j])
        while (r[j] >= cnt[k]) r[j] -= cnt[k++];
      kseg[j] = in[j] ? k : 0;
      id[j] = in[j] ? a.seg[kseg[j]].ids[r[j]] : 0;
    }
#pragma unroll
    for (int j = 0; j < IDS_K; ++j) {
      const IdSeg &sg = a.seg[kseg[j]];
      has[j] = in[j];
      if (has[j] && id[j] == CRGC_NO_ACTOR && sg.none_ok) has[j] = false;
      else if (has[j] && reserved_id(id[j])) {
        set_err(g.ctr, ERR_RESERVED_ID);
        has[j] = false;
      }
      if (has[j] && g.n_shards > 1 && !is_home(g, id[j])) {
        // not home here: resolve only as the far end of a local edge / supervisor
        bool want = false;
        if (sg.partner) {
          const uint64_t p = sg.partner[r[j]];
          want = p != CRGC_NO_ACTOR && is_home(g, p);
        }
        if (!want && sg.need) want = sg.need[r[j]] != 0;
        has[j] = want;
      }
      h[j] = mix64(id[j]) & g.hmask;
      b0[j] = has[j] ? load_bucket(&g.htab[h[j]]) : make_uint4(0, 0, 0, 0);
    }
    bool settle = false;
#pragma unroll
    for (int j = 0; j < IDS_K; ++j) {
      bucket[j] = 0;
      slot[j] = SLOT_INVALID;
      st[j] = has[j] ? id_probe_from(g, id[j], h[j], b0[j], bucket[j], slot[j]) : RS_NONE;
      settle |= st[j] == RS_INSERTED || st[j] == RS_PENDING;
    }
    // Slot allocation (one atomic per workgroup) only in rounds that created or
    // wait for a shadow: a steady-state wakeup mostly finds existing ones.
    // Every claim of the round is published before any wait (a pending key may
    // have been claimed by another thread's later id), so waits always end.
    if (__syncthreads_or(settle)) {
      uint32_t nins = 0, nhome = 0;
#pragma unroll
      for (int j = 0; j < IDS_K; ++j)
        if (st[j] == RS_INSERTED) {
          ++nins;
          nhome += is_home(g, id[j]) ? 1u : 0u;
        }
      // A new shadow starts with a reverse-candidate segment of IDS_RCAP
      // entries: most take their first in-edges in this same merge, which would
      // otherwise all go through k_rv_grow's overflow path (crgc_edges.hip §3).
      // Homes take slots from slot_top, proxies (sharded graphs) from proxy_top
      // in their own region above pbase.
      // Slot reuse (unsharded): new shadows take the swept slots of the free
      // list first (crgc_reuse.hip; the list is fixed during a merge, so the
      // taken count may pass its end), then fresh slots from slot_top.
      uint32_t nfree = 0;
      unsigned long long kf = 0;
      // (the host passes no free list while it knows the list is empty:
      // crgc_api.hip ids_view)
      const bool reuse = g.freel != nullptr;
      if (reuse) {
        unsigned long long *const fc[1] = {&g.ctr->free_used};
        const uint64_t fn = g.ctr->free_n;
        const uint32_t vf[1] = {nhome};
        unsigned long long bf[1];
        block_append<1>(fc, vf, bf);
        kf = bf[0];
        nfree = kf >= fn ? 0u : (uint32_t)min<uint64_t>(nhome, fn - kf);
      }
      unsigned long long *const ctrs[4] = {&g.ctr->slot_top, &g.ctr->inserted, &g.ctr->rpool_top,
                                           &g.ctr->proxy_top};
      const uint32_t v[4] = {nhome - nfree, nhome, nins * IDS_RCAP, nins - nhome};
      unsigned long long base[4];
      block_append<4>(ctrs, v, base);
      unsigned long long kh = base[0], kp = base[3], ro = base[2];
      const bool rfit = ro + (uint64_t)nins * IDS_RCAP <= g.rpcap;
#pragma unroll
      for (int j = 0; j < IDS_K; ++j) {
        if (st[j] != RS_INSERTED) continue;
        const bool home = is_home(g, id[j]);
        uint64_t s;
        if (home && nfree) {  // a purged slot of a collected shadow (reset by k_free_list)
          s = g.freel[kf++];
          --nfree;
        } else {
          s = region_slot(g, home, home ? kh++ : kp++);
        }
        if (s == ~0ull) {
          set_err(g.ctr, ERR_SLOTS_FULL);
          slot[j] = SLOT_INVALID;
        } else {
          slot[j] = (uint32_t)s;
          g.vid[s] = id[j];
          g.flags[s] = home ? FL_ALIVE : (FL_ALIVE | FL_PROXY);
          if (!home) g.psh[s] = (uint8_t)shard_of(id[j], g.n_shards);
          if (rfit) {
            g.radj[s] = make_uint2((uint32_t)ro, rseg_pack(0, IDS_RCAP));
          }
        }
        ro += IDS_RCAP;
        atomicExch(&g.htab[bucket[j]].val, slot[j]);
      }
#pragma unroll
      for (int j = 0; j < IDS_K; ++j) {
        if (st[j] == RS_PENDING) {
          slot[j] = SLOT_INVALID;
          for (uint32_t spin = 0; spin < (1u << 24); ++spin) {
            const uint32_t v2 = atomicOr(&g.htab[bucket[j]].val, 0u);
            if (v2 != VAL_PENDING) {
              slot[j] = v2;
              break;
            }
            __builtin_amdgcn_s_sleep(1);
          }
          if (slot[j] == SLOT_INVALID) set_err(g.ctr, ERR_SPIN);
        } else if (st[j] == RS_NONE) {
          slot[j] = SLOT_INVALID;
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < IDS_K; ++j)
        if (st[j] == RS_NONE) slot[j] = SLOT_INVALID;
    }
#pragma unroll
    for (int j = 0; j < IDS_K; ++j)
      if (in[j]) a.seg[kseg[j]].slots[r[j]] = slot[j];
  }
}

hipError_t launch_ids(const DevGraph &g, const IdArgs &a, hipStream_t s) {
  launch_begin();
  uint64_t n = 0;
  for (int k = 0; k < a.nseg; ++k) n += a.seg[k].n;
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_ids, dim3(grid_for((n + IDS_K - 1) / IDS_K, IDS_THREADS, 1024)), dim3(IDS_THREADS), 0, s, g, a);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Entries — ShadowGraph.mergeEntry, ShadowGraph.java:75-125.  One thread per
// entry over slots resolved by k_ids, in two kernels so the edge pipeline can
// start as soon as its atoms exist (it runs on a side stream beside the
// vertex updates, crgc_api.hip merge_entries_one):
//   k_entries_atoms   validation, the edge atoms, their exact count
//   k_entries_vertex  receive counts and the LWW tags (vertex state only)
// ---------------------------------------------------------------------------
// An entry's offsets are well formed (:85-123 read at most F records of each
// kind); a batch whose final offsets exceed n*F, or do not start at 0, is
// refused whole, so the atoms [0, C + U) are exactly the valid entries' atoms.
__device__ inline bool entry_ok(const EntryArgs &a, uint64_t i, bool report, Counters *c) {
  const uint32_t c0 = a.c_off[i], c1 = a.c_off[i + 1];
  const uint32_t s0 = a.s_off[i], s1 = a.s_off[i + 1];
  const uint32_t u0 = a.u_off[i], u1 = a.u_off[i + 1];
  const uint64_t cmax = a.n * a.F;
  if (c1 < c0 || s1 < s0 || u1 < u0 || c1 > cmax || s1 > cmax || u1 > cmax || a.c_off[a.n] > cmax ||
      a.u_off[a.n] > cmax || a.c_off[0] || a.s_off[0] || a.u_off[0]) {
    if (report) set_err(c, ERR_BAD_OFFSETS);
    return false;
  }
  if (c1 - c0 > a.F || s1 - s0 > a.F || u1 - u0 > a.F) {
    if (report) set_err(c, ERR_TOO_MANY);
    return false;
  }
  return true;
}

__global__ __launch_bounds__(256) void k_entries_atoms(DevGraph g, EntryArgs a) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= a.n) return;
  const bool ok = entry_ok(a, i, true, g.ctr);
  if (i == 0 && a.n_atoms) {  // atoms [0, C) created, [C, C + U) updated: the edge pipeline's exact count
    const uint64_t cmax = a.n * a.F;
    const uint64_t C = min((uint64_t)a.c_off[a.n], cmax), U = min((uint64_t)a.u_off[a.n], cmax);
    *a.n_atoms = C + U;
  }
  if (!ok) {
    a.self_slot[i] = SLOT_INVALID;
    return;
  }
  const uint32_t me = a.self_slot[i];
  const bool sh = g.n_shards > 1;
  const bool self_home = !sh || is_home(g, a.self[i]);
  // Created refs (:85-93): outgoing[owner][target] += 1.
  const uint32_t c0 = a.c_off[i], c1 = a.c_off[i + 1];
  for (uint32_t k = c0; k < c1; ++k) {
    const uint32_t os = a.co_slot[k], ts = a.ct_slot[k];
    a.atom_o[k] = os;
    a.atom_t[k] = ts;
    a.atom_d[k] = ((sh || vs(me)) && vs(os) && vs(ts)) ? 1 : 0;
  }
  // Deactivated refs (:120-122): outgoing[self][target] -= 1.
  const uint32_t ctot = a.c_off[a.n];
  const uint32_t u0 = a.u_off[i], u1 = a.u_off[i + 1];
  for (uint32_t k = u0; k < u1; ++k) {
    const uint32_t ts = a.u_slot[k];
    const uint64_t at = (uint64_t)ctot + k;
    a.atom_o[at] = me;
    a.atom_t[at] = ts;
    a.atom_d[at] = (vs(ts) && vs(me) && self_home && refob_deactivated(a.u_info[k])) ? -1 : 0;
  }
}

// Receive counts and last-write-wins tags.  The first entry of this merge to
// tag a slot (the atomicMax returns an older epoch) writes the field at once;
// any later one finds this merge's epoch and lists the slot in its block's
// conflict region, where k_entries_lww rewrites the field from the true
// winner (the tag's entry).  Most shadows appear once per batch, so the winners
// need no second random pass over every entry's tag.
__device__ inline void entry_flags(const DevGraph &g, uint32_t me, uint8_t ef, uint8_t f0) {
  uint8_t f = f0 & (uint8_t)~(FL_BUSY | FL_ROOT);
  f |= FL_INTERNED | FL_LOCAL;
  if (ef & CRGC_ENTRY_BUSY) f |= FL_BUSY;
  if (ef & CRGC_ENTRY_ROOT) f |= FL_ROOT;
  g.flags[me] = f;
}

__global__ __launch_bounds__(256) void k_entries_vertex(DevGraph g, EntryArgs a) {
  __shared__ uint32_t s_nv, s_ns;
  if (threadIdx.x == 0) s_nv = s_ns = 0;
  __syncthreads();
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  uint32_t *cv = a.conf_v + (uint64_t)blockIdx.x * 256;
  uint32_t *cs_ = a.conf_s + (uint64_t)blockIdx.x * 256 * a.F;
  if (i < a.n && entry_ok(a, i, false, g.ctr)) {  // a refused entry is reported (and its self cleared) by k_entries_atoms
    const uint32_t me = a.self_slot[i];
    const unsigned long long tag = (a.epoch << 32) | (unsigned long long)(i + 1);
    const int16_t rc = a.recv[i];
    // Sharded graphs: every record is applied by the home shard of the shadow
    // it writes (self, edge owner, spawned child, updated target).  k_ids only
    // resolved the ids this shard needs, so a valid slot of a child / owner is
    // a home slot; self may be a proxy (the supervisor of a child homed here).
    const bool sh = g.n_shards > 1;
    const bool self_home = !sh || is_home(g, a.self[i]);
    // Local information (:77-82): recv delta and the busy/root LWW tag.
    if (vs(me) && self_home) {
      // The flag byte is read beside the tag's atomic, not after it returns:
      // only the slot's first tagger of this merge writes it here (the
      // others go to the conflict list), so the early read is the value that
      // writer would read.
      const uint8_t f0 = g.flags[me];
      if (rc != 0) atomicAdd(&g.recv[me], (int32_t)rc);
      const unsigned long long old = atomicMax(&g.vseq[me], tag);
      if ((old >> 32) != a.epoch) entry_flags(g, me, a.flags[i], f0);
      else cv[atomicAdd(&s_nv, 1u)] = me;
    }
    // Spawned actors (:96-104): child.supervisor = self, last write wins.
    const uint32_t s0 = a.s_off[i], s1 = a.s_off[i + 1];
    for (uint32_t k = s0; k < s1; ++k) {
      const uint32_t cs = a.spawn_slot[k];
      if (!(vs(cs) && vs(me))) continue;
      const unsigned long long old = atomicMax(&g.sseq[cs], tag);
      if ((old >> 32) != a.epoch) g.sup[cs] = me;
      else cs_[atomicAdd(&s_ns, 1u)] = cs;
    }
    // Updated refs (:107-119): target.recv -= count.
    const uint32_t u0 = a.u_off[i], u1 = a.u_off[i + 1];
    for (uint32_t k = u0; k < u1; ++k) {
      const uint32_t ts = a.u_slot[k];
      const int32_t cnt = refob_count(a.u_info[k]);
      const bool tgt_ok = sh ? (vs(ts) && is_home(g, a.u_ref[k])) : (vs(ts) && vs(me));
      if (tgt_ok && cnt > 0) atomicAdd(&g.recv[ts], -cnt);
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {  // <= 256 slots, <= 256 * F children
    a.conf_n[2 * blockIdx.x] = s_nv;
    a.conf_n[2 * blockIdx.x + 1] = s_ns;
  }
}

// The slots several entries of this merge tagged: the tag's entry (the last
// in batch order) writes the field.  One block per k_entries_vertex block.
__global__ __launch_bounds__(256) void k_entries_lww(DevGraph g, EntryArgs a) {
  const uint32_t nv = a.conf_n[2 * blockIdx.x], ns = a.conf_n[2 * blockIdx.x + 1];
  const uint32_t *cv = a.conf_v + (uint64_t)blockIdx.x * 256;
  const uint32_t *cs_ = a.conf_s + (uint64_t)blockIdx.x * 256 * a.F;
  for (uint32_t k = threadIdx.x; k < nv; k += 256) {
    const uint32_t me = cv[k];
    const uint64_t w = (uint64_t)(g.vseq[me] & 0xFFFFFFFFull) - 1;  // the winning entry
    entry_flags(g, me, a.flags[w], g.flags[me]);
  }
  for (uint32_t k = threadIdx.x; k < ns; k += 256) {
    const uint32_t cs = cs_[k];
    const uint64_t w = (uint64_t)(g.sseq[cs] & 0xFFFFFFFFull) - 1;
    g.sup[cs] = a.self_slot[w];
  }
}

// Sharded graphs: which shards need an entry's self (its home, and the homes
// of its spawned children, where it becomes their supervisor), and which
// updated refs are the far end of a deactivation edge owned by self.
__global__ __launch_bounds__(256) void k_entries_shard_prep(DevGraph g, EntryArgs a) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= a.n) return;
  const uint64_t cmax = a.n * a.F;
  const uint64_t self = a.self[i];
  bool need = is_home(g, self);
  const uint32_t s0 = a.s_off[i], s1 = min((uint64_t)a.s_off[i + 1], cmax);
  for (uint32_t k = s0; k < s1 && k < s0 + a.F; ++k) need |= is_home(g, a.spawned[k]);
  a.self_need[i] = need;
  const uint32_t u0 = a.u_off[i], u1 = min((uint64_t)a.u_off[i + 1], cmax);
  for (uint32_t k = u0; k < u1 && k < u0 + a.F; ++k)
    a.u_partner[k] = refob_deactivated(a.u_info[k]) ? self : CRGC_NO_ACTOR;
}

// phase 0: (sharded prep) ids, atoms — the edge pipeline may start after it;
// phase 1: vertex updates, LWW winners.
hipError_t launch_entries(const DevGraph &g, const EntryArgs &a, hipStream_t s, int phase) {
  launch_begin();
  if (a.n == 0) return hipSuccess;
  const uint64_t nf = a.n * a.F;
  const int blocks = (int)((a.n + 255) / 256);
  const bool sh = g.n_shards > 1;
  if (phase == 1) {
    hipLaunchKernelGGL(k_entries_vertex, dim3(blocks), dim3(256), 0, s, g, a);
    hipLaunchKernelGGL(k_entries_lww, dim3(blocks), dim3(256), 0, s, g, a);
    return hipGetLastError();
  }
  if (sh) hipLaunchKernelGGL(k_entries_shard_prep, dim3(blocks), dim3(256), 0, s, g, a);
  IdArgs ia{};
  ia.nseg = 5;
  ia.seg[0] = IdSeg{a.self, a.self_slot, a.n, nullptr, false, nullptr, sh ? a.self_need : nullptr};
  ia.seg[1] = IdSeg{a.c_target, a.ct_slot, nf, a.c_off + a.n, false, a.c_owner, nullptr};
  ia.seg[2] = IdSeg{a.c_owner, a.co_slot, nf, a.c_off + a.n, false, nullptr, nullptr};
  ia.seg[3] = IdSeg{a.spawned, a.spawn_slot, nf, a.s_off + a.n, false, nullptr, nullptr};
  ia.seg[4] = IdSeg{a.u_ref, a.u_slot, nf, a.u_off + a.n, false, sh ? a.u_partner : nullptr,
                    nullptr};
  if (hipError_t e = hipGetLastError()) return e;  // before the nested helper drops it
  if (hipError_t e = launch_ids(g, ia, s)) return e;
  hipLaunchKernelGGL(k_entries_atoms, dim3(blocks), dim3(256), 0, s, g, a);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Deltas — ShadowGraph.mergeDelta, ShadowGraph.java:127-156.  One thread per
// delta shadow, in arrival order (seq).  Flags only when the shadow is
// interned (:139-146); isLocal is never set (:135).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_deltas_apply(DevGraph g, DeltaArgs a) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= a.n) return;
  const uint32_t o0 = a.out_off[i], o1 = a.out_off[i + 1];
  bool ok = true;
  // the atoms [0, nout) are exactly the valid shadows' outgoing entries: a
  // batch whose offsets do not start at 0 or run past nout is refused whole
  if (o1 < o0 || o1 > a.nout || a.out_off[0] || a.out_off[a.n] != a.nout) {
    set_err(g.ctr, ERR_BAD_OFFSETS);
    ok = false;
  }
  const uint32_t me = ok ? a.self_slot[i] : SLOT_INVALID;
  if (!ok) a.self_slot[i] = SLOT_INVALID;
  const unsigned long long tag = (a.epoch << 32) | (unsigned long long)(i + 1);
  const uint8_t fl = a.flags[i];
  const int32_t rc = a.recv[i];
  if (vs(me)) {
    if (rc != 0) atomicAdd(&g.recv[me], rc);
    if (fl & CRGC_DELTA_INTERNED) atomicMax(&g.vseq[me], tag);
  }
  const uint32_t ss = a.sup_slot[i];  // SLOT_INVALID: no supervisor in this delta
  const bool sup_ok = vs(ss) && vs(me);
  a.sup_slot[i] = sup_ok ? ss : SLOT_INVALID;
  if (sup_ok) atomicMax(&g.sseq[me], tag);
  if (!ok) return;
  for (uint32_t k = o0; k < o1; ++k) {
    const uint32_t ts = a.ot_slot[k];
    a.atom_o[k] = me;
    a.atom_t[k] = ts;
    a.atom_d[k] = (vs(ts) && vs(me)) ? a.out_count[k] : 0;
  }
}

__global__ __launch_bounds__(256) void k_deltas_lww(DevGraph g, DeltaArgs a) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= a.n) return;
  const uint32_t me = a.self_slot[i];
  if (!vs(me)) return;
  const unsigned long long tag = (a.epoch << 32) | (unsigned long long)(i + 1);
  const uint8_t df = a.flags[i];
  if ((df & CRGC_DELTA_INTERNED) && g.vseq[me] == tag) {
    uint8_t f = g.flags[me] & (uint8_t)~(FL_BUSY | FL_ROOT);
    f |= FL_INTERNED;
    if (df & CRGC_DELTA_BUSY) f |= FL_BUSY;
    if (df & CRGC_DELTA_ROOT) f |= FL_ROOT;
    g.flags[me] = f;
  }
  const uint32_t ss = a.sup_slot[i];
  if (vs(ss) && g.sseq[me] == tag) g.sup[me] = ss;
}

// Sharded graphs: the owning delta shadow of every outgoing entry.
__global__ __launch_bounds__(256) void k_deltas_shard_prep(DeltaArgs a, uint64_t n_out) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= a.n) return;
  const uint32_t o0 = a.out_off[i], o1 = min((uint64_t)a.out_off[i + 1], n_out);
  for (uint32_t k = o0; k < o1; ++k) a.o_partner[k] = a.id[i];
}

// phase 0: (sharded prep) ids, apply — the edge pipeline may start after it;
// phase 1: LWW winners.
hipError_t launch_deltas(const DevGraph &g, const DeltaArgs &a, uint64_t n_out, hipStream_t s, int phase) {
  launch_begin();
  if (a.n == 0) return hipSuccess;
  const int blocks = (int)((a.n + 255) / 256);
  if (phase == 1) {
    hipLaunchKernelGGL(k_deltas_lww, dim3(blocks), dim3(256), 0, s, g, a);
    return hipGetLastError();
  }
  const bool sh = g.n_shards > 1;
  if (sh && n_out)
    hipLaunchKernelGGL(k_deltas_shard_prep, dim3(blocks), dim3(256), 0, s, a, n_out);
  // A delta shadow's own fields, supervisor and out-edges all live with it, so
  // its id is resolved at home only; supervisor and targets also as proxies.
  IdArgs ia{};
  ia.nseg = 3;
  ia.seg[0] = IdSeg{a.id, a.self_slot, a.n, nullptr, false, nullptr, nullptr};
  ia.seg[1] = IdSeg{a.sup, a.sup_slot, a.n, nullptr, true, a.id, nullptr};
  ia.seg[2] = IdSeg{a.out_target, a.ot_slot, n_out, a.out_off + a.n, false,
                    sh ? a.o_partner : nullptr, nullptr};
  if (hipError_t e = hipGetLastError()) return e;  // before the nested helper drops it
  if (hipError_t e = launch_ids(g, ia, s)) return e;
  hipLaunchKernelGGL(k_deltas_apply, dim3(blocks), dim3(256), 0, s, g, a);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Undo logs — ShadowGraph.mergeUndoLog, ShadowGraph.java:158-174.
// ---------------------------------------------------------------------------
// Existence of every admitted actor and created-ref target, looked up at its
// home shard (exists[0..n) actors, exists[n..n+nc) targets).  The host ORs the
// shards' answers and reports the reference's ConcurrentModificationException
// (a target of an admitted actor not in the graph) before any
// mutation.
__global__ __launch_bounds__(256) void k_undo_exist(DevGraph g, UndoArgs a) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= a.n + a.nc) return;
  const uint64_t id = i < a.n ? a.actor[i] : a.c_target[i - a.n];
  a.exists[i] = (is_home(g, id) && id_find(g, id) != SLOT_NONE) ? 1 : 0;
}

// 1. every shadow at the downed location becomes halted (:163-165)
__global__ __launch_bounds__(256) void k_undo_halt(DevGraph g, uint16_t loc, uint64_t slot_top) {
  const uint64_t v = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (v >= slot_top) return;
  const uint8_t f = g.flags[v];
  if ((f & FL_ALIVE) && !(f & FL_PROXY) && (uint16_t)(g.vid[v] >> 48) == loc)
    g.flags[v] = f | FL_HALTED;
}

// 2. undelivered messages of admitted actors (:166-169), at their home
__global__ __launch_bounds__(256) void k_undo_recv(DevGraph g, UndoArgs a) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= a.n || a.msg[i] == 0 || !is_home(g, a.actor[i])) return;
  const uint32_t s = id_find(g, a.actor[i]);
  if (s != SLOT_NONE) atomicAdd(&g.recv[s], a.msg[i]);
}

// 3. created refs of admitted actors (:170-172), one thread per entry, at the
//    owner's home; a target homed elsewhere gets a proxy slot here.
__global__ __launch_bounds__(256) void k_undo_edges(DevGraph g, UndoArgs a) {
  const uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x;  // every lane reaches id_resolve
  const bool valid = k < a.nc;
  const uint64_t owner = valid ? a.c_actor[k] : 0;
  const uint32_t s = (valid && is_home(g, owner)) ? id_find(g, owner) : SLOT_NONE;
  const bool has = s != SLOT_NONE;
  const uint32_t t = id_resolve(g, has, has ? a.c_target[k] : 0);
  if (!valid) return;
  a.atom_o[k] = s;
  a.atom_t[k] = t;
  a.atom_d[k] = (has && vs(t)) ? a.c_count[k] : 0;
}

hipError_t launch_undo_check(const DevGraph &g, const UndoArgs &a, hipStream_t s) {
  launch_begin();
  if (a.n + a.nc == 0) return hipSuccess;
  hipLaunchKernelGGL(k_undo_exist, dim3((a.n + a.nc + 255) / 256), dim3(256), 0, s, g, a);
  return hipGetLastError();
}

hipError_t launch_undo_apply(const DevGraph &g, const UndoArgs &a, uint64_t slot_top,
                             hipStream_t s) {
  launch_begin();
  if (slot_top)
    hipLaunchKernelGGL(k_undo_halt, dim3((slot_top + 255) / 256), dim3(256), 0, s, g,
                       a.location, slot_top);
  if (a.n) hipLaunchKernelGGL(k_undo_recv, dim3((a.n + 255) / 256), dim3(256), 0, s, g, a);
  if (a.nc) hipLaunchKernelGGL(k_undo_edges, dim3((a.nc + 255) / 256), dim3(256), 0, s, g, a);
  return hipGetLastError();
}

// The edge pipeline (outgoing[o][t] += d) is crgc_edges.hip.

// A chunk of a host batch: its offsets relative to its first entry.
__global__ __launch_bounds__(256) void k_rebase(uint32_t *c_off, uint32_t *s_off, uint32_t *u_off, uint64_t n,
                                                uint32_t c0, uint32_t s0, uint32_t u0) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  c_off[i] -= c0;
  s_off[i] -= s0;
  u_off[i] -= u0;
}

// A large device batch's sub-merge boundaries: the three record offsets at
// every multiple of `ch` (and at n), gathered for one device-to-host copy.
__global__ __launch_bounds__(256) void k_bounds(const uint32_t *c_off, const uint32_t *s_off,
                                                const uint32_t *u_off, uint64_t n, uint64_t ch, uint64_t k,
                                                uint32_t *out) {
  const uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (j > k) return;
  const uint64_t at = min(n, j * ch);
  out[3 * j] = c_off[at];
  out[3 * j + 1] = s_off[at];
  out[3 * j + 2] = u_off[at];
}

hipError_t launch_bounds(const uint32_t *c_off, const uint32_t *s_off, const uint32_t *u_off, uint64_t n,
                         uint64_t ch, uint64_t k, uint32_t *out, hipStream_t s) {
  launch_begin();
  hipLaunchKernelGGL(k_bounds, dim3((k + 1 + 255) / 256), dim3(256), 0, s, c_off, s_off, u_off, n, ch, k, out);
  return hipGetLastError();
}

// A sub-merge's offset arrays, copied and rebased in one pass.
__global__ __launch_bounds__(256) void k_rebase_copy(const uint32_t *c_src, const uint32_t *s_src,
                                                     const uint32_t *u_src, uint32_t *c_off, uint32_t *s_off,
                                                     uint32_t *u_off, uint64_t n, uint32_t c0, uint32_t s0,
                                                     uint32_t u0) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  c_off[i] = c_src[i] - c0;
  s_off[i] = s_src[i] - s0;
  u_off[i] = u_src[i] - u0;
}

hipError_t launch_rebase_copy(const uint32_t *c_src, const uint32_t *s_src, const uint32_t *u_src, uint32_t *c_off,
                              uint32_t *s_off, uint32_t *u_off, uint64_t n, uint32_t c0, uint32_t s0, uint32_t u0,
                              hipStream_t s) {
  launch_begin();
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_rebase_copy, dim3((n + 255) / 256), dim3(256), 0, s, c_src, s_src, u_src, c_off, s_off, u_off,
                     n, c0, s0, u0);
  return hipGetLastError();
}

hipError_t launch_rebase(uint32_t *c_off, uint32_t *s_off, uint32_t *u_off, uint64_t n, uint32_t c0, uint32_t s0,
                         uint32_t u0, hipStream_t s) {
  launch_begin();
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_rebase, dim3((n + 255) / 256), dim3(256), 0, s, c_off, s_off, u_off, n, c0, s0, u0);
  return hipGetLastError();
}

// Up to 11 byte ranges from page-locked host memory (device-visible pointers)
// into HBM, read by the shader over PCIe: a registered batch's chunk, copied
// on the copy stream while the chunk before it merges.  One runtime copy per
// array from registered memory costs ~0.2 ms of overhead at ~1 MB
// (profiles/r3g/pcie_probe.txt), so the chunks are copied by this kernel
// instead.  Source and destination share their alignment mod 16 (the caller
// places the destination so): the body moves in 16-B groups, the ends by byte.
constexpr int COPY_IN_FLIGHT = 8;
constexpr int COPY_WG = 32;

__global__ __launch_bounds__(256) void k_copy_ranges(HostCopy c) {
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  const uint64_t tid = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  for (int r = 0; r < c.n; ++r) {
    const char *s = c.src[r];
    char *d = c.dst[r];
    const uint64_t len = c.bytes[r];
    const uint64_t head = min(len, (uint64_t)((16 - ((uintptr_t)s & 15)) & 15));
    const uint64_t body = (len - head) & ~15ull;
    if (tid < head) d[tid] = s[tid];
    const uint4 *s4 = (const uint4 *)(s + head);
    uint4 *d4 = (uint4 *)(d + head);
    // COPY_IN_FLIGHT 16-B reads per lane issued before any store: a few
    // workgroups keep the link full (the latency is ~2 us), so the merge
    // kernels running beside the copy keep their CUs (see launch_copy_ranges)
    const uint64_t n4 = body / 16;
    uint64_t i = tid;
    for (; i + (COPY_IN_FLIGHT - 1) * stride < n4; i += COPY_IN_FLIGHT * stride) {
      uint4 v[COPY_IN_FLIGHT];
#pragma unroll
      for (int k = 0; k < COPY_IN_FLIGHT; ++k) v[k] = s4[i + k * stride];
#pragma unroll
      for (int k = 0; k < COPY_IN_FLIGHT; ++k) d4[i + k * stride] = v[k];
    }
    for (; i < n4; i += stride) d4[i] = s4[i];
    const uint64_t tail = len - head - body;
    if (tid < tail) d[head + body + tid] = s[head + body + tid];
  }
}

hipError_t launch_copy_ranges(const HostCopy &c, hipStream_t s) {
  launch_begin();
  uint64_t tot = 0;
  for (int r = 0; r < c.n; ++r) tot += c.bytes[r];
  if (!tot) return hipSuccess;
  // enough 16-B requests in flight to fill the link (32 x 256 lanes x 8 x 16 B =
  // 1 MiB), few CUs taken from the merge: with 128 workgroups of one read per
  // lane, the merge kernels beside the copy ran 5-25x slower (k_rebase 134 us
  // against 5, profiles/r4ab) — their waves queued behind PCIe reads on the
  // copy's CUs
  hipLaunchKernelGGL(k_copy_ranges, dim3(grid_for(tot / 16, 256, COPY_WG)), dim3(256), 0, s, c);
  return hipGetLastError();
}

int grid_for(uint64_t threads, int block, int cap) {
  uint64_t b = (threads + block - 1) / block;
  if (b < 1) b = 1;
  if (b > (uint64_t)cap) b = cap;
  return (int)b;
}

}  // namespace crgc
