// crgc_trace.hip — ShadowGraph.trace on gfx950 (ShadowGraph.java:205-289).
//
// Mark = level-synchronous reachability over
//   { (o -> t) : outgoing[o][t] > 0 }  U  { (c -> supervisor(c)) }
// from the pseudo-roots, never expanding halted shadows (:226-229).
// Reachability does not depend on visiting order, so a level-synchronous
// sweep marks exactly the reference's `to` set.
//
// Frontier state, no atomics on the per-edge path:
//   vis     1 bit / slot   marked set as of the start of the level
//   front   1 byte / slot  candidates for the next level: a discovered target
//                          gets a plain byte store (idempotent, so concurrent
//                          stores from any XCD merge correctly at write-back),
//                          skipped when the byte is already set
//   dirty   1 byte / 2048 slots, only in sparse levels: which blocks to scan
//
// No hot global counters either (one word saturates at ~88 atomics/us on
// MI355X): frontier ranges go to per-block regions with level-tagged counts,
// statistics to per-workgroup partials reduced by a single block.
#include <hip/hip_ext.h>

#include "crgc_host.hpp"

namespace crgc {

constexpr uint32_t RANGE_MAX = 256;  // longer segments (hubs) are cut into pieces
constexpr int FB = 4;               // k_frontier: chunks of 64 frontier shadows per load group
constexpr uint32_t NO_SLOT = ~0u;
constexpr int STAT_FRONT = 0, STAT_SUP = 1, STAT_EDGES = 2, STAT_LIVE = 3;
constexpr int STAT_MF = 3;  // during the mark: the level's frontier out-edges (STAT_LIVE after)

__device__ inline bool sparse_level(const Counters *c, int L, uint32_t thr) {
  if (L <= 1) return false;
  return c->ring[(L - 2) % LEVEL_RING] < thr;
}

// The slots a pull level walks: the shadows' own and, in a sharded graph, the
// proxy region (a shard of C4 over 8 holds ~6x more proxies than shadows, so a
// frontier of slot_top / div is far too narrow for a pull to pay there: round
// 5's C4 logical-shard trace spent 13 of its 18 ms of k_expand in such pulls).
__device__ inline uint64_t pull_span(const Counters *c) { return c->slot_top + c->proxy_top; }

// Direction choice for level L (same answer in k_frontier and k_expand): pull
// when the previous frontier was large; the level is then dense, so every
// block of the slot range is scanned and `fx` is complete.
// A level that pulled in the previous trace pulls again (LevelArgs::pull_pred):
// decided before k_frontier, so it lists no push ranges the pull would not read
// (a level-1 frontier of 5e6 shadows listed 8 B of ranges each, then pulled).
template <bool PRED = true>
__device__ inline bool pull_level(const Counters *c, int L, const LevelArgs &a) {
  if (!(a.flags & LV_PULL) || L < 1) return false;
  if (sparse_level(c, L, a.sparse_thresh) || sparse_level(c, L + 1, a.sparse_thresh)) return false;
  if (PRED && L < 64 && ((a.pull_pred >> L) & 1ull)) return true;
  const uint64_t prev = c->ring[(L - 1) % LEVEL_RING];
  return a.pull_div ? prev * a.pull_div >= pull_span(c) : prev >= a.pull_thresh;
}

// Levels whose k_frontier scans every block write `fx`, so k_expand can still
// pull when the frontier it finds is large although the previous one was not
// (the decision above is made before the level's own frontier is counted).
// Level 0 (the pseudo-roots) scans every block too, so it writes `fx` as well.
__device__ inline bool fx_level(const Counters *c, int L, const LevelArgs &a) {
  if (!(a.flags & LV_PULL) || (!a.pull_cur_div && !a.alpha)) return false;
  if (L == 0) return a.alpha != 0;
  return !sparse_level(c, L, a.sparse_thresh) && !sparse_level(c, L + 1, a.sparse_thresh);
}

// k_expand's direction, once k_tail has counted the level: pull when k_frontier
// already chose to (no ranges listed), else by Beamer's rule (direction-optimising
// BFS): pull when the frontier's out-edges m_f exceed the unexplored edges m_u
// over alpha — a pull level reads in-candidate lists that stop at their first hit
// and probe a frontier bitmap that stays in the XCD's L2, a push level does a
// random candidate-byte read-modify-write per edge.
// (PRED = false: the direction the rules give without the prediction — what
// the next trace predicts from, so a prediction lapses once its level narrows)
template <bool PRED = true>
__device__ inline bool pull_now(const Counters *c, int L, const LevelArgs &a) {
  if (pull_level<PRED>(c, L, a)) return true;
  if (!fx_level(c, L, a)) return false;
  if (!a.alpha) return c->ring[L % LEVEL_RING] * a.pull_cur_div >= pull_span(c);
  const uint64_t mu = a.e_total > c->mf_sum ? a.e_total - c->mf_sum : 0;
  return c->mf_level * a.alpha > mu;
}

// Whether level L lists its frontier for k_tail (same answer in k_frontier and
// k_tail): the level may be narrow (sparse, or after a narrow level).
__device__ inline bool listing_level(const Counters *c, int L, const LevelArgs &a) {
  if (!(a.flags & LV_TAIL) || (a.flags & LV_ROOTS) || L < 1) return false;
  return sparse_level(c, L, a.sparse_thresh) || c->ring[(L - 1) % LEVEL_RING] <= a.tail_max;
}


// Workgroup sum of a 64-bit value per thread; every thread gets it.
__device__ inline uint64_t block_sum64(uint64_t v) {
  __shared__ uint64_t part[4];
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d);
  if (lane_id() == 0) part[threadIdx.x >> 6] = v;
  __syncthreads();
  const uint64_t s = part[0] + part[1] + part[2] + part[3];
  __syncthreads();
  return s;
}

// Workgroup reduction of one value per wave; thread 0 gets the sum.
__device__ inline uint64_t block_sum4(uint64_t v) {
  __shared__ uint64_t part[4];
  const uint64_t w = __shfl(wave_incl_scan((uint32_t)v), 63);  // per-wave totals fit u32
  if (lane_id() == 0) part[threadIdx.x >> 6] = w;
  __syncthreads();
  const uint64_t s = part[0] + part[1] + part[2] + part[3];
  __syncthreads();  // `part` is reused by the next call
  return s;
}

// Bit j of the result: flag byte j of the 32 in f4 has (any bit of) `bit`.
// Four bytes per word by a multiply (bits 0, 8, 16, 24 -> 21 .. 24; the partial
// products never overlap), not 32 byte extractions held in registers.
__device__ inline uint32_t flag_bits(const uint4 (&f4)[2], uint8_t bit) {
  const uint32_t w[8] = {f4[0].x, f4[0].y, f4[0].z, f4[0].w, f4[1].x, f4[1].y, f4[1].z, f4[1].w};
  const uint32_t sh = __builtin_ctz(bit);
  uint32_t m = 0;
#pragma unroll
  for (int q = 0; q < 8; ++q) m |= ((((w[q] >> sh) & 0x01010101u) * 0x00204081u) >> 21 & 0xFu) << (4 * q);
  return m;
}

// Bit i of an 8-bit value -> bit 4i.
__device__ inline uint32_t spread8(uint32_t x) {
  x = (x | (x << 12)) & 0x000F000Fu;
  x = (x | (x << 6)) & 0x03030303u;
  return (x | (x << 3)) & 0x11111111u;
}

// ---------------------------------------------------------------------------
// k_frontier: one wave per 2048-slot block.  Candidate bytes (or, at level 0,
// the pseudo-root predicate) -> new frontier bits -> vis (the wave owns those
// words); frontier shadows are compacted in LDS with a ballot/popc scan; their
// supervisor edges are followed; their edge segments go to the block's region
// of `qn` (light) or, cut into RANGE_MAX pieces, to `qh` (hubs).
// ---------------------------------------------------------------------------
template <bool ROOTS, bool INVESTIGATE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(6, 8))) void k_frontier(DevGraph g, LevelArgs a) {
  __shared__ uint16_t s_front[4][BLK_SLOTS];  // offsets in the block: 16 KiB, so LDS allows 8 waves/SIMD
  Counters *c = g.ctr;
  const int L = a.level;
  if (c->tail_state) return;  // k_tail finished the mark (or bailed to a later level)
  if (blockIdx.x == 0 && threadIdx.x == 0) c->ring[(L + 1) % LEVEL_RING] = 0;
  uint64_t *stat = g.blkstat + (uint64_t)blockIdx.x * 4;
  if (!ROOTS && c->ring[(L - 1) % LEVEL_RING] == 0) {  // previous level was empty
    if (threadIdx.x == 0) stat[STAT_FRONT] = stat[STAT_MF] = 0;
    return;
  }
  const bool sp_cur = !ROOTS && sparse_level(c, L, a.sparse_thresh);
  const bool sp_next = sparse_level(c, L + 1, a.sparse_thresh);
  // Level 0 scans the shadows' own blocks; later levels the proxy region too
  // (sharded graphs: a proxy block only marks and lists its proxies).
  const VBlocks vbs = vblocks(g, !ROOTS);
  const int wv = threadIdx.x >> 6;
  const int lane = lane_id();
  const uint32_t gw = blockIdx.x * 4 + wv;
  const uint32_t nw = gridDim.x * 4;
  uint8_t *Fc = g.front[L & 1];
  uint8_t *Fn = g.front[(L + 1) & 1];
  uint8_t *Dc = g.dirty[L & 1];
  uint8_t *Dn = g.dirty[(L + 1) & 1];
  unsigned long long *qh_cnt = &c->qh[L & 1];
  const uint32_t tag = (uint32_t)(L + 1) << 12;
  const bool pull = !ROOTS && pull_level(c, L, a);
  const bool write_fx = pull || fx_level(c, L, a);
  const bool listing = !ROOTS && listing_level(c, L, a);
  // The pseudo-root level, binned: its supervisor pushes go to the block's
  // region of `tl_buf` (no level-0 listing uses it) and k_bin_place bins them
  // with the edge targets, instead of ~1e6 random candidate-byte stores here.
  const bool sup_list = ROOTS && !INVESTIGATE && (a.flags & LV_SUPBIN) && a.nbins > 0;
  uint32_t nsl = 0;
  const bool sharded = !ROOTS && g.n_shards > 1;
  // candidates from `cb` (k_expand(L-1) pulled and wrote them as bits)
  const bool from_cb = !ROOTS && (a.flags & LV_CBITS) && c->cb_level == (unsigned long long)L;
  const bool cb_two = from_cb && L == 1 && c->cb_two;
  const bool cb_ovf = cb_two && c->bin_ovf;
  const uint64_t st = c->slot_top;
  // pull levels without listing, proxies or Beamer's m_f: the per-lane path below
  const bool lane_pull = pull && !listing && !sharded && !a.alpha;
  uint32_t n_front = 0, n_sup = 0, n_edges = 0;

  for (uint32_t vb = gw; vb < vbs.n; vb += nw) {
    const uint32_t blk = vbs.at(vb);
    if (sp_cur && Dc[blk] == 0) continue;
    const uint64_t base = (uint64_t)blk * BLK_SLOTS + (uint64_t)lane * 32;
    const uint32_t word = g.vis[(uint64_t)blk * 64 + lane];
    uint32_t m = 0;
    uint4 f4[2] = {make_uint4(0, 0, 0, 0), make_uint4(0, 0, 0, 0)};  // the lane's 32 flag bytes
    bool have_f = false;
    if (ROOTS) {
      f4[0] = *(const uint4 *)(g.flags + base);
      f4[1] = *(const uint4 *)(g.flags + base + 16);
      have_f = true;
      const uint8_t *fb = (const uint8_t *)f4;
      if (INVESTIGATE) {
        // investigateRemotelyHeldActors: every shadow at `location` (:305-310)
#pragma unroll
        for (int j = 0; j < 32; ++j)
          if ((fb[j] & (FL_ALIVE | FL_PROXY)) == FL_ALIVE &&
              (uint16_t)(g.vid[base + j] >> 48) == a.location)
            m |= 1u << j;
      } else {
        // isPseudoRoot (:201-203): 32 flag bytes + 32 receive counts per lane
        uint32_t nz = 0;
        if (a.flags & LV_ROOTS_CO) {
          // The block's counts lane-interleaved (load q, lane l: slots
          // q*256 + 4l .. +3, so a load instruction reads 1 KiB of consecutive
          // counts, not 16 B of each of 64 lines), then transposed by ballots:
          // bit k of lane l's nibble of load q belongs to lane q*8 + l/8, bit
          // 4 (l % 8) + k.
          const int4 *rp = (const int4 *)(g.recv + (uint64_t)blk * BLK_SLOTS);
          int4 r4[8];
#pragma unroll
          for (int q = 0; q < 8; ++q) r4[q] = rp[q * 64 + lane];
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            const uint32_t b0 = (uint32_t)(__ballot(r4[q].x != 0) >> (8 * (lane & 7))) & 0xFFu;
            const uint32_t b1 = (uint32_t)(__ballot(r4[q].y != 0) >> (8 * (lane & 7))) & 0xFFu;
            const uint32_t b2 = (uint32_t)(__ballot(r4[q].z != 0) >> (8 * (lane & 7))) & 0xFFu;
            const uint32_t b3 = (uint32_t)(__ballot(r4[q].w != 0) >> (8 * (lane & 7))) & 0xFFu;
            const uint32_t w = spread8(b0) | (spread8(b1) << 1) | (spread8(b2) << 2) | (spread8(b3) << 3);
            if ((lane >> 3) == q) nz = w;
          }
        } else {
          int4 r4[8];
          const int4 *rp = (const int4 *)(g.recv + base);
#pragma unroll
          for (int q = 0; q < 8; ++q) r4[q] = rp[q];
          const int32_t *rb = (const int32_t *)r4;
#pragma unroll
          for (int j = 0; j < 32; ++j) nz |= rb[j] != 0 ? (1u << j) : 0u;
        }
        m = flag_bits(f4, FL_ALIVE) & ~flag_bits(f4, FL_HALTED) & ~flag_bits(f4, FL_PROXY) &
            (flag_bits(f4, FL_ROOT) | flag_bits(f4, FL_BUSY) | ~flag_bits(f4, FL_INTERNED) | nz);
      }
    } else if (from_cb) {
      // the pull level before wrote this level's candidates as bits (words
      // past slot_top are never written: masked)
      uint32_t bits = g.cb[(uint64_t)blk * 64 + lane];
      if (cb_two) {  // level 1 after a binned level 0
        bits |= g.cb2[(uint64_t)blk * 64 + lane];
        if (cb_ovf && Dc[blk]) {  // a full slice's targets in this block went out as bytes
          uint4 *fp = (uint4 *)(Fc + base);
          const uint4 x0 = fp[0], x1 = fp[1];
          const uint32_t xs[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
#pragma unroll
          for (int q = 0; q < 8; ++q)
#pragma unroll
            for (int k = 0; k < 4; ++k) bits |= ((xs[q] >> (8 * k)) & 0xFFu) ? (1u << (4 * q + k)) : 0u;
          fp[0] = make_uint4(0, 0, 0, 0);
          fp[1] = make_uint4(0, 0, 0, 0);
          wave_lds_fence();  // (every lane has read the block's dirty byte)
          if (lane == 0) Dc[blk] = 0;
        }
      }
      if (base + 32 > st) bits &= base >= st ? 0u : ((1u << (uint32_t)(st - base)) - 1u);
      m = bits & ~word;
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
    if (!ROOTS && vbs.proxy(vb)) {
      // A proxy block: its proxies are marked (k_xscan exports the newly
      // marked ones after the round); proxies have no edges, so nothing else —
      // and they do not count in the level's frontier (a level that only
      // reaches proxies ends the round).
      continue;
    }

    // Compact this block's frontier slots into LDS (ballot/popc scan).
    const uint32_t cnt = __popc(m);
    const uint32_t incl = wave_incl_scan(cnt);
    const uint32_t total = __shfl(incl, 63);
    uint32_t pos = incl - cnt;
    // The frontier slots' halted / proxy bits travel with their LDS entries
    // (bits 11, 12), so the per-shadow loop below gathers no flag bytes.
    uint32_t halted = 0, proxy = 0;
    if (m) {
      if (!have_f) {
        f4[0] = *(const uint4 *)(g.flags + base);
        f4[1] = *(const uint4 *)(g.flags + base + 16);
      }
      halted = flag_bits(f4, FL_HALTED);
      proxy = flag_bits(f4, FL_PROXY);
    }
    // expandable frontier = frontier minus halted shadows (this wave owns the words)
    if (write_fx) g.fx[(uint64_t)blk * 64 + lane] = m & ~halted;
    if (lane_pull) {
      // Pull level: no edge ranges to list, only supervisor edges (:258-267).
      // The block's supervisors are read in 8 coalesced 16-B loads per lane
      // (load q, lane l: slots q*256 + 4l .. +3, whose frontier bits come from
      // lane q*8 + l/8 by one shuffle), then their marked words in two groups
      // of 16 loads in flight: three dependent round trips per block instead
      // of two per 64*FB frontier shadows after an LDS compaction.
      n_front += cnt;
      const uint32_t e = INVESTIGATE ? 0u : (m & ~halted);
      if (__ballot(e != 0)) {
        const uint4 *sp4 = (const uint4 *)(g.sup + (uint64_t)blk * BLK_SLOTS);
        uint4 s4[8];
        uint32_t eb = 0;  // 4 bits per load
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const uint32_t b4 = (__shfl(e, q * 8 + (lane >> 3)) >> ((lane & 7) * 4)) & 0xFu;
          eb |= b4 << (4 * q);
          s4[q] = b4 ? sp4[q * 64 + lane] : make_uint4(~0u, ~0u, ~0u, ~0u);
        }
        const uint32_t *ss = (const uint32_t *)s4;
        uint32_t sv = 0;
#pragma unroll
        for (int j = 0; j < 32; ++j) sv |= (((eb >> j) & 1u) && ss[j] < 0xFFFFFFF0u) ? (1u << j) : 0u;
        n_sup += __popc(sv);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          uint32_t w[16];
#pragma unroll
          for (int k = 0; k < 16; ++k) {
            const int j = 16 * h + k;
            w[k] = ((sv >> j) & 1u) ? g.vis[ss[j] >> 5] : ~0u;
          }
#pragma unroll
          for (int k = 0; k < 16; ++k) {
            const uint32_t s = ss[16 * h + k];
            if (!((w[k] >> (s & 31)) & 1u)) {
              Fn[s] = 1;
              if (sp_next) Dn[s >> 11] = 1;  // blind: no dependent read
            }
          }
        }
      }
      continue;
    }
    while (m) {
      const int j = __ffs(m) - 1;
      m &= m - 1;
      s_front[wv][pos++] = (uint16_t)((lane * 32 + j) | (((halted >> j) & 1u) << 11) | (((proxy >> j) & 1u) << 12));
    }
    n_front += cnt;
    wave_lds_fence();
    if (listing && total) {  // into the block's own region: no shared counter
      for (uint32_t i = lane; i < total; i += 64)
        g.tl_buf[(uint64_t)blk * BLK_SLOTS + i] = blk * BLK_SLOTS + (s_front[wv][i] & (BLK_SLOTS - 1));
      if (lane == 0) g.tl_tag[blk] = tag | total;
    }

    // Frontier shadows -> supervisor marks + edge ranges (push levels).
    uint32_t nlight = 0;
    uint2 *region = g.qn_buf + (uint64_t)blk * BLK_SLOTS;
    // FB chunks of 64 frontier shadows at a time: every per-shadow load of the
    // group (flags, degree, segment, supervisor) is issued before any store,
    // then the supervisors' marked words, so a dense block costs two memory
    // round trips per 64*FB shadows instead of two per 64.
    for (uint32_t c0 = 0; c0 < total; c0 += 64 * FB) {
      uint32_t v[FB], nz[FB], sp[FB];
      uint8_t f[FB];  // FL_HALTED / FL_PROXY, from the LDS entry
      uint2 ad[FB];
#pragma unroll
      for (int b = 0; b < FB; ++b) {
        const uint32_t idx = c0 + b * 64 + lane;
        const uint32_t e = idx < total ? s_front[wv][idx] : 0u;
        v[b] = idx < total ? blk * BLK_SLOTS + (e & (BLK_SLOTS - 1)) : NO_SLOT;
        f[b] = (uint8_t)(((e >> 11) & 1u) ? FL_HALTED : 0) | (uint8_t)(((e >> 12) & 1u) ? FL_PROXY : 0);
      }
#pragma unroll
      for (int b = 0; b < FB; ++b) {
        const bool valid = v[b] != NO_SLOT;
        nz[b] = (valid && a.alpha) ? g.nzdeg[v[b]] : 0;  // Beamer's m_f only: the sweep counts traced edges
        ad[b] = (valid && !pull) ? g.adj[v[b]] : make_uint2(0, 0);
        sp[b] = (valid && !INVESTIGATE) ? g.sup[v[b]] : NO_SLOT;
      }
      uint32_t sw[FB];
#pragma unroll
      for (int b = 0; b < FB; ++b) {
        // halted: marked, not expanded (:226); supervisor edge (:258-267) unless null / collected
        if (v[b] == NO_SLOT || (f[b] & FL_HALTED)) {
          nz[b] = 0;
          ad[b] = make_uint2(0, 0);
          sp[b] = NO_SLOT;
        }
        if (sp[b] >= 0xFFFFFFF0u) sp[b] = NO_SLOT;
        sw[b] = sp[b] != NO_SLOT ? g.vis[sp[b] >> 5] : ~0u;
      }
#pragma unroll
      for (int b = 0; b < FB; ++b) {
        n_edges += nz[b];  // this level's frontier out-edges (Beamer's m_f)
        const bool push_s = sp[b] != NO_SLOT && !((sw[b] >> (sp[b] & 31)) & 1u);
        if (sp[b] != NO_SLOT) n_sup++;
        if (sup_list) {
          const uint64_t bl = __ballot(push_s);
          if (push_s) g.tl_buf[(uint64_t)blk * BLK_SLOTS + nsl + __popcll(bl & lanemask_lt())] = sp[b];
          nsl += __popcll(bl);
        } else if (push_s) {
          const uint32_t s = sp[b];
          Fn[s] = 1;
          if (sp_next) Dn[s >> 11] = 1;  // blind: no dependent read
        }
        const uint32_t len = ad[b].y;
        const bool light = len > 0 && len <= RANGE_MAX;
        const uint64_t ball = __ballot(light);
        if (light) region[nlight + __popcll(ball & lanemask_lt())] = ad[b];
        nlight += __popcll(ball);
        const uint32_t pieces = len > RANGE_MAX ? (len + RANGE_MAX - 1) / RANGE_MAX : 0;
        if (__ballot(pieces != 0)) {  // hubs are rare: a wave-aggregated append
          const unsigned long long hi = wave_atomic_add(qh_cnt, pieces);
          for (uint32_t k = 0; k < pieces; ++k) {
            const uint32_t pl = min(RANGE_MAX, len - k * RANGE_MAX);
            if (hi + k < g.qh_cap) g.qh_buf[hi + k] = make_uint2(ad[b].x + k * RANGE_MAX, pl);
            else set_err(c, ERR_QUEUE_FULL);
          }
        }
      }
    }
    if (lane == 0 && nlight) g.qn_tag[blk] = tag | nlight;
    if (sup_list) {
      if (lane == 0 && nsl) g.tl_tag[blk] = (1u << 12) | nsl;
      nsl = 0;
    }
    wave_lds_fence();
  }
  const uint64_t tf = block_sum4(n_front);
  const uint64_t ts = block_sum4(n_sup);
  const uint64_t te = block_sum4(n_edges);
  if (threadIdx.x == 0) {
    stat[STAT_FRONT] = tf;
    stat[STAT_SUP] += ts;
    stat[STAT_MF] = te;  // this level's only (the sweep reuses the slot afterwards)
  }
}

// U edges of one lane (:231-241).  Each phase issues all its loads
// before any is waited on: the vis words, then the candidate bytes of the
// targets still unmarked, then the stores — two dependent round trips per
// group of edges instead of two per edge (a byte store may alias any load, so
// per-edge marking would serialise them).
// Candidate bytes are stored blind: no marked-word filter, no read of the
// byte first.  A byte stored for a marked target is dropped by the next
// k_frontier (bits & ~vis), and a byte store is idempotent across XCDs, so the
// edge load is the only round trip an edge costs (mark -13 % on the C2 wakeup
// against filter + read-before-store: profiles/r2e/ab.json).
// smask / slice: with target slices (LevelArgs::xslices > 1) a workgroup
// stores only the candidates of its slice, ((t >> 11) & smask) == slice.
template <int U>
__device__ inline void expand_edges(const DevGraph &g, uint8_t *Fn, uint8_t *Dn, bool sp_next,
                                    const uint64_t (&ed)[U], uint32_t &nb, uint32_t smask, uint32_t slice) {
  uint32_t t[U];
  bool go[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    t[u] = edge_target(ed[u]);
    go[u] = edge_count(ed[u]) > 0 && ((t[u] >> 11) & smask) == slice;
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    nb += go[u] ? 1 : 0;
    if (go[u]) Fn[t[u]] = 1;
  }
  if (sp_next) {  // the block's dirty byte, stored blind like the candidate byte
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (go[u]) Dn[t[u] >> 11] = 1;
  }
}

// ---------------------------------------------------------------------------
// k_expand: every wave of the grid walks the level's ranges, 64 light ranges
// per step (degree scan + binary search in LDS assigns edges to lanes) or one
// hub piece per step, U independent edge loads per lane.
// ---------------------------------------------------------------------------
// The edge stream is read once per level: non-temporal, so it does not evict
// the marked words and candidate bytes the level keeps re-reading.
__device__ inline uint64_t pool_load(const uint64_t *p) { return __builtin_nontemporal_load(p); }

constexpr int EXPAND_U = 4;  // independent edge loads per lane per step

// The workgroup's byte count (2x, per thread) into its partial: one add per
// workgroup, after every wave of it is done.
__device__ inline void expand_bytes_out(const DevGraph &g, uint32_t nb2) {
  __shared__ unsigned long long s_nb;
  if (threadIdx.x == 0) s_nb = 0;
  __syncthreads();
  const uint32_t w = wave_sum(nb2);
  if (lane_id() == 0 && w) atomicAdd(&s_nb, (unsigned long long)w);
  __syncthreads();
  if (threadIdx.x == 0) g.xbytes[blockIdx.x] += s_nb / 2;
}

// Bits 0, 8, 16, 24 of a pull thread's `found` -> bits 0 .. 3.
__device__ inline uint32_t found_nibble(uint32_t f) {
  return (f & 1u) | ((f >> 7) & 2u) | ((f >> 14) & 4u) | ((f >> 21) & 8u);
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_expand(DevGraph g, LevelArgs a) {
  constexpr int U = EXPAND_U;
  __shared__ uint32_t s_start[4][65];
  __shared__ uint32_t s_off[4][64];
  Counters *c = g.ctr;
  const int L = a.level;
  if (c->tail_state) return;
  if (L > 0 && c->ring[(L - 1) % LEVEL_RING] == 0) return;  // nothing was found this level
  const uint64_t nh = min(c->qh[L & 1], (unsigned long long)g.qh_cap);
  const bool sp_next = sparse_level(c, L + 1, a.sparse_thresh);
  uint8_t *Fn = g.front[(L + 1) & 1];
  uint8_t *Dn = g.dirty[(L + 1) & 1];
  const int wv = threadIdx.x >> 6;
  const int lane = lane_id();
  uint64_t gw = (uint64_t)blockIdx.x * 4 + wv;
  uint64_t nw = (uint64_t)gridDim.x * 4;
  const uint32_t want = (uint32_t)(L + 1);
  const uint64_t nblk = (c->slot_top + BLK_SLOTS - 1) / BLK_SLOTS;
  // A candidate byte stored for an already-marked target is dropped by the next
  // k_frontier (bits & ~vis), so the filter is an optimisation only.
  // Bytes this launch reads and writes, by element width (the roofline
  // numerator): twice the count, so 8.5-B items stay integral.
  uint32_t nb2 = 0;

  if (pull_now(c, L, a)) {
    if (L < 64 && blockIdx.x == 0 && threadIdx.x == 0 && pull_now<false>(c, L, a)) c->pulled |= 1ull << L;
    // Pull: each unmarked, not-yet-found shadow looks for an expandable
    // frontier shadow among its in-candidates whose edge to it has a
    // positive count (RC_POS), and stops at the first.  A thread owns 4
    // consecutive slots (their candidate bytes are one u32), so loads of
    // flags / bytes / radj are coalesced across the wave.
    // (sharded graphs: the proxy region's quads after the shadows' own — a
    // proxy reached from the expandable frontier is marked like any target)
    const uint64_t nqh = (c->slot_top + 3) / 4;
    const uint64_t nq = nqh + (c->proxy_top + 3) / 4;
    const uint64_t gs = (uint64_t)gridDim.x * 256;
    // Candidates as bits (LV_CBITS, unsharded graphs): this pass reads every
    // slot's candidate byte anyway, so it hands level L+1 the complete set —
    // supervisor bytes | finds — as words of `cb` (eight threads' nibbles, one
    // word; every word below slot_top is written) and clears the bytes it
    // read.  k_frontier(L+1) then reads 1 bit per slot instead of reading and
    // clearing a byte.
    const bool to_cb = (a.flags & LV_CBITS) && g.n_shards <= 1 && c->proxy_top == 0;
    if (to_cb && blockIdx.x == 0 && threadIdx.x == 0) c->cb_level = (unsigned long long)(L + 1);
    // (Loading the hints and in-candidate ranges with the flags while a
    // quarter of the slots are unmarked, and the hints' frontier bits with
    // the lists' first chunks, made level 1 slower: 146 -> 181 us, r3g/ab4.)
    // The loop bound is wave-uniform (a wave's 64 quads are consecutive), so
    // the nibble exchange below runs with every lane.
    const uint64_t qw0 = (uint64_t)blockIdx.x * 256 + (threadIdx.x & ~63u);
    for (uint64_t qw = qw0; qw < nq; qw += gs) {
      const uint64_t q = qw + (uint64_t)lane;
      uint32_t nib = 0;  // (to_cb) this quad's candidates for level L+1
      do {
      if (q >= nq) break;
      const uint64_t v0 = q < nqh ? q * 4 : g.pbase + (q - nqh) * 4;
      const uint32_t fl = *(const uint32_t *)(g.flags + v0);
      const uint32_t cand = *(const uint32_t *)(Fn + v0);
      const uint32_t vb = (g.vis[v0 >> 5] >> (v0 & 31)) & 0xFu;
      nb2 += 17;  // flags + candidate bytes (4 + 4 B) + an eighth of a marked word
      uint32_t todo = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        todo |= (((fl >> (8 * j)) & FL_ALIVE) && !((cand >> (8 * j)) & 0xFFu) && !((vb >> j) & 1u))
                    ? (1u << j) : 0u;
      if (to_cb && cand) {
#pragma unroll
        for (int j = 0; j < 4; ++j) nib |= ((cand >> (8 * j)) & 0xFFu) ? (1u << j) : 0u;
        *(uint32_t *)(Fn + v0) = 0;
        nb2 += 8;
      }
      if (!todo) break;
      uint32_t found = 0;
      // Hints first: the owner a pull level found last time, if its edge is
      // still positive (hints are cleared when it stops being) and it is in
      // the expandable frontier now — one L2-resident bit, no candidate list.
      {
        const uint4 h4 = *(const uint4 *)(g.par + v0);
        const uint32_t hs[4] = {h4.x, h4.y, h4.z, h4.w};
        nb2 += 32;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const uint32_t h = hs[j];
          if (((todo >> j) & 1u) && h < 0xFFFFFFF0u && ((g.fx[h >> 5] >> (h & 31)) & 1u)) {
            found |= 1u << (8 * j);
            todo &= ~(1u << j);
            nb2 += 8;
          }
        }
      }
      if (!todo) {
        if (to_cb) {
          nib |= found_nibble(found);
        } else {
          *(uint32_t *)(Fn + v0) = cand | found;
          nb2 += 8;
        }
        break;
      }
      const uint4 r01 = *(const uint4 *)(g.radj + v0);
      const uint4 r23 = *(const uint4 *)(g.radj + v0 + 2);
      const uint32_t ro[4] = {r01.x, r01.z, r23.x, r23.z};
      const uint32_t rl[4] = {rseg_len(r01.y), rseg_len(r01.w), rseg_len(r23.y), rseg_len(r23.w)};
      nb2 += 64;  // four in-candidate ranges
      // The thread's (up to) 4 lists are walked together, one round trip for
      // the candidates and one for their frontier bits per round, until every
      // list has a hit or is exhausted.  Each list is read as aligned 16-B
      // chunks (one request for up to four candidates; entries outside
      // [ro, ro + rl) belong to other segments and are masked).
      uint32_t p[4], e[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        p[j] = ro[j];
        e[j] = ro[j] + rl[j];
      }
      uint32_t live = todo;
      while (live) {
        uint4 u4[4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
          u4[j] = ((live >> j) & 1u) && p[j] < e[j] ? *(const uint4 *)(g.rpool + (p[j] & ~3u))
                                                    : make_uint4(0, 0, 0, 0);
        uint32_t u[4][4];
        uint32_t w[4][4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const uint32_t a0 = p[j] & ~3u;
          const uint32_t uu[4] = {u4[j].x, u4[j].y, u4[j].z, u4[j].w};
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const bool in = ((live >> j) & 1u) && a0 + k >= p[j] && a0 + k < e[j];
            u[j][k] = in ? uu[k] : 0u;
            nb2 += in ? 8 : 0;
          }
        }
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const uint32_t sl = u[j][k] & ~RC_POS;
            w[j][k] = (u[j][k] & RC_POS) ? g.fx[sl >> 5] >> (sl & 31) : 0u;  // 0: no RC_POS
            nb2 += (u[j][k] & RC_POS) ? 8 : 0;
          }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          p[j] = (p[j] & ~3u) + 4;
          bool hit = false;
          uint32_t who = 0;
#pragma unroll
          for (int k = 3; k >= 0; --k)
            if (w[j][k] & 1u) {
              hit = true;
              who = u[j][k] & ~RC_POS;
            }
          if (hit && ((live >> j) & 1u)) {
            found |= 1u << (8 * j);
            g.par[v0 + j] = who;  // the next trace tries this owner first
            nb2 += 8;
          }
          if (hit || p[j] >= e[j]) live &= ~(1u << j);
        }
      }
      if (to_cb) {
        nib |= found_nibble(found);
      } else if (found) {
        *(uint32_t *)(Fn + v0) = cand | found;
        nb2 += 8;
      }
      } while (false);
      if (to_cb) {
        // lanes 8k .. 8k+7 hold the nibbles of word (qw + 8k) / 8
        uint32_t w = nib << (4 * (lane & 7));
        w |= __shfl_xor(w, 1);
        w |= __shfl_xor(w, 2);
        w |= __shfl_xor(w, 4);
        if ((lane & 7) == 0 && q < nq) {
          g.cb[q >> 3] = w;
          nb2 += 8;  // an eighth of a candidate word per slot, times 4 slots, times 2
        }
      }
    }
    expand_bytes_out(g, (a.flags & LV_NOBYTES) ? 0u : nb2);
    return;
  }

  // Push with target slices: the grid is split into S sub-grids, workgroup b
  // in slice b % S (blocks are dealt round-robin over the 8 XCDs, so a slice
  // stays on S / 8 of them); every sub-grid walks all the level's edges and
  // stores only its slice's candidate bytes, so a candidate line is dirtied by
  // one slice's XCDs instead of by all eight (partial-line write-backs).
  const uint32_t S = a.xslices > 1 ? a.xslices : 1u;
  const uint32_t smask = S - 1, slice = blockIdx.x & smask;
  gw = (uint64_t)(blockIdx.x / S) * 4 + wv;
  nw = (uint64_t)(gridDim.x / S) * 4;
  if (blockIdx.x >= (gridDim.x / S) * S) nw = 0;  // a partial last set of slices: idle
  // light ranges: chunk (block b, k-th 64) of every block's region; chunk ids
  // run over blocks first so consecutive waves take different blocks, and wave
  // gw takes ids gw, gw + nw, gw + 2 nw, ...  It reads the tags of 64 of its
  // ids at once (one per lane) and walks the chunks that have ranges: one tag
  // round trip per 64 ids, not one per id (a sparse level's scan of nblk * 32
  // ids was a chain of dependent L2 reads).
  const uint64_t ncid = nblk * 32;
  for (uint64_t cb = gw; nw && cb < ncid; cb += nw * 64) {
    const uint64_t mc = cb + (uint64_t)lane * nw;
    uint32_t mt = 0;
    if (mc < ncid) {
      const uint32_t t = g.qn_tag[mc % nblk];
      const uint32_t mk = (uint32_t)(mc / nblk);
      if ((t >> 12) == want && (t & 0xFFFu) > mk * 64) mt = t;
    }
    nb2 += mc < ncid ? 8 : 0;
    uint64_t todo = __ballot(mt != 0);
    while (todo) {
      const int jl = __ffsll((unsigned long long)todo) - 1;
      todo &= todo - 1;
      const uint64_t cid = cb + (uint64_t)jl * nw;
      const uint64_t b = cid % nblk;
      const uint32_t k = (uint32_t)(cid / nblk);
      const uint32_t cnt = __shfl(mt, jl) & 0xFFFu;
      const uint32_t qi = k * 64 + lane;
      const uint2 r = qi < cnt ? g.qn_buf[b * BLK_SLOTS + qi] : make_uint2(0, 0);
      nb2 += qi < cnt ? 16 : 0;
      const uint32_t incl = wave_incl_scan(r.y);
      const uint32_t dtot = __shfl(incl, 63);
      s_start[wv][lane] = incl - r.y;
      s_off[wv][lane] = r.x;
      wave_lds_fence();
      for (uint32_t e0 = 0; e0 < dtot; e0 += 64 * U) {
        uint64_t ed[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const uint32_t e = e0 + u * 64 + lane;
          ed[u] = 0;  // count 0: neither traced nor counted
          if (e < dtot) {
            int lo = 0, hi = 63;
            while (lo < hi) {
              const int mid = (lo + hi + 1) >> 1;
              if (s_start[wv][mid] <= e) lo = mid;
              else hi = mid - 1;
            }
            ed[u] = pool_load(&g.pool[(uint64_t)s_off[wv][lo] + (e - s_start[wv][lo])]);
            nb2 += 16;
          }
        }
        uint32_t nb = 0;
        expand_edges(g, Fn, Dn, sp_next, ed, nb, smask, slice);
        nb2 += 2 * nb;
      }
      wave_lds_fence();
    }
  }
  // hub pieces: one per step
  for (uint64_t hi = gw; nw && hi < nh; hi += nw) {
    const uint2 r = g.qh_buf[hi];
    nb2 += lane == 0 ? 16 : 0;
    for (uint32_t e0 = 0; e0 < r.y; e0 += 64 * U) {
      uint64_t ed[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t e = e0 + u * 64 + lane;
        ed[u] = e < r.y ? pool_load(&g.pool[(uint64_t)r.x + e]) : 0;
        nb2 += e < r.y ? 16 : 0;
      }
      uint32_t nb = 0;
      expand_edges(g, Fn, Dn, sp_next, ed, nb, smask, slice);
      nb2 += 2 * nb;
    }
  }
  expand_bytes_out(g, (a.flags & LV_NOBYTES) ? 0u : nb2);
}


// ---------------------------------------------------------------------------
// The pseudo-root level's push, binned.  Level 0 of a wide trace pushes ~1e7
// candidate bytes to random slots of a ~10 MB byte map that no XCD's 4 MB L2
// holds: the edge stream takes ~22 us, the random byte stores ~215 us (C2,
// profiles/r3g/lv1).  Binned, the stores become sequential.
//   k_bin_place  one walk over the level's units (light chunks, hub pieces) by
//                BIN_WG workgroups of 16 waves; each wave sorts a window of its
//                targets by bin in LDS, reserves each bin's run in its
//                (bin, workgroup) slice — a fixed-capacity piece of the region,
//                bin-major — from an LDS cursor (nbins <= 256 ranges of
//                2^bin_shift slots), and stores the runs from consecutive lanes
//                (r4o: level 0 138 -> 133 us); a target past its slice's
//                capacity is stored as a byte at once.  The slice counts go out
//                at the end.  No barrier per unit, no global atomic.
//   k_bin_apply  two workgroups per bin, each over half its slices (16-B
//                loads, the slice counts in LDS) into an LDS bitmap of the
//                bin's slot range, whose bits become candidate bytes.
// The line footprint of the open slices is what the place pass pays for: with
// 2048 workgroups of 4 waves (round 4's first count-then-place form) the
// ~344k slices' partly written lines did not fit the L2s and left them partly
// written, and a count pass + scan sized the slices exactly (level 0: 60 + 15
// + 131 + 28 us, profiles/r4d); 512 workgroups of 16 waves keep the same waves
// with a quarter of the slices, and fixed-capacity slices need no count pass.
// Staging the targets in per-bin LDS rings and storing whole 64-B groups
// (a lock-free ring: exchange, group flush by the last position's lane,
// eviction, final flush) was correct but slower, 150 -> 220 us: the 8-B LDS
// exchanges and flush checks cost more than the stores they combined
// (profiles/r4i).
// Used only when the level-0 frontier is >= 1/32 of the slots (the place pass
// derives it and sets the mode word for k_bin_apply; not binned, it stores the
// bytes at once).
// ---------------------------------------------------------------------------
__device__ inline bool bin_mode(const Counters *c, const LevelArgs &a) {
  return a.nbins > 0 && a.nbins <= BIN_MAX && c->ring[0] * 32 >= c->slot_top;
}

constexpr int BIN_T = 1024;  // threads of a k_bin_place / k_bin_apply workgroup
constexpr int BIN_NW = BIN_T / 64;

// B16 (bins of 2^16 slots, C2 scale): a target is stored as its 16-bit offset
// in the bin, halving the place pass's writes and the apply pass's reads
// (57 MB of 4-B slots per launch for a 13 MB byte map).
template <bool B16>
__global__ __launch_bounds__(BIN_T) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_bin_place(DevGraph g, LevelArgs a) {
  constexpr int U = EXPAND_U;  // (8 edge loads per lane did not pay with the sorted stores' registers)
  __shared__ uint32_t s_start[BIN_NW][65];
  __shared__ uint32_t s_off[BIN_NW][64];
  __shared__ uint32_t s_ulist[BIN_T], s_utag[BIN_T], s_wcnt[BIN_NW], s_nact;
  __shared__ uint32_t lc[BIN_MAX];  // the next position of each bin's slice of this workgroup
  // per wave: a bin table (counts, then prefix | slice reservation << 9 in one
  // word: a window's prefix is <= 64 U = 256, a reservation is clamped to
  // bin_slice < 2^23, so BIN_MAX = 512 bins fit the LDS of two tables of 256)
  // and the window's targets sorted by bin
  __shared__ uint32_t s_wa[BIN_NW][BIN_MAX];
  __shared__ uint32_t s_ws[BIN_NW][64 * U];
  Counters *c = g.ctr;
  const bool binned = !c->tail_state && bin_mode(c, a);
  // k_bin_apply runs after this kernel (stream order) and reads the word
  if (blockIdx.x == 0 && threadIdx.x == 0) a.bin_mode_w[0] = binned ? 1u : 0u;
  if (c->tail_state) return;
  const uint32_t NB = a.nbins;
  const uint32_t SC = a.bin_slice;
  uint8_t *Fn = g.front[1];
  uint8_t *Dn1 = g.dirty[1];  // level 1's blocks with candidate bytes (a full slice's targets)
  const int wv = threadIdx.x >> 6, lane = lane_id(), tid = threadIdx.x;
  const uint64_t G = gridDim.x, wg = blockIdx.x;
  const uint64_t nblk = (c->slot_top + BLK_SLOTS - 1) / BLK_SLOTS;
  const uint64_t ncid = nblk * 32;
  const uint64_t nh = min(c->qh[0], (unsigned long long)g.qh_cap);
  // k_frontier(0)'s supervisor pushes (LV_SUPBIN): chunks (block b, k-th 256)
  // of the blocks' tl_buf regions, after the edge units
  const uint64_t nsc = ((a.flags & LV_SUPBIN) && !(a.flags & LV_INVESTIGATE)) ? nblk * (BLK_SLOTS / 256) : 0;
  const uint64_t nunits = ncid + nh + nsc;
  uint32_t nb2 = 0;
  if (binned)
    for (uint32_t k = tid; k < NB; k += BIN_T) lc[k] = 0;
  __syncthreads();

  // (not binned: the candidate byte at once; a binned level goes through `edges`)
  auto put = [&](uint32_t t) { Fn[t] = 1; };
  // A window of the wave's targets (64 U), binned: counted per bin in the
  // wave's table, a slice range reserved per (wave, bin) at once, the targets
  // sorted by bin in LDS, then stored by consecutive lanes in sorted order, so
  // a bin's run of targets goes out as consecutive addresses of its slice
  // (one memory request per run instead of one per target).
  auto edges = [&](const uint64_t (&ed)[U]) {
    if (!binned) {
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (edge_count(ed[u]) > 0) put(edge_target(ed[u]));
      return;
    }
    uint32_t *A = s_wa[wv], *S = s_ws[wv];
    for (uint32_t k = lane; k < NB; k += 64) A[k] = 0;
    wave_lds_fence();
    uint32_t t[U], r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      t[u] = edge_target(ed[u]);
      const uint32_t b = t[u] >> a.bin_shift;
      r[u] = 0xFFFFFFFFu;
      if (edge_count(ed[u]) > 0) {
        if (b < NB) r[u] = atomicAdd(&A[b], 1u);
        else {
          Fn[t[u]] = 1;  // (a slot past the bins: never, slot_top is synced)
          Dn1[t[u] >> 11] = 1;
          c->bin_ovf = 1;
        }
      }
    }
    wave_lds_fence();
    uint32_t run = 0;
    for (uint32_t k0 = 0; k0 < NB; k0 += 64) {  // A: counts -> prefix | reservation << 9
      const uint32_t k = k0 + lane;
      const uint32_t cnt = k < NB ? A[k] : 0u;
      const uint32_t incl = wave_incl_scan(cnt);
      const uint32_t pre = run + incl - cnt;
      if (k < NB) A[k] = pre | (min(cnt ? atomicAdd(&lc[k], cnt) : 0u, SC) << 9);
      run += __shfl(incl, 63);
    }
    wave_lds_fence();
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (r[u] != 0xFFFFFFFFu) S[(A[t[u] >> a.bin_shift] & 511u) + r[u]] = t[u];
    wave_lds_fence();
    for (uint32_t i = lane; i < run; i += 64) {
      const uint32_t tt = S[i], b = tt >> a.bin_shift, e = A[b];
      const uint32_t pos = (e >> 9) + i - (e & 511u);  // slice position = reservation + rank in the bin
      if (pos < SC) {
        const uint64_t at = ((uint64_t)b * G + wg) * SC + pos;
        if (B16) {
          reinterpret_cast<uint16_t *>(a.bins)[at] = (uint16_t)(tt - (b << 16));
          nb2 += 4;
        } else {
          a.bins[at] = tt;
          nb2 += 8;
        }
      } else {
        Fn[tt] = 1;  // past the slice: the byte at once
        Dn1[tt >> 11] = 1;  // (k_frontier(1) reads the bytes of such blocks besides the bits)
        c->bin_ovf = 1;
      }
    }
    wave_lds_fence();  // the table and the sorted window are reused by the next window
  };
  auto unit = [&](uint64_t un, uint32_t tag) {
    if (un < ncid) {  // light ranges: chunk (block b, k-th 64)
      const uint64_t b = un % nblk;
      const uint32_t k = (uint32_t)(un / nblk);
      const uint32_t cnt = tag & 0xFFFu;
      const uint32_t qi = k * 64 + lane;
      const uint2 rr = qi < cnt ? g.qn_buf[b * BLK_SLOTS + qi] : make_uint2(0, 0);
      nb2 += qi < cnt ? 16 : 0;
      const uint32_t incl = wave_incl_scan(rr.y);
      const uint32_t dtot = __shfl(incl, 63);
      s_start[wv][lane] = incl - rr.y;
      s_off[wv][lane] = rr.x;
      wave_lds_fence();
      for (uint32_t e0 = 0; e0 < dtot; e0 += 64 * U) {
        uint64_t ed[U];
#pragma unroll
        for (int uu = 0; uu < U; ++uu) {
          const uint32_t e = e0 + uu * 64 + lane;
          ed[uu] = 0;
          if (e < dtot) {
            int lo = 0, hi = 63;
            while (lo < hi) {
              const int mid = (lo + hi + 1) >> 1;
              if (s_start[wv][mid] <= e) lo = mid;
              else hi = mid - 1;
            }
            ed[uu] = pool_load(&g.pool[(uint64_t)s_off[wv][lo] + (e - s_start[wv][lo])]);
            nb2 += 16;
          }
        }
        edges(ed);
      }
      wave_lds_fence();
    } else if (un >= ncid + nh) {  // supervisor pushes: up to 256 of a block's
      const uint64_t sc = un - ncid - nh;
      const uint64_t b = sc % nblk;
      const uint32_t k = (uint32_t)(sc / nblk);
      const uint32_t cnt = tag & 0xFFFu;
      uint64_t ed[U];
#pragma unroll
      for (int uu = 0; uu < U; ++uu) {
        const uint32_t i = k * 256 + uu * 64 + lane;
        ed[uu] = i < cnt ? ((1ull << 32) | g.tl_buf[b * BLK_SLOTS + i]) : 0;  // count 1: a candidate
        nb2 += i < cnt ? 8 : 0;
      }
      edges(ed);
    } else {  // a hub piece
      const uint2 rr = g.qh_buf[un - ncid];
      nb2 += lane == 0 ? 16 : 0;
      for (uint32_t e0 = 0; e0 < rr.y; e0 += 64 * U) {
        uint64_t ed[U];
#pragma unroll
        for (int uu = 0; uu < U; ++uu) {
          const uint32_t e = e0 + uu * 64 + lane;
          ed[uu] = e < rr.y ? pool_load(&g.pool[(uint64_t)rr.x + e]) : 0;
          nb2 += e < rr.y ? 16 : 0;
        }
        edges(ed);
      }
    }
  };

  // Unit ids are dealt round-robin over the workgroups (workgroup w, window i,
  // thread t: id (BIN_T i + t) G + w): light chunks with work cluster at the
  // low ids (k = 0 .. 3 of every block at level 0), so consecutive windows
  // would leave most workgroups idle.  Within a window every wave takes every
  // BIN_NW-th unit with work, at its own pace: nothing waits on another wave.
  for (uint64_t ub = 0; ub * G < nunits; ub += BIN_T) {
    const uint64_t u = (ub + tid) * G + wg;
    uint32_t tag = 0;
    bool act = false;
    if (u < ncid) {
      tag = g.qn_tag[u % nblk];
      act = (tag >> 12) == 1u && (tag & 0xFFFu) > (uint32_t)(u / nblk) * 64;
      nb2 += 8;
    } else if (u >= ncid + nh && u < nunits) {
      const uint64_t sc = u - ncid - nh;
      tag = g.tl_tag[sc % nblk];
      act = (tag >> 12) == 1u && (tag & 0xFFFu) > (uint32_t)(sc / nblk) * 256;
      nb2 += 8;
    } else if (u < nunits) {
      act = true;
    }
    const uint64_t ball = __ballot(act);
    if (lane == 0) s_wcnt[wv] = __popcll(ball);
    __syncthreads();
    uint32_t off = 0;
    for (int w = 0; w < wv; ++w) off += s_wcnt[w];
    if (act) {
      const uint32_t i = off + __popcll(ball & lanemask_lt());
      s_ulist[i] = (uint32_t)tid;
      s_utag[i] = tag;
    }
    if (tid == 0) {
      uint32_t n = 0;
      for (int w = 0; w < BIN_NW; ++w) n += s_wcnt[w];
      s_nact = n;
    }
    __syncthreads();
    const uint32_t nact = s_nact;
    for (uint32_t r = wv; r < nact; r += BIN_NW) unit((ub + s_ulist[r]) * G + wg, s_utag[r]);
    __syncthreads();  // s_ulist is rewritten by the next window
  }
  if (binned)
    for (uint32_t k = tid; k < NB; k += BIN_T) a.bin_cnt[(uint64_t)k * G + wg] = min(lc[k], SC);
  expand_bytes_out(g, (a.flags & LV_NOBYTES) ? 0u : nb2);
}

// BIN_SPLIT workgroups per bin, each over every BIN_SPLIT-th slice into a
// bitmap of its own; the bits become candidate bytes by byte stores (a wave
// covers 64 consecutive slots: one masked 64-B write), which the bin's other
// workgroups' stores to the same lines cannot undo.  (One workgroup per bin
// read-modify-wrote 16-B groups: 168 workgroups on a 256-CU chip, 34 us.)
constexpr uint32_t BIN_SPLIT = 2;

template <bool B16>
__global__ __launch_bounds__(BIN_T) void k_bin_apply(DevGraph g, LevelArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t bm[];  // 2^bin_shift bits, then the slice counts
  if (!a.bins || a.bin_mode_w[0] == 0) return;  // level 0 was not binned
  const uint32_t b = blockIdx.x / BIN_SPLIT, h = blockIdx.x % BIN_SPLIT, tid = threadIdx.x;
  const uint32_t span = 1u << a.bin_shift, words = span / 32;
  // a slice is SC entries: SC / 4 16-B groups of u32 targets, or SC / 8 of u16 offsets
  const uint32_t G = a.bin_grid, SC = a.bin_slice, S4 = B16 ? SC / 8 : SC / 4;
  constexpr uint32_t PER = B16 ? 8 : 4;  // entries per 16-B group
  const uint32_t NS = (G - h + BIN_SPLIT - 1) / BIN_SPLIT;  // this workgroup's slices: w = h + BIN_SPLIT k
  uint32_t *cnt = bm + words;
  for (uint32_t k = tid; k < words; k += BIN_T) bm[k] = 0;
  for (uint32_t k = tid; k < NS; k += BIN_T) cnt[k] = a.bin_cnt[(uint64_t)b * G + h + BIN_SPLIT * k];
  __syncthreads();
  uint32_t nb2 = 0;
  // its slices, four at a time per wave (their counts from LDS: the loop
  // bounds are wave-uniform), each slice's filled part in 16-B groups
  const uint4 *src = (const uint4 *)((const char *)a.bins + (uint64_t)b * G * SC * (B16 ? 2 : 4));
  const uint32_t base = b << a.bin_shift;
  for (uint32_t k0 = (uint32_t)(tid >> 6); k0 < NS; k0 += BIN_NW * 4) {
    uint32_t n[4], mx = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t k = k0 + j * BIN_NW;
      n[j] = k < NS ? cnt[k] : 0u;
      mx = max(mx, n[j]);
    }
    for (uint32_t i = (uint32_t)lane_id() * PER; i - (uint32_t)lane_id() * PER < mx; i += 64 * PER) {
      uint4 v4[4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        v4[j] = i < n[j] ? src[(uint64_t)(h + BIN_SPLIT * (k0 + j * BIN_NW)) * S4 + i / PER] : make_uint4(0, 0, 0, 0);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t v[4] = {v4[j].x, v4[j].y, v4[j].z, v4[j].w};
#pragma unroll
        for (int k = 0; k < (int)PER; ++k)
          if (i + k < n[j]) {
            const uint32_t t = B16 ? (v[k / 2] >> (16 * (k & 1))) & 0xFFFFu : v[k] - base;
            atomicOr(&bm[t >> 5], 1u << (t & 31));
            nb2 += B16 ? 4 : 8;
          }
      }
    }
  }
  __syncthreads();
  uint8_t *Fn = g.front[1];
  const uint64_t lo = (uint64_t)b << a.bin_shift;
  const uint64_t top = slot_end(g);  // (sharded graphs: bins over the proxy region too)
  const uint64_t hi = min(lo + span, top);
  // Candidate bits (LV_CBITS, unsharded; the supervisor pushes binned too): each
  // of a bin's two workgroups stores its bitmap as words of cb / cb2, which
  // k_frontier(1) ORs, instead of a byte per candidate.  Targets past a full
  // slice went out as bytes with their block's dirty byte (dirty[1]), which
  // k_frontier(1) also reads.
  static_assert(BIN_SPLIT == 2, "one candidate bitmap per k_bin_apply workgroup of a bin");
  Counters *c = g.ctr;
  if ((a.flags & LV_CBITS) && g.n_shards <= 1 && c->proxy_top == 0 &&
      (a.flags & (LV_SUPBIN | LV_INVESTIGATE))) {
    uint32_t *dst = h == 0 ? g.cb : g.cb2;
    // (bins are sized from an upper bound of slot_top: a bin past the slots
    // in use has hi < lo and stores nothing)
    const uint64_t w0 = lo >> 5, nwd = hi > lo ? (hi - lo + 31) >> 5 : 0;
    for (uint64_t k = tid; k < nwd; k += BIN_T) dst[w0 + k] = bm[k];
    nb2 += 8 * (uint32_t)((nwd + BIN_T - 1 - tid) / BIN_T);
    if (blockIdx.x == 0 && tid == 0) {
      c->cb_level = 1;
      c->cb_two = 1;
    }
    const uint32_t ws = wave_sum(nb2);
    if (lane_id() == 0 && ws) atomicAdd((unsigned long long *)&g.xbytes[blockIdx.x], (unsigned long long)(ws / 2));
    return;
  }
  for (uint64_t q = lo + tid; q < hi; q += BIN_T) {
    const uint32_t rel = (uint32_t)(q - lo);
    if ((bm[rel >> 5] >> (rel & 31)) & 1u) {
      Fn[q] = 1;
      nb2 += 2;
    }
  }
  const uint32_t ws = wave_sum(nb2);
  if (lane_id() == 0 && ws) atomicAdd((unsigned long long *)&g.xbytes[blockIdx.x], (unsigned long long)(ws / 2));
}

// ---------------------------------------------------------------------------
// k_tail: one workgroup finishes the mark once a sparse level's frontier is
// narrow (deep chains and rings, the last levels of a wide trace): rounds over
// a queue in place of level-kernel triples.  It replaces k_expand of the level
// it starts at (the frontier listed by k_frontier), and hands back to the level
// kernels when a round discovers more than tail_max shadows: the pending ones
// become candidate bytes of level L+2.
// A round is latency-bound (one chain link per round), so its state stays on
// chip: the first TAIL_LQ entries of both queues live in LDS (the rest spill to
// g.tq), and for graphs of up to TAIL_LVIS_WORDS x 32 slots so does the marked
// bitmap (claims are LDS atomics; written back before the kernel ends).  A
// shadow with at most TAIL_LIGHT out-edges is walked by its own thread, so a
// round over light shadows needs no workgroup scan.
// ---------------------------------------------------------------------------
constexpr int TAIL_THREADS = 1024;
constexpr uint32_t TAIL_LQ = 1024;
constexpr uint32_t TAIL_LIGHT = 16;
constexpr uint32_t TAIL_LVIS_WORDS = 32 * 1024;  // 128 KiB: graphs of up to 1,048,576 slots

// Exclusive scan over a workgroup of T threads (T / 64 <= 16 waves); `total` gets the sum.
template <int T>
__device__ inline uint32_t tail_scan_n(uint32_t v, uint32_t *s_w, uint32_t &total) {
  const int lane = lane_id(), w = threadIdx.x >> 6;
  const uint32_t incl = wave_incl_scan(v);
  if (lane == 63) s_w[w] = incl;
  __syncthreads();
  if (threadIdx.x < 64) {
    const uint32_t x = threadIdx.x < T / 64 ? s_w[threadIdx.x] : 0;
    const uint32_t xi = wave_incl_scan(x);
    if (threadIdx.x < T / 64) s_w[16 + threadIdx.x] = xi - x;
    if (threadIdx.x == T / 64 - 1) s_w[32] = xi;
  }
  __syncthreads();
  total = s_w[32];
  const uint32_t r = s_w[16 + w] + incl - v;
  __syncthreads();
  return r;
}

// Exclusive scan over the workgroup; `total` gets the sum.
__device__ inline uint32_t tail_scan(uint32_t v, uint32_t *s_w, uint32_t &total) {
  const int lane = lane_id(), w = threadIdx.x >> 6;
  const uint32_t incl = wave_incl_scan(v);
  if (lane == 63) s_w[w] = incl;
  __syncthreads();
  if (threadIdx.x < 64) {
    const uint32_t x = threadIdx.x < TAIL_THREADS / 64 ? s_w[threadIdx.x] : 0;
    const uint32_t xi = wave_incl_scan(x);
    if (threadIdx.x < TAIL_THREADS / 64) s_w[16 + threadIdx.x] = xi - x;
    if (threadIdx.x == TAIL_THREADS / 64 - 1) s_w[32] = xi;
  }
  __syncthreads();
  total = s_w[32];
  const uint32_t r = s_w[16 + w] + incl - v;
  __syncthreads();
  return r;
}

// A queue whose first TAIL_LQ entries are in LDS.
struct TailQ {
  uint32_t *l, *g;
  __device__ uint32_t get(uint32_t i) const { return i < TAIL_LQ ? l[i] : g[i]; }
  __device__ void put(uint32_t i, uint32_t v) const {
    if (i < TAIL_LQ) l[i] = v;
    else g[i] = v;
  }
};

struct TailLds {
  uint32_t *start, *off, *w, *next, *vis;
};

struct TailOut {
  uint32_t n_sup = 0, n_edges = 0, rounds = 0, n = 0;
  int32_t claims = 0;
  bool bailed = false;
  bool chained = false;  // handed to chain mode: the pending claims stay marked, unexpanded
};

// Claims for the next round; without queue room a claim becomes a candidate
// byte of the resume level instead (and the round ends in a bail).  Walks: a
// thread keeps the first shadow it claims while processing one and processes
// it next itself, in the same round (a chain link per step instead of per
// round); any further claim goes to the next round's queue.
// Claims of up to N targets at once (bit k of `valid`: t[k] is a target): the
// marked words of all of them are loaded together, then the atomics of those
// still unmarked are issued together, so a batch costs two round trips instead
// of two per target (a walked shadow's edges were claimed one after another:
// the C2 tail took 48 us for a 440-shadow frontier, 37 us now).  With `keep`, the first
// target claimed is kept for the thread to walk next; the rest are queued.
template <bool LV, int N>
__device__ inline void tail_claim_batch(const DevGraph &g, const TailLds &sh, const uint32_t (&t)[N],
                                        uint32_t valid, const TailQ &nxt, uint8_t *Fb, uint8_t *Db,
                                        int32_t &claims, uint32_t *keep) {
  // (atomics without the probe: the C2 tail 37 -> 40 us, profiles/r3g/ab4)
  uint32_t w[N];
#pragma unroll
  for (int k = 0; k < N; ++k)
    w[k] = ((valid >> k) & 1u) ? (LV ? sh.vis[t[k] >> 5] : g.vis[t[k] >> 5]) : ~0u;
  uint32_t go = 0;
#pragma unroll
  for (int k = 0; k < N; ++k) go |= ((w[k] >> (t[k] & 31)) & 1u) ? 0u : (1u << k);
  if (!go) return;
#pragma unroll
  for (int k = 0; k < N; ++k)
    w[k] = ((go >> k) & 1u) ? atomicOr(LV ? &sh.vis[t[k] >> 5] : &g.vis[t[k] >> 5], 1u << (t[k] & 31)) : ~0u;
#pragma unroll
  for (int k = 0; k < N; ++k) {
    if ((w[k] >> (t[k] & 31)) & 1u) continue;  // marked already, or not a target
    if (t[k] >= g.pbase) continue;  // a proxy (sharded graphs): marked, nothing to walk (k_xscan exports it)
    if (keep && *keep == NO_SLOT) {
      *keep = t[k];
      ++claims;
      continue;
    }
    const uint32_t pos = atomicAdd(sh.next, 1u);
    if (pos < TAIL_QCAP) {
      nxt.put(pos, t[k]);
      ++claims;
    } else {
      atomicAnd(LV ? &sh.vis[t[k] >> 5] : &g.vis[t[k] >> 5], ~(1u << (t[k] & 31)));
      Fb[t[k]] = 1;
      Db[t[k] >> 11] = 1;
    }
  }
}

// A kept shadow that is not walked after all (a hub): queued like a claim.
template <bool LV>
__device__ inline void tail_enqueue_claimed(const DevGraph &g, const TailLds &sh, uint32_t t, const TailQ &nxt,
                                            uint8_t *Fb, uint8_t *Db, int32_t &claims) {
  const uint32_t pos = atomicAdd(sh.next, 1u);
  if (pos < TAIL_QCAP) {
    nxt.put(pos, t);
  } else {
    atomicAnd(LV ? &sh.vis[t >> 5] : &g.vis[t >> 5], ~(1u << (t & 31)));
    Fb[t] = 1;
    Db[t >> 11] = 1;
    --claims;
  }
}

template <bool LV>
__device__ inline void tail_rounds(const DevGraph &g, const LevelArgs &a, const TailLds &sh, TailQ cur,
                                   TailQ nxt, uint32_t n, TailOut &o) {
  const int L = a.level;
  const bool investigate = a.flags & LV_INVESTIGATE;
  uint8_t *Fn = g.front[(L + 1) & 1];  // k_frontier(L)'s supervisor pushes, redone here
  uint8_t *Dn = g.dirty[(L + 1) & 1];
  uint8_t *Fb = g.front[L & 1];        // bail: candidates of level L+2
  uint8_t *Db = g.dirty[L & 1];
  bool first = true;
  __shared__ uint32_t s_deep;  // a walk ran chain_after links: hand the rest to chain mode
  __shared__ uint32_t s_bail;  // this round's hubs had more than tail_edge_max edges: they went back
  __shared__ uint32_t s_back;  // ... this many of them, as candidates of level L+2
  if (threadIdx.x == 0) s_back = 0;
  for (;;) {
    if (threadIdx.x == 0) {
      *sh.next = 0;
      s_deep = 0;
      s_bail = 0;
    }
    __syncthreads();
    for (uint32_t c0 = 0; c0 < n; c0 += TAIL_THREADS) {
      const uint32_t i = c0 + threadIdx.x;
      bool have = i < n;
      uint32_t v = have ? cur.get(i) : 0;
      bool vfirst = first;
      bool vsup = false;  // the last shadow walked had its supervisor edge counted here (n_sup)
      uint2 ad = make_uint2(0, 0);
      uint32_t steps = 0;
      while (have) {
        have = false;
        ++steps;
        // every per-shadow field in one round trip (a walk step is one chain link)
        const uint8_t f = g.flags[v];
        const uint2 adv = g.adj[v];
        const uint32_t supv = investigate ? NO_SLOT : g.sup[v];
        const bool expand = !(f & FL_HALTED);  // (:226-229)
        ad = make_uint2(0, 0);
        uint32_t keep = NO_SLOT;
        // targets: [0] the supervisor (:258-267), [1 ..] the out-edges of a
        // light shadow (:231-241), all claimed in one batch
        uint32_t tg[TAIL_LIGHT + 1];
        uint32_t valid = 0;
        tg[0] = 0;
        if (expand) {
          ad = adv;
          const uint32_t s = supv;
          vsup = false;
          if (s < 0xFFFFFFF0u) {
            if (vfirst) {
              Fn[s] = 0;
              Dn[s >> 11] = 0;
            } else {
              ++o.n_sup;
              vsup = true;
            }
            tg[0] = s;
            valid = 1;
          }
        }
        const bool light = ad.y <= TAIL_LIGHT;  // this thread walks its shadow's out-edges
#pragma unroll
        for (uint32_t u = 0; u < TAIL_LIGHT; ++u) {
          const uint64_t ed = (light && u < ad.y) ? g.pool[(uint64_t)ad.x + u] : 0;
          tg[u + 1] = edge_target(ed);
          valid |= edge_count(ed) > 0 ? (2u << u) : 0u;
        }
        tail_claim_batch<LV, TAIL_LIGHT + 1>(g, sh, tg, valid, nxt, Fb, Db, o.claims, &keep);
        if (keep != NO_SLOT) {
          if (a.chain_after && steps >= a.chain_after) {  // a long chain: queue it, chain mode takes over
            tail_enqueue_claimed<LV>(g, sh, keep, nxt, Fb, Db, o.claims);
            s_deep = 1;
          } else if (ad.y <= TAIL_LIGHT) {  // walk on
            v = keep;
            vfirst = false;
            have = true;
          } else {  // this shadow's edges go to the workgroup pass below: queue the kept one
            tail_enqueue_claimed<LV>(g, sh, keep, nxt, Fb, Db, o.claims);
          }
        }
      }
      const bool heavy = ad.y > TAIL_LIGHT;
      if (__syncthreads_or(heavy)) {  // heavy shadows: the workgroup shares their edges
        uint32_t total;
        const uint32_t st = tail_scan(heavy ? ad.y : 0u, sh.w, total);
        if (!first && a.tail_edge_max && total > a.tail_edge_max) {
          // Hubs reached by the walk (a sharded graph's hubs: mostly edges to
          // proxies, each a global claim): this one workgroup would take
          // ~1 us per 1000 edges, the level kernels spread them over the
          // chip.  The hubs go back unexpanded, as candidates of level L+2
          // (k_frontier marks them again and k_expand walks their edges), and
          // the round ends in a bail.  (They were claimed, and counted, in the
          // previous round; the first round's frontier was bounded at the
          // takeover.)
          if (heavy) {
            atomicAnd(LV ? &sh.vis[v >> 5] : &g.vis[v >> 5], ~(1u << (v & 31)));
            Fb[v] = 1;
            Db[v >> 11] = 1;
            --o.claims;
            if (vsup) --o.n_sup;  // k_frontier(L+2) follows (and counts) its supervisor edge again
            atomicAdd(&s_back, 1u);
          }
          if (threadIdx.x == 0) s_bail = 1;
          __syncthreads();
          continue;
        }
        sh.start[threadIdx.x] = st;
        sh.off[threadIdx.x] = ad.x;
        __syncthreads();
        for (uint32_t e0 = threadIdx.x; e0 < total; e0 += 4 * TAIL_THREADS) {
          uint32_t t4[4], v4 = 0;
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const uint32_t e = e0 + k * TAIL_THREADS;
            t4[k] = 0;
            if (e < total) {
              int lo = 0, hi = TAIL_THREADS - 1;  // last item whose start <= e
              while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (sh.start[mid] <= e) lo = mid;
                else hi = mid - 1;
              }
              const uint64_t ed = g.pool[(uint64_t)sh.off[lo] + (e - sh.start[lo])];
              t4[k] = edge_target(ed);
              v4 |= edge_count(ed) > 0 ? (1u << k) : 0u;
            }
          }
          tail_claim_batch<LV, 4>(g, sh, t4, v4, nxt, Fb, Db, o.claims, nullptr);
        }
        __syncthreads();
      }
    }
    __syncthreads();
    const uint32_t nn = *sh.next;
    first = false;
    ++o.rounds;
    if (nn == 0 && !s_bail) break;
    if (nn > a.tail_max || s_bail) {
      // hand the pending shadows to the level kernels as level L+2 candidates
      const uint32_t m = min(nn, (uint32_t)TAIL_QCAP);
      for (uint32_t i = threadIdx.x; i < m; i += TAIL_THREADS) {
        const uint32_t t = nxt.get(i);
        atomicAnd(LV ? &sh.vis[t >> 5] : &g.vis[t >> 5], ~(1u << (t & 31)));
        Fb[t] = 1;
        Db[t >> 11] = 1;
      }
      o.bailed = true;
      n = m + s_back;  // (the hubs handed back are candidates of level L+2 too)
      break;
    }
    if (s_deep && nn <= a.tail_max) {
      // A deep, narrow mark (chains): hand the pending claims to chain mode
      // (crgc_chain.hip), which marks whole chains by pointer jumping.  They
      // stay marked; chain mode expands them and counts their edges.
      for (uint32_t i = threadIdx.x; i < nn; i += TAIL_THREADS) {
        const uint32_t t = nxt.get(i);
        atomicOr(&g.cm[t >> 5], 1u << (t & 31));
        atomicOr(&g.pb[0][t >> 5], 1u << (t & 31));
      }
      o.chained = true;
      n = nn;
      break;
    }
    const TailQ tmp = cur;
    cur = nxt;
    nxt = tmp;
    n = nn;
    __syncthreads();
  }
  o.n = n;
}

__global__ __launch_bounds__(TAIL_THREADS) void k_tail(DevGraph g, LevelArgs a) {
  __shared__ uint32_t s_start[TAIL_THREADS + 1];
  __shared__ uint32_t s_off[TAIL_THREADS];
  __shared__ uint32_t s_w[40];
  __shared__ uint32_t s_next;
  __shared__ unsigned long long s_red[2 * (TAIL_THREADS / 64)];
  __shared__ uint32_t s_q[2][TAIL_LQ];
  __shared__ uint32_t s_vis[TAIL_LVIS_WORDS];
  Counters *c = g.ctr;
  const int L = a.level;
  // Level count = sum of k_frontier's per-workgroup frontier counts, and its
  // frontier's out-edges (Beamer's m_f) for k_expand's direction: both loaded
  // in one round trip (before the state check, which they do not depend on)
  // and summed with wave shuffles.
  unsigned long long pf = 0, pm = 0;
  for (uint32_t b = threadIdx.x; b < a.frontier_grid; b += TAIL_THREADS) {
    pf += g.blkstat[b * 4 + STAT_FRONT];
    pm += g.blkstat[b * 4 + STAT_MF];
  }
  if (c->tail_state) return;
  for (int d = 32; d > 0; d >>= 1) {
    pf += __shfl_xor(pf, d);
    pm += __shfl_xor(pm, d);
  }
  if (lane_id() == 0) {
    s_red[threadIdx.x >> 6] = pf;
    s_red[16 + (threadIdx.x >> 6)] = pm;
  }
  __syncthreads();
  uint64_t n0 = 0, mf = 0;
  for (int k = 0; k < TAIL_THREADS / 64; ++k) {
    n0 += s_red[k];
    mf += s_red[16 + k];
  }
  if (!listing_level(c, L, a) || n0 == 0 || n0 > a.tail_start || (a.tail_edge_max && mf > a.tail_edge_max)) {
    if (threadIdx.x == 0) {  // the level kernels go on
      c->mf_level = mf;
      c->mf_sum += mf;
      c->ring[L % LEVEL_RING] = n0;
      c->marked += n0;
      c->qh[(L + 1) & 1] = 0;  // next level's hub queue (last read by k_expand(L-1))
      if (n0 == 0) c->mark_done = 1;
    }
    return;
  }
  // Take over: gather the listed frontier from the per-block regions.
  TailQ cur{s_q[0], g.tq}, nxt{s_q[1], g.tq + TAIL_QCAP};
  const uint64_t top = c->slot_top;
  {
    const uint32_t nblk = (uint32_t)((top + BLK_SLOTS - 1) / BLK_SLOTS);
    const uint32_t want = (uint32_t)(L + 1);
    // 8 tags per thread in flight, one workgroup scan per 8 x 1024 blocks
    // (one per 1024 blocks was a chain of dependent loads: 5 at C2 scale)
    constexpr int TG = 8;
    uint32_t base = 0;
    for (uint32_t b0 = 0; b0 < nblk; b0 += TG * TAIL_THREADS) {
      uint32_t cnt[TG], sum = 0;
#pragma unroll
      for (int k = 0; k < TG; ++k) {
        const uint32_t b = b0 + k * TAIL_THREADS + threadIdx.x;
        const uint32_t t = b < nblk ? g.tl_tag[b] : 0;
        cnt[k] = (t >> 12) == want ? (t & 0xFFFu) : 0u;
        sum += cnt[k];
      }
      uint32_t tot;
      uint32_t off = base + tail_scan(sum, s_w, tot);
#pragma unroll
      for (int k = 0; k < TG; ++k) {
        const uint32_t b = b0 + k * TAIL_THREADS + threadIdx.x;
        for (uint32_t i = 0; i < cnt[k]; ++i)
          if (off + i < TAIL_QCAP) cur.put(off + i, g.tl_buf[(uint64_t)b * BLK_SLOTS + i]);
        off += cnt[k];
      }
      base += tot;
    }
  }
  // (the LDS copy must cover every slot a walk can claim: proxies too)
  const uint64_t vend = slot_end(g);
  const bool lv = vend <= (uint64_t)TAIL_LVIS_WORDS * 32;
  const uint32_t nw = (uint32_t)((vend + 31) / 32);
  if (lv)
    for (uint32_t k = threadIdx.x; k < nw; k += TAIL_THREADS) s_vis[k] = g.vis[k];
  __syncthreads();
  const TailLds sh{s_start, s_off, s_w, &s_next, s_vis};
  TailOut o;
  if (lv) tail_rounds<true>(g, a, sh, cur, nxt, (uint32_t)n0, o);
  else tail_rounds<false>(g, a, sh, cur, nxt, (uint32_t)n0, o);
  __syncthreads();
  if (lv)
    for (uint32_t k = threadIdx.x; k < nw; k += TAIL_THREADS) g.vis[k] = s_vis[k];
  // statistics: claims became marked shadows (k_frontier(L) counted level L)
  uint32_t tot_claims, tot_sup;
  tail_scan((uint32_t)o.claims, s_w, tot_claims);
  tail_scan(o.n_sup, s_w, tot_sup);
  if (threadIdx.x == 0) {
    const uint64_t marked_new = (uint64_t)tot_claims - (o.bailed ? o.n : 0);  // queued claims undone
    c->ring[L % LEVEL_RING] = n0;
    c->marked += n0 + marked_new;
    g.blkstat[STAT_SUP] += tot_sup;
    c->tail_from = L;
    if (o.chained) {
      c->tail_level = L + o.rounds;
      c->tail_state = TAIL_CHAINS;  // the host runs chain mode, which finishes the mark
    } else if (o.bailed) {
      c->ring[L % LEVEL_RING] = 1;  // level L+2 runs sparse over the dirty blocks
      c->ring[(L + 1) % LEVEL_RING] = o.n;
      c->qh[L & 1] = 0;
      c->tail_level = L + 2;
      c->tail_state = TAIL_BAILED;
    } else {
      c->tail_level = L + o.rounds;  // levels 0 .. L+rounds-1 were non-empty
      c->tail_state = TAIL_DONE;
      c->mark_done = 1;
    }
  }
}

// ---------------------------------------------------------------------------
// k_walk: WALK_WG workgroups finish a sharded mark round's narrow levels in
// one launch (the multi-workgroup form of k_tail's takeover).  One workgroup
// walking a shard's narrow levels ran ~1 G edges/s, and every level the level
// kernels run costs three dependent launches (~25 us with nothing to do:
// ~30 such levels per shard and C4 wakeup over 8 logical shards,
// profiles/r5o).  Here each level is a pass over a global queue by all
// workgroups (a chunk of WALK_T shadows per workgroup and step; light shadows
// by their own thread, heavy ones' edges shared by the workgroup), claims by
// atomicOr on the marked bitmap, new shadows appended to the next queue
// (wave-aggregated), then a grid barrier.  It takes over where k_tail would
// (the listed frontier of a narrow level), hands back to the level kernels as
// k_tail does when a level finds more than tail_max shadows, and writes the
// same controller state.  Every workgroup computes the takeover decision from
// the same per-workgroup statistics, so all take the same path; WALK_WG is
// far below one workgroup per CU, and every barrier wait is bounded (a
// workgroup that never arrives — not resident — fails the mark with
// ERR_WALK_STUCK instead of hanging the grid).
// ---------------------------------------------------------------------------
constexpr int WALK_WG = 64;
constexpr int WALK_T = 256;
constexpr uint32_t WALK_LIGHT = 16;
constexpr uint32_t WALK_PIECE = 256;  // edges of a heavy shadow's piece

// A load that reads the device-coherent value (past this CU's L1): what
// other workgroups of the launch wrote before the last barrier.
template <class T>
__device__ inline T ld_agent(const T *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Grid barrier over the launch's workgroups: arrival counter, generation word.
// Returns false when the wait ran out (every workgroup then leaves the walk).
__device__ inline bool walk_sync(Counters *c, uint32_t nwg, uint32_t &gen) {
  __shared__ uint32_t s_ok;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t ok = 1;
    __threadfence();  // this workgroup's queue appends and claims, before the arrival
    if (atomicAdd(&c->walk_bar, 1u) == nwg - 1) {
      atomicExch(&c->walk_bar, 0u);
      __threadfence();
      atomicAdd(&c->walk_gen, 1u);
    } else {
      uint64_t k = 0;
      while (__hip_atomic_load(&c->walk_gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gen) {
        if (++k > (1ull << 24) || __hip_atomic_load(&c->walk_fail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
          ok = 0;
          atomicExch(&c->walk_fail, 1u);
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
    }
    __threadfence();  // the other workgroups' writes, after the wait
    ++gen;
    s_ok = ok;
  }
  __syncthreads();
  return s_ok != 0;
}

__global__ __launch_bounds__(WALK_T) void k_walk(DevGraph g, LevelArgs a) {
  __shared__ unsigned long long s_red[2 * (WALK_T / 64)];
  __shared__ uint32_t s_start[WALK_T + 1], s_off[WALK_T], s_w[40];
  Counters *c = g.ctr;
  const int L = a.level;
  const uint32_t tid = threadIdx.x, lane = lane_id(), wg = blockIdx.x, nwg = gridDim.x;
  // the level count and its frontier's out-edges, as k_tail sums them
  unsigned long long pf = 0, pm = 0;
  for (uint32_t b = tid; b < a.frontier_grid; b += WALK_T) {
    pf += g.blkstat[b * 4 + STAT_FRONT];
    pm += g.blkstat[b * 4 + STAT_MF];
  }
  if (c->tail_state) return;
  for (int d = 32; d > 0; d >>= 1) {
    pf += __shfl_xor(pf, d);
    pm += __shfl_xor(pm, d);
  }
  if (lane == 0) {
    s_red[tid >> 6] = pf;
    s_red[WALK_T / 64 + (tid >> 6)] = pm;
  }
  __syncthreads();
  uint64_t n0 = 0, mf = 0;
  for (int k = 0; k < WALK_T / 64; ++k) {
    n0 += s_red[k];
    mf += s_red[WALK_T / 64 + k];
  }
  if (!listing_level(c, L, a) || n0 == 0 || n0 > a.tail_start) {
    if (wg == 0 && tid == 0) {  // the level kernels go on
      c->mf_level = mf;
      c->mf_sum += mf;
      c->ring[L % LEVEL_RING] = n0;
      c->marked += n0;
      c->qh[(L + 1) & 1] = 0;
      if (n0 == 0) c->mark_done = 1;
    }
    return;
  }
  uint32_t gen = __hip_atomic_load(&c->walk_gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  uint32_t *qb[2] = {g.tq, g.tq + TAIL_QCAP};
  uint8_t *Fn = g.front[(L + 1) & 1];  // k_frontier(L)'s supervisor pushes, redone here
  uint8_t *Dn = g.dirty[(L + 1) & 1];
  uint8_t *Fb = g.front[L & 1];        // bail: candidates of level L+2
  uint8_t *Db = g.dirty[L & 1];
  const bool investigate = a.flags & LV_INVESTIGATE;
  // Take over: the listed frontier of level L into queue 0 (walk_n[0]); the
  // other two counts zeroed for the first levels
  {
    if (wg == 0 && tid == 0) c->walk_n[1] = c->walk_n[2] = c->walk_np[0] = c->walk_np[1] = 0;
    const uint64_t nblk = (c->slot_top + BLK_SLOTS - 1) / BLK_SLOTS;
    const uint32_t want = (uint32_t)(L + 1);
    for (uint64_t b = (uint64_t)wg * WALK_T + tid; b - tid < nblk; b += (uint64_t)nwg * WALK_T) {
      const uint32_t t = b < nblk ? g.tl_tag[b] : 0u;
      const uint32_t cnt = (t >> 12) == want ? (t & 0xFFFu) : 0u;
      const uint32_t incl = wave_incl_scan(cnt), tot = __shfl(incl, 63);
      unsigned long long at = 0;
      if (lane == 63 && tot) at = atomicAdd(&c->walk_n[0], (unsigned long long)tot);
      at = __shfl(at, 63) + incl - cnt;
      for (uint32_t i = 0; i < cnt; ++i)
        if (at + i < TAIL_QCAP) qb[0][at + i] = g.tl_buf[b * BLK_SLOTS + i];
    }
  }
  bool ok = walk_sync(c, nwg, gen);
  uint32_t claims = 0, n_sup = 0;
  uint32_t r = 0;  // walk levels done
  bool bailed = false;
  uint64_t n_bail = 0;
  for (; ok; ++r) {
    const uint64_t n = min(ld_agent(&c->walk_n[r % 3]), (unsigned long long)TAIL_QCAP);
    const uint32_t *cur = qb[r & 1];
    uint32_t *nxt = qb[(r + 1) & 1];
    unsigned long long *nn_ctr = &c->walk_n[(r + 1) % 3];
    if (wg == 0 && tid == 0) {
      c->walk_n[(r + 2) % 3] = 0;    // read at level r - 1, appended at r + 1
      c->walk_np[(r + 1) & 1] = 0;   // read at level r - 1, appended at r + 1
    }
    // chunks of WALK_T shadows, dealt to the workgroups
    for (uint64_t c0 = (uint64_t)wg * WALK_T; c0 < n; c0 += (uint64_t)nwg * WALK_T) {
      const uint64_t i = c0 + tid;
      const bool have = i < n;
      const uint32_t v = have ? ld_agent(&cur[i]) : 0u;
      uint8_t f = 0;
      uint2 ad = make_uint2(0, 0);
      uint32_t supv = NO_SLOT;
      if (have) {
        f = g.flags[v];
        ad = g.adj[v];
        supv = investigate ? NO_SLOT : g.sup[v];
      }
      const bool expand = have && !(f & FL_HALTED);  // (:226-229)
      if (!expand) ad = make_uint2(0, 0);
      // targets: the supervisor (:258-267), the out-edges of a light shadow (:231-241)
      uint32_t tg[WALK_LIGHT + 1];
      uint32_t valid = 0;
      tg[0] = 0;
      if (expand && supv < 0xFFFFFFF0u) {
        if (r == 0) {  // level L's supervisor pushes were made by k_frontier: undo them
          Fn[supv] = 0;
          Dn[supv >> 11] = 0;
        } else {
          ++n_sup;
        }
        tg[0] = supv;
        valid = 1;
      }
      const bool light = ad.y <= WALK_LIGHT;
#pragma unroll
      for (uint32_t u = 0; u < WALK_LIGHT; ++u) {
        const uint64_t ed = (light && u < ad.y) ? g.pool[(uint64_t)ad.x + u] : 0;
        tg[u + 1] = edge_target(ed);
        valid |= edge_count(ed) > 0 ? (2u << u) : 0u;
      }
      // claims: marked words together, then the atomics of the still unmarked
      uint32_t w[WALK_LIGHT + 1];
#pragma unroll
      for (uint32_t k = 0; k <= WALK_LIGHT; ++k) w[k] = ((valid >> k) & 1u) ? g.vis[tg[k] >> 5] : ~0u;
      uint32_t go = 0;
#pragma unroll
      for (uint32_t k = 0; k <= WALK_LIGHT; ++k) go |= ((w[k] >> (tg[k] & 31)) & 1u) ? 0u : (1u << k);
      uint32_t mine = 0;  // claimed shadows (not proxies) of this thread, by target index
#pragma unroll
      for (uint32_t k = 0; k <= WALK_LIGHT; ++k)
        if ((go >> k) & 1u) {
          const uint32_t old = atomicOr(&g.vis[tg[k] >> 5], 1u << (tg[k] & 31));
          if (!((old >> (tg[k] & 31)) & 1u) && tg[k] < g.pbase) mine |= 1u << k;
        }
      // append this thread's claims to the next queue (one atomic per wave)
      {
        const uint32_t cnt = __popc(mine);
        const uint32_t incl = wave_incl_scan(cnt), tot = __shfl(incl, 63);
        unsigned long long at = 0;
        if (lane == 63 && tot) at = atomicAdd(nn_ctr, (unsigned long long)tot);
        at = __shfl(at, 63) + incl - cnt;
        for (uint32_t m = mine; m; m &= m - 1) {
          const uint32_t k = __ffs(m) - 1;
          if (at < TAIL_QCAP) {
            nxt[at] = tg[k];
            ++claims;
          } else {  // no queue room: a candidate of the resume level instead (the level bails)
            atomicAnd(&g.vis[tg[k] >> 5], ~(1u << (tg[k] & 31)));
            Fb[tg[k]] = 1;
            Db[tg[k] >> 11] = 1;
          }
          ++at;
        }
      }
      // heavy shadows: their edges as pieces of <= WALK_PIECE for every
      // workgroup after the barrier (a hub walked by its own workgroup kept the
      // others waiting at the barrier, profiles/r5r)
      const uint32_t np = (expand && ad.y > WALK_LIGHT) ? (ad.y + WALK_PIECE - 1) / WALK_PIECE : 0u;
      {
        const uint32_t incl = wave_incl_scan(np), tot = __shfl(incl, 63);
        unsigned long long at = 0;
        if (lane == 63 && tot) at = atomicAdd(&c->walk_np[r & 1], (unsigned long long)tot);
        at = __shfl(at, 63) + incl - np;
        for (uint32_t k = 0; k < np; ++k, ++at)
          if (at < g.wpc_cap)  // (always: a level has <= TAIL_QCAP shadows, pcap edges)
            g.wpc[at] = make_uint2(ad.x + k * WALK_PIECE, min(WALK_PIECE, ad.y - k * WALK_PIECE));
      }
    }
    ok = walk_sync(c, nwg, gen);
    if (!ok) break;
    {
      // the pieces, one per wave at a time (4 edges per lane in flight)
      const uint64_t npc = min(ld_agent(&c->walk_np[r & 1]), (unsigned long long)g.wpc_cap);
      const uint64_t gwv = (uint64_t)wg * (WALK_T / 64) + (tid >> 6), nwv = (uint64_t)nwg * (WALK_T / 64);
      for (uint64_t pi = gwv; pi < npc; pi += nwv) {
        const unsigned long long raw = ld_agent(reinterpret_cast<const unsigned long long *>(g.wpc + pi));
        const uint2 pc = make_uint2((uint32_t)raw, (uint32_t)(raw >> 32));
        for (uint32_t e0 = 0; e0 < pc.y; e0 += 256) {
          uint32_t t[4];
          bool go[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const uint32_t e = e0 + u * 64 + lane;
            const uint64_t ed = e < pc.y ? g.pool[(uint64_t)pc.x + e] : 0ull;
            t[u] = edge_target(ed);
            go[u] = edge_count(ed) > 0;
          }
          uint32_t w4[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) w4[u] = go[u] ? g.vis[t[u] >> 5] : ~0u;
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            bool got = false;
            if (go[u] && !((w4[u] >> (t[u] & 31)) & 1u)) {
              const uint32_t old = atomicOr(&g.vis[t[u] >> 5], 1u << (t[u] & 31));
              got = !((old >> (t[u] & 31)) & 1u) && t[u] < g.pbase;
            }
            const uint64_t bal = __ballot(got);
            unsigned long long at = 0;
            if (lane == 0 && bal) at = atomicAdd(nn_ctr, (unsigned long long)__popcll(bal));
            at = __shfl(at, 0) + __popcll(bal & lanemask_lt());
            if (got) {
              if (at < TAIL_QCAP) {
                nxt[at] = t[u];
                ++claims;
              } else {
                atomicAnd(&g.vis[t[u] >> 5], ~(1u << (t[u] & 31)));
                Fb[t[u]] = 1;
                Db[t[u] >> 11] = 1;
              }
            }
          }
        }
      }
    }
    ok = walk_sync(c, nwg, gen);
    if (!ok) break;
    const uint64_t nn = ld_agent(&c->walk_n[(r + 1) % 3]);
    if (nn == 0) {
      ++r;
      break;
    }
    if (nn > a.tail_max || nn > (uint64_t)TAIL_QCAP) {
      // hand the pending shadows to the level kernels as level L+2 candidates
      const uint64_t m = min(nn, (uint64_t)TAIL_QCAP);
      for (uint64_t i = (uint64_t)wg * WALK_T + tid; i < m; i += (uint64_t)nwg * WALK_T) {
        const uint32_t t = ld_agent(&nxt[i]);
        atomicAnd(&g.vis[t >> 5], ~(1u << (t & 31)));
        Fb[t] = 1;
        Db[t >> 11] = 1;
      }
      bailed = true;
      n_bail = m;
      ++r;
      break;
    }
  }
  // totals, then the controller state (workgroup 0 after a last barrier)
  {
    uint32_t tc, ts;
    const uint32_t x0 = tail_scan_n<WALK_T>(claims, s_w, tc);
    const uint32_t x1 = tail_scan_n<WALK_T>(n_sup, s_w, ts);
    (void)x0;
    (void)x1;
    if (tid == 0) {
      if (tc) atomicAdd(&c->walk_claims, (unsigned long long)tc);
      if (ts) atomicAdd(&c->walk_sup, (unsigned long long)ts);
    }
  }
  const bool fin = walk_sync(c, nwg, gen) && ok;
  if (wg != 0 || tid != 0) return;
  if (!fin) {
    set_err(c, ERR_WALK_STUCK);
    c->tail_state = TAIL_DONE;  // the host reads the error word and fails the trace
    c->mark_done = 1;
    return;
  }
  const uint64_t claimed = ld_agent(&c->walk_claims), sup = ld_agent(&c->walk_sup);
  c->walk_claims = c->walk_sup = 0;
  c->ring[L % LEVEL_RING] = n0;
  c->marked += n0 + claimed - (bailed ? n_bail : 0);  // queued claims undone by a bail
  g.blkstat[STAT_SUP] += sup;
  c->tail_from = L;
  if (bailed) {
    c->ring[L % LEVEL_RING] = 1;  // level L+2 runs sparse over the dirty blocks
    c->ring[(L + 1) % LEVEL_RING] = n_bail;
    c->qh[L & 1] = 0;
    c->tail_level = L + 2;
    c->tail_state = TAIL_BAILED;
  } else {
    c->tail_level = L + r;  // levels 0 .. L+r-1 were non-empty
    c->tail_state = TAIL_DONE;
    c->mark_done = 1;
  }
}

// Whether k_walk's WALK_WG workgroups can all be resident on `device` (its
// grid barriers assume so).  Occupancy alone cannot promise it while other
// streams keep CUs busy: CRGC_WALK stays a test hook, off by default.
bool walk_fits(int device) {
  int per_cu = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_walk, WALK_T, 0) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return (int64_t)per_cu * cus >= WALK_WG;
}

int level_grid(uint64_t slot_top) {
  const uint64_t blocks = (slot_top + BLK_SLOTS - 1) / BLK_SLOTS;  // wave-blocks
  uint64_t wg = (blocks + 3) / 4;
  if (wg < 1) wg = 1;
  if (wg > STAT_WG) wg = STAT_WG;
  return (int)wg;
}

hipError_t launch_level(const DevGraph &g, const LevelArgs &a0, bool roots, bool investigate,
                        uint64_t slot_top, hipStream_t s, hipEvent_t *ev) {
  launch_begin();
  LevelArgs a = a0;
  const int grid = level_grid(slot_top);
  a.frontier_grid = grid;
  if (investigate) a.flags |= LV_INVESTIGATE;
  if (roots) a.flags |= LV_ROOTS;
  // Timed launches carry their start / stop events in the dispatch itself
  // (hipExtLaunchKernelGGL): no separate event packets between the kernels.
  hipEvent_t e[6] = {};
  if (ev)
    for (int k = 0; k < 6; ++k) e[k] = ev[k];
  auto frontier = [&](auto kern) {
    hipExtLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, s, e[0], e[1], 0, g, a);
  };
  if (roots && investigate) frontier(k_frontier<true, true>);
  else if (roots) frontier(k_frontier<true, false>);
  else if (investigate) frontier(k_frontier<false, true>);
  else frontier(k_frontier<false, false>);
  // level controller: the level count, and the narrow-frontier takeover
  if (a.flags & LV_WALK) {
    // (k_walk's grid barriers assume its WALK_WG workgroups are resident at
    // once: the host enables it only when occupancy allows, walk_fits(); a
    // workgroup that still never arrives fails the mark with ERR_WALK_STUCK.
    // A cooperative launch would guarantee residency, but a process that had
    // made one crashed in the runtime's exit handlers in a round-6 test run)
    hipExtLaunchKernelGGL(k_walk, dim3(WALK_WG), dim3(WALK_T), 0, s, e[2], e[3], 0, g, a);
  } else
    hipExtLaunchKernelGGL(k_tail, dim3(1), dim3(TAIL_THREADS), 0, s, e[2], e[3], 0, g, a);
  // 8 WGs of 4 waves per CU
  if (roots && a.nbins) {
    // the pseudo-root level, binned when it is wide: place and apply, timed
    // together as its expand
    const size_t lds = (size_t)(1u << a.bin_shift) / 8 + (size_t)a.bin_grid * 4;
    if (a.bin_shift == 16) {
      hipExtLaunchKernelGGL(k_bin_place<true>, dim3(a.bin_grid), dim3(BIN_T), 0, s, e[4], nullptr, 0, g, a);
      hipExtLaunchKernelGGL(k_bin_apply<true>, dim3(a.nbins * BIN_SPLIT), dim3(BIN_T), lds, s, nullptr, e[5], 0, g, a);
    } else {
      hipExtLaunchKernelGGL(k_bin_place<false>, dim3(a.bin_grid), dim3(BIN_T), 0, s, e[4], nullptr, 0, g, a);
      hipExtLaunchKernelGGL(k_bin_apply<false>, dim3(a.nbins * BIN_SPLIT), dim3(BIN_T), lds, s, nullptr, e[5], 0, g, a);
    }
    return hipGetLastError();
  }
  auto expand = [&](auto kern) {
    hipExtLaunchKernelGGL(kern, dim3(STAT_WG), dim3(256), 0, s, e[4], e[5], 0, g, a);
  };
  expand(k_expand);
  return hipGetLastError();
}

// Per-trace reset in one launch: the marked bitmap, the per-block level tags
// and proxy listings of the blocks this trace can touch, the per-workgroup
// statistics, and the trace counters (marked .. the end of the level ring).
// nh blocks from slot 0 and np blocks from the proxy region (pbase).
__global__ __launch_bounds__(256) void k_trace_reset(DevGraph g, uint64_t nh, uint64_t np, uint32_t ctr_from,
                                                     uint32_t ctr_words) {
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  const uint64_t t0 = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  const uint64_t nblk = nh + np, p0 = g.pbase / BLK_SLOTS;
  auto at = [&](uint64_t vb) { return vb < nh ? vb : p0 + (vb - nh); };
  uint4 *vis4 = reinterpret_cast<uint4 *>(g.vis);  // 2048 slots = 64 words = 16 uint4 per block
  uint4 *sent4 = reinterpret_cast<uint4 *>(g.xsent);
  for (uint64_t i = t0; i < nblk * 16; i += stride) {
    vis4[at(i / 16) * 16 + i % 16] = make_uint4(0, 0, 0, 0);
    if (sent4 && i >= nh * 16) sent4[at(i / 16) * 16 + i % 16] = make_uint4(0, 0, 0, 0);
  }
  for (uint64_t vb = t0; vb < nblk; vb += stride) {
    const uint64_t i = at(vb);
    g.qn_tag[i] = 0;
    g.tl_tag[i] = 0;
  }
  for (uint64_t i = t0; i < (uint64_t)STAT_WG * 4; i += stride) g.blkstat[i] = 0;
  for (uint64_t i = t0; i < (uint64_t)STAT_WG; i += stride) g.xbytes[i] = 0;
  unsigned long long *cw = reinterpret_cast<unsigned long long *>(g.ctr) + ctr_from;
  for (uint64_t i = t0; i < ctr_words; i += stride) cw[i] = 0;
}

hipError_t launch_trace_reset(const DevGraph &g, uint64_t nh, uint64_t np, uint32_t ctr_from, uint32_t ctr_words,
                              hipStream_t s) {
  launch_begin();
  hipLaunchKernelGGL(k_trace_reset, dim3(grid_for(std::max<uint64_t>((nh + np) * 16, ctr_words), 256, 2048)),
                     dim3(256), 0, s, g, nh, np, ctr_from, ctr_words);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Sweep (:270-284): unmarked shadows are garbage; a local one is told StopMsg
// when its supervisor is marked and it is not halted.  A local garbage shadow
// without a supervisor is the reference's NullPointerException: counted, and
// the gather pass then leaves the graph untouched.
//   k_sweep   one wave per 2048-slot block: garbage / kill slots into the
//             block's own region of out_a / out_b, counts per block
//   k_sweep_scan   one workgroup: exclusive offsets of the per-block counts
//   k_sweep_gather one wave per block: slots -> ids, packed densely; unless an
//             NPE was seen, removes the garbage from shadowMap (:276)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_sweep(DevGraph g, int should_kill) {
  Counters *c = g.ctr;
  if (!c->mark_done) return;
  const uint64_t slot_top = c->slot_top;
  const uint32_t nblk = (uint32_t)((slot_top + BLK_SLOTS - 1) / BLK_SLOTS);
  const int lane = lane_id();
  const uint32_t gw = blockIdx.x * 4 + (threadIdx.x >> 6);
  const uint32_t nw = gridDim.x * 4;
  uint32_t n_live = 0, n_npe = 0, n_req = 0;
  uint64_t n_edges = 0;
  for (uint32_t blk = gw; blk < nblk; blk += nw) {
    const uint64_t base = (uint64_t)blk * BLK_SLOTS + (uint64_t)lane * 32;
    const uint32_t word = g.vis[(uint64_t)blk * 64 + lane];
    const uint4 f4[2] = {*(const uint4 *)(g.flags + base), *(const uint4 *)(g.flags + base + 16)};
    const uint32_t fa = flag_bits(f4, FL_ALIVE), fp = flag_bits(f4, FL_PROXY);
    const uint32_t alive = fa & ~fp;  // (proxies live in their own region: none here)
    const uint32_t halted = flag_bits(f4, FL_HALTED), local = flag_bits(f4, FL_LOCAL);
    uint32_t kill = 0, req = 0;
    // traced edges (:231): the nonzero out-counts of the marked, unhalted shadows
    // Coalesced: load q of lane l holds slots q*256 + 4l .. +3, whose bits come
    // from lane q*8 + l/8 by one shuffle (a 128-B run per lane touched 64 lines
    // per load instruction).
    const uint32_t ex = alive & word & ~halted;
    if (__ballot(ex != 0)) {
      const uint4 *zp = (const uint4 *)(g.nzdeg + (uint64_t)blk * BLK_SLOTS);
      uint32_t b4[8];
      uint4 z[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        b4[q] = (__shfl(ex, q * 8 + (lane >> 3)) >> ((lane & 7) * 4)) & 0xFu;
        z[q] = b4[q] ? zp[q * 64 + lane] : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int q = 0; q < 8; ++q)
        n_edges += (uint64_t)((b4[q] & 1u) ? z[q].x : 0u) + ((b4[q] & 2u) ? z[q].y : 0u) +
                   (uint64_t)((b4[q] & 4u) ? z[q].z : 0u) + ((b4[q] & 8u) ? z[q].w : 0u);
    }
    const uint32_t garbage = alive & ~word;
    n_live += __popc(alive & word);
    uint32_t gm = garbage;
    while (gm) {
      const int j = __ffs(gm) - 1;
      gm &= gm - 1;
      // (bit masks, not fb[j]: a runtime index into the flag registers cost
      // this kernel ~20 VGPRs, and occupancy)
      if ((local >> j) & 1u) {
        const uint32_t s = g.sup[base + j];
        if (s == SLOT_NONE) {
          n_npe++;
        } else if (should_kill && !((halted >> j) & 1u) && s < 0xFFFFFFF0u) {
          if ((g.vis[s >> 5] >> (s & 31)) & 1u) {
            kill |= 1u << j;
          } else if ((g.flags[s] & (FL_ALIVE | FL_PROXY)) == (FL_ALIVE | FL_PROXY)) {
            // an unmarked proxy says nothing: its home shard knows the mark
            req |= 1u << j;
          }
        }
      }
    }
    if (g.n_shards > 1) {
      const uint32_t rc = __popc(req), ri = wave_incl_scan(rc);
      uint32_t rp = ri - rc;
      uint32_t *ra = g.rq_buf + (uint64_t)blk * BLK_SLOTS;
      while (req) {
        const int j = __ffs(req) - 1;
        req &= req - 1;
        ra[rp++] = (uint32_t)(base + j);
      }
      if (lane == 63) g.rq_cnt[blk] = ri;
      n_req += rc;
    }
    const uint32_t gc = __popc(garbage), kc = __popc(kill);
    const uint32_t gi = wave_incl_scan(gc), ki = wave_incl_scan(kc);
    uint32_t gp = gi - gc, kp = ki - kc;
    uint32_t *ga = (uint32_t *)g.out_a + (uint64_t)blk * BLK_SLOTS;
    uint32_t *ka = (uint32_t *)g.out_b + (uint64_t)blk * BLK_SLOTS;
    gm = garbage;
    while (gm) {
      const int j = __ffs(gm) - 1;
      gm &= gm - 1;
      ga[gp++] = (uint32_t)(base + j);
    }
    uint32_t km = kill;
    while (km) {
      const int j = __ffs(km) - 1;
      km &= km - 1;
      ka[kp++] = (uint32_t)(base + j);
    }
    if (lane == 63) {
      g.sweep_cnt[2 * (uint64_t)blk] = gi;
      g.sweep_cnt[2 * (uint64_t)blk + 1] = ki;
    }
  }
  const uint64_t tl = block_sum4(n_live);
  const uint64_t tn = block_sum4(n_npe);
  const uint64_t tr = block_sum4(n_req);
  const uint64_t te = block_sum64(n_edges);
  if (threadIdx.x == 0) {
    g.blkstat[(uint64_t)blockIdx.x * 4 + STAT_LIVE] = tl;
    g.blkstat[(uint64_t)blockIdx.x * 4 + STAT_EDGES] = te;  // the only writer of this partial
    if (tn) atomicAdd(&c->npe, (unsigned long long)tn);
    if (tr) atomicAdd(&c->n_req, (unsigned long long)tr);
  }
}

// One workgroup: exclusive offsets over the per-block (garbage, kill) counts,
// totals into the counters, and the live count from the sweep partials.
// Each thread owns a contiguous run of blocks, so the counts are loaded in one
// pass and placed by one workgroup scan (latency-bound: one round trip, not
// one per 1024 blocks).  Slots are u32, so every count fits 32 bits.  It also
// sums the trace's per-workgroup sup / traced-edge / expand-byte partials into
// the counters (the sweep wrote the edge partials).
__global__ __launch_bounds__(1024) void k_sweep_scan(DevGraph g, uint32_t sweep_grid) {
  __shared__ uint64_t wsum[3][16];
  __shared__ uint64_t wst[3][16];
  Counters *c = g.ctr;
  uint64_t su = 0, ed = 0, xb = 0;
  for (uint32_t b = threadIdx.x; b < STAT_WG; b += 1024) {
    su += g.blkstat[b * 4 + STAT_SUP];
    ed += g.blkstat[b * 4 + STAT_EDGES];
    xb += g.xbytes[b];
  }
  if (!c->mark_done) return;  // enqueued behind a level chunk that did not finish the mark
  for (int d = 32; d > 0; d >>= 1) {
    su += __shfl_xor(su, d);
    ed += __shfl_xor(ed, d);
    xb += __shfl_xor(xb, d);
  }
  const uint64_t nblk = (c->slot_top + BLK_SLOTS - 1) / BLK_SLOTS;
  const int lane = lane_id(), wv = threadIdx.x >> 6;
  const uint64_t per = (nblk + 1023) / 1024;
  const uint64_t b_lo = min(nblk, (uint64_t)threadIdx.x * per), b_hi = min(nblk, b_lo + per);
  uint32_t live = 0, gs = 0, ks = 0;
  for (uint32_t b = threadIdx.x; b < sweep_grid; b += 1024) live += (uint32_t)g.blkstat[b * 4 + STAT_LIVE];
#pragma unroll 4
  for (uint64_t b = b_lo; b < b_hi; ++b) {
    const uint2 gk = *(const uint2 *)(g.sweep_cnt + 2 * b);
    gs += gk.x;
    ks += gk.y;
  }
  const uint32_t gi = wave_incl_scan(gs), ki = wave_incl_scan(ks), li = wave_incl_scan(live);
  if (lane == 63) {
    wsum[0][wv] = gi;
    wsum[1][wv] = ki;
    wsum[2][wv] = li;
    wst[0][wv] = su;
    wst[1][wv] = ed;
    wst[2][wv] = xb;
  }
  __syncthreads();
  uint64_t go = 0, ko = 0, gtot = 0, ktot = 0, ltot = 0;
  for (int w = 0; w < 16; ++w) {
    if (w < wv) {
      go += wsum[0][w];
      ko += wsum[1][w];
    }
    gtot += wsum[0][w];
    ktot += wsum[1][w];
    ltot += wsum[2][w];
  }
  go += gi - gs;
  ko += ki - ks;
#pragma unroll 4
  for (uint64_t b = b_lo; b < b_hi; ++b) {
    const uint2 gk = *(const uint2 *)(g.sweep_cnt + 2 * b);
    *(ulonglong2 *)(g.sweep_off + 2 * b) = make_ulonglong2(go, ko);
    go += gk.x;
    ko += gk.y;
  }
  if (threadIdx.x == 0) {
    c->n_live = ltot;
    c->n_garbage = gtot;
    c->n_kill = ktot;
    uint64_t t[3] = {0, 0, 0};
    for (int w = 0; w < 16; ++w)
      for (int k = 0; k < 3; ++k) t[k] += wst[k][w];
    c->sup_edges = t[0];
    c->edges_scanned = t[1];
    c->expand_bytes = t[2];
  }
}

__global__ __launch_bounds__(256) void k_sweep_gather(DevGraph g, HostLists hl) {
  Counters *c = g.ctr;
  if (!c->mark_done) return;
  const bool commit = c->npe == 0;
  // the ids straight into the caller's host buffers as well, when they fit (one
  // kernel less than a copy behind the gather; the host checks the counts)
  uint64_t *const hg = (hl.g && commit && c->n_garbage <= hl.gcap) ? hl.g : nullptr;
  uint64_t *const hk = (hl.k && commit && c->n_kill <= hl.kcap) ? hl.k : nullptr;
  const uint64_t nblk = (c->slot_top + BLK_SLOTS - 1) / BLK_SLOTS;
  const uint64_t gw = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const uint64_t nw = (uint64_t)gridDim.x * 4;
  for (uint64_t blk = gw; blk < nblk; blk += nw) {
    const uint32_t gn = g.sweep_cnt[2 * blk], kn = g.sweep_cnt[2 * blk + 1];
    if (gn == 0) continue;
    const uint64_t go = g.sweep_off[2 * blk], ko = g.sweep_off[2 * blk + 1];
    const uint32_t *ga = (const uint32_t *)g.out_a + blk * BLK_SLOTS;
    const uint32_t *ka = (const uint32_t *)g.out_b + blk * BLK_SLOTS;
    for (uint32_t i = lane_id(); i < gn; i += 64) {
      const uint32_t v = ga[i];
      const uint64_t id = g.vid[v];
      g.out_ids[go + i] = id;
      if (hg) hg[go + i] = id;
      if (commit) {
        uint64_t bucket = KEY_EMPTY;
        id_find(g, id, &bucket);
        if (bucket != KEY_EMPTY) g.htab[bucket].key = KEY_TOMB;
        g.flags[v] = 0;
        if (g.gslot) g.gslot[g.gslot_at + go + i] = v;  // slot reuse: purged, listed free (crgc_reuse.hip)
      }
    }
    for (uint32_t i = lane_id(); i < kn; i += 64) {
      const uint64_t id = g.vid[ka[i]];
      g.out_kill[ko + i] = id;
      if (hk) hk[ko + i] = id;
    }
  }
}

// The garbage / kill ids straight into the caller's device-accessible host
// buffers (page-locked or registered), behind the sweep on the same stream, so
// a trace needs one host synchronisation, not two (counters, then copies of
// their size).  A list longer than its buffer, an NPE or a mark that is not done
// yet copies nothing; the host then takes the copy path (and its E2BIG).
__global__ __launch_bounds__(256) void k_copy_lists(DevGraph g, uint64_t *gdst, uint64_t gcap, uint64_t *kdst,
                                                    uint64_t kcap) {
  const Counters *c = g.ctr;
  if (!c->mark_done || c->npe) return;
  const uint64_t ng = c->n_garbage, nk = c->n_kill;
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  const uint64_t t0 = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (gdst && ng <= gcap)
    for (uint64_t i = t0; i < ng; i += stride) gdst[i] = g.out_ids[i];
  if (kdst && nk <= kcap)
    for (uint64_t i = t0; i < nk; i += stride) kdst[i] = g.out_kill[i];
}

hipError_t launch_copy_lists(const DevGraph &g, uint64_t *gdst, uint64_t gcap, uint64_t *kdst, uint64_t kcap,
                             hipStream_t s) {
  launch_begin();
  hipLaunchKernelGGL(k_copy_lists, dim3(64), dim3(256), 0, s, g, gdst, gcap, kdst, kcap);
  return hipGetLastError();
}

// The counters the host loop reads after a level chunk (everything before the
// level ring, and ring[r0 .. r0 + rn) mod LEVEL_RING) stored by the device into
// the pinned host mirror: one small kernel instead of D2H copies into pageable
// vectors, each of which waited for the stream and went through a staging buffer.
__global__ __launch_bounds__(256) void k_publish(const Counters *c, Counters *hdst, uint32_t r0, uint32_t rn) {
  constexpr uint32_t PRE = (uint32_t)(offsetof(Counters, ring) / 8);
  const unsigned long long *src = (const unsigned long long *)c;
  unsigned long long *dst = (unsigned long long *)hdst;
  for (uint32_t i = threadIdx.x; i < PRE; i += 256) dst[i] = src[i];
  for (uint32_t i = threadIdx.x; i < rn; i += 256) {
    const uint32_t k = (r0 + i) % LEVEL_RING;
    hdst->ring[k] = c->ring[k];
  }
}

hipError_t launch_publish(const Counters *c, Counters *hdst, uint32_t r0, uint32_t rn, hipStream_t s) {
  launch_begin();
  hipLaunchKernelGGL(k_publish, dim3(1), dim3(256), 0, s, c, hdst, r0, rn);
  return hipGetLastError();
}

hipError_t launch_sweep(const DevGraph &g, int should_kill, uint64_t slot_top, hipStream_t s,
                        int phase, const HostLists &hl) {
  launch_begin();
  const int grid = level_grid(slot_top);
  if (phase & 1) {
    hipLaunchKernelGGL(k_sweep, dim3(grid), dim3(256), 0, s, g, should_kill);
    hipLaunchKernelGGL(k_sweep_scan, dim3(1), dim3(1024), 0, s, g, (uint32_t)grid);
  }
  if (phase & 2) hipLaunchKernelGGL(k_sweep_gather, dim3(grid), dim3(256), 0, s, g, hl);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Sharded graphs: exchange lists.  A shard lists slots per
// 2048-slot block (newly marked proxies during the mark, garbage whose kill
// waits on a remote supervisor mark during the sweep); these kernels turn a
// listing into actor ids packed by destination shard, one region per shard
// in shard order, ready for the all-to-all.
//   k_list_count    per-destination counts (LDS histogram, one atomic per
//                   destination per workgroup) -> Counters::xcnt
//   k_list_scatter  ids (and the listed slot, for requests) into
//                   send[off(d) + ...]; off = exclusive scan of xcnt
// MODE 0: export (id of the listed proxy);  MODE 1: request (id of the
// listed garbage shadow's supervisor, plus the garbage slot).
// ---------------------------------------------------------------------------
template <int MODE>
__device__ inline uint64_t listed_id(const DevGraph &g, uint32_t v) {
  return MODE == 0 ? g.vid[v] : g.vid[g.sup[v]];
}

template <int MODE>
__global__ __launch_bounds__(256) void k_list_count(DevGraph g, const uint32_t *buf, const uint32_t *cnt,
                                                    uint64_t nblk) {
  __shared__ uint32_t hist[MAX_SHARDS];
  for (uint32_t d = threadIdx.x; d < MAX_SHARDS; d += 256) hist[d] = 0;
  __syncthreads();
  const uint64_t gw = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6), nw = (uint64_t)gridDim.x * 4;
  for (uint64_t blk = gw; blk < nblk; blk += nw) {
    const uint32_t n = cnt[blk];
    for (uint32_t i = lane_id(); i < n; i += 64)
      atomicAdd(&hist[shard_of(listed_id<MODE>(g, buf[blk * BLK_SLOTS + i]), g.n_shards)], 1u);
  }
  __syncthreads();
  for (uint32_t d = threadIdx.x; d < g.n_shards; d += 256)
    if (hist[d]) atomicAdd(&g.ctr->xcnt[d], (unsigned long long)hist[d]);
}

template <int MODE>
__global__ __launch_bounds__(256) void k_list_scatter(DevGraph g, uint32_t *buf, uint32_t *cnt,
                                                      uint64_t nblk, uint64_t *send, uint32_t *send_slot) {
  __shared__ uint32_t hist[MAX_SHARDS];
  __shared__ unsigned long long base[MAX_SHARDS];
  for (uint32_t d = threadIdx.x; d < MAX_SHARDS; d += 256) hist[d] = 0;
  __syncthreads();
  const uint64_t gw = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6), nw = (uint64_t)gridDim.x * 4;
  for (uint64_t blk = gw; blk < nblk; blk += nw) {
    const uint32_t n = cnt[blk];
    for (uint32_t i = lane_id(); i < n; i += 64)
      atomicAdd(&hist[shard_of(listed_id<MODE>(g, buf[blk * BLK_SLOTS + i]), g.n_shards)], 1u);
  }
  __syncthreads();
  if (threadIdx.x < g.n_shards) {
    const uint32_t d = threadIdx.x;
    unsigned long long off = 0;
    for (uint32_t e = 0; e < d; ++e) off += g.ctr->xcnt[e];
    base[d] = off + (hist[d] ? atomicAdd(&g.ctr->xpos[d], (unsigned long long)hist[d]) : 0ull);
    hist[d] = 0;
  }
  __syncthreads();
  for (uint64_t blk = gw; blk < nblk; blk += nw) {
    const uint32_t n = cnt[blk];
    for (uint32_t i = lane_id(); i < n; i += 64) {
      const uint32_t v = buf[blk * BLK_SLOTS + i];
      const uint64_t id = listed_id<MODE>(g, v);
      const uint32_t d = shard_of(id, g.n_shards);
      const uint64_t at = base[d] + atomicAdd(&hist[d], 1u);
      send[at] = id;
      if (MODE == 1) send_slot[at] = v;
    }
  }
}

hipError_t launch_list(const DevGraph &g, int mode, bool scatter, uint32_t *buf, uint32_t *cnt,
                       uint64_t nblk, uint64_t *send, uint32_t *send_slot, hipStream_t s) {
  launch_begin();
  if (nblk == 0) return hipSuccess;
  const int grid = (int)((nblk + 3) / 4);
  if (!scatter) {
    if (mode == 0) hipLaunchKernelGGL(k_list_count<0>, dim3(grid), dim3(256), 0, s, g, buf, cnt, nblk);
    else hipLaunchKernelGGL(k_list_count<1>, dim3(grid), dim3(256), 0, s, g, buf, cnt, nblk);
  } else {
    if (mode == 0)
      hipLaunchKernelGGL(k_list_scatter<0>, dim3(grid), dim3(256), 0, s, g, buf, cnt, nblk, send, send_slot);
    else
      hipLaunchKernelGGL(k_list_scatter<1>, dim3(grid), dim3(256), 0, s, g, buf, cnt, nblk, send, send_slot);
  }
  return hipGetLastError();
}

// ---- mark rounds in home-slot form (sharded graphs) -------------------------
// A proxy caches its actor's slot at the home shard (g.phs), resolved once by
// an id exchange and dropped when the home compacts (renumbers) its slots.
// A marked proxy with a cached home slot travels as that slot: a list of u32
// slots, or — when that is longer — a bitmap over the home's slots; one
// without travels as its id.

// Proxies homed at the shards in `mask` forget their home slots, and every
// proxy is looked at again by the next listing (res_top).
__global__ __launch_bounds__(256) void k_phs_reset(DevGraph g, uint64_t mask) {
  const uint64_t top = g.pbase + g.ctr->proxy_top, stride = (uint64_t)gridDim.x * 256;
  for (uint64_t v = g.pbase + (uint64_t)blockIdx.x * 256 + threadIdx.x; v < top; v += stride)
    if ((g.flags[v] & FL_PROXY) && ((mask >> g.psh[v]) & 1ull)) g.phs[v] = PHS_NONE;
  if (blockIdx.x == 0 && threadIdx.x == 0) g.ctr->res_top = 0;
}

// Proxies below res_top have asked already (or were reset and res_top is 0):
// after a resolution every proxy so far has.
__global__ void k_res_done(Counters *c) { c->res_top = c->proxy_top; }

__device__ inline bool unresolved_proxy(const DevGraph &g, uint64_t v) {
  return (g.flags[v] & (FL_ALIVE | FL_PROXY)) == (FL_ALIVE | FL_PROXY) && g.phs[v] == PHS_NONE;
}

// Unresolved proxies by home shard: counts (xcnt), then ids + local slots
// (send / send_slot, grouped by destination; cursors xpos).
template <bool SCATTER>
__global__ __launch_bounds__(256) void k_res_list(DevGraph g, uint64_t *send, uint32_t *send_slot) {
  __shared__ uint32_t hist[MAX_SHARDS];
  __shared__ unsigned long long base[MAX_SHARDS];
  for (uint32_t d = threadIdx.x; d < MAX_SHARDS; d += 256) hist[d] = 0;
  __syncthreads();
  // the proxies created since the last resolution (all of them after a reset):
  // steady-state traces list only the new ones
  const uint64_t top = g.pbase + g.ctr->proxy_top, stride = (uint64_t)gridDim.x * 256;
  const uint64_t v0 = g.pbase + g.ctr->res_top + (uint64_t)blockIdx.x * 256 + threadIdx.x;
  for (uint64_t v = v0; v < top; v += stride)
    if (unresolved_proxy(g, v)) atomicAdd(&hist[g.psh[v]], 1u);
  __syncthreads();
  if (!SCATTER) {
    for (uint32_t d = threadIdx.x; d < g.n_shards; d += 256)
      if (hist[d]) atomicAdd(&g.ctr->xcnt[d], (unsigned long long)hist[d]);
    return;
  }
  if (threadIdx.x < g.n_shards) {
    const uint32_t d = threadIdx.x;
    unsigned long long off = 0;
    for (uint32_t e = 0; e < d; ++e) off += g.ctr->xcnt[e];
    base[d] = off + (hist[d] ? atomicAdd(&g.ctr->xpos[d], (unsigned long long)hist[d]) : 0ull);
    hist[d] = 0;
  }
  __syncthreads();
  for (uint64_t v = v0; v < top; v += stride) {
    if (!unresolved_proxy(g, v)) continue;
    const uint64_t id = g.vid[v];
    const uint32_t d = g.psh[v];
    const uint64_t at = base[d] + atomicAdd(&hist[d], 1u);
    send[at] = id;
    send_slot[at] = (uint32_t)v;
  }
}

// At the home: the slot of each asked id (PHS_ABSENT: no live home shadow).
__global__ __launch_bounds__(256) void k_res_answer(DevGraph g, const uint64_t *ids, uint64_t n, uint32_t *ans) {
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
    const uint32_t v = id_find(g, ids[i]);
    ans[i] = (v < 0xFFFFFFF0u && (g.flags[v] & (FL_ALIVE | FL_PROXY)) == FL_ALIVE) ? v : PHS_ABSENT;
  }
}

__global__ __launch_bounds__(256) void k_phs_set(DevGraph g, const uint32_t *slots, const uint32_t *ans,
                                                 uint64_t n) {
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) g.phs[slots[i]] = ans[i];
}

hipError_t launch_resolve(const DevGraph &g, int step, uint64_t mask, uint64_t *send, uint32_t *slots,
                          const uint64_t *ids, uint64_t n, uint32_t *ans, uint64_t n_proxy, hipStream_t s) {
  launch_begin();
  const int vgrid = grid_for(std::max<uint64_t>(n_proxy, 1), 256, 4096);
  switch (step) {
    case 5: hipLaunchKernelGGL(k_res_done, dim3(1), dim3(1), 0, s, g.ctr); break;
    case 0: hipLaunchKernelGGL(k_phs_reset, dim3(vgrid), dim3(256), 0, s, g, mask); break;
    case 1: hipLaunchKernelGGL(k_res_list<false>, dim3(vgrid), dim3(256), 0, s, g, send, slots); break;
    case 2: hipLaunchKernelGGL(k_res_list<true>, dim3(vgrid), dim3(256), 0, s, g, send, slots); break;
    case 3:
      if (n) hipLaunchKernelGGL(k_res_answer, dim3(grid_for(n, 256, 4096)), dim3(256), 0, s, g, ids, n, ans);
      break;
    default:
      if (n) hipLaunchKernelGGL(k_phs_set, dim3(grid_for(n, 256, 4096)), dim3(256), 0, s, g, slots, ans, n);
  }
  return hipGetLastError();
}

// The proxies marked since the last export (marked, not yet sent: vis &
// ~xsent over the proxy region), by destination: ids of the unresolved (xcnt),
// home slots of the resolved (xcnt2); then the scatter into the byte layout the
// host derived from the all-gathered counts, which records them as sent.  A
// streaming pass over the region's marked / sent words and, for the new marks
// only, their home shards and home slots (round 4 listed marked proxies into
// per-block regions as the level kernels found them and packed the lists: a
// chain of dependent loads per entry, ~0.8 ms per shard for C4's first round
// over 8 logical shards).
// One wave per quarter q of a 2048-proxy block: lane l holds the block's word l
// (marked and sent) when l / 16 == q; step k (8q .. 8q + 7) covers slots 64k .. 64k+63 (slot 64k + l: word 2k + l / 32,
// bit l % 32, by one shuffle), so the loads of a step are coalesced; XU steps
// per load group.  The count pass derives each new mark's key (form << 6 |
// destination; 0xFF: none — its home is marked already) from the home shard,
// the home slot and the replicated home bitmaps, stores it as a byte and leaves
// its workgroup's count per key in `wgc`; k_xscan_sum turns those into each
// workgroup's run of each segment (an exclusive scan), and the scatter pass
// (same grid, so the same blocks per workgroup) reads the key bytes back, so
// the random bitmap probes run once.
template <bool SCATTER>
__global__ __launch_bounds__(256) void k_xscan(DevGraph g, char *send, XSend x, uint32_t *wgc) {
  __shared__ uint32_t hist[2 * MAX_SHARDS];
  __shared__ unsigned long long base[2 * MAX_SHARDS];
  const uint32_t G = g.n_shards;
  uint32_t *mine = wgc + (uint64_t)blockIdx.x * 2 * G;  // this workgroup's counts: [form][destination]
  for (uint32_t q = threadIdx.x; q < 2 * MAX_SHARDS; q += 256) {
    hist[q] = 0;
    if (SCATTER) {  // this workgroup's run of each segment: k_xscan_sum's exclusive scan
      const uint32_t f = q / MAX_SHARDS, d = q % MAX_SHARDS;
      base[q] = d < G ? mine[f * G + d] : 0ull;
    }
  }
  __syncthreads();
  const uint64_t gw = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6), nw = (uint64_t)gridDim.x * 4;
  const uint64_t np = g.ctr->proxy_top;
  const uint64_t nb = (np + BLK_SLOTS - 1) / BLK_SLOTS;
  const uint64_t w0 = g.pbase / 32;  // the region's first marked word (pbase is block-aligned)
  const uint32_t lane = lane_id();
  constexpr uint32_t XU = 4;
  // A wave's unit is 1 / xq of a block (xq = 4: 512 slots, words 16q .. 16q +
  // 15, steps 8q .. 8q + 7): a new mark's key is a chain of dependent loads
  // (psh, phs, the home bitmap), so xq times the waves hide xq times the
  // latency (a wave per block walked its 32 steps alone: 22 / 40 us per count /
  // scatter pass on C2 over 8 logical shards, profiles/r6i; 13 / 18 us at 4)
  const uint32_t XQ = x.xq, wpu = 64 / XQ, spu = 32 / XQ;
  const uint64_t nu = nb * XQ;
  for (uint64_t un = gw; un < nu; un += nw) {
    const uint64_t blk = un / XQ;
    const uint32_t q = (uint32_t)(un % XQ);
    const uint64_t w = w0 + blk * 64 + lane;
    uint32_t mw = 0, sw = 0;
    if (lane / wpu == q) {  // this lane's word is in the unit
      mw = g.vis[w];
      sw = g.xsent[w];
    }
    const uint32_t nm = mw & ~sw;
    if (!__ballot(nm != 0)) continue;
    for (uint32_t k0 = spu * q; k0 < spu * q + spu; k0 += XU) {
      uint32_t v[XU], key[XU];
      bool any = false;
#pragma unroll
      for (uint32_t u = 0; u < XU; ++u) {
        const uint32_t word = __shfl(nm, 2 * (k0 + u) + (lane >> 5));
        const uint64_t sl = g.pbase + blk * BLK_SLOTS + (k0 + u) * 64 + lane;
        v[u] = ((word >> (lane & 31)) & 1u) && sl - g.pbase < np ? (uint32_t)sl : NO_SLOT;
        any |= __ballot(v[u] != NO_SLOT) != 0;
      }
      if (!any) continue;
      if (!SCATTER) {
        uint32_t hs[XU];
#pragma unroll
        for (uint32_t u = 0; u < XU; ++u) {
          const uint32_t d = v[u] != NO_SLOT ? g.psh[v[u]] : 0u;
          hs[u] = v[u] != NO_SLOT && x.use_slots ? g.phs[v[u]] : PHS_NONE;
          key[u] = v[u] == NO_SLOT ? ~0u : ((hs[u] < PHS_ABSENT ? 64u : 0u) | d);
        }
        if (x.gvis) {  // marks their homes already have stay here
#pragma unroll
          for (uint32_t u = 0; u < XU; ++u)
            if (key[u] != ~0u && (key[u] >> 6)) {
              const uint32_t d = key[u] & 63;
              const uint64_t gwd = x.gvis_off[d] + (hs[u] >> 5);
              if (gwd < x.gvis_off[d + 1] && ((x.gvis[gwd] >> (hs[u] & 31)) & 1u)) key[u] = ~0u;
            }
        }
#pragma unroll
        for (uint32_t u = 0; u < XU; ++u) {
          if (v[u] != NO_SLOT) g.xkey[v[u]] = key[u] == ~0u ? (uint8_t)0xFF : (uint8_t)key[u];
          for (uint64_t pend = __ballot(key[u] != ~0u); pend;) {
            const uint32_t kk = __shfl(key[u], __ffsll((unsigned long long)pend) - 1);
            const uint64_t m = __ballot(key[u] == kk);
            if (lane == (uint32_t)(__ffsll((unsigned long long)m) - 1))
              atomicAdd(&hist[(kk >> 6) * MAX_SHARDS + (kk & 63)], (uint32_t)__popcll(m));
            pend &= ~m;
          }
        }
        continue;
      }
      // scatter: the keys back, then the home slot (a resolved mark) or the id
#pragma unroll
      for (uint32_t u = 0; u < XU; ++u) {
        const uint8_t kb = v[u] != NO_SLOT ? g.xkey[v[u]] : (uint8_t)0xFF;
        key[u] = kb == 0xFF ? ~0u : (uint32_t)kb;
      }
      uint64_t val[XU];
#pragma unroll
      for (uint32_t u = 0; u < XU; ++u)
        val[u] = key[u] == ~0u ? 0ull : (key[u] >> 6) ? (uint64_t)g.phs[v[u]] : g.vid[v[u]];
#pragma unroll
      for (uint32_t u = 0; u < XU; ++u) {
        // this lane's position: its wave's run of the key, at the key's next
        // position in this workgroup's range (consecutive lanes, consecutive
        // addresses: one store per run)
        uint64_t at = 0;
        for (uint64_t pend = __ballot(key[u] != ~0u); pend;) {
          const uint32_t kk = __shfl(key[u], __ffsll((unsigned long long)pend) - 1);
          const uint64_t m = __ballot(key[u] == kk);
          const uint32_t leader = (uint32_t)(__ffsll((unsigned long long)m) - 1);
          const bool bm = (kk >> 6) && x.bitmap[kk & 63];
          uint32_t r0 = 0;
          if (lane == leader && !bm) r0 = atomicAdd(&hist[(kk >> 6) * MAX_SHARDS + (kk & 63)], (uint32_t)__popcll(m));
          r0 = __shfl(r0, leader);
          if (key[u] == kk) at = base[(kk >> 6) * MAX_SHARDS + (kk & 63)] + r0 + __popcll(m & lanemask_lt());
          pend &= ~m;
        }
        if (key[u] == ~0u) continue;
        const uint32_t d = key[u] & 63;
        if (!(key[u] >> 6)) {  // (the id only for the unresolved)
          ((uint64_t *)(send + x.id_off[d]))[at] = val[u];
        } else if (x.bitmap[d]) {
          const uint32_t hs = (uint32_t)val[u];
          atomicOr((uint32_t *)(send + x.sl_off[d]) + (hs >> 5), 1u << (hs & 31));
        } else {
          ((uint32_t *)(send + x.sl_off[d]))[at] = (uint32_t)val[u];
        }
      }
    }
    if (SCATTER && nm) g.xsent[w] = sw | nm;
  }
  if (!SCATTER) {  // (one global atomic per workgroup and key serialised ~4 400 workgroups on
                   // 2G words: ~50 us per pass at C4 over 8 logical shards; k_xscan_sum scans)
    __syncthreads();
    for (uint32_t q = threadIdx.x; q < 2 * G; q += 256) mine[q] = hist[(q / G) * MAX_SHARDS + q % G];
  }
}

// Per key (one workgroup each): the exclusive scan of the workgroups' counts
// in place, the total into xcnt / xcnt2.  XS consecutive workgroups' counts per
// thread: k_xscan's largest grid (8192) in one pass (one per thread was a pass
// per 1024: 8.4 us at C2 over 8 logical shards, 15.3 at C4 half size with
// quarter-block units, profiles/r6y, r6ac).
__global__ __launch_bounds__(1024) void k_xscan_sum(DevGraph g, uint32_t *wgc, uint32_t nwg) {
  constexpr uint32_t XS = 8;
  __shared__ uint32_t s_w[40];
  const uint32_t G = g.n_shards, q = blockIdx.x;
  uint32_t run = 0;
  for (uint32_t w0 = 0; w0 < nwg; w0 += 1024 * XS) {
    const uint32_t wb = w0 + threadIdx.x * XS;
    uint32_t n[XS], sum = 0;
#pragma unroll
    for (uint32_t k = 0; k < XS; ++k) {
      n[k] = wb + k < nwg ? wgc[(uint64_t)(wb + k) * 2 * G + q] : 0u;
      sum += n[k];
    }
    uint32_t tot;
    uint32_t ex = run + tail_scan(sum, s_w, tot);
#pragma unroll
    for (uint32_t k = 0; k < XS; ++k)
      if (wb + k < nwg) {
        wgc[(uint64_t)(wb + k) * 2 * G + q] = ex;
        ex += n[k];
      }
    run += tot;
  }
  if (threadIdx.x == 0) {
    const uint32_t f = q / G, d = q % G;
    (f ? g.ctr->xcnt2 : g.ctr->xcnt)[d] = run;
  }
}

int xscan_grid(uint64_t nblk, uint32_t xq) { return (int)std::max<uint64_t>(1, std::min<uint64_t>((nblk * xq + 3) / 4, 8192)); }

hipError_t launch_xlist(const DevGraph &g, bool scatter, uint64_t nblk, char *send, const XSend &x,
                        uint32_t *wgc, hipStream_t s) {
  launch_begin();
  if (nblk == 0) return hipSuccess;
  const int grid = xscan_grid(nblk, x.xq);
  if (scatter) {
    hipLaunchKernelGGL(k_xscan<true>, dim3(grid), dim3(256), 0, s, g, send, x, wgc);
  } else {
    hipLaunchKernelGGL(k_xscan<false>, dim3(grid), dim3(256), 0, s, g, send, x, wgc);
    hipLaunchKernelGGL(k_xscan_sum, dim3(2 * g.n_shards), dim3(1024), 0, s, g, wgc, (uint32_t)grid);
  }
  return hipGetLastError();
}

// Received marks become candidates of level L (a sparse level: the dirty map
// names their blocks); ring[L-1] gets their number so the level kernels run.
// Work item i: source r = the last with x.start[r] <= i; its ids first, then
// its home slots (or bitmap words).
__device__ inline uint32_t import_mark(const DevGraph &g, uint8_t *Fc, uint8_t *Dc, uint32_t v, uint64_t top) {
  if (v >= top) return 0;
  if ((g.flags[v] & (FL_ALIVE | FL_PROXY)) != FL_ALIVE) return 0;
  if ((g.vis[v >> 5] >> (v & 31)) & 1u) return 0;
  Fc[v] = 1;
  Dc[v >> 11] = 1;
  return 1;
}

// XI work items per thread, their loads issued together (one item per thread
// was a chain of three dependent loads: 0.2 ms per shard for C4's second
// round over 8 logical shards, profiles/r5o).
__global__ __launch_bounds__(256) void k_ximport(DevGraph g, const char *recv, XRecv x, int L) {
  constexpr int XI = 4;
  uint8_t *Fc = g.front[L & 1];
  uint8_t *Dc = g.dirty[L & 1];
  const uint64_t top = g.ctr->slot_top;
  uint32_t found = 0;
  const uint64_t total = x.start[x.G], stride = (uint64_t)gridDim.x * 256;
  for (uint64_t i0 = (uint64_t)blockIdx.x * 256 + threadIdx.x; i0 < total; i0 += stride * XI) {
    uint32_t v[XI];
#pragma unroll
    for (int u = 0; u < XI; ++u) {
      const uint64_t i = i0 + u * stride;
      v[u] = NO_SLOT;
      if (i >= total) continue;
      uint32_t r = 0;
      while (r + 1 < x.G && x.start[r + 1] <= i) ++r;
      const uint64_t k = i - x.start[r];
      const char *seg = recv + x.off[r];
      if (k < x.n_id[r]) {
        const uint32_t s = id_find(g, ((const uint64_t *)seg)[k]);
        if (s < 0xFFFFFFF0u) v[u] = s;
        continue;
      }
      const uint64_t j = k - x.n_id[r];
      const uint32_t w = ((const uint32_t *)(seg + 8 * x.n_id[r]))[j];
      if (!x.bitmap[r]) {
        v[u] = w;
      } else {
        for (uint32_t m = w; m; m &= m - 1) found += import_mark(g, Fc, Dc, (uint32_t)(j * 32) + __ffs(m) - 1, top);
      }
    }
    uint8_t f[XI];
    uint32_t vw[XI];
#pragma unroll
    for (int u = 0; u < XI; ++u) {
      const bool in = v[u] < top;
      f[u] = in ? g.flags[v[u]] : (uint8_t)0;
      vw[u] = in ? g.vis[v[u] >> 5] : ~0u;
    }
#pragma unroll
    for (int u = 0; u < XI; ++u)
      if (v[u] < top && (f[u] & (FL_ALIVE | FL_PROXY)) == FL_ALIVE && !((vw[u] >> (v[u] & 31)) & 1u)) {
        Fc[v[u]] = 1;
        Dc[v[u] >> 11] = 1;
        ++found;
      }
  }
  const uint64_t t = block_sum4(found);
  if (threadIdx.x == 0 && t) atomicAdd(&g.ctr->ring[(L - 1) % LEVEL_RING], (unsigned long long)t);
}

// A mark round's start (one launch instead of four memsets): the trace state a
// fresh sparse level L needs — the two level counts before it and its hub queue
// zeroed (not when the round continues a capped one: level L's candidates and
// counts are the previous round's) — and no narrow-frontier state.
__global__ void k_round_start(Counters *c, int L, int fresh) {
  if (fresh) {
    c->ring[(L - 2) % LEVEL_RING] = 0;
    c->ring[(L - 1) % LEVEL_RING] = 0;
    c->qh[L & 1] = 0;
  }
  c->tail_state = 0;
}

hipError_t launch_round_start(Counters *c, int level, bool fresh, hipStream_t s) {
  launch_begin();
  hipLaunchKernelGGL(k_round_start, dim3(1), dim3(1), 0, s, c, level, fresh ? 1 : 0);
  return hipGetLastError();
}

__global__ __launch_bounds__(256) void k_zero_u64(unsigned long long *p, uint32_t n) {
  for (uint32_t i = threadIdx.x; i < n; i += 256) p[i] = 0;
}

hipError_t launch_zero_u64(void *p, uint32_t n, hipStream_t s) {
  launch_begin();
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_zero_u64, dim3(1), dim3(256), 0, s, (unsigned long long *)p, n);
  return hipGetLastError();
}

hipError_t launch_ximport(const DevGraph &g, const char *recv, const XRecv &x, int level, hipStream_t s) {
  launch_begin();
  const uint64_t n = x.start[x.G];
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_ximport, dim3(grid_for((n + 3) / 4, 256, 4096)), dim3(256), 0, s, g, recv, x, level);
  return hipGetLastError();
}

// Kill requests answered at the supervisor's home: is it marked?
__global__ __launch_bounds__(256) void k_req_answer(DevGraph g, const uint64_t *ids, uint64_t n,
                                                    uint8_t *ans) {
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
    const uint32_t v = id_find(g, ids[i]);
    ans[i] = (v < 0xFFFFFFF0u && ((g.vis[v >> 5] >> (v & 31)) & 1u)) ? 1 : 0;
  }
}

// Requests whose supervisor is marked join the kill list (after the gather).
__global__ __launch_bounds__(256) void k_kill_fix(DevGraph g, const uint32_t *slots, const uint8_t *ans,
                                                  uint64_t n) {
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t b = (uint64_t)blockIdx.x * 256 + (threadIdx.x & ~63u); b < n; b += stride) {
    const uint64_t i = b + lane_id();
    const bool k = i < n && ans[i];
    const unsigned long long at = wave_append(&g.ctr->n_kill, k);
    if (k) g.out_kill[at] = g.vid[slots[i]];
  }
}

hipError_t launch_requests(const DevGraph &g, int phase, const uint64_t *ids, uint64_t n, uint8_t *ans,
                           const uint32_t *slots, hipStream_t s) {
  launch_begin();
  if (n == 0) return hipSuccess;
  const int grid = grid_for(n, 256, 4096);
  if (phase == 0) hipLaunchKernelGGL(k_req_answer, dim3(grid), dim3(256), 0, s, g, ids, n, ans);
  else hipLaunchKernelGGL(k_kill_fix, dim3(grid), dim3(256), 0, s, g, slots, ans, n);
  return hipGetLastError();
}

// Other shards' garbage: this shard's proxies of it die with it (their ids
// will name a new incarnation if they ever reappear — SURVEY E9).
__global__ __launch_bounds__(256) void k_invalidate(DevGraph g, const uint64_t *ids, uint64_t n) {
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  uint32_t dead = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
    uint64_t bucket = KEY_EMPTY;
    const uint32_t v = id_find(g, ids[i], &bucket);
    if (v >= 0xFFFFFFF0u || bucket == KEY_EMPTY) continue;
    if ((g.flags[v] & (FL_ALIVE | FL_PROXY)) != (FL_ALIVE | FL_PROXY)) continue;
    g.htab[bucket].key = KEY_TOMB;
    g.flags[v] = 0;
    ++dead;
  }
  const uint64_t t = block_sum4(dead);  // the proxy region's dead slots (the rebuild trigger)
  if (threadIdx.x == 0 && t) atomicAdd(&g.ctr->proxy_dead, (unsigned long long)t);
}

hipError_t launch_invalidate(const DevGraph &g, const uint64_t *ids, uint64_t n, hipStream_t s) {
  launch_begin();
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_invalidate, dim3(grid_for(n, 256, 4096)), dim3(256), 0, s, g, ids, n);
  return hipGetLastError();
}

// Marked home shadows (investigateRemotelyHeldActors' to.size(), :329) -> n_out.
__global__ __launch_bounds__(256) void k_count_marked(DevGraph g) {
  const uint64_t nblk = (g.ctr->slot_top + BLK_SLOTS - 1) / BLK_SLOTS;
  const uint64_t gw = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6), nw = (uint64_t)gridDim.x * 4;
  uint32_t k = 0;
  for (uint64_t blk = gw; blk < nblk; blk += nw) {
    const uint64_t base = blk * BLK_SLOTS + (uint64_t)lane_id() * 32;
    const uint32_t word = g.vis[blk * 64 + lane_id()];
    if (!word) continue;
    const uint4 f4[2] = {*(const uint4 *)(g.flags + base), *(const uint4 *)(g.flags + base + 16)};
    const uint8_t *fb = (const uint8_t *)f4;
    uint32_t home = 0;
#pragma unroll
    for (int j = 0; j < 32; ++j) home |= ((fb[j] & (FL_ALIVE | FL_PROXY)) == FL_ALIVE) ? (1u << j) : 0u;
    k += __popc(word & home);
  }
  const uint64_t t = block_sum4(k);
  if (threadIdx.x == 0 && t) atomicAdd(&g.ctr->n_out, (unsigned long long)t);
}

hipError_t launch_count_marked(const DevGraph &g, uint64_t slot_top, hipStream_t s) {
  launch_begin();
  hipLaunchKernelGGL(k_count_marked, dim3(level_grid(slot_top)), dim3(256), 0, s, g);
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
  launch_begin();
  hipLaunchKernelGGL(k_local_roots, dim3(grid_for(slot_top, 256, 8192)), dim3(256), 0, s, g);
  return hipGetLastError();
}

}  // namespace crgc
