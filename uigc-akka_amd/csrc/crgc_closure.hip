// crgc_closure.hip — the mark of ShadowGraph.trace (ShadowGraph.java:205-268)
// as a closure over parent hints, for unsharded graphs whose marks are wide.
//
// The reference's marked set is the least set that holds the pseudo-roots
// (:201-203) and is closed under { (o -> t) : outgoing[o][t] > 0, o marked and
// not halted } and { (c -> supervisor(c)) : c marked and not halted }
// (:226-268).  Any process that only marks shadows with such a reason and stops
// once no unmarked shadow has one reaches exactly that set, whatever its order.
// The level-synchronous BFS (crgc_trace.hip) is one such process; this is
// another, built for wakeups where the graph barely changes between traces:
//
//   step 0, ROOTS  the pseudo-roots (one wave per 2048-slot block, as k_frontier
//                  level 0), their supervisors as candidate bytes
//   HINT           every unmarked shadow whose parent hint `par` (an owner whose
//                  edge to it has a positive count: set by pull searches, cleared
//                  by the merge when that count stops being positive) is marked
//                  and not halted (`em`, an L2-resident bitmap), and every
//                  candidate byte, becomes marked; their supervisors become
//                  candidates of the next step.  Repeated while it finds some.
//   EXACT          once hints find nothing: every unmarked shadow searches its
//                  in-candidate list (RC_POS entries: positive counts) for a
//                  marked, unhalted owner, and records the owner as its hint;
//                  the found ones are candidates of the next (HINT) step.  An
//                  EXACT step that finds nothing ends the mark: no unmarked
//                  shadow has a reason, so the marked set is the closure.
//
// No O(E) push: in steady state a trace costs a handful of streaming passes over
// the slots plus one random L2 bit probe per shadow.  Every step is the same
// kernel; its mode follows from the previous step's (mode, count) word in the
// counter ring, so the host enqueues a chunk of steps and synchronises once.
// Candidate maps alternate by step parity (a step reads and clears one, stores
// into the other), so a clear never races a store.
#include <hip/hip_ext.h>

#include "crgc_host.hpp"

namespace crgc {

namespace {

constexpr unsigned long long CL_MASK = (1ull << 48) - 1;
enum : uint32_t { CL_ROOTS = 1, CL_HINT = 2, CL_EXACT = 3, CL_DONE = 4 };
constexpr int CL_FB = 4;             // newly marked shadows: chunks of 64 per load group
constexpr uint32_t CL_PULL_K = 4;    // EXACT: in-candidates per list per round
constexpr int STAT_SUP_ = 1, STAT_EDGES_ = 2;  // crgc_trace.hip's per-workgroup partials
constexpr uint32_t NO_HINT = ~0u;

// Mode of step k, from step k-1's word: mode << 56 | shadows marked or found +
// candidate bytes stored.
__device__ inline uint32_t cl_mode(const Counters *c, uint32_t k) {
  if (k == 0) return CL_ROOTS;
  const unsigned long long p = c->ring[(k - 1) % LEVEL_RING];
  const uint32_t pm = (uint32_t)(p >> 56);
  const bool any = (p & CL_MASK) != 0;
  if (pm == CL_ROOTS) return CL_HINT;
  if (pm == CL_HINT) return any ? CL_HINT : CL_EXACT;
  if (pm == CL_EXACT) return any ? CL_HINT : CL_DONE;
  return CL_DONE;
}

__device__ inline uint32_t cand_bits(const uint4 &x0, const uint4 &x1) {
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
  return bits;
}

__device__ inline uint64_t block_sum(uint64_t v) {
  __shared__ uint64_t part[4];
  const uint64_t w = __shfl(wave_incl_scan((uint32_t)v), 63);
  if (lane_id() == 0) part[threadIdx.x >> 6] = w;
  __syncthreads();
  const uint64_t s = part[0] + part[1] + part[2] + part[3];
  __syncthreads();
  return s;
}

}  // namespace

__global__ __launch_bounds__(256) void k_closure(DevGraph g, uint32_t k) {
  __shared__ uint16_t s_new[4][BLK_SLOTS];  // newly marked slots of the wave's block
  Counters *c = g.ctr;
  const uint32_t mode = cl_mode(c, k);
  unsigned long long *word = &c->ring[k % LEVEL_RING];
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    atomicOr(word, (unsigned long long)mode << 56);
    if (mode == CL_DONE) c->mark_done = 1;
  }
  if (mode == CL_DONE) return;
  const uint64_t slot_top = c->slot_top;
  uint8_t *Fc = g.front[k & 1];        // this step's candidates (read and cleared)
  uint8_t *Fn = g.front[(k + 1) & 1];  // the next step's
  uint32_t n_new = 0, n_store = 0, n_sup = 0, n_edges = 0, n_root = 0;

  if (mode == CL_EXACT) {
    // A thread owns 4 consecutive slots (their flags / candidate bytes are
    // one u32), walking their in-candidate lists together, CL_PULL_K entries
    // per list per round: one round trip for the entries, one for the owners'
    // `em` bits, until every list has a hit or is exhausted.
    const uint64_t nq = (slot_top + 3) / 4;
    const uint64_t gs = (uint64_t)gridDim.x * 256;
    for (uint64_t q = (uint64_t)blockIdx.x * 256 + threadIdx.x; q < nq; q += gs) {
      const uint64_t v0 = q * 4;
      const uint32_t fl = *(const uint32_t *)(g.flags + v0);
      const uint32_t vb = (g.vis[v0 >> 5] >> (v0 & 31)) & 0xFu;
      uint32_t todo = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        todo |= ((((fl >> (8 * j)) & (FL_ALIVE | FL_PROXY)) == FL_ALIVE) && !((vb >> j) & 1u)) ? (1u << j) : 0u;
      if (!todo) continue;
      const uint4 r01 = *(const uint4 *)(g.radj + v0);
      const uint4 r23 = *(const uint4 *)(g.radj + v0 + 2);
      const uint32_t ro[4] = {r01.x, r01.z, r23.x, r23.z};
      const uint32_t rl[4] = {r01.y, r01.w, r23.y, r23.w};
      uint32_t live = todo, pos = 0, found = 0;
      while (live) {
        uint32_t u[4][CL_PULL_K];
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int kk = 0; kk < (int)CL_PULL_K; ++kk)
            u[j][kk] = ((live >> j) & 1u) && pos + kk < rl[j] ? g.rpool[(uint64_t)ro[j] + pos + kk] : 0u;
        uint32_t w[4][CL_PULL_K];
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int kk = 0; kk < (int)CL_PULL_K; ++kk) {
            const uint32_t sl = u[j][kk] & ~RC_POS;
            w[j][kk] = (u[j][kk] & RC_POS) ? g.fx[sl >> 5] >> (sl & 31) : 0u;
          }
        pos += CL_PULL_K;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          bool hit = false;
          uint32_t who = 0;
#pragma unroll
          for (int kk = (int)CL_PULL_K - 1; kk >= 0; --kk)
            if (w[j][kk] & 1u) {
              hit = true;
              who = u[j][kk] & ~RC_POS;
            }
          if (hit && ((live >> j) & 1u)) {
            found |= 1u << (8 * j);
            g.par[v0 + j] = who;  // later traces try this owner first
          }
          if (hit || pos >= rl[j]) live &= ~(1u << j);
        }
      }
      if (found) {
        *(uint32_t *)(Fn + v0) = found;  // this thread's bytes: nothing else stores them this step
        n_store += __popc(found);
      }
    }
  } else {
    // ROOTS / HINT: one wave per 2048-slot block, 32 slots per lane.
    const uint32_t nblk = (uint32_t)((slot_top + BLK_SLOTS - 1) / BLK_SLOTS);
    const int wv = threadIdx.x >> 6, lane = lane_id();
    const uint32_t gw = blockIdx.x * 4 + wv, nw = gridDim.x * 4;
    for (uint32_t blk = gw; blk < nblk; blk += nw) {
      const uint64_t base = (uint64_t)blk * BLK_SLOTS + (uint64_t)lane * 32;
      const uint64_t wi = (uint64_t)blk * 64 + lane;
      uint32_t w = 0, cb = 0;
      if (mode == CL_HINT) {
        w = g.vis[wi];
        uint4 *fp = (uint4 *)(Fc + base);
        const uint4 x0 = fp[0], x1 = fp[1];
        cb = cand_bits(x0, x1);
        if (cb) {
          fp[0] = make_uint4(0, 0, 0, 0);
          fp[1] = make_uint4(0, 0, 0, 0);
        }
      }
      uint32_t nm = 0, halted = 0;
      const bool look = mode == CL_ROOTS || w != ~0u;
      if (look) {
        const uint4 f4[2] = {*(const uint4 *)(g.flags + base), *(const uint4 *)(g.flags + base + 16)};
        const uint8_t *fb = (const uint8_t *)f4;
        uint32_t alive = 0;
#pragma unroll
        for (int j = 0; j < 32; ++j) {
          alive |= ((fb[j] & (FL_ALIVE | FL_PROXY)) == FL_ALIVE) ? (1u << j) : 0u;
          halted |= (fb[j] & FL_HALTED) ? (1u << j) : 0u;
        }
        if (mode == CL_ROOTS) {
          // isPseudoRoot (:201-203)
          int4 r4[8];
          const int4 *rp = (const int4 *)(g.recv + base);
#pragma unroll
          for (int q = 0; q < 8; ++q) r4[q] = rp[q];
          const int32_t *rb = (const int32_t *)r4;
#pragma unroll
          for (int j = 0; j < 32; ++j) {
            const uint8_t f = fb[j];
            const bool root = ((f & (FL_ROOT | FL_BUSY)) || !(f & FL_INTERNED) || rb[j] != 0);
            nm |= root ? (1u << j) : 0u;
          }
          nm &= alive & ~halted;
          n_root += __popc(nm);
        } else {
          nm = cb & alive & ~w;
          uint32_t todo = alive & ~w & ~nm;
          // parent hints: all of a half's hint loads, then all their bit probes
#pragma unroll
          for (int hf = 0; hf < 2; ++hf) {
            const uint32_t t16 = (todo >> (16 * hf)) & 0xFFFFu;
            if (!t16) continue;
            uint32_t p[16];
#pragma unroll
            for (int j = 0; j < 16; ++j) p[j] = ((t16 >> j) & 1u) ? g.par[base + 16 * hf + j] : NO_HINT;
            uint32_t e[16];
#pragma unroll
            for (int j = 0; j < 16; ++j) e[j] = p[j] < 0xFFFFFFF0u ? g.fx[p[j] >> 5] : 0u;
#pragma unroll
            for (int j = 0; j < 16; ++j)
              if (p[j] < 0xFFFFFFF0u && ((e[j] >> (p[j] & 31)) & 1u)) nm |= 1u << (16 * hf + j);
          }
        }
      }
      if (mode == CL_ROOTS) {
        g.vis[wi] = nm;  // every word: the reset left zeros, `em` starts here
        g.fx[wi] = nm;
      } else if (nm) {
        w |= nm;
        g.vis[wi] = w;
        g.fx[wi] = w & ~halted;  // the lane owns both words
      }
      n_new += __popc(nm);
      // Newly marked, unhalted shadows: their out-edge counts (the traced-edge
      // statistic) and supervisor edges (:258-267), 64 * CL_FB shadows per load
      // group, listed through LDS.
      const uint32_t ex = nm & ~halted;
      const uint32_t cnt = __popc(ex);
      const uint32_t incl = wave_incl_scan(cnt);
      const uint32_t total = __shfl(incl, 63);
      if (total == 0) continue;
      uint32_t pos = incl - cnt, m = ex;
      while (m) {
        const int j = __ffs(m) - 1;
        m &= m - 1;
        s_new[wv][pos++] = (uint16_t)(lane * 32 + j);
      }
      wave_lds_fence();
      for (uint32_t c0 = 0; c0 < total; c0 += 64 * CL_FB) {
        uint32_t v[CL_FB], sp[CL_FB], sw[CL_FB];
#pragma unroll
        for (int b = 0; b < CL_FB; ++b) {
          const uint32_t idx = c0 + b * 64 + lane;
          v[b] = idx < total ? blk * BLK_SLOTS + s_new[wv][idx] : NO_HINT;
        }
#pragma unroll
        for (int b = 0; b < CL_FB; ++b) {
          n_edges += v[b] != NO_HINT ? g.nzdeg[v[b]] : 0u;
          sp[b] = v[b] != NO_HINT ? g.sup[v[b]] : NO_HINT;
        }
#pragma unroll
        for (int b = 0; b < CL_FB; ++b) sw[b] = sp[b] < 0xFFFFFFF0u ? g.vis[sp[b] >> 5] : ~0u;
#pragma unroll
        for (int b = 0; b < CL_FB; ++b) {
          if (sp[b] < 0xFFFFFFF0u) {
            n_sup++;
            if (!((sw[b] >> (sp[b] & 31)) & 1u)) {  // a stale word only costs a redundant byte
              Fn[sp[b]] = 1;
              n_store++;
            }
          }
        }
      }
      wave_lds_fence();
    }
  }
  const uint64_t t_new = block_sum(n_new), t_store = block_sum(n_store);
  const uint64_t t_sup = block_sum(n_sup), t_edges = block_sum(n_edges), t_root = block_sum(n_root);
  if (threadIdx.x == 0) {
    if (t_new + t_store) atomicAdd(word, (unsigned long long)(t_new + t_store));
    if (t_new) atomicAdd(&c->marked, (unsigned long long)t_new);
    if (t_root) atomicAdd(&c->cl_roots, (unsigned long long)t_root);
    uint64_t *stat = g.blkstat + (uint64_t)blockIdx.x * 4;
    stat[STAT_SUP_] += t_sup;
    stat[STAT_EDGES_] += t_edges;
  }
}

hipError_t launch_closure(const DevGraph &g, uint32_t step, uint64_t slot_top, hipStream_t s) {
  hipLaunchKernelGGL(k_closure, dim3(level_grid(slot_top)), dim3(256), 0, s, g, step);
  return hipGetLastError();
}

}  // namespace crgc
