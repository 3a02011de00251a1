// crgc_chain.hip — chain mode: the end of a deep, narrow mark by pointer jumping.
//
// A mark whose frontier stays narrow for many levels (long chains of actors,
// BASELINE.json config 3) costs one dependent step per link when walked
// (k_tail: ~1.3 us per link).  Reachability does not depend on visiting order
// (ShadowGraph.java:224-268 marks the same `to` set whatever order its
// worklist takes), so once k_tail has walked `chain_after` rounds it hands the
// rest of the mark here:
//
//   nx0[v]  the unique out-target t != v with count > 0 (:231-241), NONE when v
//           has none, COMPLEX (bit in `cx`) when it has several
//   sp0[v]  the supervisor (:258-267), NONE when null / collected / investigate
//   (a halted shadow has neither: it is marked, never expanded, :226-229)
//
// Each outer iteration closes the marked set along nx0 by doubling — round k
// marks J_k(u) for every marked u, where J_0 = nx0 and J_{k+1} = J_k o J_k, so
// after round k everything within 2^(k+1) links of a marked shadow is marked,
// and a round that marks nothing means the closure is reached — then along
// sp0 the same way, then expands the complex shadows marked so far edge by
// edge (one wave per shadow).  It repeats until an iteration marks nothing.
// Cost: O(V log L) per iteration instead of L dependent steps per chain.
#include "crgc_host.hpp"

namespace crgc {

constexpr uint32_t CH_NONE = 0xFFFFFFFFu;
constexpr int STAT_SUP_SLOT = 1;  // crgc_trace.hip STAT_SUP of block 0
constexpr uint32_t CH_COMPLEX = 0xFFFFFFFEu;

__device__ inline bool bit_of(const uint32_t *bm, uint32_t v) { return (bm[v >> 5] >> (v & 31)) & 1u; }

// Marks t if it is not marked yet; returns whether this call marked it.
__device__ inline bool chain_mark(const DevGraph &g, const ChainArgs &ca, uint32_t *pb_out, uint32_t t) {
  const uint32_t bit = 1u << (t & 31);
  if (g.vis[t >> 5] & bit) return false;
  if (atomicOr(&g.vis[t >> 5], bit) & bit) return false;
  atomicOr(&g.cm[t >> 5], bit);
  if (bit_of(ca.cx, t)) atomicOr(&pb_out[t >> 5], bit);
  return true;
}

__device__ inline void chain_count(const ChainArgs &ca, uint32_t mine, uint32_t *flag) {
  const uint32_t w = wave_sum(mine);
  if (lane_id() == 0 && w) {
    atomicAdd(ca.n_new, (unsigned long long)w);
    *flag = 1;
  }
}

// nx0 / sp0 / cx of every slot.  One wave per 64 consecutive slots (the cx
// words are written whole by their wave).
__global__ __launch_bounds__(256) void k_chain_init(DevGraph g, ChainArgs ca, uint64_t top) {
  const uint64_t nwv = (uint64_t)gridDim.x * 4;
  for (uint64_t c0 = ((uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 64; c0 < top; c0 += nwv * 64) {
    const uint64_t v = c0 + lane_id();
    uint32_t nx = CH_NONE, sp = CH_NONE;
    bool cplx = false;
    if (v < top) {
      const uint8_t f = g.flags[v];
      if ((f & (FL_ALIVE | FL_PROXY | FL_HALTED)) == FL_ALIVE) {
        const uint2 ad = g.adj[v];
        for (uint32_t e = 0; e < ad.y && !cplx; ++e) {
          const uint64_t ed = g.pool[(uint64_t)ad.x + e];
          const uint32_t t = edge_target(ed);
          if (edge_count(ed) <= 0 || t == (uint32_t)v) continue;
          if (nx == CH_NONE) nx = t;
          else if (t != nx) cplx = true;
        }
        const uint32_t s = g.sup[v];
        if (!ca.investigate && s < 0xFFFFFFF0u) sp = s;
      }
      ca.nx0[v] = cplx ? CH_COMPLEX : nx;
      ca.sp0[v] = sp;
    }
    const uint64_t b = __ballot(cplx);
    if (lane_id() == 0) {
      ca.cx[c0 >> 5] = (uint32_t)b;
      ca.cx[(c0 >> 5) + 1] = (uint32_t)(b >> 32);
    }
  }
}

// One doubling round: marked u marks src[u]; dst[u] = src[src[u]].  Exits at
// once when the previous round of its sequence marked nothing.
__global__ __launch_bounds__(256) void k_chain_jump(DevGraph g, ChainArgs ca, const uint32_t *src, uint32_t *dst,
                                                    uint64_t top, uint32_t fi, int first) {
  if (!first && ca.flag[fi - 1] == 0) return;
  uint32_t *pb_out = ca.pb_in;  // complex shadows marked here are expanded later this iteration
  uint32_t mine = 0;
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t u = (uint64_t)blockIdx.x * 256 + threadIdx.x; u < top; u += stride) {
    const uint32_t j = src[u];
    uint32_t jj = j;
    if (j < 0xFFFFFFF0u) {
      if (bit_of(g.vis, (uint32_t)u)) mine += chain_mark(g, ca, pb_out, j) ? 1u : 0u;
      jj = src[j];
    }
    dst[u] = jj;
  }
  chain_count(ca, mine, &ca.flag[fi]);
}

// The complex shadows pending expansion (pb_in, cleared as read): every
// out-edge with count > 0, one wave per shadow; complex targets it marks go to
// pb_out for the next iteration.
__global__ __launch_bounds__(256) void k_chain_expand(DevGraph g, ChainArgs ca, uint64_t words, uint32_t fi) {
  uint32_t mine = 0;
  const int lane = lane_id();
  const uint64_t nwv = (uint64_t)gridDim.x * 4;
  for (uint64_t w0 = ((uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 64; w0 < words; w0 += nwv * 64) {
    const uint64_t w = w0 + lane;
    uint32_t bits = w < words ? ca.pb_in[w] : 0u;
    if (bits) ca.pb_in[w] = 0;
    uint64_t busy = __ballot(bits != 0);
    while (busy) {
      const int k = __ffsll((unsigned long long)busy) - 1;
      busy &= busy - 1;
      uint32_t kb = __shfl(bits, k);
      while (kb) {
        const uint32_t v = (uint32_t)((w0 + k) * 32 + (__ffs(kb) - 1));
        kb &= kb - 1;
        // k_tail hands over every pending claim: halted ones are marked, never expanded (:226-229)
        if ((g.flags[v] & (FL_ALIVE | FL_PROXY | FL_HALTED)) != FL_ALIVE) continue;
        const uint2 ad = g.adj[v];
        for (uint32_t e = lane; e < ad.y; e += 64) {
          const uint64_t ed = g.pool[(uint64_t)ad.x + e];
          if (edge_count(ed) > 0) mine += chain_mark(g, ca, ca.pb_out, edge_target(ed)) ? 1u : 0u;
        }
      }
    }
  }
  chain_count(ca, mine, &ca.flag[fi]);
}

// Statistics of the shadows chain mode expanded (cm: handed over by k_tail or
// marked here): supervisor edges (:258), into the level kernels' partials (the
// sweep counts traced edges); cm and the pending maps are left zero.
__global__ __launch_bounds__(256) void k_chain_stats(DevGraph g, ChainArgs ca, uint64_t words) {
  uint64_t su = 0;
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t w = (uint64_t)blockIdx.x * 256 + threadIdx.x; w < words; w += stride) {
    uint32_t bits = g.cm[w];
    g.pb[0][w] = 0;
    g.pb[1][w] = 0;
    if (!bits) continue;
    g.cm[w] = 0;
    while (bits) {
      const uint32_t v = (uint32_t)(w * 32 + (__ffs(bits) - 1));
      bits &= bits - 1;
      if ((g.flags[v] & (FL_ALIVE | FL_PROXY | FL_HALTED)) != FL_ALIVE) continue;
      if (!ca.investigate && g.sup[v] < 0xFFFFFFF0u) ++su;
    }
  }
  __shared__ unsigned long long s_su;
  if (threadIdx.x == 0) s_su = 0;
  __syncthreads();
  if (su) atomicAdd(&s_su, (unsigned long long)su);
  __syncthreads();
  if (threadIdx.x == 0) {
    if (s_su) atomicAdd((unsigned long long *)&g.blkstat[STAT_SUP_SLOT], s_su);
  }
}

// The mark is complete: counters as k_tail leaves them after a finished mark.
__global__ void k_chain_done(DevGraph g, ChainArgs ca, uint32_t rounds) {
  Counters *c = g.ctr;
  c->marked += *ca.n_new;
  c->chain_marked += *ca.n_new;
  c->chain_rounds += rounds;
  c->tail_level += rounds;
  c->tail_state = TAIL_DONE;
  c->mark_done = 1;
}

hipError_t launch_chain(const DevGraph &g, const ChainArgs &ca, int step, const uint32_t *src, uint32_t *dst,
                        uint64_t top, uint32_t fi, int first, uint32_t rounds, hipStream_t s) {
  launch_begin();
  const uint64_t words = (top + 31) / 32;
  const int wgrid = grid_for((top + 63) / 64, 4, 4096);
  switch (step) {
    case 0: hipLaunchKernelGGL(k_chain_init, dim3(wgrid), dim3(256), 0, s, g, ca, top); break;
    case 1:
      hipLaunchKernelGGL(k_chain_jump, dim3(grid_for(top, 256, 4096)), dim3(256), 0, s, g, ca, src, dst, top, fi,
                         first);
      break;
    case 2:
      hipLaunchKernelGGL(k_chain_expand, dim3(grid_for((words + 63) / 64, 4, 4096)), dim3(256), 0, s, g, ca, words,
                         fi);
      break;
    case 3: hipLaunchKernelGGL(k_chain_stats, dim3(grid_for(words, 256, 2048)), dim3(256), 0, s, g, ca, words); break;
    default: hipLaunchKernelGGL(k_chain_done, dim3(1), dim3(1), 0, s, g, ca, rounds); break;
  }
  return hipGetLastError();
}

}  // namespace crgc
