// crgc_route.hip — an entry batch cut into per-shard parts (hash-partitioned
// graphs).
//
// Every record of an Entry is applied by the home shard of the shadow it
// writes (self; edge owner; spawned child; updated target) and names the far
// end of an edge or supervisor, which that shard resolves as a proxy (the
// filter of k_ids, crgc_merge.hip).  Instead of all-gathering every shard's
// batch (each shard then reading G batches to apply about 2/G of them), a
// shard cuts its batch into one part per destination: the entry's self and
// flags plus exactly the records that destination resolves.  The parts travel
// in one all-to-all; a destination concatenates what it receives in shard
// order and merges it as one batch.  The records of one shadow only ever meet
// at its home, in (shard, entry) order either way, so every last-write-wins
// outcome is the all-gathered form's.
//   k_route_count    per block of entries and destination: entries, created,
//                    spawned, updated records (packed 4 x 16 bits)
//   k_route_scan     per destination: exclusive prefixes over the blocks, totals
//   k_route_scatter  every entry's part for each destination it concerns
//   k_concat         receiver: the received parts as one batch, offsets rebased
#include "crgc_host.hpp"

namespace crgc {

__device__ inline uint32_t rt_hi(uint32_t x, uint64_t bound) { return (uint64_t)x > bound ? (uint32_t)bound : x; }

// Record ranges of entry i, clamped to the batch and to F records; `bad`
// reports offsets the merge kernels would reject (the sender's error word).
struct Ranges {
  uint32_t c0, c1, s0, s1, u0, u1;
  bool bad;
};

__device__ inline Ranges route_ranges(const RouteArgs &a, uint64_t i) {
  Ranges r;
  const uint32_t c0 = a.c_off[i], c1 = a.c_off[i + 1], s0 = a.s_off[i], s1 = a.s_off[i + 1];
  const uint32_t u0 = a.u_off[i], u1 = a.u_off[i + 1];
  r.bad = c1 < c0 || s1 < s0 || u1 < u0 || c1 > a.C || s1 > a.S || u1 > a.U || c1 - c0 > a.F ||
          s1 - s0 > a.F || u1 - u0 > a.F;
  r.c1 = rt_hi(c1, a.C);
  r.c0 = min(c0, r.c1);
  r.c1 = min(r.c1, r.c0 + a.F);
  r.s1 = rt_hi(s1, a.S);
  r.s0 = min(s0, r.s1);
  r.s1 = min(r.s1, r.s0 + a.F);
  r.u1 = rt_hi(u1, a.U);
  r.u0 = min(u0, r.u1);
  r.u1 = min(r.u1, r.u0 + a.F);
  return r;
}

// This thread's column of per-destination parts (sp[d * RT_THREADS]), packed
// present | created << 16 | spawned << 32 | updated << 48.
__device__ inline void route_fill(const RouteArgs &a, uint64_t i, const Ranges &r, uint64_t *sp) {
  const uint32_t G = a.G;
  for (uint32_t d = 0; d < G; ++d) sp[d * RT_THREADS] = 0;
  const uint32_t me = shard_of(a.self[i], G);
  sp[me * RT_THREADS] = 1;
  for (uint32_t k = r.c0; k < r.c1; ++k) {  // owner's home applies, target's home ensures
    const uint32_t o = shard_of(a.c_owner[k], G), t = shard_of(a.c_target[k], G);
    sp[o * RT_THREADS] += 1ull << 16;
    if (t != o) sp[t * RT_THREADS] += 1ull << 16;
  }
  for (uint32_t k = r.s0; k < r.s1; ++k) sp[shard_of(a.spawned[k], G) * RT_THREADS] += 1ull << 32;
  for (uint32_t k = r.u0; k < r.u1; ++k) {  // target's home; self's home for a deactivation
    const uint32_t h = shard_of(a.u_ref[k], G);
    sp[h * RT_THREADS] += 1ull << 48;
    if (refob_deactivated(a.u_info[k]) && h != me) sp[me * RT_THREADS] += 1ull << 48;
  }
  for (uint32_t d = 0; d < G; ++d)
    if (sp[d * RT_THREADS] >> 16) sp[d * RT_THREADS] |= 1;
}

__global__ __launch_bounds__(RT_THREADS) void k_route_count(RouteArgs a) {
  __shared__ uint64_t s_part[ROUTE_MAX_SHARDS * RT_THREADS];
  const uint64_t i = (uint64_t)blockIdx.x * RT_THREADS + threadIdx.x;
  uint64_t *sp = s_part + threadIdx.x;
  if (i < a.n) {
    const Ranges r = route_ranges(a, i);
    if (r.bad) atomicOr(a.err, 1ull);
    route_fill(a, i, r, sp);
  } else {
    for (uint32_t d = 0; d < a.G; ++d) sp[d * RT_THREADS] = 0;
  }
  __syncthreads();
  if (threadIdx.x < a.G) {  // fields stay below 2^16: <= 256 entries x F <= 255 records
    uint64_t s = 0;
    for (int t = 0; t < RT_THREADS; ++t) s += s_part[threadIdx.x * RT_THREADS + t];
    a.blk_tot[(uint64_t)threadIdx.x * a.nblk + blockIdx.x] = s;
  }
}

// One workgroup per destination: exclusive prefixes of the four counts over
// the blocks, and the destination's totals.  A thread takes RS_K consecutive
// blocks, so a C2 wakeup's ~3 900 blocks are one pass of 1024 threads (a
// 256-thread loop over them was 16 dependent rounds, 25 us: profiles/r6o).
constexpr int RS_THREADS = 1024, RS_K = 4;
__global__ __launch_bounds__(RS_THREADS) void k_route_scan(RouteArgs a) {
  __shared__ uint32_t s_w[RS_THREADS / 64][4];
  __shared__ uint64_t s_carry[4];
  const uint32_t d = blockIdx.x;
  const int lane = lane_id(), wv = threadIdx.x >> 6;
  if (threadIdx.x < 4) s_carry[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t *bt = a.blk_tot + (uint64_t)d * a.nblk;
  uint64_t *bp = a.blk_pre + (uint64_t)d * a.nblk * 4;
  for (uint64_t b0 = 0; b0 < a.nblk; b0 += (uint64_t)RS_THREADS * RS_K) {
    const uint64_t b = b0 + (uint64_t)threadIdx.x * RS_K;
    uint64_t p[RS_K];
#pragma unroll
    for (int k = 0; k < RS_K; ++k) p[k] = b + k < a.nblk ? bt[b + k] : 0ull;
    uint32_t f[4] = {0, 0, 0, 0}, inc[4];  // (a pass's sums stay below 4096 x 2^16)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
#pragma unroll
      for (int k = 0; k < RS_K; ++k) f[q] += (uint32_t)((p[k] >> (16 * q)) & 0xFFFFu);
      inc[q] = wave_incl_scan(f[q]);
    }
    if (lane == 63)
      for (int q = 0; q < 4; ++q) s_w[wv][q] = inc[q];
    __syncthreads();
    uint64_t pre[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      pre[q] = s_carry[q] + inc[q] - f[q];
      for (int w = 0; w < wv; ++w) pre[q] += s_w[w][q];
    }
#pragma unroll
    for (int k = 0; k < RS_K; ++k) {
      if (b + k >= a.nblk) break;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        bp[(b + k) * 4 + q] = pre[q];
        pre[q] += (p[k] >> (16 * q)) & 0xFFFFu;
      }
    }
    __syncthreads();
    if (threadIdx.x < 4) {
      uint64_t t = 0;
      for (int w = 0; w < RS_THREADS / 64; ++w) t += s_w[w][threadIdx.x];
      s_carry[threadIdx.x] += t;
    }
    __syncthreads();
  }
  if (threadIdx.x < 4) a.totals[d * 4 + threadIdx.x] = s_carry[threadIdx.x];
}

__global__ __launch_bounds__(RT_THREADS) void k_route_scatter(RouteArgs a, const RoutePart *parts) {
  __shared__ uint64_t s_part[ROUTE_MAX_SHARDS * RT_THREADS];
  __shared__ uint32_t s_w[4][2];
  const uint32_t G = a.G;
  const uint64_t i = (uint64_t)blockIdx.x * RT_THREADS + threadIdx.x;
  const bool valid = i < a.n;
  uint64_t *sp = s_part + threadIdx.x;
  Ranges r{};
  if (valid) {
    r = route_ranges(a, i);
    route_fill(a, i, r, sp);
  } else {
    for (uint32_t d = 0; d < G; ++d) sp[d * RT_THREADS] = 0;
  }
  const uint32_t me = valid ? shard_of(a.self[i], G) : 0;
  const int lane = lane_id(), wv = threadIdx.x >> 6;
  for (uint32_t d = 0; d < G; ++d) {
    // intra-block exclusive prefix of this destination's packed counts (two
    // 32-bit halves: every field of a block's sum stays below 2^16)
    const uint64_t v = sp[d * RT_THREADS];
    const uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
    const uint32_t ilo = wave_incl_scan(lo), ihi = wave_incl_scan(hi);
    if (lane == 63) {
      s_w[wv][0] = ilo;
      s_w[wv][1] = ihi;
    }
    __syncthreads();
    uint32_t plo = 0, phi = 0;
    for (int w = 0; w < wv; ++w) {
      plo += s_w[w][0];
      phi += s_w[w][1];
    }
    __syncthreads();
    if (!(v & 1)) continue;
    const uint32_t xlo = plo + ilo - lo, xhi = phi + ihi - hi;
    const uint64_t *pre = a.blk_pre + ((uint64_t)d * a.nblk + blockIdx.x) * 4;
    const uint64_t pos = pre[0] + (xlo & 0xFFFFu), cb = pre[1] + (xlo >> 16);
    const uint64_t sb = pre[2] + (xhi & 0xFFFFu), ub = pre[3] + (xhi >> 16);
    const RoutePart P = parts[d];
    P.self[pos] = a.self[i];
    P.recv[pos] = a.recv[i];
    P.flags[pos] = a.flags[i];
    P.c_off[pos] = (uint32_t)cb;
    P.s_off[pos] = (uint32_t)sb;
    P.u_off[pos] = (uint32_t)ub;
    uint64_t j = cb;
    for (uint32_t k = r.c0; k < r.c1; ++k) {
      const uint64_t o = a.c_owner[k], t = a.c_target[k];
      if (shard_of(o, G) == d || shard_of(t, G) == d) {
        P.c_owner[j] = o;
        P.c_target[j] = t;
        ++j;
      }
    }
    j = sb;
    for (uint32_t k = r.s0; k < r.s1; ++k)
      if (shard_of(a.spawned[k], G) == d) P.spawned[j++] = a.spawned[k];
    j = ub;
    for (uint32_t k = r.u0; k < r.u1; ++k) {
      const int16_t info = a.u_info[k];
      if (shard_of(a.u_ref[k], G) == d || (refob_deactivated(info) && me == d)) {
        P.u_ref[j] = a.u_ref[k];
        P.u_info[j] = info;
        ++j;
      }
    }
  }
  if (blockIdx.x == 0 && threadIdx.x < G) {  // closing offsets of every part
    const RoutePart P = parts[threadIdx.x];
    const uint64_t *t = a.totals + (uint64_t)threadIdx.x * 4;
    if (t[0]) {
      P.c_off[t[0]] = (uint32_t)t[1];
      P.s_off[t[0]] = (uint32_t)t[2];
      P.u_off[t[0]] = (uint32_t)t[3];
    }
  }
}

hipError_t launch_route(const RouteArgs &a, int phase, const RoutePart *parts, hipStream_t s) {
  launch_begin();
  if (a.n == 0) return hipSuccess;
  const int blocks = (int)a.nblk;
  if (phase == 0) {
    hipLaunchKernelGGL(k_route_count, dim3(blocks), dim3(RT_THREADS), 0, s, a);
    hipLaunchKernelGGL(k_route_scan, dim3(a.G), dim3(RS_THREADS), 0, s, a);
  } else {
    hipLaunchKernelGGL(k_route_scatter, dim3(blocks), dim3(RT_THREADS), 0, s, a, parts);
  }
  return hipGetLastError();
}

// Receiver: the parts (in shard order) as one batch with rebased offsets.
__global__ __launch_bounds__(256) void k_concat(const ConcatPart *parts, uint32_t G, RoutePart dst, uint64_t N,
                                                uint64_t Ct, uint64_t St, uint64_t Ut) {
  __shared__ ConcatPart P[ROUTE_MAX_SHARDS];
  {
    const uint64_t *src = reinterpret_cast<const uint64_t *>(parts);
    uint64_t *d = reinterpret_cast<uint64_t *>(P);
    for (uint32_t k = threadIdx.x; k < G * (sizeof(ConcatPart) / 8); k += 256) d[k] = src[k];
  }
  __syncthreads();
  const uint64_t stride = (uint64_t)gridDim.x * 256, t0 = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  for (uint64_t j = t0; j < N; j += stride) {
    uint32_t r = 0;
    while (r + 1 < G && P[r + 1].pn <= j) ++r;
    const ConcatPart &p = P[r];
    const uint64_t li = j - p.pn;
    dst.self[j] = reinterpret_cast<const uint64_t *>(p.base + p.off[0])[li];
    dst.recv[j] = reinterpret_cast<const int16_t *>(p.base + p.off[1])[li];
    dst.flags[j] = reinterpret_cast<const uint8_t *>(p.base + p.off[2])[li];
    dst.c_off[j] = reinterpret_cast<const uint32_t *>(p.base + p.off[3])[li] + (uint32_t)p.pC;
    dst.s_off[j] = reinterpret_cast<const uint32_t *>(p.base + p.off[6])[li] + (uint32_t)p.pS;
    dst.u_off[j] = reinterpret_cast<const uint32_t *>(p.base + p.off[8])[li] + (uint32_t)p.pU;
  }
  if (t0 == 0) {
    dst.c_off[N] = (uint32_t)Ct;
    dst.s_off[N] = (uint32_t)St;
    dst.u_off[N] = (uint32_t)Ut;
  }
  for (uint64_t j = t0; j < Ct; j += stride) {
    uint32_t r = 0;
    while (r + 1 < G && P[r + 1].pC <= j) ++r;
    const ConcatPart &p = P[r];
    const uint64_t li = j - p.pC;
    dst.c_owner[j] = reinterpret_cast<const uint64_t *>(p.base + p.off[4])[li];
    dst.c_target[j] = reinterpret_cast<const uint64_t *>(p.base + p.off[5])[li];
  }
  for (uint64_t j = t0; j < St; j += stride) {
    uint32_t r = 0;
    while (r + 1 < G && P[r + 1].pS <= j) ++r;
    const ConcatPart &p = P[r];
    dst.spawned[j] = reinterpret_cast<const uint64_t *>(p.base + p.off[7])[j - p.pS];
  }
  for (uint64_t j = t0; j < Ut; j += stride) {
    uint32_t r = 0;
    while (r + 1 < G && P[r + 1].pU <= j) ++r;
    const ConcatPart &p = P[r];
    const uint64_t li = j - p.pU;
    dst.u_ref[j] = reinterpret_cast<const uint64_t *>(p.base + p.off[9])[li];
    dst.u_info[j] = reinterpret_cast<const int16_t *>(p.base + p.off[10])[li];
  }
}

hipError_t launch_concat(const ConcatPart *parts, uint32_t G, const RoutePart &dst, uint64_t N, uint64_t C,
                         uint64_t S, uint64_t U, hipStream_t s) {
  launch_begin();
  const uint64_t work = std::max(std::max(N, C), std::max(S, U));
  hipLaunchKernelGGL(k_concat, dim3(grid_for(work, 256, 4096)), dim3(256), 0, s, parts, G, dst, N, C, S, U);
  return hipGetLastError();
}

}  // namespace crgc
