// crgc_vertex.hip — the vertex half of a merge: receive-count deltas and the
// last-write-wins fields (isBusy / isRoot / interned / isLocal, supervisor) of
// every record, as atoms partitioned by slot and reduced per slot in LDS.
//
// ShadowGraph.mergeEntry / mergeDelta (ShadowGraph.java:75-156) apply a batch's
// records one by one; every write is a sum (recvCount, Java int wraparound) or
// a last write (the flags, the supervisor).  Here a record's vertex effects are
// atoms {slot, seq | kind, recv delta, value}: `seq` is the record's position
// in the call (1-based), VX_FLAGS carries the flag bits the record sets,
// VX_SUP a supervisor slot.  One workgroup per slot bucket reduces its atoms
// 1024 at a time in an LDS table (sums by LDS atomicAdd, winners by LDS 64-bit
// atomicMax of seq << 8 | flags and seq << 32 | supervisor) and writes each
// slot once with plain stores — the workgroup owns every atom of its slots.
// Winners of different rounds, and of earlier merge calls, are ordered by the
// per-slot tags vseq / sseq (epoch << 32 | seq), read and written by that same
// workgroup: no device-scope atomics anywhere.
#include "crgc_host.hpp"

namespace crgc {

constexpr int VX_THREADS = 256;  // partition kernels
constexpr int VX_WG = 1024;      // bucket kernel
constexpr uint32_t VX_CH = 1024;
constexpr uint32_t VX_TAB = 2048;

__device__ inline uint32_t vx_bucket(const VxArgs &a, uint32_t slot) { return (slot * 0x9E3779B1u) >> a.bshift; }

__device__ inline uint64_t vx_count(const VxArgs &a) { return a.n_dev ? min(*a.n_dev, a.max_atoms) : a.max_atoms; }

__device__ inline bool vx_valid(uint32_t slot) { return slot < 0xFFFFFFF0u; }

__global__ __launch_bounds__(VX_THREADS) void k_vx_count(VxArgs a) {
  extern __shared__ uint32_t hist[];
  const uint64_t n = vx_count(a);
  for (uint32_t k = threadIdx.x; k < a.nbk; k += VX_THREADS) hist[k] = 0;
  __syncthreads();
  const uint64_t per = (n + a.nblk - 1) / a.nblk;
  const uint64_t i0 = (uint64_t)blockIdx.x * per, i1 = min(n, i0 + per);
  for (uint64_t i = i0 + threadIdx.x; i < i1; i += VX_THREADS) {
    const uint32_t s = a.atoms[i].x;
    if (vx_valid(s)) atomicAdd(&hist[vx_bucket(a, s)], 1u);
  }
  __syncthreads();
  for (uint32_t k = threadIdx.x; k < a.nbk; k += VX_THREADS) a.hist[(uint64_t)k * a.nblk + blockIdx.x] = hist[k];
}

__global__ __launch_bounds__(VX_THREADS) void k_vx_scatter(VxArgs a) {
  extern __shared__ uint32_t cur[];
  const uint64_t n = vx_count(a);
  for (uint32_t k = threadIdx.x; k < a.nbk; k += VX_THREADS) cur[k] = 0;
  __syncthreads();
  const uint64_t per = (n + a.nblk - 1) / a.nblk;
  const uint64_t i0 = (uint64_t)blockIdx.x * per, i1 = min(n, i0 + per);
  for (uint64_t i = i0 + threadIdx.x; i < i1; i += VX_THREADS) {
    const uint4 v = a.atoms[i];
    if (!vx_valid(v.x)) continue;
    const uint32_t b = vx_bucket(a, v.x);
    a.part[a.hoff[(uint64_t)b * a.nblk + blockIdx.x] + atomicAdd(&cur[b], 1u)] = v;
  }
}

struct VxLds {
  uint64_t ftag[VX_TAB];  // seq << 8 | flag bits of the round's last flag record (0: none)
  uint64_t stag[VX_TAB];  // seq << 32 | supervisor slot of the round's last supervisor record
  uint32_t key[VX_TAB];   // slot (~0: free)
  int32_t recv[VX_TAB];
  uint32_t plist[VX_CH];
  uint32_t np;
};

__global__ __launch_bounds__(VX_WG) void k_vx_apply(DevGraph g, VxArgs a) {
  __shared__ VxLds L;
  const uint32_t b = blockIdx.x, tid = threadIdx.x;
  const uint64_t a0 = a.hoff[(uint64_t)b * a.nblk];
  const uint64_t a1 = b + 1 == a.nbk ? *a.tot : a.hoff[(uint64_t)(b + 1) * a.nblk];
  if (a0 == a1) return;
  const uint64_t top = g.ctr->slot_top;
  for (uint32_t k = tid; k < VX_TAB; k += VX_WG) {
    L.key[k] = 0xFFFFFFFFu;
    L.recv[k] = 0;
    L.ftag[k] = 0;
    L.stag[k] = 0;
  }
  const unsigned long long ep = a.epoch << 32;
  for (uint64_t c0 = a0; c0 < a1; c0 += VX_CH) {
    const uint32_t m = (uint32_t)min((uint64_t)VX_CH, a1 - c0);
    if (tid == 0) L.np = 0;
    __syncthreads();
    if (tid < m) {
      const uint4 v = a.part[c0 + tid];
      uint32_t h = (uint32_t)mix64(v.x) & (VX_TAB - 1);
      for (;;) {
        const uint32_t k = atomicCAS(&L.key[h], 0xFFFFFFFFu, v.x);
        if (k == 0xFFFFFFFFu) L.plist[atomicAdd(&L.np, 1u)] = h;
        if (k == 0xFFFFFFFFu || k == v.x) break;
        h = (h + 1) & (VX_TAB - 1);
      }
      const uint32_t seq = v.y & VX_SEQ;
      if (v.z) atomicAdd(&L.recv[h], (int32_t)v.z);
      if (v.y & VX_FLAGS)
        atomicMax((unsigned long long *)&L.ftag[h], ((unsigned long long)seq << 8) | (v.w & 0xFFu));
      if (v.y & VX_SUP) atomicMax((unsigned long long *)&L.stag[h], ((unsigned long long)seq << 32) | v.w);
    }
    __syncthreads();
    const uint32_t np = L.np;
    if (tid < np) {
      const uint32_t h = L.plist[tid];
      const uint32_t s = L.key[h];
      if (s < top) {  // (slots come from k_ids; malformed batches are reported, never followed)
        if (const int32_t d = L.recv[h]) g.recv[s] = (int32_t)((uint32_t)g.recv[s] + (uint32_t)d);
        if (const unsigned long long f = L.ftag[h]) {
          const unsigned long long tag = ep | (f >> 8);
          if (tag > g.vseq[s]) {
            g.vseq[s] = tag;
            g.flags[s] = (uint8_t)((g.flags[s] & (uint8_t)~(FL_BUSY | FL_ROOT)) | (uint8_t)(f & 0xFFu));
          }
        }
        if (const unsigned long long sp = L.stag[h]) {
          const unsigned long long tag = ep | (sp >> 32);
          if (tag > g.sseq[s]) {
            g.sseq[s] = tag;
            g.sup[s] = (uint32_t)sp;
          }
        }
      }
      L.key[h] = 0xFFFFFFFFu;
      L.recv[h] = 0;
      L.ftag[h] = 0;
      L.stag[h] = 0;
    }
    __syncthreads();
  }
}

hipError_t launch_vertex(const DevGraph &g, const VxArgs &a, hipStream_t s) {
  if (a.max_atoms == 0) return hipSuccess;
  const size_t lds = (size_t)a.nbk * 4;
  ScanSet q{};
  q.k = 1;
  q.n = (uint64_t)a.nbk * a.nblk;
  q.in[0] = a.hist;
  q.out[0] = a.hoff;
  q.total[0] = a.tot;
  q.bsum = a.bsum;
  hipLaunchKernelGGL(k_vx_count, dim3((unsigned)a.nblk), dim3(VX_THREADS), lds, s, a);
  if (hipError_t e = run_scan(q, s)) return e;
  hipLaunchKernelGGL(k_vx_scatter, dim3((unsigned)a.nblk), dim3(VX_THREADS), lds, s, a);
  hipLaunchKernelGGL(k_vx_apply, dim3(a.nbk), dim3(VX_WG), 0, s, g, a);
  return hipGetLastError();
}

}  // namespace crgc
