// crgc_undo.hip — UndoLog folding on the device.
//
// Every DeltaMsg a collector receives is also folded into the sender's
// UndoLog (LocalGC.scala:133; UndoLog.mergeDeltaGraph, UndoLog.java:39-67),
// and every IngressEntry into the log of its egress node (UndoLog.java:69-93).
// A log is `admitted: actor -> (messageCount, createdRefs: target -> count)`;
// here it lives in HBM as two open-addressing tables:
//   ids    actor / target id -> bucket (the bucket index is the slot), with
//          the field's existence (`adm`) and its messageCount
//   pairs  (actor bucket << 32 | target bucket) -> count
// Folds are commutative sums (absent == 0), so one thread per delta shadow /
// ingress field applies its records with atomics; counts that sum to zero
// are dropped at export, which is what updateOutgoing's zero-deletion leaves
// (UndoLog.java:95-104).
#include "crgc_host.hpp"

namespace crgc {

constexpr uint64_t UA_EMPTY = ~0ull;

__device__ inline uint64_t ua_hash(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return k;
}

// Find-or-insert `key` (never UA_EMPTY) in keys[cap]; *ins set on insertion.
__device__ inline uint32_t ua_intern(uint64_t *keys, uint64_t cap, uint64_t key, uint32_t *ins) {
  uint64_t h = ua_hash(key) & (cap - 1);
  for (;;) {
    const uint64_t k = keys[h];
    if (k == key) return (uint32_t)h;
    if (k == UA_EMPTY) {
      const uint64_t prev = atomicCAS((unsigned long long *)&keys[h], (unsigned long long)UA_EMPTY,
                                      (unsigned long long)key);
      if (prev == UA_EMPTY) {
        ++*ins;
        return (uint32_t)h;
      }
      if (prev == key) return (uint32_t)h;
    }
    h = (h + 1) & (cap - 1);
  }
}

__device__ inline void ua_count_inserts(const UndoAccDev &u, uint32_t ids, uint32_t pairs) {
  const uint32_t ti = __shfl(wave_incl_scan(ids), 63), tp = __shfl(wave_incl_scan(pairs), 63);
  if (lane_id() == 0) {
    if (ti) atomicAdd(u.n_ids, (unsigned long long)ti);
    if (tp) atomicAdd(u.n_pairs, (unsigned long long)tp);
  }
}

__device__ inline void ua_add(int32_t *p, int32_t v) { atomicAdd((unsigned int *)p, (unsigned int)v); }

// UndoLog.mergeDeltaGraph over a batch of DeltaGraphs: shadows the sender did
// not intern give back their receive counts and created refs (:43-66).
__global__ __launch_bounds__(256) void k_ua_fold_deltas(UndoAccDev u, UaDeltaArgs a) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  uint32_t ni = 0, np = 0;
  if (i < a.n && !(a.flags[i] & CRGC_DELTA_INTERNED)) {
    const uint32_t ab = ua_intern(u.keys, u.cap, a.id[i], &ni);
    u.adm[ab] = 1;
    ua_add(&u.msg[ab], -a.recv[i]);  // messageCount -= recvCount (:58)
    const uint32_t k0 = a.out_off[i], k1 = min(a.out_off[i + 1], (uint32_t)a.nout);
    for (uint32_t k = k0; k < k1; ++k) {  // createdRefs[target] -= count (:61-65)
      const uint32_t tb = ua_intern(u.keys, u.cap, a.out_target[k], &ni);
      const uint32_t pb = ua_intern(u.pkeys, u.pcap, (uint64_t)ab << 32 | tb, &np);
      ua_add(&u.pcnt[pb], -a.out_count[k]);
    }
  }
  ua_count_inserts(u, ni, np);
}

// UndoLog.mergeIngressEntry: admitted fields added back (:70-89); sign -1
// undoes (tests).
__global__ __launch_bounds__(256) void k_ua_fold_fields(UndoAccDev u, UaFieldArgs a) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  uint32_t ni = 0, np = 0;
  if (i < a.n) {
    const uint32_t ab = ua_intern(u.keys, u.cap, a.actor[i], &ni);
    u.adm[ab] = 1;
    ua_add(&u.msg[ab], a.sign * a.msg[i]);
    const uint32_t k0 = a.c_off[i], k1 = min(a.c_off[i + 1], (uint32_t)a.nc);
    for (uint32_t k = k0; k < k1; ++k) {
      const uint32_t tb = ua_intern(u.keys, u.cap, a.c_target[k], &ni);
      const uint32_t pb = ua_intern(u.pkeys, u.pcap, (uint64_t)ab << 32 | tb, &np);
      ua_add(&u.pcnt[pb], a.sign * a.c_count[k]);
    }
  }
  ua_count_inserts(u, ni, np);
}

hipError_t launch_ua_fold_deltas(const UndoAccDev &u, const UaDeltaArgs &a, hipStream_t s) {
  launch_begin();
  if (a.n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_ua_fold_deltas, dim3((a.n + 255) / 256), dim3(256), 0, s, u, a);
  return hipGetLastError();
}

hipError_t launch_ua_fold_fields(const UndoAccDev &u, const UaFieldArgs &a, hipStream_t s) {
  launch_begin();
  if (a.n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_ua_fold_fields, dim3((a.n + 255) / 256), dim3(256), 0, s, u, a);
  return hipGetLastError();
}

// ---- growth: rehash into larger tables --------------------------------------
__global__ __launch_bounds__(256) void k_ua_init(UndoAccDev u) {
  const uint64_t st = (uint64_t)gridDim.x * 256;
  for (uint64_t b = (uint64_t)blockIdx.x * 256 + threadIdx.x; b < u.cap; b += st) {
    u.keys[b] = UA_EMPTY;
    u.adm[b] = 0;
    u.msg[b] = 0;
  }
  for (uint64_t b = (uint64_t)blockIdx.x * 256 + threadIdx.x; b < u.pcap; b += st) {
    u.pkeys[b] = UA_EMPTY;
    u.pcnt[b] = 0;
  }
}

__global__ __launch_bounds__(256) void k_ua_rehash_ids(UndoAccDev o, UndoAccDev n, uint32_t *map) {
  const uint64_t st = (uint64_t)gridDim.x * 256;
  uint32_t ni = 0;
  for (uint64_t b = (uint64_t)blockIdx.x * 256 + threadIdx.x; b < o.cap; b += st) {
    const uint64_t k = o.keys[b];
    if (k == UA_EMPTY) continue;
    const uint32_t nb = ua_intern(n.keys, n.cap, k, &ni);
    map[b] = nb;
    n.adm[nb] = o.adm[b];
    n.msg[nb] = o.msg[b];
  }
}

__global__ __launch_bounds__(256) void k_ua_rehash_pairs(UndoAccDev o, UndoAccDev n, const uint32_t *map) {
  const uint64_t st = (uint64_t)gridDim.x * 256;
  uint32_t np = 0;
  for (uint64_t b = (uint64_t)blockIdx.x * 256 + threadIdx.x; b < o.pcap; b += st) {
    const uint64_t k = o.pkeys[b];
    if (k == UA_EMPTY) continue;
    const uint64_t a = map ? map[k >> 32] : (k >> 32), t = map ? map[k & 0xFFFFFFFFu] : (k & 0xFFFFFFFFu);
    const uint32_t nb = ua_intern(n.pkeys, n.pcap, a << 32 | t, &np);
    n.pcnt[nb] = o.pcnt[b];
  }
}

hipError_t launch_ua_init(const UndoAccDev &u, hipStream_t s) {
  launch_begin();
  hipLaunchKernelGGL(k_ua_init, dim3(grid_for(std::max(u.cap, u.pcap), 256, 4096)), dim3(256), 0, s, u);
  return hipGetLastError();
}

// ids too (map != null: old id bucket -> new) or pairs only
hipError_t launch_ua_rehash(const UndoAccDev &o, const UndoAccDev &n, uint32_t *map, bool ids, hipStream_t s) {
  launch_begin();
  if (ids)
    hipLaunchKernelGGL(k_ua_rehash_ids, dim3(grid_for(o.cap, 256, 4096)), dim3(256), 0, s, o, n, map);
  hipLaunchKernelGGL(k_ua_rehash_pairs, dim3(grid_for(o.pcap, 256, 4096)), dim3(256), 0, s, o, n,
                     (const uint32_t *)(ids ? map : nullptr));
  return hipGetLastError();
}

// ---- export: the log as a crgc_undo_log -------------------------------------
// Fields in bucket order; each field's created refs with nonzero counts.
__global__ __launch_bounds__(256) void k_ua_prep(UndoAccDev u, UaExportArgs x) {
  const uint64_t st = (uint64_t)gridDim.x * 256;
  for (uint64_t b = (uint64_t)blockIdx.x * 256 + threadIdx.x; b < u.cap; b += st) {
    x.admf[b] = u.adm[b] ? 1u : 0u;
    x.deg[b] = 0;
  }
}

__global__ __launch_bounds__(256) void k_ua_degree(UndoAccDev u, UaExportArgs x) {
  const uint64_t st = (uint64_t)gridDim.x * 256;
  for (uint64_t b = (uint64_t)blockIdx.x * 256 + threadIdx.x; b < u.pcap; b += st) {
    const uint64_t k = u.pkeys[b];
    if (k != UA_EMPTY && u.pcnt[b] != 0) atomicAdd(&x.deg[k >> 32], 1u);
  }
}

__global__ __launch_bounds__(256) void k_ua_fields(UndoAccDev u, UaExportArgs x) {
  const uint64_t st = (uint64_t)gridDim.x * 256;
  for (uint64_t b = (uint64_t)blockIdx.x * 256 + threadIdx.x; b < u.cap; b += st) {
    if (!u.adm[b]) continue;
    const uint64_t i = x.aidx[b];
    x.actor[i] = u.keys[b];
    x.msg[i] = u.msg[b];
    x.c_off[i] = (uint32_t)x.roff[b];
    x.deg[b] = 0;  // reused as the fill cursor
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) x.c_off[*x.n_fields] = (uint32_t)*x.n_created;
}

__global__ __launch_bounds__(256) void k_ua_created(UndoAccDev u, UaExportArgs x) {
  const uint64_t st = (uint64_t)gridDim.x * 256;
  for (uint64_t b = (uint64_t)blockIdx.x * 256 + threadIdx.x; b < u.pcap; b += st) {
    const uint64_t k = u.pkeys[b];
    if (k == UA_EMPTY || u.pcnt[b] == 0) continue;
    const uint64_t a = k >> 32;
    const uint64_t pos = x.roff[a] + atomicAdd(&x.deg[a], 1u);
    x.c_target[pos] = u.keys[k & 0xFFFFFFFFu];
    x.c_count[pos] = u.pcnt[b];
  }
}

hipError_t launch_ua_export(const UndoAccDev &u, const UaExportArgs &x, int phase, hipStream_t s) {
  launch_begin();
  const int gi = grid_for(u.cap, 256, 4096), gp = grid_for(u.pcap, 256, 4096);
  if (phase == 0) {  // counts: admitted fields, created refs per field, and their scans
    hipLaunchKernelGGL(k_ua_prep, dim3(gi), dim3(256), 0, s, u, x);
    hipLaunchKernelGGL(k_ua_degree, dim3(gp), dim3(256), 0, s, u, x);
    ScanSet q{};
    q.in[0] = x.admf;
    q.out[0] = x.aidx;
    q.total[0] = x.n_fields;
    q.in[1] = x.deg;
    q.out[1] = x.roff;
    q.total[1] = x.n_created;
    q.k = 2;
    q.n = u.cap;
    q.bsum = x.bsum;
    return run_scan(q, s);
  }
  hipLaunchKernelGGL(k_ua_fields, dim3(gi), dim3(256), 0, s, u, x);
  hipLaunchKernelGGL(k_ua_created, dim3(gp), dim3(256), 0, s, u, x);
  return hipGetLastError();
}

}  // namespace crgc
