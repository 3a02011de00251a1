// rand_probe.hip — the random-access ceilings the merge kernels are bound by.
//
// The merge (k_ids, k_entries_vertex, k_ep_owner) and the pull levels make
// independent random 4- to 16-B accesses into tables far larger than any
// cache; their bound is the chip's rate of random memory transactions, not
// HBM bytes.  This probe measures that rate on the box for the access forms
// the kernels use (loads, no-return and returning atomics, CAS, stores, a
// dependent pair), over tables of 128 MB (inside the Infinity Cache), 1 GB
// (the C2 id table), 4 GB and 32 GB (the C4 edge table).  Built here (tools/_build/rand_probe), run on
// the GPU box by tools/gpu_r4.sh step `rand`; one line per (form, table).
// Nothing here is product code.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

__device__ inline uint64_t mix(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

constexpr int IN_FLIGHT = 8;

// OP: 0 load 8 B, 1 load 16 B, 2 store 4 B, 3 atomicAdd 8 B (no return),
//     4 atomicAdd 8 B (returned value used), 5 atomicCAS 8 B (returned),
//     6 dependent pair of 8-B loads (the second address from the first value)
template <int OP>
__global__ __launch_bounds__(256) void k_rand(uint64_t *tab, uint64_t mask, uint32_t rounds, uint64_t seed,
                                              uint64_t *sink) {
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t acc = 0;
  for (uint32_t r = 0; r < rounds; ++r) {
    uint64_t idx[IN_FLIGHT];
#pragma unroll
    for (int k = 0; k < IN_FLIGHT; ++k) idx[k] = mix(seed ^ (tid * 0x100000001B3ull + r * IN_FLIGHT + k)) & mask;
    if (OP == 0) {
      uint64_t v[IN_FLIGHT];
#pragma unroll
      for (int k = 0; k < IN_FLIGHT; ++k) v[k] = tab[idx[k]];
#pragma unroll
      for (int k = 0; k < IN_FLIGHT; ++k) acc += v[k];
    } else if (OP == 1) {
      const uint4 *t4 = (const uint4 *)tab;
      uint4 v[IN_FLIGHT];
#pragma unroll
      for (int k = 0; k < IN_FLIGHT; ++k) v[k] = t4[idx[k] >> 1];
#pragma unroll
      for (int k = 0; k < IN_FLIGHT; ++k) acc += v[k].x ^ v[k].w;
    } else if (OP == 2) {
      uint32_t *t32 = (uint32_t *)tab;
#pragma unroll
      for (int k = 0; k < IN_FLIGHT; ++k) t32[idx[k] * 2] = (uint32_t)tid;
    } else if (OP == 3) {
#pragma unroll
      for (int k = 0; k < IN_FLIGHT; ++k) atomicAdd((unsigned long long *)&tab[idx[k]], 1ull);
    } else if (OP == 4) {
      uint64_t v[IN_FLIGHT];
#pragma unroll
      for (int k = 0; k < IN_FLIGHT; ++k) v[k] = atomicAdd((unsigned long long *)&tab[idx[k]], 1ull);
#pragma unroll
      for (int k = 0; k < IN_FLIGHT; ++k) acc += v[k];
    } else if (OP == 5) {
      uint64_t v[IN_FLIGHT];
#pragma unroll
      for (int k = 0; k < IN_FLIGHT; ++k)
        v[k] = atomicCAS((unsigned long long *)&tab[idx[k]], 0xFFFFFFFFFFFFFFFFull, tid);
#pragma unroll
      for (int k = 0; k < IN_FLIGHT; ++k) acc += v[k];
    } else {
      uint64_t v[IN_FLIGHT];
#pragma unroll
      for (int k = 0; k < IN_FLIGHT; ++k) v[k] = tab[idx[k]];
#pragma unroll
      for (int k = 0; k < IN_FLIGHT; ++k) v[k] = tab[(v[k] ^ idx[k]) & mask];
#pragma unroll
      for (int k = 0; k < IN_FLIGHT; ++k) acc += v[k];
    }
  }
  if (acc == 0x5EED5EED5EED5EEDull) sink[0] = acc;  // keeps the loads; never true in practice
}

template <int OP>
static float run(uint64_t *tab, uint64_t entries, uint32_t rounds, uint64_t *sink, hipEvent_t e0, hipEvent_t e1) {
  const int grid = 4096, block = 256;
  hipLaunchKernelGGL(k_rand<OP>, dim3(grid), dim3(block), 0, 0, tab, entries - 1, rounds, 7ull, sink);  // warm
  hipEventRecord(e0, 0);
  hipLaunchKernelGGL(k_rand<OP>, dim3(grid), dim3(block), 0, 0, tab, entries - 1, rounds, 11ull, sink);
  hipEventRecord(e1, 0);
  if (hipEventSynchronize(e1) != hipSuccess) return -1.f;
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  return ms;
}

int main() {
  // 128 MB: inside the Infinity Cache; 1 GB: the C2 id table; 4 GB: the C2
  // edge table; 32 GB: the C4 edge table and pool (TLB reach)
  const uint64_t sizes_mb[4] = {128, 1024, 4096, 32768};
  const uint32_t rounds = 16;
  const double ops = 4096.0 * 256 * rounds * IN_FLIGHT;
  uint64_t *sink = nullptr;
  if (hipMalloc(&sink, 64) != hipSuccess) return 1;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  printf("%-34s %8s %10s %12s %14s\n", "form", "table", "ms", "Gops/s", "GB/s@64B-line");
  for (uint64_t mb : sizes_mb) {
    const uint64_t entries = mb << 17;  // 8-B entries, a power of two
    uint64_t *tab = nullptr;
    if (hipMalloc(&tab, entries * 8) != hipSuccess) return 2;
    if (hipMemset(tab, 0xFF, entries * 8) != hipSuccess) return 3;
    const char *names[7] = {"load 8 B", "load 16 B", "store 4 B", "atomicAdd 8 B (no return)",
                            "atomicAdd 8 B (returned)", "atomicCAS 8 B (returned)", "dependent pair of 8-B loads"};
    float ms[7];
    ms[0] = run<0>(tab, entries, rounds, sink, e0, e1);
    ms[1] = run<1>(tab, entries, rounds, sink, e0, e1);
    ms[2] = run<2>(tab, entries, rounds, sink, e0, e1);
    if (hipMemset(tab, 0, entries * 8) != hipSuccess) return 3;
    ms[3] = run<3>(tab, entries, rounds, sink, e0, e1);
    ms[4] = run<4>(tab, entries, rounds, sink, e0, e1);
    if (hipMemset(tab, 0xFF, entries * 8) != hipSuccess) return 3;
    ms[5] = run<5>(tab, entries, rounds, sink, e0, e1);
    if (hipMemset(tab, 0, entries * 8) != hipSuccess) return 3;
    ms[6] = run<6>(tab, entries, rounds, sink, e0, e1);
    for (int k = 0; k < 7; ++k) {
      const double n = ops * (k == 6 ? 2 : 1);
      printf("%-34s %6lluMB %10.3f %12.2f %14.1f\n", names[k], (unsigned long long)mb, ms[k], n / (ms[k] * 1e6),
             n * 64 / (ms[k] * 1e6));
    }
    hipFree(tab);
  }
  const hipError_t e = hipGetLastError();
  printf("status: %s\n", hipGetErrorName(e));
  return e == hipSuccess ? 0 : 4;
}
