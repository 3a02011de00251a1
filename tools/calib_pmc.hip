// calib_pmc.hip — TOOLING: calibrates rocprofv3 FETCH_SIZE / WRITE_SIZE on
// MI355X (gfx950) for the access shapes of the trace kernels, on known byte
// counts (VERDICT r1 "What's weak" 2a: the x2 correction of MI355X_MICROARCH.md
// holds for 16-B/lane streaming reads only).
//
//   stream16      16-B/lane coalesced reads            (the guide's calibrated case)
//   stream8_nt    8-B/lane non-temporal reads          (k_expand's edge stream)
//   rand1_mall    random 1-B reads of a 16 MiB map     (candidate bytes; MALL-resident)
//   rand1_hbm     random 1-B reads of a 1 GiB map      (beyond the Infinity Cache)
//   rmw1_mall     random 1-B read, store if zero       (k_expand's candidate RMW)
//   rand4_l2      random 4-B reads of a 1.6 MiB bitmap (marked-word probes; L2-resident)
//   store16       16-B/lane coalesced stores           (WRITE_SIZE reference)
//
// Each kernel runs twice (a warm-up launch, then the measured one); the program
// prints one JSON line per measured launch: algorithmic bytes, accesses and
// time (HIP events).  profiles/calib_summary.py joins it with the counter CSVs.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

__device__ inline uint32_t mixh(uint64_t x) {
  x ^= x >> 30;
  x *= 0xbf58476d1ce4e5b9ull;
  x ^= x >> 27;
  x *= 0x94d049bb133111ebull;
  x ^= x >> 31;
  return (uint32_t)x;
}

__global__ void k_stream16(const uint4 *p, uint64_t n, uint32_t *out) {
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
    const uint4 v = p[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

__global__ void k_stream8_nt(const uint64_t *p, uint64_t n, uint32_t *out) {
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
    const uint64_t v = __builtin_nontemporal_load(p + i);
    acc ^= (uint32_t)v ^ (uint32_t)(v >> 32);
  }
  if (acc == 0x12345678u) out[0] = acc;
}

// 4 independent random reads per lane per step (k_expand issues U = 4)
__global__ void k_rand1(const uint8_t *tab, uint64_t mask, uint64_t n, uint32_t *out) {
  uint32_t acc = 0;
  for (uint64_t i = (blockIdx.x * 256ull + threadIdx.x) * 4; i < n; i += (uint64_t)gridDim.x * 1024) {
    uint8_t b[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) b[u] = tab[mixh(i + u) & mask];
#pragma unroll
    for (int u = 0; u < 4; ++u) acc += b[u];
  }
  if (acc == 0x12345678u) out[0] = acc;
}

__global__ void k_rmw1(uint8_t *tab, uint64_t mask, uint64_t n) {
  for (uint64_t i = (blockIdx.x * 256ull + threadIdx.x) * 4; i < n; i += (uint64_t)gridDim.x * 1024) {
    uint64_t a[4];
    uint8_t b[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      a[u] = mixh(i + u) & mask;
      b[u] = tab[a[u]];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (b[u] == 0) tab[a[u]] = 1;
  }
}

__global__ void k_rand4(const uint32_t *tab, uint64_t mask, uint64_t n, uint32_t *out) {
  uint32_t acc = 0;
  for (uint64_t i = (blockIdx.x * 256ull + threadIdx.x) * 4; i < n; i += (uint64_t)gridDim.x * 1024) {
    uint32_t b[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) b[u] = tab[mixh(i + u) & mask];
#pragma unroll
    for (int u = 0; u < 4; ++u) acc ^= b[u];
  }
  if (acc == 0x12345678u) out[0] = acc;
}

__global__ void k_store16(uint4 *p, uint64_t n) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256)
    p[i] = make_uint4((uint32_t)i, 1, 2, 3);
}

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
      return 1;                                                            \
    }                                                                      \
  } while (0)

int main() {
  const uint64_t GB = 1ull << 30, MAP_MALL = 16ull << 20, BM_L2 = 1664ull << 10;  // 1.6 MiB
  const uint64_t N_RAND = 16ull << 20;                                             // random accesses
  void *big = nullptr, *mall = nullptr, *l2 = nullptr;
  uint32_t *out = nullptr;
  CK(hipMalloc(&big, GB));
  CK(hipMalloc(&mall, MAP_MALL));
  CK(hipMalloc(&l2, 2ull << 20));
  CK(hipMalloc(&out, 64));
  CK(hipMemset(big, 1, GB));
  CK(hipMemset(mall, 0, MAP_MALL));
  CK(hipMemset(l2, 0, 2ull << 20));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int grid = 2048;
  auto run = [&](const char *name, uint64_t bytes, uint64_t accesses, auto launch) -> int {
    for (int rep = 0; rep < 2; ++rep) {
      if (rep == 1) CK(hipEventRecord(e0));
      launch();
      CK(hipGetLastError());
      if (rep == 1) CK(hipEventRecord(e1));
      CK(hipDeviceSynchronize());
    }
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("{\"kernel\": \"%s\", \"algorithmic_bytes\": %llu, \"accesses\": %llu, \"ms\": %.4f}\n", name,
           (unsigned long long)bytes, (unsigned long long)accesses, ms);
    return 0;
  };
  int rc = 0;
  rc |= run("k_stream16", GB, GB / 16, [&] { hipLaunchKernelGGL(k_stream16, dim3(grid), dim3(256), 0, 0, (const uint4 *)big, GB / 16, out); });
  rc |= run("k_stream8_nt", GB, GB / 8, [&] { hipLaunchKernelGGL(k_stream8_nt, dim3(grid), dim3(256), 0, 0, (const uint64_t *)big, GB / 8, out); });
  rc |= run("k_rand1<mall>", N_RAND, N_RAND, [&] { hipLaunchKernelGGL(k_rand1, dim3(grid), dim3(256), 0, 0, (const uint8_t *)mall, MAP_MALL - 1, N_RAND, out); });
  rc |= run("k_rand1<hbm>", N_RAND, N_RAND, [&] { hipLaunchKernelGGL(k_rand1, dim3(grid), dim3(256), 0, 0, (const uint8_t *)big, GB - 1, N_RAND, out); });
  rc |= run("k_rmw1", 2 * N_RAND, N_RAND, [&] { hipLaunchKernelGGL(k_rmw1, dim3(grid), dim3(256), 0, 0, (uint8_t *)mall, MAP_MALL - 1, N_RAND); });
  rc |= run("k_rand4", 4 * N_RAND, N_RAND, [&] { hipLaunchKernelGGL(k_rand4, dim3(grid), dim3(256), 0, 0, (const uint32_t *)l2, (BM_L2 / 4) - 1 > 0 ? (1ull << 18) - 1 : 0, N_RAND, out); });
  rc |= run("k_store16", GB, GB / 16, [&] { hipLaunchKernelGGL(k_store16, dim3(grid), dim3(256), 0, 0, (uint4 *)big, GB / 16); });
  hipFree(big);
  hipFree(mall);
  hipFree(l2);
  hipFree(out);
  return rc;
}
