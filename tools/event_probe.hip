// event_probe.hip — what a timing event costs between back-to-back kernels on
// one stream (the C2 kernel trace shows ~5 us of idle GPU before and after
// every launch that carries start / stop events, none between untimed ones:
// profiles/r5an).  Not product code: it prices the ways a level kernel can be
// timed, so the trace keeps the cheapest form the bench's roofline allows.
//
// Each case launches K short streaming kernels (~256 workgroups) back to back
// and reports the wall per launch from one event pair around all of them:
//   plain        no events
//   ext-events   hipExtLaunchKernelGGL carrying start / stop events (the product's form)
//   ext-start    the start event only in the dispatch
//   record       hipEventRecord before and after each launch
//   record-1     hipEventRecord after each launch only (the previous stop is the next start)
//   *-fence      the same with events created without hipEventDisableSystemFence
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cstdio>
#include <vector>

__global__ __launch_bounds__(256) void k_stream(const uint4 *a, uint4 *b, size_t n) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) b[i] = a[i];
}

static float wall(hipEvent_t a, hipEvent_t b) {
  float t = 0;
  (void)hipEventElapsedTime(&t, a, b);
  return t;
}

int main() {
  hipStream_t s;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return 1;
  const size_t n = (8u << 20) / 16;  // 8 MB per kernel: ~3 us of streaming
  uint4 *a = nullptr, *b = nullptr;
  if (hipMalloc(&a, n * 16) != hipSuccess || hipMalloc(&b, n * 16) != hipSuccess) return 1;
  (void)hipMemset(a, 1, n * 16);
  const int K = 200;
  hipEvent_t t0, t1;
  (void)hipEventCreate(&t0);
  (void)hipEventCreate(&t1);
  for (int fence = 0; fence < 2; ++fence) {
    std::vector<hipEvent_t> ev(2 * K + 2);
    for (auto &e : ev) (void)hipEventCreateWithFlags(&e, fence ? hipEventDefault : hipEventDisableSystemFence);
    for (int mode = 0; mode < 5; ++mode) {
      if (fence && mode == 0) continue;
      float best = 1e30f, kern = 0;
      for (int rep = 0; rep < 5; ++rep) {
        (void)hipEventRecord(t0, s);
        for (int k = 0; k < K; ++k) {
          switch (mode) {
            case 0: hipExtLaunchKernelGGL(k_stream, dim3(256), dim3(256), 0, s, nullptr, nullptr, 0, a, b, n); break;
            case 1: hipExtLaunchKernelGGL(k_stream, dim3(256), dim3(256), 0, s, ev[2 * k], ev[2 * k + 1], 0, a, b, n); break;
            case 2: hipExtLaunchKernelGGL(k_stream, dim3(256), dim3(256), 0, s, ev[2 * k], nullptr, 0, a, b, n); break;
            case 3:
              (void)hipEventRecord(ev[2 * k], s);
              hipLaunchKernelGGL(k_stream, dim3(256), dim3(256), 0, s, a, b, n);
              (void)hipEventRecord(ev[2 * k + 1], s);
              break;
            case 4:
              if (k == 0) (void)hipEventRecord(ev[0], s);
              hipLaunchKernelGGL(k_stream, dim3(256), dim3(256), 0, s, a, b, n);
              (void)hipEventRecord(ev[k + 1], s);
              break;
          }
        }
        (void)hipEventRecord(t1, s);
        (void)hipStreamSynchronize(s);
        const float w = wall(t0, t1);
        if (w < best) {
          best = w;
          kern = 0;
          if (mode == 1 || mode == 3)
            for (int k = 0; k < K; ++k) kern += wall(ev[2 * k], ev[2 * k + 1]);
          if (mode == 4)
            for (int k = 0; k < K; ++k) kern += wall(ev[k], ev[k + 1]);
        }
      }
      static const char *names[] = {"plain", "ext-events", "ext-start", "record", "record-1"};
      printf("%-12s%-6s %7.2f us per launch; timed kernel avg %6.2f us\n", names[mode], fence ? "-fence" : "",
             best * 1e3 / K, kern * 1e3 / K);
    }
    for (auto &e : ev) (void)hipEventDestroy(e);
  }
  printf("last error: %s\n", hipGetErrorName(hipGetLastError()));
  return 0;
}
