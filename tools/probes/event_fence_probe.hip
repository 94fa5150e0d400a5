// event_fence_probe.hip — what the timing events and the stream wait add to
// the wall time of one launch shaped like the bench's timed HMC call (1024
// blocks x 256 threads, ~85 us of dependent FMAs per thread, 21 MB of
// samples written as [chain][transition][coordinate]): host wall time
// (steady_clock) around record + launch + record + wait, and the events'
// elapsed time, for event flags default / hipEventDisableSystemFence /
// hipEventReleaseToDevice and for no events at all. Variants interleave
// (round robin), after 50 ms of warm-up launches; median of 200 each. After
// the fence-free variant a blocking D2H copy checks that the samples are
// visible to the host.
//   hipcc --offload-arch=gfx950 -O3 -o bin/event_fence_probe event_fence_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

constexpr int CH = 4096, DIM = 64, NT = 20;

__global__ void work_kernel(float* out, int iters, float seed) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const int c = t / DIM, d = t % DIM;
  float x = seed + (float)d * 1e-3f, y = 1.0f;
  for (int n = 0; n < NT; ++n) {
    for (int i = 0; i < iters; ++i) x = __builtin_fmaf(x, 0.999999f, 1e-7f);
    y = x + (float)n;
    out[((long long)c * NT + n) * DIM + d] = y;
  }
}

int main(int argc, char** argv) {
  hipSetDevice(0);
  hipSetDeviceFlags(hipDeviceScheduleSpin);
  const int iters = argc > 1 ? atoi(argv[1]) : 400;
  float* d;
  const size_t n = (size_t)CH * NT * DIM;
  if (hipMalloc(&d, n * 4) != hipSuccess) return 1;
  hipStream_t st;
  hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  hipEvent_t ev[3][2];
  const unsigned flags[3] = {0u, hipEventDisableSystemFence, hipEventReleaseToDevice};
  for (int k = 0; k < 3; ++k)
    for (int j = 0; j < 2; ++j)
      if (hipEventCreateWithFlags(&ev[k][j], flags[k]) != hipSuccess) {
        printf("{\"error\": \"event flags %u refused\"}\n", flags[k]);
        return 2;
      }
  const dim3 grid(CH * DIM / 256), block(256);
  auto t_end = std::chrono::steady_clock::now() + std::chrono::milliseconds(50);
  while (std::chrono::steady_clock::now() < t_end) hipLaunchKernelGGL(work_kernel, grid, block, 0, st, d, iters, 1.0f);
  hipStreamSynchronize(st);
  // variants: 0..2 events of that kind + stream wait, 3 no events + stream
  // wait, 4 default events + hipEventSynchronize(stop)
  constexpr int NV = 5;
  std::vector<double> wall[NV], evt[NV];
  for (int r = 0; r < 200; ++r) {
    for (int v = 0; v < NV; ++v) {
      const int k = v == 4 ? 0 : v;
      const auto t0 = std::chrono::steady_clock::now();
      if (v != 3) hipEventRecord(ev[k][0], st);
      hipLaunchKernelGGL(work_kernel, grid, block, 0, st, d, iters, (float)r);
      if (v != 3) hipEventRecord(ev[k][1], st);
      if (v == 4) hipEventSynchronize(ev[k][1]);
      else hipStreamSynchronize(st);
      const auto t1 = std::chrono::steady_clock::now();
      wall[v].push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
      if (v != 3) {
        float ms = 0.f;
        hipEventElapsedTime(&ms, ev[k][0], ev[k][1]);
        evt[v].push_back(ms * 1e3);
      }
    }
  }
  // visibility after a fence-free pair: the host reads the last launch's values
  hipEventRecord(ev[1][0], st);
  hipLaunchKernelGGL(work_kernel, grid, block, 0, st, d, iters, 7.0f);
  hipEventRecord(ev[1][1], st);
  hipStreamSynchronize(st);
  std::vector<float> h(n);
  hipMemcpy(h.data(), d, n * 4, hipMemcpyDeviceToHost);
  std::vector<float> chk(DIM * NT);
  hipLaunchKernelGGL(work_kernel, grid, block, 0, st, d, iters, 7.0f);
  hipStreamSynchronize(st);
  std::vector<float> h2(n);
  hipMemcpy(h2.data(), d, n * 4, hipMemcpyDeviceToHost);
  long long diff = 0;
  for (size_t i = 0; i < n; ++i) diff += h[i] != h2[i];
  auto med = [](std::vector<double> v) {
    if (v.empty()) return -1.0;
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
  };
  const char* names[NV] = {"default_events", "events_disable_system_fence", "events_release_to_device", "no_events",
                           "default_events_event_sync"};
  printf("{\"iters\": %d", iters);
  for (int v = 0; v < NV; ++v)
    printf(", \"%s\": {\"wall_us\": %.2f, \"event_us\": %.2f, \"wall_min_us\": %.2f}", names[v], med(wall[v]),
           med(evt[v]), *std::min_element(wall[v].begin(), wall[v].end()));
  printf(", \"fence_free_then_copy_mismatches\": %lld}\n", diff);
  return 0;
}
