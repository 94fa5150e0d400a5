// empty_launch_probe.hip — the floor of a launch's event-timed duration on
// this box: an empty kernel at the HMC bench's grid (256 blocks x 256
// threads), and one that only loads and stores 1 MiB (the bench's state),
// HIP events around each launch, median of 50.
//   hipcc --offload-arch=gfx950 -O3 -o bin/empty_launch_probe empty_launch_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

__global__ void empty_kernel(float* p) {
  if (p == nullptr && threadIdx.x == 1023) p[0] = 0.0f;  // never true: keeps the launch
}
__global__ void copy_kernel(float* p) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  p[i] = p[i] * 1.0001f;
}

int main() {
  float* d;
  if (hipMalloc(&d, 1 << 20) != hipSuccess) return 1;
  hipMemset(d, 0, 1 << 20);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipStream_t st;
  hipStreamCreate(&st);
  auto run = [&](int which) {
    std::vector<float> t;
    for (int r = 0; r < 60; ++r) {
      hipEventRecord(a, st);
      if (which == 0) hipLaunchKernelGGL(empty_kernel, dim3(256), dim3(256), 0, st, d);
      else hipLaunchKernelGGL(copy_kernel, dim3(1024), dim3(256), 0, st, d);
      hipEventRecord(b, st);
      hipStreamSynchronize(st);
      float ms = 0;
      hipEventElapsedTime(&ms, a, b);
      if (r >= 10) t.push_back(ms * 1000.0f);
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
  };
  const float e = run(0), c = run(1);
  printf("{\"empty_kernel_event_us\": %.2f, \"load_store_1MiB_event_us\": %.2f}\n", e, c);
  return 0;
}
