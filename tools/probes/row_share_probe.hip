#include <hip/hip_runtime.h>
#include <cstdio>
template <int CTRL>
__global__ void k(int* out) {
  int lane = threadIdx.x;
  out[lane] = __builtin_amdgcn_update_dpp(-1, lane, CTRL, 0xf, 0xf, false);
}
template <int CTRL> int run(const char* name) {
  int* d; hipMalloc(&d, 64 * sizeof(int));
  hipLaunchKernelGGL(k<CTRL>, dim3(1), dim3(64), 0, 0, d);
  int h[64]; hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  printf("%-12s", name);
  for (int i = 0; i < 64; ++i) printf(" %d", h[i]);
  printf("\n");
  hipFree(d);
  return 0;
}
int main() {
  run<0x150>("row_share0"); run<0x153>("row_share3"); run<0x15F>("row_share15");

  return 0;
}
