// Prints, for each DPP control, which source lane each destination lane reads.
#include <hip/hip_runtime.h>
#include <cstdio>
template <int CTRL>
__global__ void k(int* out) {
  int lane = threadIdx.x;
  int v = __builtin_amdgcn_update_dpp(-1, lane, CTRL, 0xf, 0xf, false);
  out[lane] = v;
}
template <int CTRL> void run(const char* name) {
  int* d; hipMalloc(&d, 64 * sizeof(int));
  hipLaunchKernelGGL(k<CTRL>, dim3(1), dim3(64), 0, 0, d);
  int h[64]; hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  printf("%-12s", name);
  for (int i : {0, 1, 2, 14, 15, 16, 17, 31, 32, 33, 62, 63}) printf(" %d<-%d", i, h[i]);
  printf("\n");
  hipFree(d);
}
int main() {
  run<0x130>("wave_shl1"); run<0x134>("wave_rol1"); run<0x138>("wave_shr1"); run<0x13C>("wave_ror1");
  run<0x101>("row_shl1"); run<0x111>("row_shr1"); run<0x142>("row_bcast15"); run<0x143>("row_bcast31");
  return 0;
}
