// What v_mov_b32_dpp row_newbcast:n returns on gfx950 (a row-broadcast attempt
// failed parity).  One wave: lane l holds 100 + l; prints each lane's result for n = 0, 1, 5.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(int* out) {
  const int l = threadIdx.x, v = 100 + l;
  out[0 * 64 + l] = __builtin_amdgcn_update_dpp(0, v, 0x150 | 0, 0xf, 0xf, false);
  out[1 * 64 + l] = __builtin_amdgcn_update_dpp(0, v, 0x150 | 1, 0xf, 0xf, false);
  out[2 * 64 + l] = __builtin_amdgcn_update_dpp(0, v, 0x150 | 5, 0xf, 0xf, false);
  out[3 * 64 + l] = __builtin_amdgcn_update_dpp(-1, v, 0x150 | 1, 0xf, 0xf, true);
}
int main() {
  int* d;
  hipMalloc(&d, 4 * 64 * sizeof(int));
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  int h[256];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  for (int r = 0; r < 4; ++r) {
    printf("case %d:", r);
    for (int l = 0; l < 64; ++l) printf(" %d", h[r * 64 + l]);
    printf("\n");
  }
  hipFree(d);
  return 0;
}
