#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void k(unsigned* out) {
  unsigned l = threadIdx.x;
  unsigned x = 100 + l;
  out[0*64+l] = __builtin_amdgcn_mov_dpp((int)x, 0x121, 0xF, 0xF, true); // row_ror:1
  out[1*64+l] = __builtin_amdgcn_mov_dpp((int)x, 0x113, 0xF, 0xF, true); // row_shr:3
  out[2*64+l] = __builtin_amdgcn_mov_dpp((int)x, 0x102, 0xF, 0xF, true); // row_shl:2
  out[3*64+l] = __builtin_amdgcn_mov_dpp((int)x, 0x155, 0xF, 0xF, true); // row_share:5
  auto s16 = __builtin_amdgcn_permlane16_swap(x, x + 1000, false, false);
  out[4*64+l] = s16[0]; out[5*64+l] = s16[1];
  auto s32 = __builtin_amdgcn_permlane32_swap(x, x + 1000, false, false);
  out[6*64+l] = s32[0]; out[7*64+l] = s32[1];
}
int main() {
  unsigned* d; hipMalloc(&d, 8*64*4);
  k<<<1,64>>>(d);
  unsigned h[8*64]; hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
  const char* nm[8] = {"ror1","shr3","shl2","share5","p16a","p16b","p32a","p32b"};
  for (int r = 0; r < 8; r++) { printf("%s:", nm[r]); for (int l = 0; l < 64; l++) printf(" %u", h[r*64+l]); printf("\n"); }
  return 0;
}
