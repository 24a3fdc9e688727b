// Semantics probe for v_permlane16_swap_b32 / v_permlane32_swap_b32 (gfx950):
// prints, for the 4x4 row transpose used by the engine, which (register, row)
// each output row came from.  Expect s_j row a == S[a] row j.
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void k(unsigned* out) {
  const unsigned l = threadIdx.x;
  unsigned s[4];
  for (int i = 0; i < 4; ++i) s[i] = i * 1000 + l;  // register i, lane l
  auto r0 = __builtin_amdgcn_permlane32_swap(s[0], s[2], false, false);
  auto r1 = __builtin_amdgcn_permlane32_swap(s[1], s[3], false, false);
  s[0] = r0[0]; s[2] = r0[1]; s[1] = r1[0]; s[3] = r1[1];
  auto q0 = __builtin_amdgcn_permlane16_swap(s[0], s[1], false, false);
  auto q1 = __builtin_amdgcn_permlane16_swap(s[2], s[3], false, false);
  s[0] = q0[0]; s[1] = q0[1]; s[2] = q1[0]; s[3] = q1[1];
  for (int i = 0; i < 4; ++i) out[i * 64 + l] = s[i];
}
int main() {
  unsigned* d; hipMalloc(&d, 4 * 64 * 4);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  unsigned h[256]; hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  int bad = 0;
  for (int j = 0; j < 4; ++j)
    for (int l = 0; l < 64; ++l) {
      const unsigned a = l >> 4, b = l & 15, want = a * 1000 + (j * 16 + b);
      if (h[j * 64 + l] != want) { if (bad < 8) printf("s%d lane %d: got %u want %u\n", j, l, h[j * 64 + l], want); ++bad; }
    }
  printf("permlane transpose: %s (%d mismatches)\n", bad ? "FAIL" : "OK", bad);
  for (int j = 0; j < 4; ++j) printf("s%d lanes 0,16,32,48: %u %u %u %u\n", j, h[j*64], h[j*64+16], h[j*64+32], h[j*64+48]);
  return 0;
}
