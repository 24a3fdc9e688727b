// Diagnostics for the cross-lane / byte-permute primitives used by the engine.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
extern "C" __global__ void prim_kernel(uint32_t* out) {
  const int lane = threadIdx.x;
  const uint32_t v = 0x1000u + lane;
  out[0 * 64 + lane] = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, true);
  out[1 * 64 + lane] = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, true);
  out[2 * 64 + lane] = (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x101F);
  out[3 * 64 + lane] = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x128, 0xF, 0xF, true);
  out[4 * 64 + lane] = (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x401F);
  out[5 * 64 + lane] = (uint32_t)__shfl_xor((int)v, 32);
  const uint32_t x = 0xA1B2C3D4u;
  const uint32_t lb = (1u << 16) | 0x80u | ((uint32_t)(lane & 31) << 2);
  out[6 * 64 + lane] = __builtin_amdgcn_perm(x, lb, 0x0C020400u);
  out[7 * 64 + lane] = __builtin_amdgcn_perm(x, lb, 0x0C020700u);
  out[8 * 64 + lane] = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x130, 0xF, 0xF, true);  // wave_shl:1
  out[9 * 64 + lane] = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x134, 0xF, 0xF, true);  // wave_rol:1
  out[10 * 64 + lane] = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x138, 0xF, 0xF, true); // wave_shr:1
  out[11 * 64 + lane] = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x13C, 0xF, 0xF, true); // wave_ror:1
}
int main() {
  uint32_t* d; hipMalloc(&d, 12 * 64 * 4);
  hipLaunchKernelGGL(prim_kernel, dim3(1), dim3(64), 0, 0, d);
  uint32_t h[12 * 64]; hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  const char* names[] = {"dpp_xor1", "dpp_xor2", "swz_xor4", "dpp_ror8", "swz_xor16", "shfl_xor32", "perm_b0", "perm_b3"};
  for (int r = 0; r < 8; ++r) {
    int bad = 0;
    for (int l = 0; l < 64; ++l) {
      uint32_t want;
      int x[] = {1, 2, 4, 8, 16, 32};
      if (r < 6) want = 0x1000u + (l ^ x[r]);
      else if (r == 6) want = (1u << 16) | (0xD4u << 8) | (0x80u | ((l & 31) << 2));
      else want = (1u << 16) | (0xA1u << 8) | (0x80u | ((l & 31) << 2));
      if (h[r * 64 + l] != want) bad++;
    }
    printf("%-10s %s   lanes0-7:", names[r], bad ? "MISMATCH" : "ok");
    for (int l = 0; l < 8; ++l) printf(" %x", h[r * 64 + l]);
    printf("  lanes 16,32,48: %x %x %x\n", h[r*64+16], h[r*64+32], h[r*64+48]);
  }
  const char* n2[] = {"wave_shl1", "wave_rol1", "wave_shr1", "wave_ror1"};
  for (int r = 8; r < 12; ++r) {
    printf("%-10s lanes0-3: %x %x %x %x  lane62,63: %x %x\n", n2[r - 8], h[r*64], h[r*64+1], h[r*64+2], h[r*64+3], h[r*64+62], h[r*64+63]);
  }
  return 0;
}
