// Semantics check of the gfx950 cross-lane primitives used by the attention
// kernels (v_permlane16_swap / v_permlane32_swap, DPP row_ror / row_half_mirror /
// quad_perm): prints, per primitive, the source lane every lane ends up holding.
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void k(int* o) {
  const int l = threadIdx.x;
  unsigned x = l, y = 100 + l;
  auto r = __builtin_amdgcn_permlane16_swap(x, y, false, false);
  auto q = __builtin_amdgcn_permlane32_swap(x, y, false, false);
  o[0 * 64 + l] = r[0];
  o[1 * 64 + l] = r[1];
  o[2 * 64 + l] = q[0];
  o[3 * 64 + l] = q[1];
  o[4 * 64 + l] = __builtin_amdgcn_update_dpp(0, l, 0x128, 0xF, 0xF, false);   // row_ror:8
  o[5 * 64 + l] = __builtin_amdgcn_update_dpp(0, l, 0x141, 0xF, 0xF, false);   // row_half_mirror
  o[6 * 64 + l] = __builtin_amdgcn_update_dpp(0, l, 0x4E, 0xF, 0xF, false);    // quad_perm [2,3,0,1]
  o[7 * 64 + l] = __builtin_amdgcn_update_dpp(0, l, 0xB1, 0xF, 0xF, false);    // quad_perm [1,0,3,2]
}

int main() {
  int* d; (void)hipMalloc(&d, 8 * 64 * 4);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  int h[8 * 64];
  (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  const char* names[8] = {"p16swap.vdst", "p16swap.vsrc", "p32swap.vdst", "p32swap.vsrc",
                          "dpp.row_ror8", "dpp.row_half_mirror", "dpp.qp2301", "dpp.qp1032"};
  for (int i = 0; i < 8; ++i) {
    printf("%-20s", names[i]);
    for (int l = 0; l < 64; ++l) printf(" %d", h[i * 64 + l]);
    printf("\n");
  }
  return 0;
}
