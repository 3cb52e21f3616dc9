// XCD placement probe: which XCD (HW_REG_XCC_ID) runs each workgroup of a 1-D grid, and for a 2-D
// grid. Prints the first 32 block -> XCD assignments and the histogram of (block % 8) vs XCD.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void where(int* out) {
  if (threadIdx.x == 0) {
    // HW_REG_XCC_ID: hwRegId 20, offset 0, size 16 -> simm16 = id | (offset << 6) | ((size-1) << 11)
    const unsigned v = __builtin_amdgcn_s_getreg((20) | (0 << 6) | ((16 - 1) << 11));
    out[blockIdx.y * gridDim.x + blockIdx.x] = (int)(v & 0xf);
  }
}

int main() {
  for (int nb : {2048, 40000}) {
    int* d;
    hipMalloc(&d, sizeof(int) * nb);
    where<<<nb, 256>>>(d);
    std::vector<int> h(nb);
    hipMemcpy(h.data(), d, sizeof(int) * nb, hipMemcpyDeviceToHost);
    printf("grid %d: first 32:", nb);
    for (int i = 0; i < 32; ++i) printf(" %d", h[i]);
    int match = 0;
    for (int i = 0; i < nb; ++i) match += h[i] == (i % 8);
    int hist[8][8] = {};
    for (int i = 0; i < nb; ++i) hist[i % 8][h[i] & 7]++;
    printf("\n  blocks with xcd == b %% 8: %d of %d\n", match, nb);
    for (int r = 0; r < 8; ++r) {
      printf("  b%%8=%d:", r);
      for (int c = 0; c < 8; ++c) printf(" %6d", hist[r][c]);
      printf("\n");
    }
    hipFree(d);
  }
  return 0;
}
