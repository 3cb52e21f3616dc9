// Instruction-fetch probe: a long straight-line VALU body (no memory ops) run 3 times inside one
// launch; per-pass s_memrealtime ticks (10 ns). Pass 1 pays for cold instruction fetch.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int N>
__global__ void body(float* out, float s, unsigned long long* t) {
  float a = s + threadIdx.x, b = s * 2.f, c = s * 3.f, d = s * 4.f;
  unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (int p = 0; p < 3; ++p) {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      a = __builtin_fmaf(a, 1.0001f, b);
      b = __builtin_fmaf(b, 0.9999f, c);
      c = __builtin_fmaf(c, 1.0002f, d);
      d = __builtin_fmaf(d, 0.9998f, a);
    }
    asm volatile("" ::: "memory");
    unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0 && blockIdx.x == 0) t[p] = t1 - t0;
    t0 = t1;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a + b + c + d;
}

int main() {
  float* out;
  unsigned long long* t;
  hipMalloc(&out, 1 << 20);
  hipMalloc(&t, 64);
  unsigned long long h[3];
  for (int rep = 0; rep < 3; ++rep) {
    body<1024><<<8, 1024>>>(out, 1.f, t);
    hipMemcpy(h, t, 24, hipMemcpyDeviceToHost);
    printf("4096 fma body (~32 KB code), 8 WG x 1024: passes %.2f %.2f %.2f us\n", h[0] * .01, h[1] * .01, h[2] * .01);
    body<256><<<8, 1024>>>(out, 1.f, t);
    hipMemcpy(h, t, 24, hipMemcpyDeviceToHost);
    printf("1024 fma body (~8 KB code),  8 WG x 1024: passes %.2f %.2f %.2f us\n", h[0] * .01, h[1] * .01, h[2] * .01);
    body<256><<<8, 64>>>(out, 1.f, t);
    hipMemcpy(h, t, 24, hipMemcpyDeviceToHost);
    printf("1024 fma body (~8 KB code),  8 WG x 64:   passes %.2f %.2f %.2f us\n", h[0] * .01, h[1] * .01, h[2] * .01);
  }
  return 0;
}
