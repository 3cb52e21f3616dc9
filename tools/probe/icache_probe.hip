// Instruction-fetch probe: a straight-line body of N dependent-free VALU ops (no memory ops), run
// twice back to back inside one launch on a fresh CU; pass 1 pays for cold instruction fetch.
// Timestamps are pinned by data dependencies (s_memrealtime, 10 ns ticks).
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ __forceinline__ unsigned long long stamp(float dep) {
  unsigned long long t;
  asm volatile("s_memrealtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t) : "v"(dep) : "memory");
  return t;
}

template <int N>
__global__ void body(float* out, float s, unsigned long long* t) {
  float a = s + threadIdx.x, b = s * 2.f, c = s * 3.f, d = s * 4.f;
  unsigned long long ts[3];
  ts[0] = stamp(a);
  for (int p = 0; p < 2; ++p) {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      a = __builtin_fmaf(a, 1.0001f, 0.5f);
      b = __builtin_fmaf(b, 0.9999f, 0.25f);
      c = __builtin_fmaf(c, 1.0002f, 0.125f);
      d = __builtin_fmaf(d, 0.9998f, 0.0625f);
    }
    ts[p + 1] = stamp(a + b + c + d);
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a + b + c + d;
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    t[0] = ts[1] - ts[0];
    t[1] = ts[2] - ts[1];
  }
}

int main() {
  float* out;
  unsigned long long* t;
  hipMalloc(&out, 1 << 22);
  hipMalloc(&t, 64);
  unsigned long long h[2];
  for (int rep = 0; rep < 3; ++rep) {
    body<2048><<<8, 256>>>(out, 1.f, t);
    hipMemcpy(h, t, 16, hipMemcpyDeviceToHost);
    printf("8192 VALU ops (~64 KB code): pass1 %.2f us  pass2 %.2f us\n", h[0] * .01, h[1] * .01);
    body<512><<<8, 256>>>(out, 1.f, t);
    hipMemcpy(h, t, 16, hipMemcpyDeviceToHost);
    printf("2048 VALU ops (~16 KB code): pass1 %.2f us  pass2 %.2f us\n", h[0] * .01, h[1] * .01);
    body<128><<<8, 256>>>(out, 1.f, t);
    hipMemcpy(h, t, 16, hipMemcpyDeviceToHost);
    printf(" 512 VALU ops  (~4 KB code): pass1 %.2f us  pass2 %.2f us\n", h[0] * .01, h[1] * .01);
  }
  return 0;
}
