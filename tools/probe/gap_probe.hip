// Launch-gap probe: per-kernel time of N dependent tiny kernels launched on a stream vs replayed from
// a captured hipGraph, for a kernel that does ~nothing and for one that stores a value the next one
// reads (the k-means rounds' pattern). Prints us per kernel.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void tiny(float* p, int i) {
  if (threadIdx.x == 0 && blockIdx.x == 0) p[i & 1023] = p[(i + 1023) & 1023] + 1.f;
}

int main() {
  float* d;
  hipMalloc(&d, 4096 * sizeof(float));
  hipMemset(d, 0, 4096 * sizeof(float));
  hipStream_t s;
  hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int N = 1000;
  for (int grid : {1, 96, 1024}) {
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(a, s);
      for (int i = 0; i < N; ++i) tiny<<<grid, 256, 0, s>>>(d, i);
      hipEventRecord(b, s);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      if (rep) printf("stream  grid=%4d: %.3f us/kernel\n", grid, ms * 1e3 / N);
    }
    hipGraph_t g;
    hipGraphExec_t ge;
    hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
    for (int i = 0; i < N; ++i) tiny<<<grid, 256, 0, s>>>(d, i);
    hipStreamEndCapture(s, &g);
    hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    for (int rep = 0; rep < 3; ++rep) {
      hipEventRecord(a, s);
      hipGraphLaunch(ge, s);
      hipEventRecord(b, s);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      if (rep) printf("graph   grid=%4d: %.3f us/kernel\n", grid, ms * 1e3 / N);
    }
    hipGraphExecDestroy(ge);
    hipGraphDestroy(g);
  }
  return 0;
}
