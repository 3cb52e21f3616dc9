// CU-mask probe: (1) which XCDs (HW_REG_XCC_ID) run the workgroups of a stream created with
// hipExtStreamCreateWithCUMask for a few masks (is "CUs 0..31" one XCD, or CU i on XCD i % 8?);
// (2) a chain of dependent small kernels, each reading the 32 KB its predecessor wrote (the
// MiniBatch step's pattern: a few dozen workgroups, tiny hand-offs through memory), on the default
// stream vs a one-XCD masked stream: us per kernel. Prints to stdout.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>
#include <cstring>
#include <vector>

__global__ void where(int* out) {
  if (threadIdx.x == 0) {
    const unsigned v = __builtin_amdgcn_s_getreg((20) | (0 << 6) | ((16 - 1) << 11));
    out[blockIdx.x] = (int)(v & 0xf);
  }
}

// 32 workgroups: each reads its 1 KB slice of `in` (written by the previous kernel), adds, writes out
__global__ void hop(const float* __restrict__ in, float* __restrict__ out, int i) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  float v = in[t];
  // a dependent second trip: an index read from what the predecessor wrote
  const int j = ((int)v + t * 7) & 8191;
  out[t] = v + in[j] * 0.5f + (float)i;
}

static void xcd_hist(hipStream_t s, const char* name) {
  int* d;
  hipMalloc(&d, sizeof(int) * 256);
  where<<<256, 64, 0, s>>>(d);
  hipStreamSynchronize(s);
  std::vector<int> h(256);
  hipMemcpy(h.data(), d, sizeof(int) * 256, hipMemcpyDeviceToHost);
  int hist[16] = {};
  for (int x : h) hist[x & 15]++;
  printf("%-28s XCD histogram of 256 blocks:", name);
  for (int x = 0; x < 8; ++x) printf(" %d", hist[x]);
  printf("\n");
  hipFree(d);
}

static float chain(hipStream_t s, float* a, float* b, int N) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int i = 0; i < 50; ++i) hop<<<32, 256, 0, s>>>(i & 1 ? b : a, i & 1 ? a : b, i);
  hipEventRecord(e0, s);
  for (int i = 0; i < N; ++i) hop<<<32, 256, 0, s>>>(i & 1 ? b : a, i & 1 ? a : b, i);
  hipEventRecord(e1, s);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  return ms * 1e3f / N;
}

int main() {
  int dev = 0;
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, dev);
  printf("CUs: %d\n", p.multiProcessorCount);
  const int ncu = p.multiProcessorCount;
  const int words = (ncu + 31) / 32;
  hipStream_t def;
  hipStreamCreateWithFlags(&def, hipStreamNonBlocking);
  xcd_hist(def, "unmasked");
  struct M {
    const char* name;
    std::vector<uint32_t> m;
  };
  std::vector<M> masks;
  {
    std::vector<uint32_t> m(words, 0);
    m[0] = 0xffffffffu;  // CUs 0..31
    masks.push_back({"CUs 0..31", m});
  }
  {
    std::vector<uint32_t> m(words, 0);
    for (int c = 0; c < ncu; c += 8) m[c / 32] |= 1u << (c % 32);  // CU i with i % 8 == 0
    masks.push_back({"CUs 0,8,16,...", m});
  }
  {
    std::vector<uint32_t> m(words, 0);
    for (int c = 0; c < 8; ++c) m[0] |= 1u << c;  // CUs 0..7
    masks.push_back({"CUs 0..7", m});
  }
  float *a, *b;
  hipMalloc(&a, sizeof(float) * 8192);
  hipMalloc(&b, sizeof(float) * 8192);
  hipMemset(a, 0, sizeof(float) * 8192);
  hipMemset(b, 0, sizeof(float) * 8192);
  printf("chain of dependent 32-workgroup kernels, default stream: %.3f us/kernel\n", chain(def, a, b, 2000));
  for (auto& mk : masks) {
    hipStream_t s;
    if (hipExtStreamCreateWithCUMask(&s, (uint32_t)mk.m.size(), mk.m.data()) != hipSuccess) {
      printf("%s: hipExtStreamCreateWithCUMask failed\n", mk.name);
      continue;
    }
    xcd_hist(s, mk.name);
    printf("chain on %-20s: %.3f us/kernel\n", mk.name, chain(s, a, b, 2000));
    hipStreamDestroy(s);
  }
  printf("chain of dependent 32-workgroup kernels, default stream: %.3f us/kernel\n", chain(def, a, b, 2000));
  return 0;
}
