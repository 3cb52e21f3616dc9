// Latency probe: dependent single-lane loads at the start of a kernel, after a writer kernel.
// Reports s_memrealtime ticks (10 ns) per load for several address patterns.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void writer(float* buf, size_t n) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i < n; i += (size_t)gridDim.x * blockDim.x) buf[i] = (float)(i & 7);
}

// offsets in floats; each load's address depends on the previous value (which is 0..7 -> *0)
__global__ void probe(const float* buf, const long* offs, int m, unsigned long long* out) {
  if (threadIdx.x != 0) return;
  long dep = 0;
  unsigned long long t = __builtin_amdgcn_s_memrealtime();
  for (int q = 0; q < m; ++q) {
    float v = buf[offs[q] + dep];
    dep = (long)(v * 0.0f);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    unsigned long long t2 = __builtin_amdgcn_s_memrealtime();
    out[q] = t2 - t;
    t = t2;
  }
}

int main() {
  const size_t n = 64ull << 20;  // 256 MB of floats
  float* buf;
  hipMalloc(&buf, n * 4);
  std::vector<long> offs;
  // same line x4, +64 B, +4 KB, +64 KB, +2 MB, +32 MB, back to first
  long pat[] = {0, 0, 0, 16, 1024, 1024 + 16, 16384, 524288, 524288 + 1024, 8388608, 0, 16384};
  for (long p : pat) offs.push_back(p);
  long* d_offs;
  hipMalloc(&d_offs, offs.size() * sizeof(long));
  hipMemcpy(d_offs, offs.data(), offs.size() * sizeof(long), hipMemcpyHostToDevice);
  unsigned long long* d_out;
  hipMalloc(&d_out, 64 * 8);
  std::vector<unsigned long long> h(offs.size());
  for (int rep = 0; rep < 4; ++rep) {
    writer<<<1024, 256>>>(buf, n);
    probe<<<1, 64>>>(buf, d_offs, (int)offs.size(), d_out);
    hipMemcpy(h.data(), d_out, offs.size() * 8, hipMemcpyDeviceToHost);
    printf("after writer rep %d:", rep);
    for (size_t q = 0; q < offs.size(); ++q) printf(" %lld:%.2fus", (long long)offs[q], h[q] * 0.01);
    printf("\n");
    probe<<<1, 64>>>(buf, d_offs, (int)offs.size(), d_out);
    hipMemcpy(h.data(), d_out, offs.size() * 8, hipMemcpyDeviceToHost);
    printf("probe again     %d:", rep);
    for (size_t q = 0; q < offs.size(); ++q) printf(" %lld:%.2fus", (long long)offs[q], h[q] * 0.01);
    printf("\n");
  }
  return 0;
}
