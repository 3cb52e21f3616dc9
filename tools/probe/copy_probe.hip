// Copy-bandwidth probe: which streaming-copy shape reaches the highest HBM rate on this box.
// Variants: contiguous chunk per workgroup vs grid-stride, nontemporal vs plain, 16 B x U per lane.
// Prints GB/s (read + write bytes) per variant for a 1 GiB and a 4 GiB buffer.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float v4f __attribute__((ext_vector_type(4)));

template <int U, bool NT>
__global__ __launch_bounds__(256) void chunk_copy(const v4f* __restrict__ src, v4f* __restrict__ dst,
                                                  long n16, long per) {
  const long b0 = (long)blockIdx.x * per;
  const long b1 = b0 + per < n16 ? b0 + per : n16;
  for (long i = b0 + threadIdx.x; i < b1; i += U * 256) {
    v4f v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long j = i + u * 256;
      if (j < b1) v[u] = NT ? __builtin_nontemporal_load(src + j) : src[j];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long j = i + u * 256;
      if (j < b1) {
        if (NT)
          __builtin_nontemporal_store(v[u], dst + j);
        else
          dst[j] = v[u];
      }
    }
  }
}

template <int U, bool NT>
__global__ __launch_bounds__(256) void stride_copy(const v4f* __restrict__ src, v4f* __restrict__ dst,
                                                   long n16) {
  const long step = (long)gridDim.x * 256 * U;
  for (long i = (long)blockIdx.x * 256 * U + threadIdx.x; i < n16; i += step) {
    v4f v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long j = i + u * 256;
      if (j < n16) v[u] = NT ? __builtin_nontemporal_load(src + j) : src[j];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long j = i + u * 256;
      if (j < n16) {
        if (NT)
          __builtin_nontemporal_store(v[u], dst + j);
        else
          dst[j] = v[u];
      }
    }
  }
}

template <class F>
static float timeit(F f) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int r = 0; r < 3; ++r) f();
  hipEventRecord(a);
  for (int r = 0; r < 10; ++r) f();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms / 10;
}

int main() {
  for (size_t bytes : {1ull << 30, 4ull << 30}) {
    v4f *s, *d;
    if (hipMalloc(&s, bytes) != hipSuccess || hipMalloc(&d, bytes) != hipSuccess) return 1;
    hipMemset(s, 1, bytes);
    const long n16 = (long)(bytes / 16);
    auto report = [&](const char* name, float ms) {
      printf("%-34s %5.1f GiB: %7.1f GB/s\n", name, bytes / 1073741824.0, 2.0 * bytes / (ms * 1e-3) / 1e9);
    };
    for (int blocks : {2048, 4096, 16384}) {
      long per = (n16 + blocks - 1) / blocks;
      per = (per + 1023) / 1024 * 1024;
      const unsigned g = (unsigned)((n16 + per - 1) / per);
      char nm[64];
      snprintf(nm, sizeof nm, "chunk U4 NT blocks=%d", blocks);
      report(nm, timeit([&] { chunk_copy<4, true><<<g, 256>>>(s, d, n16, per); }));
      snprintf(nm, sizeof nm, "chunk U4 plain blocks=%d", blocks);
      report(nm, timeit([&] { chunk_copy<4, false><<<g, 256>>>(s, d, n16, per); }));
    }
    for (unsigned g : {1024u, 2048u, 4096u, 8192u}) {
      char nm[64];
      snprintf(nm, sizeof nm, "stride U4 NT grid=%u", g);
      report(nm, timeit([&] { stride_copy<4, true><<<g, 256>>>(s, d, n16); }));
      snprintf(nm, sizeof nm, "stride U4 plain grid=%u", g);
      report(nm, timeit([&] { stride_copy<4, false><<<g, 256>>>(s, d, n16); }));
      snprintf(nm, sizeof nm, "stride U8 plain grid=%u", g);
      report(nm, timeit([&] { stride_copy<8, false><<<g, 256>>>(s, d, n16); }));
      snprintf(nm, sizeof nm, "stride U2 plain grid=%u", g);
      report(nm, timeit([&] { stride_copy<2, false><<<g, 256>>>(s, d, n16); }));
    }
    report("hipMemcpyDtoD", timeit([&] { hipMemcpyAsync(d, s, bytes, hipMemcpyDeviceToDevice, 0); }));
    hipFree(s);
    hipFree(d);
  }
  return 0;
}
