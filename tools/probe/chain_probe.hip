// Dependent-add latency probe: one fp32 add chain per lane, 1024 adds, at several active-lane counts,
// operands from registers and from LDS (ds_read_b128 batches). Reports shader clocks per add.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void chain_reg(int active, float* out, long long* clk) {
  float acc = threadIdx.x, x0 = 1.0001f, x1 = 0.9999f;
  long long t0 = 0, t1 = 0;
  if ((int)threadIdx.x < active) {
    t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 64
    for (int i = 0; i < 1024; ++i) acc = acc + ((i & 1) ? x0 : x1);
    t1 = __builtin_amdgcn_s_memtime();
  }
  out[threadIdx.x] = acc;
  if (threadIdx.x == 0) clk[0] = t1 - t0;
}

__global__ void chain_lds(int active, float* out, long long* clk) {
  __shared__ float s[8 * 1092];
  for (int e = threadIdx.x; e < 8 * 1092; e += blockDim.x) s[e] = 1e-3f * (e & 15);
  __syncthreads();
  float acc = 0.f;
  long long t0 = 0, t1 = 0;
  const int lane = threadIdx.x;
  if (lane < active) {
    const float* p = s + (lane & 7) * 1092;
    t0 = __builtin_amdgcn_s_memtime();
    clk[2] = __builtin_amdgcn_s_memrealtime();
    for (int m = 0; m < 1024; m += 64) {
      float4 v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) v[u] = *reinterpret_cast<const float4*>(p + m + 4 * u);
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        acc = acc + v[u].x;
        acc = acc + v[u].y;
        acc = acc + v[u].z;
        acc = acc + v[u].w;
      }
    }
    t1 = __builtin_amdgcn_s_memtime();
    clk[3] = __builtin_amdgcn_s_memrealtime();
  }
  out[threadIdx.x] = acc;
  if (threadIdx.x == 0) clk[0] = t1 - t0;
}

int main() {
  float* out;
  long long* clk;
  hipMalloc(&out, 4096 * 4);
  hipMalloc(&clk, 64);
  long long h;
  for (int active : {1, 8, 64}) {
    for (int rep = 0; rep < 2; ++rep) {
      chain_reg<<<1, 64>>>(active, out, clk);
      hipMemcpy(&h, clk, 8, hipMemcpyDeviceToHost);
      printf("reg chain, %2d lanes: %.2f clk/add   ", active, h / 1024.0);
      chain_lds<<<1, 64>>>(active, out, clk);
      hipMemcpy(&h, clk, 8, hipMemcpyDeviceToHost);
      printf("lds chain: %.2f clk/add\n", h / 1024.0);
    }
  }
  chain_lds<<<1, 1024>>>(8, out, clk);
  long long hh[4];
  hipMemcpy(hh, clk, 32, hipMemcpyDeviceToHost);
  printf("lds chain in a 1024-thread block (other waves idle): %.2f clk/add, %.2f us for 1024 adds\n",
         hh[0] / 1024.0, (hh[3] - hh[2]) * 0.01);
  return 0;
}
