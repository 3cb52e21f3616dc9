// gdd_bf16.hip — the bf16 full labels pass (predict(precision="bf16"); SURVEY §8(d) config 5: "fp32
// vs bf16 MFMA distance kernel"), r06 form. Its own translation unit: it is built with
// -mllvm -amdgpu-mfma-vgpr-form (Makefile), so the MFMA accumulators live in VGPRs and the epilogue
// reads them without v_accvgpr_read copies; the fp32 kernels of gdd_kmeans.hip keep the default.
//
// HBM design point: X is read once (460 MB at 2.45M x 47: ~58 us at 8 TB/s). The r03 kernel
// (gdd_kmeans.hip k_assign_bf16p, GDD_FORCE=bf16_v1) ran at 0.36 of that roof; its counters
// (rocprofv3, profiles/r06_bf16_pmc.json) put the limit in the VALU: ~925 vector instructions per
// 32-point tile, each 4 cycles of its SIMD (SQ_ACTIVE_INST_VALU = SQ_INSTS_VALU quad-cycles). Here:
//   * a tile's 32 x dim floats are ONE contiguous span of X, copied into the wave's LDS slot as is
//     (float4 stores, row stride dim: no index arithmetic); B-fragments read row r's features
//     16 st + 8 h .. + 7 straight from it (two ds_read_b128 when dim % 4 == 0, else eight
//     ds_read_b32), features past dim masked to zero;
//   * the argmin runs on integer keys. The first free K slot (feature dim; the pass needs
//     dim % 16 != 0) carries -||x||^2 / 2 in the B-fragment and 1.0 in every centre's A-fragment,
//     so the chain yields x.c - ||x||^2 / 2 and fma(-2, acc, ||c||^2) is the squared distance,
//     non-negative up to rounding: its float bits order as signed integers. The centre's in-tile
//     index goes into the 5 low significand bits (one v_and_or_b32), the lane's 16 keys reduce by
//     v_min3_i32, one compare per centre tile — per centre an fma and an and_or, where the r03
//     epilogue spent an fma, a compare and two selects (plus a copy out of the accumulator).
// Accuracy: the labels are those of bf16 dot products (tests/test_gpu_kmeans.py and
// tests/test_gpu_configs.py bound every label that differs from the exact fp32 one by the bf16
// rounding, 2^-7 ||x|| ||c|| per product). The shift by ||x||^2 is the same for every centre of a
// point, so its own bf16 rounding cannot reorder them; dropping 5 of the 24 significand bits moves a
// distance by < 2^-18 of itself; keys that tie may pick either centre, and a distance that rounds
// below zero (a point on a centre) is a negative key, i.e. a winner, as it should be.
#include <algorithm>
#include <type_traits>

#include "gdd_common.hpp"

namespace gdd {
namespace {

using floatx16 = __attribute__((ext_vector_type(16))) float;
typedef float floatx4_t __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));

inline size_t frag_bytes(int ktiles, int nsteps) {
  return (size_t)ktiles * nsteps * 64 * 16 + (size_t)ktiles * 32 * sizeof(float);
}

inline size_t bf16q_lds(int ktiles, int nsteps, int dim) {
  return frag_bytes(ktiles, nsteps) + (size_t)4 * (32 * dim + 16) * sizeof(float);
}

// the A-fragments of every centre tile ([tile][k-step][lane] x 8 bf16: centre ct*32 + (lane & 31),
// features 16 st + 8 (lane >> 5) ..) with 1.0 at feature dim (the -||x||^2 / 2 slot), and the norms
// (+inf past k), once per call
__global__ void k_bf16q_frags(int dim, int nsteps, int ktiles, int k, const float* __restrict__ C,
                              const float* __restrict__ cn2, bf16x8_t* __restrict__ frags,
                              float* __restrict__ cn_out) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e < ktiles * nsteps * 64) {
    const int l = e & 63, rest = e >> 6;
    const int st = rest % nsteps, ct = rest / nsteps;
    const int c = ct * 32 + (l & 31), f0 = 16 * st + 8 * (l >> 5);
    bf16x8_t v;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int f = f0 + j;
      v[j] = (__bf16)(f == dim ? 1.0f : ((c < k && f < dim) ? C[(int64_t)c * dim + f] : 0.f));
    }
    frags[e] = v;
  }
  if (e < ktiles * 32) cn_out[e] = e < k ? cn2[e] : __builtin_inff();
}

__device__ __forceinline__ int key_with_index(float d, int idx) {
  int out;
  // one v_and_or_b32 (the mask comes from an SGPR: a VOP3 literal is not available on gfx950)
  asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(out) : "v"(d), "s"(0xffffffe0u), "n"(idx));
  return out;
}

template <int PER, int NST, bool VEC4>
__global__ __launch_bounds__(256) void k_assign_bf16q(int64_t n, int dim, int ktiles,
                                                      const float* __restrict__ X,
                                                      const bf16x8_t* __restrict__ frags,
                                                      const float* __restrict__ cn_in,
                                                      const float* __restrict__ C,
                                                      int32_t* __restrict__ labels,
                                                      float* __restrict__ sq_dist) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  bf16x8_t* Af = reinterpret_cast<bf16x8_t*>(smem);
  float* Cn = reinterpret_cast<float*>(smem + (size_t)ktiles * NST * 64 * 16);
  float* Pt = Cn + ktiles * 32;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, r = lane & 31;
  const int slot = 32 * dim + 16;  // floats per wave slot (a multiple of 4: dim x 32 is)
  {  // the prebuilt fragments and norms: coalesced 16-byte copies
    const int nfr = ktiles * NST * 64;
    for (int e = tid; e < nfr; e += 256) Af[e] = frags[e];
    for (int c = tid; c < ktiles * 32; c += 256) Cn[c] = cn_in[c];
  }
  float* my = Pt + wave * slot;
  if (lane < 16) my[32 * dim + lane] = 0.f;  // past the last row: read by row 31's masked features
  __syncthreads();
  const int nf4 = 8 * dim;  // float4 per full tile (32 rows x dim floats)
  const int64_t ntiles = (n + 31) / 32, nfull = n / 32;
  const int64_t step = (int64_t)gridDim.x * 4;
  // every load unconditional (a tile past the full ones re-reads the last full tile, unused), so the
  // compiler's vmcnt waits count exactly PER loads per tile and the next tile's stay in flight
  auto fetch = [&](int64_t tt, floatx4_t (&v)[PER]) {
    const int64_t tc = min(tt, nfull - 1);
    const floatx4_t* src = reinterpret_cast<const floatx4_t*>(X + tc * 32 * dim);
#pragma unroll
    for (int q = 0; q < PER; ++q) v[q] = __builtin_nontemporal_load(src + min(lane + 64 * q, nf4 - 1));
  };
  auto stage = [&](int64_t tt, const floatx4_t (&v)[PER]) {
    if (tt < nfull) {
      floatx4_t* d4 = reinterpret_cast<floatx4_t*>(my);
#pragma unroll
      for (int q = 0; q < PER; ++q)
        if (lane + 64 * q < nf4) d4[lane + 64 * q] = v[q];
    } else {  // the partial last tile
      const int64_t m = (n - tt * 32) * dim;
      for (int e = lane; e < 32 * dim; e += 64) my[e] = e < m ? X[tt * 32 * dim + e] : 0.f;
    }
  };
  const int lastf = dim - 16 * (NST - 1) - 8 * h;  // features of the last k-step this lane keeps
  auto compute = [&](int64_t tt) {
    const float* row = my + r * dim;
    float x[NST][8];
    float xx = 0.f;  // this lane's half of ||x||^2 (fp32)
#pragma unroll
    for (int st = 0; st < NST; ++st) {
      if constexpr (VEC4) {
        const floatx4_t lo = *reinterpret_cast<const floatx4_t*>(row + 16 * st + 8 * h);
        const floatx4_t hi = *reinterpret_cast<const floatx4_t*>(row + 16 * st + 8 * h + 4);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          x[st][j] = lo[j];
          x[st][4 + j] = hi[j];
        }
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) x[st][j] = row[16 * st + 8 * h + j];
      }
      if (st == NST - 1) {
#pragma unroll
        for (int j = 0; j < 8; ++j) x[st][j] = j < lastf ? x[st][j] : 0.f;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) xx = __builtin_fmaf(x[st][j], x[st][j], xx);
    }
    const float oxx = __shfl_xor(xx, 32);
    const float shift = -0.5f * (h ? oxx + xx : xx + oxx);  // the same value on both halves
    bf16x8_t b[NST];
#pragma unroll
    for (int st = 0; st < NST; ++st) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float v = x[st][j];
        if (st == NST - 1 && j == lastf) v = shift;  // feature dim: the free K slot
        b[st][j] = (__bf16)v;
      }
    }
    int bestk = 0x7fffffff;
    int bestct = 0;
    auto chain = [&](int c) {
      floatx16 acc = {};
#pragma unroll
      for (int st = 0; st < NST; ++st)
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(Af[(c * NST + st) * 64 + lane], b[st], acc, 0, 0, 0);
      return acc;
    };
    auto epilogue = [&](const floatx16& acc, int ct) {
      const floatx4_t* cp = reinterpret_cast<const floatx4_t*>(Cn + ct * 32 + 4 * h);
      int e[16];
      const floatx4_t cn0 = cp[0], cn1 = cp[2], cn2 = cp[4], cn3 = cp[6];  // rows 8g + 4h .. +3
#define GDD_KEY(g, j) e[4 * g + j] = key_with_index(__builtin_fmaf(-2.f, acc[4 * g + j], cn##g[j]), 8 * g + j)
      GDD_KEY(0, 0); GDD_KEY(0, 1); GDD_KEY(0, 2); GDD_KEY(0, 3);
      GDD_KEY(1, 0); GDD_KEY(1, 1); GDD_KEY(1, 2); GDD_KEY(1, 3);
      GDD_KEY(2, 0); GDD_KEY(2, 1); GDD_KEY(2, 2); GDD_KEY(2, 3);
      GDD_KEY(3, 0); GDD_KEY(3, 1); GDD_KEY(3, 2); GDD_KEY(3, 3);
#undef GDD_KEY
      int m = min(e[0], min(e[1], e[2]));
#pragma unroll
      for (int q = 3; q < 15; q += 2) m = min(m, min(e[q], e[q + 1]));
      m = min(m, e[15]);
      if (m < bestk) {
        bestk = m;
        bestct = ct;
      }
    };
    int ct = 0;
    for (; ct + 2 <= ktiles; ct += 2) {
      const floatx16 a0 = chain(ct);
      const floatx16 a1 = chain(ct + 1);
      epilogue(a0, ct);
      epilogue(a1, ct + 1);
    }
    if (ct < ktiles) epilogue(chain(ct), ct);
    int bestc = bestct * 32 + (bestk & 31) + 4 * h;
    const int ok = __shfl_xor(bestk, 32);
    const int oc = __shfl_xor(bestc, 32);
    if (ok < bestk || (ok == bestk && oc < bestc)) {
      bestk = ok;
      bestc = oc;
    }
    const int64_t p = tt * 32 + r;
    if (h == 0 && p < n) {
      labels[p] = bestc;
      if (sq_dist) sq_dist[p] = skl_sqdist(row, C + (int64_t)bestc * dim, dim);
    }
  };
  // two tiles' loads in flight per wave (three or four measured the same: the pass did not wait on HBM)
  floatx4_t va[PER], vb[PER];
  int64_t t = (int64_t)blockIdx.x * 4 + wave;
  fetch(t, va);
  fetch(t + step, vb);
  while (t < ntiles) {
    stage(t, va);
    fetch(t + 2 * step, va);
    compute(t);
    t += step;
    if (t >= ntiles) break;
    stage(t, vb);
    fetch(t + 2 * step, vb);
    compute(t);
    t += step;
  }
}

}  // namespace

int bf16q_launch(int64_t n, int dim, const float* X, int k, const float* C, const float* c_norm2,
                 int32_t* labels, float* sq_dist, void* ws, size_t ws_bytes, hipStream_t s) {
  const int nsteps = (dim + 15) / 16, ktiles = (k + 31) / 32;
  GDD_REQUIRE(n >= 32 && dim % 16 != 0 && nsteps <= 4 && k > 0, "bf16 labels pass: unsupported shape");
  GDD_REQUIRE((reinterpret_cast<uintptr_t>(X) & 15) == 0, "bf16 labels pass: X must be 16-byte aligned");
  GDD_REQUIRE(frag_bytes(ktiles, nsteps) <= ws_bytes, "bf16 labels pass: workspace too small");
  const size_t lds = bf16q_lds(ktiles, nsteps, dim);
  GDD_REQUIRE(lds <= 150 * 1024, "bf16 labels pass: centres do not fit the LDS");
  bf16x8_t* frags = static_cast<bf16x8_t*>(ws);
  float* cn = reinterpret_cast<float*>(static_cast<char*>(ws) + (size_t)ktiles * nsteps * 64 * 16);
  const int nfr = std::max(ktiles * nsteps * 64, ktiles * 32);
  k_bf16q_frags<<<(nfr + 255) / 256, 256, 0, s>>>(dim, nsteps, ktiles, k, C, c_norm2, frags, cn);
  GDD_LAUNCHED();
  const int64_t ntiles = (n + 31) / 32;
  const int per_need = (8 * dim + 63) / 64;
  auto go = [&](auto kern) -> int {
    GDD_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    int res = 0;
    const int rc = occupancy_blocks((const void*)kern, 256, lds, &res);
    if (rc) return rc;
    const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>((ntiles + 3) / 4, (int64_t)res));
    kern<<<grid, 256, lds, s>>>(n, dim, ktiles, X, frags, cn, C, labels, sq_dist);
    GDD_LAUNCHED();
    return GDD_OK;
  };
  auto pick_per = [&](auto N_, auto V_) -> int {
    constexpr int N = decltype(N_)::value;
    constexpr bool V = decltype(V_)::value;
    if (per_need <= 1) return go(k_assign_bf16q<1, N, V>);
    if (per_need <= 2) return go(k_assign_bf16q<2, N, V>);
    if (per_need <= 4) return go(k_assign_bf16q<4, N, V>);
    if (per_need <= 6) return go(k_assign_bf16q<6, N, V>);
    return go(k_assign_bf16q<8, N, V>);
  };
  using T_ = std::true_type;
  using F_ = std::false_type;
  const bool v4 = dim % 4 == 0;
  switch (nsteps) {
    case 1: return v4 ? pick_per(std::integral_constant<int, 1>(), T_()) : pick_per(std::integral_constant<int, 1>(), F_());
    case 2: return v4 ? pick_per(std::integral_constant<int, 2>(), T_()) : pick_per(std::integral_constant<int, 2>(), F_());
    case 3: return v4 ? pick_per(std::integral_constant<int, 3>(), T_()) : pick_per(std::integral_constant<int, 3>(), F_());
    default: return v4 ? pick_per(std::integral_constant<int, 4>(), T_()) : pick_per(std::integral_constant<int, 4>(), F_());
  }
}

}  // namespace gdd
