// gdd_bf16.hip — the bf16 full labels pass (predict(precision="bf16"); SURVEY §8(d) config 5: "fp32
// vs bf16 MFMA distance kernel"), r06 form. Its own translation unit: it is built with
// -mllvm -amdgpu-mfma-vgpr-form (Makefile), so the MFMA accumulators live in VGPRs and the epilogue
// reads them without v_accvgpr_read copies; the fp32 kernels of gdd_kmeans.hip keep the default.
//
// HBM design point: X is read once (460 MB at 2.45M x 47: ~58 us at 8 TB/s; torch's own X.sum() takes
// 121 us on the same box). The r03 kernel (gdd_kmeans.hip k_assign_bf16p, GDD_FORCE=bf16_v1) ran at
// 0.36 of that roof; its counters (rocprofv3, profiles/r06_bf16_pmc.json) put the limit in the VALU:
// ~780 vector instructions per 32-point tile, each 4 cycles of its SIMD. Here ~340:
//   * one launch: every block builds the centres' A-fragments ([tile][k-step][lane] x 8 bf16) and
//     their -||c||^2 / 2 in its LDS from C, after issuing its first X loads (r06 first form: a
//     separate fragment kernel, ~5 us plus a launch gap per call);
//   * a tile's 32 x dim floats are ONE contiguous span of X, copied into the wave's LDS slot as is
//     (float4 stores, row stride dim: no index arithmetic); B-fragments read row r's features
//     16 st + 8 h .. + 7 straight from it (two ds_read_b128 when dim % 4 == 0, else eight
//     ds_read_b32), features past dim masked to zero;
//   * the whole distance comes out of the MFMA chain: the accumulator STARTS at -||c||^2 / 2 (fp32,
//     exact), and the first free K slot (feature dim; the pass needs dim % 16 != 0) carries
//     -(||x||^2 / 2 + delta) in the B-fragment against 1.0 in every centre's A-fragment, so the
//     chain yields acc = -(d / 2 + delta), d the squared distance;
//   * the argmin runs on integer keys: acc < 0 always (below), and the bits of negative floats order
//     as signed integers like their magnitudes, so the smallest key is the nearest centre. The
//     centre's in-tile index goes into the 5 low significand bits (one v_and_or_b32 per centre: a
//     larger index adds magnitude, the lower index wins a tie), and a balanced v_min3_i32 tree takes
//     the tile's 16 keys per lane (8 per centre tile) — per centre 1.5 VALU, where the r03 epilogue
//     spent an fma, a compare and two selects (plus a copy out of the accumulator).
// Accuracy: the labels are those of bf16 dot products (tests/test_gpu_kmeans.py and
// tests/test_gpu_configs.py bound every label that differs from the exact fp32 one by the bf16
// rounding, 2^-7 ||x|| ||c|| per product). delta = 2^-5 ||x||^2 + 2^-100 keeps acc strictly negative:
// a centre whose acc crossed zero would need d / 2 < 2^-7 ||x|| ||c|| + 2^-7 ||x||^2 (the products'
// rounding; the shift's: ||x||^2 summed from the bf16-rounded features, <= 2^-8 ||x||^2 off, then
// rounded to bf16) - delta, impossible for ||c|| <= 2.9 ||x|| (the right side is negative) and for
// larger ||c|| (then d >= (||c|| - ||x||)^2 is far above it); the shift is the same for every centre
// of a point, so neither it nor its bf16 rounding reorders them. Dropping 5 of the 24 significand
// bits moves a key by < 2^-18 of |acc|; keys that tie may pick either centre.
#include <algorithm>
#include <type_traits>

#include "gdd_common.hpp"

namespace gdd {
namespace {

using floatx16 = __attribute__((ext_vector_type(16))) float;
typedef float floatx4_t __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));

inline size_t bf16q_lds(int ktiles, int nsteps, int dim, int waves) {
  return (size_t)ktiles * nsteps * 64 * 16 + (size_t)ktiles * 32 * sizeof(float) +
         (size_t)waves * (32 * dim + 16) * sizeof(float);
}

// the key: acc's bits with the in-tile index in the 5 low significand bits (one v_and_or_b32). Plain C,
// not inline asm: an asm operand that reads an MFMA result directly is invisible to the compiler's
// hazard recognizer (no wait states after the MFMA: stale accumulator values — r06, measured)
__device__ __forceinline__ int key_with_index(float d, int idx) {
  return (int)((__float_as_uint(d) & 0xffffffe0u) | (unsigned)idx);
}

// W waves per block, D tiles' loads in flight per wave, WPE the waves per SIMD the registers allow
// DIM > 0: the feature count fixed at compile time (the configs' logit widths 47, 41, 40: the last
// k-step's masks and the free slot then fold to one select per lane half), else the argument
template <int PER, int NST, bool VEC4, int W, int D, int WPE, int DIM = 0>
__global__ __launch_bounds__(64 * W) __attribute__((amdgpu_waves_per_eu(WPE))) void k_assign_bf16q(
    int64_t n, int dim_arg, int k, int ktiles, const float* __restrict__ X, const float* __restrict__ C,
    const float* __restrict__ cn2, int32_t* __restrict__ labels, float* __restrict__ sq_dist) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int dim = DIM > 0 ? DIM : dim_arg;
  bf16x8_t* Af = reinterpret_cast<bf16x8_t*>(smem);
  float* Cn = reinterpret_cast<float*>(smem + (size_t)ktiles * NST * 64 * 16);
  float* Pt = Cn + ktiles * 32;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, r = lane & 31;
  const int slot = 32 * dim + 16;  // floats per wave slot (a multiple of 4: dim x 32 is)
  float* my = Pt + wave * slot;
  const int nf4 = 8 * dim;  // float4 per full tile (32 rows x dim floats)
  const int64_t ntiles = (n + 31) / 32, nfull = n / 32;
  const int64_t step = (int64_t)gridDim.x * W;
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
    }
    // the B-fragments first (the free slot still zero), then this lane's half of ||x||^2 from them: one
    // v_dot2c_f32_bf16 per pair of features instead of two fp32 fmas (the shift's error, ~2^-8 ||x||^2,
    // stays inside delta: header)
    bf16x8_t b[NST];
    float xx = 0.f;
#pragma unroll
    for (int st = 0; st < NST; ++st) {
#pragma unroll
      for (int j = 0; j < 8; ++j) b[st][j] = (__bf16)x[st][j];
      const bf16x2_t* pr = reinterpret_cast<const bf16x2_t*>(&b[st]);
#pragma unroll
      for (int q = 0; q < 4; ++q) xx = __builtin_amdgcn_fdot2_f32_bf16(pr[q], pr[q], xx, false);
    }
    const float oxx = __shfl_xor(xx, 32);
    const float xsq = h ? oxx + xx : xx + oxx;  // the same value on both halves
    const float shift = -__builtin_fmaf(0.53125f, xsq, 0x1p-100f);  // -(||x||^2 / 2 + delta), header
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (j == lastf) b[NST - 1][j] = (__bf16)shift;  // feature dim: the free K slot
    int bestk = 0x7fffffff;
    int bestct = 0;
    auto chain = [&](int c) {
      floatx16 acc;  // rows 8g + 4h .. + 3 of centre tile c: -||c||^2 / 2
      const floatx4_t* cp = reinterpret_cast<const floatx4_t*>(Cn + c * 32 + 4 * h);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const floatx4_t v = cp[2 * g];
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[4 * g + j] = v[j];
      }
#pragma unroll
      for (int st = 0; st < NST; ++st)
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(Af[(c * NST + st) * 64 + lane], b[st], acc, 0, 0, 0);
      return acc;
    };
    auto epilogue = [&](const floatx16& acc, int ct) {
      int e[16];  // acc = -(d / 2 + delta) < 0: its bits order as signed integers like d
#pragma unroll
      for (int q = 0; q < 16; ++q) e[q] = key_with_index(acc[q], 8 * (q >> 2) + (q & 3));
      // a balanced v_min3_i32 tree (8 per centre tile), the running best folded into its root
      const int m1 = min(e[0], min(e[1], e[2])), m2 = min(e[3], min(e[4], e[5]));
      const int m3 = min(e[6], min(e[7], e[8])), m4 = min(e[9], min(e[10], e[11]));
      const int m5 = min(e[12], min(e[13], e[14]));
      const int m6 = min(m1, min(m2, m3)), m7 = min(m4, min(m5, e[15]));
      const int m = min(bestk, min(m6, m7));
      if (m != bestk) bestct = ct;
      bestk = m;
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
  // D = 2: two tiles' loads in flight per wave (three or four measured the same: the pass does not wait
  // on HBM); D = 1 (the 8-wave form): one, the registers go to occupancy instead
  floatx4_t va[PER], vb[PER];
  int64_t t = (int64_t)blockIdx.x * W + wave;
  fetch(t, va);
  if constexpr (D == 2) fetch(t + step, vb);
  {  // the centre tiles, while the first X loads are in flight: A-fragments (centre ct * 32 + (lane &
     // 31), features 16 st + 8 (lane >> 5) .., 1.0 at feature dim, zero past it and past k) and
     // -||c||^2 / 2 (-inf past k: never the minimum). U fragments per thread per round, their loads
     // issued together (L2 latency once per round, not per fragment). Without given norms each
     // fragment leaves its 8 features' sum of squares in the (not yet used) wave slots, summed per
     // centre in a fixed order after the barrier: ||c||^2 in fp32, deterministic.
    constexpr int U = W == 8 ? 4 : 6;  // (8 waves: within the 128 VGPRs of WPE = 4)
    float* part = Pt;  // [centre][2 NST] partial sums (bf16q_norms_fit: they fit the wave slots)
    const int nfr = ktiles * NST * 64;
    for (int e0 = tid; e0 < nfr; e0 += 64 * W * U) {
      float v[U][8];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = e0 + u * 64 * W, l = e & 63, rest = e >> 6;
        const int st = rest % NST, ct = rest / NST;
        const int c = ct * 32 + (l & 31), f0 = 16 * st + 8 * (l >> 5);
#pragma unroll
        for (int j = 0; j < 8; ++j)
          v[u][j] = (e < nfr && c < k && f0 + j < dim) ? C[(int64_t)c * dim + f0 + j] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = e0 + u * 64 * W, l = e & 63, rest = e >> 6;
        if (e >= nfr) break;
        const int st = rest % NST, ct = rest / NST;
        const int f0 = 16 * st + 8 * (l >> 5);
        bf16x8_t fr;
        float ss = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          fr[j] = (__bf16)(f0 + j == dim ? 1.0f : v[u][j]);
          ss = __builtin_fmaf(v[u][j], v[u][j], ss);
        }
        Af[e] = fr;
        if (!cn2) part[(ct * 32 + (l & 31)) * (2 * NST) + 2 * st + (l >> 5)] = ss;
      }
    }
    __syncthreads();
    for (int c = tid; c < ktiles * 32; c += 64 * W) {
      float v = __builtin_inff();
      if (c < k) {
        if (cn2) {
          v = cn2[c];
        } else {
          v = 0.f;
#pragma unroll
          for (int q = 0; q < 2 * NST; ++q) v += part[c * (2 * NST) + q];
        }
      }
      Cn[c] = -0.5f * v;
    }
    __syncthreads();
    if (lane < 16) my[32 * dim + lane] = 0.f;  // past the last row: read by row 31's masked features
  }
  if constexpr (D == 1) {
    while (t < ntiles) {
      stage(t, va);
      fetch(t + step, va);
      compute(t);
      t += step;
    }
    return;
  }
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

bool bf16q_norms_fit(int dim, int k) {
  const int nsteps = (dim + 15) / 16, ktiles = (k + 31) / 32;
  return (int64_t)ktiles * 32 * 2 * nsteps <= (int64_t)4 * (32 * dim + 16);  // the 4-wave slots
}

int bf16q_launch(int64_t n, int dim, const float* X, int k, const float* C, const float* c_norm2,
                 int32_t* labels, float* sq_dist, hipStream_t s) {
  const int nsteps = (dim + 15) / 16, ktiles = (k + 31) / 32;
  GDD_REQUIRE(n >= 32 && dim % 16 != 0 && nsteps <= 4 && k > 0, "bf16 labels pass: unsupported shape");
  GDD_REQUIRE((reinterpret_cast<uintptr_t>(X) & 15) == 0, "bf16 labels pass: X must be 16-byte aligned");
  GDD_REQUIRE(c_norm2 || bf16q_norms_fit(dim, k), "bf16 labels pass: this k needs the norms given");
  // at three k-steps (the configs' logit widths 41 .. 47) with many centre tiles, 8-wave blocks with
  // one tile's loads in flight and at most 128 VGPRs (4 waves per SIMD): Reddit's k = 769 at 0.84 of
  // the 4-wave form's time, products' k = 196 the same within noise (r06, tools/micro_bf16.py).
  // GDD_FORCE=bf16_w4 / bf16_w8: either form at any k (A/B, tests)
  const bool f3 = nsteps == 3 && dim % 4 != 0 && (8 * dim + 63) / 64 == 6;
  const bool w8 = f3 && !forced("bf16_w4") && (ktiles > 8 || forced("bf16_w8"));
  const int waves = w8 ? 8 : 4;
  const size_t lds = bf16q_lds(ktiles, nsteps, dim, waves);
  GDD_REQUIRE(lds <= 150 * 1024, "bf16 labels pass: centres do not fit the LDS");
  const int64_t ntiles = (n + 31) / 32;
  const int per_need = (8 * dim + 63) / 64;
  auto go = [&](auto kern) -> int {
    GDD_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    int res = 0;
    const int rc = occupancy_blocks((const void*)kern, 64 * waves, lds, &res);
    if (rc) return rc;
    const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>((ntiles + waves - 1) / waves, (int64_t)res));
    kern<<<grid, 64 * waves, lds, s>>>(n, dim, k, ktiles, X, C, c_norm2, labels, sq_dist);
    GDD_LAUNCHED();
    return GDD_OK;
  };
  auto pick_per = [&](auto N_, auto V_) -> int {
    constexpr int N = decltype(N_)::value;
    constexpr bool V = decltype(V_)::value;
    if (per_need <= 1) return go(k_assign_bf16q<1, N, V, 4, 2, 1>);
    if (per_need <= 2) return go(k_assign_bf16q<2, N, V, 4, 2, 1>);
    if (per_need <= 4) return go(k_assign_bf16q<4, N, V, 4, 2, 1>);
    if (per_need <= 6) {
      if constexpr (N == 3 && !V) {  // dims 41 .. 47
        if (w8) return dim == 41 ? go(k_assign_bf16q<6, 3, false, 8, 1, 4, 41>)
                                 : dim == 47 ? go(k_assign_bf16q<6, 3, false, 8, 1, 4, 47>)
                                             : go(k_assign_bf16q<6, 3, false, 8, 1, 4>);
        if (dim == 47) return go(k_assign_bf16q<6, 3, false, 4, 2, 1, 47>);
        if (dim == 41) return go(k_assign_bf16q<6, 3, false, 4, 2, 1, 41>);
      }
      if constexpr (N == 3 && V)
        if (dim == 40) return go(k_assign_bf16q<6, 3, true, 4, 2, 1, 40>);
      return go(k_assign_bf16q<6, N, V, 4, 2, 1>);
    }
    return go(k_assign_bf16q<8, N, V, 4, 2, 1>);
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
