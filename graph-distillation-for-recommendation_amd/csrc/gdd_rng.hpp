// gdd_rng.hpp — numpy's legacy RandomState (MT19937) draws, restated for the native host loops.
//
// The reference's k-means consumes numpy.random.RandomState (sklearn check_random_state). To run the
// MiniBatchKMeans loop natively, the host code must draw the exact same numbers in the same order:
//   mt19937 genrand_int32 + tempering        numpy/random/src/mt19937/mt19937.{h,c}
//   legacy random_sample (53-bit double)      mt19937_next_double: (a>>5)*2^26 + (b>>6), / 2^53
//   randint(low, high, size), int64 dtype     _bounded_integers.pyx _rand_int64 ->
//                                             random_bounded_uint64_fill, masked rejection on
//                                             32-bit draws when high-low-1 < 2^32
//   permutation(n) / shuffle                  RandomState._shuffle_raw + random_interval
//   choice(n, replace=False, size=m)          permutation(n)[:m]
//   choice(n, p=p)                            cdf = cumsum(p); cdf /= cdf[-1]; searchsorted(u, 'right')
// Host-only code (no device state). Verified against numpy draw-for-draw in tests/test_rng.py.
#pragma once

#include <cstdint>
#include <cstring>
#include <vector>

namespace gdd {

struct MTState {  // layout of gdd_mt_state in gdd.h
  uint32_t key[624];
  int32_t pos;
  int32_t has_gauss;
  double gauss;
};

class LegacyRNG {
 public:
  explicit LegacyRNG(MTState* s) : s_(s) {}

  uint32_t next32() {
    if (s_->pos >= 624) generate();
    uint32_t y = s_->key[s_->pos++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
  }

  double next_double() {
    const int32_t a = (int32_t)(next32() >> 5), b = (int32_t)(next32() >> 6);
    return (a * 67108864.0 + b) / 9007199254740992.0;
  }

  static uint64_t gen_mask(uint64_t max) {
    uint64_t m = max;
    m |= m >> 1;
    m |= m >> 2;
    m |= m >> 4;
    m |= m >> 8;
    m |= m >> 16;
    m |= m >> 32;
    return m;
  }

  uint64_t next64() {
    const uint64_t hi = next32();
    return (hi << 32) | next32();
  }

  // RandomState.randint(low, high, size) with the default int64 dtype
  void randint(int64_t low, int64_t high, int64_t count, int64_t* out) {
    const uint64_t rng = (uint64_t)(high - 1 - low);
    const uint64_t off = (uint64_t)low;
    if (rng == 0) {
      for (int64_t i = 0; i < count; ++i) out[i] = low;
      return;
    }
    if (rng <= 0xFFFFFFFFull) {
      if (rng == 0xFFFFFFFFull) {
        for (int64_t i = 0; i < count; ++i) out[i] = (int64_t)(off + next32());
        return;
      }
      const uint32_t mask = (uint32_t)gen_mask(rng);
      for (int64_t i = 0; i < count; ++i) {
        uint32_t v;
        while ((v = (next32() & mask)) > (uint32_t)rng) {
        }
        out[i] = (int64_t)(off + v);
      }
      return;
    }
    const uint64_t mask = gen_mask(rng);
    for (int64_t i = 0; i < count; ++i) {
      uint64_t v;
      if (rng == 0xFFFFFFFFFFFFFFFFull) {
        v = next64();
      } else {
        while ((v = (next64() & mask)) > rng) {
        }
      }
      out[i] = (int64_t)(off + v);
    }
  }

  uint64_t random_interval(uint64_t max) {
    if (max == 0) return 0;
    const uint64_t mask = gen_mask(max);
    uint64_t v;
    if (max <= 0xffffffffull) {
      while ((v = (next32() & mask)) > max) {
      }
    } else {
      while ((v = (next64() & mask)) > max) {
      }
    }
    return v;
  }

  // RandomState.permutation(n)
  std::vector<int64_t> permutation(int64_t n) {
    std::vector<int64_t> a(n);
    for (int64_t i = 0; i < n; ++i) a[i] = i;
    for (int64_t i = n - 1; i >= 1; --i) {
      const int64_t j = (int64_t)random_interval((uint64_t)i);
      const int64_t t = a[j];
      a[j] = a[i];
      a[i] = t;
    }
    return a;
  }

  // RandomState.choice(n, p=w/w.sum()) for fp32 unit weights: p_i = fp32(1/n) as doubles
  int64_t choice_uniform_weights(int64_t n) {
    const double p = (double)(1.0f / (float)n);  // sample_weight / sample_weight.sum() in fp32
    std::vector<double> cdf(n);
    double run = 0.0;
    for (int64_t i = 0; i < n; ++i) {
      run = run + p;
      cdf[i] = run;
    }
    const double last = cdf[n - 1];
    for (int64_t i = 0; i < n; ++i) cdf[i] = cdf[i] / last;
    const double u = next_double();
    // searchsorted(side='right'): first index with cdf[idx] > u
    int64_t a = 0, b = n;
    while (a < b) {
      const int64_t m = (a + b) >> 1;
      if (cdf[m] <= u)
        a = m + 1;
      else
        b = m;
    }
    return a;
  }

 private:
  void generate() {
    static const uint32_t mag01[2] = {0x0u, 0x9908b0dfu};
    uint32_t* mt = s_->key;
    int kk;
    uint32_t y;
    for (kk = 0; kk < 624 - 397; kk++) {
      y = (mt[kk] & 0x80000000u) | (mt[kk + 1] & 0x7fffffffu);
      mt[kk] = mt[kk + 397] ^ (y >> 1) ^ mag01[y & 0x1u];
    }
    for (; kk < 623; kk++) {
      y = (mt[kk] & 0x80000000u) | (mt[kk + 1] & 0x7fffffffu);
      mt[kk] = mt[kk + (397 - 624)] ^ (y >> 1) ^ mag01[y & 0x1u];
    }
    y = (mt[623] & 0x80000000u) | (mt[0] & 0x7fffffffu);
    mt[623] = mt[396] ^ (y >> 1) ^ mag01[y & 0x1u];
    s_->pos = 0;
  }

  MTState* s_;
};

}  // namespace gdd
