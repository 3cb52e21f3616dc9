// gdd_devrng.hpp — numpy legacy RandomState (MT19937) draws on the device, one workgroup at a time.
//
// The same draws as gdd_rng.hpp (host), restated for a cooperating workgroup so that the
// MiniBatchKMeans loop can draw its batch indices and reassignment permutations without a host
// round trip:
//   twist      mt19937_gen (numpy/random/src/mt19937/mt19937.c) in four dependency phases:
//              i < 227 reads only old words; 227 <= i < 454 reads new[i-227] from phase 1;
//              454 <= i < 623 reads new[i-227] from phase 2; i = 623 reads new[0] and new[396]
//   randint    RandomState.randint(low, high, size) int64, masked rejection on 32-bit draws
//              (_bounded_integers.pyx _rand_int64 -> random_bounded_uint64_fill): each tempered
//              word is accepted iff (w & mask) <= rng; a workgroup prefix count over the words of
//              the current key block places the accepted values in draw order
//   shuffle    RandomState.permutation(n) (legacy _shuffle_raw + random_interval): one lane walks
//              the tempered words to get j_i for i = n-1..1; the first m entries of the permuted
//              arange are then traced backwards through the swaps, one lane per entry
// Requirements: blockDim.x is a multiple of 64 and >= 256 (the twist's widest phase is 227 words;
// randint walks the key block in windows of blockDim.x words); every thread of the block calls in.
#pragma once

#include <climits>
#include <cstdint>

namespace gdd {

struct DevMT {  // key block + position, as gdd_mt_state without the gaussian cache
  uint32_t key[624];
  int32_t pos;
  int32_t pad;
};

__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= (y >> 18);
  return y;
}

__device__ __forceinline__ uint32_t mt_mix(uint32_t a, uint32_t b, uint32_t c) {
  const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
  return c ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
}

// regenerate the 624-word key block in LDS (mt19937_gen). Word kk >= 227 depends on the NEW word
// kk - 227, so thread t < 227 carries the chain t -> 227 + t -> 454 + t in registers: every read
// is of an old word, all reads precede all writes, and word 623 (which needs new words 0 and 396)
// follows. Three barriers.
__device__ inline void mt_twist_block(uint32_t* key) {
  const int t = threadIdx.x;
  uint32_t n0 = 0, n1 = 0, n2 = 0, o623 = 0;
  if (t < 227) {
    n0 = mt_mix(key[t], key[t + 1], key[t + 397]);
    n1 = mt_mix(key[227 + t], key[228 + t], n0);
    if (t < 169) n2 = mt_mix(key[454 + t], key[455 + t], n1);
    if (t == 0) o623 = key[623];
  }
  __syncthreads();
  if (t < 227) {
    key[t] = n0;
    key[227 + t] = n1;
    if (t < 169) key[454 + t] = n2;
  }
  __syncthreads();
  if (t == 0) key[623] = mt_mix(o623, key[0], key[396]);
  __syncthreads();
}

// the same with ONE wave (no block barriers): lane l carries the chains of t = l, l+64, l+128,
// l+192 (< 227); all old words are read before any write (a wave's LDS operations execute in
// order; the empty asm keeps the compiler from moving reads past writes it cannot relate).
__device__ inline void mt_twist_wave(uint32_t* key) {
  const int lane = threadIdx.x & 63;
  uint32_t n0[4], n1[4], n2[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int t = lane + 64 * g;
    const int tc = t < 227 ? t : 0;
    n0[g] = mt_mix(key[tc], key[tc + 1], key[tc + 397]);
    n1[g] = mt_mix(key[227 + tc], key[228 + tc], n0[g]);
    const int t3 = tc < 169 ? tc : 0;
    n2[g] = mt_mix(key[454 + t3], key[455 + t3], n1[g]);
  }
  const uint32_t o623 = key[623];
  asm volatile("" ::: "memory");
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int t = lane + 64 * g;
    if (t < 227) {
      key[t] = n0[g];
      key[227 + t] = n1[g];
      if (t < 169) key[454 + t] = n2[g];
    }
  }
  asm volatile("" ::: "memory");
  if (lane == 0) key[623] = mt_mix(o623, key[0], key[396]);
  asm volatile("" ::: "memory");
}

// exclusive prefix count of `flag` over the block; returns the prefix, *total = block count.
// scratch: >= blockDim.x/64 + 1 ints of LDS.
__device__ inline int block_prefix_count(bool flag, int* scratch, int* total) {
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, nw = blockDim.x >> 6;
  const unsigned long long m = __ballot(flag);
  const int before = __popcll(m & ((1ull << lane) - 1ull));
  if (lane == 0) scratch[wave] = __popcll(m);
  __syncthreads();
  int base = 0, tot = 0;
  for (int w = 0; w < nw; ++w) {
    const int c = scratch[w];
    base += w < wave ? c : 0;
    tot += c;
  }
  __syncthreads();
  *total = tot;
  return base + before;
}

__device__ __forceinline__ uint32_t mask32(uint32_t x) {
  x |= x >> 1;
  x |= x >> 2;
  x |= x >> 4;
  x |= x >> 8;
  x |= x >> 16;
  return x;
}

// LDS scratch of the block draws: the key block, the position, the prefix-count scratch
struct MTScratch {
  uint32_t key[624];
  int pos;
  int last;
  int cnt[20];
};

__device__ inline void mt_load(const DevMT* __restrict__ src, MTScratch* s) {
  for (int i = threadIdx.x; i < 624; i += blockDim.x) s->key[i] = src->key[i];
  if (threadIdx.x == 0) s->pos = src->pos;
  __syncthreads();
}

__device__ inline void mt_store(const MTScratch* s, DevMT* __restrict__ dst) {
  for (int i = threadIdx.x; i < 624; i += blockDim.x) dst->key[i] = s->key[i];
  if (threadIdx.x == 0) {
    dst->pos = s->pos;
    dst->pad = 0;
  }
}

// key block `nw` = the twist of block `old` (both LDS, distinct): thread t < 227 carries the chain
// t -> 227 + t -> 454 + t in registers; word 623 follows once new words 0 and 396 are in. Two
// barriers; needs blockDim.x >= 227.
__device__ inline void mt_twist_into(const uint32_t* __restrict__ old, uint32_t* __restrict__ nw) {
  const int t = threadIdx.x;
  if (t < 227) {
    const uint32_t n0 = mt_mix(old[t], old[t + 1], old[t + 397]);
    const uint32_t n1 = mt_mix(old[227 + t], old[228 + t], n0);
    nw[t] = n0;
    nw[227 + t] = n1;
    if (t < 169) nw[454 + t] = mt_mix(old[454 + t], old[455 + t], n1);
  }
  __syncthreads();
  if (t == 0) nw[623] = mt_mix(old[623], nw[0], nw[396]);
  __syncthreads();
}

// LDS of mt_randint_ring: five key blocks (block b of the stream in slot b % 5) + scratch
constexpr int kMtRing = 5;
constexpr size_t kMtRingBytes = sizeof(uint32_t) * (kMtRing * 624 + 64);

// out[0..count) = randint(low, high, count) with every thread busy: each pass takes the next
// 2048 words (2048 / blockDim.x consecutive words per thread), the key blocks they span twisted
// ahead into the ring, acceptance flags, one block prefix of the per-thread counts, ordered
// stores. `ring` slot 0 holds the current key block and `pos` its position (numpy's pos: 624 =
// exhausted). The final state goes to `state_out`. blockDim.x: a power of two in [256, 1024].
__device__ inline void mt_randint_ring(uint32_t* ring, int pos, int64_t low, int64_t high,
                                       int64_t count, int64_t* __restrict__ out,
                                       DevMT* __restrict__ state_out) {
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, nwv = blockDim.x >> 6;
  int* scr = reinterpret_cast<int*>(ring + kMtRing * 624);  // 16 wave totals, the last word
  const uint32_t rng = (uint32_t)(high - 1 - low);
  int last_block = 0, last_pos = pos;
  if (rng == 0) {
    for (int64_t i = t; i < count; i += blockDim.x) out[i] = low;
  } else {
    const uint32_t mask = mask32(rng);
    const int wpt = 2048 / (int)blockDim.x;  // 2, 4 or 8
    int base = 0, ready = 0;
    int64_t produced = 0;
    while (produced < count) {
      const int hib = base + (pos + 2047) / 624;
      while (ready < hib) {
        mt_twist_into(ring + (ready % kMtRing) * 624, ring + ((ready + 1) % kMtRing) * 624);
        ++ready;
      }
      const int r0 = pos + wpt * t;  // this thread's first word, relative to block `base`
      uint32_t v[8];
      unsigned okb = 0;
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        v[u] = 0;
        if (u < wpt) {
          const int r = r0 + u, b = base + r / 624;
          v[u] = mt_temper(ring[(b % kMtRing) * 624 + (r - (r / 624) * 624)]) & mask;
          okb |= (v[u] <= rng ? 1u : 0u) << u;
        }
      }
      const int cnt = __popc(okb);
      // exclusive prefix of cnt over the block: wave scan, then the wave totals
      int inc = cnt;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(inc, o);
        if (lane >= o) inc += y;
      }
      if (lane == 63) scr[wave] = inc;
      __syncthreads();
      int wb = 0, tot = 0;
      for (int w = 0; w < nwv; ++w) {
        const int c = scr[w];
        wb += w < wave ? c : 0;
        tot += c;
      }
      int rank = wb + inc - cnt;
      const int64_t need = count - produced;
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        if ((okb >> u) & 1u) {
          if (rank < need) out[produced + rank] = low + (int64_t)v[u];
          if (rank == need - 1) scr[32] = r0 + u;
          ++rank;
        }
      }
      __syncthreads();
      if (tot >= need) {
        const int wl = scr[32];  // the last word consumed, relative to block `base`
        last_block = base + wl / 624;
        last_pos = wl - (wl / 624) * 624 + 1;
        produced = count;
      } else {
        produced += tot;
        const int nx = pos + 2048;
        base += nx / 624;
        pos = nx - (nx / 624) * 624;
      }
    }
  }
  const uint32_t* kb = ring + (last_block % kMtRing) * 624;
  for (int i = t; i < 624; i += blockDim.x) state_out->key[i] = kb[i];
  if (t == 0) {
    state_out->pos = last_pos;
    state_out->pad = 0;
  }
}

// the next batch in its own workgroup: load the state into the ring, draw, store the new state
__device__ inline void mt_randint_from(const DevMT* __restrict__ in, uint32_t* ring, int64_t low,
                                       int64_t high, int64_t count, int64_t* __restrict__ out,
                                       DevMT* __restrict__ state_out) {
  for (int i = threadIdx.x; i < 624; i += blockDim.x) ring[i] = in->key[i];
  const int pos = in->pos;
  __syncthreads();
  mt_randint_ring(ring, pos, low, high, count, out, state_out);
}

// out[0..count) = randint(low, high, count) (high - low - 1 < 2^32)
__device__ inline void mt_randint_block(MTScratch* s, int64_t low, int64_t high, int64_t count,
                                 int64_t* __restrict__ out) {
  const uint32_t rng = (uint32_t)(high - 1 - low);
  if (rng == 0) {  // no draws
    for (int64_t i = threadIdx.x; i < count; i += blockDim.x) out[i] = low;
    return;
  }
  const uint32_t mask = mask32(rng);
  const int t = threadIdx.x;
  int64_t produced = 0;
  while (produced < count) {
    if (s->pos >= 624) {
      mt_twist_block(s->key);
      if (t == 0) s->pos = 0;
      __syncthreads();
    }
    const int pos = s->pos;
    const int avail = min(624 - pos, (int)blockDim.x);  // this pass's window of words
    uint32_t v = 0;
    bool ok = false;
    if (t < avail) {
      v = mt_temper(s->key[pos + t]) & mask;
      ok = v <= rng;
    }
    int total;
    const int e = block_prefix_count(ok, s->cnt, &total);
    const int64_t need = count - produced;
    if (ok && e < need) out[produced + e] = low + (int64_t)v;
    if (total >= need) {
      if (ok && e == need - 1) s->last = t;
      __syncthreads();
      if (t == 0) s->pos = pos + s->last + 1;
      produced = count;
    } else {
      if (t == 0) s->pos = pos + avail;
      produced += total;
    }
    __syncthreads();
  }
}

// perm[0..m) = RandomState.permutation(n)[:m]. J: n ints of 16-byte aligned LDS (swap partners).
__device__ inline void mt_permutation_prefix_block(MTScratch* s, int64_t n, int m, int* J,
                                            int64_t* __restrict__ perm) {
  const int t = threadIdx.x;
  // wave 0 walks the words up to 64 at a time; the block regenerates the key block when it runs
  // dry. In a window of wn words that cannot take i below the smallest value with the current
  // mask, word u is accepted iff v_u <= i - (accepted before u): v_u <= i - (wn-1) is surely
  // accepted, v_u > i surely rejected, and the few words in between are settled in order. At the
  // bottom of a mask range (i a power of two) words go one by one until the first acceptance.
  if (t == 0) s->last = (int)n - 1;  // the next i to draw for
  __syncthreads();
  const int lane = t & 63;
  while (true) {
    if (s->last < 1) break;
    if (s->pos >= 624) {
      mt_twist_block(s->key);
      if (t == 0) s->pos = 0;
      __syncthreads();
    }
    if (t < 64) {
      int i = s->last, pos = s->pos;
      while (i >= 1 && pos < 624) {
        const uint32_t mk = mask32((uint32_t)i);
        const int m_lo = (int)((mk >> 1) + 1);  // smallest i drawn with this mask
        // a window of wn words cannot accept more than wn, so i stays >= m_lo and the mask fixed
        const int wn = min(64, min(624 - pos, i - m_lo));
        if (wn >= 1) {
          const bool valid = lane < wn;
          const uint32_t v = valid ? (mt_temper(s->key[pos + lane]) & mk) : 0xffffffffu;
          // lane u draws for i_u in [i - u, i]: v <= i - (wn - 1) accepts for sure, v > i never
          const unsigned long long sure = __ballot(valid && v + (uint32_t)(wn - 1) <= (uint32_t)i);
          unsigned long long maybe =
              __ballot(valid && v + (uint32_t)(wn - 1) > (uint32_t)i && v <= (uint32_t)i);
          unsigned long long acc = sure;
          while (maybe) {
            const int u = __ffsll((long long)maybe) - 1;
            maybe &= maybe - 1;
            const int c = __popcll(acc & ((1ull << u) - 1ull));
            const uint32_t vu = (uint32_t)__shfl((int)v, u);
            if (vu <= (uint32_t)(i - c)) acc |= 1ull << u;
          }
          if ((acc >> lane) & 1ull) J[i - __popcll(acc & ((1ull << lane) - 1ull))] = (int)v;
          i -= __popcll(acc);
          pos += wn;
        } else {
          // i == m_lo: word by word until one is accepted (the mask shrinks after it)
          int i0 = i, p0 = pos;
          if (lane == 0) {
            while (p0 < 624) {
              const uint32_t v = mt_temper(s->key[p0++]) & mk;
              if (v <= (uint32_t)i0) {
                J[i0] = (int)v;
                --i0;
                break;
              }
            }
          }
          i = __shfl(i0, 0);
          pos = __shfl(p0, 0);
        }
      }
      if (t == 0) {
        s->last = i;
        s->pos = pos;
      }
    }
    __syncthreads();
  }
  // trace entry p of the permuted arange back through the swaps (applied for i = n-1 .. 1);
  // J is read eight entries per step (two 16-byte LDS reads, one broadcast to all lanes)
  if (t == 0) J[0] = 0;  // swap 0 <-> 0: the identity, so i = 0 can ride along in the batches
  __syncthreads();
  const int nn = (int)n;
  for (int p = t; p < m; p += blockDim.x) {
    int q = p;
    int i0 = 0;
    for (; i0 + 8 <= nn; i0 += 8) {
      const int4 a = *reinterpret_cast<const int4*>(J + i0);
      const int4 b = *reinterpret_cast<const int4*>(J + i0 + 4);
      const int jj[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = i0 + u;
        q = (q == i) ? jj[u] : ((q == jj[u]) ? i : q);
      }
    }
    for (int i = i0; i < nn; ++i) {
      const int j = J[i];
      q = (q == i) ? j : ((q == j) ? i : q);
    }
    perm[p] = q;
  }
  __syncthreads();
}

// out[0..count) = randint(low, high, count) by ONE wave (no block barriers; the other waves are
// free meanwhile). Same words, same acceptance as mt_randint_block. A key block at a time: lane l
// reads words pos + 64 j + l (j < 10, every read issued before the first use), and one ballot per
// 64-word slice places the accepted values in order. Writes s->pos from lane 0.
__device__ inline void mt_randint_wave(MTScratch* s, int64_t low, int64_t high, int64_t count,
                                       int64_t* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const unsigned long long below = (1ull << lane) - 1ull;
  const uint32_t rng = (uint32_t)(high - 1 - low);
  if (rng == 0) {
    for (int64_t i = lane; i < count; i += 64) out[i] = low;
    return;
  }
  const uint32_t mask = mask32(rng);
  int pos = __builtin_amdgcn_readfirstlane(s->pos);
  int64_t produced = 0;
  while (produced < count) {
    if (pos >= 624) {
      mt_twist_wave(s->key);
      pos = 0;
    }
    uint32_t v[10];
    unsigned live = 0;  // bit j: word pos + 64 j + lane is inside the key block
#pragma unroll
    for (int j = 0; j < 10; ++j) {
      const int idx = pos + 64 * j + lane;
      v[j] = idx < 624 ? mt_temper(s->key[idx]) & mask : 0u;
      live |= (idx < 624 ? 1u : 0u) << j;
    }
    int64_t base = produced;
    bool done = false;
#pragma unroll
    for (int j = 0; j < 10; ++j) {
      if (!done) {
        const bool ok = ((live >> j) & 1u) && v[j] <= rng;
        const unsigned long long b = __ballot(ok);
        const int64_t r = base + __popcll(b & below);
        if (ok && r < count) out[r] = low + (int64_t)v[j];
        if (base + __popcll(b) >= count) {  // the last draw is in this slice
          const unsigned long long lb = __ballot(ok && r == count - 1);
          pos = pos + 64 * j + __ffsll((long long)lb);  // through the last word used
          done = true;
        }
        base += __popcll(b);
      }
    }
    if (done) {
      produced = count;
    } else {
      produced = base;
      pos = 624;
    }
    asm volatile("" ::: "memory");
  }
  if (lane == 0) s->pos = pos;
}

// J[i] = random_interval(i) for i = n-1 .. 1: the draws of the legacy shuffle behind
// RandomState.permutation(n), by ONE wave (twists included), 64 words per window. Word u of a
// window is accepted iff (w_u & mask32(i_u)) <= i_u with i_u = i - (#accepted before u), a
// sequential recurrence. Solved as a fixed point: guess the acceptances, recount the prefix, repeat
// until nothing changes. Each pass settles at least one more leading word, so the loop ends within
// 64 passes and its fixed point is the sequential answer; a window usually settles in a few passes
// (only words within a few of the threshold ever flip). Words after i reaches 0 are not consumed.
// Writes s->pos from lane 0.
__device__ inline void mt_shuffle_draws_wave(MTScratch* s, int n, int* J) {
  const int lane = threadIdx.x & 63;
  const unsigned long long below = (1ull << lane) - 1ull;
  int i = n - 1;
  int pos = __builtin_amdgcn_readfirstlane(s->pos);
  while (i >= 1) {
    if (pos >= 624) {
      mt_twist_wave(s->key);
      pos = 0;
    }
    const int wn = min(64, 624 - pos);
    const uint32_t word = lane < wn ? mt_temper(s->key[pos + lane]) : 0u;
    unsigned long long acc = 0;
    int iu = i;
    bool live = lane < wn;
    while (true) {
      live = lane < wn && iu >= 1;
      const uint32_t mu = 0xffffffffu >> __builtin_clz((uint32_t)(iu > 1 ? iu : 1));
      const unsigned long long nacc = __ballot(live && (word & mu) <= (uint32_t)iu);
      if (nacc == acc) break;
      acc = nacc;
      iu = i - __popcll(acc & below);
    }
    if ((acc >> lane) & 1ull) J[iu] = (int)(word & (0xffffffffu >> __builtin_clz((uint32_t)iu)));
    const unsigned long long lv = __ballot(live);  // a prefix of the window
    i -= __popcll(acc);
    pos += __popcll(lv);
    asm volatile("" ::: "memory");
  }
  if (lane == 0) s->pos = pos;
}

// the key block and position by one wave (the others may be busy)
__device__ inline void mt_store_wave(const MTScratch* s, DevMT* __restrict__ dst) {
  const int lane = threadIdx.x & 63;
  for (int i = lane; i < 624; i += 64) dst->key[i] = s->key[i];
  if (lane == 0) {
    dst->pos = s->pos;
    dst->pad = 0;
  }
}

// RandomState.permutation(n)[p] from the shuffle's draws J (J[0] must be 0), for one p by one
// wave: tracing position p back through the swaps (applied for i = n-1 .. 1), the swaps below p
// never touch it, swap p sends it to J[p], and after that it moves (to i) only at a swap i whose
// partner J[i] is its current position. The wave scans J 64 entries at a time.
__device__ inline int shuffle_trace_wave(const int* J, int n, int p) {
  const int lane = threadIdx.x & 63;
  int q = J[p];
  int i0 = p + 1;
  while (i0 < n) {
    const int i = i0 + lane;
    const unsigned long long b = __ballot(i < n && J[i < n ? i : 0] == q);
    if (b) {
      q = i0 + __ffsll((long long)b) - 1;
      i0 = q + 1;
    } else {
      i0 += 64;
    }
  }
  return q;
}

// shuffle_trace_wave reading J 256 entries per step (lane l: one 16-byte read of entries
// a0 + 4l .. a0 + 4l + 3, a0 = the current start rounded down to a multiple of 4; J 16-byte aligned).
// Entries before the start or past n are masked; reads past n stay inside the workgroup's LDS.
__device__ inline int shuffle_trace_wave4(const int* J, int n, int p) {
  const int lane = threadIdx.x & 63;
  int q = J[p];
  int i0 = p + 1;
  while (i0 < n) {
    const int a0 = i0 & ~3;
    const int e0 = a0 + 4 * lane;
    const int4 v = *reinterpret_cast<const int4*>(J + e0);
    const int vv[4] = {v.x, v.y, v.z, v.w};
    int hit = INT_MAX;
#pragma unroll
    for (int u = 3; u >= 0; --u)
      if (e0 + u >= i0 && e0 + u < n && vv[u] == q) hit = e0 + u;
    const unsigned long long b = __ballot(hit != INT_MAX);
    if (b) {
      q = __shfl(hit, __ffsll((long long)b) - 1);  // the first match: the lowest lane's lowest entry
      i0 = q + 1;
    } else {
      i0 = a0 + 256;
    }
  }
  return q;
}

// "draw the next batch in this launch": an extra workgroup of the assignment kernel runs
// randint(0, n, bs) from `in` into rows / `out` (rows == nullptr: nothing to draw)
struct RngNext {
  const DevMT* in;
  DevMT* out;
  int64_t* rows;
  int64_t n;
  int64_t bs;
};

}  // namespace gdd
