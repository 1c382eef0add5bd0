// Host-side: the Flatland-compatible malfunction stream.
//
// The reference builds its env with ParamMalfunctionGen(MalfunctionParameters(rate, lo, hi))
// (test_model.py:14-19, main.py:28-33) and resets it with the same seed every episode
// (switch_env.py:99 <- distr_q.py:195, 296).  Flatland (absent here, unpinned in
// requirements.txt:5) then draws, per step and per agent in handle order, from the env's
// np_random -- a legacy numpy RandomState (MT19937) seeded by flatland.utils.seeding.np_random
// (gym's seeding: sha512 of str(seed), the first 8 bytes as two little-endian words,
// init_by_array):
//
//   u = np_random.rand()                                     (two 32-bit outputs)
//   if u < 1 - exp(-rate): n = np_random.randint(lo, hi + 1) + 1   (masked rejection, >= 1 output)
//   else:                  n = 0
//
// Nothing in those draws depends on the trains' dynamics, so the proposals of an episode are a
// pure function of the seed: this file expands them once per env into a [steps][T] byte table
// (num_broken_steps, 0 = none) that the kernels read instead of the counter-based draw.  Before
// the first step the reset consumes the timetable's draws: one randint(0, window) per agent
// (flatland_patch/timetable_generators.py:115).  The rail and line generators are built with
// their own seeds (test_model.py:36-41) and are assumed to draw from their own RandomState.
// Parity with real Flatland is unpinned (no Flatland source or fixture); the stream itself is
// checked against numpy's RandomState in tests/test_mfstream.py.
#pragma once
#include <stdint.h>

namespace sfl {

struct Mt19937 {
  uint32_t key[624];
  int pos;
};

inline void mt_seed(Mt19937& g, uint32_t s) {
  for (int i = 0; i < 624; ++i) {
    g.key[i] = s;
    s = 1812433253u * (s ^ (s >> 30)) + (uint32_t)(i + 1);
  }
  g.pos = 624;
}

// numpy's mt19937_init_by_array (RandomState.seed(list))
inline void mt_init_by_array(Mt19937& g, const uint32_t* init_key, int n) {
  mt_seed(g, 19650218u);
  uint32_t* mt = g.key;
  int i = 1, j = 0;
  for (int k = 624 > n ? 624 : n; k; --k) {
    mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1664525u)) + init_key[j] + (uint32_t)j;
    ++i;
    ++j;
    if (i >= 624) {
      mt[0] = mt[623];
      i = 1;
    }
    if (j >= n) j = 0;
  }
  for (int k = 623; k; --k) {
    mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1566083941u)) - (uint32_t)i;
    ++i;
    if (i >= 624) {
      mt[0] = mt[623];
      i = 1;
    }
  }
  mt[0] = 0x80000000u;
  g.pos = 624;
}

inline void mt_twist(Mt19937& g) {
  uint32_t* k = g.key;
  auto mix = [](uint32_t a, uint32_t b, uint32_t c) {
    const uint32_t y = (a & 0x80000000u) | (b & 0x7FFFFFFFu);
    return c ^ (y >> 1) ^ ((0u - (y & 1u)) & 0x9908B0DFu);
  };
  int i = 0;
  for (; i < 624 - 397; ++i) k[i] = mix(k[i], k[i + 1], k[i + 397]);
  for (; i < 623; ++i) k[i] = mix(k[i], k[i + 1], k[i + 397 - 624]);
  k[623] = mix(k[623], k[0], k[396]);
  g.pos = 0;
}

inline uint32_t mt_next32(Mt19937& g) {
  if (g.pos == 624) mt_twist(g);
  uint32_t y = g.key[g.pos++];
  y ^= y >> 11;
  y ^= (y << 7) & 0x9D2C5680u;
  y ^= (y << 15) & 0xEFC60000u;
  y ^= y >> 18;
  return y;
}

// RandomState.rand()
inline double mt_double(Mt19937& g) {
  const int32_t a = (int32_t)(mt_next32(g) >> 5), b = (int32_t)(mt_next32(g) >> 6);
  return (a * 67108864.0 + b) / 9007199254740992.0;
}

// RandomState.randint(low, high) for high - low - 1 < 2^32: masked rejection on 32-bit outputs
// (numpy random_bounded_uint64_fill, use_masked); a one-value range draws nothing
inline int64_t mt_randint(Mt19937& g, int64_t low, int64_t high) {
  const uint64_t rng = (uint64_t)(high - 1 - low);
  if (rng == 0) return low;
  if (rng == 0xFFFFFFFFull) return low + (int64_t)mt_next32(g);
  uint32_t mask = (uint32_t)rng;
  mask |= mask >> 1;
  mask |= mask >> 2;
  mask |= mask >> 4;
  mask |= mask >> 8;
  mask |= mask >> 16;
  uint32_t v;
  while ((v = mt_next32(g) & mask) > (uint32_t)rng) {
  }
  return low + (int64_t)v;
}

// One env's proposals: key[nkey] the seeding words, windows[n_pre] the timetable's randint(0, w)
// bounds consumed at reset, prob = 1 - exp(-rate), out[steps][T] bytes.  Returns 0, or -1 when a
// proposal does not fit a byte.
inline int mf_schedule_flatland(const uint32_t* key, int nkey, const int32_t* windows, int n_pre, int T, double prob,
                                int32_t lo, int32_t hi, int steps, uint8_t* out) {
  Mt19937 g;
  mt_init_by_array(g, key, nkey);
  for (int i = 0; i < n_pre; ++i) (void)mt_randint(g, 0, windows[i]);
  for (int t = 0; t < steps; ++t)
    for (int h = 0; h < T; ++h) {
      int64_t n = 0;
      if (mt_double(g) < prob) n = mt_randint(g, lo, (int64_t)hi + 1) + 1;
      if (n < 0 || n > 255) return -1;
      out[(size_t)t * T + h] = (uint8_t)n;
    }
  return 0;
}

}  // namespace sfl
