// numpy-compatible random streams on the device (and host).
//
// The reference's epsilon-greedy branch (distr_q.py:314-317) draws from
// ``np.random.default_rng(seed)`` — a PCG64 (XSL-RR 128/64) generator — with
// ``rng.random()`` (53-bit double from one 64-bit output) and
// ``rng.integers(0, 2**31-1)`` (Lemire's method on 32-bit halves that the
// bit generator buffers across calls), then seeds a *fresh* generator for
// gymnasium's ``Discrete.sample(mask)`` through ``SeedSequence(seed)``.  These
// are numpy's published algorithms (numpy/random/src/pcg64/pcg64.h,
// numpy/random/bit_generator.pyx SeedSequence, distributions.c
// buffered_bounded_lemire_uint32), restated here so every env keeps its own
// stream in HBM; tests/test_hostsim.py checks them against numpy itself.
#pragma once
#include <stdint.h>

#ifndef SFL_FN
#if defined(__HIPCC__)
#define SFL_FN __host__ __device__ inline __attribute__((always_inline))
#else
#define SFL_FN inline
#endif
#endif

namespace sfl {

struct Pcg64 {
  uint64_t shi, slo;  // 128-bit state
  uint64_t ihi, ilo;  // 128-bit increment
  uint32_t has;       // has_uint32
  uint32_t buf;       // uinteger
};

SFL_FN uint64_t mulhi64(uint64_t a, uint64_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __umul64hi(a, b);
#else
  return (uint64_t)(((unsigned __int128)a * b) >> 64);
#endif
}

SFL_FN void pcg_step(Pcg64& g) {
  const uint64_t MH = 0x2360ED051FC65DA4ull, ML = 0x4385DF649FCCF645ull;
  uint64_t lo = g.slo * ML;
  uint64_t hi = mulhi64(g.slo, ML) + g.slo * MH + g.shi * ML;
  uint64_t nlo = lo + g.ilo;
  hi += g.ihi + (nlo < lo ? 1ull : 0ull);
  g.slo = nlo;
  g.shi = hi;
}

SFL_FN uint64_t pcg_next64(Pcg64& g) {
  pcg_step(g);
  uint64_t x = g.shi ^ g.slo;
  unsigned rot = (unsigned)(g.shi >> 58);
  return (x >> rot) | (x << ((64u - rot) & 63u));
}

SFL_FN uint32_t pcg_next32(Pcg64& g) {
  if (g.has) {
    g.has = 0;
    return g.buf;
  }
  uint64_t v = pcg_next64(g);
  g.has = 1;
  g.buf = (uint32_t)(v >> 32);
  return (uint32_t)v;
}

SFL_FN double pcg_double(Pcg64& g) { return (double)(pcg_next64(g) >> 11) * (1.0 / 9007199254740992.0); }

// value in [0, rng] (numpy random_bounded_uint64 for rng < 2^32, unmasked)
SFL_FN uint32_t pcg_bounded(Pcg64& g, uint32_t rng) {
  if (rng == 0) return 0;
  if (rng == 0xFFFFFFFFu) return pcg_next32(g);
  const uint32_t excl = rng + 1u;
  uint64_t m = (uint64_t)pcg_next32(g) * excl;
  uint32_t left = (uint32_t)m;
  if (left < excl) {
    const uint32_t thr = (0xFFFFFFFFu - rng) % excl;
    while (left < thr) {
      m = (uint64_t)pcg_next32(g) * excl;
      left = (uint32_t)m;
    }
  }
  return (uint32_t)(m >> 32);
}

// Generator(PCG64(SeedSequence(value))) for a non-negative value < 2^32
SFL_FN void pcg_from_seedseq(uint32_t value, Pcg64& g) {
  uint32_t hc = 0x43b0d7e5u;
  uint32_t pool[4];
  for (int i = 0; i < 4; ++i) {
    uint32_t v = (i == 0) ? value : 0u;
    v ^= hc;
    hc *= 0x931e8875u;
    v *= hc;
    v ^= v >> 16;
    pool[i] = v;
  }
  for (int src = 0; src < 4; ++src) {
    for (int dst = 0; dst < 4; ++dst) {
      if (src == dst) continue;
      uint32_t v = pool[src];
      v ^= hc;
      hc *= 0x931e8875u;
      v *= hc;
      v ^= v >> 16;
      uint32_t r = 0xca01f9ddu * pool[dst] - 0x4973f715u * v;
      r ^= r >> 16;
      pool[dst] = r;
    }
  }
  uint32_t w[8];
  uint32_t hb = 0x8b51f9ddu;
  for (int i = 0; i < 8; ++i) {
    uint32_t d = pool[i & 3];
    d ^= hb;
    hb *= 0x58f38dedu;
    d *= hb;
    d ^= d >> 16;
    w[i] = d;
  }
  const uint64_t s_hi = (uint64_t)w[0] | ((uint64_t)w[1] << 32);
  const uint64_t s_lo = (uint64_t)w[2] | ((uint64_t)w[3] << 32);
  const uint64_t q_hi = (uint64_t)w[4] | ((uint64_t)w[5] << 32);
  const uint64_t q_lo = (uint64_t)w[6] | ((uint64_t)w[7] << 32);
  // pcg_setseq_128_srandom_r(initstate = s, initseq = q)
  g.ihi = (q_hi << 1) | (q_lo >> 63);
  g.ilo = (q_lo << 1) | 1ull;
  g.shi = 0;
  g.slo = 0;
  pcg_step(g);
  uint64_t lo = g.slo + s_lo;
  g.shi = g.shi + s_hi + (lo < g.slo ? 1ull : 0ull);
  g.slo = lo;
  pcg_step(g);
  g.has = 0;
  g.buf = 0;
}

// splitmix-style counter hash for the malfunction draws (oracle/flatland_lite.py mf_draw)
SFL_FN uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

SFL_FN uint64_t mf_draw(uint64_t seed, uint64_t tick, uint64_t handle) {
  return mix64(seed * 0x9E3779B97F4A7C15ull + tick * 0xD1B54A32D192ED03ull + handle * 0x8CB92BA72F3D8DD7ull +
               0x632BE59BD9B4E019ull);
}

}  // namespace sfl
