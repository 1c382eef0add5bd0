// TEST-ONLY host build of the same per-env kernel body (sfl_core.h) behind the
// same C-ABI: libsfl_hostsim.so.  Used by tests/ to check the product
// algorithm against the CPU oracle in a container without a GPU.  Never loaded
// by the product package (network-distributed-q-learning_amd/_lib.py only
// loads libsfl.so and requires a HIP device).
#include <omp.h>
#include <stdlib.h>
#include <string.h>

#include <string>

#include "sfl_engine.h"

namespace {

struct HostBackend {
  static constexpr bool kHasWave = false;  // the host build runs the lane-per-env body only
  std::string err;
  static int device_count(int* n) {
    *n = 0;
    return 0;
  }
  const char* error() const { return err.c_str(); }
  int init(int) { return 0; }
  void* alloc(size_t bytes) { return calloc(1, bytes); }
  void free(void* p) { ::free(p); }
  void h2d(void* d, const void* s, size_t n) { memcpy(d, s, n); }
  void d2h(void* d, const void* s, size_t n) { memcpy(d, s, n); }
  void d2h_async(void* d, const void* s, size_t n) { memcpy(d, s, n); }
  float elapsed_ms() { return 0.f; }
  void memset(void* p, int v, size_t n) { ::memset(p, v, n); }
  void fill_f64(double* p, double v, size_t n) {
    for (size_t i = 0; i < n; ++i) p[i] = v;
  }
  void qinit(const sfl::SflMap& m, const sfl::SflState& s, uint32_t n_rows, const uint32_t* port,
             const uint32_t* state, const double* vals) {
    for (uint32_t e = 0; e < s.E; ++e)
      for (uint32_t r = 0; r < n_rows; ++r) {
        const uint32_t g = port[r], st = state[r];
        const int w = m.q_w[g];
        double* row = s.q + (size_t)e * m.q_per_env + m.q_off[g] + (size_t)st * w;
        for (int j = 0; j < w; ++j) {
          const double v = vals[(size_t)r * 4 + j];
          row[j] = (v != v) ? m.default_q : v;
        }
        const uint32_t rid = m.row_base[g] + st;
        s.touched[(size_t)e * m.touched_words + (rid >> 5)] |= 1u << (rid & 31u);
      }
  }
  int run(const sfl::SflMap& m, const sfl::SflState& s, const sfl::SflCtl& c, int /*variant*/, float* ms) {
#pragma omp parallel for schedule(dynamic, 1)
    for (int64_t e = 0; e < (int64_t)s.E; ++e) {
      if (m.T <= 32) sfl::env_run<1>(m, s, c, (uint32_t)e);
      else if (m.T <= 64) sfl::env_run<2>(m, s, c, (uint32_t)e);
      else sfl::env_run<4>(m, s, c, (uint32_t)e);
    }
    *ms = 0.f;
    return 0;
  }
  int run_ext(const sfl::SflMap& m, const sfl::SflState& s, const sfl::SflCtl& c, float* ms) {
#pragma omp parallel for schedule(dynamic, 1)
    for (int64_t e = 0; e < (int64_t)s.E; ++e) {
      if (m.T <= 32) sfl::env_run_ext<1>(m, s, c, (uint32_t)e);
      else if (m.T <= 64) sfl::env_run_ext<2>(m, s, c, (uint32_t)e);
      else sfl::env_run_ext<4>(m, s, c, (uint32_t)e);
    }
    *ms = 0.f;
    return 0;
  }
  int sync() { return 0; }
  uint64_t n_wait = 0;  // (nothing to wait for: the host build runs on the caller's thread)
  const uint32_t* seedseq_table() { return nullptr; }  // the host build draws every sub-generator
  void reduce_launch(const uint64_t* dec, const uint64_t* ticks, const uint64_t* bytes, const uint32_t* err, uint32_t E,
                     uint64_t* out) {
    out[0] = out[1] = out[2] = out[3] = 0;
    for (uint32_t e = 0; e < E; ++e) {
      out[0] += dec[e];
      out[1] += ticks[e];
      out[2] += bytes[e];
      out[3] |= err[e];
    }
  }
  void replicate(void* base, size_t bytes, uint32_t n) {
    for (uint32_t i = 1; i < n; ++i) memcpy((char*)base + (size_t)i * bytes, base, bytes);
  }
  int part_local(const sfl::SflMap& m, const sfl::SflState& s, const sfl::SflCtl& c, const sfl::SflPart& P, int /*variant*/,
                 float* ms) {
#pragma omp parallel for schedule(dynamic, 1)
    for (int64_t e = 0; e < (int64_t)s.E; ++e) {
      if (m.T <= 32) sfl::env_run_part<1>(m, s, c, P, (uint32_t)e);
      else if (m.T <= 64) sfl::env_run_part<2>(m, s, c, P, (uint32_t)e);
      else sfl::env_run_part<4>(m, s, c, P, (uint32_t)e);
    }
    part_compact(P, s, c);
    *ms = 0.f;
    return 0;
  }
  // k_part_compact (sfl.hip) in env order: each env's staged records into the segments as one group per
  // destination (sfl_part.h env_groups; at most k_msg records per segment: an env with a group past that is
  // deferred whole, its places below the end get void records), the launch totals of the envs that ran,
  // the headers and the checkpoint counts
  static void part_compact(const sfl::SflPart& P, const sfl::SflState& s, const sfl::SflCtl& c) {
    const int W = P.world;
    const uint32_t k = P.k_msg;
    std::vector<uint32_t> nm(W, 0u);
    uint32_t n_open = 0, n_def = 0;
    uint64_t t[4] = {0, 0, 0, 0};
    for (uint32_t e = 0; e < s.E; ++e) {
      const uint32_t flags = s.eflags[e];
      if (!(flags & sfl::F_DEFER)) {
        t[0] += c.launch_dec[e];
        t[1] += c.launch_ticks[e];
        t[2] += c.launch_bytes[e];
      }
      t[3] |= s.err[e];
      const int rd = P.req_dst[e];
      const uint32_t nu = P.upd_n[e];
      int32_t dst[sfl::PART_GROUP_MAX];
      uint32_t pos[sfl::PART_GROUP_MAX], size[sfl::PART_GROUP_MAX], at[sfl::PART_GROUP_MAX];
      for (uint32_t r = 0; r < nu; ++r) dst[r] = P.owner[P.upd_st[(size_t)e * P.upd_env + r].port >> 2];
      const uint32_t n = sfl::env_groups(rd, nu, dst, pos, size, at, [&](int d, uint32_t z) {
        const uint32_t b = nm[d];
        nm[d] += z;
        return b;
      });
      bool fits = true;
      for (uint32_t r = 0; r < n; ++r)
        if (at[r] >= k) fits = false;
      for (uint32_t r = 0; r < n; ++r) {
        sfl::PartMsg& x = P.msg_out[(size_t)dst[r] * (k + 1) + 1 + at[r]];
        if (fits) {
          x = r < nu ? P.upd_st[(size_t)e * P.upd_env + r] : sfl::msg_of_req(P.req_st[e]);
          x.kind |= sfl::msg_tag(size[r], pos[r]);
          if (r == nu) P.req_ix[e] = (uint32_t)dst[r] * (k + 1) + 1u + at[r];
        } else if (at[r] < k) {
          x.genv = 0u;
          x.kind = sfl::MSG_VOID | sfl::msg_tag(1u, 0u);
        }
      }
      if ((bool)(flags & sfl::F_DEFER) == fits) s.eflags[e] = flags ^ sfl::F_DEFER;
      n_open += (rd >= 0 || !fits) ? 1u : 0u;
      n_def += fits ? 0u : 1u;
    }
    uint32_t* co = (uint32_t*)(P.cnt_out + 4);
    for (int g = 0; g < W; ++g) {
      P.msg_out[(size_t)g * (k + 1)].genv = nm[g] < k ? nm[g] : k;
      co[sfl::PART_C_MSG(W) + g] = nm[g];
      co[sfl::PART_C_PEAK(W) + g] = std::max(co[sfl::PART_C_PEAK(W) + g], nm[g]);
    }
    co[sfl::PART_C_OPEN(W)] = n_open;
    co[sfl::PART_C_DEFER(W)] = n_def;
    co[sfl::PART_C_DEFER_SUM(W)] += n_def;
    for (int i = 0; i < 3; ++i) P.cnt_out[i] += t[i];
    P.cnt_out[3] |= t[3];
  }
  int set_stream(void*) { return 0; }  // one host thread: nothing to order
  void part_eblk(const sfl::SflState&, const sfl::SflPart&, int) {}
  void part_caps(const sfl::SflPart&) {}  // (the host build reads the SflPart itself)
  // k_part_owner: every received group by one thread (the groups are independent: one env's records each)
  void part_owner(const sfl::SflMap& m, const sfl::SflPart& P, const sfl::PartMsg* in, sfl::PartRep* out) {
    for (int g = 0; g < P.world; ++g) {
      const size_t base = (size_t)g * (P.k_msg + 1);
      const int64_t n = in[base].genv;
#pragma omp parallel for
      for (int64_t i = 1; i <= n; ++i) {
        const uint32_t len = sfl::msg_group(in[base + i].kind);
        if (sfl::msg_pos(in[base + i].kind) != 0u || sfl::msg_type(in[base + i].kind) == sfl::MSG_VOID) continue;
        sfl::part_owner_group(m, P, in + base + i, len, out + base + i,
                              [&](const sfl::PartReq& r, sfl::PartRep& rep) { sfl::part_answer_one(m, P, r, rep); });
      }
    }
  }
};

}  // namespace

using Backend = HostBackend;
#include "sfl_capi.inc"

// RNG self-test hooks for tests/test_hostsim.py (numpy parity of the device streams)
extern "C" {
int sflh_rng_selftest(uint32_t seedseq_value, uint32_t n, uint64_t* out64, uint32_t* out32, double* outd,
                      uint32_t bound, uint32_t* outb) {
  sfl::Pcg64 g;
  sfl::pcg_from_seedseq(seedseq_value, g);
  for (uint32_t i = 0; i < n; ++i) out64[i] = sfl::pcg_next64(g);
  sfl::pcg_from_seedseq(seedseq_value, g);
  for (uint32_t i = 0; i < n; ++i) out32[i] = sfl::pcg_next32(g);
  sfl::pcg_from_seedseq(seedseq_value, g);
  for (uint32_t i = 0; i < n; ++i) outd[i] = sfl::pcg_double(g);
  sfl::pcg_from_seedseq(seedseq_value, g);
  for (uint32_t i = 0; i < n; ++i) outb[i] = sfl::pcg_bounded(g, bound);
  return 0;
}
// OpenMP threads of the host build (bench.py's CPU baseline runs it on every host core)
int sflh_set_threads(int n) {
  if (n > 0) omp_set_num_threads(n);
  return omp_get_max_threads();
}
// the counter-based malfunction proposal (mf_propose with the map's integer threshold / modulo forms) for n
// (tick, handle) pairs: tests/test_rng.py checks it against the oracle's float compare and 64-bit remainder
int sflh_mf_propose(double rate, int32_t mf_min, int32_t mf_max, uint64_t seed, uint32_t n, const int32_t* ticks,
                    const int32_t* handles, uint32_t* out) {
  sfl::SflMap m{};
  m.mf_rate = rate;
  m.mf_min = mf_min;
  m.mf_max = mf_max;
  m.mf_steps = 0;
  sfl::mf_prepare(m);
  for (uint32_t i = 0; i < n; ++i) out[i] = sfl::mf_propose(m, seed, 0u, ticks[i], handles[i]);
  return 0;
}
int sflh_mf_draw(uint64_t seed, uint64_t tick, uint64_t handle, uint64_t* z) {
  *z = sfl::mf_draw(seed, tick, handle);
  return 0;
}
}
