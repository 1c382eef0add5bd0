// Wave-cooperative SwitchFL kernel body (gfx950): one environment per 64-lane wavefront.
//
// Same operations, in the same per-env order, as env_run in sfl_core.h (the lane-per-env
// body, kept for T > 64 and for the host test build), but the env's hot state lives in
// VGPRs for the whole launch:
//   * lane h holds train h (cell, packed bits, plan, ports, delay);
//   * lane p % 64, register p / 64 holds the semaphore record of port p (32-bit packed);
//   * lane s % 64, register s / 64 holds agent_num_interactions of switch s.
// A Flatland tick runs train-parallel (one lane per train); conflict resolution, the
// purge of arrived trains, extend_semaphores and the decision queue are wave ballots and
// per-lane scans of the lanes' own records.  A decision is wave-uniform: cross-lane reads
// are v_readlane, the read-only map tables are scalar loads through the constant cache,
// and only the Q-table, the (switch, train) slots and the distance maps reach L2/HBM.
// Nothing is replicated across envs in a wave, so there is no divergence between envs.
#pragma once
#include <hip/hip_runtime.h>

#include "sfl_core.h"

namespace sfl {
namespace wave {

#define SFL_AS_G __attribute__((address_space(1)))
#define SFL_AS_C __attribute__((address_space(4)))

template <class T, int N>
using vec_t = T __attribute__((ext_vector_type(N)));

// global memory written by this kernel (explicit global address space: no flat accesses)
template <class T>
__device__ __forceinline__ T ld(const T* p, size_t i) {
  return ((const SFL_AS_G T*)p)[i];
}
template <class T>
__device__ __forceinline__ void st(T* p, size_t i, T v) {
  ((SFL_AS_G T*)p)[i] = v;
}
// read-only map tables at a wave-uniform index: scalar loads (K$)
template <class T>
__device__ __forceinline__ T ldc(const T* p, size_t i) {
  return ((const SFL_AS_C T*)p)[i];
}
__device__ __forceinline__ uint32_t ldc_u8(const uint8_t* p, uint32_t i) {
  return (ldc((const uint32_t*)p, i >> 2) >> (8u * (i & 3u))) & 0xFFu;
}
__device__ __forceinline__ uint32_t ldc_u16(const uint16_t* p, uint32_t i) {
  return (ldc((const uint32_t*)p, i >> 1) >> (16u * (i & 1u))) & 0xFFFFu;
}
__device__ __forceinline__ int32_t ldc_i16(const int16_t* p, uint32_t i) {
  return (int32_t)(int16_t)ldc_u16((const uint16_t*)p, i);
}

// wave-uniform values
__device__ __forceinline__ uint32_t uni(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }
__device__ __forceinline__ int32_t uni(int32_t x) { return (int32_t)__builtin_amdgcn_readfirstlane((int)x); }
__device__ __forceinline__ uint64_t uni(uint64_t x) {
  return ((uint64_t)uni((uint32_t)(x >> 32)) << 32) | (uint64_t)uni((uint32_t)x);
}
__device__ __forceinline__ int64_t uni(int64_t x) { return (int64_t)uni((uint64_t)x); }
__device__ __forceinline__ double unid(double x) {
  return __longlong_as_double((long long)uni((uint64_t)__double_as_longlong(x)));
}
__device__ __forceinline__ uint32_t rl(uint32_t v, int lane) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, lane);
}
__device__ __forceinline__ int32_t rl(int32_t v, int lane) { return (int32_t)__builtin_amdgcn_readlane((int)v, lane); }

// semaphore record in a VGPR: t0 11 | t1 11 | owner 8 | in 1 | present 1
__device__ __forceinline__ uint32_t r_pack(uint32_t owner, uint32_t in, int32_t t0, int32_t t1) {
  return ((uint32_t)t0 & 0x7FFu) | (((uint32_t)t1 & 0x7FFu) << 11) | ((owner & 0xFFu) << 22) | ((in & 1u) << 30) |
         (1u << 31);
}
__device__ __forceinline__ bool r_present(uint32_t r) { return (r >> 31) != 0u; }
__device__ __forceinline__ uint32_t r_in(uint32_t r) { return (r >> 30) & 1u; }
__device__ __forceinline__ uint32_t r_owner(uint32_t r) { return (r >> 22) & 0xFFu; }
__device__ __forceinline__ int32_t r_t0(uint32_t r) { return ((int32_t)(r << 21)) >> 21; }
__device__ __forceinline__ int32_t r_t1(uint32_t r) { return ((int32_t)(r << 10)) >> 21; }
__device__ __forceinline__ uint32_t r_from64(uint64_t x) {
  return sem_present(x) ? r_pack(sem_owner(x), sem_in(x), sem_t0(x), sem_t1(x)) : 0u;
}
__device__ __forceinline__ uint64_t r_to64(uint32_t r) {
  return r_present(r) ? sem_pack(r_owner(r), r_in(r), r_t0(r), r_t1(r)) : 0ull;
}

__device__ __forceinline__ int ctz64(uint64_t x) { return __builtin_ctzll(x); }
__device__ __forceinline__ int popc64(uint64_t x) { return __builtin_popcountll(x); }

// PPL semaphore registers (ports <= 64*PPL) and SPL counter registers (switches <= 64*SPL) per lane
template <int PPL, int SPL>
struct WEnv {
  const SflMap& m;
  const SflState& s;
  const uint32_t e, E;
  const int lane;
  const bool mine;  // lane < T: this lane holds train `lane`
  // train `lane`
  int32_t pos;
  uint32_t bits, plan;
  uint32_t nprv;  // next port | prev port << 16
  uint32_t sdec;  // source port | decision switch << 16
  int32_t delay;
  vec_t<uint32_t, PPL> sem;
  vec_t<uint32_t, SPL> cnt;
  uint32_t lerr;  // error bits seen by this lane (OR-reduced on store)
  // wave-uniform env scalars
  int32_t now;
  uint32_t flags, epoch;
  uint64_t q_mask, arr_mask, fl_mask, mf_mask;
  Pcg64 rng;
  double cum;
  int32_t n_mf, ep_dec, ep_ticks;
  int64_t step_ctr, dec_total;

  __device__ WEnv(const SflMap& m_, const SflState& s_, uint32_t e_, int lane_)
      : m(m_), s(s_), e(e_), E(s_.E), lane(lane_), mine(lane_ < m_.T) {}

  __device__ __forceinline__ size_t ix(size_t i) const { return i * (size_t)E + e; }

  // ---- cross-lane access (index wave-uniform) -------------------------------------
  __device__ __forceinline__ uint32_t sget(int p) const { return rl(sem[p >> 6], p & 63); }
  __device__ __forceinline__ void sset(int p, uint32_t r) {
    const int k = p >> 6;
    const bool me = lane == (p & 63);
#pragma unroll
    for (int i = 0; i < PPL; ++i)
      if (i == k) sem[i] = me ? r : sem[i];
  }
  __device__ __forceinline__ uint32_t cget(int sw) const { return rl(cnt[sw >> 6], sw & 63); }
  __device__ __forceinline__ void cset(int sw, uint32_t v) {
    const int k = sw >> 6;
    const bool me = lane == (sw & 63);
#pragma unroll
    for (int i = 0; i < SPL; ++i)
      if (i == k) cnt[i] = me ? v : cnt[i];
  }
  // counter of a per-lane switch index (flush): bpermute per register; call with all lanes active
  __device__ __forceinline__ uint32_t cget_var(int sw) const {
    uint32_t r = 0;
#pragma unroll
    for (int i = 0; i < SPL; ++i) {
      const uint32_t v = (uint32_t)__shfl((int)cnt[i], sw & 63, 64);
      r = (i == (sw >> 6)) ? v : r;
    }
    return r;
  }
  template <class T>
  __device__ __forceinline__ void tset(T& x, int h, T v) {
    x = (lane == h) ? v : x;
  }
  __device__ __forceinline__ uint32_t state_of(int h) const { return tb_state(rl(bits, h)); }

  // ---- grid (U: wave-uniform arguments -> scalar loads) ---------------------------------
  template <bool U>
  __device__ __forceinline__ uint32_t grid_at(int cell) const {
    return U ? ldc_u16(m.grid, (uint32_t)cell) : (uint32_t)ld(m.grid, (size_t)cell);
  }
  __device__ __forceinline__ int move_cell(int cell, int d) const {
    int r = cell / m.W, cc = cell - r * m.W;
    r += (d == 2) - (d == 0);
    cc += (d == 1) - (d == 3);
    if (r < 0 || r >= m.H || cc < 0 || cc >= m.W) return -1;
    return r * m.W + cc;
  }
  struct Move {
    int cell, dir;
    bool valid, cell_ok;
  };
  // flatland-lite check_action_on_agent
  template <bool U>
  __device__ __forceinline__ Move check_action(uint32_t a, int cell, int dir) const {
    const uint32_t nib = (grid_at<U>(cell) >> ((3 - dir) * 4)) & 15u;
    const int n = __builtin_popcount(nib);
    int nd = dir, valid = -1;
    if (a == A_LEFT) {
      nd = dir + 3;
      if (n <= 1) valid = 0;
    } else if (a == A_RIGHT) {
      nd = dir + 1;
      if (n <= 1) valid = 0;
    }
    nd &= 3;
    if (a == A_FWD && n == 1) {
      nd = 3 - (31 - __builtin_clz(nib));
      valid = 1;
    }
    Move mv;
    mv.cell = move_cell(cell, nd);
    mv.dir = nd;
    mv.cell_ok = mv.cell >= 0 && grid_at<U>(mv.cell) != 0;
    mv.valid = valid < 0 ? (((nib >> (3 - nd)) & 1u) != 0) : (valid != 0);
    return mv;
  }
  template <bool U>
  __device__ __forceinline__ bool action_ok(uint32_t a, int cell, int dir) const {
    Move mv = check_action<U>(a, cell, dir);
    return mv.cell_ok && mv.valid;
  }
  // distance map lookup (wave-uniform)
  __device__ __forceinline__ int32_t dist(int h, int cell, int dir) {
    if (cell < 0) {
      lerr |= E_INF_DIST;
      return 0;
    }
    const int32_t k = ldc(m.tr_k, (size_t)h);
    const int32_t d = ldc(m.dist, (((size_t)k * m.H * m.W) + (size_t)cell) * 4 + dir);
    if (d >= DIST_INF) lerr |= E_INF_DIST;
    return d;
  }

  // ---- semaphores (wave-uniform) ----------------------------------------------------------
  // observer.py:44-151 (a record's dir field always equals map_direction(port))
  __device__ __forceinline__ bool port_blocked(int next_p, int out_p, int h) const {
    uint32_t r = sget(next_p);
    if (r_present(r) && r_owner(r) != (uint32_t)h && r_t0(r) <= now && now <= r_t1(r)) {
      if (!r_in(r)) return true;
      if (state_of((int)r_owner(r)) == S_MALF) return true;
    }
    r = sget(out_p);
    if (r_present(r) && r_owner(r) != (uint32_t)h && r_t0(r) <= now && now <= r_t1(r)) {
      if (r_in(r)) return true;
      if (state_of((int)r_owner(r)) == S_MALF) return true;
    }
    return false;
  }
  // set if absent, else (io == ovr_io or t0 in the future) -> retime in place (io kept)
  __device__ __forceinline__ void put_keep(int p, int h, uint32_t in, int32_t span, uint32_t ovr_in) {
    const uint32_t r = sget(p);
    if (!r_present(r)) sset(p, r_pack(h, in, now, now + span));
    else if (r_in(r) == ovr_in || r_t0(r) > now) sset(p, r_pack(h, r_in(r), now, now + span));
  }
  // set if absent, else (ovr_in matches or t0 in the future) -> replace whole record
  __device__ __forceinline__ void put_replace(int p, int h, uint32_t in, int32_t span, int ovr_in) {
    const uint32_t r = sget(p);
    if (!r_present(r) || (ovr_in >= 0 && r_in(r) == (uint32_t)ovr_in) || r_t0(r) > now)
      sset(p, r_pack(h, in, now, now + span));
  }

  // ---- Q-table ------------------------------------------------------------------------------
  __device__ __forceinline__ double* qrow(int sw, int slot, uint32_t state) const {
    const int g = 4 * sw + slot;
    return s.q + (size_t)e * m.q_per_env + ldc(m.q_off, (size_t)g) + (size_t)state * ldc_u8(m.q_w, (uint32_t)g);
  }
  __device__ __forceinline__ void touch(int sw, int slot, uint32_t state) const {
    const uint32_t row = ldc(m.row_base, (size_t)(4 * sw + slot)) + state;
    atomicOr(&s.touched[(size_t)e * m.touched_words + (row >> 5)], 1u << (row & 31u));
  }
  __device__ __forceinline__ double row_val(int sw, int slot, const vec_t<double, 4>& row, int a) const {
    const int na = (int)ldc_u8(m.sw_na, (uint32_t)sw);
    if (a == na - 1) return row[(int)ldc_u8(m.q_w, (uint32_t)(4 * sw + slot)) - 1];
    if ((int)ldc_u8(m.act_src, (uint32_t)(sw * 8 + a)) == slot) return row[(int)ldc_u8(m.act_j, (uint32_t)(sw * 8 + a))];
    return m.default_q;
  }
  __device__ __forceinline__ double lr_of(uint32_t n) const {
    return n < (uint32_t)m.ntab ? ldc(m.lr_tab, (size_t)n) : m.lr0 * pow(m.lr_decay, (double)n);
  }
  __device__ __forceinline__ double lr_of_var(uint32_t n) const {
    return n < (uint32_t)m.ntab ? ld(m.lr_tab, (size_t)n) : m.lr0 * pow(m.lr_decay, (double)n);
  }

  // ---- launch-boundary state transfer ---------------------------------------------------------
  __device__ __forceinline__ void load() {
    if (mine) {
      pos = ld(s.tr_pos, ix(lane));
      bits = ld(s.tr_bits, ix(lane));
      plan = ld(s.tr_plan, ix(lane));
      nprv = (uint32_t)ld(s.tr_next, ix(lane)) | ((uint32_t)ld(s.tr_prev, ix(lane)) << 16);
      sdec = (uint32_t)ld(s.tr_src, ix(lane)) | ((uint32_t)ld(s.tr_dec, ix(lane)) << 16);
      delay = ld(s.tr_delay, ix(lane));
    } else {
      pos = -1;
      bits = 0;
      plan = 0;
      nprv = 0xFFFFFFFFu;
      sdec = 0xFFFFFFFFu;
      delay = 0;
    }
#pragma unroll
    for (int k = 0; k < PPL; ++k) {
      const int p = k * 64 + lane;
      sem[k] = p < m.NP ? r_from64(ld(s.sem, ix(p))) : 0u;
    }
#pragma unroll
    for (int k = 0; k < SPL; ++k) {
      const int sw = k * 64 + lane;
      cnt[k] = sw < m.S ? ld(s.counts, ix(sw)) : 0u;
    }
    now = uni(ld(s.elapsed, e));
    flags = uni(ld(s.eflags, e));
    epoch = uni(ld(s.epoch, e));
    lerr = uni(ld(s.err, e));
    auto mask = [&](int k) {
      return uni((uint64_t)ld(s.masks, (size_t)(k * MAXW + 0) * E + e) |
                 ((uint64_t)ld(s.masks, (size_t)(k * MAXW + 1) * E + e) << 32));
    };
    q_mask = mask(0);
    arr_mask = mask(1);
    fl_mask = mask(2);
    mf_mask = mask(3);
    rng.shi = uni(ld(s.rng, ix(0)));
    rng.slo = uni(ld(s.rng, ix(1)));
    rng.ihi = uni(ld(s.rng, ix(2)));
    rng.ilo = uni(ld(s.rng, ix(3)));
    const uint64_t hb = uni(ld(s.rng, ix(4)));
    rng.has = (uint32_t)(hb >> 32);
    rng.buf = (uint32_t)hb;
    cum = unid(ld(s.cum_reward, e));
    n_mf = uni(ld(s.n_mf, e));
    ep_dec = uni(ld(s.ep_dec, e));
    ep_ticks = uni(ld(s.ep_ticks, e));
    step_ctr = uni(ld(s.step_ctr, e));
    dec_total = uni(ld(s.dec_total, e));
  }
  __device__ __forceinline__ void store(int32_t phase) {
    if (mine) {
      st(s.tr_pos, ix(lane), pos);
      st(s.tr_bits, ix(lane), bits);
      st(s.tr_plan, ix(lane), plan);
      st(s.tr_next, ix(lane), (uint16_t)(nprv & 0xFFFFu));
      st(s.tr_prev, ix(lane), (uint16_t)(nprv >> 16));
      st(s.tr_src, ix(lane), (uint16_t)(sdec & 0xFFFFu));
      st(s.tr_dec, ix(lane), (uint16_t)(sdec >> 16));
      st(s.tr_delay, ix(lane), delay);
    }
#pragma unroll
    for (int k = 0; k < PPL; ++k) {
      const int p = k * 64 + lane;
      if (p < m.NP) st(s.sem, ix(p), r_to64(sem[k]));
    }
#pragma unroll
    for (int k = 0; k < SPL; ++k) {
      const int sw = k * 64 + lane;
      if (sw < m.S) st(s.counts, ix(sw), cnt[k]);
    }
    uint32_t err = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b)
      if (__ballot((lerr >> b) & 1u)) err |= 1u << b;
    if (lane == 0) {
      st(s.phase, e, phase);
      st(s.elapsed, e, now);
      st(s.eflags, e, flags);
      st(s.epoch, e, epoch);
      st(s.err, e, err);
      st(s.masks, (size_t)(0 * MAXW + 0) * E + e, (uint32_t)q_mask);
      st(s.masks, (size_t)(0 * MAXW + 1) * E + e, (uint32_t)(q_mask >> 32));
      st(s.masks, (size_t)(1 * MAXW + 0) * E + e, (uint32_t)arr_mask);
      st(s.masks, (size_t)(1 * MAXW + 1) * E + e, (uint32_t)(arr_mask >> 32));
      st(s.masks, (size_t)(2 * MAXW + 0) * E + e, (uint32_t)fl_mask);
      st(s.masks, (size_t)(2 * MAXW + 1) * E + e, (uint32_t)(fl_mask >> 32));
      st(s.masks, (size_t)(3 * MAXW + 0) * E + e, (uint32_t)mf_mask);
      st(s.masks, (size_t)(3 * MAXW + 1) * E + e, (uint32_t)(mf_mask >> 32));
      st(s.rng, ix(0), rng.shi);
      st(s.rng, ix(1), rng.slo);
      st(s.rng, ix(4), ((uint64_t)rng.has << 32) | rng.buf);
      st(s.cum_reward, e, cum);
      st(s.n_mf, e, n_mf);
      st(s.ep_dec, e, ep_dec);
      st(s.ep_ticks, e, ep_ticks);
      st(s.step_ctr, e, step_ctr);
      st(s.dec_total, e, dec_total);
    }
  }

  // ---- episode reset (switch_env.py:93-158, _init_ports 507-568) --------------------------------
  __device__ __forceinline__ void reset() {
    now = 0;
    if (mine) {
      pos = -1;
      bits = tb_make(ld(m.tr_init_dir, lane), S_WAITING, A_NONE, 0, 0, 0);
      plan = 0;
      nprv = (nprv & 0xFFFF0000u) | (uint32_t)(uint16_t)ld(m.tr_init_port, lane);
      delay = ld(m.tr_init_delay, lane);
    }
    sem = 0u;
    for (int h = 0; h < m.T; ++h) {
      const int32_t ed = ldc(m.tr_ed, (size_t)h);
      sset(ldc_i16(m.tr_init_port, (uint32_t)h), r_pack(h, 1, ed - 2, ed + ldc(m.tr_init_dist, (size_t)h)));
    }
    flags &= ~(F_TERM | F_TRUNC | F_OWN_SCAN | F_INFLIGHT);
    q_mask = arr_mask = fl_mask = mf_mask = 0;
    // new (switch, train) epoch: slots from older episodes read as empty
    epoch = (epoch + 1u) & 0xFFu;
    if (epoch == 0) {
      for (int i = lane; i < m.S * m.T; i += 64) st(s.slot, ix(i), slot_make(PEND_NONE, 0, 0));
      epoch = 1;
    }
    cum = 0.0;
    n_mf = 0;
    ep_dec = 0;
    ep_ticks = 0;
    step_ctr = 0;
  }

  // ---- one Flatland tick + switchfl bookkeeping (switch_env.py:296-401, 427-485;
  //      flatland_lite.RailEnv.step), train-parallel: lane h = train h ----------------------------
  __device__ __forceinline__ void tick() {
    const int32_t t = ++now;
    const uint64_t seed = s.seed[e];
    const int h = lane;
    // pass 1: plan pop + prediction, malfunction draw, action preprocessing, desired move
    bool mover = false;
    int32_t desired = -1, pred = -1;
    uint32_t aux = 0;
    int32_t t_init_cell = 0, t_target = -1, t_ed = 0;
    uint32_t t_init_dir = 0;
    if (mine) {
      t_init_cell = ld(m.tr_init_cell, h);
      t_init_dir = ld(m.tr_init_dir, h);
      t_target = ld(m.tr_target, h);
      t_ed = ld(m.tr_ed, h);
      const uint32_t b = bits;
      const int32_t p0 = pos;
      uint32_t st_ = tb_state(b), dir = tb_dir(b), prev = tb_prev(b), saved = tb_saved(b), mf = tb_mf(b);
      uint32_t given = A_NOTHING;
      pred = p0;
      if (!tb_done(b)) {
        const uint32_t pl = plan;
        if (pl_len(pl) == 0) {
          given = A_FWD;
        } else {
          given = pl_front(pl);
          prev = given;
          plan = pl_pop(pl);
        }
        if (p0 >= 0) {
          Move mv = check_action<false>(given, p0, (int)dir);
          aux |= 1u << 12;
          if (mv.valid) {
            aux |= 1u << 13;
            pred = mv.cell;
          }
        }
      }
      if (st_ != S_DONE && mf == 0 && m.mf_rate > 0.0) {
        const uint64_t z = mf_draw(seed, (uint64_t)t, (uint64_t)h);
        const double u = (double)(z >> 11) * (1.0 / 9007199254740992.0);
        if (u < m.mf_rate)
          mf = (uint32_t)(m.mf_min + (int32_t)(mix64(z ^ 0xA0761D6478BD642Full) % (uint64_t)(m.mf_max - m.mf_min + 1))) + 1u;
      }
      // preprocess_action
      uint32_t pa = given;
      if (pa == A_NOTHING && st_ == S_MOVING) pa = A_FWD;
      if (st_ == S_WAITING) pa = A_NOTHING;
      const int pc = p0 >= 0 ? p0 : t_init_cell;
      const int pd = p0 >= 0 ? (int)dir : (int)t_init_dir;
      if ((pa == A_LEFT || pa == A_RIGHT) && !action_ok<false>(pa, pc, pd)) pa = A_FWD;
      if (is_moving_action(pa) && !action_ok<false>(pa, pc, pd)) pa = A_STOP;
      if (is_moving_action(pa) && saved == 0 && st_ != S_DONE) saved = pa;
      const bool update_allowed = (mf == 0) && pa != A_STOP;
      desired = p0;
      uint32_t ddir = dir;
      if (st_ == S_DONE) {
      } else if (p0 < 0 && saved != 0) {
        desired = t_init_cell;
        ddir = t_init_dir;
        mover = true;
      } else if (saved != 0 && update_allowed) {
        Move mv = check_action<false>(saved, p0, (int)dir);
        desired = mv.cell;
        ddir = (uint32_t)mv.dir;
        pa = saved;
        mover = desired != p0;
      }
      aux |= pa | (ddir << 4) | (given << 8);
      bits = tb_make(dir, st_, prev, saved, mf, tb_done(b));
    }
    // pass 2: motion check, least fixed point (flatland_lite.motion_check): the lowest handle
    // wanting a cell wins it; a cell can be entered if free or its occupant moves out
    const uint64_t M = __ballot(mover);
    uint64_t A = 0;
    if (M) {
      bool win = mover;
      int occ = -1;
      uint64_t cand_j = M | __ballot(pos >= 0);
      while (cand_j) {
        const int j = ctz64(cand_j);
        cand_j &= cand_j - 1ull;
        const int32_t dj = rl(desired, j);
        const int32_t pj = rl(pos, j);
        if (mover) {
          if (((M >> j) & 1ull) && j < h && dj == desired) win = false;
          if (pj >= 0 && pj == desired && j != h) occ = j;
        }
      }
      while (true) {
        const bool cand = mover && win && !((A >> h) & 1ull) &&
                          (occ < 0 || (((M >> occ) & 1ull) && ((A >> occ) & 1ull)));
        const uint64_t nb = __ballot(cand);
        if (!nb) break;
        A |= nb;
      }
    }
    // pass 3: state machine + positions, deviation fix
    const bool over = t >= m.max_episode_steps;
    bool done = false, isdone = !mine, newly = false, dep = false;
    if (mine) {
      const uint32_t b = bits;
      const int32_t p0 = pos;
      uint32_t st_ = tb_state(b), dir = tb_dir(b), saved = tb_saved(b), mf = tb_mf(b);
      const uint32_t pa = aux & 15u;
      const bool in_mf = mf > 0;
      bool ma = in_mf ? false : (mover && ((A >> h) & 1ull));
      const bool valid_move = is_moving_action(pa) && ma;
      const bool ed_reached = t >= t_ed;
      const uint32_t prev_st = st_;
      switch (st_) {
        case S_WAITING: st_ = in_mf ? S_MF_OFF : (ed_reached ? S_READY : S_WAITING); break;
        case S_READY: st_ = in_mf ? S_MF_OFF : (valid_move ? S_MOVING : S_READY); break;
        case S_MF_OFF: st_ = (mf == 0) ? (ed_reached ? S_READY : S_WAITING) : S_MF_OFF; break;
        case S_MOVING:
          if (in_mf) st_ = S_MALF;
          else if (pa == A_STOP) st_ = S_STOPPED;
          else if (p0 >= 0 && p0 == t_target) st_ = S_DONE;
          else if (!ma) st_ = S_STOPPED;
          break;
        case S_STOPPED: st_ = in_mf ? S_MALF : (valid_move ? S_MOVING : S_STOPPED); break;
        case S_MALF: st_ = (mf == 0) ? (valid_move ? S_MOVING : S_STOPPED) : S_MALF; break;
        default: break;
      }
      ma = ma && st_ != S_DONE;
      int32_t np = p0;
      if (on_map_state(st_)) {
        if (off_map_state(prev_st)) {
          np = t_init_cell;
          dir = t_init_dir;
        } else if (ma) {
          np = desired;
          dir = (aux >> 4) & 3u;
          if (np == t_target) st_ = S_DONE;
        }
      }
      if (st_ == S_DONE && !((arr_mask >> h) & 1ull)) {
        newly = true;  // arrived: position None, arrival_time set
        np = -1;
      }
      if (mf > 0) mf -= 1;
      if (np >= 0) saved = 0;
      done = (st_ == S_DONE) || over;
      isdone = st_ == S_DONE;
      pos = np;
      // switchfl: deviation fix
      if ((aux >> 12) & 1u) {
        const uint32_t given = (aux >> 8) & 15u;
        if (pred != np && ((aux >> 13) & 1u) && given != A_STOP) {
          plan = pl_push_front(plan, given, lerr);
          if (ld(m.cell_sw, (size_t)pred) >= 0) nprv = (nprv & 0xFFFF0000u) | (sdec & 0xFFFFu);
        }
      }
      dep = t == t_ed - 2;
      bits = tb_make(dir, st_, tb_prev(b), saved, mf, done ? 1u : 0u);
    }
    arr_mask |= __ballot(newly);
    // delete the semaphores of done trains (switch_env.py:370-376): each lane its own records
    const uint64_t DONE = __ballot(done);
    if (DONE) {
#pragma unroll
      for (int k = 0; k < PPL; ++k)
        if (r_present(sem[k]) && ((DONE >> r_owner(sem[k])) & 1ull)) sem[k] = 0u;
    }
    // departure semaphores, in handle order (switch_env.py:379-384)
    uint64_t D = __ballot(dep);
    while (D) {
      const int j = ctz64(D);
      D &= D - 1ull;
      const int32_t ed = ldc(m.tr_ed, (size_t)j);
      sset((int)(rl(nprv, j) & 0xFFFFu), r_pack(j, 1, ed - 2, ed + ldc(m.tr_init_dist, (size_t)j)));
    }
    // pass 4: extend_semaphores (rail_network.py:229-244)
    const uint32_t st4 = tb_state(bits);
    const uint64_t SM = __ballot(mine && (st4 == S_STOPPED || st4 == S_MALF));
    if (SM) {
#pragma unroll
      for (int k = 0; k < PPL; ++k) {
        const uint32_t r = sem[k];
        if (r_present(r) && ((SM >> r_owner(r)) & 1ull)) sem[k] = r_pack(r_owner(r), r_in(r), t, t + (r_t1(r) - r_t0(r)));
      }
    }
    uint64_t MA = __ballot(mine && st4 == S_MALF);
    while (MA) {
      const int j = ctz64(MA);
      MA &= MA - 1ull;
      const int p = (int)(rl(nprv, j) & 0xFFFFu);
      if (!r_present(sget(p))) sset(p, r_pack(j, 1, t, t + ldc(m.tr_init_dist, (size_t)j)));
    }
    // malfunction count (switch_env.py:399-401)
    const uint64_t MF = __ballot(mine && tb_mf(bits) > 0);
    n_mf += popc64(MF & ~mf_mask);
    mf_mask = MF;
    // _check_active_switch (switch_env.py:427-485)
    bool act = false;
    if (mine && pos >= 0 && st4 != S_WAITING) {
      const uint32_t nxt = pl_len(plan) ? pl_front(plan) : A_FWD;
      Move mv = check_action<false>(nxt, pos, (int)tb_dir(bits));
      if (mv.cell >= 0) {
        const int sw_at = ld(m.cell_sw, (size_t)mv.cell);
        if (sw_at >= 0) {
          int sw = -1;
          if (st4 == S_READY || st4 == S_MOVING) sw = sw_at;
          else if ((st4 == S_STOPPED || st4 == S_MALF) && tb_prev(bits) == A_STOP) sw = sw_at;
          else if (st4 == S_STOPPED || st4 == S_MALF) sw = (int)((nprv & 0xFFFFu) >> 2);
          if (sw >= m.S) {  // next port is None: the reference would raise here
            lerr |= E_PORT;
          } else if (sw >= 0) {
            act = true;
            sdec = (sdec & 0xFFFFu) | ((uint32_t)sw << 16);
          }
        }
      }
    }
    q_mask = __ballot(act);
    const uint64_t full = (m.T == 64) ? ~0ull : ((1ull << m.T) - 1ull);
    const uint64_t ALL = __ballot(isdone);
    ep_ticks += 1;
    if ((ALL & full) == full || over) flags |= F_TERM;
  }

  // ---- decision (wave-uniform): observe (observer.py:246-308), epsilon-greedy
  //      (distr_q.py:312-319), _apply_action (switch_env.py:203-294) ---------------------------
  struct Dec {
    int sw, h, slot;
    uint32_t state;
    int action, j;
    int32_t reward, r_new;
    int next_sw;
    uint64_t slotword;
    vec_t<double, 4> row;
  };

  __device__ __forceinline__ void decide(Dec& d, bool greedy) {
    // agent_iter: lowest queued train (switch_env.py:418-421, 616-622)
    const int h = ctz64(q_mask);
    q_mask &= q_mask - 1ull;
    const uint32_t sd = rl(sdec, h);
    const int sw = (int)(sd >> 16);
    const int np = (int)ldc_u8(m.sw_np, (uint32_t)sw);
    const int na = (int)ldc_u8(m.sw_na, (uint32_t)sw);
    const uint32_t npv = rl(nprv, h);
    const int pin = (int)(npv & 0xFFFFu);
    const int pprev = (int)(npv >> 16);
    int slot = pin & 3;
    if ((pin >> 2) != sw || slot >= np) {  // observer.py:294-301 (the reference would raise)
      lerr |= E_PORT;
      slot = 0;
    }
    d.slotword = uni(ld(s.slot, ix((size_t)sw * m.T + h)));
    // observe
    uint32_t free_bits = 0;
    for (int j = 0; j < np; ++j) {
      const int p = 4 * sw + j;
      if (!port_blocked(ldc_i16(m.port_nb, (uint32_t)p), p, h)) free_bits |= 1u << j;
    }
    const uint32_t b = rl(bits, h);
    const int32_t p0 = rl(pos, h);
    const int32_t la = ldc(m.tr_la, (size_t)h);
    const int32_t dl = now - la + dist(h, p0, (int)tb_dir(b));
    const int32_t avail = la - ldc(m.tr_ed, (size_t)h);
    const uint32_t lvl = dl <= 0 ? 0u : (dl <= avail * 20 ? 1u : 2u);
    const uint32_t state = ((free_bits * (uint32_t)m.K) + (uint32_t)ldc(m.tr_k, (size_t)h)) * 3u + lvl;
    uint32_t amask = 1u << (na - 1);
    for (int a = 0; a < na - 1; ++a)
      if ((int)ldc_u8(m.act_src, (uint32_t)(sw * 8 + a)) == slot &&
          ((free_bits >> ldc_u8(m.act_dst, (uint32_t)(sw * 8 + a))) & 1u))
        amask |= 1u << a;
    const int w = (int)ldc_u8(m.q_w, (uint32_t)(4 * sw + slot));
    const double* rp = qrow(sw, slot, state);
#pragma unroll
    for (int j = 0; j < 4; ++j) d.row[j] = j < w ? unid(ld(rp, (size_t)j)) : 0.0;
    const int32_t reward = slot_rew(d.slotword, epoch);
    // epsilon-greedy
    int action = -1;
    bool explore = false;
    if (!greedy) {
      const uint32_t n = cget(sw);
      const double eps = n < (uint32_t)m.ntab ? ldc(m.eps_tab, (size_t)n) : m.eps0 * pow(m.eps_decay, (double)n);
      if (pcg_double(rng) < eps) {
        explore = true;
        const uint32_t sub_seed = pcg_bounded(rng, 2147483646u);
        Pcg64 sub;
        pcg_from_seedseq(sub_seed, sub);
        const uint32_t nvalid = (uint32_t)__builtin_popcount(amask);
        const uint32_t pick = pcg_bounded(sub, nvalid - 1u);
        uint32_t mk = amask;
        for (uint32_t k = 0; k < pick; ++k) mk &= mk - 1u;
        action = __builtin_ctz(mk);
      }
    }
    if (!explore) {
      if (lane == 0) touch(sw, slot, state);
      // np.argmax over the full row, falling back to the first allowed maximum (distr_q.py:468-490)
      int best = 0;
      double mx = row_val(sw, slot, d.row, 0);
      for (int a = 1; a < na; ++a) {
        const double v = row_val(sw, slot, d.row, a);
        if (v > mx) {
          mx = v;
          best = a;
        }
      }
      if ((amask >> best) & 1u) {
        action = best;
      } else {
        double amx = 0.0;
        for (int a = 0; a < na; ++a) {
          if (!((amask >> a) & 1u)) continue;
          const double v = row_val(sw, slot, d.row, a);
          if (action < 0 || v > amx) {
            action = a;
            amx = v;
          }
        }
      }
    }
    if (action < 0 || action >= na) lerr |= E_BAD_ACTION;
    // _apply_action
    const int stop = na - 1;
    bool moving = false;
    uint32_t turn = A_FWD;
    int in_p = pin, out_p = pin;
    if (action != stop && (pin >> 2) == sw) {
      const int src = (int)ldc_u8(m.act_src, (uint32_t)(sw * 8 + action));
      if (src == slot) {
        moving = true;
        turn = ldc_u8(m.act_turn, (uint32_t)(sw * 8 + action));
        in_p = 4 * sw + src;
        out_p = 4 * sw + (int)ldc_u8(m.act_dst, (uint32_t)(sw * 8 + action));
      }
    }
    int next_sw = sw, target = -1;
    if (moving) {
      // transition_train / transition_semaphore (rail_network.py:246-278, 303-416)
      target = ldc_i16(m.port_nb, (uint32_t)out_p);
      if (tb_state(b) != S_MALF) {
        // free the train's records on the ports of its current and previous switch
        const int x1 = pin >> 2;
        const int x2 = pprev != (int)PORT_NONE ? (pprev >> 2) : -1;
#pragma unroll
        for (int k = 0; k < PPL; ++k) {
          const int x = (k * 64 + lane) >> 2;
          if ((x == x1 || x == x2) && r_present(sem[k]) && r_owner(sem[k]) == (uint32_t)h) sem[k] = 0u;
        }
      }
      const int32_t d_ot = ldc_i16(m.port_len, (uint32_t)out_p);
      put_keep(out_p, h, 0, 3, 0);
      put_keep(target, h, 1, d_ot + 1, 1);
      const int u = ldc_i16(m.port_unique, (uint32_t)target);
      if (u >= 0) {
        if (u != in_p && u != out_p && u != target) put_replace(u, h, 0, d_ot + 1, 0);
        put_replace(u, h, 0, d_ot, -1);
        const int far = ldc_i16(m.port_nb, (uint32_t)u);
        if (far != in_p && far != out_p && far != u)
          put_replace(far, h, 1, d_ot + ldc_i16(m.port_len, (uint32_t)u) + 1, 1);
      }
      if (target != in_p && target != out_p) put_replace(target, h, 0, d_ot + 1, 0);
      tset(sdec, h, (sd & 0xFFFF0000u) | (uint32_t)in_p);
      tset(nprv, h, (uint32_t)target | ((uint32_t)out_p << 16));
      next_sw = target >> 2;
    }
    uint32_t p = rl(plan, h);
    if (moving && pl_len(p) > 0) {
      p = (p & 0xF0u) | 1u;  // plan[:1]
      p = pl_push_back(p, turn, lerr);
    } else if (!moving) {
      p = pl_push_front(p, A_STOP, lerr);
    } else {
      p = pl_push_back(p, A_FWD, lerr);
      p = pl_push_back(p, turn, lerr);
    }
    tset(plan, h, p);
    bool all_blocked;
    if (moving) {
      all_blocked = port_blocked(target, out_p, h);
    } else {
      all_blocked = true;
      for (int a = 0; a < na - 1; ++a) {
        if ((int)ldc_u8(m.act_src, (uint32_t)(sw * 8 + a)) != slot) continue;
        const int o = 4 * sw + (int)ldc_u8(m.act_dst, (uint32_t)(sw * 8 + a));
        if (!port_blocked(ldc_i16(m.port_nb, (uint32_t)o), o, h)) all_blocked = false;
      }
    }
    // reward_func.py:23-78: project the position along the non-STOP plan
    int pc = p0, pd = (int)tb_dir(b);
    const uint32_t nn = pl_len(p);
    for (uint32_t i = 0; i < nn; ++i) {
      const uint32_t a = pl_at(p, i);
      if (a == A_STOP) continue;
      if (pc < 0) break;
      Move mv = check_action<true>(a, pc, pd);
      pc = mv.cell;
      pd = mv.dir;
    }
    const int32_t cur = now - la + dist(h, pc, pd);
    const int32_t diff = rl(delay, h) - cur;
    d.r_new = (pl_front(p) == A_STOP && !all_blocked) ? diff - 1300 : diff;
    tset(delay, h, cur);
    d.sw = sw;
    d.h = h;
    d.slot = slot;
    d.state = state;
    d.action = action;
    d.j = (action == stop) ? (w - 1) : (int)ldc_u8(m.act_j, (uint32_t)(sw * 8 + action));
    d.reward = reward;
    d.next_sw = next_sw;
  }

  // ---- post-step part of the learn loop (distr_q.py:322-362) -----------------------------------
  // The (switch, train) slot of the deciding switch is consumed and the successor slot gets
  // the new pending update and the reward the train will see there (AECEnv.last).
  __device__ __forceinline__ void post(const Dec& d, bool greedy) {
    const int T = m.T;
    if (greedy) {
      if (lane == 0) st(s.slot, ix((size_t)d.next_sw * T + d.h), slot_make(PEND_NONE, d.r_new, epoch));
      return;
    }
    const uint32_t pend = slot_pend(d.slotword, epoch);
    if (pend != PEND_NONE) {
      const int ps = (int)(pend & 0xFFFu);
      const int pslot = (int)((pend >> 12) & 3u);
      const uint32_t pstate = (pend >> 14) & 0x3FFFu;
      const int pj = (int)((pend >> 28) & 3u);
      const double lr = lr_of(cget(ps));
      double* qp = qrow(ps, pslot, pstate) + pj;
      const double qv = unid(ld(qp, 0));
      const double r = (double)d.reward;
      double nv;
      if (d.sw != ps) {
        // max(row) over the full, unmasked successor row (distr_q.py:449-466)
        const int na = (int)ldc_u8(m.sw_na, (uint32_t)d.sw);
        double mq = row_val(d.sw, d.slot, d.row, 0);
        for (int a = 1; a < na; ++a) {
          const double v = row_val(d.sw, d.slot, d.row, a);
          mq = v > mq ? v : mq;
        }
        const double a1 = (1.0 - lr) * qv;
        const double b1 = lr * (r + m.gamma * mq);
        nv = a1 + b1;
      } else {
        const double a1 = (1.0 - lr) * qv;
        const double b1 = lr * r;
        nv = a1 + b1;
      }
      if (lane == 0) {
        st(qp, 0, nv);
        touch(ps, pslot, pstate);
        if (d.sw != ps) touch(d.sw, d.slot, d.state);
      }
    }
    if (lane == 0) {
      st(s.slot, ix((size_t)d.sw * T + d.h), slot_make(PEND_NONE, slot_rew(d.slotword, epoch), epoch));
      st(s.slot, ix((size_t)d.next_sw * T + d.h),
         slot_make(pend_make((uint32_t)d.sw, (uint32_t)d.slot, d.state, (uint32_t)d.j), d.r_new, epoch));
    }
    // destination bonus for newly arrived trains (distr_q.py:344-356); lanes take switches.
    // Distinct slots of one train never hold the same Q cell (same cell => same action =>
    // same successor switch => same slot), so the lanes' updates are independent.
    uint64_t fresh = arr_mask & ~fl_mask;
    fl_mask |= fresh;
    while (fresh) {
      const int tr = ctz64(fresh);
      fresh &= fresh - 1ull;
      for (int base = 0; base < m.S; base += 64) {
        const int sw2 = base + lane;
        const bool valid = sw2 < m.S;
        const uint64_t slw = valid ? ld(s.slot, ix((size_t)sw2 * T + tr)) : 0ull;
        const uint32_t pe = valid ? slot_pend(slw, epoch) : PEND_NONE;
        const int ps = pe == PEND_NONE ? 0 : (int)(pe & 0xFFFu);
        const uint32_t n = cget_var(ps);  // all lanes active: a bpermute reads 0 from inactive lanes
        if (pe == PEND_NONE) continue;
        const int pslot = (int)((pe >> 12) & 3u);
        const uint32_t pstate = (pe >> 14) & 0x3FFFu;
        const int pj = (int)((pe >> 28) & 3u);
        const double lr = lr_of_var(n);
        const int g = 4 * ps + pslot;
        double* qp = s.q + (size_t)e * m.q_per_env + ld(m.q_off, (size_t)g) + (size_t)pstate * ld(m.q_w, (size_t)g) + pj;
        const double a1 = (1.0 - lr) * ld(qp, 0);
        const double b1 = lr * (1000.0 + m.gamma * 0.0);
        st(qp, 0, a1 + b1);
        const uint32_t row = ld(m.row_base, (size_t)g) + pstate;
        atomicOr(&s.touched[(size_t)e * m.touched_words + (row >> 5)], 1u << (row & 31u));
        st(s.slot, ix((size_t)sw2 * T + tr), slot_make(PEND_NONE, slot_rew(slw, epoch), epoch));
      }
    }
    cset(d.sw, cget(d.sw) + 1u);
  }

  // order-independent checksum of the semaphore table (trace/debug only)
  __device__ __forceinline__ uint64_t sem_checksum() const {
    uint64_t c0 = 0;
#pragma unroll
    for (int k = 0; k < PPL; ++k) {
      const int p = k * 64 + lane;
      if (p < m.NP && r_present(sem[k])) c0 += mix64(((uint64_t)p << 42) ^ r_to64(sem[k]));
    }
    for (int off = 1; off < 64; off <<= 1) c0 += (uint64_t)__shfl_xor((long long)c0, off, 64);
    return c0;
  }
};

// driver: one env per wavefront until its episode target / decision budget (env_run in sfl_core.h)
template <int PPL, int SPL>
__device__ void run(const SflMap& m, const SflState& s, const SflCtl& c) {
  using V = WEnv<PPL, SPL>;
  const int lane = (int)__lane_id();
  const uint32_t e = uni((uint32_t)((blockIdx.x * blockDim.x + threadIdx.x) >> 6));
  if (e >= s.E) return;
  V v(m, s, e, lane);
  v.load();
  int32_t phase = uni(ld(s.phase, e));
  int32_t ep_t = uni(ld(s.ep_t, e)), n_test = uni(ld(s.n_test, e));
  uint64_t dec = 0, ticks = 0, abytes = 0;
  typename V::Dec d;
  d.sw = d.h = d.slot = d.action = d.j = d.reward = d.r_new = d.next_sw = 0;
  d.state = 0;
  d.slotword = 0;
  d.row = 0.0;
  const bool test_mode = c.mode == 1;
  while (true) {
    if (phase == PH_RESET) {
      // learn: optional greedy round before episode t (distr_q.py:278-281)
      if (test_mode) {
        if (c.ep_target >= 0 && n_test >= c.ep_target) break;
        v.flags |= F_GREEDY;
      } else {
        if (c.ep_target >= 0 && ep_t >= c.ep_target) break;
        if (c.exploit_freq > 0 && (ep_t + 1) % c.exploit_freq == 0 && !(v.flags & F_EXPLOIT_DONE)) v.flags |= F_GREEDY;
        else v.flags &= ~F_GREEDY;
      }
      v.reset();
      phase = PH_TICK;
    } else if (phase == PH_TICK) {
      abytes += 36ull * (uint64_t)(m.T - popc64(v.arr_mask));
      v.tick();
      ticks++;
      if (v.flags & F_TERM) phase = (v.flags & F_INFLIGHT) ? PH_POST : PH_END;
      else if (v.q_mask) phase = (v.flags & F_INFLIGHT) ? PH_POST : PH_DECIDE;
    } else if (phase == PH_DECIDE || phase == PH_POST) {
      bool post_now = phase == PH_POST;
      const bool greedy = (v.flags & F_GREEDY) != 0;
      if (phase == PH_DECIDE) {
        v.decide(d, greedy);
        abytes += 220ull + 48ull * ldc_u8(m.sw_np, (uint32_t)d.sw) + 8ull * ldc_u8(m.sw_na, (uint32_t)d.sw);
        v.flags |= F_INFLIGHT;
        if (!v.q_mask) phase = PH_TICK;  // ticks happen between the step and the update
        else post_now = true;
      }
      if (post_now) {
        v.post(d, greedy);
        if (c.trace && (int32_t)e == c.trace_env) {
          const uint64_t cs = v.sem_checksum();
          if (lane == 0) {
            const uint64_t n = *c.trace_n;
            if (n < (uint64_t)c.trace_cap) {
              uint64_t* tp = c.trace + 4 * n;
              tp[0] = (uint64_t)(uint32_t)v.now | ((uint64_t)(uint32_t)d.sw << 16) | ((uint64_t)(uint32_t)d.h << 32) |
                      ((uint64_t)(uint32_t)d.action << 48);
              tp[1] = (uint64_t)d.state | ((uint64_t)(uint32_t)d.reward << 32);
              tp[2] = cs;
              tp[3] = (uint64_t)(uint32_t)d.next_sw;
            }
            *c.trace_n = n + 1;
          }
        }
        v.flags &= ~F_INFLIGHT;
        v.cum += (double)d.reward;
        v.ep_dec += 1;
        v.dec_total += 1;
        v.step_ctr += 1;
        if (v.step_ctr > m.max_steps) v.flags |= F_TRUNC;
        dec++;
        phase = (v.flags & (F_TERM | F_TRUNC)) ? PH_END : PH_DECIDE;
        if (c.dec_budget > 0 && (int64_t)dec >= c.dec_budget) break;
      }
    } else {  // PH_END
      const int arrived = popc64(v.arr_mask);
      const size_t cap = (size_t)(c.stats_cap > 0 ? c.stats_cap : 1);
      const bool greedy = (v.flags & F_GREEDY) != 0;
      if (c.st_cum && c.stats_cap > 0 && (!greedy || test_mode)) {
        const int32_t idx = (greedy && test_mode) ? n_test : ep_t;
        const size_t row = (size_t)(idx - c.stats_base) % cap;
        if (lane == 0) {
          st(c.st_cum, row * s.E + e, v.cum);
          st(c.st_arrived, row * s.E + e, (int32_t)arrived);
          st(c.st_mf, row * s.E + e, v.n_mf);
          st(c.st_dec, row * s.E + e, v.ep_dec);
          st(c.st_ticks, row * s.E + e, v.ep_ticks);
        }
        if (v.mine) st(c.st_delays, (row * m.T + lane) * s.E + e, v.delay);
      }
      if (greedy && !test_mode && c.sx_cum && c.stats_cap > 0 && lane == 0) {
        const size_t row = (size_t)(ep_t - c.stats_base) % cap;
        st(c.sx_cum, row * s.E + e, v.cum);
        st(c.sx_arrived, row * s.E + e, (int32_t)arrived);
      }
      if (greedy) {
        if (test_mode) n_test += 1;
        else v.flags |= F_EXPLOIT_DONE;
      } else {
        ep_t += 1;
        v.flags &= ~F_EXPLOIT_DONE;
      }
      phase = PH_RESET;
    }
  }
  v.store(phase);
  if (lane == 0) {
    st(s.ep_t, e, ep_t);
    st(s.n_test, e, n_test);
    if (c.launch_dec) st(c.launch_dec, e, dec);
    if (c.launch_ticks) st(c.launch_ticks, e, ticks);
    if (c.launch_bytes) st(c.launch_bytes, e, abytes);
  }
}

}  // namespace wave
}  // namespace sfl
