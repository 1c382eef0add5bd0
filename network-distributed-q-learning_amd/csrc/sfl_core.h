// SwitchFL + network-distributed Q-learning: one lock-step environment per lane.
//
// This header is the whole hot path, written once
// as host/device code.  The HIP kernel (sfl.hip) runs ``env_run`` with one
// thread per environment; tests also compile it for the host (sfl_hostsim.cpp)
// to check it against the CPU oracle without a GPU.  Reference behaviour it
// restates, with citations at each function:
//   switchfl/distr_q.py        learn / test / update / max_q / max_action
//   switchfl/switch_env.py     reset / _apply_action / _move_trains / _check_active_switch
//   switchfl/rail_network.py   transition_train / transition_semaphore / extend_semaphores
//   switchfl/observer.py       check_port_blocked / compute_delay / observe
//   switchfl/reward_func.py    StandardRewardFunction
//   oracle/flatland_lite.py    the frozen Flatland RailEnv.step spec
//
// Memory layout (DESIGN.md §"HBM layout"): every per-env quantity is SoA with
// the env index fastest (``field[i * E + e]``) so a wave's 64 lanes touching
// the same field of their own envs coalesce; the Q-table is env-major (one
// contiguous block per env) because rows are gathered at data-dependent
// offsets.
#pragma once
#include <stdint.h>
#include "sfl_rng.h"

#if !defined(__HIPCC__)
#include <math.h>
#endif

namespace sfl {

enum : uint32_t { A_NOTHING = 0, A_LEFT = 1, A_FWD = 2, A_RIGHT = 3, A_STOP = 4, A_NONE = 15 };
enum : uint32_t { S_WAITING = 0, S_READY = 1, S_MF_OFF = 2, S_MOVING = 3, S_STOPPED = 4, S_MALF = 5, S_DONE = 6 };
enum : int32_t { PH_RESET = 0, PH_TICK = 1, PH_DECIDE = 2, PH_POST = 3, PH_END = 4 };
enum : uint32_t { F_TERM = 1, F_TRUNC = 2, F_GREEDY = 4, F_EXPLOIT_DONE = 8, F_OWN_SCAN = 16, F_INFLIGHT = 32 };
// (64: F_REQ, sfl_part.h; 128: F_EXT_OBS, an observation was emitted in external-action mode and its
// action is due)
enum : uint32_t { F_EXT_OBS = 128 };
enum : uint32_t {
  E_INF_DIST = 1,      // observer.py:35-36 would raise ValueError
  E_PLAN_OVF = 2,      // train plan longer than the packed ring
  E_PORT = 4,          // active train's next port not at the deciding switch (observer.py:294-301)
  E_BAD_ACTION = 8,    // action outside the switch's action space (switch_env.py:213-215)
  // (16: E_MSG_OVF, sfl_part.h)
  E_LR_TABLE = 32,     // device: a decayed lr beyond the host table; the device pow is not the host
                       // libm's, so the run stops rather than lose bit-exactness (raise ntab)
};

constexpr int32_t DIST_INF = 0x3FFFFFFF;
constexpr int OWN_MAX = 16;
constexpr int MAXW = 4;  // train bitmask words (T <= 128)
constexpr uint32_t PEND_NONE = 0xFFFFFFFFu;
constexpr uint16_t PORT_NONE = 0xFFFFu;

struct SflMap {
  int32_t H, W, S, T, K, NP, HW, cell_bits;  // cell_bits: bits of a cell index (HW - 1)
  int32_t max_episode_steps, mf_min, mf_max, ntab;
  int32_t delay_thr;  // StandardObserver.delay_threshold (observer.py:221)
  double mf_rate, gamma, eps0, eps_decay, lr0, lr_decay, default_q;
  // the counter-based malfunction draw without its f64 conversion and 64-bit division (mf_propose):
  // u < mf_rate  <=>  (z >> 11) < mf_thresh = ceil(mf_rate * 2^53), and x % mf_n via mf_magic = (2^64 - 1) / mf_n
  uint64_t mf_thresh, mf_magic;
  uint32_t mf_n;
  int64_t max_steps;
  uint64_t q_per_env;
  uint32_t rows_per_env, touched_words;
  const uint16_t* grid;
  const int16_t* cell_sw;
  const uint8_t* sw_np;
  const uint8_t* sw_na;
  const uint8_t* act_src;
  const uint8_t* act_dst;
  const uint8_t* act_turn;
  const uint8_t* act_j;
  const uint8_t* first_other;
  const uint8_t* port_side;
  const uint8_t* slot_nroutes;
  const uint8_t* slot_route_act;
  const uint8_t* q_w;
  const int16_t* port_nb;
  const int16_t* port_len;
  const int16_t* port_unique;
  const uint64_t* q_off;
  const uint32_t* row_base;
  const int32_t* dist;
  const int32_t* tr_ed;
  const int32_t* tr_la;
  const int32_t* tr_k;
  const int32_t* tr_target;
  const int32_t* tr_init_cell;
  const int32_t* tr_init_dist;
  const int32_t* tr_init_delay;
  const uint8_t* tr_init_dir;
  const int16_t* tr_init_port;
  const double* eps_tab;
  const double* lr_tab;
  // packed copies for the one-env-per-wave kernel (sfl_wave.h), built at create time
  const uint32_t* sw_pack;    // [S][16]: np | na<<4; src/dst 2b per action; turn/j 2b; q_w 4b per slot; row map per slot;
                              // neighbour port of ports 0-3 (16 b each) in words 8-9; 10-15 spare
  const uint32_t* port_pack;  // [NP][4]: nb | len<<16; unique | q_w<<16; row_base; q_off
  const uint32_t* move_tab;   // [H*W][4 dir][4 action&3]: check_action result (see move_pack)
  const uint32_t* move2c_tab; // [H*W][4 dir][4 action&3][4 rail action t]: move_tab's word of rail action t at the
                              // destination of (cell, dir, action); off the grid: that destination (cell -1)
  const int32_t* tr_pack;     // [T][8]: ed, la, k, target, init_cell, init_dist, init_delay, init_dir | init_port<<16
  const uint32_t* seedseq32;  // [2^31] first 32-bit output of Generator(PCG64(SeedSequence(v))), or null
  const uint32_t* port_tr;    // [NP][4]: transition recipe of an out port o: nb(o) | unique(nb(o)) << 16;
                              //          nb(unique) | len(o) << 16; len(unique); 0  (int16 fields, -1 = none)
  // Flatland-compatible malfunction stream (sfl_mfgen.h): [E][mf_steps][T] num_broken_steps proposed at
  // step t (row t - 1) of an episode, 0 = none; mf_steps == 0: the counter-based draw (mf_draw)
  const uint8_t* mf_tab;
  int32_t mf_steps;
};

// x % n for 1 <= n < 2^32 with M = floor((2^64 - 1) / n): q = hi64(x * M) is floor(x / n) or one less (M is
// within 1 of 2^64 / n and x < 2^64), so one correction makes the remainder exact.  On the GPU the 64-bit `%`
// is a ~200-instruction expansion; this is a 64 x 64 high product and a few integer ops (c3: +0.7 %, same box,
// profiles/r05i_mf_fastmod_ab.txt).
SFL_FN uint32_t mod_small(uint64_t x, uint32_t n, uint64_t M) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint64_t q = __umul64hi(x, M);
#else
  const uint64_t q = (uint64_t)(((unsigned __int128)x * M) >> 64);
#endif
  uint64_t r = x - q * (uint64_t)n;
  if (r >= n) r -= n;
  return (uint32_t)r;
}

// mf_propose's integer forms of the map's malfunction parameters (set when the map is built, sfl_engine.h)
inline void mf_prepare(SflMap& m) {
  const double R = ldexp(m.mf_rate, 53);
  m.mf_thresh = !(m.mf_rate > 0.0) ? 0ull : (R >= 9007199254740992.0 ? (1ull << 53) : (uint64_t)ceil(R));
  const int64_t n = (int64_t)m.mf_max - (int64_t)m.mf_min + 1;
  m.mf_n = (n >= 1 && n < (1ll << 32)) ? (uint32_t)n : 0u;
  m.mf_magic = m.mf_n ? ~0ull / m.mf_n : 0ull;
}

// the malfunction proposed to train h of env e at step t, given its state and counter (both streams)
SFL_FN uint32_t mf_propose(const SflMap& m, uint64_t seed, uint32_t e, int32_t t, int h) {
  if (m.mf_steps > 0) {
    if (t < 1 || t > m.mf_steps) return 0u;
    return m.mf_tab[((size_t)e * (uint32_t)m.mf_steps + (uint32_t)(t - 1)) * (uint32_t)m.T + (uint32_t)h];
  }
  if (!(m.mf_rate > 0.0)) return 0u;
  const uint64_t z = mf_draw(seed, (uint64_t)t, (uint64_t)h);
  // u = (z >> 11) * 2^-53 is exact, so u < mf_rate  <=>  (z >> 11) < ceil(mf_rate * 2^53)  (oracle/flatland_lite.py)
  if ((z >> 11) >= m.mf_thresh) return 0u;
  const uint64_t x = mix64(z ^ 0xA0761D6478BD642Full);
  const uint32_t r = m.mf_n ? mod_small(x, m.mf_n, m.mf_magic)
                            : (uint32_t)(x % (uint64_t)(m.mf_max - m.mf_min + 1));  // (mf_max < mf_min: as before)
  return (uint32_t)(m.mf_min + (int32_t)r) + 1u;
}

struct SflState {
  uint32_t E;
  int32_t* phase;
  int32_t* elapsed;
  uint32_t* eflags;
  int32_t* ep_t;        // learning episodes completed in the current learn() call
  int32_t* n_test;      // greedy test episodes completed in the current test() call
  uint32_t* epoch;      // (switch, train) slot epoch
  uint64_t* rng;        // [5][E]: state hi/lo, inc hi/lo, has<<32|buf
  uint64_t* seed;       // env seed (reset / malfunction stream)
  double* cum_reward;
  int32_t* n_mf;
  int32_t* ep_dec;
  int32_t* ep_ticks;
  int64_t* step_ctr;
  int64_t* dec_total;
  uint32_t* masks;      // [4][MAXW][E]: active, arrived, flushed, malfunction-last-tick
  uint32_t* err;
  int32_t* tr_pos;      // [T][E] cell index or -1 (off map)
  uint32_t* tr_bits;    // [T][E] dir | state | prev action | saved action | mf counter | done
  uint32_t* tr_plan;    // [T][E] packed rail-action queue
  uint16_t* tr_next;    // [T][E] _train2next_port
  uint16_t* tr_prev;    // [T][E] _train_prev_port (persists across resets, like the reference)
  uint16_t* tr_src;     // [T][E] _train_source_port (persists across resets)
  uint16_t* tr_dec;     // [T][E] switch of the train's queued decision
  int32_t* tr_delay;    // [T][E] train_to_last_node delay
  uint16_t* own;        // [T*OWN_MAX][E] ports a train may own (lazily validated)
  uint8_t* own_n;       // [T][E]
  int32_t* sc_desired;  // [T][E] tick scratch
  int32_t* sc_pred;     // [T][E]
  uint32_t* sc_aux;     // [T][E]
  uint8_t* occ;         // [H*W][E] occupying train or 0xFF
  uint8_t* claim;       // [H*W][E] motion-check claim or 0xFF
  uint64_t* sem;        // [NP][E] semaphore records
  uint64_t* slot;       // pending update | reward | epoch: [S*T][E] (k_run), [E][T][S] (k_wave)
  uint32_t* counts;     // [S][E] agent_num_interactions
  double* q;            // [E][q_per_env]
  uint32_t* touched;    // [E][touched_words] Q-table key set
};

struct SflCtl {
  int32_t mode;          // 0 = learn, 1 = greedy test
  int32_t exploit_freq;  // learn: greedy round before episode t when (t+1) % f == 0
  int32_t ep_target;     // stop once this many episodes of the mode are done (-1: unlimited)
  int32_t stats_cap;     // rows in the stats buffers: row = (episode index - stats_base) % cap
  int32_t stats_base;
  int64_t dec_budget;    // decisions per env in this launch (<= 0: unlimited)
  double* st_cum;        // [cap][E]
  int32_t* st_arrived;   // [cap][E]
  int32_t* st_mf;        // [cap][E]
  int32_t* st_dec;       // [cap][E]
  int32_t* st_ticks;     // [cap][E]
  int32_t* st_delays;    // [cap][T][E]
  double* sx_cum;        // exploit rounds [cap][E]
  int32_t* sx_arrived;   // [cap][E]
  uint64_t* launch_dec;  // [E] decisions made in this launch
  uint64_t* launch_ticks;  // [E]
  uint64_t* launch_bytes;  // [E] algorithmic bytes (SURVEY.md §8(d) model) of this launch
  uint64_t* trace;       // optional per-decision trace of one env: [trace_cap][4]
  uint64_t* trace_n;     // records written
  int32_t trace_env;
  int32_t trace_cap;
  const struct SflExt* ext;  // external-action mode (mode 2) buffers, device memory; null otherwise
  uint64_t* phase_cyc;       // [8] per-phase cycles of sampled wavefronts (learn / test launches), or null
};

// External-action mode (sfl_env_step): the env alone, stepped one decision per call by a policy on the
// host -- the PettingZoo AEC protocol agent_iter / last / step(action) / observe (switch_env.py:616-675)
// driven by any learner (distr_q.py:302-320).  Per env and call: the action for the observation the
// previous call emitted is applied (_apply_action, then the Flatland ticks up to the next decision if
// no switch is active), and the env runs on to its next decision, whose observation is emitted; an
// episode end is reported instead (agent = -1) and the next call starts the next episode.
struct SflExt {
  const int32_t* actions;  // [E] in: action for the pending observation (< 0: none)
  int32_t* agent;          // [E] deciding switch (-1: the episode ended in this call)
  int32_t* train;          // [E] active train
  int32_t* slot;           // [E] in-port slot of the active train at the switch
  uint32_t* state;         // [E] observation index ((free_bits * K + k) * 3 + delay level)
  uint32_t* mask;          // [E] action mask bits
  int32_t* reward;         // [E] AECEnv.last() reward of (switch, train)
  int32_t* now;            // [E] elapsed ticks at the observation
  int32_t* next_sw;        // [E] successor switch of the applied action (-1: none applied)
  int32_t* step_now;       // [E] elapsed ticks when the applied action's step() returned
  uint32_t* arrived;       // [MAXW][E] arrived trains (bitmask) after the step / at the episode end
  int32_t* n_mf;           // [E] malfunctions counted in the episode
  int32_t* delays;         // [T][E] train_to_last_node delays at the episode end
  int32_t* truncated;      // [E] the episode ended by max_steps truncation (1) or termination (0)
};

// ---------------------------------------------------------------------------
// small helpers
// ---------------------------------------------------------------------------
SFL_FN int popc32(uint32_t x) { return __builtin_popcount(x); }
SFL_FN int ctz32(uint32_t x) { return __builtin_ctz(x); }

// tr_bits layout
SFL_FN uint32_t tb_dir(uint32_t b) { return b & 3u; }
SFL_FN uint32_t tb_state(uint32_t b) { return (b >> 2) & 7u; }
SFL_FN uint32_t tb_prev(uint32_t b) { return (b >> 5) & 15u; }
SFL_FN uint32_t tb_saved(uint32_t b) { return (b >> 9) & 15u; }
SFL_FN uint32_t tb_mf(uint32_t b) { return (b >> 13) & 0xFFu; }
SFL_FN uint32_t tb_done(uint32_t b) { return (b >> 21) & 1u; }
SFL_FN uint32_t tb_make(uint32_t dir, uint32_t state, uint32_t prev, uint32_t saved, uint32_t mf, uint32_t done) {
  return (dir & 3u) | ((state & 7u) << 2) | ((prev & 15u) << 5) | ((saved & 15u) << 9) | ((mf & 0xFFu) << 13) |
         ((done & 1u) << 21);
}

// packed plan: bits 0-3 length, action k in bits 4+4k
SFL_FN uint32_t pl_len(uint32_t p) { return p & 15u; }
SFL_FN uint32_t pl_front(uint32_t p) { return (p >> 4) & 15u; }
SFL_FN uint32_t pl_pop(uint32_t p) { return ((p >> 8) << 4) | (pl_len(p) - 1u); }
SFL_FN uint32_t pl_push_front(uint32_t p, uint32_t a, uint32_t& err) {
  uint32_t n = pl_len(p);
  if (n >= 7u) { err |= E_PLAN_OVF; return p; }
  return (((p >> 4) << 8) | (a << 4)) | (n + 1u);
}
SFL_FN uint32_t pl_push_back(uint32_t p, uint32_t a, uint32_t& err) {
  uint32_t n = pl_len(p);
  if (n >= 7u) { err |= E_PLAN_OVF; return p; }
  return (p & ~15u) | (a << (4u + 4u * n)) | (n + 1u);
}
SFL_FN uint32_t pl_at(uint32_t p, uint32_t i) { return (p >> (4u + 4u * i)) & 15u; }

// semaphore record: t0 16 | t1 16 | owner 8 | in 1 | present 1
SFL_FN uint64_t sem_pack(uint32_t owner, uint32_t is_in, int32_t t0, int32_t t1) {
  return (uint64_t)(uint16_t)(int16_t)t0 | ((uint64_t)(uint16_t)(int16_t)t1 << 16) | ((uint64_t)(owner & 0xFFu) << 32) |
         ((uint64_t)(is_in & 1u) << 40) | (1ull << 41);
}
SFL_FN bool sem_present(uint64_t r) { return (r >> 41) & 1ull; }
SFL_FN int32_t sem_t0(uint64_t r) { return (int32_t)(int16_t)(uint16_t)(r & 0xFFFFull); }
SFL_FN int32_t sem_t1(uint64_t r) { return (int32_t)(int16_t)(uint16_t)((r >> 16) & 0xFFFFull); }
SFL_FN uint32_t sem_owner(uint64_t r) { return (uint32_t)((r >> 32) & 0xFFull); }
SFL_FN uint32_t sem_in(uint64_t r) { return (uint32_t)((r >> 40) & 1ull); }
SFL_FN uint64_t sem_retime(uint64_t r, uint32_t owner, int32_t t0, int32_t t1) {
  return sem_pack(owner, sem_in(r), t0, t1);
}
// the wavefront kernels' 32-bit record (LDS, and their env-major state between launches):
// t0 14 (signed) | t1 - t0 9 | owner 7 | in 1 | present 1 (choose_variant checks that the map's
// ticks and spans fit)
constexpr uint32_t R_T0_BITS = 14, R_DUR_BITS = 9, R_OWNER_SHIFT = R_T0_BITS + R_DUR_BITS;
constexpr uint32_t R_T0_MASK = (1u << R_T0_BITS) - 1u, R_DUR_MASK = (1u << R_DUR_BITS) - 1u;
SFL_FN uint64_t wave_rec_to64(uint32_t r) {
  if (!(r >> 31)) return 0ull;
  const int32_t t0 = ((int32_t)(r << (32 - R_T0_BITS))) >> (32 - R_T0_BITS);
  return sem_pack((r >> R_OWNER_SHIFT) & 0x7Fu, (r >> 30) & 1u, t0, t0 + (int32_t)((r >> R_T0_BITS) & R_DUR_MASK));
}

// (switch, train) slot: pending 32 | reward 24 (signed) | epoch 8
SFL_FN uint32_t slot_pend(uint64_t v, uint32_t epoch) { return ((uint32_t)(v >> 56) == (epoch & 0xFFu)) ? (uint32_t)v : PEND_NONE; }
SFL_FN int32_t slot_rew(uint64_t v, uint32_t epoch) {
  if ((uint32_t)(v >> 56) != (epoch & 0xFFu)) return 0;
  int32_t r = (int32_t)((v >> 32) & 0xFFFFFFull);
  return (r << 8) >> 8;
}
SFL_FN uint64_t slot_make(uint32_t pend, int32_t rew, uint32_t epoch) {
  return (uint64_t)pend | ((uint64_t)((uint32_t)rew & 0xFFFFFFu) << 32) | ((uint64_t)(epoch & 0xFFu) << 56);
}
// pending: switch 12 | slot 2 | state 14 | j 2 (+ all-ones = none)
SFL_FN uint32_t pend_make(uint32_t s, uint32_t slot, uint32_t state, uint32_t j) {
  return (s & 0xFFFu) | ((slot & 3u) << 12) | ((state & 0x3FFFu) << 14) | ((j & 3u) << 28);
}

SFL_FN bool is_moving_action(uint32_t a) { return a == A_LEFT || a == A_FWD || a == A_RIGHT; }

// flatland-lite check_action_on_agent for (action, cell, dir), packed for move_tab:
// new cell + 1 (20 bits; 0 = off the grid) | new dir << 20 | transition valid << 22 | new cell valid << 23.
// Actions NOTHING (0) and STOP (4) behave alike, so a table row is indexed by action & 3.
SFL_FN uint32_t move_pack(const uint16_t* grid, int H, int W, uint32_t a, int cell, int dir) {
  const uint32_t nib = ((uint32_t)grid[cell] >> ((3 - dir) * 4)) & 15u;
  const int n = popc32(nib);
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
  int r = cell / W, c = cell - r * W;
  r += (nd == 2) - (nd == 0);
  c += (nd == 1) - (nd == 3);
  const int nc = (r < 0 || r >= H || c < 0 || c >= W) ? -1 : r * W + c;
  const bool ok = nc >= 0 && grid[nc] != 0;
  const bool v = valid < 0 ? (((nib >> (3 - nd)) & 1u) != 0) : (valid != 0);
  return (uint32_t)(nc + 1) | ((uint32_t)nd << 20) | ((v ? 1u : 0u) << 22) | ((ok ? 1u : 0u) << 23);
}
SFL_FN bool on_map_state(uint32_t s) { return s == S_MOVING || s == S_STOPPED || s == S_MALF; }
SFL_FN bool off_map_state(uint32_t s) { return s == S_WAITING || s == S_READY || s == S_MF_OFF; }

// ---------------------------------------------------------------------------
// environment view
// ---------------------------------------------------------------------------
template <int NW>
struct Env {
  static constexpr int kNW = NW;  // train bitmask words held in registers (T <= 32*NW)
  const SflMap& m;
  const SflState& s;
  const uint32_t e;
  const uint32_t E;
  uint32_t err;
  int32_t now;      // rail_env._elapsed_steps
  uint32_t flags;
  uint32_t epoch;
  // train bitmasks kept in registers for the whole launch: 0 decision queue, 1 arrived,
  // 2 destination bonus paid, 3 in malfunction at the previous tick
  uint32_t msk[4][NW];

  SFL_FN Env(const SflMap& m_, const SflState& s_, uint32_t e_) : m(m_), s(s_), e(e_), E(s_.E), err(0), now(0), flags(0), epoch(0) {
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int w = 0; w < NW; ++w) msk[k][w] = 0;
  }
  SFL_FN void masks_load() {
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int w = 0; w < NW; ++w) msk[k][w] = s.masks[((size_t)k * MAXW + w) * E + e];
  }
  SFL_FN void masks_store() const {
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int w = 0; w < NW; ++w) s.masks[((size_t)k * MAXW + w) * E + e] = msk[k][w];
  }
  // constant-index access to the register masks (a runtime index would spill them to scratch)
  SFL_FN bool mbit(int k, int h) const {
    bool r = false;
#pragma unroll
    for (int w = 0; w < NW; ++w)
      if (w == (h >> 5)) r = (msk[k][w] >> (h & 31)) & 1u;
    return r;
  }
  SFL_FN void mset(int k, int h) {
#pragma unroll
    for (int w = 0; w < NW; ++w)
      if (w == (h >> 5)) msk[k][w] |= 1u << (h & 31);
  }
  SFL_FN void mclr(int k, int h) {
#pragma unroll
    for (int w = 0; w < NW; ++w)
      if (w == (h >> 5)) msk[k][w] &= ~(1u << (h & 31));
  }
  SFL_FN size_t ix(size_t i) const { return i * (size_t)E + e; }

  // grid -----------------------------------------------------------------
  SFL_FN uint32_t exits(int cell, int d) const { return ((uint32_t)m.grid[cell] >> ((3 - d) * 4)) & 15u; }
  SFL_FN int move_cell(int cell, int d) const {
    int r = cell / m.W, c = cell - r * m.W;
    r += (d == 2) - (d == 0);
    c += (d == 1) - (d == 3);
    if (r < 0 || r >= m.H || c < 0 || c >= m.W) return -1;
    return r * m.W + c;
  }
  struct Move {
    int cell;
    int dir;
    bool valid;    // transition_valid
    bool cell_ok;  // new_cell_valid
  };
  // flatland-lite check_action_on_agent
  SFL_FN Move check_action(uint32_t a, int cell, int dir) const {
    uint32_t nib = exits(cell, dir);
    int n = popc32(nib);
    int nd = dir;
    int valid = -1;
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
    mv.cell_ok = mv.cell >= 0 && m.grid[mv.cell] != 0;
    mv.valid = valid < 0 ? (((nib >> (3 - nd)) & 1u) != 0) : (valid != 0);
    return mv;
  }
  SFL_FN bool action_ok(uint32_t a, int cell, int dir) const {
    Move mv = check_action(a, cell, dir);
    return mv.cell_ok && mv.valid;
  }
  SFL_FN int32_t dist(int h, int cell, int dir) {
    if (cell < 0) { err |= E_INF_DIST; return 0; }
    int32_t d = m.dist[(((size_t)m.tr_k[h] * m.H * m.W) + (size_t)cell) * 4 + dir];
    if (d >= DIST_INF) err |= E_INF_DIST;
    return d;
  }

  // train fields -------------------------------------------------------------
  SFL_FN uint32_t& bits(int h) const { return s.tr_bits[ix(h)]; }
  SFL_FN int32_t& pos(int h) const { return s.tr_pos[ix(h)]; }
  SFL_FN uint32_t& plan(int h) const { return s.tr_plan[ix(h)]; }
  SFL_FN uint16_t& next_port(int h) const { return s.tr_next[ix(h)]; }
  SFL_FN uint16_t& prev_port(int h) const { return s.tr_prev[ix(h)]; }
  SFL_FN uint16_t& src_port(int h) const { return s.tr_src[ix(h)]; }
  SFL_FN uint32_t state_of(int h) const { return tb_state(s.tr_bits[ix(h)]); }

  // semaphores ---------------------------------------------------------------
  SFL_FN uint64_t& sem(int p) const { return s.sem[ix(p)]; }
  SFL_FN void own_add(int h, int p) {
    if (flags & F_OWN_SCAN) return;
    uint8_t& n = s.own_n[ix(h)];
    uint32_t cnt = n;
    for (uint32_t k = 0; k < cnt; ++k)
      if (s.own[ix((size_t)h * OWN_MAX + k)] == (uint16_t)p) return;
    if (cnt == OWN_MAX) {  // compact: drop entries the train no longer owns
      uint32_t w = 0;
      for (uint32_t k = 0; k < cnt; ++k) {
        uint16_t q = s.own[ix((size_t)h * OWN_MAX + k)];
        uint64_t r = sem(q);
        if (sem_present(r) && sem_owner(r) == (uint32_t)h) s.own[ix((size_t)h * OWN_MAX + w++)] = q;
      }
      cnt = w;
      if (cnt == OWN_MAX) {  // still full: fall back to full scans for this env
        flags |= F_OWN_SCAN;
        return;
      }
    }
    s.own[ix((size_t)h * OWN_MAX + cnt)] = (uint16_t)p;
    n = (uint8_t)(cnt + 1);
  }
  SFL_FN void sem_set(int p, uint64_t rec) {
    sem(p) = rec;
    own_add((int)sem_owner(rec), p);
  }
  // set if absent, else (io == ovr_io or t0 in the future) -> retime in place (io kept)
  SFL_FN void sem_put_keep(int p, int h, uint32_t is_in, int32_t span, uint32_t ovr_in) {
    uint64_t r = sem(p);
    if (!sem_present(r)) sem_set(p, sem_pack(h, is_in, now, now + span));
    else if (sem_in(r) == ovr_in || sem_t0(r) > now) sem_set(p, sem_retime(r, h, now, now + span));
  }
  // set if absent, else (ovr_in matches or t0 in the future) -> replace whole record
  SFL_FN void sem_put_replace(int p, int h, uint32_t is_in, int32_t span, int ovr_in) {
    uint64_t r = sem(p);
    if (!sem_present(r)) sem_set(p, sem_pack(h, is_in, now, now + span));
    else if ((ovr_in >= 0 && sem_in(r) == (uint32_t)ovr_in) || sem_t0(r) > now)
      sem_set(p, sem_pack(h, is_in, now, now + span));
  }
  SFL_FN void free_switch_ports(int sw, int h) {
    if (sw < 0 || sw >= m.S) {
      err |= E_PORT;
      return;
    }
    const int np = m.sw_np[sw];
    for (int j = 0; j < np; ++j) {
      uint64_t r = sem(4 * sw + j);
      if (sem_present(r) && sem_owner(r) == (uint32_t)h) sem(4 * sw + j) = 0;
    }
  }
  // delete every semaphore owned by h (switch_env.py:370-376)
  SFL_FN void purge_train(int h) {
    if (flags & F_OWN_SCAN) {
      for (int p = 0; p < m.NP; ++p) {
        uint64_t r = sem(p);
        if (sem_present(r) && sem_owner(r) == (uint32_t)h) sem(p) = 0;
      }
      return;
    }
    uint8_t& n = s.own_n[ix(h)];
    for (uint32_t k = 0; k < n; ++k) {
      uint16_t p = s.own[ix((size_t)h * OWN_MAX + k)];
      uint64_t r = sem(p);
      if (sem_present(r) && sem_owner(r) == (uint32_t)h) sem(p) = 0;
    }
    n = 0;
  }
  // extend_semaphores for one stopped/malfunctioning train (rail_network.py:233-238)
  SFL_FN void extend_train(int h) {
    if (flags & F_OWN_SCAN) {
      for (int p = 0; p < m.NP; ++p) {
        uint64_t r = sem(p);
        if (sem_present(r) && sem_owner(r) == (uint32_t)h) sem(p) = sem_retime(r, h, now, now + (sem_t1(r) - sem_t0(r)));
      }
      return;
    }
    const uint32_t n = s.own_n[ix(h)];
    for (uint32_t k = 0; k < n; ++k) {
      uint16_t p = s.own[ix((size_t)h * OWN_MAX + k)];
      uint64_t r = sem(p);
      if (sem_present(r) && sem_owner(r) == (uint32_t)h) sem(p) = sem_retime(r, h, now, now + (sem_t1(r) - sem_t0(r)));
    }
  }
  // observer.py:44-151 (a record's dir field always equals map_direction(port))
  SFL_FN bool port_blocked(int next_p, int out_p, int h) const {
    uint64_t r = sem(next_p);
    if (sem_present(r) && sem_owner(r) != (uint32_t)h && sem_t0(r) <= now && now <= sem_t1(r)) {
      if (!sem_in(r)) return true;
      if (state_of((int)sem_owner(r)) == S_MALF) return true;
    }
    r = sem(out_p);
    if (sem_present(r) && sem_owner(r) != (uint32_t)h && sem_t0(r) <= now && now <= sem_t1(r)) {
      if (sem_in(r)) return true;
      if (state_of((int)sem_owner(r)) == S_MALF) return true;
    }
    return false;
  }

  // Q-table --------------------------------------------------------------------
  SFL_FN double* qrow(int sw, int slot, uint32_t state) const {
    const int g = 4 * sw + slot;
    return s.q + (size_t)e * m.q_per_env + m.q_off[g] + (size_t)state * m.q_w[g];
  }
  SFL_FN void touch(int sw, int slot, uint32_t state) const {
    const uint32_t row = m.row_base[4 * sw + slot] + state;
    s.touched[(size_t)e * m.touched_words + (row >> 5)] |= 1u << (row & 31u);
  }
  SFL_FN double eps_of(uint32_t n) const { return n < (uint32_t)m.ntab ? m.eps_tab[n] : m.eps0 * pow(m.eps_decay, (double)n); }
  // beyond the table: eps only decides `random() < eps` (an ulp of pow moves that by ~1e-17 in
  // probability), but lr enters the Q values, so on the device a decaying lr past the table is an error
  SFL_FN double lr_of(uint32_t n, uint32_t& e) const {
    if (n < (uint32_t)m.ntab) return m.lr_tab[n];
#if defined(__HIP_DEVICE_COMPILE__)
    if (m.lr_decay != 1.0) e |= E_LR_TABLE;
#endif
    return m.lr0 * pow(m.lr_decay, (double)n);
  }

  // rng ------------------------------------------------------------------------
  SFL_FN Pcg64 rng_load() const {
    Pcg64 g;
    g.shi = s.rng[ix(0)];
    g.slo = s.rng[ix(1)];
    g.ihi = s.rng[ix(2)];
    g.ilo = s.rng[ix(3)];
    uint64_t hb = s.rng[ix(4)];
    g.has = (uint32_t)(hb >> 32);
    g.buf = (uint32_t)hb;
    return g;
  }
  SFL_FN void rng_store(const Pcg64& g) const {
    s.rng[ix(0)] = g.shi;
    s.rng[ix(1)] = g.slo;
    s.rng[ix(4)] = ((uint64_t)g.has << 32) | g.buf;
  }
};

// constant-index bit ops on small register arrays (runtime indices would spill them to scratch)
template <int N>
SFL_FN bool bget(const uint32_t (&a)[N], int i) {
  bool r = false;
#pragma unroll
  for (int w = 0; w < N; ++w)
    if (w == (i >> 5)) r = (a[w] >> (i & 31)) & 1u;
  return r;
}
template <int N>
SFL_FN void bset(uint32_t (&a)[N], int i) {
#pragma unroll
  for (int w = 0; w < N; ++w)
    if (w == (i >> 5)) a[w] |= 1u << (i & 31);
}

// ---------------------------------------------------------------------------
// episode reset (switch_env.py:93-158, _init_ports 507-568)
// ---------------------------------------------------------------------------
template <class V>
SFL_FN void env_reset(V& v) {
  const SflMap& m = v.m;
  const SflState& s = v.s;
  v.now = 0;
  for (int h = 0; h < m.T; ++h) {
    int32_t p = v.pos(h);
    if (p >= 0 && s.occ[v.ix(p)] == (uint8_t)h) s.occ[v.ix(p)] = 0xFF;
    v.pos(h) = -1;
    v.bits(h) = tb_make(m.tr_init_dir[h], S_WAITING, A_NONE, 0, 0, 0);
    v.plan(h) = 0;
    v.next_port(h) = (uint16_t)m.tr_init_port[h];
    s.tr_delay[v.ix(h)] = m.tr_init_delay[h];
    s.own_n[v.ix(h)] = 0;
  }
  for (int p = 0; p < m.NP; ++p) v.sem(p) = 0;
  v.flags &= ~(F_TERM | F_TRUNC | F_OWN_SCAN | F_INFLIGHT);
  for (int h = 0; h < m.T; ++h) {
    const int p = m.tr_init_port[h];
    v.sem_set(p, sem_pack(h, 1, m.tr_ed[h] - 2, m.tr_ed[h] + m.tr_init_dist[h]));
  }
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int w = 0; w < V::kNW; ++w) v.msk[k][w] = 0;
  // new (switch, train) epoch: slots from older episodes read as empty
  v.epoch = (v.epoch + 1u) & 0xFFu;
  if (v.epoch == 0) {
    for (int i = 0; i < m.S * m.T; ++i) s.slot[v.ix(i)] = slot_make(PEND_NONE, 0, 0);
    v.epoch = 1;
  }
  s.cum_reward[v.e] = 0.0;
  s.n_mf[v.e] = 0;
  s.ep_dec[v.e] = 0;
  s.ep_ticks[v.e] = 0;
  s.step_ctr[v.e] = 0;
}

// ---------------------------------------------------------------------------
// one Flatland tick + switchfl bookkeeping + _check_active_switch
// (switch_env.py:296-401, 427-485; flatland_lite.RailEnv.step)
// ---------------------------------------------------------------------------
// sc_aux layout: pa 0-3 | ddir 4-5 | mover 6 | allowed 7 | given 8-11 | has_pred 12 | pred_valid 13
template <class V>
SFL_FN void env_tick(V& v) {
  const SflMap& m = v.m;
  const SflState& s = v.s;
  const int32_t t = ++v.now;
  const uint64_t seed = s.seed[v.e];
  constexpr int NW = V::kNW;
  uint32_t movers[NW] = {};

  // pass 1: plan pop + prediction (switch_env.py:304-339), malfunction draw, action
  // preprocessing, desired move, cell claims (flatland step, first agent loop)
  for (int h = 0; h < m.T; ++h) {
    uint32_t b = v.bits(h);
    const int32_t pos = v.pos(h);
    uint32_t st = tb_state(b), dir = tb_dir(b), prev = tb_prev(b), saved = tb_saved(b), mf = tb_mf(b);
    uint32_t aux = 0;
    uint32_t given = A_NOTHING;
    int32_t pred = pos;
    if (!tb_done(b)) {
      uint32_t p = v.plan(h);
      if (pl_len(p) == 0) {
        given = A_FWD;
      } else {
        given = pl_front(p);
        prev = given;
        v.plan(h) = pl_pop(p);
      }
      if (pos >= 0) {
        typename V::Move mv = v.check_action(given, pos, (int)dir);
        aux |= 1u << 12;
        if (mv.valid) {
          aux |= 1u << 13;
          pred = mv.cell;
        }
      }
    }
    if (st != S_DONE && mf == 0) mf = mf_propose(m, seed, v.e, t, h);
    // preprocess_action
    uint32_t pa = given;
    if (pa == A_NOTHING && st == S_MOVING) pa = A_FWD;
    if (st == S_WAITING) pa = A_NOTHING;
    const int pc = pos >= 0 ? pos : m.tr_init_cell[h];
    const int pd = pos >= 0 ? (int)dir : (int)m.tr_init_dir[h];
    if ((pa == A_LEFT || pa == A_RIGHT) && !v.action_ok(pa, pc, pd)) pa = A_FWD;
    if (is_moving_action(pa) && !v.action_ok(pa, pc, pd)) pa = A_STOP;
    if (is_moving_action(pa) && saved == 0 && st != S_DONE) saved = pa;
    const bool update_allowed = (mf == 0) && pa != A_STOP;
    int32_t desired = pos;
    uint32_t ddir = dir;
    bool mover = false;
    if (st == S_DONE) {
    } else if (pos < 0 && saved != 0) {
      desired = m.tr_init_cell[h];
      ddir = m.tr_init_dir[h];
      mover = true;
    } else if (saved != 0 && update_allowed) {
      typename V::Move mv = v.check_action(saved, pos, (int)dir);
      desired = mv.cell;
      ddir = (uint32_t)mv.dir;
      pa = saved;
      mover = desired != pos;
    }
    if (mover) {
      bset(movers, h);
      uint8_t& c = s.claim[v.ix(desired)];
      if (c == 0xFF) c = (uint8_t)h;
    }
    aux |= pa | (ddir << 4) | ((mover ? 1u : 0u) << 6) | (given << 8);
    s.sc_aux[v.ix(h)] = aux;
    s.sc_desired[v.ix(h)] = desired;
    s.sc_pred[v.ix(h)] = pred;
    v.bits(h) = tb_make(dir, st, prev, saved, mf, tb_done(b));
  }

  // pass 2: motion check, least fixed point (flatland_lite.motion_check)
  uint32_t allowed[NW] = {};
  bool changed = true;
  while (changed) {
    changed = false;
#pragma unroll
    for (int w = 0; w < V::kNW; ++w) {
      uint32_t pend = movers[w] & ~allowed[w];
      while (pend) {
        const int h = w * 32 + ctz32(pend);
        pend &= pend - 1u;
        const int32_t d = s.sc_desired[v.ix(h)];
        if (s.claim[v.ix(d)] != (uint8_t)h) continue;
        const uint8_t j = s.occ[v.ix(d)];
        if (j == 0xFF || (bget(movers, j) && bget(allowed, j))) {
          allowed[w] |= 1u << (h & 31);
          changed = true;
        }
      }
    }
  }

  // pass 3: state machine + positions (flatland step, second agent loop), then
  // deviation fix, purge of done trains and departure semaphores (switch_env.py:353-384)
  const bool episode_over_by_time = t >= m.max_episode_steps;
  bool all_done = true;
  for (int h = 0; h < m.T; ++h) {
    uint32_t b = v.bits(h);
    const int32_t pos = v.pos(h);
    const uint32_t aux = s.sc_aux[v.ix(h)];
    const int32_t desired = s.sc_desired[v.ix(h)];
    uint32_t st = tb_state(b), dir = tb_dir(b), saved = tb_saved(b), mf = tb_mf(b);
    const uint32_t pa = aux & 15u;
    const bool mover = (aux >> 6) & 1u;
    if (mover && s.claim[v.ix(desired)] == (uint8_t)h) s.claim[v.ix(desired)] = 0xFF;
    const bool in_mf = mf > 0;
    bool ma = in_mf ? false : (mover && bget(allowed, h));
    const bool valid_move = is_moving_action(pa) && ma;
    const bool ed_reached = t >= m.tr_ed[h];
    const uint32_t prev_st = st;
    switch (st) {
      case S_WAITING: st = in_mf ? S_MF_OFF : (ed_reached ? S_READY : S_WAITING); break;
      case S_READY: st = in_mf ? S_MF_OFF : (valid_move ? S_MOVING : S_READY); break;
      case S_MF_OFF: st = (mf == 0) ? (ed_reached ? S_READY : S_WAITING) : S_MF_OFF; break;
      case S_MOVING:
        if (in_mf) st = S_MALF;
        else if (pa == A_STOP) st = S_STOPPED;
        else if (pos >= 0 && pos == m.tr_target[h]) st = S_DONE;
        else if (!ma) st = S_STOPPED;
        break;
      case S_STOPPED: st = in_mf ? S_MALF : (valid_move ? S_MOVING : S_STOPPED); break;
      case S_MALF: st = (mf == 0) ? (valid_move ? S_MOVING : S_STOPPED) : S_MALF; break;
      default: break;
    }
    ma = ma && st != S_DONE;
    int32_t npos = pos;
    if (on_map_state(st)) {
      if (off_map_state(prev_st)) {
        npos = m.tr_init_cell[h];
        dir = m.tr_init_dir[h];
      } else if (ma) {
        npos = desired;
        dir = (aux >> 4) & 3u;
        if (npos == m.tr_target[h]) st = S_DONE;
      }
    }
    if (st == S_DONE && !v.mbit(1, h)) {
      v.mset(1, h);  // arrived (position None, arrival_time set)
      npos = -1;
    }
    if (npos != pos) {
      if (pos >= 0 && s.occ[v.ix(pos)] == (uint8_t)h) s.occ[v.ix(pos)] = 0xFF;
      if (npos >= 0) s.occ[v.ix(npos)] = (uint8_t)h;
    }
    if (mf > 0) mf -= 1;
    if (npos >= 0) saved = 0;
    const bool done = (st == S_DONE) || episode_over_by_time;
    all_done = all_done && st == S_DONE;
    v.pos(h) = npos;
    // switchfl: deviation fix
    if ((aux >> 12) & 1u) {
      const int32_t exp = s.sc_pred[v.ix(h)];
      const uint32_t given = (aux >> 8) & 15u;
      if (exp != npos && ((aux >> 13) & 1u) && given != A_STOP) {
        v.plan(h) = pl_push_front(v.plan(h), given, v.err);
        if (m.cell_sw[exp] >= 0) v.next_port(h) = v.src_port(h);
      }
    }
    if (done) v.purge_train(h);
    if (t == m.tr_ed[h] - 2) {
      const int p = v.next_port(h);
      v.sem_set(p, sem_pack(h, 1, m.tr_ed[h] - 2, m.tr_ed[h] + m.tr_init_dist[h]));
    }
    v.bits(h) = tb_make(dir, st, tb_prev(b), saved, mf, done ? 1u : 0u);
  }

  // pass 4: extend_semaphores (rail_network.py:229-244), malfunction count
  // (switch_env.py:399-401), _check_active_switch (switch_env.py:427-485)
  const bool terminated = all_done || episode_over_by_time;
  int32_t new_mf = 0;
  for (int h = 0; h < m.T; ++h) {
    const uint32_t b = v.bits(h);
    const uint32_t st = tb_state(b);
    if (st == S_STOPPED || st == S_MALF) v.extend_train(h);
    if (st == S_MALF) {
      const int p = v.next_port(h);
      if (!sem_present(v.sem(p))) v.sem_set(p, sem_pack(h, 1, t, t + m.tr_init_dist[h]));
    }
    if (tb_mf(b) > 0) {
      if (!v.mbit(3, h)) new_mf++;
      v.mset(3, h);
    } else {
      v.mclr(3, h);
    }
    const int32_t pos = v.pos(h);
    if (pos < 0 || st == S_WAITING) continue;
    const uint32_t p = v.plan(h);
    const uint32_t nxt = pl_len(p) ? pl_front(p) : A_FWD;
    typename V::Move mv = v.check_action(nxt, pos, (int)tb_dir(b));
    if (mv.cell < 0) continue;
    const int sw_at = m.cell_sw[mv.cell];
    if (sw_at < 0) continue;
    int sw;
    if (st == S_READY || st == S_MOVING) sw = sw_at;
    else if ((st == S_STOPPED || st == S_MALF) && tb_prev(b) == A_STOP) sw = sw_at;
    else if (st == S_STOPPED || st == S_MALF) sw = v.next_port(h) >> 2;
    else continue;
    if (sw >= m.S) {  // next port is None: the reference would raise here
      v.err |= E_PORT;
      continue;
    }
    v.mset(0, h);
    s.tr_dec[v.ix(h)] = (uint16_t)sw;
  }
  s.n_mf[v.e] += new_mf;
  s.ep_ticks[v.e] += 1;
  if (terminated) v.flags |= F_TERM;
}

template <class V>
SFL_FN bool queue_empty(const V& v) {
  uint32_t any = 0;
#pragma unroll
  for (int w = 0; w < V::kNW; ++w) any |= v.msk[0][w];
  return any == 0;
}

// ---------------------------------------------------------------------------
// decision: observe (observer.py:246-308), epsilon-greedy (distr_q.py:312-319),
// _apply_action (switch_env.py:203-294)
// ---------------------------------------------------------------------------
struct Decision {
  int32_t sw, h, slot;
  uint32_t state;
  int32_t action, j;
  int32_t reward;
  int32_t next_sw;
};

// value of full-row action a (the full row is default_q except the compact entries)
template <class V>
SFL_FN double row_val(const V& v, int sw, int slot, const double* row, int a) {
  const SflMap& m = v.m;
  const int na = m.sw_na[sw];
  if (a == na - 1) return row[m.q_w[4 * sw + slot] - 1];
  if (m.act_src[sw * 8 + a] == (uint8_t)slot) return row[m.act_j[sw * 8 + a]];
  return m.default_q;
}

// np.argmax over the full row, falling back to the first allowed maximum (distr_q.py:468-490)
template <class V>
SFL_FN int max_action(const V& v, int sw, int slot, const double* row, const uint32_t amask) {
  const int na = v.m.sw_na[sw];
  int best = 0;
  double mx = row_val(v, sw, slot, row, 0);
  for (int a = 1; a < na; ++a) {
    const double val = row_val(v, sw, slot, row, a);
    if (val > mx) {
      mx = val;
      best = a;
    }
  }
  if ((amask >> best) & 1u) return best;
  int arg = -1;
  double amx = 0.0;
  for (int a = 0; a < na; ++a) {
    if (!((amask >> a) & 1u)) continue;
    const double val = row_val(v, sw, slot, row, a);
    if (arg < 0 || val > amx) {
      arg = a;
      amx = val;
    }
  }
  return arg;
}

// max(row) over the full, unmasked row (distr_q.py:449-466)
template <class V>
SFL_FN double row_max(const V& v, int sw, int slot, const double* row) {
  const int na = v.m.sw_na[sw];
  double mx = row_val(v, sw, slot, row, 0);
  for (int a = 1; a < na; ++a) {
    const double val = row_val(v, sw, slot, row, a);
    mx = val > mx ? val : mx;
  }
  return mx;
}

// rail_network.py:246-278 + 303-416
template <class V>
SFL_FN int transition_train(V& v, int h, int in_p, int out_p) {
  const SflMap& m = v.m;
  const int target = m.port_nb[out_p];
  if (v.state_of(h) != S_MALF) {
    v.free_switch_ports(v.next_port(h) >> 2, h);
    const uint16_t pp = v.prev_port(h);
    if (pp != PORT_NONE) v.free_switch_ports(pp >> 2, h);
  }
  const int32_t d_ot = m.port_len[out_p];
  v.sem_put_keep(out_p, h, 0, 3, 0);
  v.sem_put_keep(target, h, 1, d_ot + 1, 1);
  const int u = m.port_unique[target];
  if (u >= 0) {
    if (u != in_p && u != out_p && u != target) v.sem_put_replace(u, h, 0, d_ot + 1, 0);
    v.sem_put_replace(u, h, 0, d_ot, -1);
    const int far = m.port_nb[u];
    if (far != in_p && far != out_p && far != u) v.sem_put_replace(far, h, 1, d_ot + m.port_len[u] + 1, 1);
  }
  if (target != in_p && target != out_p) v.sem_put_replace(target, h, 0, d_ot + 1, 0);
  v.src_port(h) = (uint16_t)in_p;
  v.next_port(h) = (uint16_t)target;
  v.prev_port(h) = (uint16_t)out_p;
  return target >> 2;
}

// The decision of one agent_iter step, up to the point where the Q row is needed: the
// observation (observer.py:246-308) and the epsilon draw (distr_q.py:312-319).
struct Obs {
  int32_t h, sw, slot, explore, action;
  uint32_t state, amask;
  int32_t reward;
};

template <class V>
SFL_FN void decide_observe(V& v, Obs& o, bool greedy) {
  const SflMap& m = v.m;
  const SflState& s = v.s;
  // agent_iter: lowest queued train (switch_env.py:418-421, 616-622)
  int h = -1;
#pragma unroll
  for (int w = 0; w < V::kNW; ++w) {
    const uint32_t mk = v.msk[0][w];
    if (h < 0 && mk) {
      h = w * 32 + ctz32(mk);
      v.msk[0][w] = mk & (mk - 1u);
    }
  }
  if (h < 0) h = 0;
  const int sw = s.tr_dec[v.ix(h)];
  const int np = m.sw_np[sw];
  const int na = m.sw_na[sw];
  const int pin = v.next_port(h);
  int slot = pin & 3;
  if ((pin >> 2) != sw || slot >= np) {  // observer.py:294-301 (the reference would raise)
    v.err |= E_PORT;
    slot = 0;
  }
  // observe
  uint32_t free_bits = 0;
  for (int j = 0; j < np; ++j) {
    const int p = 4 * sw + j;
    if (!v.port_blocked(m.port_nb[p], p, h)) free_bits |= 1u << j;
  }
  const uint32_t b = v.bits(h);
  const int32_t pos = v.pos(h);
  const int32_t delay = v.now - m.tr_la[h] + v.dist(h, pos, (int)tb_dir(b));
  const int32_t avail = m.tr_la[h] - m.tr_ed[h];
  const uint32_t lvl = delay <= 0 ? 0u : (delay <= (int64_t)avail * m.delay_thr ? 1u : 2u);
  const uint32_t state = ((free_bits * (uint32_t)m.K) + (uint32_t)m.tr_k[h]) * 3u + lvl;
  uint32_t amask = 1u << (na - 1);
  for (int a = 0; a < na - 1; ++a)
    if (m.act_src[sw * 8 + a] == (uint8_t)slot && ((free_bits >> m.act_dst[sw * 8 + a]) & 1u)) amask |= 1u << a;
  o.h = h;
  o.sw = sw;
  o.slot = slot;
  o.state = state;
  o.amask = amask;
  o.reward = slot_rew(s.slot[v.ix((size_t)sw * m.T + h)], v.epoch);
  o.explore = 0;
  o.action = -1;
  // epsilon-greedy: the exploratory branch needs no Q value
  if (!greedy) {
    Pcg64 g = v.rng_load();
    const double eps = v.eps_of(s.counts[v.ix(sw)]);
    if (pcg_double(g) < eps) {
      o.explore = 1;
      const uint32_t sub_seed = pcg_bounded(g, 2147483646u);
      Pcg64 sub;
      pcg_from_seedseq(sub_seed, sub);
      const uint32_t nvalid = (uint32_t)popc32(amask);
      uint32_t pick = pcg_bounded(sub, nvalid - 1u);
      uint32_t mk = amask;
      for (uint32_t k = 0; k < pick; ++k) mk &= mk - 1u;
      o.action = ctz32(mk);
    }
    v.rng_store(g);
  }
}

// _apply_action (switch_env.py:203-294) for the chosen action
template <class V>
SFL_FN void decide_apply(V& v, const Obs& o, int action, Decision& d) {
  const SflMap& m = v.m;
  const SflState& s = v.s;
  const int h = o.h, sw = o.sw, slot = o.slot;
  const int na = m.sw_na[sw];
  const int pin = v.next_port(h);
  const uint32_t b = v.bits(h);
  const int32_t pos = v.pos(h);
  if (action < 0 || action >= na) v.err |= E_BAD_ACTION;
  const int stop = na - 1;
  bool moving = false;
  uint32_t turn = A_FWD;
  int in_p = pin, out_p = pin;
  if (action != stop && action >= 0 && action < na && (pin >> 2) == sw) {  // (no table read for a bad action)
    const int src = m.act_src[sw * 8 + action];
    if (src == slot) {
      moving = true;
      turn = m.act_turn[sw * 8 + action];
      in_p = 4 * sw + src;
      out_p = 4 * sw + m.act_dst[sw * 8 + action];
    }
  }
  int next_sw = sw;
  int target = -1;
  if (moving) {
    next_sw = transition_train(v, h, in_p, out_p);
    target = m.port_nb[out_p];
  }
  uint32_t p = v.plan(h);
  if (moving && pl_len(p) > 0) {
    p = (p & 0xF0u) | 1u;  // plan[:1]
    p = pl_push_back(p, turn, v.err);
  } else if (!moving) {
    p = pl_push_front(p, A_STOP, v.err);
  } else {
    p = pl_push_back(p, A_FWD, v.err);
    p = pl_push_back(p, turn, v.err);
  }
  v.plan(h) = p;
  bool all_blocked;
  if (moving) {
    all_blocked = v.port_blocked(target, out_p, h);
  } else {
    all_blocked = true;
    for (int a = 0; a < na - 1; ++a) {
      if (m.act_src[sw * 8 + a] != (uint8_t)slot) continue;
      const int o2 = 4 * sw + m.act_dst[sw * 8 + a];
      if (!v.port_blocked(m.port_nb[o2], o2, h)) all_blocked = false;
    }
  }
  // reward_func.py:23-78: project the position along the non-STOP plan
  int pc = pos, pd = (int)tb_dir(b);
  const uint32_t n = pl_len(p);
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t a = pl_at(p, i);
    if (a == A_STOP) continue;
    if (pc < 0) break;
    typename V::Move mv = v.check_action(a, pc, pd);
    pc = mv.cell;
    pd = mv.dir;
  }
  const int32_t cur = v.now - m.tr_la[h] + v.dist(h, pc, pd);
  const int32_t diff = s.tr_delay[v.ix(h)] - cur;
  const int32_t r_new = (pl_front(p) == A_STOP && !all_blocked) ? diff - 1300 : diff;
  uint64_t& sl = s.slot[v.ix((size_t)next_sw * m.T + h)];
  sl = slot_make(slot_pend(sl, v.epoch), r_new, v.epoch);
  s.tr_delay[v.ix(h)] = cur;

  d.sw = sw;
  d.h = h;
  d.slot = slot;
  d.state = o.state;
  d.action = action;
  d.j = (action == stop) ? (m.q_w[4 * sw + slot] - 1) : m.act_j[sw * 8 + action];
  d.reward = o.reward;
  d.next_sw = next_sw;
}

template <class V>
SFL_FN void env_decide(V& v, Decision& d, bool greedy) {
  Obs o;
  decide_observe(v, o, greedy);
  int action = o.action;
  if (!o.explore) {
    v.touch(o.sw, o.slot, o.state);
    action = max_action(v, o.sw, o.slot, v.qrow(o.sw, o.slot, o.state), o.amask);
  }
  decide_apply(v, o, action, d);
}

// Q-table access of the post step.  LocalQ: this env's own table (the fused kernels);
// the graph-partitioned mode (sfl_part.h) sends the same operations to the switch's owner.
template <class V>
struct LocalQ {
  V& v;
  SFL_FN void touch(int sw, int slot, uint32_t state) { v.touch(sw, slot, state); }
  SFL_FN double row_max_of(const Decision& d) { return row_max(v, d.sw, d.slot, v.qrow(d.sw, d.slot, d.state)); }
  // q <- (1 - lr) * q + lr * target, the reference's operation order (distr_q.py:436-447)
  SFL_FN void update(int ps, int pslot, uint32_t pstate, int pj, double lr, double target, int /*stage*/) {
    double* q = v.qrow(ps, pslot, pstate) + pj;
    const double a = (1.0 - lr) * *q;
    const double bb = lr * target;
    *q = a + bb;
  }
};

// post-step part of the learn loop (distr_q.py:322-362).  stage: 0 for the pending update,
// 1 + i for the destination bonus of the i-th newly arrived train (operations of one stage
// never touch the same Q cell; stages must be applied in order).
template <class V, class Q>
SFL_FN void env_post(V& v, const Decision& d, Q& q) {
  const SflMap& m = v.m;
  const SflState& s = v.s;
  uint64_t& here = s.slot[v.ix((size_t)d.sw * m.T + d.h)];
  const uint32_t pend = slot_pend(here, v.epoch);
  if (pend != PEND_NONE) {
    const int ps = (int)(pend & 0xFFFu);
    const int pslot = (int)((pend >> 12) & 3u);
    const uint32_t pstate = (pend >> 14) & 0x3FFFu;
    const int pj = (int)((pend >> 28) & 3u);
    q.touch(ps, pslot, pstate);
    const double lr = v.lr_of(s.counts[v.ix(ps)], v.err);
    const double r = (double)d.reward;
    if (d.sw != ps) {
      q.touch(d.sw, d.slot, d.state);
      const double mq = q.row_max_of(d);
      q.update(ps, pslot, pstate, pj, lr, r + m.gamma * mq, 0);
    } else {
      q.update(ps, pslot, pstate, pj, lr, r, 0);
    }
    here = slot_make(PEND_NONE, slot_rew(here, v.epoch), v.epoch);
  }
  uint64_t& nxt = s.slot[v.ix((size_t)d.next_sw * m.T + d.h)];
  nxt = slot_make(pend_make((uint32_t)d.sw, (uint32_t)d.slot, d.state, (uint32_t)d.j), slot_rew(nxt, v.epoch), v.epoch);
  // destination bonus for newly arrived trains (distr_q.py:344-356)
  int stage = 1;
#pragma unroll
  for (int w = 0; w < V::kNW; ++w) {
    uint32_t fresh = v.msk[1][w] & ~v.msk[2][w];
    if (!fresh) continue;
    v.msk[2][w] |= fresh;
    while (fresh) {
      const int tr = w * 32 + ctz32(fresh);
      fresh &= fresh - 1u;
      for (int sw2 = 0; sw2 < m.S; ++sw2) {
        uint64_t& sl = s.slot[v.ix((size_t)sw2 * m.T + tr)];
        const uint32_t pe = slot_pend(sl, v.epoch);
        if (pe == PEND_NONE) continue;
        const int ps = (int)(pe & 0xFFFu);
        const int pslot = (int)((pe >> 12) & 3u);
        const uint32_t pstate = (pe >> 14) & 0x3FFFu;
        const int pj = (int)((pe >> 28) & 3u);
        q.touch(ps, pslot, pstate);
        const double lr = v.lr_of(s.counts[v.ix(ps)], v.err);
        q.update(ps, pslot, pstate, pj, lr, 1000.0 + m.gamma * 0.0, stage);
        sl = slot_make(PEND_NONE, slot_rew(sl, v.epoch), v.epoch);
      }
      ++stage;
    }
  }
  s.counts[v.ix(d.sw)] += 1u;
}

template <class V>
SFL_FN void env_post(V& v, const Decision& d) {
  LocalQ<V> q{v};
  env_post(v, d, q);
}

// order-independent checksum of the semaphore table (trace/debug only)
template <class V>
SFL_FN uint64_t sem_checksum(const V& v) {
  uint64_t c = 0;
  for (int p = 0; p < v.m.NP; ++p) {
    const uint64_t r = v.sem(p);
    if (sem_present(r)) c += mix64(((uint64_t)p << 42) ^ r);
  }
  return c;
}

template <class V>
SFL_FN void trace_decision(const V& v, const SflCtl& c, const Decision& d) {
  const uint64_t n = *c.trace_n;
  if (n < (uint64_t)c.trace_cap) {
    uint64_t* t = c.trace + 4 * n;
    t[0] = (uint64_t)(uint32_t)v.now | ((uint64_t)(uint32_t)d.sw << 16) | ((uint64_t)(uint32_t)d.h << 32) |
           ((uint64_t)(uint32_t)d.action << 48);
    t[1] = (uint64_t)d.state | ((uint64_t)(uint32_t)d.reward << 32);
    t[2] = sem_checksum(v);
    t[3] = (uint64_t)(uint32_t)d.next_sw;
  }
  *c.trace_n = n + 1;
}

// any lane of the wave (host build: a wave of one lane)
SFL_FN bool wave_any(bool pred) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __ballot(pred) != 0ull;
#else
  return pred;
#endif
}

// ---------------------------------------------------------------------------
// driver: one env until its episode target / decision budget
// ---------------------------------------------------------------------------
template <int NW>
SFL_FN void env_run(const SflMap& m, const SflState& s, const SflCtl& c, uint32_t e) {
  using V = Env<NW>;
  V v(m, s, e);
  v.flags = s.eflags[e];
  v.now = s.elapsed[e];
  v.epoch = s.epoch[e];
  v.err = s.err[e];
  int32_t phase = s.phase[e];
  uint64_t dec = 0, ticks = 0, abytes = 0;
  Decision d;
  d.sw = d.h = d.slot = d.action = d.j = d.reward = d.next_sw = 0;
  d.state = 0;
  double cum = s.cum_reward[e];
  const bool test_mode = c.mode == 1;
  v.masks_load();
  while (true) {
    const bool busy = wave_any(phase == PH_DECIDE || phase == PH_POST);
    if (phase == PH_RESET) {
      // learn: optional greedy round before episode t (distr_q.py:278-281)
      if (test_mode) {
        if (c.ep_target >= 0 && s.n_test[e] >= c.ep_target) break;
        v.flags |= F_GREEDY;
      } else {
        if (c.ep_target >= 0 && s.ep_t[e] >= c.ep_target) break;
        const int32_t t = s.ep_t[e];
        if (c.exploit_freq > 0 && (t + 1) % c.exploit_freq == 0 && !(v.flags & F_EXPLOIT_DONE)) v.flags |= F_GREEDY;
        else v.flags &= ~F_GREEDY;
      }
      env_reset(v);
      cum = 0.0;
      phase = PH_TICK;
    } else if (phase == PH_TICK) {
      // Wave-synchronised ticking: a lane that needs a Flatland tick waits while any lane of
      // its wave still has queued decisions, so the (expensive) tick body runs once per
      // round for the whole wave instead of in almost every iteration.  Scheduling only:
      // each env's own sequence of operations is unchanged.
      if (!busy) {
        int live = m.T;
#pragma unroll
        for (int w = 0; w < V::kNW; ++w) live -= popc32(v.msk[1][w]);
        abytes += 36ull * (uint64_t)live;
        env_tick(v);
        ticks++;
        if (v.flags & F_TERM) phase = (v.flags & F_INFLIGHT) ? PH_POST : PH_END;
        else if (!queue_empty(v)) phase = (v.flags & F_INFLIGHT) ? PH_POST : PH_DECIDE;
      }
    } else if (phase == PH_DECIDE || phase == PH_POST) {
      bool post_now = phase == PH_POST;
      if (phase == PH_DECIDE) {
        env_decide(v, d, (v.flags & F_GREEDY) != 0);
        abytes += 220ull + 48ull * m.sw_np[d.sw] + 8ull * m.sw_na[d.sw];
        v.flags |= F_INFLIGHT;
        if (queue_empty(v)) phase = PH_TICK;  // ticks happen between the step and the update
        else post_now = true;
      }
      if (post_now) {
        if (!(v.flags & F_GREEDY)) env_post(v, d);
        if (c.trace && (int32_t)e == c.trace_env) trace_decision(v, c, d);
        v.flags &= ~F_INFLIGHT;
        cum += (double)d.reward;
        s.ep_dec[e] += 1;
        s.dec_total[e] += 1;
        s.step_ctr[e] += 1;
        if (s.step_ctr[e] > m.max_steps) v.flags |= F_TRUNC;
        dec++;
        phase = (v.flags & (F_TERM | F_TRUNC)) ? PH_END : PH_DECIDE;
        if (c.dec_budget > 0 && (int64_t)dec >= c.dec_budget) break;
      }
    } else {  // PH_END
      int arrived = 0;
#pragma unroll
      for (int w = 0; w < V::kNW; ++w) arrived += popc32(v.msk[1][w]);
      const size_t cap = (size_t)(c.stats_cap > 0 ? c.stats_cap : 1);
      if (v.flags & F_GREEDY) {
        if (test_mode) {
          const int32_t i = s.n_test[e];
          if (c.st_cum && c.stats_cap > 0) {
            const size_t row = (size_t)(i - c.stats_base) % cap;
            c.st_cum[row * s.E + e] = cum;
            c.st_arrived[row * s.E + e] = arrived;
            c.st_mf[row * s.E + e] = s.n_mf[e];
            c.st_dec[row * s.E + e] = s.ep_dec[e];
            c.st_ticks[row * s.E + e] = s.ep_ticks[e];
            for (int h = 0; h < m.T; ++h) c.st_delays[(row * m.T + h) * s.E + e] = s.tr_delay[v.ix(h)];
          }
          s.n_test[e] += 1;
        } else {
          const int32_t i = s.ep_t[e];
          if (c.sx_cum && c.stats_cap > 0) {
            const size_t row = (size_t)(i - c.stats_base) % cap;
            c.sx_cum[row * s.E + e] = cum;
            c.sx_arrived[row * s.E + e] = arrived;
          }
          v.flags |= F_EXPLOIT_DONE;
        }
      } else {
        const int32_t i = s.ep_t[e];
        if (c.st_cum && c.stats_cap > 0) {
          const size_t row = (size_t)(i - c.stats_base) % cap;
          c.st_cum[row * s.E + e] = cum;
          c.st_arrived[row * s.E + e] = arrived;
          c.st_mf[row * s.E + e] = s.n_mf[e];
          c.st_dec[row * s.E + e] = s.ep_dec[e];
          c.st_ticks[row * s.E + e] = s.ep_ticks[e];
          for (int h = 0; h < m.T; ++h) c.st_delays[(row * m.T + h) * s.E + e] = s.tr_delay[v.ix(h)];
        }
        s.ep_t[e] += 1;
        v.flags &= ~F_EXPLOIT_DONE;
      }
      phase = PH_RESET;
    }
  }
  v.masks_store();
  s.phase[e] = phase;
  s.elapsed[e] = v.now;
  s.eflags[e] = v.flags;
  s.epoch[e] = v.epoch;
  s.err[e] = v.err;
  s.cum_reward[e] = cum;
  if (c.launch_dec) c.launch_dec[e] = dec;
  if (c.launch_ticks) c.launch_ticks[e] = ticks;
  if (c.launch_bytes) c.launch_bytes[e] = abytes;
}

// ---------------------------------------------------------------------------
// external-action mode (SflExt): one env, one decision per call, the action from the host
// ---------------------------------------------------------------------------
// The env's operations are env_run's in the same order (reset, ticks, observe, apply, the deferred
// post point after the ticks), without the learner: no epsilon draw, no Q-table, no pending updates;
// the post point only counts the step and checks max_steps (switch_env.py:652-657).
template <int NW>
SFL_FN void env_run_ext(const SflMap& m, const SflState& s, const SflCtl& c, uint32_t e) {
  using V = Env<NW>;
  const SflExt& x = *c.ext;
  V v(m, s, e);
  v.flags = s.eflags[e];
  v.now = s.elapsed[e];
  v.epoch = s.epoch[e];
  v.err = s.err[e];
  int32_t phase = s.phase[e];
  uint64_t ticks = 0;
  Decision d;
  d.sw = d.h = d.slot = d.action = d.j = d.reward = d.next_sw = 0;
  d.state = 0;
  v.masks_load();
  x.agent[e] = -1;
  x.next_sw[e] = -1;
  x.step_now[e] = -1;
  int32_t act = x.actions[e];
  bool applied = false;
  if (act == -2) {  // SFL_ACTION_RESET (sfl.h), env.reset() mid-episode: the episode-end reset, where the env stands
    phase = PH_RESET;
    v.flags &= ~(F_EXT_OBS | F_INFLIGHT);
    act = -1;
  }
  while (true) {
    if (phase == PH_RESET) {
      env_reset(v);
      phase = PH_TICK;
    } else if (phase == PH_TICK) {
      env_tick(v);
      ticks++;
      if (v.flags & F_TERM) phase = (v.flags & F_INFLIGHT) ? PH_POST : PH_END;
      else if (!queue_empty(v)) phase = (v.flags & F_INFLIGHT) ? PH_POST : PH_DECIDE;
    } else if (phase == PH_DECIDE) {
      const bool apply = (v.flags & F_EXT_OBS) && !applied && act >= 0;
      uint32_t keep[NW];
#pragma unroll
      for (int w = 0; w < NW; ++w) keep[w] = v.msk[0][w];
      Obs o;
      decide_observe(v, o, true);
      // an action outside the switch's action space is refused before it touches the env (the reference's
      // assert, switch_env.py:213-215): E_BAD_ACTION, and the same observation is emitted again
      const bool bad = apply && act >= m.sw_na[o.sw];
      if (bad) v.err |= E_BAD_ACTION;
      if (!apply || bad) {
        // emit the observation of the queue's first train (agent_iter + last(); the queue is left
        // as it is: the next call observes it again and applies the action)
#pragma unroll
        for (int w = 0; w < NW; ++w) v.msk[0][w] = keep[w];
        x.agent[e] = o.sw;
        x.train[e] = o.h;
        x.slot[e] = o.slot;
        x.state[e] = o.state;
        x.mask[e] = o.amask;
        x.reward[e] = o.reward;
        x.now[e] = v.now;
        v.flags |= F_EXT_OBS;
        break;
      }
      decide_apply(v, o, act, d);
      v.flags &= ~F_EXT_OBS;
      v.flags |= F_INFLIGHT;
      applied = true;
      x.next_sw[e] = d.next_sw;
      phase = queue_empty(v) ? PH_TICK : PH_POST;  // no active switch left: move the trains first
    } else if (phase == PH_POST) {
      // the step() of the applied action returns here (after the ticks when the queue emptied)
      if (c.trace && (int32_t)e == c.trace_env) trace_decision(v, c, d);
      v.flags &= ~F_INFLIGHT;
      x.step_now[e] = v.now;
      s.ep_dec[e] += 1;
      s.dec_total[e] += 1;
      s.step_ctr[e] += 1;
      if (s.step_ctr[e] > m.max_steps) v.flags |= F_TRUNC;
      phase = (v.flags & (F_TERM | F_TRUNC)) ? PH_END : PH_DECIDE;
    } else {  // PH_END: report the episode (the learner records arrivals, delays, malfunctions)
      x.truncated[e] = (v.flags & F_TRUNC) ? 1 : 0;
      x.agent[e] = -1;
      v.flags &= ~F_EXT_OBS;
      phase = PH_RESET;
      break;
    }
  }
  // the episode's delays and malfunction count as they stand (its final values when agent == -1)
  for (int h = 0; h < m.T; ++h) x.delays[(size_t)h * s.E + e] = s.tr_delay[v.ix(h)];
  x.n_mf[e] = s.n_mf[e];
  if (x.agent[e] >= 0) x.truncated[e] = 0;
#pragma unroll
  for (int w = 0; w < MAXW; ++w) x.arrived[(size_t)w * s.E + e] = w < NW ? v.msk[1][w < NW ? w : 0] : 0u;
  v.masks_store();
  s.phase[e] = phase;
  s.elapsed[e] = v.now;
  s.eflags[e] = v.flags;
  s.epoch[e] = v.epoch;
  s.err[e] = v.err;
  if (c.launch_dec) c.launch_dec[e] = applied ? 1u : 0u;
  if (c.launch_ticks) c.launch_ticks[e] = ticks;
  if (c.launch_bytes) c.launch_bytes[e] = 0;
}

}  // namespace sfl
