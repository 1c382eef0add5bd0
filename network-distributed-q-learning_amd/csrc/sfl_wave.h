// Wave-cooperative SwitchFL kernel body (gfx950): one environment per 64-lane wavefront.
//
// Same operations, in the same per-env order, as env_run in sfl_core.h (the lane-per-env
// body, kept for T > 64 and for the host test build), but the env's hot state lives in
// VGPRs for the whole launch:
//   * lane h holds train h (cell, packed bits, plan, ports, delay, its timetable constants);
//   * lane p % 64, register p / 64 holds the semaphore record of port p (32-bit packed);
//   * lane s % 64, register s / 64 holds agent_num_interactions of switch s.
// A Flatland tick runs train-parallel (one lane per train); conflict resolution, the
// purge of arrived trains, extend_semaphores and the decision queue are wave ballots and
// per-lane scans of the lanes' own records.  A decision is wave-uniform: cross-lane reads
// are v_readlane, the read-only map tables are packed per switch / port / train
// (SflMap::sw_pack, port_pack, tr_pack) and read with one scalar load each, check_action is
// a table lookup (move_tab), and only the Q-table, the (switch, train) slots and the distance
// maps reach L2/HBM.  Loads whose results are needed later (the Q row, the pending update's
// Q cell, the slot word) are issued early and made wave-uniform only where they are used.
#pragma once
#include <hip/hip_runtime.h>

#include <type_traits>

#include "sfl_core.h"
#include "sfl_part.h"
#include "sfl_experiment.h"

namespace sfl {
namespace wave {

#ifndef SFL_PF_RING
// grouped shapes with two train slots per lane: prefetch records per env (0: one per train).  A ring
// of 10 fits four 16-env blocks per CU (40.4 KB each), and 4 waves per SIMD then have to live in
// 128 VGPRs: with the env's Q / key-set / slot base pointers held in registers 86 spilled (c3
// 1,097 M vs 1,308 M at 3 waves); recomputed from the env index at each use (qbase / tbase /
// sbase) 57, mostly in the episode-end bookkeeping: 1,351 M vs 1,298 M (3 waves, no ring).  Round 6: 12 -- the
// largest ring that still fits four blocks per CU (40,448 B per block; up to 16 records the staged offsets stay one
// register per lane) -- c3 1,640-1,644 M vs 1,611-1,615 M for 10, +1.8 %; 11: 1,558 M, 8: 1,576 M
// (profiles/r06p_pf_ring_ab.txt)
#define SFL_PF_RING 12
#endif
#ifndef SFL_PF_RING64
#define SFL_PF_RING64 16  // one env per wavefront with two train slots per lane (c5, k_wave2): see WEnv::RING
#endif
#ifndef SFL_TICK_HOLD
#define SFL_TICK_HOLD 2  // run_groups: ticks wait while this many groups of the wave can still decide
#endif
#ifndef SFL_TICK_REMMIN
#define SFL_TICK_REMMIN 5  // ... and one of them has fewer than this many decisions left (0: hold regardless)
#endif
#ifdef SFL_PROFILE
// tuning builds only: wall cycles per phase summed over waves (reset, tick, decide, post, total,
// decide = observe + egreedy + apply)
static __device__ unsigned long long g_prof[32];  // (one per translation unit: sfl_kwave_v7.hip has its own)
#define SFL_PCNT(k) (prof[k] += 1)
#define SFL_LAP0() (lap_t = (uint64_t)__builtin_amdgcn_s_memtime())
#define SFL_LAP(k)                                                 \
  do {                                                             \
    const uint64_t _t = (uint64_t)__builtin_amdgcn_s_memtime();   \
    lap[k] += _t - lap_t;                                          \
    lap_t = _t;                                                    \
  } while (0)
#define SFL_PT(var) const uint64_t var = (uint64_t)__builtin_amdgcn_s_memtime()
#define SFL_PACC(k, t0) prof[k] += (uint64_t)__builtin_amdgcn_s_memtime() - (t0)
#else
#define SFL_PT(var)
#define SFL_PACC(k, t0)
#define SFL_PCNT(k)
#define SFL_LAP0()
#define SFL_LAP(k)
#endif

// Wave priorities (s_setprio: the SIMD's issue arbiter prefers higher-priority waves): a wave in a tick above one
// in a decision above one in its post step / bookkeeping.  Round 5 (profiles/r05ag_wave_priority_ab.txt): tick 2,
// decide 1 -- c3 +2.1 %, c2 at 4,096 envs +3.8 %, c2 at 65,536 envs +4.1 %, c5 fused +1.3 %; the tick must rank above
// the decision (equal priorities lose the gain); the prefetch's own priority adds nothing; the partitioned local
// step keeps the default priority (-1 % with them).
#ifndef SFL_SETPRIO_PF
#define SFL_SETPRIO_PF 0  // while the batch prefetch issues its loads (0: the caller's)
#endif
#ifndef SFL_SETPRIO_TICK
#define SFL_SETPRIO_TICK 2  // during a tick (0: unchanged)
#endif
#ifndef SFL_SETPRIO_DECIDE
#define SFL_SETPRIO_DECIDE 1  // during a decision (0: unchanged)
#endif
template <int P>
struct PrioGuard {  // s_setprio P for the scope (P = 0: nothing)
  __device__ __forceinline__ PrioGuard() {
    if constexpr (P > 0) __builtin_amdgcn_s_setprio(P);
  }
  __device__ __forceinline__ ~PrioGuard() {
    if constexpr (P > 0) __builtin_amdgcn_s_setprio(0);
  }
};
constexpr uint32_t PF_NONE = 0xFFFFFFFFu;
// batch-prefetch record per train: doubles -- the pending cell, the slot word, the staged row's max;
// words -- distance-map values at the train's cell (observation), at its projected cell if it stops
// (reward of STOP), if it moves with final rail action 1..3 (reward of a route), and the row's
// argmax | first allowed argmax << 8 under the staged observation (the row's columns themselves are
// not kept: a decision on a staged row needs only its max and argmaxes)
constexpr int PF_D = 3, PF_WI = 3;  // doubles and 32-bit words of a prefetch record (stored apart: [TW][3] each)
constexpr int PF_WORDS = 2 * PF_D + PF_WI;
// (doubles: pending cell value, slot word, row max; words: 0 distance at the cell | along the STOP
// plan << 16, 1 route final action 1 | 2 << 16, 2 route final action 3 | argmax pack << 16 (int16
// distances, see d16))
// distances staged as int16: off the grid -> INT16_MIN, unreachable -> INT16_MAX (choose_variant
// checks that every finite distance of the map is below 32767)
__device__ __forceinline__ uint32_t d16(int32_t d) {
  const int32_t v = d == (int32_t)0x80000000 ? -32768 : (d >= 32767 ? 32767 : d);
  return (uint32_t)v & 0xFFFFu;
}
__device__ __forceinline__ int32_t d16_lo(uint32_t w) {
  const int32_t v = (int32_t)(int16_t)(w & 0xFFFFu);
  return v == -32768 ? (int32_t)0x80000000 : (v == 32767 ? DIST_INF : v);
}
__device__ __forceinline__ int32_t d16_hi(uint32_t w) { return d16_lo(w >> 16); }
// epsilon staged with the batch (round 6): the grouped shapes (G < 64, <= 64 switches) stage, with each queued
// train's record, eps_tab[n] of its decision switch as the switch's interaction count n stands at staging (record
// double 3); the decision compares against it instead of loading eps_tab[n] behind the count (one dependent vector
// load off the decision's chain).  A switch decided on since the staging has a stale value (its count moved): the
// env's LDS word lrng[5] marks those switches, and their decisions load eps_tab[n] as before.  Measured and NOT the
// default (profiles/r06e_eps_staging_ab.txt, same box, parity ok): c3 1,590-1,593 M vs 1,611-1,612 M, c2 at 4,096
// envs 335.5 M vs 345.6 M -- the staged value's live range and the lrng[5] read-modify-write cost the variant-7 kernel
// 12 more spill instructions (40 -> 52, scripts/spills.py), some of them in the decision and staging paths, and the
// staging adds a counter read and a load to every staged record.  1: on (A/B builds)
#ifndef SFL_EPS_PF
#define SFL_EPS_PF 0
#endif
#ifndef SFL_WAVE_BLOCK
#define SFL_WAVE_BLOCK 256  // threads per k_wave block (envs per block x 64)
#endif
#ifndef SFL_GROUP_BLOCK
#define SFL_GROUP_BLOCK SFL_WAVE_BLOCK  // threads per k_wave_g block (run_groups: envs per block x G)
#endif
constexpr int32_t PF_OFFGRID = (int32_t)0x80000000;  // projection left the grid

#define SFL_AS_G __attribute__((address_space(1)))
#define SFL_AS_C __attribute__((address_space(4)))

template <class T, int N>
using vec_t = T __attribute__((ext_vector_type(N)));
using u4 = vec_t<uint32_t, 4>;
using u8 = vec_t<uint32_t, 8>;

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
template <class V>
__device__ __forceinline__ V ldcv(const void* p, size_t i) {
  return ((const SFL_AS_C V*)p)[i];
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

// semaphore record in a VGPR / LDS word and in the env-major state between launches (R_* in
// sfl_core.h): t0 14 (signed) | t1 - t0 9 | owner 7 | in 1 | present 1 (ticks -8192..8191 and
// spans up to 511: choose_variant checks the map's timetable and port lengths)
__device__ __forceinline__ uint32_t r_pack(uint32_t owner, uint32_t in, int32_t t0, int32_t t1) {
  return ((uint32_t)t0 & R_T0_MASK) | (((uint32_t)(t1 - t0) & R_DUR_MASK) << R_T0_BITS) | ((owner & 0x7Fu) << R_OWNER_SHIFT) |
         ((in & 1u) << 30) | (1u << 31);
}
__device__ __forceinline__ bool r_present(uint32_t r) { return (r >> 31) != 0u; }
__device__ __forceinline__ uint32_t r_in(uint32_t r) { return (r >> 30) & 1u; }
__device__ __forceinline__ uint32_t r_owner(uint32_t r) { return (r >> R_OWNER_SHIFT) & 0x7Fu; }
__device__ __forceinline__ int32_t r_t0(uint32_t r) { return ((int32_t)(r << (32 - R_T0_BITS))) >> (32 - R_T0_BITS); }
__device__ __forceinline__ uint32_t r_dur(uint32_t r) { return (r >> R_T0_BITS) & R_DUR_MASK; }
__device__ __forceinline__ int32_t r_t1(uint32_t r) { return r_t0(r) + (int32_t)r_dur(r); }
// the same record restarted at tick t (extend_semaphores: span kept)
__device__ __forceinline__ uint32_t r_retime(uint32_t r, int32_t t) { return (r & ~R_T0_MASK) | ((uint32_t)t & R_T0_MASK); }
__device__ __forceinline__ uint64_t r_to64(uint32_t r) {
  return r_present(r) ? sem_pack(r_owner(r), r_in(r), r_t0(r), r_t1(r)) : 0ull;
}

// decay**n beyond the host-computed tables (rare): out of line, so the f64 pow expansion does
// not set the register budget of the whole kernel
__device__ __attribute__((noinline)) double pow_ool(double base, double n) { return pow(base, n); }

__device__ __forceinline__ int ctz64(uint64_t x) { return __builtin_ctzll(x); }
__device__ __forceinline__ int popc64(uint64_t x) { return __builtin_popcountll(x); }

// Train masks.  A map with up to 64 trains keeps one train per lane and 64-bit masks; up to 128
// trains, lane l holds trains l and l + 64 (TPL = 2 "train slots" per lane) and a mask is two
// words.  The helpers below are overloaded on both, so the TPL = 1 code is the plain uint64_t code.
struct M2 {
  uint64_t w[2];
};
__device__ __forceinline__ M2 operator|(M2 a, M2 b) { return M2{{a.w[0] | b.w[0], a.w[1] | b.w[1]}}; }
__device__ __forceinline__ M2 operator&(M2 a, M2 b) { return M2{{a.w[0] & b.w[0], a.w[1] & b.w[1]}}; }
__device__ __forceinline__ M2 operator~(M2 a) { return M2{{~a.w[0], ~a.w[1]}}; }
__device__ __forceinline__ M2& operator|=(M2& a, M2 b) { return a = a | b; }
__device__ __forceinline__ M2& operator&=(M2& a, M2 b) { return a = a & b; }
__device__ __forceinline__ bool operator==(M2 a, M2 b) { return a.w[0] == b.w[0] && a.w[1] == b.w[1]; }
// one 32-bit word for up to 32 trains (bit indices >= 32 read as 0)
__device__ __forceinline__ bool many(uint32_t m) { return m != 0u; }
__device__ __forceinline__ int mctz(uint32_t m) { return __builtin_ctz(m); }
__device__ __forceinline__ void mclear_low(uint32_t& m) { m &= m - 1u; }
__device__ __forceinline__ int mpopc(uint32_t m) { return __builtin_popcount(m); }
__device__ __forceinline__ bool mbit(uint32_t m, int i) { return (i < 32) & (((m >> (i & 31)) & 1u) != 0u); }
__device__ __forceinline__ uint32_t mone(uint32_t, int i) { return 1u << i; }
__device__ __forceinline__ uint32_t mbelow(uint32_t, int i) { return (1u << i) - 1u; }
__device__ __forceinline__ int mhighest(uint32_t m) { return 31 - __builtin_clz(m); }
__device__ __forceinline__ uint32_t mfirst(uint32_t, int n) { return n >= 32 ? ~0u : (1u << n) - 1u; }
__device__ __forceinline__ bool many(uint64_t m) { return m != 0ull; }
__device__ __forceinline__ bool many(M2 m) { return (m.w[0] | m.w[1]) != 0ull; }
__device__ __forceinline__ int mctz(uint64_t m) { return ctz64(m); }
__device__ __forceinline__ int mctz(M2 m) { return m.w[0] ? ctz64(m.w[0]) : 64 + ctz64(m.w[1]); }
__device__ __forceinline__ void mclear_low(uint64_t& m) { m &= m - 1ull; }
__device__ __forceinline__ void mclear_low(M2& m) {
  if (m.w[0]) m.w[0] &= m.w[0] - 1ull;
  else m.w[1] &= m.w[1] - 1ull;
}
__device__ __forceinline__ int mpopc(uint64_t m) { return popc64(m); }
__device__ __forceinline__ int mpopc(M2 m) { return popc64(m.w[0]) + popc64(m.w[1]); }
__device__ __forceinline__ bool mbit(uint64_t m, int i) { return ((m >> i) & 1ull) != 0ull; }
__device__ __forceinline__ bool mbit(M2 m, int i) { return (((i & 64) ? m.w[1] : m.w[0]) >> (i & 63)) & 1ull; }
__device__ __forceinline__ uint64_t mone(uint64_t, int i) { return 1ull << i; }
__device__ __forceinline__ M2 mone(M2, int i) { return (i & 64) ? M2{{0ull, 1ull << (i & 63)}} : M2{{1ull << i, 0ull}}; }
// bits below i (i < 64 for one word, < 128 for two)
__device__ __forceinline__ uint64_t mbelow(uint64_t, int i) { return (1ull << i) - 1ull; }
__device__ __forceinline__ M2 mbelow(M2, int i) {
  return (i & 64) ? M2{{~0ull, (1ull << (i & 63)) - 1ull}} : M2{{(1ull << i) - 1ull, 0ull}};
}
__device__ __forceinline__ int mhighest(uint64_t m) { return 63 - __builtin_clzll(m); }
__device__ __forceinline__ int mhighest(M2 m) { return m.w[1] ? 127 - __builtin_clzll(m.w[1]) : 63 - __builtin_clzll(m.w[0]); }
__device__ __forceinline__ uint64_t mfirst(uint64_t, int n) { return n >= 64 ? ~0ull : (1ull << n) - 1ull; }
__device__ __forceinline__ M2 mfirst(M2, int n) {
  return n >= 128 ? M2{{~0ull, ~0ull}} : n >= 64 ? M2{{~0ull, (n == 64) ? 0ull : (1ull << (n - 64)) - 1ull}} : M2{{(1ull << n) - 1ull, 0ull}};
}
// index of the i-th set bit (i < popcount; per lane): binary search on popcounts, branch-free
__device__ __forceinline__ int mselect(uint32_t m, int i) {
  int base = 0;
#pragma unroll
  for (int w = 16; w >= 1; w >>= 1) {
    const int c = __builtin_popcount(m & ((1u << w) - 1u));
    const bool up = i >= c;
    i = up ? i - c : i;
    m = up ? m >> w : m;
    base = up ? base + w : base;
  }
  return base;
}
__device__ __forceinline__ int mselect(uint64_t m, int i) {
  const int c = __builtin_popcount((uint32_t)m);
  return i >= c ? 32 + mselect((uint32_t)(m >> 32), i - c) : mselect((uint32_t)m, i);
}
__device__ __forceinline__ int mselect(M2 m, int i) {
  const int c = popc64(m.w[0]);
  return i >= c ? 64 + mselect(m.w[1], i - c) : mselect(m.w[0], i);
}
// train masks: one 32-bit word for up to 32 trains, one 64-bit word for up to 64, two (M2) for up to 128
template <int BITS>
struct MaskOf {
  using type = typename std::conditional<(BITS <= 32), uint32_t,
                                         typename std::conditional<(BITS <= 64), uint64_t, M2>::type>::type;
};

// max over each quad of lanes (DPP quad permutes; the result is valid in every lane of the quad)
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double x) {
  const long long u = __double_as_longlong(x);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)u, CTRL, 0xF, 0xF, false);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(u >> 32), CTRL, 0xF, 0xF, false);
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
__device__ __forceinline__ double quad_max(double x) {
  x = fmax(x, dpp_f64<0xB1>(x));  // quad_perm [1,0,3,2]
  return fmax(x, dpp_f64<0x4E>(x));  // quad_perm [2,3,0,1]
}

// packed switch record (SflMap::sw_pack), wave-uniform
struct SwRec {
  u8 w;
  __device__ __forceinline__ int np() const { return (int)(w[0] & 15u); }
  __device__ __forceinline__ int na() const { return (int)((w[0] >> 4) & 15u); }
  __device__ __forceinline__ int src(int a) const { return (int)((w[1] >> (2 * a)) & 3u); }
  __device__ __forceinline__ int dst(int a) const { return (int)((w[1] >> (16 + 2 * a)) & 3u); }
  __device__ __forceinline__ uint32_t turn(int a) const { return (w[2] >> (2 * a)) & 3u; }
  __device__ __forceinline__ int j(int a) const { return (int)((w[2] >> (16 + 2 * a)) & 3u); }
  __device__ __forceinline__ int q_w(int slot) const { return (int)((w[3] >> (4 * slot)) & 15u); }
  // compact row of an in-port slot: full-row action of column c in bits 4c..4c+3 (c < q_w),
  // first full-row action valued default_q in bits 16..19 (15: none)
  __device__ __forceinline__ uint32_t row_desc(int slot) const { return w[4 + slot]; }
};
// packed port record (SflMap::port_pack)
struct PortRec {
  u4 w;
  __device__ __forceinline__ int nb() const { return (int)(int16_t)(w[0] & 0xFFFFu); }
  __device__ __forceinline__ int len() const { return (int)(int16_t)(w[0] >> 16); }
  __device__ __forceinline__ int unique() const { return (int)(int16_t)(w[1] & 0xFFFFu); }
  __device__ __forceinline__ int q_w() const { return (int)(w[1] >> 16); }
  __device__ __forceinline__ uint32_t row_base() const { return w[2]; }
  __device__ __forceinline__ uint32_t q_off() const { return w[3]; }
};
// G lanes per env (a lane group; G = 64: one env per wavefront, G = 32 / 16: two / four envs per
// wavefront, for maps with few trains).  PPL semaphore words (ports <= G*PPL) and SPL counter words
// (switches <= G*SPL) per lane.  With G = 64 the env's control values are wave-uniform and live in
// SGPRs (uni, readlane, ballot, scalar loads of the map tables); with G < 64 they are group-uniform
// VGPRs: a cross-lane read is a ds_bpermute inside the group, a ballot is the group's slice of the
// wave's, and the map tables are read with vector loads (the groups of a wave sit on different
// switches).  Branches on group-uniform values diverge across the groups of a wave, which the
// flat loop of run_groups (one tick / post / decision per group and iteration) keeps balanced.
// PART: the graph-partitioned mode's local step (sfl_part.h, G = 64 only): the env's Q rows live on
// their switches' owner ranks, so a decision is observed in one launch (request to the owner) and
// applied in the next (with the owner's reply), and the post step's Q operations are update
// records to the owners
// LM (run_groups only, sfl_engine.h variant 11): the map's move table and distance map (int16) live in the block's LDS
template <int PPL, int SPL, int TWc, bool PART = false, int G = 64, bool LM = false>
struct WEnv {
  static_assert(G == 64 || G == 32 || G == 16 || G == 8, "lane group of 8, 16, 32 or 64 lanes");
  static_assert(G == 64 || !PART, "the partitioned local step runs one env per wavefront");
  const SflMap& m;
  const SflState& s;
  const uint32_t e, E;
  const int lane;   // lane in the env's group (0 .. G-1)
  const int gbase;  // first wavefront lane of the group
  const SflPart* P;  // PART only
  static constexpr int TPL = (TWc + G - 1) / G;  // train slots per lane: trains lane, lane + G, ...
  // prefetch records: one per queued train; PART stages only the train that decides in the launch.
  // RING (shapes with two train slots per lane): PF_SLOTS records hold the first queued trains of a
  // batch in queue order (record i = the i-th decision after the prefetch) and the batch is staged
  // again when they are used up.  c5 (k_wave2, one env per 64-thread block): 16 records instead of
  // 128 take an env's LDS from 13.9 to 9.8 KB, so 16 envs fit a CU instead of 11, at 4 waves per
  // SIMD in 128 VGPRs (1 spilled): 598 M -> 729 M agent-env-steps/s (ring of 32: 673 M).  c3 (G = 16):
  // off by default, see SFL_PF_RING
  static constexpr int RING_N = G < 64 ? SFL_PF_RING : SFL_PF_RING64;
  static constexpr bool RING = !PART && TPL > 1 && RING_N > 0 && RING_N < TWc;
  static constexpr int PF_SLOTS = PART ? 1 : (RING ? RING_N : TWc);
  // (SFL_EPS_PF) the record's doubles: + the staged epsilon
  static constexpr bool EPS_PF = SFL_EPS_PF && !PART && G < 64 && G * SPL <= 64;
  static constexpr int PFD = EPS_PF ? PF_D + 1 : PF_D;
  static constexpr int PFW = 2 * PFD + PF_WI;
  __device__ __forceinline__ static int pfx(int h) { return PART ? 0 : h; }
  // RING: record i is staged by lane i % G (register slot i / G) in one pass per G records -- the lanes
  // stage the batch's queued trains in queue order, so a batch of up to G decisions is one set of
  // dependent loads instead of one per train slot; otherwise train h's lane stages it (slot h / G)
  static constexpr bool PF_BY_RANK = RING;
  static constexpr int PFS = PF_BY_RANK ? (PF_SLOTS + G - 1) / G : TPL;
  int pf_n = 0;  // RING: decisions since the batch was staged (= the record of the next one)
  static constexpr int kG = G;
  static_assert(TPL * G <= 128, "at most 128 train slots per env");
  using Mask = typename MaskOf<(TWc <= 32 ? 32 : TPL * G)>::type;
  bool mine[TPL];  // lane + G k < T: slot k holds train lane + G k
  // the lane's trains (slot k = train lane + G k)
  int32_t pos[TPL];
  uint32_t bits[TPL], plan[TPL];
  uint32_t nprv[TPL];  // next port | prev port << 16
  uint32_t sdec[TPL];  // source port | decision switch << 16
  int32_t delay[TPL];
  // timetable constants of train `lane` (tr_pack)
  // timetable constants of the lane's train (tr_pack row) live in LDS and are read where used
  const int32_t* ltt;  // [TW][8]
  // G < 64: the block's LDS copies of the per-switch and per-port map records (sw_pack [S][16],
  // port_pack and port_tr [4S][4]); G = 64 reads them with scalar loads
  const uint32_t* tsw = nullptr;
  static constexpr int SW_LDS = 12;  // words of a switch record in the block's LDS copy (10 used of sw_pack's 16)
  const uint32_t* tpp = nullptr;
  const uint32_t* tpt = nullptr;
  // LM: the block's LDS copies of move_tab ([HW][4] rows of 4 words) and of the distance map as int16 pairs (d16)
  const uint32_t* lmv = nullptr;
  const uint32_t* ldist = nullptr;
  // this env's semaphore records and switch counters in LDS (one region per wave):
  // uniform reads are broadcast ds_reads, writes one lane's ds_write, and the lane-parallel
  // scans read entries k*64 + lane (conflict-free)
  uint32_t* lsem;  // [64*PPL]
  uint32_t* lcnt;  // [64*SPL]
  // batch prefetch (see prefetch()): per queued train (lane), the staged Q row, the pending
  // update's Q cell value and the slot word in LDS, and the staged offsets in VGPRs
  double* lpf;       // [TW][PFD]: pending cell value | slot word (as bits) | row max (| staged epsilon)
  uint32_t* lpi;     // [TW][PF_WI]: int16 distances, argmaxes
  uint32_t pf_roff[PFS];  // offset of the staged row in the env's Q block (PF_NONE: none)
  uint32_t pf_qoff[PFS];  // offset of the staged pending cell (PF_NONE: none)
  bool pf_ok;        // uniform: this batch has been prefetched
  uint32_t lerr;  // error bits seen by this lane (OR-reduced on store)
  // this env's blocks: Q-table, key-set bitmap, (switch, train) slots (env-major [T][S] here,
  // so one env's slots are contiguous and a flush over switches is one coalesced access)
  double* qb;
  uint32_t* touchb;
  uint64_t* slotb;
  // wave-uniform env scalars
  int32_t now;
  uint32_t flags, epoch;
  Mask q_mask, arr_mask, fl_mask, mf_mask;
  // the epsilon-greedy stream (numpy PCG64 state, increment, buffered half) lives in LDS: it is
  // touched once per decision and would otherwise hold ten registers across the whole loop
  uint64_t* lrng;  // [6]: state hi, lo, inc hi, lo, has << 32 | buf, (EPS_PF) switches decided since the staging
  int64_t cum;     // cumulative reward: a sum of integer rewards, exact in f64 (converted on store)
  int32_t n_mf, ep_dec, ep_ticks;
  int32_t step_ctr;
  uint32_t n_dec;  // decisions in this launch (dec_total += n_dec on store)
  // PART: this launch's messages, staged in the env's own slots (k_part_compact packs them)
  int32_t req_dst_v = -1;  // destination of the request (-1: none)
  uint32_t n_upd = 0;      // update records staged
  uint32_t stg = 0;        // next update stage of this launch (the posts' records in program order)
  // PART: the launch's loaded semaphore records, [64 * PPL] words of the env's LDS region
  // (store() writes back only what changed).  Held in registers they were spilled, and every conditional
  // store of the write-back then waited for its predecessors (a scratch reload's vmcnt counts stores too)
  uint32_t* lsem0 = nullptr;
  // PART: switches whose counter changed in this launch, a bitmap of (G * SPL) / 32 words after lsem0 (cset sets
  // the bit; store() writes back only those counters)
  uint32_t* ldirty = nullptr;
  // PART: the launch's loaded train records, [TPL][6][64] words (pos, bits, plan, next | prev, src | dec, delay)
  // after ldirty: store() writes back only the fields that changed (a round moves few trains; round 3 wrote all
  // eight arrays of every train, ~50 of the 60 write requests per env and round)
  uint32_t* ltr0 = nullptr;
  // PART: this lane's word of the env's scalar block (SflPart::eblk; lane i holds word i), loaded by load()
  uint32_t eb_w = 0;
  // PART: the reply to the env's last request (action, max lo / hi words), loaded by load() right behind the
  // state (its place, req_ix, with the state batch): the apply pass reads registers instead of two dependent loads
  uint32_t rep_a = 0, rep_lo = 0, rep_hi = 0;
  __device__ __forceinline__ uint32_t ebw(int i) const { return rl(eb_w, i); }  // (G = 64: wave-uniform)
  __device__ __forceinline__ uint64_t ebw64(int i) const { return (uint64_t)ebw(i) | ((uint64_t)ebw(i + 1) << 32); }
  // product phase timers (the TIMED kernels that learn() / test() run; sfl_get_phase_cycles): decide<true>
  // stamps the end of its observe and epsilon-greedy sections on a sampled wavefront (tm_on); run_groups
  // reads the stamps from a deciding lane after the (divergent) decide block
  bool tm_on = false;
  uint64_t tm_obs_t = 0, tm_eg_t = 0;
#ifdef SFL_PROFILE
  uint64_t prof[9] = {};  // decide: observe, epsilon-greedy, apply; events: prefetch, row hit/miss, pend hit/miss, decisions
  uint64_t lap[16] = {};  // finer segments (see SFL_LAP call sites)
  uint64_t lap_t = 0;
#endif

  // lds: this env's region; ltt_shared: the block's copy of the timetable rows (G < 64), or null for
  // the env's own copy after its region
  __device__ WEnv(const SflMap& m_, const SflState& s_, uint32_t e_, int wlane, uint32_t* lds, const SflPart* P_ = nullptr,
                  int32_t* ltt_shared = nullptr)
      : m(m_), s(s_), e(e_), E(s_.E), lane(wlane & (G - 1)), gbase(wlane & ~(G - 1)), P(P_), lsem(lds), lcnt(lds + G * PPL),
        lpf((double*)(lds + G * (PPL + SPL))) {
#pragma unroll
    for (int k = 0; k < TPL; ++k) mine[k] = lane + G * k < m_.T;
#pragma unroll
    for (int k = 0; k < PFS; ++k) pf_roff[k] = pf_qoff[k] = PF_NONE;
    lpi = (uint32_t*)(lpf + PF_SLOTS * PFD);
    lrng = (uint64_t*)(lds + G * (PPL + SPL) + PF_SLOTS * PFW);
    // PART: the timetable rows are read from the map (L2-resident): a launch runs one or two
    // decisions, so a per-launch LDS copy would cost more than it saves
    if constexpr (PART) ltt = m.tr_pack;
    else ltt = ltt_shared ? ltt_shared : (const int32_t*)(lds + G * (PPL + SPL) + PF_SLOTS * PFW + 12);
    pf_ok = false;
    if constexpr (PART) {  // the rows this rank owns, of this env (the env-local table is freed)
      const size_t ge = (size_t)P_->env_base + e_;
      qb = P_->q_own + ge * P_->q_own_per_env;
      touchb = P_->touched_own + ge * P_->own_words;
    } else {
      qb = s.q + (size_t)e * m.q_per_env;
      touchb = s.touched + (size_t)e * m.touched_words;
    }
    slotb = s.slot + (size_t)e * (uint32_t)(m.S * m.T);
  }
  __device__ __forceinline__ uint32_t slot_ix(int sw, int h) const { return (uint32_t)(h * m.S + sw); }

  __device__ __forceinline__ size_t ix(size_t i) const { return i * (size_t)E + e; }
  // per-train / per-port / per-switch state between launches: env-major ([E][T], [E][NP], [E][S];
  // sfl_get_env_state), so a wave's load and store of its env are contiguous (the lane-per-env
  // body keeps the env index fastest instead)
  __device__ __forceinline__ size_t tix(int h) const { return (size_t)e * (uint32_t)m.T + (uint32_t)h; }
  __device__ __forceinline__ size_t pix(int p) const { return (size_t)e * (uint32_t)m.NP + (uint32_t)p; }
  // the semaphore state between launches: 32-bit records, env-major (the array is sized for the
  // lane-per-env body's 64-bit ones)
  __device__ __forceinline__ uint32_t* sem_words() const { return (uint32_t*)s.sem; }
  // PART: switch sw's agent is owned by this rank, so its rows are read and written here directly
  // (P->local_sw; otherwise its rows go through the owner's messages)
  __device__ __forceinline__ bool local_sw(int sw) const {
    if constexpr (!PART) return true;
    else return LDC(P->local_sw, (size_t)sw) != 0u;
  }
  __device__ __forceinline__ bool local_sw_var(int sw) const {  // per-lane sw
    if constexpr (!PART) return true;
    else return ld(P->local_sw, (size_t)sw) != 0u;
  }
  // the Q block offset / first key-set row of in-port g (group-uniform g): the map's layout, or
  // (PART) this rank's owned table
  __device__ __forceinline__ uint32_t qoff_of(int g, const PortRec& pr) const {
    if constexpr (PART) return (uint32_t)LDC(P->q_off_own, (size_t)g);
    else return pr.q_off();
  }
  __device__ __forceinline__ uint32_t rowb_of(int g, const PortRec& pr) const {
    if constexpr (PART) return LDC(P->row_own, (size_t)g);
    else return pr.row_base();
  }
  __device__ __forceinline__ size_t cix(int sw) const { return (size_t)e * (uint32_t)m.S + (uint32_t)sw; }

  // ---- group primitives -------------------------------------------------------------
  // the lane index in the group, re-read (v_mbcnt) where it is used: values derived from it are then
  // recomputed inside the loop (one or two VALU) instead of hoisted out of it and spilled -- a
  // scratch reload is a vector-memory round trip (~600 cycles measured, VmemLatency)
  __device__ __forceinline__ int lid() const {
    int x = (int)__lane_id();
    asm volatile("" : "+v"(x));
    return G == 64 ? x : (x & (G - 1));
  }
  __device__ __forceinline__ bool mine_(int k) const { return lid() + G * k < m.T; }
  // a group-uniform value: in an SGPR for G = 64 (readfirstlane), as is for G < 64
  template <class T>
  __device__ __forceinline__ T U(T x) const {
    if constexpr (G == 64) return uni(x);
    else return x;
  }
  __device__ __forceinline__ double Ud(double x) const {
    if constexpr (G == 64) return unid(x);
    else return x;
  }
  // lane i of the group (i group-uniform)
  __device__ __forceinline__ uint32_t RL(uint32_t v, int i) const {
    if constexpr (G == 64) return rl(v, i);
    else return (uint32_t)__builtin_amdgcn_ds_bpermute((gbase + i) << 2, (int)v);
  }
  __device__ __forceinline__ int32_t RL(int32_t v, int i) const { return (int32_t)RL((uint32_t)v, i); }
  // the group's lanes with p set (bit i = lane i of the group)
  __device__ __forceinline__ uint64_t BAL(bool p) const {
    if constexpr (G == 64) return __ballot(p);
    else return (__ballot(p) >> gbase) & ((1ull << G) - 1ull);
  }
  // one ballot per train slot: bit h = train h
  __device__ __forceinline__ Mask mbal(const bool (&p)[TPL]) const {
    if constexpr (TPL * G <= 64 || TWc <= 32) {
      uint64_t r = 0;
#pragma unroll
      for (int k = 0; k < TPL; ++k) r |= BAL(p[k]) << (G * k);
      return (Mask)r;  // (32-bit masks: trains < 32 only)
    } else {
      return M2{{BAL(p[0]), BAL(p[1])}};
    }
  }
  // read-only map tables at a group-uniform index: scalar loads (K$) for G = 64, vector loads else
  template <class T>
  __device__ __forceinline__ T LDC(const T* p, size_t i) const {
    if constexpr (G == 64) return ldc(p, i);
    else return ld(p, i);
  }
  template <class V>
  __device__ __forceinline__ V LDCV(const void* p, size_t i) const {
    if constexpr (G == 64) return ldcv<V>(p, i);
    else return ld((const V*)p, i);
  }

  // ---- cross-lane access (index group-uniform) --------------------------------------
  __device__ __forceinline__ uint32_t sget(int p) const { return U(lsem[p]); }
  __device__ __forceinline__ void sset(int p, uint32_t r) {
    lsem[p] = r;  // wave-uniform value from every lane (one address): no lane-0 exec region
  }
  __device__ __forceinline__ uint32_t& sem(int k) const { return lsem[k * G + lid()]; }  // lane-parallel
  __device__ __forceinline__ uint32_t cget(int sw) const { return U(lcnt[sw]); }
  __device__ __forceinline__ void cset(int sw, uint32_t v) {
    lcnt[sw] = v;  // wave-uniform value from every lane
    if constexpr (PART) {
      if (lid() == 0) atomicOr(&ldirty[sw >> 5], 1u << (sw & 31));
    }
  }
  __device__ __forceinline__ uint32_t cget_var(int sw) const { return lcnt[sw]; }  // per-lane index
  // train h's value of a per-train register (h wave-uniform)
  template <class T>
  __device__ __forceinline__ T trl(const T (&x)[TPL], int h) const {
    if constexpr (TPL == 1) {
      return RL(x[0], h);
    } else {
      T v = x[0];
#pragma unroll
      for (int k = 1; k < TPL; ++k) v = (h / G == k) ? x[k] : v;
      return RL(v, h & (G - 1));
    }
  }
  // train h's value with h varying per lane (a ds_bpermute from lane h % G of the group per slot)
  template <class T>
  __device__ __forceinline__ T trl_v(const T (&x)[TPL], int h) const {
    const int a = (gbase + (h & (G - 1))) << 2;
    T v = (T)__builtin_amdgcn_ds_bpermute(a, (int)x[0]);
#pragma unroll
    for (int k = 1; k < TPL; ++k) {
      const T w = (T)__builtin_amdgcn_ds_bpermute(a, (int)x[k]);
      v = (h / G == k) ? w : v;
    }
    return v;
  }
  // record i of a prefetch register (lane i % G, slot i / G; i group-uniform)
  template <class T, int N>
  __device__ __forceinline__ T rec_of(const T (&x)[N], int i) const {
    if constexpr (N == 1) {
      return RL(x[0], i);
    } else {
      T v = x[0];
#pragma unroll
      for (int k = 1; k < N; ++k) v = (i / G == k) ? x[k] : v;
      return RL(v, i & (G - 1));
    }
  }
  template <class T>
  __device__ __forceinline__ void tset(T (&x)[TPL], int h, T v) {
#pragma unroll
    for (int k = 0; k < TPL; ++k) x[k] = (lid() + G * k == h) ? v : x[k];
  }
  __device__ __forceinline__ uint32_t state_of(int h) const { return tb_state(trl(bits, h)); }
  // malfunctioning trains (check_port_blocked's owner test)
  __device__ __forceinline__ Mask malf_mask() const {
    bool p[TPL];
#pragma unroll
    for (int k = 0; k < TPL; ++k) p[k] = mine_(k) && tb_state(bits[k]) == S_MALF;
    return mbal(p);
  }

  // ---- map records --------------------------------------------------------------------
  __device__ __forceinline__ SwRec sw_rec(int sw) const {
    if constexpr (G == 64) return SwRec{LDCV<u8>(m.sw_pack, (size_t)sw * 2u)};
    else return SwRec{*(const u8*)(tsw + SW_LDS * sw)};
  }
  // neighbour ports of the switch's ports 0-3 (16 bits each)
  __device__ __forceinline__ vec_t<uint32_t, 2> sw_nb(int sw) const {
    if constexpr (G == 64) return LDCV<vec_t<uint32_t, 2>>(m.sw_pack, (size_t)sw * 8u + 4u);
    else return *(const vec_t<uint32_t, 2>*)(tsw + SW_LDS * sw + 8);
  }
  __device__ __forceinline__ PortRec port_rec(int p) const {
    if constexpr (G == 64) return PortRec{LDCV<u4>(m.port_pack, (size_t)p)};
    else return PortRec{*(const u4*)(tpp + 4 * p)};
  }
  __device__ __forceinline__ int port_nb(int p) const { return (int)(int16_t)(port_rec(p).w[0] & 0xFFFFu); }
  __device__ __forceinline__ u4 port_tr_rec(int o) const {
    if constexpr (G == 64) return LDCV<u4>(m.port_tr, (size_t)o);
    else return *(const u4*)(tpt + 4 * o);
  }
  // lane-parallel (per-lane index) reads of the same records: vector loads for G = 64, LDS else
  __device__ __forceinline__ u4 sw_v4(int sw, int q) const {
    if constexpr (G == 64) return ld((const u4*)m.sw_pack, (size_t)sw * 4u + (uint32_t)q);
    else return *(const u4*)(tsw + SW_LDS * sw + 4 * q);
  }
  __device__ __forceinline__ vec_t<uint32_t, 2> sw_nb_v(int sw) const {
    if constexpr (G == 64) return ld((const vec_t<uint32_t, 2>*)m.sw_pack, (size_t)sw * 8u + 4u);
    else return *(const vec_t<uint32_t, 2>*)(tsw + SW_LDS * sw + 8);
  }
  __device__ __forceinline__ u4 port_v(int p) const {
    if constexpr (G == 64) return ld((const u4*)m.port_pack, (size_t)p);
    else return *(const u4*)(tpp + 4 * p);
  }
  // timetable row of train h (group-uniform h): scalar loads for G = 64, the LDS rows else
  __device__ __forceinline__ vec_t<int32_t, 8> tr_row(int h) const {
    if constexpr (G == 64) return LDCV<vec_t<int32_t, 8>>(m.tr_pack, (size_t)h);
    else return *(const vec_t<int32_t, 8>*)(ltt + 8 * h);
  }
  __device__ __forceinline__ int32_t tr_init_dist(int h) const {
    if constexpr (G == 64) return LDC(m.tr_pack, (size_t)h * 8 + 5);
    else return ltt[8 * h + 5];
  }
  struct Move {
    int cell, dir;
    bool valid, cell_ok;
    int sw;  // switch at the destination cell; -1: none; 0xFF: not packed (look it up)
  };
  __device__ __forceinline__ static Move unpack_move(uint32_t w) {
    Move mv;
    mv.cell = (int)(w & 0xFFFFFu) - 1;
    mv.dir = (int)((w >> 20) & 3u);
    mv.valid = (w >> 22) & 1u;
    mv.cell_ok = (w >> 23) & 1u;
    mv.sw = (int)(w >> 24);
    return mv;
  }
  // cell_sw of a move's destination cell (packed in the move table when the map has <= 254 switches)
  __device__ __forceinline__ int dest_sw(const Move& mv) const {
    if (m.S <= 254) return mv.sw == 0xFF ? -1 : mv.sw;
    return mv.cell >= 0 ? (int)ld(m.cell_sw, (size_t)mv.cell) : -1;
  }
  // flatland-lite check_action_on_agent as a table lookup; U: wave-uniform arguments (scalar load)
  template <bool UNI>
  __device__ __forceinline__ Move check_action(uint32_t a, int cell, int dir) const {
    const uint32_t i = ((uint32_t)cell * 4u + (uint32_t)dir) * 4u + (a & 3u);
    if constexpr (LM) return unpack_move(lmv[i]);
    else return unpack_move(UNI ? LDC(m.move_tab, i) : ld(m.move_tab, i));
  }
  // the move-table row (all four rail actions) of (cell, dir) = cd, per lane
  __device__ __forceinline__ u4 move_row(uint32_t cd) const {
    if constexpr (LM) return *(const u4*)(lmv + 4u * cd);
    else return ld((const u4*)m.move_tab, (size_t)cd);
  }
  // distance-map entry i (int32 semantics: DIST_INF for unreachable)
  __device__ __forceinline__ int32_t dist_at(uint32_t i, bool uni) const {
    if constexpr (LM) return d16_lo(ldist[i >> 1] >> (16u * (i & 1u)));
    else return uni ? LDC(m.dist, i) : ld(m.dist, i);
  }
  template <bool UNI>
  __device__ __forceinline__ bool action_ok(uint32_t a, int cell, int dir) const {
    Move mv = check_action<UNI>(a, cell, dir);
    return mv.cell_ok && mv.valid;
  }
  // distance map lookup (wave-uniform)
  __device__ __forceinline__ int32_t dist(int k, int cell, int dir) {
    if (cell < 0) {
      lerr |= E_INF_DIST;
      return 0;
    }
    const int32_t d = dist_at(((uint32_t)k * (uint32_t)m.HW + (uint32_t)cell) * 4u + (uint32_t)dir, true);
    if (d >= DIST_INF) lerr |= E_INF_DIST;
    return d;
  }

  // per-lane projection step of reward_func.py:41-56 (STOP entries are skipped, and a cell off
  // the grid ends the walk) and distance lookup with the off-grid marker
  __device__ __forceinline__ void project(uint32_t a, int& pc, int& pd) const {
    // lane-parallel (prefetch): a clamped lookup and selects instead of a divergent branch
    const bool go = (a != A_STOP) & (pc >= 0);
    const Move mv = check_action<false>(a, pc >= 0 ? pc : 0, pd);
    pc = go ? mv.cell : pc;
    pd = go ? mv.dir : pd;
  }
  __device__ __forceinline__ int32_t dist_v(int k, int cell, int dir) const {
    const int32_t d = dist_at(((uint32_t)k * (uint32_t)m.HW + (uint32_t)(cell >= 0 ? cell : 0)) * 4u + (uint32_t)dir, false);
    return cell < 0 ? PF_OFFGRID : d;
  }
  // distance staged by prefetch (dist() semantics: off the grid or unreachable sets E_INF_DIST)
  __device__ __forceinline__ int32_t dist_staged(int32_t d) {
    if (d == PF_OFFGRID) {
      lerr |= E_INF_DIST;
      return 0;
    }
    if (d >= DIST_INF) lerr |= E_INF_DIST;
    return d;
  }

  // ---- semaphores (wave-uniform) ----------------------------------------------------------
  // observer.py:44-151 (a record's dir field always equals map_direction(port))
  // does record r block a train h entering through its port (io = 0: the next port) or leaving
  // through it (io = 1: the out port)?  0/1 in integer VALU: present, owned by another train,
  // inside its [t0, t1] window, and of the opposite direction or owned by a malfunctioning train
  __device__ __forceinline__ uint32_t rec_blocks(uint32_t r, uint32_t h, Mask malf, uint32_t io) const {
    const uint32_t ow = r_owner(r);
    const uint32_t win = (uint32_t)(now - r_t0(r)) <= r_dur(r) ? 1u : 0u;  // t0 <= now <= t1
    const uint32_t other = ((ow ^ h) + 0x7Fu) >> 7;  // owner != h (both < 128)
    const uint32_t mf = mbit(malf, (int)ow) ? 1u : 0u;
    return (r >> 31) & win & other & ((r_in(r) ^ io ^ 1u) | mf);
  }
  // put_keep / put_replace as value transforms of a record (vector ALU, wave-uniform values)
  struct PutF {
    uint32_t h, in;
    int32_t now, span, ovr;  // ovr: in-flag that is overridden (-1: none)
    bool keep;               // put_keep: an overridden record keeps its in-flag
    __device__ __forceinline__ uint32_t operator()(uint32_t r) const {
      // selects on bitwise conditions: the record copies live in VGPRs, so a short-circuit
      // condition would become an exec-mask region
      const uint32_t nr = r_pack(h, keep ? r_in(r) : in, now, now + span);
      const uint32_t fresh = r_pack(h, in, now, now + span);
      const bool retime = ((ovr >= 0) & (r_in(r) == (uint32_t)ovr)) | (r_t0(r) > now);
      return !r_present(r) ? fresh : (retime ? nr : r);
    }
  };
  __device__ __forceinline__ PutF put_keep_f(int h, uint32_t in, int32_t span, uint32_t ovr_in) const {
    return PutF{(uint32_t)h, in, now, span, (int32_t)ovr_in, true};
  }
  __device__ __forceinline__ PutF put_replace_f(int h, uint32_t in, int32_t span, int ovr_in) const {
    return PutF{(uint32_t)h, in, now, span, ovr_in, false};
  }
  // register copies of the records of up to four ports (index -1 = unused)
  struct SemQuad {
    uint32_t* l;
    int p[4];
    uint32_t v[4];
    __device__ __forceinline__ SemQuad(uint32_t* l_, int a, int b, int c, int d) : l(l_) {
      p[0] = a;
      p[1] = b;
      p[2] = c;
      p[3] = d;
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = l[p[i] >= 0 ? p[i] : 0];
    }
    template <class F>
    __device__ __forceinline__ void put(int port, const F& f) {
      uint32_t cur = v[0];
#pragma unroll
      for (int i = 3; i > 0; --i) cur = (p[i] == port) ? v[i] : cur;
      const uint32_t nv = f(cur);
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = (p[i] == port) ? nv : v[i];
    }
    __device__ __forceinline__ void store() const {  // uniform values, written by every lane
      {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (p[i] >= 0) l[p[i]] = v[i];
      }
    }
  };
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
  // the env's global blocks; G < 64 recomputes them from e at each use (a held 64-bit pointer is
  // two VGPRs per block for the whole loop)
  __device__ __forceinline__ double* qbase() const {
    if constexpr (PART || G == 64) return qb;
    else return s.q + (size_t)e * m.q_per_env;
  }
  __device__ __forceinline__ uint32_t* tbase() const {
    if constexpr (PART || G == 64) return touchb;
    else return s.touched + (size_t)e * m.touched_words;
  }
  __device__ __forceinline__ uint64_t* sbase() const {
    if constexpr (G == 64) return slotb;
    else return s.slot + (size_t)e * (uint32_t)(m.S * m.T);
  }
  // global-address-space atomic: a flat atomic would also count on lgkmcnt, so the decision's next
  // LDS read or scalar load would wait for its L2 round trip
  __device__ __forceinline__ void touch_row(uint32_t row) const {
    __hip_atomic_fetch_or((SFL_AS_G uint32_t*)tbase() + (row >> 5), 1u << (row & 31u), __ATOMIC_RELAXED,
                          __HIP_MEMORY_SCOPE_AGENT);
  }
  // (a decaying lr past the table is an error, E_LR_TABLE: see SflEnv::lr_of in sfl_core.h)
  __device__ __forceinline__ double lr_of(uint32_t n) {
    if (m.lr_decay == 1.0) return m.lr0;  // lr0 * 1.0**n (distr_q.py:70-79)
    if (n < (uint32_t)m.ntab) return LDC(m.lr_tab, (size_t)n);
    lerr |= E_LR_TABLE;
    return m.lr0;
  }
  __device__ __forceinline__ double lr_of_var(uint32_t n) {
    if (m.lr_decay == 1.0) return m.lr0;
    if (n < (uint32_t)m.ntab) return ld(m.lr_tab, (size_t)n);
    lerr |= E_LR_TABLE;
    return m.lr0;
  }

  // ---- launch-boundary state transfer ---------------------------------------------------------
  __device__ __forceinline__ void load() {
    // every per-lane load is issued unconditionally (clamped index) before any result is used: as conditional
    // loads each sat in its own exec-masked block and waited for its own HBM round trip (16 + 4 + 2 x 8 in a
    // row for c5's partitioned local step, which loads the state every round)
    uint32_t tw[TPL][8];
    uint32_t ixr = 0;
    if constexpr (PART) {  // (first: the env's scalars and its reply's place travel with the state batch)
      eb_w = ld(P->eblk, (size_t)e * PART_EB + (uint32_t)lane);
      ixr = ld(P->req_ix, (size_t)e);
    }
#pragma unroll
    for (int k = 0; k < TPL; ++k) {
      const size_t ti = tix(mine[k] ? lane + G * k : 0);
      tw[k][0] = (uint32_t)ld(s.tr_pos, ti);
      tw[k][1] = ld(s.tr_bits, ti);
      tw[k][2] = ld(s.tr_plan, ti);
      tw[k][3] = ld(s.tr_next, ti);
      tw[k][4] = ld(s.tr_prev, ti);
      tw[k][5] = ld(s.tr_src, ti);
      tw[k][6] = ld(s.tr_dec, ti);
      tw[k][7] = (uint32_t)ld(s.tr_delay, ti);
    }
    uint32_t rw[PPL], nw[SPL];
#pragma unroll
    for (int k = 0; k < PPL; ++k) rw[k] = ld(sem_words(), pix(k * G + lane < m.NP ? k * G + lane : 0));
#pragma unroll
    for (int k = 0; k < SPL; ++k) nw[k] = ld(s.counts, cix(k * G + lane < m.S ? k * G + lane : 0));
#pragma unroll
    for (int k = 0; k < TPL; ++k) {
      const int hk = lane + G * k;
      if (mine[k]) {
        pos[k] = (int32_t)tw[k][0];
        bits[k] = tw[k][1];
        plan[k] = tw[k][2];
        nprv[k] = tw[k][3] | (tw[k][4] << 16);
        sdec[k] = tw[k][5] | (tw[k][6] << 16);
        delay[k] = (int32_t)tw[k][7];
        if constexpr (PART) {
          uint32_t* t0 = ltr0 + (k * 6) * 64 + lane;
          t0[0] = (uint32_t)pos[k];
          t0[64] = bits[k];
          t0[128] = plan[k];
          t0[192] = nprv[k];
          t0[256] = sdec[k];
          t0[320] = (uint32_t)delay[k];
        }
        if constexpr (!PART) {
          *(vec_t<int32_t, 4>*)(ltt + 8 * hk) = ld((const vec_t<int32_t, 4>*)m.tr_pack, (size_t)hk * 2u);
          *(vec_t<int32_t, 4>*)(ltt + 8 * hk + 4) = ld((const vec_t<int32_t, 4>*)m.tr_pack, (size_t)hk * 2u + 1u);
        }
      } else {
        pos[k] = -1;
        bits[k] = 0;
        plan[k] = 0;
        nprv[k] = 0xFFFFFFFFu;
        sdec[k] = 0xFFFFFFFFu;
        delay[k] = 0;
      }
    }
#pragma unroll
    for (int k = 0; k < PPL; ++k) {
      const uint32_t r = k * G + lane < m.NP ? rw[k] : 0u;
      sem(k) = r;
      if constexpr (PART) lsem0[k * G + lane] = r;
    }
#pragma unroll
    for (int k = 0; k < SPL; ++k) {
      const uint32_t n = k * G + lane < m.S ? nw[k] : 0u;
      lcnt[k * G + lane] = n;
    }
    if constexpr (PART) {
      if (lane < 2 * SPL) ldirty[lane] = 0u;
      // the env's scalars: one 64-lane load of its block (see sfl_part.h EB_*), issued above
      {  // the reply, if a request is open (a stale index of an env without one stays inside the buffer)
        const uint32_t ix = U(ixr);
        const vec_t<int32_t, 4> rw =
            ld((const vec_t<int32_t, 4>*)(P->rep_in + (ix < P->world * (P->cap_msg + 1u) ? ix : 0u)), 0);
        rep_a = (uint32_t)rw[0];
        rep_lo = (uint32_t)rw[2];
        rep_hi = (uint32_t)rw[3];
      }
      now = (int32_t)ebw(EB_ELAPSED);
      flags = ebw(EB_EFLAGS);
      epoch = ebw(EB_EPOCH);
      lerr = ebw(EB_ERR);
      auto mask = [&](int k) -> Mask {
        if constexpr (TPL * G <= 64 || TWc <= 32) return (Mask)ebw64(EB_MASKS + k * MAXW);
        else return M2{{ebw64(EB_MASKS + k * MAXW), ebw64(EB_MASKS + k * MAXW + 2)}};
      };
      q_mask = mask(0);
      arr_mask = mask(1);
      fl_mask = mask(2);
      mf_mask = mask(3);
      {  // lanes 0-4: rng word `lane` (two dwords of the block, read across lanes)
        const int l = lane < 5 ? lane : 0;
        const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_bpermute((EB_RNG + 2 * l) << 2, (int)eb_w);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_bpermute((EB_RNG + 2 * l + 1) << 2, (int)eb_w);
        if (lane < 5) lrng[lane] = (uint64_t)lo | ((uint64_t)hi << 32);
      }
      cum = (int64_t)__longlong_as_double((long long)ebw64(EB_CUM));
      n_mf = (int32_t)ebw(EB_N_MF);
      ep_dec = (int32_t)ebw(EB_EP_DEC);
      ep_ticks = (int32_t)ebw(EB_EP_TICKS);
      step_ctr = (int32_t)ebw(EB_STEP_CTR);
      n_dec = 0;
      return;
    }
    now = U(ld(s.elapsed, e));
    flags = U(ld(s.eflags, e));
    epoch = U(ld(s.epoch, e));
    lerr = U(ld(s.err, e));
    auto word = [&](int k, int w) {
      return U((uint64_t)ld(s.masks, (size_t)(k * MAXW + 2 * w) * E + e) |
                 ((uint64_t)ld(s.masks, (size_t)(k * MAXW + 2 * w + 1) * E + e) << 32));
    };
    auto mask = [&](int k) -> Mask {
      if constexpr (TPL * G <= 64 || TWc <= 32) return (Mask)word(k, 0);
      else return M2{{word(k, 0), word(k, 1)}};
    };
    q_mask = mask(0);
    arr_mask = mask(1);
    fl_mask = mask(2);
    mf_mask = mask(3);
    if (lane < 5) lrng[lane] = ld(s.rng, ix((size_t)lane));
    cum = (int64_t)Ud(ld(s.cum_reward, e));
    n_mf = U(ld(s.n_mf, e));
    ep_dec = U(ld(s.ep_dec, e));
    ep_ticks = U(ld(s.ep_ticks, e));
    step_ctr = (int32_t)U(ld(s.step_ctr, e));
    n_dec = 0;
  }
  // returns the env's error bits (OR over lanes); PART writes its scalars with store_eblk
  __device__ __forceinline__ uint32_t store(int32_t phase) {
    if constexpr (PART) {  // only the changed fields (the LDS reads first, then the stores)
      uint32_t o[TPL][6];
#pragma unroll
      for (int k = 0; k < TPL; ++k)
#pragma unroll
        for (int i = 0; i < 6; ++i) o[k][i] = ltr0[(k * 6 + i) * 64 + lane];
#pragma unroll
      for (int k = 0; k < TPL; ++k) {
        const int hk = lane + G * k;
        if (!mine[k]) continue;
        if ((uint32_t)pos[k] != o[k][0]) st(s.tr_pos, tix(hk), pos[k]);
        if (bits[k] != o[k][1]) st(s.tr_bits, tix(hk), bits[k]);
        if (plan[k] != o[k][2]) st(s.tr_plan, tix(hk), plan[k]);
        if ((nprv[k] ^ o[k][3]) & 0xFFFFu) st(s.tr_next, tix(hk), (uint16_t)(nprv[k] & 0xFFFFu));
        if ((nprv[k] ^ o[k][3]) >> 16) st(s.tr_prev, tix(hk), (uint16_t)(nprv[k] >> 16));
        if ((sdec[k] ^ o[k][4]) & 0xFFFFu) st(s.tr_src, tix(hk), (uint16_t)(sdec[k] & 0xFFFFu));
        if ((sdec[k] ^ o[k][4]) >> 16) st(s.tr_dec, tix(hk), (uint16_t)(sdec[k] >> 16));
        if ((uint32_t)delay[k] != o[k][5]) st(s.tr_delay, tix(hk), delay[k]);
      }
    }
#pragma unroll
    for (int k = 0; k < TPL && !PART; ++k) {
      const int hk = lane + G * k;
      if (mine[k]) {
        st(s.tr_pos, tix(hk), pos[k]);
        st(s.tr_bits, tix(hk), bits[k]);
        st(s.tr_plan, tix(hk), plan[k]);
        st(s.tr_next, tix(hk), (uint16_t)(nprv[k] & 0xFFFFu));
        st(s.tr_prev, tix(hk), (uint16_t)(nprv[k] >> 16));
        st(s.tr_src, tix(hk), (uint16_t)(sdec[k] & 0xFFFFu));
        st(s.tr_dec, tix(hk), (uint16_t)(sdec[k] >> 16));
        st(s.tr_delay, tix(hk), delay[k]);
      }
    }
    // (PART: a round changes a handful of records and one counter; only those are written back)
    // (the LDS reads first, then the stores: one wait instead of one per record)
    uint32_t rw[PPL], r0[PART ? PPL : 1], nw[SPL], n0[PART ? SPL : 1];
#pragma unroll
    for (int k = 0; k < PPL; ++k) {
      rw[k] = sem(k);
      if constexpr (PART) r0[k] = lsem0[k * G + lane];
    }
#pragma unroll
    for (int k = 0; k < SPL; ++k) {
      nw[k] = lcnt[k * G + lane];
      if constexpr (PART) n0[k] = (ldirty[(k * G + lane) >> 5] >> ((k * G + lane) & 31)) & 1u;
    }
#pragma unroll
    for (int k = 0; k < PPL; ++k) {
      const int p = k * G + lane;
      if (p < m.NP && (!PART || rw[k] != r0[PART ? k : 0])) st(sem_words(), pix(p), rw[k]);
    }
#pragma unroll
    for (int k = 0; k < SPL; ++k) {
      const int sw = k * G + lane;
      if (sw < m.S && (!PART || n0[PART ? k : 0] != 0u)) st(s.counts, cix(sw), nw[k]);
    }
    uint32_t err = 0;
#pragma unroll
    for (int b = 0; b < 6; ++b)
      if (BAL((lerr >> b) & 1u)) err |= 1u << b;
    if (PART) return err;
    if (lane == 0) {
      st(s.phase, e, phase);
      st(s.elapsed, e, now);
      st(s.eflags, e, flags);
      st(s.epoch, e, epoch);
      st(s.err, e, err);
      auto put = [&](int k, const Mask& mk) {
        uint64_t w[2];
        constexpr int NWD = (TPL * G <= 64 || TWc <= 32) ? 1 : 2;
        if constexpr (NWD == 1) {
          w[0] = mk;
          w[1] = 0ull;
        } else {
          w[0] = mk.w[0];
          w[1] = mk.w[1];
        }
#pragma unroll
        for (int j = 0; j < 2 * NWD; ++j) st(s.masks, (size_t)(k * MAXW + j) * E + e, (uint32_t)(w[j >> 1] >> (32 * (j & 1))));
      };
      put(0, q_mask);
      put(1, arr_mask);
      put(2, fl_mask);
      put(3, mf_mask);
      st(s.rng, ix(0), lrng[0]);
      st(s.rng, ix(1), lrng[1]);
      st(s.rng, ix(4), lrng[4]);
      st(s.cum_reward, e, (double)cum);
      st(s.n_mf, e, n_mf);
      st(s.ep_dec, e, ep_dec);
      st(s.ep_ticks, e, ep_ticks);
      st(s.step_ctr, e, (int64_t)step_ctr);
      st(s.dec_total, e, ld(s.dec_total, e) + (int64_t)n_dec);
    }
    return err;
  }
  // PART: the env's scalar block (sfl_part.h EB_*) after the round: staged in LDS (the lsem0 region, read by
  // store() before), then one store instruction, lane i writing word i
  __device__ __forceinline__ void store_eblk(int32_t phase, uint32_t err, int32_t ep_t, int32_t n_test, int64_t dec_done,
                                             int32_t req_dst, uint32_t upd_n, uint64_t l_dec, uint64_t l_ticks,
                                             uint64_t l_bytes) {
    if constexpr (PART) {
      uint32_t* sg = lsem0;
      auto put4 = [&](int i, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {  // uniform values, written by every lane
        u4 v;
        v[0] = a;
        v[1] = b;
        v[2] = c;
        v[3] = d;
        *(u4*)(sg + i) = v;
      };
      auto lo = [](uint64_t x) { return (uint32_t)x; };
      auto hi = [](uint64_t x) { return (uint32_t)(x >> 32); };
      const uint64_t dtot = ebw64(EB_DEC_TOTAL) + (uint64_t)n_dec;
      const uint64_t cumd = (uint64_t)__double_as_longlong((double)cum);
      const uint64_t r0 = lrng[0], r1 = lrng[1], r2 = lrng[2], r3 = lrng[3], r4 = lrng[4];
      uint64_t mw[4][2];
      auto mwords = [&](int k, const Mask& mk) {
        if constexpr (TPL * G <= 64 || TWc <= 32) {
          mw[k][0] = (uint64_t)mk;
          mw[k][1] = 0ull;
        } else {
          mw[k][0] = mk.w[0];
          mw[k][1] = mk.w[1];
        }
      };
      mwords(0, q_mask);
      mwords(1, arr_mask);
      mwords(2, fl_mask);
      mwords(3, mf_mask);
      static_assert(EB_PHASE == 0 && EB_EP_DEC == 8 && EB_STEP_CTR == 10 && EB_RNG == 16 && EB_MASKS == 26 &&
                        EB_DEC_DONE == 42 && EB_USED == 52 && MAXW == 4,
                    "block layout");
      put4(0, (uint32_t)phase, (uint32_t)now, flags, epoch);
      put4(4, err, (uint32_t)ep_t, (uint32_t)n_test, (uint32_t)n_mf);
      put4(8, (uint32_t)ep_dec, (uint32_t)ep_ticks, (uint32_t)step_ctr, 0u);
      put4(12, lo(dtot), hi(dtot), lo(cumd), hi(cumd));
      put4(16, lo(r0), hi(r0), lo(r1), hi(r1));
      put4(20, lo(r2), hi(r2), lo(r3), hi(r3));
      put4(24, lo(r4), hi(r4), lo(mw[0][0]), hi(mw[0][0]));
      put4(28, lo(mw[0][1]), hi(mw[0][1]), lo(mw[1][0]), hi(mw[1][0]));
      put4(32, lo(mw[1][1]), hi(mw[1][1]), lo(mw[2][0]), hi(mw[2][0]));
      put4(36, lo(mw[2][1]), hi(mw[2][1]), lo(mw[3][0]), hi(mw[3][0]));
      put4(40, lo(mw[3][1]), hi(mw[3][1]), lo((uint64_t)dec_done), hi((uint64_t)dec_done));
      put4(44, (uint32_t)req_dst, upd_n, lo(l_dec), hi(l_dec));
      put4(48, lo(l_ticks), hi(l_ticks), lo(l_bytes), hi(l_bytes));
      const uint32_t v = sg[lane < EB_USED ? lane : 0];
      if (lane < EB_USED) st(P->eblk, (size_t)e * PART_EB + (uint32_t)lane, v);
    }
  }

  // ---- episode reset (switch_env.py:93-158, _init_ports 507-568) --------------------------------
  __device__ __forceinline__ void reset() {
    now = 0;
#pragma unroll
    for (int k = 0; k < TPL; ++k) {
      if (mine[k]) {
        const int hk = lane + G * k;
        const uint32_t t_init = (uint32_t)ltt[8 * hk + 7];
        pos[k] = -1;
        bits[k] = tb_make(t_init & 0xFFu, S_WAITING, A_NONE, 0, 0, 0);
        plan[k] = 0;
        nprv[k] = (nprv[k] & 0xFFFF0000u) | (t_init >> 16);
        delay[k] = ltt[8 * hk + 6];
      }
    }
#pragma unroll
    for (int k = 0; k < PPL; ++k) sem(k) = 0u;
    for (int h = 0; h < m.T; ++h) {
      const vec_t<int32_t, 8> tr = LDCV<vec_t<int32_t, 8>>(m.tr_pack, (size_t)h);
      sset((int)((uint32_t)tr[7] >> 16), r_pack(h, 1, tr[0] - 2, tr[0] + tr[5]));
    }
    flags &= ~(F_TERM | F_TRUNC | F_OWN_SCAN | F_INFLIGHT);
    q_mask = arr_mask = fl_mask = mf_mask = Mask{};
    // new (switch, train) epoch: slots from older episodes read as empty
    epoch = (epoch + 1u) & 0xFFu;
    if (epoch == 0) {
      for (int i = lane; i < m.S * m.T; i += G) st(sbase(), (size_t)i, slot_make(PEND_NONE, 0, 0));
      epoch = 1;
    }
    cum = 0;
    n_mf = 0;
    ep_dec = 0;
    ep_ticks = 0;
    step_ctr = 0;
  }

  // ---- one Flatland tick + switchfl bookkeeping (switch_env.py:296-401, 427-485;
  //      flatland_lite.RailEnv.step), train-parallel: lane h = train h ----------------------------
  __device__ __forceinline__ void tick() {
    PrioGuard<PART ? 0 : SFL_SETPRIO_TICK> prio;  // (the partitioned local step: no gain, profiles/r05ag_*)
    SFL_LAP0();
    if constexpr (xp::kNoTick) {
      ++now;
      return;
    }
    pf_ok = false;
    const int32_t t = ++now;
    const uint64_t seed = s.seed[e];
    // the trains' timetable rows (LDS)
    vec_t<int32_t, 4> tt0[TPL], tt1[TPL];
#pragma unroll
    for (int k = 0; k < TPL; ++k) {
      tt0[k] = *(const vec_t<int32_t, 4>*)(ltt + 8 * (mine_(k) ? lid() + G * k : 0));
      tt1[k] = *(const vec_t<int32_t, 4>*)(ltt + 8 * (mine_(k) ? lid() + G * k : 0) + 4);
    }
    // pass 1: plan pop + prediction, malfunction draw, action preprocessing, desired move
    // (the slots' move-table rows loaded together, clamped: inside each slot's exec-masked block the
    // second load waited for the first slot's work)
    u4 mrows[TPL];
#pragma unroll
    for (int k = 0; k < TPL; ++k) {
      const bool ok = mine_(k);
      const int pc = pos[k] >= 0 ? pos[k] : tt1[k][0];
      const int pd = pos[k] >= 0 ? (int)tb_dir(bits[k]) : (int)((uint32_t)tt1[k][3] & 0xFFu);
      mrows[k] = move_row((uint32_t)(ok ? pc : 0) * 4u + (uint32_t)(ok ? pd : 0));
    }
    bool mover[TPL];
    int32_t desired[TPL], pred[TPL];
    uint32_t aux[TPL];
#pragma unroll
    for (int k = 0; k < TPL; ++k) {
      const int h = lid() + G * k;
      const int32_t t_init_cell = tt1[k][0];
      const uint32_t t_init_dir = (uint32_t)tt1[k][3] & 0xFFu;
      mover[k] = false;
      desired[k] = -1;
      pred[k] = -1;
      aux[k] = 0;
      if (mine_(k)) {
        const uint32_t b = bits[k];
        const int32_t p0 = pos[k];
        uint32_t st_ = tb_state(b), dir = tb_dir(b), prev = tb_prev(b), saved = tb_saved(b), mf = tb_mf(b);
        uint32_t given = A_NOTHING;
        pred[k] = p0;
        // every check_action of this pass is at (pc, pd): one 16-byte load of the move-table row
        const int pc = p0 >= 0 ? p0 : t_init_cell;
        const int pd = p0 >= 0 ? (int)dir : (int)t_init_dir;
        const u4 mrow = mrows[k];
        auto mv_of = [&](uint32_t a) -> Move {
          const uint32_t q = a & 3u;
          return unpack_move(q == 0 ? mrow[0] : q == 1 ? mrow[1] : q == 2 ? mrow[2] : mrow[3]);
        };
        if (!tb_done(b)) {
          const uint32_t pl = plan[k];
          if (pl_len(pl) == 0) {
            given = A_FWD;
          } else {
            given = pl_front(pl);
            prev = given;
            plan[k] = pl_pop(pl);
          }
          if (p0 >= 0) {
            const Move mv = mv_of(given);
            aux[k] |= 1u << 12;
            if (mv.valid) {
              aux[k] |= 1u << 13;
              pred[k] = mv.cell;
              if (dest_sw(mv) >= 0) aux[k] |= 1u << 14;  // the predicted cell is a switch cell
            }
          }
        }
        if (st_ != S_DONE && mf == 0) mf = mf_propose(m, seed, e, t, h);
        // preprocess_action
        uint32_t pa = given;
        if (pa == A_NOTHING && st_ == S_MOVING) pa = A_FWD;
        if (st_ == S_WAITING) pa = A_NOTHING;
        if (pa == A_LEFT || pa == A_RIGHT) {
          const Move mv = mv_of(pa);
          if (!(mv.cell_ok && mv.valid)) pa = A_FWD;
        }
        if (is_moving_action(pa)) {
          const Move mv = mv_of(pa);
          if (!(mv.cell_ok && mv.valid)) pa = A_STOP;
        }
        if (is_moving_action(pa) && saved == 0 && st_ != S_DONE) saved = pa;
        const bool update_allowed = (mf == 0) && pa != A_STOP;
        desired[k] = p0;
        uint32_t ddir = dir;
        if (st_ == S_DONE) {
        } else if (p0 < 0 && saved != 0) {
          desired[k] = t_init_cell;
          ddir = t_init_dir;
          mover[k] = true;
        } else if (saved != 0 && update_allowed) {
          const Move mv = mv_of(saved);
          desired[k] = mv.cell;
          ddir = (uint32_t)mv.dir;
          pa = saved;
          mover[k] = desired[k] != p0;
        }
        aux[k] |= pa | (ddir << 4) | (given << 8);
        bits[k] = tb_make(dir, st_, prev, saved, mf, tb_done(b));
      }
    }
    SFL_LAP(11);
    // pass 2: motion check, least fixed point (flatland_lite.motion_check): the lowest handle
    // wanting a cell wins it; a cell can be entered if free or its occupant moves out
    const Mask M = mbal(mover);
    Mask A{};
    if (many(M)) {
      // Bit-sliced equality instead of a loop over trains: for each bit of the cell index, one
      // ballot (per train slot) of the movers' desired cells and one of the on-map trains'
      // cells; a train ANDs in each ballot or its complement by its own desired cell's bit,
      // leaving exactly the movers that want the same cell (`same`) and the train that occupies
      // it (`occs`).  One extra bit keeps an off-grid target (-1) apart from every cell.
      bool onmap[TPL];
#pragma unroll
      for (int k = 0; k < TPL; ++k) onmap[k] = mine_(k) && pos[k] >= 0;
      Mask same[TPL], occs[TPL];
      const Mask occ0 = mbal(onmap);
#pragma unroll
      for (int k = 0; k < TPL; ++k) {
        same[k] = M;
        occs[k] = occ0;
      }
      for (int bi = 0; bi < m.cell_bits; ++bi) {
        bool pd_[TPL], pp_[TPL];
#pragma unroll
        for (int k = 0; k < TPL; ++k) {
          pd_[k] = mover[k] && (((uint32_t)desired[k] >> bi) & 1u);
          pp_[k] = onmap[k] && (((uint32_t)pos[k] >> bi) & 1u);
        }
        const Mask bd = mbal(pd_), bp = mbal(pp_);
#pragma unroll
        for (int k = 0; k < TPL; ++k) {
          const bool one = ((uint32_t)desired[k] >> bi) & 1u;
          same[k] &= one ? bd : ~bd;
          occs[k] &= one ? bp : ~bp;
        }
      }
      if (m.cell_bits < 32) {  // the sign bit of an off-grid target
        bool pn[TPL];
#pragma unroll
        for (int k = 0; k < TPL; ++k) pn[k] = mover[k] && desired[k] < 0;
        const Mask bd = mbal(pn);
#pragma unroll
        for (int k = 0; k < TPL; ++k) {
          same[k] &= desired[k] < 0 ? bd : ~bd;
          if (desired[k] < 0) occs[k] = Mask{};
        }
      }
      // the lowest handle wanting a cell wins it; the occupant is the (last) train on it
      bool win[TPL];
      int occ[TPL];
#pragma unroll
      for (int k = 0; k < TPL; ++k) {
        const int h = lid() + G * k;
        win[k] = mover[k] && !many(same[k] & mbelow(Mask{}, h));
        const Mask occset = occs[k] & ~mone(Mask{}, h);
        occ[k] = (mover[k] && many(occset)) ? mhighest(occset) : -1;
      }
      while (true) {
        bool cand[TPL];
#pragma unroll
        for (int k = 0; k < TPL; ++k) {
          const int h = lid() + G * k;
          cand[k] = mover[k] && win[k] && !mbit(A, h) && (occ[k] < 0 || (mbit(M, occ[k]) && mbit(A, occ[k])));
        }
        const Mask nb = mbal(cand);
        if (!many(nb)) break;
        A |= nb;
      }
    }
    SFL_LAP(12);
    // pass 3: state machine + positions, deviation fix
    const bool over = t >= m.max_episode_steps;
    bool done[TPL], isdone[TPL], newly[TPL], dep[TPL];
#pragma unroll
    for (int k = 0; k < TPL; ++k) {
      const int h = lid() + G * k;
      const int32_t t_ed = tt0[k][0], t_target = tt0[k][3], t_init_cell = tt1[k][0];
      const uint32_t t_init_dir = (uint32_t)tt1[k][3] & 0xFFu;
      done[k] = false;
      isdone[k] = !mine_(k);
      newly[k] = false;
      dep[k] = false;
      if (mine_(k)) {
        const uint32_t b = bits[k];
        const int32_t p0 = pos[k];
        uint32_t st_ = tb_state(b), dir = tb_dir(b), saved = tb_saved(b), mf = tb_mf(b);
        const uint32_t pa = aux[k] & 15u;
        const bool in_mf = mf > 0;
        bool ma = in_mf ? false : (mover[k] && mbit(A, h));
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
            np = desired[k];
            dir = (aux[k] >> 4) & 3u;
            if (np == t_target) st_ = S_DONE;
          }
        }
        if (st_ == S_DONE && !mbit(arr_mask, h)) {
          newly[k] = true;  // arrived: position None, arrival_time set
          np = -1;
        }
        if (mf > 0) mf -= 1;
        if (np >= 0) saved = 0;
        done[k] = (st_ == S_DONE) || over;
        isdone[k] = st_ == S_DONE;
        pos[k] = np;
        // switchfl: deviation fix
        if ((aux[k] >> 12) & 1u) {
          const uint32_t given = (aux[k] >> 8) & 15u;
          if (pred[k] != np && ((aux[k] >> 13) & 1u) && given != A_STOP) {
            plan[k] = pl_push_front(plan[k], given, lerr);
            if ((aux[k] >> 14) & 1u) nprv[k] = (nprv[k] & 0xFFFF0000u) | (sdec[k] & 0xFFFFu);
          }
        }
        dep[k] = t == t_ed - 2;
        bits[k] = tb_make(dir, st_, tb_prev(b), saved, mf, done[k] ? 1u : 0u);
      }
    }
    arr_mask |= mbal(newly);
    SFL_LAP(13);
    // delete the semaphores of done trains (switch_env.py:370-376): each lane its own records
    const Mask DONE = mbal(done);
    if (many(DONE)) {
#pragma unroll
      for (int k = 0; k < PPL; ++k) {
        const uint32_t r = sem(k);
        sem(k) = (r_present(r) & mbit(DONE, (int)r_owner(r))) ? 0u : r;
      }
    }
    // departure semaphores, in handle order (switch_env.py:379-384)
    Mask D = mbal(dep);
    while (many(D)) {
      const int j = mctz(D);
      mclear_low(D);
      const int32_t ed = ltt[8 * j];
      sset((int)(trl(nprv, j) & 0xFFFFu), r_pack(j, 1, ed - 2, ed + tr_init_dist(j)));
    }
    // pass 4: extend_semaphores (rail_network.py:229-244)
    bool smp[TPL], map_[TPL], mfp[TPL];
#pragma unroll
    for (int k = 0; k < TPL; ++k) {
      const uint32_t st4 = tb_state(bits[k]);
      smp[k] = mine_(k) && (st4 == S_STOPPED || st4 == S_MALF);
      map_[k] = mine_(k) && st4 == S_MALF;
      mfp[k] = mine_(k) && tb_mf(bits[k]) > 0;
    }
    const Mask SM = mbal(smp);
    if (many(SM)) {
#pragma unroll
      for (int k = 0; k < PPL; ++k) {
        const uint32_t r = sem(k);
        const bool ext = r_present(r) & mbit(SM, (int)r_owner(r));
        sem(k) = ext ? r_retime(r, t) : r;
      }
    }
    Mask MA = mbal(map_);
    while (many(MA)) {
      const int j = mctz(MA);
      mclear_low(MA);
      const int p = (int)(trl(nprv, j) & 0xFFFFu);
      if (!r_present(sget(p))) sset(p, r_pack(j, 1, t, t + tr_init_dist(j)));
    }
    // malfunction count (switch_env.py:399-401)
    const Mask MF = mbal(mfp);
    n_mf += mpopc(MF & ~mf_mask);
    mf_mask = MF;
    SFL_LAP(14);
    // _check_active_switch (switch_env.py:427-485)
    // (the slots' move-table loads issued together)
    int sw_next[TPL];  // the switch at the cell the train's next rail action leads to (-1: none)
#pragma unroll
    for (int k = 0; k < TPL; ++k) {
      const bool ok = mine_(k) && pos[k] >= 0;
      const uint32_t nxt = pl_len(plan[k]) ? pl_front(plan[k]) : A_FWD;
      const Move mv = check_action<false>(nxt, ok ? pos[k] : 0, ok ? (int)tb_dir(bits[k]) : 0);
      sw_next[k] = mv.cell >= 0 ? dest_sw(mv) : -1;
    }
    bool act[TPL];
#pragma unroll
    for (int k = 0; k < TPL; ++k) {
      act[k] = false;
      const uint32_t st4 = tb_state(bits[k]);
      if (mine_(k) && pos[k] >= 0 && st4 != S_WAITING) {
        {
          const int sw_at = sw_next[k];
          if (sw_at >= 0) {
            int sw = -1;
            if (st4 == S_READY || st4 == S_MOVING) sw = sw_at;
            else if ((st4 == S_STOPPED || st4 == S_MALF) && tb_prev(bits[k]) == A_STOP) sw = sw_at;
            else if (st4 == S_STOPPED || st4 == S_MALF) sw = (int)((nprv[k] & 0xFFFFu) >> 2);
            if (sw >= m.S) {  // next port is None: the reference would raise here
              lerr |= E_PORT;
            } else if (sw >= 0) {
              act[k] = true;
              sdec[k] = (sdec[k] & 0xFFFFu) | ((uint32_t)sw << 16);
            }
          }
        }
      }
    }
    q_mask = mbal(act);
    SFL_LAP(15);
    const Mask full = mfirst(Mask{}, m.T);
    const Mask ALL = mbal(isdone);
    ep_ticks += 1;
    if ((ALL & full) == full || over) flags |= F_TERM;
  }

  // ---- batch prefetch ----------------------------------------------------------------------
  // When a tick leaves decisions queued, each queued train's lane loads, in parallel, its
  // (switch, train) slot word, the Q cell of the pending update that slot holds, and the Q row of
  // its observation as the semaphores stand now, into LDS.  The batch's decisions then run in
  // handle order as before; a decision uses a staged row only if the row it actually observes
  // (after the batch's earlier decisions changed the semaphores) is the staged one, and staged
  // Q values are dropped when the batch writes their cell (pf_written).  Slot words are never
  // stale: a decision writes only its own train's slots and a train decides once per batch.
  __device__ __forceinline__ void prefetch(bool greedy) {
    PrioGuard<PART ? 0 : SFL_SETPRIO_PF> prio;
    const Mask malf = malf_mask();
#pragma unroll
    for (int k = 0; k < PFS; ++k) pf_roff[k] = pf_qoff[k] = PF_NONE;
    pf_n = 0;
    if constexpr (EPS_PF) lrng[5] = 0ull;  // (uniform value from every lane) the staged epsilons are current
    if constexpr (PF_BY_RANK) {
      // lane i stages the i-th queued train (record i = the i-th decision of the batch); trains beyond the
      // records wait for the next staging
      const int nq = mpopc(q_mask);
#pragma unroll 1
      for (int k = 0; k < PFS; ++k) {
        const int i = lid() + G * k;
        const bool on = i < nq && i < PF_SLOTS;
        const int h = mselect(q_mask, on ? i : 0);
        const uint32_t sd = trl_v(sdec, h), npv = trl_v(nprv, h), bt = trl_v(bits, h), pl = trl_v(plan, h);
        const int32_t ps = trl_v(pos, h);
        uint32_t roff = PF_NONE, qoff = PF_NONE;
        if (on) prefetch_slot(h, i, sd, npv, bt, ps, pl, malf, greedy, roff, qoff);
#pragma unroll
        for (int j = 0; j < PFS; ++j) {
          pf_roff[j] = j == k ? roff : pf_roff[j];
          pf_qoff[j] = j == k ? qoff : pf_qoff[j];
        }
      }
      return;
    }
    // one train slot at a time (not unrolled): the slots' loads would otherwise be interleaved and
    // hold twice the registers; the slot's registers are selected by value, not indexed
    // PART: a launch decides one train per env (the round ends at the next request, and the staging
    // does not survive the launch): stage that train only
    const int h_first = PART ? mctz(q_mask) : -1;
#pragma unroll 1
    for (int k = 0; k < TPL; ++k) {
      if (!mbit(q_mask, lid() + G * k)) continue;
      if (PART && lid() + G * k != h_first) continue;
      uint32_t roff, qoff;
      prefetch_slot(lid() + G * k, pfx(lid() + G * k), pick(sdec, k), pick(nprv, k), pick(bits, k), pick(pos, k),
                    pick(plan, k), malf, greedy, roff, qoff);
#pragma unroll
      for (int j = 0; j < TPL; ++j) {
        pf_roff[j] = j == k ? roff : pf_roff[j];
        pf_qoff[j] = j == k ? qoff : pf_qoff[j];
      }
    }
  }
  template <class T>
  __device__ __forceinline__ static T pick(const T (&x)[TPL], int k) {
    T v = x[0];
#pragma unroll
    for (int j = 1; j < TPL; ++j) v = j == k ? x[j] : v;
    return v;
  }
  // train hk (one of this lane's slots) is queued: stage its decision's inputs; its registers are
  // passed by value (sdec, nprv, bits, pos, plan); returns the staged row and pending-cell offsets
  __device__ __forceinline__ void prefetch_slot(const int hk, const int rec, const uint32_t sdec_k, const uint32_t nprv_k,
                                                const uint32_t bits_k, const int32_t pos_k, const uint32_t plan_k, Mask malf,
                                                bool greedy, uint32_t& roff_out, uint32_t& qoff_out) {
    if constexpr (xp::kNoPrefetch) {
      roff_out = qoff_out = PF_NONE;
      return;
    }
    // Loads are issued by dependency level, unconditionally (clamped indices), so the chains
    // overlap: level 1 needs only this train's registers, level 2 the level-1 results, ...
    const int sw = (int)(sdec_k >> 16);
    const int pin = (int)(nprv_k & 0xFFFFu);
    const int slot = pin & 3;
    const int dir0 = (int)tb_dir(bits_k);
    const int pos0 = pos_k >= 0 ? pos_k : 0;
    double* pfl = lpf + PFD * rec;
    uint32_t* pfi = lpi + PF_WI * rec;
    // level 1: slot word, switch record, timetable row, the row block's port record, first moves
    const uint64_t slw = ld(sbase(), slot_ix(sw, hk));
    const u4 w0 = sw_v4(sw, 0);
    const u4 w4 = sw_v4(sw, 1);  // compact-row descriptors
    const vec_t<uint32_t, 2> nbw = sw_nb_v(sw);
    const vec_t<int32_t, 4> trw = *(const vec_t<int32_t, 4>*)(ltt + 8 * hk);  // ed, la, k, target
    const u4 pr = port_v(4 * sw + slot);
    const uint32_t n_plan = pl_len(plan_k);
    const uint32_t a1 = n_plan ? pl_front(plan_k) : A_FWD;
    // move-table rows (all four rail actions) at the cell and after the first rail action
    const u4 row0 = move_row((uint32_t)pos0 * 4u + (uint32_t)dir0);
    auto mv_in = [](const u4& r, uint32_t a) -> Move {
      const uint32_t q = a & 3u;
      return unpack_move(q == 0 ? r[0] : q == 1 ? r[1] : q == 2 ? r[2] : r[3]);
    };
    // distances the decision needs (reward_func.py:23-78): at the cell, along the STOP plan
    // ([STOP] + plan) and along each route's plan ([front or FWD, final rail action 1..3])
    const int32_t la = (int32_t)trw[1], k = (int32_t)trw[2];
    const int32_t dd = dist_v(k, pos_k, dir0);
    int32_t d_stop, d_rt[4];
    {
      // Both projections in one dependent level: the plan's first two moving entries (STOP entries are
      // skipped) from the move-table row at the cell and the two-step row move2c_tab[cell, dir, a] (a: the
      // route plan's first action, which is also the STOP plan's first move unless the plan starts with
      // STOP -- then the route plan moves by the final action only, row0).  A STOP plan with more than two
      // moves (rare) walks the rest with dependent loads.
      const uint32_t body = plan_k >> 4;  // entries, 4 bits each
      const uint32_t used = 0x1111111u & ((1u << (4u * (n_plan < 7u ? n_plan : 7u))) - 1u);
      uint32_t isstop = ~(body ^ 0x4444444u);  // bit 0 of a nibble: the entry is STOP (A_STOP = 4)
      isstop &= isstop >> 1;
      isstop &= isstop >> 2;
      const uint32_t mvb = used & ~isstop;
      const int nmv = __builtin_popcount(mvb);
      const uint32_t i0 = (uint32_t)__builtin_ctz(mvb | 0x10000000u);
      const uint32_t mvb1 = mvb & (mvb - 1u);
      const uint32_t i1 = (uint32_t)__builtin_ctz(mvb1 | 0x10000000u);
      const uint32_t x0 = (body >> i0) & 15u, x1 = (body >> i1) & 15u;
      const uint32_t at2 = a1 != A_STOP ? a1 : x0;
      const u4 t2 = ld((const u4*)m.move2c_tab, (size_t)(((uint32_t)pos0 * 4u + (uint32_t)dir0) * 4u + (at2 & 3u)));
      const bool on = pos_k >= 0;
      // the STOP plan's walk
      int pc = pos_k, pd = dir0;
      if (on && nmv == 1) {
        const Move mv = mv_in(row0, x0);
        pc = mv.cell;
        pd = mv.dir;
      } else if (on && nmv >= 2) {
        const Move mv = mv_in(t2, x1);
        pc = mv.cell;
        pd = mv.dir;
        if (nmv > 2) {  // the rest of the walk (entries after the second move)
          for (uint32_t i = (i1 >> 2) + 1u; i < n_plan; ++i) project(pl_at(plan_k, i), pc, pd);
        }
      }
      d_stop = dist_v(k, pc, pd);
      d_rt[0] = 0;  // final rail action 0 (DO_NOTHING) is never a route's
#pragma unroll
      for (uint32_t t = 1; t < 4; ++t) {
        const Move mv = mv_in(a1 != A_STOP ? t2 : row0, t);
        d_rt[t] = dist_v(k, on ? mv.cell : -1, on ? mv.dir : dir0);
      }
    }
    // level 2: the pending update's block; the observation (LDS) and its row
    const uint32_t pend = greedy ? PEND_NONE : slot_pend(slw, epoch);
    const bool hp = pend != PEND_NONE;
    const u4 pp = port_v(hp ? 4 * (int)(pend & 0xFFFu) + (int)((pend >> 12) & 3u) : 0);
    const int np = (int)(w0[0] & 15u);
    uint32_t fb = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int p = 4 * sw + j;
      const int nb = j < np ? (int)((nbw[j >> 1] >> (16 * (j & 1))) & 0xFFFFu) : p;
      const uint32_t blk = rec_blocks(lsem[nb], (uint32_t)hk, malf, 0u) | rec_blocks(lsem[p], (uint32_t)hk, malf, 1u);
      fb |= (blk == 0u && j < np) ? (1u << j) : 0u;
    }
    const int32_t dl = now - la + dd;
    const int32_t avail = la - (int32_t)trw[0];
    const uint32_t lvl = dl <= 0 ? 0u : (dl <= avail * m.delay_thr ? 1u : 2u);
    const uint32_t state = ((fb * (uint32_t)m.K) + (uint32_t)k) * 3u + lvl;
    const uint32_t w = pr[1] >> 16, roff = pr[3] + state * w;
    const bool row_ok = pos_k >= 0 && dd < DIST_INF && (pin >> 2) == sw && slot < np;
    const uint32_t qoff = pp[3] + ((pend >> 14) & 0x3FFFu) * (pp[1] >> 16) + ((pend >> 28) & 3u);
    // level 3: Q values
    // (PART: the rows live on their owners; nothing is staged)
    double rv[4] = {0.0, 0.0, 0.0, 0.0};
    double qv = 0.0;
    if constexpr (!PART) {
      const double* rp = qbase() + (row_ok ? roff : 0u);
#pragma unroll
      for (int c = 0; c < 4; ++c) rv[c] = ld(rp, (size_t)((uint32_t)c < w ? c : 0));
      qv = ld(qbase(), (size_t)(hp ? qoff : 0u));
    }
    // (EPS_PF) eps0 * decay**n of the decision switch at its present count (distr_q.py:59-68), with the Q loads (a
    // short live range); beyond the table the decision computes it
    if constexpr (EPS_PF) {
      const uint32_t n_s = cget_var(sw);
      double eps_v = 0.0;
      if (!greedy && n_s < (uint32_t)m.ntab) eps_v = ld(m.eps_tab, (size_t)n_s);
      pfl[3] = eps_v;
    }
    // the greedy choice on the staged row (distr_q.py:449-490, as in decide): valid whenever the
    // row is (a decision uses it only if its observation is the staged one)
    {
      const uint32_t rd = w4[slot];
      const int na = (int)((w0[0] >> 4) & 15u);
      // branch-free (selects, fixed trip counts): the lanes of a batch sit on different switches
      uint32_t am = 1u << (na - 1);
#pragma unroll
      for (int a = 0; a < 8; ++a) {
        const uint32_t ok = (uint32_t)(a < na - 1) & (uint32_t)((int)((w0[1] >> (2 * a)) & 3u) == slot) &
                            ((fb >> ((w0[1] >> (16 + 2 * a)) & 3u)) & 1u);
        am |= ok << a;
      }
      const int mind = (int)((rd >> 16) & 15u);
      double mx = mind != 15 ? m.default_q : -__builtin_huge_val();
      int best = mind != 15 ? mind : 99, arg = -1;
      double amx = 0.0;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int a = (int)((rd >> (4 * c)) & 15u);
        const double v = rv[c];
        const bool in = (uint32_t)c < w;
        // bitwise, not short-circuit, operators: no divergent branches in this lane-parallel code
        const bool b1 = in & ((v > mx) | ((v == mx) & (a < best)));
        mx = b1 ? v : mx;
        best = b1 ? a : best;
        const bool b2 = in & (((am >> a) & 1u) != 0u) & ((arg < 0) | (v > amx) | ((v == amx) & (a < arg)));
        arg = b2 ? a : arg;
        amx = b2 ? v : amx;
      }
      pfl[2] = mx;
      pfi[2] = d16(d_rt[3]) | ((uint32_t)((best & 0xFF) | ((arg & 0xFF) << 8)) << 16);
    }
    pfl[0] = qv;
    pfl[1] = __longlong_as_double((long long)slw);
    pfi[0] = d16(dd) | (d16(d_stop) << 16);
    pfi[1] = d16(d_rt[1]) | (d16(d_rt[2]) << 16);
    roff_out = (row_ok && !PART) ? roff : PF_NONE;
    qoff_out = (hp && !PART) ? qoff : PF_NONE;
  }
  // a Q cell of this env was written (uniform offset): drop staged copies that contain it
  __device__ __forceinline__ void pf_written(uint32_t off) {
#pragma unroll
    for (int k = 0; k < PFS; ++k) {
      pf_qoff[k] = (pf_qoff[k] == off) ? PF_NONE : pf_qoff[k];
      pf_roff[k] = (off - pf_roff[k] < 4u) ? PF_NONE : pf_roff[k];
    }
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
    double mq;        // max over the full decision row (successor value for the pending update)
    uint32_t qoff_pend;  // Q cell (offset in the env's block) of the pending update consumed here, or PF_NONE
    double q_pend;    // its value, loaded during the decision
    uint32_t row_pend;  // key-set row of the pending update
    uint32_t row_cur;   // key-set row of this decision's observation
    bool touch_cur;     // greedy choice: insert row_cur into the key set (max_action's __check_entry)
    uint32_t abytes;    // algorithmic bytes of the decision
  };

  // PART: true = observe pass (no reply yet): the request went to the row's owner and nothing of
  // the env changed (the next launch repeats the observation, which is deterministic, and
  // applies the reply)
  template <bool TM = false>
  __device__ __forceinline__ bool decide(Dec& d, bool greedy) {
    PrioGuard<PART ? 0 : SFL_SETPRIO_DECIDE> prio;
    // PART: a row of this rank's own switches is decided in one pass, like the fused kernel
    const bool loc = local_sw((int)(trl(sdec, mctz(q_mask)) >> 16));
    const bool observe_only = PART && !(flags & F_REQ) && !loc;
    SFL_PT(t_obs);
    SFL_LAP0();
    // agent_iter: lowest queued train (switch_env.py:418-421, 616-622)
    // (PART observe pass: the observation needs one distance, looked up directly below; the
    // staging waits for the apply pass in the next launch)
    // (PART observe pass: no staging.  Round 5 measured carrying the observe pass's record to the apply pass in the
    // env's scalar block instead of restaging it: 95.2 M vs 95.8 M per GPU on the 8-rank rehearsal -- the apply
    // pass's staging overlaps its state load; not kept.)
    if ((!pf_ok || (RING && pf_n >= PF_SLOTS)) && !observe_only) {
      prefetch(greedy);
      pf_ok = !PART;  // (PART stages only this decision's train: the next one stages its own)
      SFL_PCNT(3);
    }
    SFL_LAP(0);
    SFL_PCNT(8);
    const int h = mctz(q_mask);
    if (!observe_only) mclear_low(q_mask);
    const uint32_t sd = trl(sdec, h);
    const int sw = (int)(sd >> 16);
    const SwRec swr = sw_rec(sw);
    const vec_t<int32_t, 8> tr = tr_row(h);
    const int rec = RING ? pf_n : pfx(h);
    if constexpr (RING) pf_n += 1;
    const double* pfh = lpf + PFD * rec;
    const uint32_t* pfw = lpi + PF_WI * rec;
    // the decision's LDS reads that do not depend on its observation, issued together: the staged
    // slot word (never stale: a decision writes only its own train's slots), row column, pending
    // cell value and distances, the epsilon-greedy stream and the switch's interaction count
    const uint64_t slot_v = (uint64_t)__double_as_longlong(pfh[1]);
    const double pf_qp = pfh[0];
    const double pf_mx = pfh[2];
    const uint32_t pfd01[2] = {pfw[0], pfw[1]};
    const uint32_t pfd23[1] = {pfw[2]};
    uint64_t rng_w[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) rng_w[i] = lrng[i];
    const uint32_t n_sw = cget(sw);
    const int pidx = PF_BY_RANK ? rec : h;  // the staged offsets' record
    const uint32_t pf_roff_h = rec_of(pf_roff, pidx), pf_qoff_h = rec_of(pf_qoff, pidx);
    const int np = swr.np();
    const int na = swr.na();
    const uint32_t npv = trl(nprv, h);
    const int pin = (int)(npv & 0xFFFFu);
    const int pprev = (int)(npv >> 16);
    int slot = pin & 3;
    if ((pin >> 2) != sw || slot >= np) {  // observer.py:294-301 (the reference would raise)
      lerr |= E_PORT;
      slot = 0;
    }
    SFL_LAP(1);
    // observe: lane j < np evaluates check_port_blocked(next_port(p_j), p_j) for port j of the
    // switch (observer.py:44-151, 269-283), branch-free integer VALU, then one ballot; lane a
    // evaluates get_action_mask for route a (switch_agents.py:104-134)
    const vec_t<uint32_t, 2> nbw = sw_nb(sw);
    const int pj = 4 * sw + (lid() & 3);
    const uint32_t nbl = ((lid() & 2) ? nbw[1] : nbw[0]) >> ((lid() & 1) * 16);
    const bool pvalid = lid() < np;
    const int nbj = pvalid ? (int)(nbl & 0xFFFFu) : pj;
    const Mask malf = malf_mask();
    const uint32_t rn = lsem[nbj], ro = lsem[pj];
    const uint32_t blk = rec_blocks(rn, (uint32_t)h, malf, 0u) | rec_blocks(ro, (uint32_t)h, malf, 1u);
    const uint32_t free_bits = (uint32_t)BAL(pvalid && blk == 0u) & 15u;
    SFL_LAP(2);
    const uint32_t b = trl(bits, h);
    const int32_t p0 = trl(pos, h);
    const int32_t ed = tr[0], la = tr[1], k = tr[2];
    const int32_t d_obs = observe_only ? dist(k, p0, (int)tb_dir(b)) : dist_staged(d16_lo(U(pfd01[0])));
    const int32_t dl = now - la + d_obs;
    const int32_t avail = la - ed;
    const uint32_t lvl = dl <= 0 ? 0u : (dl <= avail * m.delay_thr ? 1u : 2u);
    const uint32_t state = ((free_bits * (uint32_t)m.K) + (uint32_t)k) * 3u + lvl;
    const uint32_t la7 = (uint32_t)lid() & 7u;
    const uint32_t srca = (swr.w[1] >> (2u * la7)) & 3u, dsta = (swr.w[1] >> (16u + 2u * la7)) & 3u;
    const uint32_t amask =
        ((uint32_t)BAL(lid() < na - 1 && srca == (uint32_t)slot && ((free_bits >> dsta) & 1u)) & 0xFFu) |
        (1u << (na - 1));
    SFL_LAP(3);
    if constexpr (TM) {  // observe done (observer.py:246-308)
      if (tm_on) tm_obs_t = (uint64_t)__builtin_amdgcn_s_memtime();
    }
    SFL_PACC(0, t_obs);
    SFL_PT(t_eg);
    // issue the Q row load and the pending update's Q cell load, then draw while they fly
    const PortRec prr = port_rec(4 * sw + slot);
    const int w = prr.q_w();
    // (PART: another rank's row has no offset here -- its owner answers -- so no scalar load waits for one)
    const uint32_t roff = (!PART || loc) ? qoff_of(4 * sw + slot, prr) + state * (uint32_t)w : PF_NONE - 1u;
    // lane c < w holds compact column c of the row (staged by prefetch unless stale)
    const bool colv = lid() < w;
    const bool row_hit = pf_roff_h == roff;  // the staged row and its greedy choice are valid
    double v_c = 0.0;
    if (row_hit) {
      SFL_PCNT(4);
    } else if (loc) {
      v_c = ld(qbase() + roff, (size_t)(colv ? lid() : 0));
      SFL_PCNT(5);
    }
    SFL_LAP(4);
    d.slotword = U(slot_v);
    const uint32_t pend = greedy ? PEND_NONE : slot_pend(d.slotword, epoch);
    d.qoff_pend = PF_NONE;
    double q_pend_v = 0.0;
    if (!observe_only && pend != PEND_NONE) {  // (observe pass: the LDS record was not staged)
      const int ps = (int)(pend & 0xFFFu);
      const int pslot = (int)((pend >> 12) & 3u);
      const uint32_t pstate = (pend >> 14) & 0x3FFFu;
      const int pj = (int)((pend >> 28) & 3u);
      const PortRec pr = port_rec(4 * ps + pslot);
      const bool loc_p = local_sw(ps);
      if (!PART || loc_p) {
        d.qoff_pend = qoff_of(4 * ps + pslot, pr) + pstate * (uint32_t)pr.q_w() + (uint32_t)pj;
        d.row_pend = rowb_of(4 * ps + pslot, pr) + pstate;
      }
      if (!loc_p) {
        // the pending update is applied by its row's owner (PART: d.qoff_pend stays PF_NONE; post_part emits the record)
      } else if (pf_qoff_h == d.qoff_pend) {
        q_pend_v = pf_qp;
        SFL_PCNT(6);
      } else {
        q_pend_v = ld(qbase(), (size_t)d.qoff_pend);
        SFL_PCNT(7);
      }
    }
    const int32_t reward = slot_rew(d.slotword, epoch);
    SFL_LAP(5);
    // epsilon-greedy
    int action = -1;
    bool explore = false;
    if (!greedy && !xp::kNoRng) {
      // (kept in VGPRs: the 128-bit LCG runs on the vector ALU's 64-bit multiply-adds; the scalar
      // unit is the contended one)
      Pcg64 rng;
      rng.shi = rng_w[0];
      rng.slo = rng_w[1];
      rng.ihi = rng_w[2];
      rng.ilo = rng_w[3];
      rng.has = U((uint32_t)(rng_w[4] >> 32));  // uniform: pcg_next32's branch on it stays scalar
      rng.buf = (uint32_t)rng_w[4];
      const uint32_t n = n_sw;
      // eps0 * decay**n (distr_q.py:59-68): host-computed table (a scalar load, K$-resident), pow beyond it
      const double ud = Ud(pcg_double(rng));
      if (xp::kEpsConst) {
        explore = ud < m.eps0;
      } else {
        // (EPS_PF) the staged value, unless the switch was decided on since the staging (its count moved)
        bool staged = false;
        double eps_st = 0.0;
        if constexpr (EPS_PF) {
          staged = !((lrng[5] >> sw) & 1ull) && n < (uint32_t)m.ntab;
          eps_st = pfh[3];
        }
        explore = ud < (staged ? eps_st
                               : (n < (uint32_t)m.ntab ? LDC(m.eps_tab, (size_t)n) : m.eps0 * pow_ool(m.eps_decay, (double)n)));
      }
      if (explore && !observe_only) {
        const uint32_t sub_seed = pcg_bounded(rng, 2147483646u);
        const uint32_t nvalid = (uint32_t)__builtin_popcount(amask);
        // Discrete.sample(mask) == valid[default_rng(sub_seed).integers(0, nvalid)]: Lemire on the
        // sub-generator's first 32-bit output (tabulated, see k_seedseq_table); the rare rejected
        // draw, and a device without the table, run the sub-generator itself
        uint32_t pick = 0;
        bool slow = nvalid > 1u;
        if (slow && m.seedseq32) {
          const uint64_t mm = (uint64_t)(xp::kNoSeedSeqLoad ? (uint32_t)mix64(U(sub_seed)) : LDC(m.seedseq32, (size_t)U(sub_seed))) * nvalid;
          // Lemire rejects when the low word is below (2^32 - n) % n < n: test against n first
          slow = (uint32_t)mm < nvalid && (uint32_t)mm < (0u - nvalid) % nvalid;
          pick = (uint32_t)(mm >> 32);
        }
        if (slow) {
          Pcg64 sub;
          pcg_from_seedseq(sub_seed, sub);
          pick = pcg_bounded(sub, nvalid - 1u);
        }
        // the pick-th allowed action: lane a holds action a, one ballot of its rank among the allowed
        const uint32_t la16 = (uint32_t)lid() & 15u;
        const bool is_pick = lid() < 16 && ((amask >> la16) & 1u) &&
                             (uint32_t)__builtin_popcount(amask & ((1u << la16) - 1u)) == pick;
        // (G = 8: lanes 0-7 hold actions 0-7; a 9-action switch's STOP, action 8, is the pick no lane makes)
        const uint64_t pb = BAL(is_pick);
        action = (G < 16 && pb == 0ull) ? 8 : ctz64(pb);
      }
      if (!observe_only) {  // uniform values, written by every lane
        lrng[0] = rng.shi;
        lrng[1] = rng.slo;
        lrng[4] = ((uint64_t)rng.has << 32) | rng.buf;
      }
    }
    if constexpr (EPS_PF) lrng[5] |= 1ull << sw;  // (uniform) this switch's count moves in post
    if constexpr (PART) {
      if (observe_only) {
        emit_req(sw, slot, state, amask, explore);
        flags |= F_REQ;
        return true;
      }
      flags &= ~F_REQ;
    }
    SFL_LAP(6);
    d.q_pend = Ud(q_pend_v);
    // np.argmax over the full row (first maximum), max(row), and the first allowed maximum
    // (distr_q.py:449-490), over the compact columns held by lanes 0..w-1 (column order = action
    // order, so the lowest lane among equal values is the first index): column c holds full-row
    // action a(c); every other action of the full row is default_q, the first of them at mind
    double mx;
    int best, arg;
    if (PART && !loc) {
      // the owner's reply: max over the full row, and the masked argmax (-1 for an exploratory request)
      best = arg = U((int)rep_a);
      mx = __longlong_as_double(((long long)U(rep_hi) << 32) | (long long)U(rep_lo));
    } else if (row_hit) {
      mx = Ud(pf_mx);
      const uint32_t ba = U(pfd23[0]) >> 16;
      best = (int)(ba & 0xFFu);
      arg = (int)((ba >> 8) & 0xFFu);
    } else {
      const uint32_t rd = swr.row_desc(slot);
      const int mind = (int)((rd >> 16) & 15u);
      const uint32_t a_c = (rd >> (4u * ((uint32_t)lid() & 3u))) & 15u;
      const double NEG = -__builtin_huge_val();
      const double vq = colv ? v_c : NEG;
      const double vm = (colv && ((amask >> a_c) & 1u)) ? v_c : NEG;
      const double mq4 = quad_max(vq), am4 = quad_max(vm);
      const double mqu = Ud(mq4), amu = Ud(am4);
      const int cb = ctz64(BAL(colv && v_c == mqu));
      const int ca = ctz64(BAL(vm == amu && colv && ((amask >> a_c) & 1u)));
      mx = __longlong_as_double(((long long)RL((uint32_t)(__double_as_longlong(v_c) >> 32), cb) << 32) |
                                (long long)RL((uint32_t)__double_as_longlong(v_c), cb));
      best = (int)((rd >> (4 * cb)) & 15u);
      if (mind != 15 && (m.default_q > mx || (m.default_q == mx && mind < best))) {
        mx = m.default_q;
        best = mind;
      }
      arg = (int)((rd >> (4 * ca)) & 15u);
    }
    d.mq = mx;
    d.row_cur = (!PART || loc) ? rowb_of(4 * sw + slot, prr) + state : 0u;
    d.touch_cur = !explore;  // the key-set insert is done by post (one lane-0 region)
    if (!explore) action = ((amask >> best) & 1u) ? best : arg;
    // the exploratory pick comes out of the vector-ALU generator: declare the action wave-uniform,
    // so the apply below branches on the scalar unit instead of through exec-mask regions
    action = U(action);
    if (action < 0 || action >= na) lerr |= E_BAD_ACTION;
    SFL_LAP(7);
    if constexpr (TM) {  // action selected (distr_q.py:312-319)
      if (tm_on) tm_eg_t = (uint64_t)__builtin_amdgcn_s_memtime();
    }
    SFL_PACC(1, t_eg);
    SFL_PT(t_ap);
    // _apply_action
    const int stop = na - 1;
    bool moving = false;
    uint32_t turn = A_FWD;
    int in_p = pin, out_p = pin;
    if (action != stop && (pin >> 2) == sw) {
      const int src = swr.src(action);
      if (src == slot) {
        moving = true;
        turn = swr.turn(action);
        in_p = 4 * sw + src;
        out_p = 4 * sw + swr.dst(action);
      }
    }
    int next_sw = sw, target = -1;
    bool blk_moving = false;
    if (moving) {
      // transition_train / transition_semaphore (rail_network.py:246-278, 303-416)
      const u4 rc = port_tr_rec(out_p);  // one scalar load (LDS read for G < 64) for the whole recipe
      target = (int)(int16_t)(rc[0] & 0xFFFFu);
      if (tb_state(b) != S_MALF) {
        // free the train's records on the ports of its current and previous switch
        const int x1 = pin >> 2;
        const int x2 = pprev != (int)PORT_NONE ? (pprev >> 2) : -1;
        // lanes 0-3: the ports of switch x1, lanes 4-7: those of x2
        const int xs = lid() < 4 ? x1 : x2;
        const bool act = lid() < 8 && xs >= 0;
        const int pc = act ? 4 * xs + (lid() & 3) : 0;
        const uint32_t r = lsem[pc];
        if (act && r_present(r) && r_owner(r) == (uint32_t)h) lsem[pc] = 0u;
      }
      // transition_semaphore's record updates on the out, target, unique-onward and far ports,
      // evaluated on register copies of the four records (one LDS round trip; writes to a port
      // that appears in several roles update every copy) and written back once
      const int32_t d_ot = (int32_t)(int16_t)(rc[1] >> 16);
      const int u = (int)(int16_t)(rc[0] >> 16);
      const bool hu = u >= 0;
      const int far = (int)(int16_t)(rc[1] & 0xFFFFu);
      const int32_t len_u = (int32_t)rc[2];
      SemQuad q4(lsem, out_p, target, u, far);
      q4.put(out_p, put_keep_f(h, 0, 3, 0));
      q4.put(target, put_keep_f(h, 1, d_ot + 1, 1));
      if (hu) {
        if (u != in_p && u != out_p && u != target) q4.put(u, put_replace_f(h, 0, d_ot + 1, 0));
        q4.put(u, put_replace_f(h, 0, d_ot, -1));
        if (far != in_p && far != out_p && far != u) q4.put(far, put_replace_f(h, 1, d_ot + len_u + 1, 1));
      }
      if (target != in_p && target != out_p) q4.put(target, put_replace_f(h, 0, d_ot + 1, 0));
      q4.store();
      // check_port_blocked(target, out_p) on the updated records (reward_func.py:62-70)
      blk_moving = (rec_blocks(q4.v[1], (uint32_t)h, malf, 0u) | rec_blocks(q4.v[0], (uint32_t)h, malf, 1u)) != 0u;
      SFL_LAP(8);
      tset(sdec, h, (sd & 0xFFFF0000u) | (uint32_t)in_p);
      tset(nprv, h, (uint32_t)target | ((uint32_t)out_p << 16));
      next_sw = target >> 2;
    }
    uint32_t p = trl(plan, h);
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
      all_blocked = U((uint32_t)blk_moving) != 0u;
    } else {
      // semaphores unchanged since the observation: no route from the in-port has a free out-port,
      // i.e. the action mask holds STOP only
      all_blocked = (amask & ((1u << (na - 1)) - 1u)) == 0u;
    }
    // reward_func.py:23-78: distance at the position projected along the non-STOP plan (staged
    // by prefetch for the STOP plan and for each final rail action of a route)
    const uint32_t tq = turn & 3u;
    const uint32_t dw = U(moving ? (tq == 3 ? pfd23[0] : pfd01[1]) : pfd01[0]);
    const int32_t dproj = moving ? (tq == 0 ? 0 : tq == 2 ? d16_hi(dw) : d16_lo(dw)) : d16_hi(dw);
    const int32_t cur = now - la + dist_staged(dproj);
    const int32_t diff = trl(delay, h) - cur;
    d.r_new = (pl_front(p) == A_STOP && !all_blocked) ? diff - 1300 : diff;
    tset(delay, h, cur);
    d.sw = sw;
    d.h = h;
    d.slot = slot;
    d.state = state;
    d.action = action;
    d.j = (action == stop) ? (w - 1) : swr.j(action);
    d.reward = reward;
    d.next_sw = next_sw;
    d.abytes = 220u + 48u * (uint32_t)np + 8u * (uint32_t)na;  // SURVEY.md §8(d) bytes of this decision
    SFL_LAP(9);
    SFL_PACC(2, t_ap);
    return false;
  }

  // ---- graph-partitioned mode: messages to the owners (sfl_part.h records) ---------------------
  // the decision's row request (the row's owner answers max(row) and the masked argmax), staged in
  // the env's request slot; k_part_compact gives it its place in the destination segment
  __device__ __forceinline__ void emit_req(int sw, int slot, uint32_t state, uint32_t amask, bool explore) {
    req_dst_v = U(ld(P->owner, (size_t)sw));
    if (lid() != 0) return;
    u4 r;
    r[0] = P->env_base + e;
    r[1] = (uint32_t)(4 * sw + slot) | (amask << 16);
    r[2] = state;
    r[3] = explore ? 1u : 0u;
    static_assert(sizeof(PartReq) == sizeof(u4), "request record");
    st((u4*)P->req_st, (size_t)e, r);
  }
  // one update record (kind 0: q <- (1 - lr) q + lr target, and the key-set insert; kind 1: the
  // key-set insert only) to the owner of switch sw, applied in stage order, staged in slot k of the
  // env's update slots (k from the wave-uniform count n_upd)
  __device__ __forceinline__ void emit_upd(uint32_t k, int sw, int slot, uint32_t state, int j, uint32_t kind, double lr,
                                           double target, int stage) {
    if (k >= P->upd_env || stage > 254) {  // (the record's stage field is 8 bits)
      lerr |= E_MSG_OVF;
      return;
    }
    u4 a, b;
    a[0] = P->env_base + e;
    a[1] = (uint32_t)(4 * sw + slot) | ((uint32_t)j << 16) | ((uint32_t)stage << 24);
    a[2] = state;
    a[3] = kind;
    b[0] = (uint32_t)__double_as_longlong(lr);
    b[1] = (uint32_t)(__double_as_longlong(lr) >> 32);
    b[2] = (uint32_t)__double_as_longlong(target);
    b[3] = (uint32_t)(__double_as_longlong(target) >> 32);
    static_assert(sizeof(PartUpd) == 2 * sizeof(u4), "update record");
    u4* u = (u4*)(P->upd_st + (size_t)e * P->upd_env + k);
    st(u, 0, a);
    st(u, 1, b);
  }

  // ---- post-step part of the learn loop (distr_q.py:322-362) -----------------------------------
  // The (switch, train) slot of the deciding switch is consumed and the successor slot gets
  // the new pending update and the reward the train will see there (AECEnv.last).
  __device__ __forceinline__ void post(const Dec& d, bool greedy) {
    if constexpr (PART) {
      post_part(d, greedy);
      return;
    }
    SFL_LAP0();
    if (greedy) {
      if (lid() == 0) {
        if (d.touch_cur) touch_row(d.row_cur);
        st(sbase(), slot_ix(d.next_sw, d.h), slot_make(PEND_NONE, d.r_new, epoch));
      }
      return;
    }
    const bool hp = d.qoff_pend != PF_NONE;
    int ps = 0;
    double nv = 0.0;
    if (hp) {
      const uint32_t pend = slot_pend(d.slotword, epoch);
      ps = (int)(pend & 0xFFFu);
      const double lr = lr_of(cget(ps));
      const double r = (double)d.reward;
      if (d.sw != ps) {
        const double a1 = (1.0 - lr) * d.q_pend;
        const double b1 = lr * (r + m.gamma * d.mq);
        nv = a1 + b1;
      } else {
        const double a1 = (1.0 - lr) * d.q_pend;
        const double b1 = lr * r;
        nv = a1 + b1;
      }
    }
    // every global write of the step from one lane-0 region
    // (xp::kNo*: timing-only experiment builds that drop one class of store, sfl_experiment.h)
    if (lid() == 0) {
      for (int rep = 0; rep < 2; ++rep) {  // (rep 1: the timing-only duplicate writes of sfl_experiment.h)
        if (rep == 1 && !(xp::kQStoreTwice || xp::kTouchTwice || xp::kSlotTwice)) break;
        if (rep == 1) asm volatile("" ::: "memory");
        if (hp) {
          if (!xp::kNoQStore && (rep == 0 || xp::kQStoreTwice)) st(qbase(), (size_t)d.qoff_pend, nv);
          if (!xp::kNoTouch && (rep == 0 || xp::kTouchTwice)) touch_row(d.row_pend);
        }
        if (!xp::kNoTouch && (rep == 0 || xp::kTouchTwice) && (d.touch_cur || (hp && d.sw != ps))) touch_row(d.row_cur);
        if (!xp::kNoSlot && (rep == 0 || xp::kSlotTwice)) {
          st(sbase(), slot_ix(d.sw, d.h), slot_make(PEND_NONE, slot_rew(d.slotword, epoch), epoch));
          st(sbase(), slot_ix(d.next_sw, d.h),
             slot_make(pend_make((uint32_t)d.sw, (uint32_t)d.slot, d.state, (uint32_t)d.j), d.r_new, epoch));
        }
      }
    }
    if (hp) pf_written(d.qoff_pend);
    // destination bonus for newly arrived trains (distr_q.py:344-356); lanes take switches.
    // Distinct slots of one train never hold the same Q cell (same cell => same action =>
    // same successor switch => same slot), so the lanes' updates are independent.
    Mask fresh = arr_mask & ~fl_mask;
    fl_mask |= fresh;
    if (many(fresh)) pf_ok = false;  // bonus writes: stage the rest of the batch again
    while (many(fresh)) {
      const int tr = mctz(fresh);
      mclear_low(fresh);
      for (int base = 0; base < m.S; base += G) {
        const int sw2 = base + lid();
        const bool valid = sw2 < m.S;
        const uint64_t slw = valid ? ld(sbase(), slot_ix(sw2, tr)) : 0ull;
        const uint32_t pe = valid ? slot_pend(slw, epoch) : PEND_NONE;
        const int ps = pe == PEND_NONE ? 0 : (int)(pe & 0xFFFu);
        const uint32_t n = cget_var(ps);  // all lanes active: a bpermute reads 0 from inactive lanes
        if (pe == PEND_NONE) continue;
        const int pslot = (int)((pe >> 12) & 3u);
        const uint32_t pstate = (pe >> 14) & 0x3FFFu;
        const int pj = (int)((pe >> 28) & 3u);
        const double lr = lr_of_var(n);
        const u4 pr = port_v(4 * ps + pslot);
        double* qp = qbase() + pr[3] + (size_t)pstate * (pr[1] >> 16) + pj;
        const double a1 = (1.0 - lr) * ld(qp, 0);
        const double b1 = lr * (1000.0 + m.gamma * 0.0);
        st(qp, 0, a1 + b1);
        touch_row(pr[2] + pstate);
        st(sbase(), slot_ix(sw2, tr), slot_make(PEND_NONE, slot_rew(slw, epoch), epoch));
      }
    }
    cset(d.sw, cget(d.sw) + 1u);
    SFL_LAP(10);
  }
  // PART: post with the Q operations on other ranks' rows as update records to their owners (env_post
  // with MsgQ in sfl_part.h; stage stg = the pending update and key-set insert, then one stage per
  // arrived train's bonus -- only stages that carry records take a number), those on this rank's
  // rows applied here as in post(); a
  // greedy decision's key-set insert on a remote row was done by its owner when it answered
  __device__ __forceinline__ void post_part(const Dec& d, bool greedy) {
    const bool loc_cur = local_sw(d.sw);
    if (greedy) {
      if (lid() == 0) {
        if (loc_cur && d.touch_cur) touch_row(d.row_cur);
        st(sbase(), slot_ix(d.next_sw, d.h), slot_make(PEND_NONE, d.r_new, epoch));
      }
      return;
    }
    const uint32_t pend = slot_pend(d.slotword, epoch);
    const bool hp = pend != PEND_NONE;
    const int ps = hp ? (int)(pend & 0xFFFu) : 0;
    const bool loc_p = local_sw(ps);
    const double lr = lr_of(cget(ps));
    const double r = (double)d.reward;
    const double target = d.sw != ps ? r + m.gamma * d.mq : r;
    // record slots taken outside the lane-0 region, so the count stays wave-uniform
    const bool upd_rec = hp && !loc_p;
    const bool touch_rec = hp && d.sw != ps && !d.touch_cur && !loc_cur;
    const uint32_t k0 = n_upd;
    n_upd += (upd_rec ? 1u : 0u) + (touch_rec ? 1u : 0u);
    if (lid() == 0) {
      if (hp) {
        if (loc_p) {
          const double a1 = (1.0 - lr) * d.q_pend;
          const double b1 = lr * target;
          st(qbase(), (size_t)d.qoff_pend, a1 + b1);
          touch_row(d.row_pend);
        } else {
          emit_upd(k0, ps, (int)((pend >> 12) & 3u), (pend >> 14) & 0x3FFFu, (int)((pend >> 28) & 3u), 0u, lr, target,
                   (int)stg);
        }
      }
      if (loc_cur) {
        if (d.touch_cur || (hp && d.sw != ps)) touch_row(d.row_cur);
      } else if (touch_rec) {
        emit_upd(k0 + (upd_rec ? 1u : 0u), d.sw, d.slot, d.state, 0, 1u, 0.0, 0.0, (int)stg);
      }
      st(sbase(), slot_ix(d.sw, d.h), slot_make(PEND_NONE, slot_rew(d.slotword, epoch), epoch));
      st(sbase(), slot_ix(d.next_sw, d.h),
         slot_make(pend_make((uint32_t)d.sw, (uint32_t)d.slot, d.state, (uint32_t)d.j), d.r_new, epoch));
    }
    Mask fresh = arr_mask & ~fl_mask;
    fl_mask |= fresh;
    if (many(fresh)) pf_ok = false;
    // stages are numbered per launch and only those that carry records take a number: a launch
    // that decides on local rows only (one rank: every row) emits none, however many posts it runs
    uint32_t stage = stg + ((upd_rec || touch_rec) ? 1u : 0u);
    while (many(fresh)) {
      const int tr = mctz(fresh);
      mclear_low(fresh);
      const uint32_t n_before = n_upd;
      for (int base = 0; base < m.S; base += G) {
        const int sw2 = base + lid();
        const bool valid = sw2 < m.S;
        const uint64_t slw = valid ? ld(sbase(), slot_ix(sw2, tr)) : 0ull;
        const uint32_t pe = valid ? slot_pend(slw, epoch) : PEND_NONE;
        const int ps2 = pe == PEND_NONE ? 0 : (int)(pe & 0xFFFu);
        const uint32_t n = cget_var(ps2);  // all lanes active: a bpermute reads 0 from inactive lanes
        const bool loc2 = local_sw_var(ps2);
        // this pass's records: slots in lane order after the ones taken so far
        const uint64_t bm = (uint64_t)BAL(pe != PEND_NONE && !loc2);
        const uint32_t k = n_upd + (uint32_t)__builtin_popcountll(bm & ((1ull << lid()) - 1ull));
        n_upd += (uint32_t)__builtin_popcountll(bm);
        if (pe == PEND_NONE) continue;
        const int pslot = (int)((pe >> 12) & 3u);
        const uint32_t pstate = (pe >> 14) & 0x3FFFu;
        const int pj = (int)((pe >> 28) & 3u);
        if (loc2) {
          const int g = 4 * ps2 + pslot;
          const u4 pr = port_v(g);
          double* qp = qbase() + (uint32_t)ld(P->q_off_own, (size_t)g) + (size_t)pstate * (pr[1] >> 16) + pj;
          const double lr2 = lr_of_var(n);
          const double a1 = (1.0 - lr2) * ld(qp, 0);
          const double b1 = lr2 * (1000.0 + m.gamma * 0.0);
          st(qp, 0, a1 + b1);
          touch_row(ld(P->row_own, (size_t)g) + pstate);
        } else {
          emit_upd(k, ps2, pslot, pstate, pj, 0u, lr_of_var(n), 1000.0 + m.gamma * 0.0, (int)stage);
        }
        st(sbase(), slot_ix(sw2, tr), slot_make(PEND_NONE, slot_rew(slw, epoch), epoch));
      }
      if (n_upd != n_before) ++stage;
    }
    stg = stage;
    cset(d.sw, cget(d.sw) + 1u);
  }

  // order-independent checksum of the semaphore table (trace/debug only)
  __device__ __forceinline__ uint64_t sem_checksum() const {
    uint64_t c0 = 0;
#pragma unroll
    for (int k = 0; k < PPL; ++k) {
      const int p = k * G + lane;
      if (p < m.NP && r_present(sem(k))) c0 += mix64(((uint64_t)p << 42) ^ r_to64(sem(k)));
    }
    for (int off = 1; off < G; off <<= 1) c0 += (uint64_t)__shfl_xor((long long)c0, off, 64);
    return c0;
  }
};

// driver: one env per wavefront until its episode target / decision budget (env_run in sfl_core.h)
// TRACE: the per-decision trace of one env (parity tests only) is compiled into a separate
// instantiation, so the production kernel does not carry its registers
// PART: one round of the graph-partitioned mode (P = its tables and this round's message
// buffers): each env applies the reply to its open request, runs to its next decision and stops
// after emitting that decision's request; c.dec_budget counts decisions since sfl_part_begin
// phase-timer buckets (SflCtl::phase_cyc, include/sfl.h sfl_get_phase_cycles)
enum { TM_TICK = 0, TM_OBS = 1, TM_EG = 2, TM_APPLY = 3, TM_POST = 4, TM_RESET = 5, TM_OTHER = 6, TM_TOTAL = 7 };
// the TIMED kernels sample one wavefront in TM_SAMPLE blocks
constexpr uint32_t TM_SAMPLE = 8;
struct PhaseTimer {
  bool on;
  uint64_t t, acc[8];
  __device__ __forceinline__ void start(bool on_) {
    on = on_;
    t = on ? (uint64_t)__builtin_amdgcn_s_memtime() : 0ull;
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = 0ull;
    acc[TM_TOTAL] = t;
  }
  __device__ __forceinline__ void lap(int k) {
    if (on) {
      const uint64_t n = (uint64_t)__builtin_amdgcn_s_memtime();
      acc[k] += n - t;
      t = n;
    }
  }
  // the decide block split at decide's stamps, read from lane `lane` (a lane that decided; -1: none did)
  template <class V>
  __device__ __forceinline__ void decide_done(const V& v, int lane) {
    if (on) {
      const uint64_t n = (uint64_t)__builtin_amdgcn_s_memtime();
      if (lane >= 0) {
        const uint64_t o = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(v.tm_obs_t >> 32), lane) << 32) |
                           (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v.tm_obs_t, lane);
        const uint64_t g = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(v.tm_eg_t >> 32), lane) << 32) |
                           (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v.tm_eg_t, lane);
        acc[TM_OBS] += o - t;
        acc[TM_EG] += g - o;
        acc[TM_APPLY] += n - g;
      } else {
        acc[TM_OTHER] += n - t;
      }
      t = n;
    }
  }
  __device__ __forceinline__ void flush(const SflCtl& c) {
    if (!on) return;
    const uint64_t end = (uint64_t)__builtin_amdgcn_s_memtime();
    acc[TM_TOTAL] = end - acc[TM_TOTAL];
    uint64_t known = 0;
#pragma unroll
    for (int k = 0; k < 6; ++k) known += acc[k];
    acc[TM_OTHER] = acc[TM_TOTAL] > known ? acc[TM_TOTAL] - known : 0ull;
    if (__lane_id() == 0)
#pragma unroll
      for (int k = 0; k < 8; ++k) atomicAdd((unsigned long long*)&c.phase_cyc[k], (unsigned long long)acc[k]);
  }
};

template <int PPL, int SPL, int TW, bool TRACE, bool PART = false, bool TIMED = false>
__device__ void run(const SflMap& m, const SflState& s, const SflCtl& c, const SflPart* P = nullptr) {
  using V = WEnv<PPL, SPL, TW, PART>;
  // semaphores, counters, prefetch records, rng, timetable (PART: one record, timetable from the map)
  // (PART: the launch's initial records / counters in place of the timetable copy)
  constexpr int LDS_WORDS =
      64 * (PPL + SPL) + V::PF_SLOTS * V::PFW + 12 + (PART ? 64 * PPL + 2 * SPL + 6 * 64 * V::TPL : TW * 8);
  const int lane = (int)__lane_id();
  const uint32_t e = uni((uint32_t)((blockIdx.x * blockDim.x + threadIdx.x) >> 6));
  if (e >= s.E) return;
  constexpr int WPB = TW > 64 ? 1 : SFL_WAVE_BLOCK / 64;  // waves (envs) per block (sfl.hip launches)
  __shared__ uint32_t lds[WPB * LDS_WORDS];
  V v(m, s, e, lane, lds + (threadIdx.x >> 6) * LDS_WORDS, P);
  if constexpr (PART) {
    v.lsem0 = lds + (threadIdx.x >> 6) * LDS_WORDS + 64 * (PPL + SPL) + V::PF_SLOTS * V::PFW + 12;
    v.ldirty = v.lsem0 + 64 * PPL;
    v.ltr0 = v.ldirty + 2 * SPL;
  }
  PhaseTimer tm;
  if constexpr (TIMED) tm.start(c.phase_cyc != nullptr && blockIdx.x % TM_SAMPLE == 0u);
  v.load();
  if constexpr (PART)
    if (v.flags & F_DEFER) return;  // its records did not fit the last round's segments: it sits this one out
  if constexpr (xp::kLoadTwice) v.load();  // experiment build: the marginal cost of the state load
  const int64_t dec_base = PART ? (int64_t)v.ebw64(EB_DEC_DONE) : 0;
  int32_t phase = PART ? (int32_t)v.ebw(EB_PHASE) : uni(ld(s.phase, e));
  int32_t ep_t = PART ? (int32_t)v.ebw(EB_EP_T) : uni(ld(s.ep_t, e));
  int32_t n_test = PART ? (int32_t)v.ebw(EB_N_TEST) : uni(ld(s.n_test, e));
  uint32_t ticks = 0, abytes = 0;
  typename V::Dec d;
  d.sw = d.h = d.slot = d.action = d.j = d.reward = d.r_new = d.next_sw = 0;
  d.state = 0;
  d.slotword = 0;
  d.mq = d.q_pend = 0.0;
  d.qoff_pend = PF_NONE;
  d.row_pend = 0;
  d.row_cur = 0;
  d.touch_cur = false;
  d.abytes = 0;
  const bool test_mode = c.mode == 1;
  const int64_t max_steps = m.max_steps, dec_budget = c.dec_budget;
#ifdef SFL_PROFILE
  uint64_t prof[5] = {0, 0, 0, 0, 0};
  const uint64_t t_begin = (uint64_t)__builtin_amdgcn_s_memtime();
#endif
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
      SFL_PT(t0);
      if constexpr (TIMED) tm.lap(TM_OTHER);
      v.reset();
      if constexpr (TIMED) tm.lap(TM_RESET);
      SFL_PACC(0, t0);
      phase = PH_TICK;
    } else if (phase == PH_TICK) {
      abytes += 36u * (uint32_t)(m.T - mpopc(v.arr_mask));
      SFL_PT(t0);
      if constexpr (TIMED) tm.lap(TM_OTHER);
      v.tick();
      if constexpr (TIMED) tm.lap(TM_TICK);
      SFL_PACC(1, t0);
      ticks++;
      if (v.flags & F_TERM) phase = (v.flags & F_INFLIGHT) ? PH_POST : PH_END;
      else if (many(v.q_mask)) phase = (v.flags & F_INFLIGHT) ? PH_POST : PH_DECIDE;
    } else if (phase == PH_DECIDE || phase == PH_POST) {
      const bool greedy = (v.flags & F_GREEDY) != 0;
      // post step + loop bookkeeping of decision d; true: the launch's decision budget is spent
      auto finish = [&]() -> bool {
        SFL_PT(t0);
        if constexpr (TIMED) tm.lap(TM_OTHER);
        v.post(d, greedy);
        if constexpr (TIMED) tm.lap(TM_POST);
        SFL_PACC(3, t0);
        if (TRACE && c.trace && (int32_t)e == c.trace_env) {
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
        v.cum += d.reward;
        v.ep_dec += 1;
        v.n_dec += 1;
        v.step_ctr += 1;
        if (v.step_ctr > max_steps) v.flags |= F_TRUNC;
        phase = (v.flags & (F_TERM | F_TRUNC)) ? PH_END : PH_DECIDE;
        return dec_budget > 0 && dec_base + (int64_t)v.n_dec >= dec_budget;
      };
      // a batch of queued decisions: decide, and post each one while more are queued (the last
      // one is posted after the ticks that follow it, switch_env.py:418-421 / distr_q.py:322-343);
      // PH_POST enters at that deferred post
      bool stop = false, do_decide = phase == PH_DECIDE;
      while (true) {
        if (do_decide) {
          if (PART && !(v.flags & F_REQ) && dec_budget > 0 && dec_base + (int64_t)v.n_dec >= dec_budget) {
            stop = true;  // this part step's decisions are done: no new request
            break;
          }
          SFL_PT(t0);
          if constexpr (TIMED) {
            tm.lap(TM_OTHER);
            v.tm_on = tm.on;
          }
          const bool requested = v.template decide<TIMED>(d, greedy);
          if constexpr (TIMED) tm.decide_done(v, 0);
          SFL_PACC(2, t0);
          if (PART && requested) {
            stop = true;  // the round ends at the request (phase stays PH_DECIDE)
            break;
          }
          abytes += d.abytes;
          v.flags |= F_INFLIGHT;
          if (!many(v.q_mask)) {
            phase = PH_TICK;
            break;
          }
        }
        do_decide = true;
        stop = finish();
        if (stop || phase != PH_DECIDE) break;
      }
      if (stop) break;
    } else {  // PH_END
      const int arrived = mpopc(v.arr_mask);
      const size_t cap = (size_t)(c.stats_cap > 0 ? c.stats_cap : 1);
      const bool greedy = (v.flags & F_GREEDY) != 0;
      if (c.st_cum && c.stats_cap > 0 && (!greedy || test_mode)) {
        const int32_t idx = (greedy && test_mode) ? n_test : ep_t;
        const size_t row = (size_t)(idx - c.stats_base) % cap;
        if (lane == 0) {
          st(c.st_cum, row * s.E + e, (double)v.cum);
          st(c.st_arrived, row * s.E + e, (int32_t)arrived);
          st(c.st_mf, row * s.E + e, v.n_mf);
          st(c.st_dec, row * s.E + e, v.ep_dec);
          st(c.st_ticks, row * s.E + e, v.ep_ticks);
        }
#pragma unroll
        for (int k = 0; k < V::TPL; ++k)
          if (v.mine[k]) st(c.st_delays, (row * m.T + lane + V::kG * k) * s.E + e, v.delay[k]);
      }
      if (greedy && !test_mode && c.sx_cum && c.stats_cap > 0 && lane == 0) {
        const size_t row = (size_t)(ep_t - c.stats_base) % cap;
        st(c.sx_cum, row * s.E + e, (double)v.cum);
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
  const uint32_t err_out = v.store(phase);
  if constexpr (xp::kStoreTwice) v.store(phase);  // experiment build: the marginal cost of the state store
  if constexpr (PART)
    v.store_eblk(phase, err_out, ep_t, n_test, dec_base + (int64_t)v.n_dec, v.req_dst_v,
                 v.n_upd < P->upd_env ? v.n_upd : P->upd_env, (uint64_t)v.n_dec, (uint64_t)ticks, (uint64_t)abytes);
  if constexpr (TIMED) tm.flush(c);
#ifdef SFL_PROFILE
  prof[4] = (uint64_t)__builtin_amdgcn_s_memtime() - t_begin;
  if (lane == 0) {
    for (int k = 0; k < 5; ++k) atomicAdd(&g_prof[k], (unsigned long long)prof[k]);
    for (int k = 0; k < 9; ++k) atomicAdd(&g_prof[5 + k], (unsigned long long)v.prof[k]);
    for (int k = 0; k < 16; ++k) atomicAdd(&g_prof[16 + k], (unsigned long long)v.lap[k]);
  }
#endif
  if (lane == 0 && !PART) {
    st(s.ep_t, e, ep_t);
    st(s.n_test, e, n_test);
    if (c.launch_dec) st(c.launch_dec, e, (uint64_t)v.n_dec);
    if (c.launch_ticks) st(c.launch_ticks, e, (uint64_t)ticks);
    if (c.launch_bytes) st(c.launch_bytes, e, (uint64_t)abytes);
  }
}

// driver for G < 64 (several envs per wavefront, one per lane group): the same per-env sequence
// as run() -- decide, post, decide, ..., the last decision of a batch posted after the ticks that
// follow it -- as a flat loop in which each iteration advances every group by at most one tick,
// one post step and one decision.  The groups of a wave diverge (one ticks while another decides);
// a batch loop as in run() would hold every group until the longest batch of the wave is done.
template <int PPL, int SPL, int TW, bool TRACE, int G, bool TIMED = false, bool LM = false>
__device__ void run_groups(const SflMap& m, const SflState& s, const SflCtl& c) {
  using V = WEnv<PPL, SPL, TW, false, G, LM>;
  // per env: semaphores, counters, prefetch records, rng; per block: the timetable rows and the
  // per-switch / per-port map records (the groups of a wave read different switches' records: LDS
  // reads instead of vector loads)
  constexpr int LDS_WORDS = (G * (PPL + SPL) + V::PF_SLOTS * V::PFW + 12 + 3) / 4 * 4;
  constexpr int EPB = SFL_GROUP_BLOCK / G;  // envs per block (sfl.hip launches)
  constexpr int SWX = G * SPL, NPX = G * PPL;  // switches / ports the shape holds
  constexpr int O_TT = EPB * LDS_WORDS, O_SW = O_TT + TW * 8, O_PP = O_SW + SWX * V::SW_LDS, O_PT = O_PP + NPX * 4;
  // LM: the move table and the distance map (int16 pairs) after the map records, within 64,512 bytes
  // (sfl_engine.h kLmBytes: two such blocks fill the CU's LDS)
  constexpr int O_LM = O_PT + NPX * 4, LM_WORDS = LM ? 16128 : 0;
  __shared__ __attribute__((aligned(16))) uint32_t lds[O_LM + LM_WORDS];
  for (int i = (int)threadIdx.x; i < m.S * V::SW_LDS; i += (int)blockDim.x)
    lds[O_SW + i] = m.sw_pack[(i / V::SW_LDS) * 16 + i % V::SW_LDS];
  for (int i = (int)threadIdx.x; i < m.NP * 4; i += (int)blockDim.x) {
    lds[O_PP + i] = m.port_pack[i];
    lds[O_PT + i] = m.port_tr[i];
  }
  const int lm_mv = LM ? m.HW * 16 : 0;  // move-table words
  if constexpr (LM) {
    const int nd = m.K * m.HW * 4;  // distance entries
    for (int i = (int)threadIdx.x; i < lm_mv; i += (int)blockDim.x) lds[O_LM + i] = m.move_tab[i];
    for (int j = (int)threadIdx.x; 2 * j < nd; j += (int)blockDim.x) {
      const uint32_t lo = d16(m.dist[2 * j]), hi = 2 * j + 1 < nd ? d16(m.dist[2 * j + 1]) : 0u;
      lds[O_LM + lm_mv + j] = lo | (hi << 16);
    }
  }
  __syncthreads();
  const uint32_t e = (uint32_t)((blockIdx.x * blockDim.x + threadIdx.x) / G);
  if (e >= s.E) return;
  V v(m, s, e, (int)__lane_id(), lds + (threadIdx.x / G) * LDS_WORDS, nullptr, (int32_t*)(lds + O_TT));
  v.tsw = lds + O_SW;
  v.tpp = lds + O_PP;
  v.tpt = lds + O_PT;
  if constexpr (LM) {
    v.lmv = lds + O_LM;
    v.ldist = lds + O_LM + lm_mv;
  }
  PhaseTimer tm;
  if constexpr (TIMED) tm.start(c.phase_cyc != nullptr && blockIdx.x % TM_SAMPLE == 0u && threadIdx.x < 64u);
  v.load();
  int32_t phase = ld(s.phase, e);
  int32_t ep_t = ld(s.ep_t, e), n_test = ld(s.n_test, e);
  uint32_t ticks = 0, abytes = 0;
  typename V::Dec d;
  d.sw = d.h = d.slot = d.action = d.j = d.reward = d.r_new = d.next_sw = 0;
  d.state = 0;
  d.slotword = 0;
  d.mq = d.q_pend = 0.0;
  d.qoff_pend = PF_NONE;
  d.row_pend = 0;
  d.row_cur = 0;
  d.touch_cur = false;
  d.abytes = 0;
  const bool test_mode = c.mode == 1;
  // 32-bit bounds (step_ctr and n_dec are 32-bit counters): held as two 64-bit values across the
  // loop they were spilled, and the decision count reloaded from scratch every post (c3: 1,356 M ->
  // 1,404 M agent-env-steps/s)
  const int32_t max_steps = m.max_steps < 0x7FFFFFFF ? (int32_t)m.max_steps : 0x7FFFFFFF;
  const uint32_t dec_budget = c.dec_budget > 0 ? (c.dec_budget < 0xFFFFFFFFll ? (uint32_t)c.dec_budget : 0xFFFFFFFFu) : 0xFFFFFFFFu;
#ifdef SFL_PROFILE
  // group activity of the flat loop (per wave, lane 0): iterations, and per iteration the groups
  // that tick / post / decide, and the iterations with any tick
  uint64_t gs[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // + wall cycles of the tick / post / decide blocks
  uint64_t tp0 = 0;
#endif
  while (true) {
#ifdef SFL_PROFILE
    {
      const uint64_t bt = __ballot(phase == PH_TICK), bp = __ballot(phase == PH_POST), bd = __ballot(phase == PH_DECIDE);
      gs[0] += 1;
      gs[1] += (uint64_t)__builtin_popcountll(bt) / G;
      gs[2] += (uint64_t)__builtin_popcountll(bp) / G;
      gs[3] += (uint64_t)__builtin_popcountll(bd) / G;
      gs[4] += (bp | bd) ? 0u : 1u;
    }
#endif
    if (phase == PH_RESET) {
      // learn: optional greedy round before episode t (distr_q.py:278-281)
      bool target = false;
      if (test_mode) {
        target = c.ep_target >= 0 && n_test >= c.ep_target;
        v.flags |= F_GREEDY;
      } else {
        target = c.ep_target >= 0 && ep_t >= c.ep_target;
        if (c.exploit_freq > 0 && (ep_t + 1) % c.exploit_freq == 0 && !(v.flags & F_EXPLOIT_DONE)) v.flags |= F_GREEDY;
        else v.flags &= ~F_GREEDY;
      }
      if (target) break;
      v.reset();
      phase = PH_TICK;
    }
    if constexpr (TIMED) tm.lap(TM_RESET);
    // the groups waiting for a tick start it once fewer than SFL_TICK_HOLD groups can still
    // decide: their ticks then run together, while the last deciding group (if any) runs its
    // batch alongside.  Measured at G = 16 (c3): hold while >= 2 decide 1,316 M, while >= 1
    // (ticks only when no group decides) 1,263 M, tick as soon as 3 / 2 groups wait 1,308 / 1,245 M,
    // never hold 14 % below the second.
    // Round 3: they also tick while every deciding group still has at least SFL_TICK_REMMIN decisions
    // left in its batch -- the ticking groups then decide alongside it instead of idling to its end.
    // scripts/sched_model.py replays c3 decision streams through this loop and prices the blocks an
    // iteration executes (profiles/r03_sched_model.txt): the rule is worth ~1.6 % there, measured
    // +0.65 % / +1.0 % on two boxes (profiles/r03_ab_sched.txt); aligning the groups perfectly would
    // give at most 28 %, and no rule tried gets more than the 1.6 %.
    const bool dec_ph = phase == PH_POST || phase == PH_DECIDE;
    const bool wave_decides = (int)__builtin_popcountll(__ballot(dec_ph)) >= SFL_TICK_HOLD * G &&
                              (SFL_TICK_REMMIN <= 0 || __ballot(dec_ph && mpopc(v.q_mask) < SFL_TICK_REMMIN) != 0ull);
#ifdef SFL_PROFILE
    tp0 = __builtin_amdgcn_s_memtime();
#endif
    if constexpr (TIMED) tm.lap(TM_OTHER);
    if (phase == PH_TICK && !wave_decides) {
      abytes += 36u * (uint32_t)(m.T - mpopc(v.arr_mask));
      v.tick();
      ticks++;
      if (v.flags & F_TERM) phase = (v.flags & F_INFLIGHT) ? PH_POST : PH_END;
      else if (many(v.q_mask)) phase = (v.flags & F_INFLIGHT) ? PH_POST : PH_DECIDE;
    }
    if constexpr (TIMED) tm.lap(TM_TICK);
#ifdef SFL_PROFILE
    {
      const uint64_t t1 = __builtin_amdgcn_s_memtime();
      gs[5] += t1 - tp0;
      tp0 = t1;
    }
#endif
    if (phase == PH_POST) {  // post step + loop bookkeeping of the decision in flight
      const bool greedy = (v.flags & F_GREEDY) != 0;
      v.post(d, greedy);
      if (TRACE && c.trace && (int32_t)e == c.trace_env) {
        const uint64_t cs = v.sem_checksum();
        if (v.lane == 0) {
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
      v.cum += d.reward;
      v.ep_dec += 1;
      v.n_dec += 1;
      v.step_ctr += 1;
      if (v.step_ctr > max_steps) v.flags |= F_TRUNC;
      phase = (v.flags & (F_TERM | F_TRUNC)) ? PH_END : PH_DECIDE;
      if (v.n_dec >= dec_budget) break;
    }
    if constexpr (TIMED) {
      tm.lap(TM_POST);
      v.tm_on = tm.on;
    }
    const uint64_t dec_lanes = TIMED ? (uint64_t)__ballot(phase == PH_DECIDE) : 0ull;
#ifdef SFL_PROFILE
    {
      const uint64_t t1 = __builtin_amdgcn_s_memtime();
      gs[6] += t1 - tp0;
      tp0 = t1;
    }
#endif
    if (phase == PH_DECIDE) {
      const bool greedy = (v.flags & F_GREEDY) != 0;
      v.template decide<TIMED>(d, greedy);
      abytes += d.abytes;
      v.flags |= F_INFLIGHT;
      phase = many(v.q_mask) ? PH_POST : PH_TICK;
    }
    if constexpr (TIMED) tm.decide_done(v, dec_lanes ? __builtin_ctzll(dec_lanes) : -1);
#ifdef SFL_PROFILE
    gs[7] += __builtin_amdgcn_s_memtime() - tp0;
#endif
    if (phase == PH_END) {
      const int arrived = mpopc(v.arr_mask);
      const size_t cap = (size_t)(c.stats_cap > 0 ? c.stats_cap : 1);
      const bool greedy = (v.flags & F_GREEDY) != 0;
      if (c.st_cum && c.stats_cap > 0 && (!greedy || test_mode)) {
        const int32_t idx = (greedy && test_mode) ? n_test : ep_t;
        const size_t row = (size_t)(idx - c.stats_base) % cap;
        if (v.lane == 0) {
          st(c.st_cum, row * s.E + e, (double)v.cum);
          st(c.st_arrived, row * s.E + e, (int32_t)arrived);
          st(c.st_mf, row * s.E + e, v.n_mf);
          st(c.st_dec, row * s.E + e, v.ep_dec);
          st(c.st_ticks, row * s.E + e, v.ep_ticks);
        }
#pragma unroll
        for (int k = 0; k < V::TPL; ++k)
          if (v.mine[k]) st(c.st_delays, (row * m.T + v.lane + G * k) * s.E + e, v.delay[k]);
      }
      if (greedy && !test_mode && c.sx_cum && c.stats_cap > 0 && v.lane == 0) {
        const size_t row = (size_t)(ep_t - c.stats_base) % cap;
        st(c.sx_cum, row * s.E + e, (double)v.cum);
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
  if constexpr (TIMED) tm.flush(c);
#ifdef SFL_PROFILE
  {  // the counts of the group that left the loop last (it saw every iteration of the wave)
    uint64_t mx = gs[0];
    for (int off = 32; off > 0; off >>= 1) mx = max(mx, (uint64_t)__shfl_xor((long long)mx, off, 64));
    const int src = __builtin_ctzll(__ballot(gs[0] == mx));
    uint64_t w[8];
    for (int k = 0; k < 8; ++k) w[k] = (uint64_t)__shfl((long long)gs[k], src, 64);
    if (__lane_id() == 0)
      for (int k = 0; k < 8; ++k) atomicAdd(&g_prof[k], (unsigned long long)w[k]);
    if (v.lane == 0) {  // per group: decide's counters (prefetches, row / pending hits, decisions) and laps
      for (int k = 3; k < 9; ++k) atomicAdd(&g_prof[5 + k], (unsigned long long)v.prof[k]);
      for (int k = 0; k < 16; ++k) atomicAdd(&g_prof[16 + k], (unsigned long long)v.lap[k]);
    }
  }
#endif
  if (v.lane == 0) {
    st(s.ep_t, e, ep_t);
    st(s.n_test, e, n_test);
    if (c.launch_dec) st(c.launch_dec, e, (uint64_t)v.n_dec);
    if (c.launch_ticks) st(c.launch_ticks, e, (uint64_t)ticks);
    if (c.launch_bytes) st(c.launch_bytes, e, (uint64_t)abytes);
  }
}

}  // namespace wave
}  // namespace sfl
