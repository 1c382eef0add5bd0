// MI355X (gfx950) build of the SwitchFL hot path: libsfl.so.
//
// One thread = one environment (sfl_core.h env_run).  A block of 256 threads is
// 4 waves; at 65,536 envs the grid is 256 blocks = one per CU, one wave per
// SIMD.  Envs are independent, so there is no inter-workgroup communication;
// the static map tables (a few hundred KB) are read by every CU and stay in
// L2 / the Infinity Cache.  Build: see build.py (hipcc --offload-arch=gfx950
// -O3 -ffp-contract=off: the Q update must be the reference's separate f64
// multiply/add, not a contracted FMA).
#include <hip/hip_runtime.h>

#include <stdio.h>

#include <algorithm>
#include <string>

#include "sfl_engine.h"
#include "sfl_kwave_g.h"
#include "sfl_wave.h"

SFL_KWAVE_V7(extern template)  // (defined in sfl_kwave_v7.hip)

#ifndef SFL_WAVE_OCC
#define SFL_WAVE_OCC 6  // waves per SIMD the one-env-per-wave kernel is register-budgeted for (6: 80 VGPRs)
#endif

namespace {

// The three parameter structs live in device memory and are passed by pointer: a by-value
// struct whose fields are reached through references would be copied to scratch per lane.
// NW = 32-bit words of the per-env train bitmasks kept in registers (T <= 32 * NW).
template <int NW>
__global__ void __launch_bounds__(256) k_run(const sfl::SflMap* __restrict__ m, const sfl::SflState* __restrict__ s,
                                             const sfl::SflCtl* __restrict__ c) {
  const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e < s->E) sfl::env_run<NW>(*m, *s, *c, e);
}

// external-action mode (sfl_env_step): the lane-per-env body without the learner, one decision per call
template <int NW>
__global__ void __launch_bounds__(256) k_run_ext(const sfl::SflMap* __restrict__ m, const sfl::SflState* __restrict__ s,
                                                 const sfl::SflCtl* __restrict__ c) {
  const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e < s->E) sfl::env_run_ext<NW>(*m, *s, *c, e);
}

// One env per wavefront (sfl_wave.h): 4 envs per block.  PPL / SPL = semaphore / counter
// registers per lane (sfl::kVariants).
// TIMED: the learn() / test() instantiation, with the sampled phase timers (sfl_wave.h PhaseTimer); the
// benchmark's sfl_step runs the untimed one
template <int PPL, int SPL, int TW, bool TRACE, bool TIMED = false>
__global__ void __launch_bounds__(SFL_WAVE_BLOCK) __attribute__((amdgpu_waves_per_eu(SFL_WAVE_OCC))) k_wave(const sfl::SflMap* __restrict__ m, const sfl::SflState* __restrict__ s,
                                              const sfl::SflCtl* __restrict__ c) {
  sfl::wave::run<PPL, SPL, TW, TRACE, false, TIMED>(*m, *s, *c);
}
// several envs per wavefront: k_wave_g (sfl_kwave_g.h).  Variant 7 -- the bench's c3 shape -- is compiled in
// its own translation unit (sfl_kwave_v7.hip) with another register-allocation-aware scheduler; this one
// only declares it (below the includes).
using sflk::k_wave_g;
// maps with 65-128 trains (two train slots per lane): one env per 64-thread block (its LDS is
// ~22 KB), register budget for the LDS-bound occupancy of 2 waves per SIMD
#ifndef SFL_WAVE2_OCC
#define SFL_WAVE2_OCC (SFL_PF_RING64 > 0 ? 4 : 2)  // waves per SIMD k_wave2 is register-budgeted for
#endif
template <int PPL, int SPL, int TW, bool TRACE, bool TIMED = false>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(SFL_WAVE2_OCC))) k_wave2(const sfl::SflMap* __restrict__ m,
                                                                                   const sfl::SflState* __restrict__ s,
                                                                                   const sfl::SflCtl* __restrict__ c) {
  sfl::wave::run<PPL, SPL, TW, TRACE, false, TIMED>(*m, *s, *c);
}

// graph-partitioned rounds, local env step on the one-env-per-wave body (sfl_wave.h, PART)
template <int PPL, int SPL, int TW>
__global__ void __launch_bounds__(SFL_WAVE_BLOCK) __attribute__((amdgpu_waves_per_eu(SFL_WAVE_OCC)))
k_wave_part(const sfl::SflMap* __restrict__ m, const sfl::SflState* __restrict__ s, const sfl::SflCtl* __restrict__ c,
            const sfl::SflPart* __restrict__ P) {
  sfl::wave::run<PPL, SPL, TW, false, true>(*m, *s, *c, P);
}
#ifndef SFL_WAVE2P_OCC
#define SFL_WAVE2P_OCC 3  // k_wave2_part: 5.2 KB of LDS per env, so the registers set its occupancy
#endif
template <int PPL, int SPL, int TW>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(SFL_WAVE2P_OCC)))
k_wave2_part(const sfl::SflMap* __restrict__ m, const sfl::SflState* __restrict__ s, const sfl::SflCtl* __restrict__ c,
             const sfl::SflPart* __restrict__ P) {
  sfl::wave::run<PPL, SPL, TW, false, true>(*m, *s, *c, P);
}

// graph-partitioned rounds (sfl_part.h): local env step (lane per env), compaction into the
// message segments, owner side (one thread per env group)
template <int NW>
__global__ void __launch_bounds__(256) k_part_local(const sfl::SflMap* __restrict__ m, const sfl::SflState* __restrict__ s,
                                                    const sfl::SflCtl* __restrict__ c, const sfl::SflPart* __restrict__ P) {
  const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e < s->E) sfl::env_run_part<NW>(*m, *s, *c, *P, e);
}
// after the local step: pack each env's staged request and update records into the destination
// segments, each env's records for one destination as a contiguous group (sfl_part.h env_groups: its
// updates in emission order, then its request) -- a block reserves its range per destination with one
// global atomic, the envs their groups in it with LDS atomics -- and add the launch totals of the envs
// that ran into P->sums.  A segment holds k_msg records this round: an env with a group that reaches past
// that place is deferred whole (F_DEFER; its places below the end get void records, its staged records go
// again next round and the local step skips it until then).  arrays: the lane-per-env body (its scalars in
// the SflState / SflPart arrays), else the wave kernels' per-env blocks (eblk).
#ifndef SFL_COMPACT_BLOCK
#define SFL_COMPACT_BLOCK 256  // threads (envs) per block of k_part_compact (64: -1.3 % on the 8-rank rehearsal)
#endif
__global__ void __launch_bounds__(SFL_COMPACT_BLOCK) k_part_compact(const sfl::SflPart* __restrict__ P, const sfl::SflState* __restrict__ s,
                                                     const sfl::SflCtl* __restrict__ c, int arrays) {
  constexpr int R = sfl::PART_GROUP_MAX;  // (register arrays: the loops over them are unrolled)
  constexpr int EARLY = 2;                // update records read with the env's words (most envs stage <= 2)
  constexpr int S_LDS = 1024;             // switches whose owners the block copies to LDS (more: read from the map)
  __shared__ uint32_t lmsg[256], bmsg[256];
  __shared__ int32_t lown[S_LDS];
  constexpr int NWV = SFL_COMPACT_BLOCK / 64;  // waves per block
  __shared__ unsigned long long lsum[NWV][4];
  __shared__ uint32_t lopen, ldefer;
  const int world = P->world, S = P->n_sw;
  for (int i = threadIdx.x; i < world; i += blockDim.x) lmsg[i] = 0u;
  if (threadIdx.x == 0) lopen = ldefer = 0u;
  for (int i = threadIdx.x; i < S && i < S_LDS; i += blockDim.x) lown[i] = P->owner[i];
  const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
  const bool valid = e < s->E;
  int rd = -1;
  uint32_t nu = 0, flags = 0, n = 0;
  int32_t dst[R];
  uint32_t pos[R], size[R], place[R];
  // the wave kernel's per-env words (its scalar block, sfl_part.h EB_*), or the lane kernel's arrays
  const uint32_t* eb = (valid && !arrays) ? P->eblk + (size_t)e * sfl::PART_EB : nullptr;
  auto eb64 = [&](int i) { return (unsigned long long)eb[i] | ((unsigned long long)eb[i + 1] << 32); };
  // the env's first update records and its request, read (clamped, unconditionally) with its words: their
  // copies into the segment below need no second read, and their destinations no dependent load
  const sfl::PartUpd* ust = P->upd_st + (size_t)(valid ? e : 0u) * P->upd_env;
  sfl::PartUpd early[EARLY];
#pragma unroll
  for (int r = 0; r < EARLY; ++r) early[r] = ust[r < (int)P->upd_env ? r : 0];
  const sfl::PartReq req = P->req_st[valid ? e : 0u];
  if (valid) {
    flags = eb ? eb[sfl::EB_EFLAGS] : s->eflags[e];
    rd = eb ? (int)eb[sfl::EB_REQ_DST] : P->req_dst[e];
    nu = eb ? eb[sfl::EB_UPD_N] : P->upd_n[e];
  }
  __syncthreads();  // (lown)
  if (valid) {
    auto own = [&](int sw) { return sw < S_LDS ? lown[sw] : P->owner[sw]; };
#pragma unroll
    for (int r = 0; r < R - 1; ++r)
      if ((uint32_t)r < nu) dst[r] = own((r < EARLY ? early[r].port : ust[r].port) >> 2);
    // each group takes its places in the block's range of its destination (LDS atomics)
    n = sfl::env_groups(rd, nu, dst, pos, size, place, [&](int d, uint32_t z) { return atomicAdd(&lmsg[d], z); });
  }
  // the launch totals of the envs that ran (a deferred env sat the local step out: its totals are the
  // last round's, already counted): wave sums, then one LDS slot per wave
  const bool ran = valid && !(flags & sfl::F_DEFER);
  unsigned long long a = !ran ? 0ull : eb ? eb64(sfl::EB_L_DEC) : c->launch_dec[e],
                     b = !ran ? 0ull : eb ? eb64(sfl::EB_L_TICKS) : c->launch_ticks[e],
                     d = !ran ? 0ull : eb ? eb64(sfl::EB_L_BYTES) : c->launch_bytes[e],
                     o = !valid ? 0ull : eb ? eb[sfl::EB_ERR] : s->err[e];
  for (int off = 32; off > 0; off >>= 1) {
    a += __shfl_xor(a, off, 64);
    b += __shfl_xor(b, off, 64);
    d += __shfl_xor(d, off, 64);
    o |= __shfl_xor(o, off, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    const int w = threadIdx.x >> 6;
    lsum[w][0] = a;
    lsum[w][1] = b;
    lsum[w][2] = d;
    lsum[w][3] = o;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < world; i += blockDim.x) bmsg[i] = lmsg[i] ? atomicAdd(P->cnt + i, lmsg[i]) : 0u;
  if (threadIdx.x < 4) {
    unsigned long long t = 0;
#pragma unroll
    for (int w = 0; w < NWV; ++w) t = threadIdx.x == 3 ? (t | lsum[w][3]) : t + lsum[w][threadIdx.x];
    if (threadIdx.x == 3) {
      if (t) atomicOr((unsigned long long*)&P->sums[3], t);
    } else if (t) {
      atomicAdd((unsigned long long*)&P->sums[threadIdx.x], t);
    }
  }
  __syncthreads();  // (bmsg: this block's reservations)
  // does every group of the env fit this round's segments?
  const uint32_t k = P->k_msg;
  bool fits = valid;
#pragma unroll
  for (int r = 0; r < R; ++r)
    if ((uint32_t)r < n && bmsg[dst[r]] + place[r] >= k) fits = false;
  const bool deferred = valid && !fits;
  const bool open = valid && (rd >= 0 || deferred);
  const uint32_t n_open = __popcll(__ballot(open)), n_def = __popcll(__ballot(deferred));
  if ((threadIdx.x & 63) == 0 && NWV > 1) {
    if (n_open) atomicAdd(&lopen, n_open);
    if (n_def) atomicAdd(&ldefer, n_def);
  }
  if (NWV > 1) __syncthreads();
  // the last block to get here writes the segment headers and hands the counts and totals to the
  // host copy (zeroing them for the next round): every block's reservations are done by then
  __shared__ bool last;
  if (threadIdx.x == 0) {
    const uint32_t no = NWV > 1 ? lopen : n_open, nd = NWV > 1 ? ldefer : n_def;
    if (no) atomicAdd(P->cnt + world + 1, no);
    if (nd) atomicAdd(P->cnt + world + 2, nd);
  }
  __threadfence();  // (a workgroup-scope fence here measured +0.8 % on the C5 round; not worth the ordering risk)
  if (threadIdx.x == 0) last = atomicAdd(P->blocks_done, 1u) == gridDim.x - 1u;
  __syncthreads();
  if (last) {
    __threadfence();
    uint32_t* co = (uint32_t*)(P->cnt_out + 4);
    for (int i = threadIdx.x; i < world; i += blockDim.x) {
      const uint32_t nm = atomicExch(P->cnt + i, 0u);
      P->msg_out[(size_t)i * (k + 1)].genv = nm < k ? nm : k;
      co[sfl::PART_C_MSG(world) + i] = nm;
      co[sfl::PART_C_PEAK(world) + i] = max(co[sfl::PART_C_PEAK(world) + i], nm);
    }
    if (threadIdx.x == 0) {
      const uint32_t no = atomicExch(P->cnt + world + 1, 0u), nd = atomicExch(P->cnt + world + 2, 0u);
      co[sfl::PART_C_OPEN(world)] = no;
      co[sfl::PART_C_DEFER(world)] = nd;
      co[sfl::PART_C_DEFER_SUM(world)] += nd;
      for (int i = 0; i < 3; ++i) P->cnt_out[i] += atomicExch((unsigned long long*)&P->sums[i], 0ull);
      P->cnt_out[3] |= atomicExch((unsigned long long*)&P->sums[3], 0ull);
      atomicExch(P->blocks_done, 0u);
    }
  }
  if (!valid) return;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    if ((uint32_t)r >= n) continue;
    const uint32_t at = bmsg[dst[r]] + place[r];
    sfl::PartMsg* x = P->msg_out + (size_t)dst[r] * (k + 1) + 1 + at;
    if (fits) {
      sfl::PartMsg y = (uint32_t)r < nu ? (r < EARLY ? early[r] : ust[r]) : sfl::msg_of_req(req);
      y.kind |= sfl::msg_tag(size[r], pos[r]);
      *x = y;
      if ((uint32_t)r == nu) P->req_ix[e] = (uint32_t)dst[r] * (k + 1) + 1u + at;  // (its reply lands there)
    } else if (at < k) {  // void records in the places below the segment's end
      x->genv = 0u;
      x->kind = sfl::MSG_VOID | sfl::msg_tag(1u, 0u);
    }
  }
  if ((bool)(flags & sfl::F_DEFER) != deferred) {
    if (eb) P->eblk[(size_t)e * sfl::PART_EB + sfl::EB_EFLAGS] = flags ^ sfl::F_DEFER;
    else s->eflags[e] = flags ^ sfl::F_DEFER;
  }
}
// the wave kernels' per-env scalar blocks (sfl_part.h EB_*) from the SflState arrays (dir 0: before the rounds)
// or back into them (dir 1: before the host reads them); one thread per env
__global__ void __launch_bounds__(256) k_part_eblk(const sfl::SflState s, uint32_t* eblk, int64_t* dec_done, int dir) {
  const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= s.E) return;
  uint32_t* b = eblk + (size_t)e * sfl::PART_EB;
  const size_t E = s.E;
  auto w32 = [&](int i, auto* a) {
    if (dir == 0) b[i] = (uint32_t)a[e];
    else a[e] = (std::remove_pointer_t<decltype(a)>)b[i];
  };
  auto w64 = [&](int i, auto* a, size_t at) {
    uint64_t x;
    if (dir == 0) {
      memcpy(&x, a + at, 8);
      b[i] = (uint32_t)x;
      b[i + 1] = (uint32_t)(x >> 32);
    } else {
      x = (uint64_t)b[i] | ((uint64_t)b[i + 1] << 32);
      memcpy(a + at, &x, 8);
    }
  };
  w32(sfl::EB_PHASE, s.phase);
  w32(sfl::EB_ELAPSED, s.elapsed);
  w32(sfl::EB_EFLAGS, s.eflags);
  w32(sfl::EB_EPOCH, s.epoch);
  w32(sfl::EB_ERR, s.err);
  w32(sfl::EB_EP_T, s.ep_t);
  w32(sfl::EB_N_TEST, s.n_test);
  w32(sfl::EB_N_MF, s.n_mf);
  w32(sfl::EB_EP_DEC, s.ep_dec);
  w32(sfl::EB_EP_TICKS, s.ep_ticks);
  w64(sfl::EB_STEP_CTR, s.step_ctr, e);
  w64(sfl::EB_DEC_TOTAL, s.dec_total, e);
  w64(sfl::EB_CUM, s.cum_reward, e);
  for (int i = 0; i < 5; ++i) w64(sfl::EB_RNG + 2 * i, s.rng, (size_t)i * E + e);
  for (int i = 0; i < 4 * sfl::MAXW; ++i) w32(sfl::EB_MASKS + i, s.masks + (size_t)i * E);
  w64(sfl::EB_DEC_DONE, dec_done, e);
  if (dir == 0) {
    b[sfl::EB_REQ_DST] = 0xFFFFFFFFu;
    for (int i = sfl::EB_UPD_N; i < sfl::PART_EB; ++i) b[i] = 0u;
  }
}
// part_answer_one (sfl_part.h) with its table reads issued together: the switch's action sources and compact
// columns (8 bytes each), the block's width and offsets, then the row's columns, then the same comparisons in
// the same order (row_max, max_action: bit-identical results).  Round 3: the generic version walks row_val
// per action, a chain of dependent L2 reads per request (12.6 us of a 178-us round).
// the map reads of an answer (they do not depend on the round's updates: k_part_owner issues them before its
// stage loop, so the answer waits for the row only)
struct AnsPre {
  int na, w;
  uint2 srcw, jw;
  uint64_t qoff;
  uint32_t rowb;
};
__device__ __forceinline__ AnsPre answer_pre(const sfl::SflMap& m, const sfl::SflPart& P, int port) {
  const int sw = port >> 2;
  AnsPre a;
  a.na = m.sw_na[sw];
  a.srcw = *(const uint2*)(m.act_src + (size_t)sw * 8);
  a.jw = *(const uint2*)(m.act_j + (size_t)sw * 8);
  a.w = m.q_w[port];
  a.qoff = P.q_off_own[port];
  a.rowb = P.row_own[port];
  return a;
}
__device__ __forceinline__ void part_answer_fast(const sfl::SflMap& m, const sfl::SflPart& P, const sfl::PartReq& r,
                                                 sfl::PartRep& out, const AnsPre& pre) {
  const int port = r.port, slot = port & 3;
  const int na = pre.na;
  const uint2 srcw = pre.srcw;
  const uint2 jw = pre.jw;
  const int w = pre.w;
  const double* row = P.q_own + (size_t)r.genv * P.q_own_per_env + pre.qoff + (size_t)r.state * (uint32_t)w;
  double rv[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) rv[c] = row[c < w ? c : 0];
  auto col = [&](int c) -> double {
    double v = rv[0];
#pragma unroll
    for (int k = 1; k < 8; ++k) v = c == k ? rv[k] : v;
    return v;
  };
  auto val = [&](int a) -> double {  // row_val
    if (a == na - 1) return col(w - 1);
    const uint32_t src = ((a < 4 ? srcw.x : srcw.y) >> (8 * (a & 3))) & 0xFFu;
    if (src == (uint32_t)slot) return col((int)(((a < 4 ? jw.x : jw.y) >> (8 * (a & 3))) & 0xFFu));
    return m.default_q;
  };
  double mx = val(0);
  int best = 0;
  for (int a = 1; a < na; ++a) {
    const double v = val(a);
    if (v > mx) {
      mx = v;
      best = a;
    }
  }
  out.mq = mx;  // (row_max: the same maximum over the same sequence)
  out.pad = 0;
  if (r.flags & 1u) {
    out.action = -1;
    return;
  }
  const uint32_t rid = pre.rowb + r.state;
  atomicOr(&P.touched_own[(size_t)r.genv * P.own_words + (rid >> 5)], 1u << (rid & 31u));
  if ((r.amask >> best) & 1u) {
    out.action = best;
    return;
  }
  int arg = -1;
  double amx = 0.0;
  for (int a = 0; a < na; ++a) {
    if (!((r.amask >> a) & 1u)) continue;
    const double v = val(a);
    if (arg < 0 || v > amx) {
      arg = a;
      amx = v;
    }
  }
  out.action = arg;
}
// owner side of a round (sfl_part.h part_owner_group's order per env): a block takes the groups that start in a
// chunk of OWN_CHUNK records of a segment (its threads hold the chunk's records and the tails of groups that
// run past its end), applies their update records stage by stage -- records of one stage touch distinct cells of
// their env; a later stage (an arrival bonus, a later post of the same launch) may revisit a cell -- with a
// block barrier between stages, then answers their requests.  One launch, every record on its own thread.
// (Round 4 ran three kernels: stage-0 updates, the later stages in one block, the answers.  A first round-5 cut
// walked each group on one thread: 30 us per round on the 8-rank rehearsal, the group's loads in one chain.)
constexpr int OWN_CHUNK = 256;
__global__ void __launch_bounds__(OWN_CHUNK) k_part_owner(const sfl::SflMap* __restrict__ m, const sfl::SflPart* __restrict__ P,
                                                          const sfl::PartMsg* __restrict__ in, sfl::PartRep* __restrict__ out) {
  constexpr int X = sfl::PART_GROUP_MAX - 1;  // a group reaches at most this far past its chunk
  __shared__ uint32_t smax;
  const size_t k = P->k_msg;
  const uint32_t chunks = (uint32_t)((k + OWN_CHUNK - 1) / OWN_CHUNK), units = (uint32_t)P->world * chunks;
  const uint32_t t = threadIdx.x;
  for (uint32_t u = blockIdx.x; u < units; u += gridDim.x) {
    const size_t base = (size_t)(u / chunks) * (k + 1);
    const size_t n = in[base].genv;
    const size_t lo = 1 + (size_t)(u % chunks) * OWN_CHUNK;
    if (lo > n) continue;  // (block-uniform)
    const size_t hi = min(lo + OWN_CHUNK, n + 1);
    // this thread's records: lo + t, and for t < X the tail record hi + t; each one the block's if its group
    // starts in [lo, hi)
    sfl::PartMsg r[2];
    bool mine[2];
    uint32_t st[2];
    const size_t ix[2] = {lo + t, hi + t};
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const bool in_range = q == 0 ? ix[0] < hi : (t < (uint32_t)X && ix[1] <= n);
      r[q] = in[base + (in_range ? ix[q] : 0)];
      const size_t gs = ix[q] - sfl::msg_pos(r[q].kind);
      const uint32_t ty = sfl::msg_type(r[q].kind);
      mine[q] = in_range && gs >= lo && gs < hi && ty != sfl::MSG_VOID;
      st[q] = (mine[q] && (ty == sfl::MSG_UPD || ty == sfl::MSG_INSERT)) ? r[q].stage : 0u;
    }
    AnsPre pre[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const uint32_t ty = sfl::msg_type(r[q].kind);
      pre[q] = answer_pre(*m, *P, (mine[q] && (ty == sfl::MSG_REQ || ty == sfl::MSG_REQ_X)) ? (int)r[q].port : 0);
    }
    if (t == 0) smax = 0u;
    __syncthreads();
    const uint32_t top = max(st[0], st[1]);
    if (top) atomicMax(&smax, top);
    __syncthreads();
    const uint32_t last = smax;
    for (uint32_t s = 0; s <= last; ++s) {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const uint32_t ty = sfl::msg_type(r[q].kind);
        if (mine[q] && (ty == sfl::MSG_UPD || ty == sfl::MSG_INSERT) && st[q] == s) sfl::part_update_one(*m, *P, r[q]);
      }
      __syncthreads();  // (this stage's writes before the next stage's reads: one CU, one L1)
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const uint32_t ty = sfl::msg_type(r[q].kind);
      if (mine[q] && (ty == sfl::MSG_REQ || ty == sfl::MSG_REQ_X))
        part_answer_fast(*m, *P, sfl::req_of_msg(r[q]), out[base + ix[q]], pre[q]);
    }
  }
}
__global__ void k_replicate(uint32_t* base, size_t words, uint32_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < words * (n - 1); i += (size_t)gridDim.x * blockDim.x)
    base[words + i] = base[i % words];
}

// The exploratory action (distr_q.py:315-317) seeds a fresh Generator(PCG64(SeedSequence(v)))
// with v = rng.integers(0, 2**31 - 1) and draws one bounded integer from it, whose Lemire step
// needs only the generator's first 32-bit output.  That output is a pure function of v, so it is
// tabulated once per device for all 2^31 values (8.6 GB of the 288 GB HBM): an exploratory
// decision then costs one load instead of ~250 dependent integer instructions.
__global__ void k_seedseq_table(uint32_t* out, uint64_t n) {
  for (uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; v < n; v += (uint64_t)gridDim.x * blockDim.x) {
    sfl::Pcg64 g;
    sfl::pcg_from_seedseq((uint32_t)v, g);
    out[v] = sfl::pcg_next32(g);
  }
}

// per-launch totals of the per-env counters (one block): decisions, ticks, bytes, OR of errors
__global__ void __launch_bounds__(1024) k_reduce_launch(const uint64_t* dec, const uint64_t* ticks, const uint64_t* bytes,
                                                        const uint32_t* err, uint32_t E, uint64_t* out) {
  __shared__ uint64_t red[4][16];
  uint64_t a = 0, b = 0, c = 0, o = 0;
  for (uint32_t e = threadIdx.x; e < E; e += blockDim.x) {
    a += dec[e];
    b += ticks[e];
    c += bytes[e];
    o |= err[e];
  }
  for (int off = 32; off > 0; off >>= 1) {
    a += __shfl_xor(a, off, 64);
    b += __shfl_xor(b, off, 64);
    c += __shfl_xor(c, off, 64);
    o |= __shfl_xor(o, off, 64);
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[0][w] = a;
    red[1][w] = b;
    red[2][w] = c;
    red[3][w] = o;
  }
  __syncthreads();
  if (threadIdx.x < 4) {
    uint64_t t = 0;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t = threadIdx.x == 3 ? (t | red[3][i]) : t + red[threadIdx.x][i];
    out[threadIdx.x] = t;
  }
}

__global__ void k_fill_f64(double* p, double v, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = v;
}

// one thread per (env, patch row); consecutive threads = consecutive rows of one env
__global__ void k_qinit(sfl::SflMap m, sfl::SflState s, uint32_t n_rows, const uint32_t* port, const uint32_t* state,
                        const double* vals) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (size_t)n_rows * s.E) return;
  const uint32_t e = (uint32_t)(i / n_rows), r = (uint32_t)(i % n_rows);
  const uint32_t g = port[r], st = state[r];
  const int w = m.q_w[g];
  double* row = s.q + (size_t)e * m.q_per_env + m.q_off[g] + (size_t)st * w;
  for (int j = 0; j < w; ++j) {
    const double v = vals[(size_t)r * 4 + j];
    row[j] = (v != v) ? m.default_q : v;
  }
  const uint32_t rid = m.row_base[g] + st;
  atomicOr(&s.touched[(size_t)e * m.touched_words + (rid >> 5)], 1u << (rid & 31u));
}

struct HipBackend {
  static constexpr bool kHasWave = true;
  hipStream_t stream = nullptr;      // the stream every call of the handle queues on
  hipStream_t own_stream = nullptr;  // the handle's own (stream unless sfl_set_stream chose the caller's)
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  void* d_params = nullptr;  // device copies of SflMap | SflState | SflCtl
  std::string err;
  int dev = 0;

  static int device_count(int* n) {
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
    *n = c;
    return 0;
  }
  bool check(hipError_t rc, const char* what) {
    if (rc == hipSuccess) return true;
    if (err.empty()) err = std::string(what) + ": " + hipGetErrorString(rc);
    return false;
  }
  const char* error() const { return err.c_str(); }
  int init(int device) {
    dev = device;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) {
      err = "no HIP device visible (this library needs an MI355X)";
      return -1;
    }
    if (!check(hipSetDevice(device), "hipSetDevice")) return -1;
    if (!check(hipStreamCreateWithFlags(&own_stream, hipStreamNonBlocking), "hipStreamCreate")) return -1;
    stream = own_stream;
    if (!check(hipEventCreate(&ev0), "hipEventCreate") || !check(hipEventCreate(&ev1), "hipEventCreate")) return -1;
    if (!check(hipMalloc(&d_params, 4096), "hipMalloc params")) return -1;
    return 0;
  }
  ~HipBackend() {
    if (ev0) hipEventDestroy(ev0);
    if (ev1) hipEventDestroy(ev1);
    if (d_params) hipFree(d_params);
    if (d_pparams) hipFree(d_pparams);
    if (own_stream) hipStreamDestroy(own_stream);
  }
  // the host's waits for the device (stream / event synchronisations): sfl_get_sync_count
  uint64_t n_wait = 0;
  hipError_t stream_wait() {
    ++n_wait;
    return hipStreamSynchronize(stream);
  }
  hipError_t event_wait(hipEvent_t ev) {
    ++n_wait;
    return hipEventSynchronize(ev);
  }
  // queue on the caller's stream (e.g. torch's current stream, which its RCCL collectives follow);
  // null: back to the handle's own
  int set_stream(void* st) {
    if (!check(stream_wait(), "sync")) return -1;
    stream = st ? (hipStream_t)st : own_stream;
    return 0;
  }
  void* alloc(size_t bytes) {
    void* p = nullptr;
    if (!check(hipMalloc(&p, bytes), "hipMalloc")) return nullptr;
    return p;
  }
  void free(void* p) {
    if (p) hipFree(p);
  }
  void h2d(void* d, const void* s, size_t n) { check(hipMemcpyAsync(d, s, n, hipMemcpyHostToDevice, stream), "h2d"); }
  void d2h(void* d, const void* s, size_t n) {
    check(hipMemcpyAsync(d, s, n, hipMemcpyDeviceToHost, stream), "d2h");
    check(stream_wait(), "d2h sync");
  }
  void memset(void* p, int v, size_t n) { check(hipMemsetAsync(p, v, n, stream), "memset"); }
  // stream-ordered copy without the synchronisation (the caller syncs once for several)
  void d2h_async(void* d, const void* s, size_t n) { check(hipMemcpyAsync(d, s, n, hipMemcpyDeviceToHost, stream), "d2h"); }
  // time between the events of the last launch (after a sync)
  float elapsed_ms() {
    float t = 0.f;
    hipEventElapsedTime(&t, ev0, ev1);
    return t;
  }
  void fill_f64(double* p, double v, size_t n) {
    k_fill_f64<<<4096, 256, 0, stream>>>(p, v, n);
    check(hipGetLastError(), "k_fill_f64");
  }
  void qinit(const sfl::SflMap& m, const sfl::SflState& s, uint32_t n_rows, const uint32_t* port,
             const uint32_t* state, const double* vals) {
    const size_t n = (size_t)n_rows * s.E;
    const unsigned blocks = (unsigned)((n + 255) / 256);
    k_qinit<<<blocks, 256, 0, stream>>>(m, s, n_rows, port, state, vals);
    check(hipGetLastError(), "k_qinit");
  }
#ifdef SFL_PROFILE
  // tuning builds: the wave kernels' phase cycles (sfl_wave.h g_prof), printed and cleared
  void print_prof() {
      unsigned long long pr[32] = {};
      hipMemcpyFromSymbol(pr, HIP_SYMBOL(sfl::wave::g_prof), sizeof pr);
      {  // variant 7's kernels count into their own translation unit's copy
        unsigned long long p7[32] = {};
        sflk::kwave_v7_prof_take(p7);
        for (int k = 0; k < 32; ++k) pr[k] += p7[k];
      }
      fprintf(stderr,
              "[sfl profile] cycles reset %.3e tick %.3e decide %.3e (observe %.3e egreedy %.3e apply %.3e) post %.3e "
              "total %.3e | prefetch %llu row hit %llu miss %llu pend hit %llu miss %llu decisions %llu\n",
              (double)pr[0], (double)pr[1], (double)pr[2], (double)pr[5], (double)pr[6], (double)pr[7], (double)pr[3],
              (double)pr[4], pr[8], pr[9], pr[10], pr[11], pr[12], pr[13]);
      fprintf(stderr, "[sfl laps]");
      for (int k = 0; k < 16; ++k) fprintf(stderr, " %d:%.3e", k, (double)pr[16 + k]);
      fprintf(stderr, "\n");
      unsigned long long z[32] = {};
      hipMemcpyToSymbol(HIP_SYMBOL(sfl::wave::g_prof), z, sizeof z);
    }
#endif
  int run(const sfl::SflMap& m, const sfl::SflState& s, const sfl::SflCtl& c, int variant, float* ms) {
    static_assert(sizeof(sfl::SflMap) + sizeof(sfl::SflState) + sizeof(sfl::SflCtl) + 64 < 4096, "params");
    const unsigned blocks = (s.E + 255) / 256;
    char* base = (char*)d_params;
    const size_t om = 0, os = (sizeof(sfl::SflMap) + 63) / 64 * 64,
                 oc = os + (sizeof(sfl::SflState) + 63) / 64 * 64;
    struct {
      sfl::SflMap m;
      char p0[(sizeof(sfl::SflMap) + 63) / 64 * 64 - sizeof(sfl::SflMap)];
      sfl::SflState s;
      char p1[(sizeof(sfl::SflState) + 63) / 64 * 64 - sizeof(sfl::SflState)];
      sfl::SflCtl c;
    } host_params;
    host_params.m = m;
    host_params.s = s;
    host_params.c = c;
    (void)om;
    check(hipMemcpyAsync(d_params, &host_params, sizeof(host_params), hipMemcpyHostToDevice, stream), "params h2d");
    check(hipEventRecord(ev0, stream), "event");
    const auto* pm = (const sfl::SflMap*)(base);
    const auto* ps = (const sfl::SflState*)(base + os);
    const auto* pc = (const sfl::SflCtl*)(base + oc);
    const unsigned wblocks = (unsigned)(((size_t)s.E * 64 + SFL_WAVE_BLOCK - 1) / SFL_WAVE_BLOCK);
#define SFL_KW(v)                                                                                                   \
  {                                                                                                             \
    constexpr sfl::WaveShape w = sfl::kVariants[v];                                                             \
    if (c.trace) k_wave<w.PPL, w.SPL, w.TW, true><<<wblocks, SFL_WAVE_BLOCK, 0, stream>>>(pm, ps, pc);          \
    else if (c.phase_cyc) k_wave<w.PPL, w.SPL, w.TW, false, true><<<wblocks, SFL_WAVE_BLOCK, 0, stream>>>(pm, ps, pc); \
    else k_wave<w.PPL, w.SPL, w.TW, false><<<wblocks, SFL_WAVE_BLOCK, 0, stream>>>(pm, ps, pc);                 \
  }
#define SFL_KW2(v)                                                                                       \
  {                                                                                                             \
    constexpr sfl::WaveShape w = sfl::kVariants[v];                                                             \
    if (c.trace) k_wave2<w.PPL, w.SPL, w.TW, true><<<s.E, 64, 0, stream>>>(pm, ps, pc);                         \
    else if (c.phase_cyc) k_wave2<w.PPL, w.SPL, w.TW, false, true><<<s.E, 64, 0, stream>>>(pm, ps, pc);         \
    else k_wave2<w.PPL, w.SPL, w.TW, false><<<s.E, 64, 0, stream>>>(pm, ps, pc);                                \
  }
#define SFL_KG(v)                                                                                               \
  {                                                                                                             \
    constexpr sfl::WaveShape w = sfl::kVariants[v];                                                             \
    const unsigned gblocks = (unsigned)(((size_t)s.E * w.G + SFL_GROUP_BLOCK - 1) / SFL_GROUP_BLOCK);             \
    if (c.trace) k_wave_g<w.PPL, w.SPL, w.TW, true, w.G, w.OCC, false, (bool)w.LM><<<gblocks, SFL_GROUP_BLOCK, 0, stream>>>(pm, ps, pc); \
    else if (c.phase_cyc)                                                                                       \
      k_wave_g<w.PPL, w.SPL, w.TW, false, w.G, w.OCC, true, (bool)w.LM><<<gblocks, SFL_GROUP_BLOCK, 0, stream>>>(pm, ps, pc); \
    else k_wave_g<w.PPL, w.SPL, w.TW, false, w.G, w.OCC, false, (bool)w.LM><<<gblocks, SFL_GROUP_BLOCK, 0, stream>>>(pm, ps, pc); \
  }
    static_assert(sfl::kVariants[5].TW > 64 && sfl::kNumVariants == 12, "variant 5 is the two-slot shape, 6-11 grouped");
    if (variant == 1) SFL_KW(1)
    else if (variant == 2) SFL_KW(2)
    else if (variant == 3) SFL_KW(3)
    else if (variant == 4) SFL_KW(4)
    else if (variant == 5) SFL_KW2(5)
    else if (variant == 6) SFL_KG(6)
    else if (variant == 7) SFL_KG(7)
    else if (variant == 8) SFL_KG(8)
    else if (variant == 9) SFL_KG(9)
    else if (variant == 10) SFL_KG(10)
    else if (variant == 11) SFL_KG(11)
#undef SFL_KG
#undef SFL_KW2
#undef SFL_KW
    else if (m.T <= 32) k_run<1><<<blocks, 256, 0, stream>>>(pm, ps, pc);
    else if (m.T <= 64) k_run<2><<<blocks, 256, 0, stream>>>(pm, ps, pc);
    else k_run<4><<<blocks, 256, 0, stream>>>(pm, ps, pc);
    if (!check(hipGetLastError(), "k_run launch")) return -1;
    check(hipEventRecord(ev1, stream), "event");
    if (!check(event_wait(ev1), "k_run")) return -1;
    float t = 0.f;
    hipEventElapsedTime(&t, ev0, ev1);
    *ms = t;
#ifdef SFL_PROFILE
    if (variant > 0) print_prof();
#endif
    return err.empty() ? 0 : -1;
  }
  // external-action mode: one call = every env applies its action and runs to its next observation
  int run_ext(const sfl::SflMap& m, const sfl::SflState& s, const sfl::SflCtl& c, float* ms) {
    struct {
      sfl::SflMap m;
      char p0[(sizeof(sfl::SflMap) + 63) / 64 * 64 - sizeof(sfl::SflMap)];
      sfl::SflState s;
      char p1[(sizeof(sfl::SflState) + 63) / 64 * 64 - sizeof(sfl::SflState)];
      sfl::SflCtl c;
    } hp;
    hp.m = m;
    hp.s = s;
    hp.c = c;
    const size_t os = (sizeof(sfl::SflMap) + 63) / 64 * 64, oc = os + (sizeof(sfl::SflState) + 63) / 64 * 64;
    char* base = (char*)d_params;
    check(hipMemcpyAsync(d_params, &hp, sizeof(hp), hipMemcpyHostToDevice, stream), "params h2d");
    check(hipEventRecord(ev0, stream), "event");
    const auto* pm = (const sfl::SflMap*)base;
    const auto* ps = (const sfl::SflState*)(base + os);
    const auto* pc = (const sfl::SflCtl*)(base + oc);
    const unsigned blocks = (s.E + 63) / 64;  // (64-thread blocks: few envs, spread over the CUs)
    if (m.T <= 32) k_run_ext<1><<<blocks, 64, 0, stream>>>(pm, ps, pc);
    else if (m.T <= 64) k_run_ext<2><<<blocks, 64, 0, stream>>>(pm, ps, pc);
    else k_run_ext<4><<<blocks, 64, 0, stream>>>(pm, ps, pc);
    if (!check(hipGetLastError(), "k_run_ext launch")) return -1;
    check(hipEventRecord(ev1, stream), "event");
    if (!check(event_wait(ev1), "k_run_ext")) return -1;
    float t = 0.f;
    hipEventElapsedTime(&t, ev0, ev1);
    *ms = t;
    return err.empty() ? 0 : -1;
  }
  int sync() { return check(stream_wait(), "sync") && err.empty() ? 0 : -1; }
  // process-wide, one per device, built on first use and kept for the life of the process
  const uint32_t* seedseq_table() {
    static uint32_t* tab[64] = {};
    if (dev < 0 || dev >= 64) return nullptr;
    if (!tab[dev]) {
      const uint64_t n = 1ull << 31;
      void* p = nullptr;
      if (hipMalloc(&p, n * 4) != hipSuccess) return nullptr;  // no table: draws fall back to compute
      k_seedseq_table<<<16384, 256, 0, stream>>>((uint32_t*)p, n);
      if (!check(hipGetLastError(), "k_seedseq_table") || !check(stream_wait(), "k_seedseq_table")) {
        hipFree(p);
        return nullptr;
      }
      tab[dev] = (uint32_t*)p;
    }
    return tab[dev];
  }
  void reduce_launch(const uint64_t* dec, const uint64_t* ticks, const uint64_t* bytes, const uint32_t* err, uint32_t E,
                     uint64_t* out) {
    k_reduce_launch<<<1, 1024, 0, stream>>>(dec, ticks, bytes, err, E, out);
    check(hipGetLastError(), "k_reduce_launch");
  }
  void replicate(void* base, size_t bytes, uint32_t n) {
    if (n > 1) k_replicate<<<4096, 256, 0, stream>>>((uint32_t*)base, bytes / 4, n);
    check(hipGetLastError(), "k_replicate");
  }
  // parameter block for the partitioned kernels: SflMap | SflState | SflCtl | SflPart
  struct PartParams {
    sfl::SflMap m;
    char p0[(sizeof(sfl::SflMap) + 63) / 64 * 64 - sizeof(sfl::SflMap)];
    sfl::SflState s;
    char p1[(sizeof(sfl::SflState) + 63) / 64 * 64 - sizeof(sfl::SflState)];
    sfl::SflCtl c;
    char p2[(sizeof(sfl::SflCtl) + 63) / 64 * 64 - sizeof(sfl::SflCtl)];
    sfl::SflPart P;
  };
  // one device parameter block per round step (0 local, 1 owner; 2 unused), uploaded only when
  // its contents change: a round's steps reuse the same buffers, so after the first round no step
  // pays a host-to-device copy and its synchronisation
  void* d_pparams = nullptr;
  PartParams pp_host[3];
  bool pp_valid[3] = {false, false, false};
  PartParams* part_params(int which, const sfl::SflMap& m, const sfl::SflState& s, const sfl::SflCtl& c,
                          const sfl::SflPart& P) {
    static_assert(3 * ((sizeof(PartParams) + 255) / 256 * 256) <= 16384, "params");
    constexpr size_t stride = (sizeof(PartParams) + 255) / 256 * 256;
    if (!d_pparams && !check(hipMalloc(&d_pparams, 16384), "hipMalloc params")) return nullptr;
    PartParams hp;
    ::memset(&hp, 0, sizeof hp);  // (the C library one, not this class's device memset) padding included: the blocks are compared bytewise
    hp.m = m;
    hp.s = s;
    hp.c = c;
    hp.P = P;
    auto* dst = (PartParams*)((char*)d_pparams + which * stride);
    if (pp_valid[which] && memcmp(&pp_host[which], &hp, sizeof hp) == 0) return dst;
    pp_host[which] = hp;
    pp_valid[which] = true;
    check(hipMemcpyAsync(dst, &pp_host[which], sizeof hp, hipMemcpyHostToDevice, stream), "params h2d");
    check(stream_wait(), "params sync");
    return dst;
  }
  // new segment capacities (sfl_part_set_caps, at a checkpoint): the uploaded parameter blocks take them now, so
  // the next rounds' launches find their blocks unchanged and upload nothing (no wait between checkpoints)
  void part_caps(const sfl::SflPart& P) {
    if (!d_pparams) return;
    constexpr size_t stride = (sizeof(PartParams) + 255) / 256 * 256;
    bool any = false;
    for (int w = 0; w < 3; ++w) {
      if (!pp_valid[w]) continue;
      pp_host[w].P.k_msg = P.k_msg;
      check(hipMemcpyAsync((char*)d_pparams + w * stride, &pp_host[w], sizeof(PartParams), hipMemcpyHostToDevice, stream),
            "params h2d");
      any = true;
    }
    if (any) check(stream_wait(), "params sync");
  }
  int part_local(const sfl::SflMap& m, const sfl::SflState& s, const sfl::SflCtl& c, const sfl::SflPart& P, int variant,
                 float* ms) {
    PartParams* pp = part_params(0, m, s, c, P);
    if (!pp) return -1;
    check(hipEventRecord(ev0, stream), "event");
    // one wave per block: a round's envs spread over as many CUs as possible
    const unsigned blocks = (s.E + 63) / 64;
    const unsigned wblocks = (unsigned)(((size_t)s.E * 64 + SFL_WAVE_BLOCK - 1) / SFL_WAVE_BLOCK);
#define SFL_KWP(v) \
  k_wave_part<sfl::kVariants[v].PPL, sfl::kVariants[v].SPL, sfl::kVariants[v].TW><<<wblocks, SFL_WAVE_BLOCK, 0, stream>>>(&pp->m, &pp->s, &pp->c, &pp->P)
    if (variant == 1) SFL_KWP(1);
    else if (variant == 2) SFL_KWP(2);
    else if (variant == 3) SFL_KWP(3);
    else if (variant == 4) SFL_KWP(4);
    else if (variant == 5)
      k_wave2_part<sfl::kVariants[5].PPL, sfl::kVariants[5].SPL, sfl::kVariants[5].TW><<<s.E, 64, 0, stream>>>(&pp->m, &pp->s, &pp->c, &pp->P);
#undef SFL_KWP
    else if (m.T <= 32) k_part_local<1><<<blocks, 64, 0, stream>>>(&pp->m, &pp->s, &pp->c, &pp->P);
    else if (m.T <= 64) k_part_local<2><<<blocks, 64, 0, stream>>>(&pp->m, &pp->s, &pp->c, &pp->P);
    else k_part_local<4><<<blocks, 64, 0, stream>>>(&pp->m, &pp->s, &pp->c, &pp->P);
    if (!check(hipGetLastError(), "k_part_local")) return -1;
    // (256 envs per block: fewer blocks reserve places and count themselves done; 64 measured -1.3 %)
    k_part_compact<<<(s.E + SFL_COMPACT_BLOCK - 1) / SFL_COMPACT_BLOCK, SFL_COMPACT_BLOCK, 0, stream>>>(&pp->P, &pp->s, &pp->c,
                                                                                                  variant > 0 ? 0 : 1);
    check(hipEventRecord(ev1, stream), "event");
    // (no synchronisation here: the caller issues the launch totals and the count copies behind
    // it and syncs once; *ms is read with elapsed_ms() after that)
    *ms = 0.f;
#ifdef SFL_PROFILE
    if (!check(event_wait(ev1), "k_part_local")) return -1;
    if (variant > 0) print_prof();
#endif
    return err.empty() ? 0 : -1;
  }
  // the wave kernels' per-env scalar blocks from / into the SflState arrays (k_part_eblk)
  void part_eblk(const sfl::SflState& s, const sfl::SflPart& P, int dir) {
    k_part_eblk<<<(s.E + 255) / 256, 256, 0, stream>>>(s, P.eblk, P.dec_done, dir);
    check(hipGetLastError(), "k_part_eblk");
  }
  // the owner side of a round on the received message segments (k_part_owner)
  void part_owner(const sfl::SflMap& m, const sfl::SflPart& P, const sfl::PartMsg* in, sfl::PartRep* out) {
    sfl::SflState s{};
    sfl::SflCtl c{};
    PartParams* pp = part_params(1, m, s, c, P);
    if (!pp) return;
    const size_t units = (size_t)P.world * ((P.k_msg + OWN_CHUNK - 1) / OWN_CHUNK);
    const unsigned blocks = (unsigned)std::min<size_t>(units, 1024);
    k_part_owner<<<blocks, OWN_CHUNK, 0, stream>>>(&pp->m, &pp->P, in, out);
    check(hipGetLastError(), "k_part_owner");
  }
};

}  // namespace

using Backend = HipBackend;
#include "sfl_capi.inc"
