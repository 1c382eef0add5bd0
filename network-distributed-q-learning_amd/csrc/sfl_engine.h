// Engine: owns one batch of lock-step environments on one device and implements
// the C-ABI of include/sfl.h.  Templated over a backend (HIP device memory +
// kernel launches in sfl.hip; host memory + a plain loop in the test-only
// host build sfl_hostsim.cpp) so both builds share every line above the
// per-env kernel body.
#pragma once
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "../../include/sfl.h"
#include "sfl_core.h"
#include "sfl_mfgen.h"
#include "sfl_part.h"

namespace sfl {

static thread_local std::string g_last_error;

inline int fail(const std::string& msg) {
  g_last_error = msg;
  return -1;
}

template <class B>
struct Handle {
  B be;
  SflMap map{};
  SflState st{};
  uint32_t E = 0;
  int device = 0;
  std::vector<void*> allocs;
  std::vector<uint64_t> seeds;
  // host copies of small per-env counters for reporting
  // launch totals reduced on the device (decisions, ticks, algorithmic bytes, OR of error flags)
  uint64_t last_dec = 0, last_ticks = 0, last_bytes = 0, total_dec = 0;
  uint32_t last_err = 0;
  uint64_t* d_sums = nullptr;  // [4]
  bool ext_stream = false;     // the caller's stream (sfl_set_stream): owner steps queue without a sync
  bool part_pending = false;              // a part_local's counts not read yet
  bool part_consumed = true;              // part_counts handed out by sfl_part_counts (the next read restarts the peaks)
  uint64_t part_reads = 0;                // host reads of the round counts (part_read): sfl_get_sync_count
  std::vector<uint32_t> part_counts;      // of the last part_local: [2 * world + 1]
  // the partitioned wave kernels' per-env scalar blocks (SflPart::eblk): which copy is current --
  // 0 the SflState arrays (the next part_local copies them in), 1 the blocks, 2 both
  int eblk_state = 0;
  uint64_t* d_launch_dec = nullptr;
  uint64_t* d_launch_ticks = nullptr;
  uint64_t* d_launch_bytes = nullptr;
  float last_kernel_ms = 0.f;
  std::vector<std::vector<uint32_t>> keep;  // host sources of async uploads, alive until the create() sync
  int variant = 0;  // 0: k_run (lane per env); v > 0: k_wave shape kVariants[v] (see choose_variant)
  std::string variant_note;  // why a device handle runs k_run ("" when k_wave, or when chosen explicitly)
  // host copies of the map fields the partitioned mode lays out its owned Q blocks with
  std::vector<uint8_t> h_sw_np, h_q_w;
  std::vector<uint64_t> h_q_off;
  std::vector<uint32_t> h_row_base;
  // graph-partitioned mode (sfl_part.h); part.world == 0: not configured
  SflPart part{};
  // external-action mode (sfl_env_begin / sfl_env_step): device buffers, the descriptor in device memory
  SflExt ext{};
  SflExt* d_ext = nullptr;
  bool env_mode = false;
  // per-phase cycles of the sampled wavefronts, accumulated over learn / test launches on the device
  // (sfl_get_phase_cycles reads them)
  uint64_t* d_phase = nullptr;

  template <class T>
  T* dalloc(size_t n) {
    if (n == 0) n = 1;
    void* p = be.alloc(n * sizeof(T));
    if (!p) return nullptr;
    allocs.push_back(p);
    return (T*)p;
  }
  template <class T>
  const T* upload(const T* src, size_t n) {
    T* d = dalloc<T>(n);
    if (d && src && n) be.h2d(d, src, n * sizeof(T));
    return d;
  }
  void dfree(void* p) {
    for (auto& a : allocs)
      if (a == p) {
        be.free(p);
        a = allocs.back();
        allocs.pop_back();
        return;
      }
  }
  ~Handle() {
    for (void* p : allocs) be.free(p);
  }
};

// One-env-per-wavefront kernel shapes (sfl_wave.h): PPL semaphore and SPL counter registers
// per lane (ports <= 64*PPL, switches <= 64*SPL).  Index 0 = the lane-per-env kernel (k_run).
// TW: trains per env the variant's LDS prefetch records are sized for (T <= TW).
// G: lanes per env (64: one env per wavefront; 32 / 16 / 8: two / four / eight envs per wavefront, run_groups).
// OCC: waves per SIMD a grouped shape's registers are budgeted for (sfl.hip k_wave_g; 0: the G = 64 kernels' own).
#ifndef SFL_G8_OCC1
// G = 8, one train slot per lane (maps with <= 8 trains, c2: 32 envs per 256-thread block).  Round 4: c2 at 65,536
// envs 1,326 M agent-env-steps/s vs 853 M at G = 16 (profiles/r04c_c2_65536_g8.json, r04b_c2_65536_g16.json); a
// G = 8 shape with four train slots per lane for c3 spilled 100 registers at 256 VGPRs: 745 M vs 1,471 M at G = 16
// (profiles/r04c_c3_65536_g8.json), not kept
#define SFL_G8_OCC1 4
#endif
struct WaveShape {
  int PPL, SPL, TW, G, OCC;
  int LM = 0;  // 1: the map's move table and distance map are copied into the block's LDS (run_groups, round 6)
};
#ifndef SFL_LM_OCC
#define SFL_LM_OCC 4  // variant 11's register budget (waves per SIMD)
#endif
#ifndef SFL_V7_OCC
#define SFL_V7_OCC 4  // variant 7 (c3): waves per SIMD its registers are budgeted for (tuning builds: 3)
#endif
constexpr WaveShape kVariants[] = {{0, 0, 0, 64, 0},    {1, 1, 32, 64, 0},  {4, 1, 32, 64, 0}, {4, 1, 64, 64, 0},
                                   {8, 2, 64, 64, 0},   {16, 4, 128, 64, 0}, {4, 1, 16, 16, 4}, {16, 4, 32, 16, SFL_V7_OCC},
                                   {2, 1, 32, 32, 4},   {8, 2, 32, 32, 4},   {8, 2, 8, 8, SFL_G8_OCC1},
                                   {2, 1, 32, 32, SFL_LM_OCC, 1}};
constexpr int kNumVariants = 12;
// Variant 11 = variant 8 with the map's move table and distance map (as int16) in LDS (LM): a batch of at most two
// wavefronts per SIMD (kLmWaves; configs[1], c2 at 4,096 envs: 2,048 wavefronts at G = 32) runs two 256-thread blocks
// per CU, which leaves each block ~63 KB of LDS beyond its env records; the tick's two move-table lookups and the
// staging's move-table and distance lookups then become LDS reads instead of dependent L2 round trips.  Chosen where
// the tables fit kLmBytes (c2: 40,000 + 20,000 bytes); SFL_LDS_MAP=0 keeps variant 8.
constexpr uint64_t kLmWaves = 2048;
constexpr int64_t kLmBytes = 64512;  // (sfl_wave.h run_groups: LM_WORDS)
inline int64_t lm_bytes(const sfl_map_desc* md) {
  const int64_t hw = (int64_t)md->H * md->W;
  return hw * 4 * 16 + ((int64_t)md->K * hw * 4 + 1) / 2 * 4;
}
#ifndef SFL_DEFAULT_G
#define SFL_DEFAULT_G 16  // lane group size chosen where a grouped shape fits (SFL_WAVE_G overrides)
#endif

// Eligibility: trains fit one or two slots per lane (T <= 128), the env fits the variant's
// registers and every semaphore record fits the 32-bit LDS word (sfl_wave.h r_pack: start tick
// -8192..8191, span <= 511).  SFL_KERNEL=scalar forces k_run.  why: when non-null, the reason a
// map is not eligible (the caller reports it; the lane-per-env body is 15-45x slower).
// A batch too small to fill the device at the default group size (fewer than kFillWaves wavefronts: 4 per SIMD
// of MI355X's 1,024) takes two envs per wavefront instead of four: c2 at its stated 4,096 envs 316 M vs 276 M
// agent-env-steps/s (G = 64: 313 M), while c3 at 16,384 envs -- 4,096 wavefronts at G = 16 -- keeps G = 16
// (1,275 M vs 982 M at G = 64; profiles/r03d_group_size_*.json).  Round 4, c2 at 4,096 envs: G = 8 229 M, 16 291 M,
// 32 326 M, 64 323 M (profiles/r04c_c2_4096_g*.json).
constexpr uint64_t kFillWaves = 4096;
inline int choose_variant(const sfl_map_desc* md, bool backend_has_wave, std::string* why = nullptr, uint64_t n_envs = 0) {
  if (!backend_has_wave) return 0;
  const char* env = getenv("SFL_KERNEL");
  if (env && strcmp(env, "scalar") == 0) return 0;
  auto no = [&](const char* r) {
    if (why) *why = r;
    return 0;
  };
  if (md->T > 128) return no("more than 128 trains");
  int32_t ed_max = 0, ed_min = 0, dist_max = 0, len_max = 0;
  for (int32_t h = 0; h < md->T; ++h) {
    ed_max = md->tr_ed[h] > ed_max ? md->tr_ed[h] : ed_max;
    ed_min = md->tr_ed[h] < ed_min ? md->tr_ed[h] : ed_min;
    dist_max = md->tr_init_dist[h] > dist_max ? md->tr_init_dist[h] : dist_max;
  }
  for (int32_t p = 0; p < md->S * 4; ++p) len_max = md->port_len[p] > len_max ? md->port_len[p] : len_max;
  const int64_t span = (int64_t)(dist_max > 2 * len_max + 2 ? dist_max : 2 * len_max + 2) + 4;
  const int64_t t_hi = (int64_t)(ed_max > md->max_episode_steps ? ed_max : md->max_episode_steps) + 2 + span;
  if (t_hi > 8191 || ed_min - 2 < -8192) return no("timetable horizon beyond 8191 ticks");
  if (span > 511) return no("a semaphore span beyond 511 ticks");
  for (size_t i = 0, n = (size_t)md->K * md->H * md->W * 4; i < n; ++i)  // (staged as int16, sfl_wave.h d16)
    if (md->dist[i] >= 32767 && md->dist[i] < DIST_INF) return no("a finite distance of 32767 cells or more");
  if (md->q_per_env >= (1ull << 32)) return no("Q-table beyond 2^32 cells per env");
  if ((int64_t)md->H * md->W >= (1 << 20) - 1) return no("grid beyond 2^20 cells");
  const char* gs = getenv("SFL_WAVE_G");
  // one train per lane, eight envs per wavefront, for maps with <= 8 trains (round 4)
  int want_g = gs ? atoi(gs) : (md->T <= 8 ? 8 : SFL_DEFAULT_G);
  if (!gs && n_envs > 0 && want_g < 32 && n_envs * (uint64_t)want_g / 64 < kFillWaves) want_g = 32;
  auto fits = [&](int v) {
    const WaveShape& w = kVariants[v];
    return md->S * 4 <= w.G * w.PPL && md->S <= w.G * w.SPL && md->T <= w.TW;
  };
  const char* lms = getenv("SFL_LDS_MAP");
  const bool lm_ok = !(lms && atoi(lms) == 0) && n_envs > 0 && n_envs * (uint64_t)want_g / 64 <= kLmWaves &&
                     lm_bytes(md) <= kLmBytes;
  for (int v = 1; v < kNumVariants; ++v) {
    if (kVariants[v].LM || kVariants[v].G != want_g || !fits(v)) continue;
    if (lm_ok)  // the same shape with the map tables in LDS, if there is one
      for (int u = 1; u < kNumVariants; ++u) {
        const WaveShape &a = kVariants[u], &b = kVariants[v];
        if (a.LM && a.PPL == b.PPL && a.SPL == b.SPL && a.TW == b.TW && a.G == b.G) return u;
      }
    return v;
  }
  for (int v = 1; v < kNumVariants; ++v)
    if (kVariants[v].G == 64 && fits(v)) return v;
  return no("more than 256 switches");
}

// the one-env-per-wavefront shape of the same map (the partitioned local step runs G = 64 only)
inline int wave64_variant(int S, int T) {
  for (int v = 1; v < kNumVariants; ++v) {
    const WaveShape& w = kVariants[v];
    if (w.G == 64 && S * 4 <= w.G * w.PPL && S <= w.G * w.SPL && T <= w.TW) return v;
  }
  return 0;
}

template <class B>
int create(const sfl_map_desc* md, const sfl_hparams* hp, uint32_t n_envs, const uint64_t* env_seeds, int device,
           Handle<B>** out) {
  if (!md || !hp || !out || n_envs == 0) return fail("sfl_create: null argument or zero envs");
  if (md->T > 32 * MAXW) return fail("sfl_create: at most 128 trains per env");
  if (md->S * 4 >= 0xFFFF) return fail("sfl_create: too many switches");
  if (md->K < 1 || md->K > 341) return fail("sfl_create: station count out of range");
  if (md->delay_threshold < -65536 || md->delay_threshold > 65536) return fail("sfl_create: delay_threshold out of range");
  auto* h = new Handle<B>();
  h->device = device;
  if (int rc = h->be.init(device)) {
    delete h;
    return fail(std::string("sfl_create: backend init failed: ") + h->be.error());
  }
  h->E = n_envs;
  h->h_sw_np.assign(md->sw_np, md->sw_np + md->S);
  h->h_q_w.assign(md->q_w, md->q_w + (size_t)md->S * 4);
  h->h_q_off.assign(md->q_off, md->q_off + (size_t)md->S * 4);
  h->h_row_base.assign(md->row_base, md->row_base + (size_t)md->S * 4);
  h->variant = choose_variant(md, B::kHasWave, &h->variant_note, n_envs);
  SflMap& m = h->map;
  const size_t HW = (size_t)md->H * md->W, NP = (size_t)md->S * 4, S = md->S, T = md->T;
  m.H = md->H;
  m.W = md->W;
  m.HW = md->H * md->W;
  m.cell_bits = 1;
  while ((1 << m.cell_bits) < m.HW) ++m.cell_bits;
  m.S = md->S;
  m.T = md->T;
  m.K = md->K;
  m.NP = (int32_t)NP;
  m.max_episode_steps = md->max_episode_steps;
  m.mf_rate = md->mf_rate;
  m.mf_min = md->mf_min;
  m.mf_max = md->mf_max;
  mf_prepare(m);  // (mf_propose's integer forms of u < mf_rate and of the duration's modulo)
  m.delay_thr = md->delay_threshold;
  m.gamma = hp->gamma;
  m.eps0 = hp->epsilon;
  m.eps_decay = hp->epsilon_decay_rate;
  // (log2 of 0 is -inf and of a negative value NaN: the device test is then never certain and takes the table)
  m.lr0 = hp->lr;
  m.lr_decay = hp->lr_decay_rate;
  m.default_q = hp->default_q;
  m.max_steps = hp->max_steps;
  m.ntab = hp->ntab;
  m.q_per_env = md->q_per_env;
  m.rows_per_env = md->rows_per_env;
  m.touched_words = (md->rows_per_env + 31u) / 32u;
  m.grid = h->upload(md->grid, HW);
  m.cell_sw = h->upload(md->cell_sw, HW);
  m.sw_np = h->upload(md->sw_np, S);
  m.sw_na = h->upload(md->sw_na, S);
  m.act_src = h->upload(md->act_src, S * 8);
  m.act_dst = h->upload(md->act_dst, S * 8);
  m.act_turn = h->upload(md->act_turn, S * 8);
  m.act_j = h->upload(md->act_j, S * 8);
  m.first_other = h->upload(md->first_other, NP);
  m.port_side = h->upload(md->port_side, NP);
  m.slot_nroutes = h->upload(md->slot_nroutes, NP);
  m.slot_route_act = h->upload(md->slot_route_act, NP * 4);
  m.q_w = h->upload(md->q_w, NP);
  m.port_nb = h->upload(md->port_nb, NP);
  m.port_len = h->upload(md->port_len, NP);
  m.port_unique = h->upload(md->port_unique, NP);
  m.q_off = h->upload(md->q_off, NP);
  m.row_base = h->upload(md->row_base, NP);
  m.dist = h->upload(md->dist, (size_t)md->K * HW * 4);
  m.tr_ed = h->upload(md->tr_ed, T);
  m.tr_la = h->upload(md->tr_la, T);
  m.tr_k = h->upload(md->tr_k, T);
  m.tr_target = h->upload(md->tr_target, T);
  m.tr_init_cell = h->upload(md->tr_init_cell, T);
  m.tr_init_dist = h->upload(md->tr_init_dist, T);
  m.tr_init_delay = h->upload(md->tr_init_delay, T);
  m.tr_init_dir = h->upload(md->tr_init_dir, T);
  m.tr_init_port = h->upload(md->tr_init_port, T);
  m.eps_tab = h->upload(hp->eps_tab, (size_t)hp->ntab);
  m.lr_tab = h->upload(hp->lr_tab, (size_t)hp->ntab);
  {
    // packed tables for the one-env-per-wave kernel: one scalar load per switch / port / train,
    // and check_action as a table lookup
    std::vector<uint32_t> swp(S * 16, 0), pp(NP * 4, 0), mv(HW * 16, 0);
    std::vector<int32_t> trp(T * 8, 0);
    bool pack_ok = true;
    for (size_t sw = 0; sw < S; ++sw) {
      uint32_t* w = &swp[sw * 16];
      const int na = md->sw_na[sw];
      w[0] = (uint32_t)md->sw_np[sw] | ((uint32_t)na << 4);
      for (int a = 0; a < 8 && a < na - 1; ++a) {  // routes (STOP = action na-1 has no entry)
        w[1] |= ((uint32_t)md->act_src[sw * 8 + a] & 3u) << (2 * a);
        w[1] |= ((uint32_t)md->act_dst[sw * 8 + a] & 3u) << (16 + 2 * a);
        w[2] |= ((uint32_t)md->act_turn[sw * 8 + a] & 3u) << (2 * a);
        w[2] |= ((uint32_t)md->act_j[sw * 8 + a] & 3u) << (16 + 2 * a);
      }
      for (int sl = 0; sl < 4; ++sl) {
        const uint32_t qw = md->q_w[sw * 4 + sl];
        w[3] |= (qw & 15u) << (4 * sl);
        // compact row descriptor: full-row action of each compact column (routes leaving
        // through this slot in action order, then STOP), and the first default-valued action
        uint32_t rd = 0, c = 0, mind = 15;
        for (int a = 0; a < na - 1; ++a) {
          if (md->act_src[sw * 8 + a] == sl) {
            if (md->act_j[sw * 8 + a] != c) rd |= 1u << 31;  // columns must follow action order
            rd |= ((uint32_t)a & 15u) << (4 * c++);
          } else if (mind == 15) {
            mind = (uint32_t)a;
          }
        }
        if (qw > 0) {
          if (c != qw - 1u) rd |= 1u << 31;
          rd |= ((uint32_t)(na - 1) & 15u) << (4 * c);
        }
        rd |= mind << 16;
        if (rd >> 31) pack_ok = false;
        w[4 + sl] = rd;
        // neighbour port of each port (observer lanes)
        w[8 + (sl >> 1)] |= (uint32_t)(uint16_t)md->port_nb[sw * 4 + sl] << (16 * (sl & 1));
      }
    }
    for (size_t p = 0; p < NP; ++p) {
      pp[p * 4 + 0] = (uint32_t)(uint16_t)md->port_nb[p] | ((uint32_t)(uint16_t)md->port_len[p] << 16);
      pp[p * 4 + 1] = (uint32_t)(uint16_t)md->port_unique[p] | ((uint32_t)md->q_w[p] << 16);
      pp[p * 4 + 2] = md->row_base[p];
      pp[p * 4 + 3] = (uint32_t)md->q_off[p];
    }
    std::vector<uint32_t> ptr_(NP * 4, 0);
    for (size_t o = 0; o < NP; ++o) {
      const int t = md->port_nb[o];
      const int u = t >= 0 ? md->port_unique[t] : -1;
      const int far = u >= 0 ? md->port_nb[u] : -1;
      ptr_[o * 4 + 0] = (uint32_t)(uint16_t)(int16_t)t | ((uint32_t)(uint16_t)(int16_t)u << 16);
      ptr_[o * 4 + 1] = (uint32_t)(uint16_t)(int16_t)far | ((uint32_t)(uint16_t)md->port_len[o] << 16);
      ptr_[o * 4 + 2] = u >= 0 ? (uint32_t)(uint16_t)md->port_len[u] : 0u;
    }
    for (size_t c = 0; c < HW; ++c)
      for (int d = 0; d < 4; ++d)
        for (int a = 0; a < 4; ++a)
        {
          // bits 24-31: the switch at the destination cell (0xFF: none, or more than 254 switches)
          uint32_t w = move_pack(md->grid, md->H, md->W, (uint32_t)a, (int)c, d);
          const int nc = (int)(w & 0xFFFFFu) - 1;
          const int swd = nc >= 0 ? md->cell_sw[nc] : -1;
          w |= (uint32_t)(swd >= 0 && md->S <= 254 ? swd : 0xFF) << 24;
          mv[(c * 4 + d) * 4 + a] = w;
        }
    for (size_t t = 0; t < T; ++t) {
      int32_t* w = &trp[t * 8];
      w[0] = md->tr_ed[t];
      w[1] = md->tr_la[t];
      w[2] = md->tr_k[t];
      w[3] = md->tr_target[t];
      w[4] = md->tr_init_cell[t];
      w[5] = md->tr_init_dist[t];
      w[6] = md->tr_init_delay[t];
      w[7] = (int32_t)((uint32_t)md->tr_init_dir[t] | ((uint32_t)(uint16_t)md->tr_init_port[t] << 16));
    }
    if (!pack_ok) {
      delete h;
      return fail("sfl_create: compact Q columns do not follow action order (map compiler mismatch)");
    }
    h->keep.push_back(std::move(swp));
    m.sw_pack = h->upload(h->keep.back().data(), h->keep.back().size());
    h->keep.push_back(std::move(pp));
    m.port_pack = h->upload(h->keep.back().data(), h->keep.back().size());
    // two steps ahead (the batch prefetch's reward projections, sfl_wave.h prefetch_slot)
    std::vector<uint32_t> mv2c(HW * 64, 0u);
    for (size_t i = 0; i < HW * 16; ++i) {
      const int nc = (int)(mv[i] & 0xFFFFFu) - 1, nd = (int)((mv[i] >> 20) & 3u);
      for (int n = 0; n < 4; ++n) mv2c[i * 4 + n] = nc < 0 ? ((uint32_t)nd << 20) : mv[((size_t)nc * 4 + nd) * 4 + n];
    }
    h->keep.push_back(std::move(mv));
    m.move_tab = h->upload(h->keep.back().data(), h->keep.back().size());
    h->keep.push_back(std::move(mv2c));
    m.move2c_tab = h->upload(h->keep.back().data(), h->keep.back().size());
    h->keep.push_back(std::move(ptr_));
    m.port_tr = h->upload(h->keep.back().data(), h->keep.back().size());
    m.seedseq32 = h->be.seedseq_table();
    h->keep.emplace_back(trp.begin(), trp.end());
    m.tr_pack = (const int32_t*)h->upload(h->keep.back().data(), h->keep.back().size());
  }

  SflState& s = h->st;
  const size_t E = n_envs;
  s.E = n_envs;
  s.phase = h->template dalloc<int32_t>(E);
  s.elapsed = h->template dalloc<int32_t>(E);
  s.eflags = h->template dalloc<uint32_t>(E);
  s.ep_t = h->template dalloc<int32_t>(E);
  s.n_test = h->template dalloc<int32_t>(E);
  s.epoch = h->template dalloc<uint32_t>(E);
  s.rng = h->template dalloc<uint64_t>(5 * E);
  s.seed = h->template dalloc<uint64_t>(E);
  s.cum_reward = h->template dalloc<double>(E);
  s.n_mf = h->template dalloc<int32_t>(E);
  s.ep_dec = h->template dalloc<int32_t>(E);
  s.ep_ticks = h->template dalloc<int32_t>(E);
  s.step_ctr = h->template dalloc<int64_t>(E);
  s.dec_total = h->template dalloc<int64_t>(E);
  s.masks = h->template dalloc<uint32_t>(4 * MAXW * E);
  s.err = h->template dalloc<uint32_t>(E);
  s.tr_pos = h->template dalloc<int32_t>(T * E);
  s.tr_bits = h->template dalloc<uint32_t>(T * E);
  s.tr_plan = h->template dalloc<uint32_t>(T * E);
  s.tr_next = h->template dalloc<uint16_t>(T * E);
  s.tr_prev = h->template dalloc<uint16_t>(T * E);
  s.tr_src = h->template dalloc<uint16_t>(T * E);
  s.tr_dec = h->template dalloc<uint16_t>(T * E);
  s.tr_delay = h->template dalloc<int32_t>(T * E);
  s.own = h->template dalloc<uint16_t>(T * OWN_MAX * E);
  s.own_n = h->template dalloc<uint8_t>(T * E);
  s.sc_desired = h->template dalloc<int32_t>(T * E);
  s.sc_pred = h->template dalloc<int32_t>(T * E);
  s.sc_aux = h->template dalloc<uint32_t>(T * E);
  s.occ = h->template dalloc<uint8_t>(HW * E);
  s.claim = h->template dalloc<uint8_t>(HW * E);
  s.sem = h->template dalloc<uint64_t>(NP * E);
  s.slot = h->template dalloc<uint64_t>(S * T * E);
  s.counts = h->template dalloc<uint32_t>(S * E);
  s.q = h->template dalloc<double>((size_t)m.q_per_env * E);
  s.touched = h->template dalloc<uint32_t>((size_t)m.touched_words * E);
  h->d_launch_dec = h->template dalloc<uint64_t>(E);
  h->d_launch_ticks = h->template dalloc<uint64_t>(E);
  h->d_launch_bytes = h->template dalloc<uint64_t>(E);
  h->d_sums = h->template dalloc<uint64_t>(4);
  h->d_phase = h->template dalloc<uint64_t>(8);
  for (void* p : h->allocs)
    if (!p) {
      delete h;
      return fail("sfl_create: device allocation failed");
    }
  if (!m.grid || !s.q) {
    delete h;
    return fail("sfl_create: device allocation failed (out of memory?)");
  }
  // initial values
  h->be.memset(s.phase, 0, E * 4);
  h->be.memset(s.elapsed, 0, E * 4);
  h->be.memset(s.eflags, 0, E * 4);
  h->be.memset(s.ep_t, 0, E * 4);
  h->be.memset(s.n_test, 0, E * 4);
  h->be.memset(s.epoch, 0, E * 4);
  h->be.memset(s.rng, 0, 5 * E * 8);
  h->be.memset(s.cum_reward, 0, E * 8);
  h->be.memset(s.n_mf, 0, E * 4);
  h->be.memset(s.ep_dec, 0, E * 4);
  h->be.memset(s.ep_ticks, 0, E * 4);
  h->be.memset(s.step_ctr, 0, E * 8);
  h->be.memset(s.dec_total, 0, E * 8);
  h->be.memset(s.masks, 0, 4 * MAXW * E * 4);
  h->be.memset(s.err, 0, E * 4);
  h->be.memset(s.tr_pos, 0xFF, T * E * 4);  // -1: off map
  h->be.memset(s.tr_bits, 0, T * E * 4);
  h->be.memset(s.tr_plan, 0, T * E * 4);
  h->be.memset(s.tr_next, 0, T * E * 2);
  h->be.memset(s.tr_prev, 0xFF, T * E * 2);  // None
  h->be.memset(s.tr_src, 0xFF, T * E * 2);   // None
  h->be.memset(s.tr_dec, 0, T * E * 2);
  h->be.memset(s.tr_delay, 0, T * E * 4);
  h->be.memset(s.own_n, 0, T * E);
  h->be.memset(s.occ, 0xFF, HW * E);
  h->be.memset(s.claim, 0xFF, HW * E);
  h->be.memset(s.sem, 0, NP * E * 8);
  h->be.memset(s.slot, 0, S * T * E * 8);
  h->be.memset(s.counts, 0, S * E * 4);
  h->be.memset(h->d_phase, 0, 8 * 8);
  h->be.memset(s.touched, 0, (size_t)m.touched_words * E * 4);
  h->be.fill_f64(s.q, m.default_q, (size_t)m.q_per_env * E);
  h->seeds.assign(env_seeds, env_seeds + E);
  h->be.h2d(s.seed, env_seeds, E * 8);
  if (int rc = h->be.sync()) {
    delete h;
    return fail(std::string("sfl_create: ") + h->be.error());
  }
  *out = h;
  return 0;
}

// Flatland-compatible malfunction stream: table[E][steps][T] proposals (sfl_mfgen.h); steps == 0
// returns to the counter-based draw
template <class B>
int set_mf_schedule(Handle<B>* h, int32_t steps, const uint8_t* table) {
  SflMap& m = h->map;
  if (steps < 0 || (steps > 0 && !table)) return fail("sfl_set_mf_schedule: bad argument");
  if (m.mf_tab) {
    h->dfree((void*)m.mf_tab);
    m.mf_tab = nullptr;
  }
  m.mf_steps = 0;
  if (steps == 0) return 0;
  const size_t n = (size_t)h->E * (size_t)steps * (size_t)m.T;
  // (a byte is the train's malfunction counter field, tb_mf)
  m.mf_tab = h->upload(table, n);
  if (!m.mf_tab) return fail("sfl_set_mf_schedule: device allocation failed");
  m.mf_steps = steps;
  return h->be.sync() ? fail(h->be.error()) : 0;
}

template <class B>
int part_host_access(Handle<B>* h, bool write);

// rng_states: [E][5] (state hi, state lo, inc hi, inc lo, has<<32|buf) — numpy's
// default_rng(seed).bit_generator.state, computed on the host.
template <class B>
int learn_begin(Handle<B>* h, const uint64_t* rng_states) {
  if (int rc = part_host_access(h, true)) return rc;
  const size_t E = h->E;
  std::vector<uint64_t> soa(5 * E);
  for (size_t e = 0; e < E; ++e)
    for (int k = 0; k < 5; ++k) soa[k * E + e] = rng_states[e * 5 + k];
  h->be.h2d(h->st.rng, soa.data(), soa.size() * 8);
  h->be.memset(h->st.counts, 0, (size_t)h->map.S * E * 4);
  h->be.memset(h->st.ep_t, 0, E * 4);
  // every env starts the learn() call with a fresh reset, and no exploit round done yet
  std::vector<int32_t> ph(E, PH_RESET);
  h->be.h2d(h->st.phase, ph.data(), E * 4);
  std::vector<uint32_t> fl(E);
  h->be.d2h(fl.data(), h->st.eflags, E * 4);
  for (auto& f : fl) f &= ~(F_EXPLOIT_DONE | F_INFLIGHT | F_GREEDY);
  h->be.h2d(h->st.eflags, fl.data(), E * 4);
  return h->be.sync() ? fail(h->be.error()) : 0;
}

template <class B>
int test_begin(Handle<B>* h) {
  if (int rc = part_host_access(h, true)) return rc;
  const size_t E = h->E;
  h->be.memset(h->st.n_test, 0, E * 4);
  std::vector<int32_t> ph(E, PH_RESET);
  h->be.h2d(h->st.phase, ph.data(), E * 4);
  return h->be.sync() ? fail(h->be.error()) : 0;
}

template <class B>
int mark_exploit_done(Handle<B>* h) {
  if (int rc = part_host_access(h, true)) return rc;
  const size_t E = h->E;
  std::vector<uint32_t> fl(E);
  h->be.d2h(fl.data(), h->st.eflags, E * 4);
  for (auto& f : fl) f |= F_EXPLOIT_DONE;
  h->be.h2d(h->st.eflags, fl.data(), E * 4);
  return h->be.sync() ? fail(h->be.error()) : 0;
}

// Q-init patch rows (distr_q.py:81-181): the same rows for every env
template <class B>
int apply_qinit(Handle<B>* h, uint32_t n_rows, const uint32_t* row_port, const uint32_t* row_state,
                const double* values /*[n_rows][4], NaN = default_q*/) {
  if (n_rows == 0) return 0;
  uint32_t* d_port = h->template dalloc<uint32_t>(n_rows);
  uint32_t* d_state = h->template dalloc<uint32_t>(n_rows);
  double* d_vals = h->template dalloc<double>((size_t)n_rows * 4);
  if (!d_port || !d_state || !d_vals) return fail("sfl_apply_qinit: allocation failed");
  h->be.h2d(d_port, row_port, n_rows * 4);
  h->be.h2d(d_state, row_state, n_rows * 4);
  h->be.h2d(d_vals, values, (size_t)n_rows * 4 * 8);
  h->be.qinit(h->map, h->st, n_rows, d_port, d_state, d_vals);
  int rc = h->be.sync();
  // release the scratch
  for (int k = 0; k < 3; ++k) {
    h->be.free(h->allocs.back());
    h->allocs.pop_back();
  }
  return rc ? fail(h->be.error()) : 0;
}

// per-launch totals: one device reduction and a 32-byte copy instead of per-env arrays
template <class B>
int reduce_launch(Handle<B>* h) {
  uint64_t out[4] = {0, 0, 0, 0};
  h->be.reduce_launch(h->d_launch_dec, h->d_launch_ticks, h->d_launch_bytes, h->st.err, h->E, h->d_sums);
  h->be.d2h(out, h->d_sums, sizeof out);
  if (h->be.sync()) return fail(h->be.error());
  h->last_dec = out[0];
  h->last_ticks = out[1];
  h->last_bytes = out[2];
  h->last_err = (uint32_t)out[3];
  h->total_dec += out[0];
  return 0;
}

// the per-env error flags, when the launch totals reported any (h->last_err)
// before the host reads (write = false) or writes (true) the per-env scalars of a partitioned handle: the
// wave kernels' blocks copied back into the SflState arrays if they are newer; after a write the next
// part_local copies the arrays into the blocks again
template <class B>
int part_host_access(Handle<B>* h, bool write) {
  if (!h->part.world || !h->part.eblk) return 0;
  if (h->eblk_state == 1) {
    h->be.part_eblk(h->st, h->part, 1);
    if (h->be.sync()) return fail(h->be.error());
    h->eblk_state = 2;
  }
  if (write) h->eblk_state = 0;
  return 0;
}

template <class B>
int scan_errors(Handle<B>* h) {
  if (!h->last_err) return 0;
  if (int rc = part_host_access(h, false)) return rc;
  std::vector<uint32_t> err(h->E);
  h->be.d2h(err.data(), h->st.err, h->E * 4);
  if (h->be.sync()) return fail(h->be.error());
  for (uint32_t e = 0; e < h->E; ++e)
    if (err[e]) {
      char buf[256];
      snprintf(buf, sizeof buf, "env %u: error flags 0x%x (1=inf distance, 2=plan overflow, 4=port mismatch, 8=bad action, "
               "16=message segment overflow, 32=decayed lr beyond the ntab table: raise ntab)",
               e, err[e]);
      return fail(buf);
    }
  return 0;
}

template <class B>
int check_errors(Handle<B>* h) {
  if (int rc = reduce_launch(h)) return rc;
  return scan_errors(h);
}

template <class B>
int run(Handle<B>* h, const SflCtl& c_in, sfl_run_args* args) {
  if (h->part.world) return fail("sfl_run: the handle is graph-partitioned; drive it with sfl_part_*");
  if (h->env_mode) return fail("sfl_run: the handle is in external-action mode (sfl_env_begin); drive it with sfl_env_step");
  SflCtl c = c_in;
  const size_t E = h->E, T = h->map.T;
  const int32_t cap = args ? args->stats_cap : 0;
  std::vector<void*> scratch;
  auto scr = [&](size_t bytes) -> void* {
    void* p = h->be.alloc(bytes ? bytes : 1);
    scratch.push_back(p);
    return p;
  };
  c.stats_cap = cap;
  c.stats_base = c_in.stats_base;
  if (args && cap > 0) {
    c.st_cum = (double*)scr((size_t)cap * E * 8);
    c.st_arrived = (int32_t*)scr((size_t)cap * E * 4);
    c.st_mf = (int32_t*)scr((size_t)cap * E * 4);
    c.st_dec = (int32_t*)scr((size_t)cap * E * 4);
    c.st_ticks = (int32_t*)scr((size_t)cap * E * 4);
    c.st_delays = (int32_t*)scr((size_t)cap * T * E * 4);
    c.sx_cum = (double*)scr((size_t)cap * E * 8);
    c.sx_arrived = (int32_t*)scr((size_t)cap * E * 4);
    for (void* p : scratch)
      if (!p) {
        for (void* q : scratch) h->be.free(q);
        return fail("sfl_run: stats allocation failed");
      }
    h->be.memset(c.sx_cum, 0, (size_t)cap * E * 8);
    h->be.memset(c.sx_arrived, 0, (size_t)cap * E * 4);
  }
  c.launch_dec = h->d_launch_dec;
  c.launch_ticks = h->d_launch_ticks;
  c.launch_bytes = h->d_launch_bytes;
  c.phase_cyc = args ? h->d_phase : nullptr;  // learn / test (not the benchmark's sfl_step): phase timers
  uint64_t* d_trace = nullptr;
  uint64_t* d_trace_n = nullptr;
  if (args && args->trace && args->trace_cap > 0) {
    d_trace = (uint64_t*)scr((size_t)args->trace_cap * 32);
    d_trace_n = (uint64_t*)scr(8);
    if (!d_trace || !d_trace_n) {
      for (void* q : scratch) h->be.free(q);
      return fail("sfl_run: trace allocation failed");
    }
    h->be.memset(d_trace_n, 0, 8);
    c.trace = d_trace;
    c.trace_n = d_trace_n;
    c.trace_env = args->trace_env;
    c.trace_cap = args->trace_cap;
  }
  float ms = 0.f;
  int rc = h->be.run(h->map, h->st, c, h->variant, &ms);
  h->last_kernel_ms = ms;
  if (!rc && args && cap > 0) {
    if (args->cum_reward) h->be.d2h(args->cum_reward, c.st_cum, (size_t)cap * E * 8);
    if (args->arrived) h->be.d2h(args->arrived, c.st_arrived, (size_t)cap * E * 4);
    if (args->malfunctions) h->be.d2h(args->malfunctions, c.st_mf, (size_t)cap * E * 4);
    if (args->decisions) h->be.d2h(args->decisions, c.st_dec, (size_t)cap * E * 4);
    if (args->ticks) h->be.d2h(args->ticks, c.st_ticks, (size_t)cap * E * 4);
    if (args->delays) h->be.d2h(args->delays, c.st_delays, (size_t)cap * T * E * 4);
    if (args->exploit_cum) h->be.d2h(args->exploit_cum, c.sx_cum, (size_t)cap * E * 8);
    if (args->exploit_arrived) h->be.d2h(args->exploit_arrived, c.sx_arrived, (size_t)cap * E * 4);
  }
  if (!rc && d_trace) {
    h->be.d2h(args->trace_n, d_trace_n, 8);
    h->be.d2h(args->trace, d_trace, (size_t)args->trace_cap * 32);
  }
  if (!rc) rc = h->be.sync();
  for (void* p : scratch) h->be.free(p);
  if (rc) return fail(std::string("sfl_run: ") + h->be.error());
  return check_errors(h);
}

// ---------------------------------------------------------------------------
// external-action mode (include/sfl.h sfl_env_begin / sfl_env_step; SflExt in sfl_core.h)
// ---------------------------------------------------------------------------
template <class B>
int env_begin(Handle<B>* h) {
  if (h->part.world) return fail("sfl_env_begin: the handle is graph-partitioned");
  const size_t E = h->E, T = h->map.T, S = h->map.S, NP = h->map.NP;
  if (!h->d_ext) {
    SflExt& x = h->ext;
    x.actions = h->template dalloc<int32_t>(E);
    x.agent = h->template dalloc<int32_t>(E);
    x.train = h->template dalloc<int32_t>(E);
    x.slot = h->template dalloc<int32_t>(E);
    x.state = h->template dalloc<uint32_t>(E);
    x.mask = h->template dalloc<uint32_t>(E);
    x.reward = h->template dalloc<int32_t>(E);
    x.now = h->template dalloc<int32_t>(E);
    x.next_sw = h->template dalloc<int32_t>(E);
    x.step_now = h->template dalloc<int32_t>(E);
    x.arrived = h->template dalloc<uint32_t>(MAXW * E);
    x.n_mf = h->template dalloc<int32_t>(E);
    x.delays = h->template dalloc<int32_t>(T * E);
    x.truncated = h->template dalloc<int32_t>(E);
    h->d_ext = h->template dalloc<SflExt>(1);
    if (!x.actions || !x.agent || !x.train || !x.slot || !x.state || !x.mask || !x.reward || !x.now || !x.next_sw ||
        !x.step_now || !x.arrived || !x.n_mf || !x.delays || !x.truncated || !h->d_ext)
      return fail("sfl_env_begin: allocation failed");
    h->be.h2d(h->d_ext, &h->ext, sizeof(SflExt));
  }
  // a fresh env (a new ASyncSwitchEnv): the lane-per-env body and its state layout, every env at reset
  h->variant = 0;
  h->env_mode = true;
  SflState& st = h->st;
  std::vector<int32_t> ph(E, PH_RESET);
  h->be.h2d(st.phase, ph.data(), E * 4);
  h->be.memset(st.eflags, 0, E * 4);
  h->be.memset(st.elapsed, 0, E * 4);
  h->be.memset(st.epoch, 0, E * 4);
  h->be.memset(st.err, 0, E * 4);
  h->be.memset(st.masks, 0, 4 * MAXW * E * 4);
  h->be.memset(st.tr_pos, 0xFF, T * E * 4);
  h->be.memset(st.tr_bits, 0, T * E * 4);
  h->be.memset(st.tr_plan, 0, T * E * 4);
  h->be.memset(st.tr_next, 0, T * E * 2);
  h->be.memset(st.tr_prev, 0xFF, T * E * 2);
  h->be.memset(st.tr_src, 0xFF, T * E * 2);
  h->be.memset(st.tr_dec, 0, T * E * 2);
  h->be.memset(st.own_n, 0, T * E);
  h->be.memset(st.occ, 0xFF, (size_t)h->map.HW * E);
  h->be.memset(st.claim, 0xFF, (size_t)h->map.HW * E);
  h->be.memset(st.sem, 0, NP * E * 8);
  h->be.memset(st.slot, 0, S * T * E * 8);
  h->be.memset(st.step_ctr, 0, E * 8);
  std::vector<int32_t> none(E, -1);
  h->be.h2d((void*)h->ext.actions, none.data(), E * 4);
  return h->be.sync() ? fail(h->be.error()) : 0;
}

template <class B>
int env_step(Handle<B>* h, sfl_env_io* io) {
  if (!h->env_mode) return fail("sfl_env_step: call sfl_env_begin first");
  if (!io || !io->agent) return fail("sfl_env_step: null argument");
  const size_t E = h->E, T = h->map.T;
  const SflExt& x = h->ext;
  if (io->actions) h->be.h2d((void*)x.actions, io->actions, E * 4);
  else h->be.memset((void*)x.actions, 0xFF, E * 4);
  SflCtl c{};
  c.mode = 2;
  c.ext = h->d_ext;
  c.launch_dec = h->d_launch_dec;
  c.launch_ticks = h->d_launch_ticks;
  c.launch_bytes = h->d_launch_bytes;
  float ms = 0.f;
  if (h->be.run_ext(h->map, h->st, c, &ms)) return fail(std::string("sfl_env_step: ") + h->be.error());
  h->last_kernel_ms = ms;
  auto get = [&](void* dst, const void* src, size_t n) {
    if (dst) h->be.d2h_async(dst, src, n);
  };
  get(io->agent, x.agent, E * 4);
  get(io->train, x.train, E * 4);
  get(io->slot, x.slot, E * 4);
  get(io->state, x.state, E * 4);
  get(io->mask, x.mask, E * 4);
  get(io->reward, x.reward, E * 4);
  get(io->now, x.now, E * 4);
  get(io->next_switch, x.next_sw, E * 4);
  get(io->step_now, x.step_now, E * 4);
  get(io->arrived, x.arrived, MAXW * E * 4);
  get(io->malfunctions, x.n_mf, E * 4);
  get(io->delays, x.delays, T * E * 4);
  get(io->truncated, x.truncated, E * 4);
  if (h->be.sync()) return fail(std::string("sfl_env_step: ") + h->be.error());
  return check_errors(h);
}

}  // namespace sfl

namespace sfl {

// ---------------------------------------------------------------------------
// graph-partitioned mode (sfl_part.h): owned Q storage and one round's three steps
// ---------------------------------------------------------------------------
template <class B>
int part_config(Handle<B>* h, int rank, int world, const int32_t* owner, uint32_t env_base, uint32_t E_tot,
                uint32_t cap_req, uint32_t cap_upd) {
  if (world < 1 || rank < 0 || rank >= world || world > 255) return fail("sfl_part_config: bad rank / world");
  if (h->part.world) return fail("sfl_part_config: already configured");
  if (env_base + h->E > E_tot) return fail("sfl_part_config: env range outside envs_total");
  if (cap_req < h->E) return fail("sfl_part_config: request capacity must hold one request per local env");
  if (cap_upd < 1 || (uint64_t)cap_req + cap_upd >= (1ull << 31) || (uint64_t)world * (cap_req + cap_upd + 1ull) >= (1ull << 32))
    return fail("sfl_part_config: bad capacities");
  // the wave kernel stages up to upd_env update records per env and round (E_MSG_OVF beyond); the
  // segments must hold every env's staged records
  const uint32_t upd_env = cap_upd / h->E < PART_UPD_ENV_MAX ? cap_upd / h->E : PART_UPD_ENV_MAX;
  if (upd_env < 2) return fail("sfl_part_config: update capacity must allow two records per local env");
  const int S = h->map.S, K = h->map.K;
  std::vector<int32_t> own(owner, owner + S);
  for (int s = 0; s < S; ++s)
    if (own[s] < 0 || own[s] >= world) return fail("sfl_part_config: owner out of range");
  std::vector<uint64_t> qo(4 * (size_t)S, 0);
  std::vector<uint32_t> ro(4 * (size_t)S, 0);
  uint64_t off = 0;
  uint32_t rows = 0;
  for (int s = 0; s < S; ++s) {
    if (own[s] != rank) continue;
    const int P = h->h_sw_np[s];
    for (int i = 0; i < P; ++i) {
      const int g = 4 * s + i;
      const uint32_t nrows = (uint32_t)(1u << P) * (uint32_t)K * 3u;
      qo[g] = off;
      ro[g] = rows;
      off += (uint64_t)nrows * h->h_q_w[g];
      rows += nrows;
    }
  }
  // the env-local Q-table is not used in this mode: release it before the owned tables
  h->be.sync();
  h->dfree(h->st.q);
  h->dfree(h->st.touched);
  h->st.q = nullptr;
  h->st.touched = nullptr;
  SflPart& P = h->part;
  P.rank = rank;
  P.world = world;
  P.n_sw = S;
  P.env_base = env_base;
  P.E_tot = E_tot;
  // a segment holds one group per env of a source rank: its request and its update records to this
  // destination (cap_req >= the largest rank's env count, cap_upd its update records)
  P.cap_msg = cap_req + cap_upd;
  P.k_msg = P.cap_msg;  // (full segments until sfl_part_set_caps)
  P.q_own_per_env = off;
  P.own_rows = rows;
  P.own_words = (rows + 31u) / 32u;
  P.owner = h->upload(own.data(), own.size());
  std::vector<uint32_t> loc(S);
  for (int s = 0; s < S; ++s) loc[s] = own[s] == rank ? 1u : 0u;
  P.local_sw = h->upload(loc.data(), loc.size());
  P.q_off_own = h->upload(qo.data(), qo.size());
  P.row_own = h->upload(ro.data(), ro.size());
  P.q_own = h->template dalloc<double>((size_t)E_tot * (off ? off : 1));
  P.touched_own = h->template dalloc<uint32_t>((size_t)E_tot * (P.own_words ? P.own_words : 1));
  P.obs = h->template dalloc<Obs>(h->E);
  P.req_ix = h->template dalloc<uint32_t>(h->E);
  P.dec_done = h->template dalloc<int64_t>(h->E);
  P.cnt = h->template dalloc<uint32_t>((size_t)world + 4);
  P.sums = h->d_sums;
  P.cnt_out = h->template dalloc<uint64_t>(4 + ((size_t)PART_NCNT(world) + 1) / 2);
  P.upd_env = upd_env;
  P.req_st = h->template dalloc<PartReq>(h->E);
  P.req_dst = h->template dalloc<int32_t>(h->E);
  P.upd_st = h->template dalloc<PartUpd>((size_t)h->E * upd_env);
  P.upd_n = h->template dalloc<uint32_t>(h->E);
  P.eblk = nullptr;
  if (!P.owner || !P.q_own || !P.touched_own || !P.obs || !P.req_ix || !P.dec_done || !P.cnt || !P.cnt_out || !P.req_st ||
      !P.req_dst || !P.upd_st || !P.upd_n)
    return fail("sfl_part_config: allocation failed (out of memory?)");
  P.blocks_done = P.cnt + world;
  h->be.memset(P.cnt, 0, ((size_t)world + 4) * 4);
  h->be.memset(P.sums, 0, 4 * 8);
  h->be.memset(P.cnt_out, 0, (4 + ((size_t)PART_NCNT(world) + 1) / 2) * 8);
  h->be.fill_f64(P.q_own, h->map.default_q, (size_t)E_tot * off);
  h->be.memset(P.touched_own, 0, (size_t)E_tot * P.own_words * 4);
  h->be.memset(P.dec_done, 0, h->E * 8);
  // a grouped shape (G < 64) becomes its one-env-per-wavefront shape: same env-major state layout
  if (h->variant > 0 && kVariants[h->variant].G != 64) h->variant = wave64_variant(h->map.S, h->map.T);
  if (h->variant > 0) {  // the wave kernels keep each env's scalars in a block between rounds
    P.eblk = h->template dalloc<uint32_t>((size_t)h->E * PART_EB);
    if (!P.eblk) return fail("sfl_part_config: allocation failed (out of memory?)");
  }
  h->eblk_state = 0;
  // the partitioned rounds run the body the handle was created for (h->variant: k_wave where
  // eligible, else the lane-per-env body), with that body's (switch, train) slot layout
  return h->be.sync() ? fail(h->be.error()) : 0;
}

// Q-init patch rows on the owned blocks (sfl_apply_qinit for a partitioned handle)
template <class B>
int part_qinit(Handle<B>* h, uint32_t n_rows, const uint32_t* row_port, const uint32_t* row_state, const double* values) {
  SflPart& P = h->part;
  const int rank = P.rank;
  std::vector<int32_t> own(h->map.S);
  h->be.d2h(own.data(), P.owner, own.size() * 4);
  if (h->be.sync()) return fail(h->be.error());
  // apply on the host copy of one env's owned table, then replicate over all envs
  std::vector<uint64_t> qo(4 * (size_t)h->map.S);
  std::vector<uint32_t> ro(4 * (size_t)h->map.S);
  h->be.d2h(qo.data(), P.q_off_own, qo.size() * 8);
  h->be.d2h(ro.data(), P.row_own, ro.size() * 4);
  if (h->be.sync()) return fail(h->be.error());
  std::vector<double> tab(P.q_own_per_env, h->map.default_q);
  std::vector<uint32_t> bits(P.own_words, 0u);
  for (uint32_t r = 0; r < n_rows; ++r) {
    const uint32_t g = row_port[r], st = row_state[r];
    if (own[g >> 2] != rank) continue;
    const int w = h->h_q_w[g];
    for (int j = 0; j < w; ++j) {
      const double v = values[(size_t)r * 4 + j];
      tab[qo[g] + (size_t)st * w + j] = (v != v) ? h->map.default_q : v;
    }
    const uint32_t rid = ro[g] + st;
    bits[rid >> 5] |= 1u << (rid & 31u);
  }
  // one env's owned table and key set, replicated over every env of the job
  if (P.q_own_per_env) {
    h->be.h2d(P.q_own, tab.data(), tab.size() * 8);
    h->be.replicate(P.q_own, tab.size() * 8, P.E_tot);
  }
  if (P.own_words) {
    h->be.h2d(P.touched_own, bits.data(), bits.size() * 4);
    h->be.replicate(P.touched_own, bits.size() * 4, P.E_tot);
  }
  return h->be.sync() ? fail(h->be.error()) : 0;
}

// one env of the job (global index): its owned Q blocks in the full per-env layout (other
// entries untouched) and its owned key-set bits OR-ed into `touched`
template <class B>
int part_get_q(Handle<B>* h, uint32_t genv, double* q, uint32_t* touched) {
  SflPart& P = h->part;
  if (genv >= P.E_tot) return fail("sfl_part_get_q: env out of range");
  std::vector<int32_t> own(h->map.S);
  std::vector<uint64_t> qo(4 * (size_t)h->map.S);
  std::vector<uint32_t> ro(4 * (size_t)h->map.S);
  std::vector<double> tab(P.q_own_per_env);
  std::vector<uint32_t> bits(P.own_words);
  h->be.d2h(own.data(), P.owner, own.size() * 4);
  h->be.d2h(qo.data(), P.q_off_own, qo.size() * 8);
  h->be.d2h(ro.data(), P.row_own, ro.size() * 4);
  if (P.q_own_per_env) h->be.d2h(tab.data(), P.q_own + (size_t)genv * P.q_own_per_env, tab.size() * 8);
  if (P.own_words) h->be.d2h(bits.data(), P.touched_own + (size_t)genv * P.own_words, bits.size() * 4);
  if (h->be.sync()) return fail(h->be.error());
  const int K = h->map.K;
  for (int s = 0; s < h->map.S; ++s) {
    if (own[s] != P.rank) continue;
    const int np = h->h_sw_np[s];
    for (int i = 0; i < np; ++i) {
      const int g = 4 * s + i;
      const uint32_t nrows = (uint32_t)(1u << np) * (uint32_t)K * 3u;
      const int w = h->h_q_w[g];
      if (q) memcpy(q + h->h_q_off[g], tab.data() + qo[g], (size_t)nrows * w * 8);
      if (touched)
        for (uint32_t r = 0; r < nrows; ++r) {
          const uint32_t lr = ro[g] + r;
          if ((bits[lr >> 5] >> (lr & 31u)) & 1u) {
            const uint32_t fr = h->h_row_base[g] + r;
            touched[fr >> 5] |= 1u << (fr & 31u);
          }
        }
    }
  }
  return 0;
}

template <class B>
int part_begin(Handle<B>* h) {
  if (!h->part.world) return fail("sfl_part_begin: handle not partitioned");
  if (int rc = part_host_access(h, true)) return rc;
  h->be.memset(h->part.dec_done, 0, h->E * 8);
  return h->be.sync() ? fail(h->be.error()) : 0;
}

// this round's segment size (records per destination, without the header): the buffers handed to the
// next rounds hold [world][k + 1] records.  Every rank of the job must use the same value.
template <class B>
int part_set_caps(Handle<B>* h, uint32_t k_msg) {
  SflPart& P = h->part;
  if (!P.world) return fail("sfl_part_set_caps: handle not partitioned");
  if (k_msg < 1 || k_msg > P.cap_msg) return fail("sfl_part_set_caps: capacity outside [1, the configured capacity]");
  P.k_msg = k_msg;
  h->be.part_caps(P);
  return h->be.error()[0] ? fail(std::string("sfl_part_set_caps: ") + h->be.error()) : 0;
}

// the host copy of the last part_local's record counts, of the peaks and deferrals and of the launch
// totals accumulated since the previous read: a checkpoint's one synchronisation
template <class B>
int part_read(Handle<B>* h) {
  SflPart& P = h->part;
  std::vector<uint64_t> out(4 + ((size_t)PART_NCNT(P.world) + 1) / 2);
  h->be.d2h_async(out.data(), P.cnt_out, out.size() * 8);
  h->be.memset(P.cnt_out, 0, out.size() * 8);
  if (h->be.sync()) return fail(std::string("sfl_part_local: ") + h->be.error());
  h->part_pending = false;
  h->part_reads++;
  h->last_kernel_ms = h->be.elapsed_ms();
  h->last_dec = out[0];
  h->last_ticks = out[1];
  h->last_bytes = out[2];
  h->last_err = (uint32_t)out[3];
  h->total_dec += out[0];
  const uint32_t* cnt = (const uint32_t*)(out.data() + 4);
  const int W = P.world;
  std::vector<uint32_t> prev;
  if (!h->part_consumed) prev.swap(h->part_counts);  // (peaks and deferrals since sfl_part_counts: merged)
  h->part_counts.assign(cnt, cnt + PART_NCNT(W));
  if (prev.size() == h->part_counts.size()) {
    for (int i = PART_C_PEAK(W); i < PART_C_OPEN(W); ++i) h->part_counts[i] = std::max(h->part_counts[i], prev[i]);
    h->part_counts[PART_C_DEFER_SUM(W)] += prev[PART_C_DEFER_SUM(W)];
  }
  h->part_consumed = false;
  return scan_errors(h);
}

// local step of a round: every env applies its reply, runs to its next decision and emits the
// request (and the update records of its post step).  With n_req, one host synchronisation for
// the record counts and launch totals; without it on the caller's stream (sfl_set_stream), none:
// sfl_part_counts reads them later (errors of the envs surface there)
template <class B>
int part_local(Handle<B>* h, int64_t budget, const void* rep_in, void* msg_out, uint64_t* n_req) {
  SflPart& P = h->part;
  if (!P.world) return fail("sfl_part_local: handle not partitioned");
  P.rep_in = (const PartRep*)rep_in;
  P.msg_out = (PartMsg*)msg_out;
  SflCtl c{};
  c.mode = 0;
  c.ep_target = -1;
  c.dec_budget = budget;
  c.launch_dec = h->d_launch_dec;
  c.launch_ticks = h->d_launch_ticks;
  c.launch_bytes = h->d_launch_bytes;
  float ms = 0.f;
  if (P.eblk && h->eblk_state == 0) h->be.part_eblk(h->st, P, 0);  // (stream-ordered before the launch)
  if (h->be.part_local(h->map, h->st, c, P, h->variant, &ms)) return fail(std::string("sfl_part_local: ") + h->be.error());
  if (P.eblk) h->eblk_state = 1;
  h->part_pending = true;
  if (!n_req) return 0;  // (sfl_part_counts reads them)
  if (int rc = part_read(h)) return rc;
  if (n_req) *n_req = h->part_counts[PART_C_OPEN(P.world)];
  return 0;
}

// the owner steps are queued without a synchronisation when the caller's stream carries the
// round (sfl_set_stream): launch errors still surface, kernel faults at the next synchronisation
template <class B>
int part_done(Handle<B>* h, const char* what) {
  if (h->ext_stream) return h->be.error()[0] ? fail(std::string(what) + ": " + h->be.error()) : 0;
  return h->be.sync() ? fail(std::string(what) + ": " + h->be.error()) : 0;
}

// the owner side of a round on the received segments: each env's update records in order, then the
// answer to its request (sfl_part.h part_owner_group)
template <class B>
int part_owner(Handle<B>* h, const void* msg_in, void* rep_out) {
  SflPart& P = h->part;
  if (!P.world) return fail("sfl_part_owner: handle not partitioned");
  h->be.part_owner(h->map, P, (const PartMsg*)msg_in, (PartRep*)rep_out);
  return part_done(h, "sfl_part_owner");
}

// which switches' rows the wave kernel decides on and updates directly: local[S] (null: the
// switches this rank owns, the default), the rest through their owners' messages.  Rows of
// another rank's switch cannot be local; marking fewer of this rank's own switches local
// rehearses a bigger job's message traffic on one rank.  The lane-per-env body always sends.
template <class B>
int part_set_local_rows(Handle<B>* h, const uint8_t* local) {
  SflPart& P = h->part;
  if (!P.world) return fail("sfl_part_set_local_rows: handle not partitioned");
  const int S = h->map.S;
  std::vector<int32_t> own(S);
  h->be.d2h(own.data(), P.owner, own.size() * 4);
  if (h->be.sync()) return fail(h->be.error());
  std::vector<uint32_t> loc(S);
  for (int s = 0; s < S; ++s) {
    const bool want = local ? local[s] != 0 : own[s] == P.rank;
    if (want && own[s] != P.rank) return fail("sfl_part_set_local_rows: switch owned by another rank marked local");
    loc[s] = want ? 1u : 0u;
  }
  h->be.h2d((void*)P.local_sw, loc.data(), loc.size() * 4);
  return h->be.sync() ? fail(h->be.error()) : 0;
}

// this rank's counts (sfl_part.h PART_C_*): of the last part_local, message records staged per destination,
// then their peaks per destination since the previous read, that round's open and deferred envs and the
// deferrals since the previous read.  cap >= world (the first counts only)
template <class B>
int part_counts(Handle<B>* h, uint32_t* out, int32_t cap) {
  if (!h->part.world) return fail("sfl_part_counts: handle not partitioned");
  const int32_t n = PART_NCNT(h->part.world);
  if (cap < h->part.world) return fail("sfl_part_counts: buffer too small");
  if (h->part_pending)
    if (int rc = part_read(h)) return rc;
  for (int32_t i = 0; i < n && i < cap; ++i) out[i] = i < (int32_t)h->part_counts.size() ? h->part_counts[i] : 0u;
  h->part_consumed = true;
  return 0;
}

}  // namespace sfl
