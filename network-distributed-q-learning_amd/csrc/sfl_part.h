// Graph-partitioned mode (BASELINE.json configs[4], SURVEY.md §8(e) "C5"): the switch agents
// are partitioned over the ranks, and each rank stores the Q rows of the switches it owns,
// for every env of the job.  Envs are sharded over the ranks as in the env-sharded mode; an
// env's decision at switch s asks owner(s) for the Q row (argmax and max), and its post step
// sends the Q update of the pending (switch, train) entry -- the bootstrap from the successor
// agent's row, distr_q.py:419-447 -- to owner(previous switch).  That is the reference's
// network-distributed learner with the successor-Q values crossing GPU boundaries.
//
// One round = every local env makes (at most) one decision:
//   local    (env_run_part): apply the reply of the previous round's request, continue the
//            env (post, ticks, episode ends) up to the next decision, observe it and stage its
//            request; post steps stage update records
//   compact  (k_part_compact): the staged records into ONE message segment per destination rank,
//            each env's records for that destination as a contiguous group (its update records in
//            emission order, then its request); at most k_msg records per segment: an env with a group
//            that does not fit is deferred whole (F_DEFER: it sends nothing this round and sits out the
//            next local step, its staged records go again), so the segments have a fixed size and the
//            exchange needs no counts from the host
//   exchange the message segments (one RCCL all-to-all; segment per destination rank)
//   owner    (part_owner_group): per received group, the env's updates in order, then the answer to
//            its request (max(row) and the masked argmax) -- one kernel, no stage ordering across
//            the segment: an env's records touch only that env's rows, and a group is walked in order
//   exchange the replies (the same segment layout, back to the requesters)
// Each env's own sequence of operations is that of env_run (sfl_core.h), so the results are
// bit-identical to the fused kernels (tests/test_partition.py).
#pragma once
#include "sfl_core.h"

namespace sfl {

enum : uint32_t { F_REQ = 64 };     // eflags: a request is waiting for its reply
enum : uint32_t { F_DEFER = 256 };  // eflags: the env's staged records did not fit this round's segments
enum : uint32_t { E_MSG_OVF = 16 };  // a message segment overflowed (capacity too small)
constexpr uint32_t PART_UPD_ENV_MAX = 16;  // staged update records per env and round, at most

// The wave kernel's per-env scalars between rounds (SflPart::eblk, [E][PART_EB] words, env-major): one
// coalesced load and one store per env and round instead of ~30 single-word accesses to as many [field][E]
// arrays, each a partial cache line (round 3: 67 of 115 write requests per env and round).  The canonical
// SflState arrays are refreshed from the block when the host reads them (part_sync) and copied into it at
// sfl_part_begin (k_part_eblk).  Word offsets:
enum : int {
  EB_PHASE = 0, EB_ELAPSED = 1, EB_EFLAGS = 2, EB_EPOCH = 3, EB_ERR = 4, EB_EP_T = 5, EB_N_TEST = 6, EB_N_MF = 7,
  EB_EP_DEC = 8, EB_EP_TICKS = 9, EB_STEP_CTR = 10 /* 2 */, EB_DEC_TOTAL = 12 /* 2 */, EB_CUM = 14 /* 2, f64 */,
  EB_RNG = 16 /* 5 x 2 */, EB_MASKS = 26 /* 4 x MAXW */, EB_DEC_DONE = 42 /* 2 */, EB_REQ_DST = 44, EB_UPD_N = 45,
  EB_L_DEC = 46 /* 2 */, EB_L_TICKS = 48 /* 2 */, EB_L_BYTES = 50 /* 2 */, EB_USED = 52
};
constexpr int PART_EB = 64;

// staged records (the env's own slots: its request, its update records) and the 32-byte message
// record of the segments; record 0 of each destination segment is a header whose first word is the
// number of records that follow
struct PartReq {
  uint32_t genv;   // global env index
  uint16_t port;   // 4 * switch + in-port slot (the row's block)
  uint16_t amask;  // allowed actions (get_action_mask)
  uint32_t state;  // observation state index within the block
  uint32_t flags;  // 1: exploratory action (no argmax, no key-set insert)
};
struct PartRep {
  int32_t action;  // masked argmax (distr_q.py:468-490); -1 for exploratory requests
  int32_t pad;
  double mq;       // max over the full row (distr_q.py:449-466)
};
struct PartUpd {
  uint32_t genv;
  uint16_t port;
  uint8_t j;      // compact column
  uint8_t stage;  // 0: pending update / key-set inserts; 1 + i: bonus of the i-th arrived train (emission order)
  uint32_t state;
  uint32_t kind;  // 0: q <- (1 - lr) q + lr target;  1: key-set insert only
  double lr;
  double target;
};
// a segment record (32 B): an update record (MSG_UPD / MSG_INSERT, the PartUpd fields) or a request
// (MSG_REQ / MSG_REQ_X: genv, port, state as PartReq, amask in `j | stage << 8`).  kind bits 8-15: the
// length of the env's group, bits 16-23: the record's place in it (its group starts pos records before it);
// a deferred env's places below the segment end carry MSG_VOID records (groups of one).
enum : uint32_t { MSG_UPD = 0u, MSG_INSERT = 1u, MSG_VOID = 2u, MSG_REQ = 3u, MSG_REQ_X = 4u };
typedef PartUpd PartMsg;
SFL_FN constexpr uint32_t msg_type(uint32_t kind) { return kind & 0xFFu; }
SFL_FN constexpr uint32_t msg_group(uint32_t kind) { return (kind >> 8) & 0xFFu; }
SFL_FN constexpr uint32_t msg_pos(uint32_t kind) { return (kind >> 16) & 0xFFu; }
SFL_FN constexpr uint32_t msg_tag(uint32_t len, uint32_t pos) { return (len << 8) | (pos << 16); }
static_assert(sizeof(PartReq) == 16 && sizeof(PartRep) == 16 && sizeof(PartUpd) == 32, "record sizes");
constexpr uint32_t PART_GROUP_MAX = PART_UPD_ENV_MAX + 1;  // records of one env in one segment, at most

struct SflPart {
  int32_t rank, world;
  int32_t n_sw;               // switches of the map (owner[] entries)
  const uint32_t* local_sw;   // [S] 1: the wave kernel reads / writes this switch's rows here directly
                              // (its owner is this rank; all 0: every row operation as a message)
  uint32_t env_base;  // global index of local env 0
  uint32_t E_tot;     // envs over all ranks
  uint32_t cap_msg;           // records per destination segment (without the header), at most:
                              // one request and PART_UPD_ENV_MAX update records per env of the largest rank
  uint32_t k_msg;             // this round's records per destination segment (<= cap_msg; the segments
                              // of a buffer are k_msg + 1 records apart): sfl_part_set_caps
  uint64_t q_own_per_env;     // doubles of owned Q per env
  uint32_t own_rows, own_words;
  const int32_t* owner;       // [S] rank owning each switch agent
  const uint64_t* q_off_own;  // [4S] block offset in the owned table (owned switches only)
  const uint32_t* row_own;    // [4S] first owned row id of the block
  double* q_own;              // [E_tot][q_own_per_env]
  uint32_t* touched_own;      // [E_tot][own_words]
  Obs* obs;                   // [E] observation waiting for its reply
  uint32_t* req_ix;           // [E] record index of that request's reply in the reply buffer
  int64_t* dec_done;          // [E] decisions since sfl_part_begin
  uint32_t* cnt;              // [world] message records staged this round (sent or not), then
                              // blocks_done, open envs, deferred envs
  uint32_t* blocks_done;      // [1] k_part_compact's finished blocks (the last one writes the headers)
  uint64_t* sums;             // [4] this round's launch totals (decisions, ticks, bytes, error bits OR)
  uint64_t* cnt_out;          // [4 + PART_NCNT(world) / 2]: sums, then the counts as u32 (PART_C_*): what the
                              // host reads at a checkpoint (the peaks and the deferral total since the last one)
  // the wave kernel's per-env staging of a round's messages (k_part_compact packs them into the
  // segments): no record index is taken with a contended atomic counter in the env kernel
  PartReq* req_st;            // [E] the env's request of this round
  int32_t* req_dst;           // [E] its destination rank, -1: no request (lane-per-env body; the wave
                              // kernels keep it in eblk)
  PartUpd* upd_st;            // [E][upd_env] the env's update records of this round
  uint32_t* upd_n;            // [E] how many (lane-per-env body)
  uint32_t upd_env;           // staged update records per env and round (E_MSG_OVF beyond)
  uint32_t* eblk;             // [E][PART_EB] the wave kernel's per-env scalars between rounds (null: the
                              // lane-per-env body, which keeps the SflState arrays)
  // round buffers (set per call)
  const PartRep* rep_in;      // [world][k_msg + 1] (a reply sits at its request's record index)
  PartMsg* msg_out;           // [world][k_msg + 1]
};

// the counts a checkpoint reads (sfl_part_counts), u32 words after the four launch totals of cnt_out
SFL_FN constexpr int PART_C_MSG(int) { return 0; }                    // [world] message records staged this round
SFL_FN constexpr int PART_C_PEAK(int w) { return w; }                 // [world] peak of C_MSG since the read
SFL_FN constexpr int PART_C_OPEN(int w) { return 2 * w; }             // envs with a request or deferred
SFL_FN constexpr int PART_C_DEFER(int w) { return 2 * w + 1; }        // envs deferred this round
SFL_FN constexpr int PART_C_DEFER_SUM(int w) { return 2 * w + 2; }    // deferrals since the read
SFL_FN constexpr int PART_NCNT(int w) { return 2 * w + 3; }

SFL_FN void fetch_or_u32(uint32_t* p, uint32_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
  atomicOr(p, v);
#else
  __atomic_fetch_or(p, v, __ATOMIC_RELAXED);
#endif
}
// the post step's Q operations as update records to the owner of the row's switch, staged in the
// env's update slots (k_part_compact / the host build's part_compact give them their segment places)
template <class V>
struct MsgQ {
  V& v;
  const SflPart& P;
  uint32_t e, genv;
  uint32_t& n;  // records staged so far this round
  double mq;    // max of the decision's own row, from the owner's reply
  SFL_FN void emit(int sw, int slot, uint32_t state, int j, uint32_t kind, double lr, double target, int stage) {
    if (n >= P.upd_env || stage > 254) {  // (the record's stage field is 8 bits)
      v.err |= E_MSG_OVF;
      return;
    }
    PartUpd& u = P.upd_st[(size_t)e * P.upd_env + n++];
    u.genv = genv;
    u.port = (uint16_t)(4 * sw + slot);
    u.j = (uint8_t)j;
    u.stage = (uint8_t)stage;
    u.state = state;
    u.kind = kind;
    u.lr = lr;
    u.target = target;
  }
  SFL_FN void touch(int sw, int slot, uint32_t state) { emit(sw, slot, state, 0, 1u, 0.0, 0.0, 0); }
  SFL_FN double row_max_of(const Decision&) { return mq; }
  SFL_FN void update(int ps, int pslot, uint32_t pstate, int pj, double lr, double target, int stage) {
    emit(ps, pslot, pstate, pj, 0u, lr, target, stage);
  }
};

// the map as row_max / max_action see it
struct MapView {
  const SflMap& m;
};

// a request as a segment record and back (sfl_part.h PartMsg: amask in j | stage << 8)
SFL_FN PartMsg msg_of_req(const PartReq& r) {
  PartMsg x;
  x.genv = r.genv;
  x.port = r.port;
  x.j = (uint8_t)(r.amask & 0xFFu);
  x.stage = (uint8_t)(r.amask >> 8);
  x.state = r.state;
  x.kind = (r.flags & 1u) ? MSG_REQ_X : MSG_REQ;
  x.lr = 0.0;
  x.target = 0.0;
  return x;
}
SFL_FN PartReq req_of_msg(const PartMsg& x) {
  PartReq r;
  r.genv = x.genv;
  r.port = x.port;
  r.amask = (uint16_t)(x.j | ((uint32_t)x.stage << 8));
  r.state = x.state;
  r.flags = msg_type(x.kind) == MSG_REQ_X ? 1u : 0u;
  return r;
}

// owner side: one request -> reply (distr_q.py:449-490 on the owned row)
SFL_FN void part_answer_one(const SflMap& m, const SflPart& P, const PartReq& r, PartRep& out) {
  const int port = r.port, sw = port >> 2, slot = port & 3;
  const double* row = P.q_own + (size_t)r.genv * P.q_own_per_env + P.q_off_own[port] + (size_t)r.state * m.q_w[port];
  const MapView mv{m};
  out.mq = row_max(mv, sw, slot, row);
  out.pad = 0;
  if (r.flags & 1u) {
    out.action = -1;
  } else {
    const uint32_t rid = P.row_own[port] + r.state;
    fetch_or_u32(&P.touched_own[(size_t)r.genv * P.own_words + (rid >> 5)], 1u << (rid & 31u));
    out.action = max_action(mv, sw, slot, row, r.amask);
  }
}

// owner side: one update record (MSG_UPD: the bootstrapped update and the key-set insert; MSG_INSERT: the
// insert only)
SFL_FN void part_update_one(const SflMap& m, const SflPart& P, const PartUpd& u) {
  const int port = u.port;
  const uint32_t rid = P.row_own[port] + u.state;
  fetch_or_u32(&P.touched_own[(size_t)u.genv * P.own_words + (rid >> 5)], 1u << (rid & 31u));
  if (msg_type(u.kind) == MSG_UPD) {
    double* q = P.q_own + (size_t)u.genv * P.q_own_per_env + P.q_off_own[port] + (size_t)u.state * m.q_w[port] + u.j;
    const double a = (1.0 - u.lr) * *q;
    const double bb = u.lr * u.target;
    *q = a + bb;
  }
}

// owner side: one env's group of a received segment, in order -- its update records as the env emitted
// them (the pending update, key-set inserts, arrival bonuses: distr_q.py:325-362), then the answer to its
// request, which may read a row those updates just wrote.  An env's records touch only that env's rows
// (q_own / touched_own of its genv), so groups are independent of each other.  (The host build walks a
// group like this; k_part_owner applies a block's groups by update stage -- records of one stage touch
// distinct cells of their env -- then answers, which is the same order per env.)
template <class Answer>
SFL_FN void part_owner_group(const SflMap& m, const SflPart& P, const PartMsg* g, uint32_t len, PartRep* rep,
                             Answer&& answer) {
  for (uint32_t i = 0; i < len; ++i) {
    const uint32_t t = msg_type(g[i].kind);
    if (t == MSG_UPD || t == MSG_INSERT) part_update_one(m, P, g[i]);
    else if (t == MSG_REQ || t == MSG_REQ_X) answer(req_of_msg(g[i]), rep[i]);
  }
}

// sender side: an env's staged records grouped per destination (k_part_compact, the host build's
// part_compact).  Record r < nu is update r, to the owner of its row's switch (dst[r], filled by the caller);
// record nu the request, to rd (if rd >= 0); dst = -1 past the last.  For each destination the env writes to,
// reserve(d, size) returns the place of its group in d's segment; place[r] = that + the record's place in the
// group (emission order, so the request comes last), pos[r] its place in the group, size[r] the group's length.
// Returns the number of records.  (One pass per destination the env writes to -- usually one or two -- over
// bit masks.)
template <class Reserve>
SFL_FN uint32_t env_groups(int rd, uint32_t nu, int32_t (&dst)[PART_GROUP_MAX], uint32_t (&pos)[PART_GROUP_MAX],
                           uint32_t (&size)[PART_GROUP_MAX], uint32_t (&place)[PART_GROUP_MAX], Reserve&& reserve) {
  const uint32_t n = nu + (rd >= 0 ? 1u : 0u);
#pragma unroll
  for (uint32_t r = 0; r < PART_GROUP_MAX; ++r) {
    dst[r] = r < nu ? dst[r] : (r == nu && rd >= 0) ? rd : -1;
    pos[r] = size[r] = place[r] = 0u;
  }
  uint32_t left = (1u << n) - 1u;  // (n <= 17)
  while (left) {
    const uint32_t r0 = (uint32_t)__builtin_ctz(left);
    int32_t d = -1;
#pragma unroll
    for (uint32_t q = 0; q < PART_GROUP_MAX; ++q) d = q == r0 ? dst[q] : d;
    uint32_t mk = 0u;
#pragma unroll
    for (uint32_t q = 0; q < PART_GROUP_MAX; ++q) mk |= (q < n && dst[q] == d) ? (1u << q) : 0u;
    const uint32_t z = (uint32_t)__builtin_popcount(mk);
    const uint32_t b = reserve(d, z);
#pragma unroll
    for (uint32_t q = 0; q < PART_GROUP_MAX; ++q) {
      if ((mk >> q) & 1u) {
        pos[q] = (uint32_t)__builtin_popcount(mk & ((1u << q) - 1u));
        size[q] = z;
        place[q] = b + pos[q];
      }
    }
    left &= ~mk;
  }
  return n;
}

// local side: one env for one round (env_run of sfl_core.h, with the Q row operations sent to
// their owners).  Stops after staging the next decision's request, or when the env has made
// its decisions for this part_step (c.dec_budget) or reached its episode target.  A deferred env
// (F_DEFER: its records did not fit the last round's segments) sits the round out unchanged.
template <int NW>
SFL_FN void env_run_part(const SflMap& m, const SflState& s, const SflCtl& c, const SflPart& P, uint32_t e) {
  if (s.eflags[e] & F_DEFER) return;
  using V = Env<NW>;
  V v(m, s, e);
  uint32_t n_upd = 0;
  P.req_dst[e] = -1;
  v.flags = s.eflags[e];
  v.now = s.elapsed[e];
  v.epoch = s.epoch[e];
  v.err = s.err[e];
  int32_t phase = s.phase[e];
  int64_t dec = P.dec_done[e];
  uint64_t ticks = 0, abytes = 0, ndec = 0;
  Decision d;
  d.sw = d.h = d.slot = d.action = d.j = d.reward = d.next_sw = 0;
  d.state = 0;
  double mq_cur = 0.0;
  double cum = s.cum_reward[e];
  const bool test_mode = c.mode == 1;
  const uint32_t genv = P.env_base + e;
  v.masks_load();
  while (true) {
    if (phase == PH_RESET) {
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
      int live = m.T;
#pragma unroll
      for (int w = 0; w < V::kNW; ++w) live -= popc32(v.msk[1][w]);
      abytes += 36ull * (uint64_t)live;
      env_tick(v);
      ticks++;
      if (v.flags & F_TERM) phase = (v.flags & F_INFLIGHT) ? PH_POST : PH_END;
      else if (!queue_empty(v)) phase = (v.flags & F_INFLIGHT) ? PH_POST : PH_DECIDE;
    } else if (phase == PH_DECIDE || phase == PH_POST) {
      bool post_now = phase == PH_POST;
      if (phase == PH_DECIDE) {
        const bool greedy = (v.flags & F_GREEDY) != 0;
        if (!(v.flags & F_REQ)) {
          if (c.dec_budget > 0 && dec >= c.dec_budget) break;
          Obs o;
          decide_observe(v, o, greedy);
          PartReq& r = P.req_st[e];
          r.genv = genv;
          r.port = (uint16_t)(4 * o.sw + o.slot);
          r.amask = (uint16_t)o.amask;
          r.state = o.state;
          r.flags = o.explore ? 1u : 0u;
          P.req_dst[e] = P.owner[o.sw];
          P.obs[e] = o;
          v.flags |= F_REQ;
          break;  // the round ends here: the owner answers before this env goes on
        }
        v.flags &= ~F_REQ;
        const Obs o = P.obs[e];
        const PartRep& rp = P.rep_in[P.req_ix[e]];
        mq_cur = rp.mq;
        decide_apply(v, o, o.explore ? o.action : rp.action, d);
        abytes += 220ull + 48ull * m.sw_np[d.sw] + 8ull * m.sw_na[d.sw];
        v.flags |= F_INFLIGHT;
        if (queue_empty(v)) phase = PH_TICK;  // ticks happen between the step and the update
        else post_now = true;
      }
      if (post_now) {
        if (!(v.flags & F_GREEDY)) {
          MsgQ<V> q{v, P, e, genv, n_upd, mq_cur};
          env_post(v, d, q);
        }
        v.flags &= ~F_INFLIGHT;
        cum += (double)d.reward;
        s.ep_dec[e] += 1;
        s.dec_total[e] += 1;
        s.step_ctr[e] += 1;
        if (s.step_ctr[e] > m.max_steps) v.flags |= F_TRUNC;
        dec++;
        ndec++;
        phase = (v.flags & (F_TERM | F_TRUNC)) ? PH_END : PH_DECIDE;
        if (c.dec_budget > 0 && dec >= c.dec_budget) break;
      }
    } else {  // PH_END
      int arrived = 0;
#pragma unroll
      for (int w = 0; w < V::kNW; ++w) arrived += popc32(v.msk[1][w]);
      const size_t cap = (size_t)(c.stats_cap > 0 ? c.stats_cap : 1);
      const bool greedy = (v.flags & F_GREEDY) != 0;
      if (c.st_cum && c.stats_cap > 0 && (!greedy || test_mode)) {
        const int32_t i = (greedy && test_mode) ? s.n_test[e] : s.ep_t[e];
        const size_t row = (size_t)(i - c.stats_base) % cap;
        c.st_cum[row * s.E + e] = cum;
        c.st_arrived[row * s.E + e] = arrived;
        c.st_mf[row * s.E + e] = s.n_mf[e];
        c.st_dec[row * s.E + e] = s.ep_dec[e];
        c.st_ticks[row * s.E + e] = s.ep_ticks[e];
        for (int h = 0; h < m.T; ++h) c.st_delays[(row * m.T + h) * s.E + e] = s.tr_delay[v.ix(h)];
      }
      if (greedy && !test_mode && c.sx_cum && c.stats_cap > 0) {
        const size_t row = (size_t)(s.ep_t[e] - c.stats_base) % cap;
        c.sx_cum[row * s.E + e] = cum;
        c.sx_arrived[row * s.E + e] = arrived;
      }
      if (greedy) {
        if (test_mode) s.n_test[e] += 1;
        else v.flags |= F_EXPLOIT_DONE;
      } else {
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
  P.dec_done[e] = dec;
  P.upd_n[e] = n_upd;
  if (c.launch_dec) c.launch_dec[e] = ndec;
  if (c.launch_ticks) c.launch_ticks[e] = ticks;
  if (c.launch_bytes) c.launch_bytes[e] = abytes;
}

}  // namespace sfl
