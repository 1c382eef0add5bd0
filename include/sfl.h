/*
 * sfl.h — C-ABI of the MI355X SwitchFL / network-distributed Q-learning hot path.
 *
 * One handle = one batch of E lock-step SwitchFL environments (all on the same
 * compiled map, each with its own seed, its own tabular Q-table and its own RNG
 * stream) resident in the HBM of one GPU.  Plain pointers and sizes only; no
 * torch types.  Every function returns 0 on success and -1 on failure, with the
 * message in sfl_last_error() (thread-local).  Calls are synchronous: they
 * return after the device work they launched has completed.  One handle is used
 * from one host thread.  Multi-GPU = one process and one handle per device.
 *
 * The interfaces these entry points replace in the reference
 * (AI4REALNET/network-distributed-q-learning):
 *
 *   sfl_create        ASyncSwitchEnv(rail_env, max_steps=...)        switchfl/switch_env.py:605-614
 *                     + DistrQLearning(env, gamma, epsilon, ...)     switchfl/distr_q.py:32-45
 *                     (RailNetwork(rail_env) graph compile is done on the host:
 *                      network-distributed-q-learning_amd/compiler.py)
 *   sfl_learn_begin   rng = np.random.default_rng(self.seed),
 *                     agent_num_interactions = {...: 0}               switchfl/distr_q.py:263, 269
 *   sfl_apply_qinit   DistrQLearning.__init_q_table                  switchfl/distr_q.py:81-181, 299-300
 *   sfl_learn         the episode loop of DistrQLearning.learn        switchfl/distr_q.py:275-366
 *   sfl_test          DistrQLearning.test (greedy episode)           switchfl/distr_q.py:184-241
 *   sfl_step          `decisions` iterations of the agent_iter loop  switchfl/distr_q.py:302-362
 *                     (learning mode, episodes restart as they end; the benchmark step)
 *   sfl_get_q / sfl_set_q   DistrQLearning.q_table / save / load     switchfl/distr_q.py:492-527
 *   sfl_get_counters  timing/progress accumulators                   switchfl/switch_env.py:67-73
 *   sfl_env_begin / sfl_env_step   the AEC protocol with an external learner:
 *                     env.reset / agent_iter / last / step(action) / observe
 *                                                                    switchfl/switch_env.py:93, 616-675
 *                     (driven by any learner, e.g. distr_q.py:302-320)
 *   sfl_get_phase_cycles   the per-phase time accumulators            switchfl/switch_env.py:67-73
 *                     (flatland_step_time, last_time, action_selection_time, update_time, reset_time ...)
 */
#ifndef SFL_H
#define SFL_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SFL_ABI_VERSION 8

typedef struct sfl_handle sfl_handle;

/* Compiled map (all arrays are host pointers; the library copies them).
 * Layouts are produced by compiler.py; see DESIGN.md "HBM layout". */
typedef struct {
  int32_t H, W;               /* grid size (square) */
  int32_t S, T, K;            /* switches, trains, distinct target stations */
  int32_t max_episode_steps;  /* Flatland timetable horizon */
  double mf_rate;             /* malfunction rate per train per tick */
  int32_t mf_min, mf_max;     /* malfunction duration bounds */
  uint64_t q_per_env;         /* doubles of compact Q-table per env */
  uint32_t rows_per_env;      /* Q rows per env (key-set bitmap) */
  const uint16_t* grid;       /* [H*W] 16-bit Flatland transitions */
  const int16_t* cell_sw;     /* [H*W] switch index or -1 */
  const uint8_t* sw_np;       /* [S] ports */
  const uint8_t* sw_na;       /* [S] actions incl. STOP */
  const uint8_t* act_src;     /* [S*8] route action -> source port slot */
  const uint8_t* act_dst;     /* [S*8] route action -> destination port slot */
  const uint8_t* act_turn;    /* [S*8] second rail action (1 left, 2 forward, 3 right) */
  const uint8_t* act_j;       /* [S*8] index of the action inside its source slot's compact row */
  const uint8_t* first_other; /* [4S] first action not leaving from this slot */
  const uint8_t* port_side;   /* [4S] map_direction(port) */
  const uint8_t* slot_nroutes;/* [4S] routes leaving from this slot */
  const uint8_t* slot_route_act; /* [4S*4] their action indices */
  const uint8_t* q_w;         /* [4S] compact row width = routes + 1 (STOP) */
  const int16_t* port_nb;     /* [4S] rail neighbour port (global id 4*switch+slot) */
  const int16_t* port_len;    /* [4S] plain cells between the two ports */
  const int16_t* port_unique; /* [4S] unique onward port of a target port, or -1 */
  const uint64_t* q_off;      /* [4S] offset (doubles) of the (switch, in-slot) block */
  const uint32_t* row_base;   /* [4S] first row id of the block */
  const int32_t* dist;        /* [K*H*W*4] distance to station, 0x3FFFFFFF = inf */
  const int32_t* tr_ed;       /* [T] earliest departure */
  const int32_t* tr_la;       /* [T] latest arrival */
  const int32_t* tr_k;        /* [T] target station */
  const int32_t* tr_target;   /* [T] target cell */
  const int32_t* tr_init_cell;/* [T] start cell */
  const int32_t* tr_init_dist;/* [T] cells to the first switch port */
  const int32_t* tr_init_delay; /* [T] delay at reset */
  const uint8_t* tr_init_dir; /* [T] start heading */
  const int16_t* tr_init_port;/* [T] first switch port */
  int32_t delay_threshold;    /* StandardObserver(delay_threshold=...) (observer.py:221, default 20): a train's
                                 delay discretises to 1 while delay <= (latest_arrival - earliest_departure)
                                 * delay_threshold (observer.py:228-244), else 2; |value| <= 65536 */
} sfl_map_desc;

typedef struct {
  double gamma, epsilon, epsilon_decay_rate, lr, lr_decay_rate, default_q;
  int64_t max_steps;          /* ASyncSwitchEnv max_steps (truncation) */
  int32_t ntab;               /* length of the two tables below */
  const double* eps_tab;      /* epsilon * decay**n, Python float arithmetic */
  const double* lr_tab;       /* lr * lr_decay**n */
} sfl_hparams;

typedef struct {
  int32_t n_episodes;         /* episodes to run in this call (learn: learning episodes) */
  int32_t exploit_freq;       /* learn: greedy round before episode t when (t+1) % f == 0 (0 = off) */
  int32_t stats_cap;          /* rows of the output buffers below (>= n_episodes to keep all) */
  int32_t pad_;
  /* optional host outputs, row = episode index % stats_cap, [row][env] ([row][train][env] for delays) */
  double* cum_reward;
  int32_t* arrived;
  int32_t* malfunctions;
  int32_t* decisions;
  int32_t* ticks;
  int32_t* delays;
  double* exploit_cum;
  int32_t* exploit_arrived;
  /* optional per-decision trace of one env (debug / parity tests): [trace_cap][4] uint64 */
  uint64_t* trace;
  uint64_t* trace_n;
  int32_t trace_env;
  int32_t trace_cap;
} sfl_run_args;

typedef struct {
  uint64_t decisions;         /* agent-env-steps over all envs since create */
  uint64_t last_launch_decisions;
  uint64_t last_launch_ticks;
  uint64_t last_launch_alg_bytes; /* sum of 220+48P+8A per decision + 36*T_live per env-tick */
  double last_kernel_ms;      /* device time of the last run/step launch (HIP events) */
  int32_t kernel_variant;     /* 0: one env per lane (k_run); v > 0: one env per lane group (k_wave shape v) */
  int32_t group_lanes;        /* lanes per env */
} sfl_counters;

int sfl_abi_version(void);
/* SHA-1 of the sources the library was built from (build.py kernel_source_sha1); the Python
 * loader refuses a library whose id differs from the sources in its tree (a stale build) */
const char* sfl_build_id(void);
const char* sfl_last_error(void);
int sfl_device_count(int* n);

int sfl_create(const sfl_map_desc* map, const sfl_hparams* hp, uint32_t n_envs, const uint64_t* env_seeds,
               int device, sfl_handle** out);
int sfl_destroy(sfl_handle* h);

int sfl_learn_begin(sfl_handle* h, const uint64_t* rng_states /* [n_envs][5] */);
int sfl_apply_qinit(sfl_handle* h, uint32_t n_rows, const uint32_t* row_port, const uint32_t* row_state,
                    const double* values /* [n_rows][4], NaN = default_q */);
int sfl_mark_exploit_done(sfl_handle* h);
int sfl_learn(sfl_handle* h, sfl_run_args* args);
int sfl_test(sfl_handle* h, sfl_run_args* args);
int sfl_step(sfl_handle* h, int64_t decisions_per_env, uint64_t* decisions_done, double* kernel_ms);

int sfl_get_q(sfl_handle* h, uint32_t env, double* q /* [q_per_env] */, uint32_t* touched /* [(rows+31)/32] */);
int sfl_set_q(sfl_handle* h, uint32_t env, const double* q, const uint32_t* touched);
int sfl_get_counters(sfl_handle* h, sfl_counters* out);
/* why this handle runs the lane-per-env body (kernel_variant 0) instead of the one-env-per-wavefront
 * kernel, e.g. "timetable horizon beyond 8191 ticks"; "" when it runs k_wave or k_run was requested */
int sfl_get_kernel_note(sfl_handle* h, char* buf, int32_t cap);
/* read back one env's state word arrays (debug / parity tests) */
int sfl_get_env_state(sfl_handle* h, uint32_t env, int32_t* elapsed, int32_t* phase, uint64_t* sem /* [4S] */,
                      int32_t* tr_pos /* [T] */, uint32_t* tr_bits /* [T] */);

/* ---- Flatland-compatible malfunction stream ----
 * Replaces the counter-based malfunction draw (the default, oracle/flatland_lite.py mf_draw) with
 * a table of the proposals Flatland's ParamMalfunctionGen draws from the env's np_random each step
 * (flatland.envs.malfunction_generators, built at test_model.py:14-19 / main.py:28-33 and
 * reseeded by RailEnv.reset(random_seed=seed) at switch_env.py:99): table[n_envs][steps][T] =
 * num_broken_steps proposed to train h at step t + 1 of an episode (0 = none); a proposal starts
 * a malfunction only for a train that is not done and not already malfunctioning (the
 * MalfunctionHandler rule).  steps == 0 returns to the counter-based draw. */
int sfl_set_mf_schedule(sfl_handle* h, int32_t steps, const uint8_t* table);
/* Host helper (no device): one env's table from its seeding words (flatland.utils.seeding.np_random:
 * key = the sha512-derived init_by_array words), the timetable's randint(0, window) draws consumed
 * at reset (flatland_patch/timetable_generators.py:115), prob = 1 - exp(-malfunction_rate),
 * durations randint(mf_min, mf_max + 1) + 1.  out[steps][T]. */
int sfl_mf_schedule_flatland(const uint32_t* key, int32_t nkey, const int32_t* windows, int32_t n_windows, int32_t T,
                             double prob, int32_t mf_min, int32_t mf_max, int32_t steps, uint8_t* out);

/* ---- graph-partitioned mode (BASELINE.json configs[4]; SURVEY.md §8(e) "C5") ----
 * The switch agents are partitioned over `world` ranks (owner[S]); rank r stores the Q rows of
 * the switches it owns for all `envs_total` envs of the job, and simulates its own envs
 * [env_base, env_base + n_envs).  A round: sfl_part_local (every local env applies the reply
 * to its last request, runs to its next decision and stages that decision's request, plus the
 * update records of its post step; the staged records are packed into one message segment per
 * destination rank, each env's records for that rank as a contiguous group: its updates in the
 * order it made them, then its request), ONE all-to-all of the message buffer, sfl_part_owner on
 * the received segments (per group: the updates in order, then the answer to the request), and an
 * all-to-all of the replies back.  Buffers are [world][k + 1] records (record 0 of a segment =
 * header holding the count; k = the capacity of sfl_part_set_caps, cap_req + cap_upd until then):
 * messages of sfl_part_record_sizes' `msg` bytes, replies of `rep` bytes, a reply at its request's
 * record index; on the GPU they are device pointers (the caller's RCCL buffers).  An env whose group
 * does not fit this round's segment is deferred whole: it sends nothing (its places below the
 * segment end carry void records), sits out the next sfl_part_local and sends the same records
 * again -- so the exchange has a fixed size and needs no counts, and results do not depend on k.
 * Replaces the reference's in-process successor lookup max_q(next_state, next_agent) and update
 * (switchfl/distr_q.py:419-466) across GPU boundaries. */
int sfl_part_config(sfl_handle* h, int32_t rank, int32_t world, const int32_t* owner /* [S] */, uint32_t env_base,
                    uint32_t envs_total, uint32_t cap_req /* >= n_envs */, uint32_t cap_upd);
int sfl_part_record_sizes(uint32_t* msg, uint32_t* rep);
int sfl_part_begin(sfl_handle* h);  /* start a part step: per-env decision counters to 0 */
/* requests_sent: the envs with a request or deferred this round (null: see sfl_set_stream) */
int sfl_part_local(sfl_handle* h, int64_t decisions_per_env, const void* replies, void* messages,
                   uint64_t* requests_sent /* null: see sfl_set_stream */);
int sfl_part_owner(sfl_handle* h, const void* messages, void* replies);
/* this rank's record counts of the last sfl_part_local: out[0 .. world) message records per
 * destination (staged, sent or deferred); then, when cap allows (2 world + 3 words): out[world .. 2 world)
 * their peaks since the previous call, out[2 world] the envs with a request or deferred, out[2 world + 1]
 * the envs deferred in that round, out[2 world + 2] the deferrals since the previous call.  cap >= world;
 * synchronises if sfl_part_local did not (and reports the envs' errors) */
int sfl_part_counts(sfl_handle* h, uint32_t* out, int32_t cap);
/* the segment capacity of the next rounds (records per destination, 1 <= k <= cap_req + cap_upd):
 * every rank of the job sets the same value, at a point where no round is in flight (the buffers of
 * a round are [world][k + 1] records).  A smaller k moves fewer bytes per round; an env that does not
 * fit waits a round (see above). */
int sfl_part_set_caps(sfl_handle* h, uint32_t k_msg);
/* how often the handle has waited for its device since create (stream / event synchronisations; 0 on
 * the host build) and read the round counts back (sfl_part_counts, sfl_part_local with requests_sent):
 * what a caller checks to see that its rounds queue without the host in the loop */
int sfl_get_sync_count(sfl_handle* h, uint64_t* waits, uint64_t* count_reads);
/* queue the handle's work on the caller's stream (a hipStream_t, e.g. torch's current stream,
 * which its RCCL collectives follow).  Then sfl_part_owner returns without a
 * synchronisation, and so does sfl_part_local when requests_sent is null (its counts are read by
 * sfl_part_counts): the rounds between two sfl_part_counts calls queue without a synchronisation.
 * null: the handle's own stream again */
int sfl_set_stream(sfl_handle* h, void* stream);
/* Which switches' rows the wave kernel decides on and updates in place: local_switches[S] (1 = in
 * place; only switches this rank owns), null = every switch this rank owns (the default after
 * sfl_part_config).  The other rows travel as requests / update records to their owners -- with
 * one rank and the default, no messages at all.  Marking fewer switches local rehearses a bigger
 * job's message traffic on one rank (all zero: every row operation as a message, like the
 * lane-per-env body).  Results are identical either way. */
int sfl_part_set_local_rows(sfl_handle* h, const uint8_t* local_switches);
/* owned Q blocks of one env of the job, written into the full per-env layout of sfl_get_q
 * (other entries untouched); owned key-set bits OR-ed into touched */
int sfl_part_get_q(sfl_handle* h, uint32_t global_env, double* q, uint32_t* touched);

/* ---- external-action mode: the AEC protocol with the policy / learner on the host ----
 * sfl_env_begin turns the handle into n_envs plain environments (no learner: no epsilon draw, no Q-table
 * access), each at a fresh reset.  Each sfl_env_step call then, per env: applies actions[e] to the
 * observation the previous call emitted (ASyncSwitchEnv.step -> _apply_action, and _move_trains_to_switch
 * when no switch is active: switch_env.py:632-666), and runs on to the env's next decision, whose
 * observation it emits (agent_iter pops it, last() / observe() read it: switch_env.py:616-630, 668-675,
 * observer.py:246-308) -- or reports the episode's end (agent = -1; the next call resets:
 * switch_env.py:93-158).  actions == null (or an action < 0) applies nothing and re-emits the pending
 * observation; SFL_ACTION_RESET resets the env where it stands (env.reset() in the middle of an episode:
 * the same reset as at an episode end, switch_env.py:93-158) and emits the new episode's first observation.
 * An action outside the deciding switch's action space is refused (E_BAD_ACTION, switch_env.py:213-215)
 * without touching the env.  Output arrays are host pointers, [n_envs] unless stated; null skips one. */
#define SFL_ACTION_RESET (-2)
typedef struct {
  const int32_t* actions;  /* in: action for each env's pending observation (< 0 or null: none) */
  int32_t* agent;          /* deciding switch index of the emitted observation; -1: the episode ended */
  int32_t* train;          /* active train (info["active_train"]) */
  int32_t* slot;           /* in-port slot of the active train at the switch */
  uint32_t* state;         /* observation index ((free_port_bits * K + station) * 3 + delay level): the
                              observation vector [r, c, sem[P], target[2P], delay[P]] (observer.py:269-308) */
  uint32_t* mask;          /* info["action_mask"] as bits (bit a: action a allowed) */
  int32_t* reward;         /* last() reward of (agent, train) (switch_env.py:289, AECEnv.last) */
  int32_t* now;            /* rail_env._elapsed_steps at the observation */
  int32_t* next_switch;    /* step() "next_switch" of the applied action (-1: none applied) */
  int32_t* step_now;       /* _elapsed_steps when that step() returned (-1: none applied) */
  uint32_t* arrived;       /* [4][n_envs] arrived-train bitmask ("arrived_trains") after this call */
  int32_t* malfunctions;   /* episode end: num_malfunctions */
  int32_t* delays;         /* episode end: [T][n_envs] train_to_last_node delays */
  int32_t* truncated;      /* episode end: 1 truncation (max_steps), 0 termination */
} sfl_env_io;
int sfl_env_begin(sfl_handle* h);
int sfl_env_step(sfl_handle* h, sfl_env_io* io);
/* Device time per phase of the learn loop since create, accumulated from in-kernel cycle counters of a
 * sample of the wavefronts (the kernels with one env per lane group; zero for the lane-per-env body):
 * cycles[0] tick (Flatland RailEnv.step + _move_trains / _check_active_switch), [1] observe (last()),
 * [2] epsilon-greedy action selection, [3] apply (_apply_action), [4] post (Q update, pending map,
 * destination bonus), [5] reset, [6] other (launch state load / store, loop control), [7] the sampled
 * wavefronts' total; their ratios split the launches' kernel time (switch_env.py:67-73 accumulators).
 * n >= 8. */
int sfl_get_phase_cycles(sfl_handle* h, uint64_t* cycles, int32_t n);
#ifdef __cplusplus
}
#endif
#endif /* SFL_H */
