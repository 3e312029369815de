/*
 * pongmi.h — C-ABI of libpongmi.so, the MI355X (gfx950) hot path of pingpong-selfplay-ai:
 * batched PongEnv2P rollout (SoA fp64 arenas), fused two-player QNet acting, device replay +
 * prioritized sampling, and the double-DQN head update.
 *
 * The reference (MaxChen228/pingpong-selfplay-ai) is pure Python and has no FFI; every entry point
 * below replaces a Python function on its hot path, cited as reference file:line. The Python
 * mirror of the reference API (pingpong-selfplay-ai_amd/{envs,models,scripts}) binds these with
 * ctypes.
 *
 * Conventions
 *  - Every pointer argument is a DEVICE pointer owned by the caller (e.g. a torch tensor's
 *    data_ptr()); the library never allocates or frees caller memory. Parameter structs
 *    (pm_env_params, pm_env_state, pm_selfplay) are HOST structs passed by pointer and copied
 *    into the launch; the pointers inside them are device pointers.
 *  - Every call is asynchronous on `stream` (a hipStream_t; NULL = the null stream) and never
 *    synchronizes the host, so a caller may capture calls into a hipGraph.
 *  - Return 0 on success, a negative PM_E* code on an argument error, or a positive hipError_t
 *    if a launch failed. pm_last_error() returns a thread-local message for the last failure.
 *  - Randomness is Philox4x32-10, keyed by a 64-bit seed, countered by (index, purpose, step):
 *    results depend only on (seed, counters), never on launch geometry.
 */
#ifndef PONGMI_H
#define PONGMI_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PM_ABI_VERSION 23

#define PM_OK 0
#define PM_E_ARG (-1)     /* null / inconsistent argument */
#define PM_E_SIZE (-2)    /* size outside the supported range */
#define PM_E_LAUNCH (-3)  /* launch failed (see pm_last_error) */
#define PM_E_COMM (-4)    /* RCCL binding / communicator failure (see pm_last_error) */

/* ---------------------------------------------------------------- environment (K1) */

/* PongEnv2P constructor parameters (envs/my_pong_env_2p.py:19-81). The last six doubles are
 * derived constants the HOST computes with the reference's own Python expressions so the device
 * reproduces them bit for bit:
 *   half_width   = paddle_width/2                     (:152,190)
 *   speed_scale  = 1.0 + speed_increment              (:230)
 *   inertia      = (2/5) * ball_mass * radius**2      (envs/physics.py:9)
 *   jt_coef      = 2*ball_mass/7.0                    (envs/physics.py:10)
 *   inv_mass     = 1.0/ball_mass, inv_inertia = 1.0/inertia (correctly rounded reciprocals: the
 *                  device divides by ball_mass and inertia as q = a*inv; q + fma(-q, b, a)*inv,
 *                  which is the correctly rounded a/b, the quotient physics.py:20-21 computes)  */
typedef struct pm_env_params {
    double paddle_width, paddle_speed, magnus_factor, restitution, friction, ball_mass, radius;
    double speed_lo, speed_hi, spin_lo, spin_hi;
    double ang0_lo, ang0_hi, ang1_lo, ang1_hi;
    double half_width, speed_scale, inertia, jt_coef, inv_mass, inv_inertia;
    int32_t max_score, speed_scale_every, enable_spin, _pad;
} pm_env_params;

/* Struct-of-arrays arena state, [n] each (PongEnv2P attributes ball_x, ball_y, ball_vx, ball_vy,
 * spin, top_paddle_x, bottom_paddle_x, scoreA, scoreB, bounce_count). `serves` counts the resets
 * an arena has consumed: it indexes the injected serve table / the Philox serve stream. */
typedef struct pm_env_state {
    double *x, *y, *vx, *vy, *spin, *top, *bot;
    int32_t *scoreA, *scoreB, *bounces, *serves;
} pm_env_state;

/* PongEnv2P.reset (envs/my_pong_env_2p.py:83-114) for every arena with mask[i] != 0 (mask NULL =
 * all). Serve (vx, vy, spin) comes from `inject` when non-NULL — layout [n][inject_cap][3],
 * entry serves[i] mod inject_cap (parity mode: the host draws it with CPython's `random` exactly
 * as the reference does) — else from Philox(seed) with counter (i, serves[i]) (production mode:
 * speed~U(speed_lo,speed_hi), angle~U(ang0) or U(ang1) by a fair coin, spin~U(spin_lo,spin_hi)).
 * serves[i] is incremented. Writes obsA/obsB [n][7] (may be NULL). `status` (nullable, device
 * int32) is reserved for error bits. */
int pm_env_reset(const pm_env_params* p, const pm_env_state* s, const uint8_t* mask, const double* inject,
                 int32_t inject_cap, uint64_t seed, float* obsA, float* obsB, int32_t* status, int32_t n,
                 void* stream);

/* PongEnv2P.step (envs/my_pong_env_2p.py:116-225, physics.py:3-23, _maybe_scale_speed :227-232,
 * _get_obs :235-263) for n arenas: aA/aB [n] in {0,1,2}; writes obsA/obsB [n][7], rA/rB [n]
 * (values -1/0/+1), done [n]. With autoreset != 0, done arenas are then reset as pm_env_reset
 * (inject / seed as above); obsA/obsB then hold the post-reset observation, and term_obsA /
 * term_obsB (nullable, both or neither) the observation returned by the terminal step (the `nB`
 * the reference stores in replay, scripts/train_iterative.py:242-243):
 *   autoreset 1: every term row is written (the step's pre-reset observation of every arena);
 *   autoreset 2: only the rows of arenas with done[i] != 0 are written, the others keep their
 *                contents (next state for replay = done ? term_obs : obs; SURVEY.md §8d's 203 B
 *                per env-step). With autoreset 0 the term rows, if given, equal obs.
 * Serves of done arenas (ABI 15): with `inject` as pm_env_reset (serves[i] indexes the table and is
 * incremented); in production (inject NULL) from Philox(seed) keyed by (i, counter) — `counter` is
 * the caller's env-step count (PongEnv2PBatch passes its own) — so the draw needs nothing from
 * memory and overlaps the state loads; serves[i] is then neither read nor written. */
int pm_env_step(const pm_env_params* p, const pm_env_state* s, const int8_t* aA, const int8_t* aB, float* obsA,
                float* obsB, float* rA, float* rB, uint8_t* done, float* term_obsA, float* term_obsB,
                int32_t autoreset, const double* inject, int32_t inject_cap, uint64_t seed, uint64_t counter,
                int32_t* status, int32_t n, void* stream);

/* collide_sphere_with_moving_plane (envs/physics.py:3-23) over n rows: in [n][8] =
 * (vn, vt, u, omega, e, mu, m, R) fp64, with I = (2/5)*m*R**2 supplied per row in inertia[n]
 * (CPython's value); out [n][3] = (vn', vt', omega'). A test/diagnostic entry point. */
int pm_collide(const double* in, const double* inertia, double* out, int32_t n, void* stream);

/* The scalar drop-ins' fast path (ABI 23): one launch per call, no copy, no stream synchronisation.
 * `out` is device-visible memory, normally a host-mapped buffer (pm_host_mapped_alloc) the host
 * polls: the kernel writes its results, then `seq` into the 32-bit word after them with a
 * system-scope release.
 *   pm_env_step1  PongEnv2P.step (envs/my_pong_env_2p.py:116-225) of arena 0 of `s` with actions
 *                 (aA, aB), no autoreset: out = obsA[7] obsB[7] rA rB done (f32), seq at word 17.
 *                 Same tick as pm_env_step at n = 1, bit for bit.
 *   pm_env_reset1 PongEnv2P.reset (:83-114) of arena 0 with the host-drawn serve (vx, vy, spin);
 *                 serves[0] incremented: out = obsA[7] obsB[7] 0 0 0, seq at word 17.
 *   pm_collide1   collide_sphere_with_moving_plane (envs/physics.py:3-23) of one row (vn, vt, u,
 *                 omega, e, mu, m, R) with I = inertia: out = (vn', vt', omega') fp64, seq at word 6. */
int pm_env_step1(const pm_env_params* p, const pm_env_state* s, int32_t aA, int32_t aB, float* out, uint32_t seq,
                 void* stream);
int pm_env_reset1(const pm_env_state* s, double vx, double vy, double spin, float* out, uint32_t seq, void* stream);
int pm_collide1(const double* row, double inertia, double* out, uint32_t seq, void* stream);
/* Pinned host memory the device reads and writes directly (hipHostMalloc, mapped + coherent):
 * returns the host pointer (NULL on failure), *dev the device address of the same bytes. */
void* pm_host_mapped_alloc(int64_t bytes, void** dev);
int pm_host_mapped_free(void* host);

/* ---------------------------------------------------------------- QNet (K2) */

/* Packed QNet parameter block (models/qnet.py:52-69), PM_QNET_NP floats, in this order:
 *   features.0.weight [64,7] | features.0.bias [64] | features.2.weight [64,64] | features.2.bias [64]
 *   fc_V.{weight_mu [1,64], bias_mu [1], weight_sigma [1,64], bias_sigma [1]}
 *   fc_A.{weight_mu [3,64], bias_mu [3], weight_sigma [3,64], bias_sigma [3]}      (the 520 "heads",
 *        in the order train_iterative.py:101-104 hands them to Adam)
 *   fc_V.{weight_epsilon [1,64], bias_epsilon [1]} | fc_A.{weight_epsilon [3,64], bias_epsilon [3]}
 * Effective (folded) weights, PM_QNET_NW floats: the plain part W1 [64,7] | b1 [64] | W2 [64,64] |
 *   b2 [64] | Wh [4,64] (row 0 = V, rows 1..3 = A) | bh [4] (4932 floats, padded to 4936), then the
 *   same weights re-ordered into MFMA operand fragments (5008 floats) for the matrix-core forward.
 *   Produce it with pm_qnet_fold; treat the fragment part as opaque. */
#define PM_QNET_NP 5452
#define PM_QNET_NHEAD 520
#define PM_QNET_HEAD_OFF 4672
#define PM_QNET_EPS_OFF 5192
#define PM_QNET_NW 9944
/* The learner's packed exchange buffer sp->grad (float32, PM_GRAD_LEN), the one thing a sharded
 * update all-reduces (SUM): the 520 head gradients of this shard's batch, then the episodes this
 * shard finished in the vector step (update 0 only) and the "an update ran" flag (1 per shard, so
 * the sum counts the ranks that trained). Every rank then applies Adam to grads / world and decays
 * epsilon by the summed episode count. */
#define PM_GRAD_EPISODES 520
#define PM_GRAD_UPDATED 521
#define PM_GRAD_LEN 528

#define PM_FOLD_EVAL 0        /* NoisyLinear eval mode: W = mu                          (qnet.py:47-49) */
#define PM_FOLD_TRAIN 1       /* train mode with the block's epsilon buffers: mu+sigma*eps (qnet.py:44-46) */
#define PM_FOLD_TRAIN_FRESH 2 /* reset_noise() then train mode (qnet.py:33-41): fresh factorised
                                 Gaussian noise from Philox(seed, counter); written back into the
                                 block's epsilon slots when params_out != NULL                   */

/* Fold `count` parameter blocks [count][PM_QNET_NP] into effective weights [count][PM_QNET_NW].
 * counter_dev (nullable, device uint64) is added to `counter` so a captured graph advances it. */
int pm_qnet_fold(const float* params, float* params_out, int32_t mode, uint64_t seed, uint64_t counter,
                 const uint64_t* counter_dev, float* w_eff, int32_t count, void* stream);

/* QNet.forward (models/qnet.py:71-75) on effective weights: x [n][7] -> q [n][3]. */
int pm_qnet_q(const float* w_eff, const float* x, float* q, int32_t n, void* stream);

/* Both players' action selection for n arenas (fused, matrix cores):
 *   A: argmax_a Q_opp(obsA) with opponent weights w_opp[opp_id[i]] (opp_id NULL = net 0)
 *      (scripts/train_iterative.py:240; tests/arena.py:294-320)
 *   B: random.random() < epsilon ? randint(0,2) : argmax_a Q_B(obsB)          (train_iterative.py:124-130)
 * argmax keeps the first maximal index (torch). epsilon is *eps_dev when eps_dev != NULL.
 * qA/qB [n][3] nullable. Philox counter for the epsilon draws: (i, counter + *counter_dev).
 * Rows are grouped by opponent net: net 0 is gathered per chunk0 arenas, nets >= 1 per chunk1
 * arenas (0 = defaults 256 / 4096; at most 4096); choose each so a chunk holds >= ~64 of its rows. */
int pm_qnet_act(const float* w_opp, const int32_t* opp_id, int32_t n_opp, const float* w_B, const float* obsA,
                const float* obsB, float epsilon, const double* eps_dev, uint64_t seed, uint64_t counter,
                const uint64_t* counter_dev, int8_t* aA, int8_t* aB, float* qA, float* qB, int32_t n,
                int32_t chunk0, int32_t chunk1, void* stream);

/* K8 — whole greedy matches in one launch (the match megakernel, csrc/pm_play.hip). Replaces the
 * per-episode loops of scripts/train_iterative.py:171-196 (eval_vs_model / eval_vs_pool),
 * tests/test_round_robin.py:290-330 and tests/arena.py:294-320 for QNet and ball-follower players.
 * Every arena resets with its serve (vx, vy, spin) and plays until a score reaches max_score, both
 * players greedy (argmax, first max) on effective weights w_nets[net] (PM_QNET_NW floats each,
 * 16-B aligned; net -1 = HardcodedBallFollower). Work is given as slots: order[s] = arena of slot
 * s, serves[s] = its serve ([m][3] f64, slot order). Block b plays slots
 * [blk_range[2b], blk_range[2b] + blk_range[2b+1]) (at most 1024 slots) with nets
 * (blk_nets[2b], blk_nets[2b+1]) for (A, B), 128 at a time, a finished slot's column taking the
 * next one. max_steps bounds the ticks of each wave over all its slots. Outputs per arena: final
 * scores, length and last[i] = sign(rB - rA) of the final tick; arenas not finished keep the
 * caller's length (initialise it to -1). *status (device, zeroed by the caller) counts invalid net /
 * arena ids, invalid ranges and episodes cut by max_steps. All pointers except p are device
 * pointers. */
int pm_play(const pm_env_params* p, const float* w_nets, int32_t n_nets, const int32_t* blk_nets,
            const int32_t* blk_range, int32_t n_blocks, const int32_t* order, const double* serves, int32_t n,
            int32_t max_steps, int32_t* scoreA, int32_t* scoreB, int32_t* length, int8_t* last, int32_t* status,
            void* stream);

/* K9 — inference-only self-play rollout, `steps` vector steps in one launch (BASELINE configs[1];
 * csrc/pm_rollout.hip). Replaces the act/step loop of scripts/train_iterative.py:239-242 with the
 * learner switched off: per vector step c = counter0 + s, modelB's heads are refolded with fresh
 * noise (reset_noise, :125; Philox(seed_net, c) as pm_qnet_fold PM_FOLD_TRAIN_FRESH), player A acts
 * greedily on wA, player B epsilon-greedily on wB's features + the fresh heads (Philox(seed_env, c)
 * as pm_qnet_act), and every arena ticks with autoreset (the step-keyed serve of pm_env_step,
 * Philox(seed_env, c)). Bit-identical to that fold -> act -> env_step sequence. wA / wB: effective
 * weights (PM_QNET_NW, 16-B aligned; wB any fold of paramsB: only its feature layers are read);
 * paramsB: modelB's parameter block (PM_QNET_NP; its eps section is not written); heads_ws: device
 * workspace of steps * PM_ROLL_HEADS floats, 16-B aligned. On return the state holds the arenas after
 * the last step and obsA / obsB [n][7] their observations. stats (nullable, device, accumulated):
 * [0] episodes finished, [1] of them won by B, [2] points won by A, [3] points won by B. The serve
 * counters (s->serves) are neither read nor written. */
#define PM_ROLL_HEADS 264
int pm_rollout(const pm_env_params* p, const pm_env_state* s, const float* wA, const float* wB, const float* paramsB,
               float epsilon, uint64_t seed_env, uint64_t seed_net, uint64_t counter0, int32_t steps, float* heads_ws,
               float* obsA, float* obsB, int64_t* stats, int32_t n, void* stream);

/* §8f3 — the collecting rollout (ABI 18): pm_rollout's launch that also pushes every vector step's
 * transitions into a replay ring from registers, as the training loop's memory.push((oB, aB, rB, nB,
 * done)) (scripts/train_iterative.py:242-243, PrioritizedReplay.push :56-63) with the learner switched
 * off (no train_step between pushes, epsilon held for the launch). Step s's arena i lands in slot
 * (pos + s * n + i) mod cap: row (s = obsB before the step, r = rB, s' = the step's terminal obsB,
 * bits(aB | done << 8)), prios[slot] = prio, and, with per_work, the PER leaf powf(prio, alpha) —
 * after the launch the sum tree's nodes are rebuilt over the whole ring (per_work then is the
 * pm_per_work_bytes(cap) tree of pm_per_sample). ep_reward [n] is carried (ep_reward += rB, zeroed
 * on done). steps * n <= cap (no slot is written twice in one launch). stats (nullable, device,
 * accumulated) holds 6 entries: pm_rollout's four, then [4] episodes with ep_reward > 0 (the loop's
 * win, :247-248), [5] the sum of ep_reward over finished episodes. Bit-identical to `steps`
 * repetitions of pm_rollout's stepped composition with pm_env_step's terminal observations pushed
 * in arena order (tests/test_gpu_rollout.py). */
typedef struct pm_roll_replay {
    float *trans;      /* [cap][PM_TRANS_F], 16-byte aligned */
    float *prios;      /* [cap] */
    void *per_work;    /* nullable: PER sum tree (pm_per_work_bytes(cap), 16-byte aligned) */
    float *ep_reward;  /* [n] */
    int64_t pos, cap;  /* 0 <= pos < cap */
    float prio, alpha; /* the pushed priority (max(prios), or 1.0 into an empty buffer) and PER alpha */
} pm_roll_replay;
int pm_rollout_push(const pm_env_params* p, const pm_env_state* s, const float* wA, const float* wB,
                    const float* paramsB, float epsilon, uint64_t seed_env, uint64_t seed_net, uint64_t counter0,
                    int32_t steps, float* heads_ws, float* obsA, float* obsB, const pm_roll_replay* rp, int64_t* stats,
                    int32_t n, void* stream);

/* ---------------------------------------------------------------- QNetRNN (K5) */

/* Packed QNetRNN parameter block (models/qnet_rnn.py:58-101), PM_RNN_NP floats: the state_dict
 * tensors in modelB.parameters() order (features_extractor.{0,2}.{weight,bias}, lstm.{weight_ih_l0,
 * weight_hh_l0, bias_ih_l0, bias_hh_l0}, fc_shared_head.0 / fc_V / fc_A {weight_mu, bias_mu,
 * weight_sigma, bias_sigma}: 174 984 floats), then the NoisyLinear epsilon buffers (shared head,
 * V, A; weight then bias). Effective weights, PM_RNN_NW floats: an opaque MFMA fragment image. */
#define PM_RNN_NP 192012
#define PM_RNN_NPARAM 174984
#define PM_RNN_NW 157456

/* Fold `count` QNetRNN blocks [count][PM_RNN_NP] into effective weights [count][PM_RNN_NW]; modes
 * as pm_qnet_fold (NoisyLinear eval: mu; train: mu + sigma*eps; train_fresh: reset_noise() first,
 * Philox(seed, counter + *counter_dev) per net, written back into params_out when non-NULL). */
int pm_rnn_fold(const float* params, float* params_out, int32_t mode, uint64_t seed, uint64_t counter,
                const uint64_t* counter_dev, float* w_eff, int32_t count, void* stream);

/* One QNetRNN.forward step (models/qnet_rnn.py:107-144, T = 1) for n rows: x [n][7], (h, c)
 * [n][128] each read and overwritten with (h_n, c_n); reset[i] != 0 (nullable) starts row i from
 * init_hidden (zeros, :146-152); q [n][3]. */
int pm_rnn_q(const float* w_eff, const float* x, float* h, float* c, const uint8_t* reset, float* q, int32_t n,
             void* stream);

/* Both players' QNetRNN action selection (train_rnn_iterative.py:371-389, :571-581) for n arenas,
 * fused on the matrix cores: A greedy with w_opp[opp_id[i]] (opp_id NULL = net 0) on obsA and
 * (hA, cA); B on obsB and (hB, cB): random.random() < epsilon ? randint(0,2) : argmax, the forward
 * advancing (hB, cB) either way. reset (nullable) zeroes both players' state first (episode
 * start). Side A is grouped per net: with opp_list / opp_cnt (nullable; per-256-arena-block lists
 * as pm_selfplay's, consistent with opp_id) every net's arenas are packed into full 128-row groups,
 * otherwise chunks of chunk0 (net 0) / chunk1 (others) arenas are compacted (0 = 256 / 2048). */
int pm_rnn_act(const float* w_opp, const int32_t* opp_id, int32_t n_opp, const float* w_B, const float* obsA,
               const float* obsB, float* hA, float* cA, float* hB, float* cB, const uint8_t* reset, float epsilon,
               const double* eps_dev, uint64_t seed, uint64_t counter, const uint64_t* counter_dev, int8_t* aA,
               int8_t* aB, float* qA, float* qB, int32_t n, int32_t chunk0, int32_t chunk1, const int32_t* opp_list,
               const int32_t* opp_cnt, void* stream);

/* ---------------------------------------------------------------- DRQN update (K6) */

/* train_step_rnn (scripts/train_rnn_iterative.py:400-531) on a sampled batch of `batch` sequences
 * of length T: zero initial state; q = Q_B(obs)[last step][act[:, T-1]]; double-DQN target
 * y = rew[:, T-1] + gamma * Q_T(next)[argmax Q_B(next)] * (1 - done[:, T-1]) with modelB in train
 * mode (NoisyLinear mu + sigma * its epsilon buffers) and targetB in eval mode (mu);
 * loss = smooth_l1(q, y) (mean); gradients of all PM_RNN_NPARAM parameters by BPTT;
 * clip_grad_norm_(max_norm); Adam; targetB <- modelB every target_update_interval steps. */
typedef struct pm_drqn_stats {
    int64_t steps;  /* updates taken (train_steps_count: target sync every target_update_interval) */
    int64_t adam_t; /* the optimizer's step count (bias correction); a new optimizer restarts it at 0 */
    float loss;     /* smooth_l1 loss of the last update */
    float norm;     /* pre-clip total gradient norm of the last update (of the rank mean) */
    float q_mean;   /* mean q of the last batch */
    int32_t status; /* latched error bits: 2 = a hand-off inside pm_drqn_grads timed out on this replica;
                     * 4 = (before round 6) pm_drqn_apply's norm arrival timed out; no longer set;
                     * 8 = an update was voided (a timeout on any rank: no Adam step, no target sync) */
} pm_drqn_stats;

typedef struct pm_drqn {
    float *params;          /* [PM_RNN_NP] modelB, updated in place */
    float *target;          /* [PM_RNN_NP] targetB */
    float *adam_m, *adam_v; /* [PM_RNN_NPARAM] */
    float *grad;            /* [PM_RNN_NPARAM + 4] gradients in packed parameter order, then at
                             * [PM_RNN_NPARAM] the number of ranks that contributed (1 per enabled
                             * replica) and at [PM_RNN_NPARAM + 1] the number of ranks whose update
                             * timed out — all summed by the all-reduce; apply divides by the first
                             * and does nothing when the second is non-zero */
    void *work;             /* pm_drqn_work_bytes(batch, T) bytes, 16-byte aligned, ZERO-FILLED before the
                             * first pm_drqn_* call that uses it (pm_drqn_init does it): the in-launch
                             * hand-offs match granule tags against an epoch kept in the workspace, and
                             * a stale granule whose tag happened to match (hipMalloc / reused memory)
                             * would be read before its producer wrote it */
    pm_drqn_stats *stats;
    const float *obs, *next; /* [batch][T][7] */
    const int32_t *act;      /* [batch][T] */
    const float *rew;        /* [batch][T] */
    const uint8_t *done;     /* [batch][T] */
    const int32_t *enable;   /* nullable device flag: 0 = this replica skips the update (grads -> 0) */
    int32_t batch;           /* multiple of 32, <= 256 */
    int32_t T;               /* 1 .. 64 */
    int64_t target_update_interval;
    double gamma, lr, beta1, beta2, adam_eps, max_norm;
    int32_t poll_limit;     /* polls per in-launch hand-off before it times out: 0 = default (2^20);
                             * < 0 = none (every hand-off times out: a test hook for the void path) */
    int32_t reserved;
} pm_drqn;

int64_t pm_drqn_work_bytes(int32_t batch, int32_t T);
/* Zero-fill d->work (pm_drqn_work_bytes(d->batch, d->T) bytes) on the stream (ABI 20): call once after
 * allocating the workspace, before the first pm_drqn_grads / pm_drqn_update on it. */
int pm_drqn_init(const pm_drqn *d, void *stream);
/* Forward + BPTT: grad <- d loss / d params of this replica's batch, grad[PM_RNN_NPARAM] <- 1
 * (all zero when *enable == 0). The NoisyLinear sigma slots are left for pm_drqn_apply, which
 * forms them as mu gradient x epsilon (linear, identical epsilon on every rank). */
int pm_drqn_grads(const pm_drqn *d, void *stream);
/* grad / grad[PM_RNN_NPARAM] -> clip_grad_norm_ -> Adam step -> target sync; stats updated.
 * Nothing happens when grad[PM_RNN_NPARAM] == 0. */
int pm_drqn_apply(const pm_drqn *d, void *stream);
/* pm_drqn_grads then pm_drqn_apply, the clip norm's shares summed by the weight-gradient tiles as they
 * store. pm_drqn_apply after an all-reduce forms the same shares of the summed gradient in the same
 * order (round 6), so with one rank the two paths give bit-identical parameters, clip active or not. */
int pm_drqn_update(const pm_drqn *d, void *stream);

/* ---------------------------------------------------------------- QNetRNN self-play (K7) */

/* scripts/train_rnn_iterative.py's hot loop (:731-798) for n arenas: both players act with their
 * QNetRNN and (h, c) carried per arena (A greedy: modelA or a pool net, both eval mode; B
 * epsilon-greedy with fresh noise per vector step), env.step, SequenceReplayBuffer.push_step
 * (:107-116: whole episodes of length >= T are kept, the latest seq_cap of them), episode
 * bookkeeping and the next opponent / serve for finished arenas, then 64 sequences sampled
 * (:118-173) into a pm_drqn batch and train_step_rnn once the buffer holds > min_episodes. */
typedef struct pm_rnn_ctrl {
    uint64_t step;       /* vector steps taken */
    int64_t episodes;    /* finished episodes (global_episode_count) */
    int64_t seq_count;   /* episodes ever stored (length >= T) */
    int64_t seq_size;    /* episodes held: the newest min(seq_count, seq_cap), less any evicted by age */
    double epsilon;
    int64_t win_A, ep_A, win_P, ep_P;
    double reward_B;     /* summed rewards of finished episodes */
    int32_t status;      /* bit 0: a sampled step had been overwritten in its arena's ring (never, by
                            construction: kept for the check); bit 1: episodes left the buffer by age
                            before seq_cap newer ones did (their steps would leave the ring: depth is
                            too small for the episode lengths seen); bit 2: a finished trajectory
                            longer than depth / 2 steps was not stored */
    int32_t train;       /* 1 when this step's DRQN update was enabled */
} pm_rnn_ctrl;

typedef struct pm_rnn_selfplay {
    pm_env_params env;
    pm_env_state st;
    int32_t *opp;          /* [n] 0 = modelA, k >= 1 = pool net k */
    float *ep_reward;      /* [n] */
    int32_t *ep_len;       /* [n] steps into the current trajectory (the episode steps push_step
                              collected since the last done; a max_steps cut does not end it) */
    int32_t *ep_steps;     /* [n] steps into the current env episode (the max_steps cut)           */
    uint8_t *reset;        /* [n] 1: zero both players' (h, c) before the next act (episode start) */
    const float *w_opp;    /* [1 + n_pool][PM_RNN_NW] modelA, pool nets (eval-mode folds) */
    float *paramsB;        /* [PM_RNN_NP] modelB (the pm_drqn params); fresh noise written back */
    float *w_B;            /* [PM_RNN_NW] */
    float *hA, *cA, *hB, *cB;  /* [n][128] */
    float *obsA, *obsB;    /* [n][7] */
    int8_t *aA, *aB;       /* [n] */
    float *trans;          /* [depth][n][PM_TRANS_F] per-arena transition rings (s, r, s', a | done << 8) */
    int64_t *seq_eps;      /* [seq_cap][2]: arena | length << 32, first step */
    int64_t *seq_mark;     /* [depth] seq_count after step s's append, at s % depth (age eviction) */
    int64_t *fin;          /* [ceil(n / 256) * 256][2] scratch: stored episodes staged per env block */
    int64_t *partials;     /* [ceil(n / 256)][8] */
    int32_t *opp_list;     /* [n] per-256-arena-block opponent lists (written by the env kernel) */
    int32_t *opp_cnt;      /* [ceil(n / 256)][1 + n_pool] (offset << 16 | count) */
    int32_t *enable;       /* [1] set by the sampler: seq_size > min_episodes */
    pm_rnn_ctrl *ctrl;
    int32_t n, n_pool, depth, T, chunk_A, chunk_P;
    int32_t max_steps;     /* max_episode_steps (:751, config default 1000; 0 = no cut): an episode still
                              running after max_steps steps ends (counters, epsilon decay, new opponent,
                              env.reset, zero (h, c)) but its trajectory does not: push_step's
                              current_episode_trajectory keeps collecting until a done (:107-116) */
    int32_t _pad;
    int64_t seq_cap, min_episodes;
    double min_epsilon, epsilon_decay, pool_ratio;
    uint64_t seed_env, seed_net;
    const float *hA_in, *cA_in; /* nullable [n][128]: where the opponents' act reads (h, c) from (it writes
                                   hA / cA); null = in place. The overlapped step (ABI 10) alternates two
                                   buffers so a speculative act of the next step can be redone */
    float *qA, *qB;        /* nullable [n][3]: the Q values each player's act chose from (ABI 19; parity
                              tests read them beside the actions of the same launch) */
} pm_rnn_selfplay;

/* Ring safety: a stored trajectory is at most depth / 2 steps long (longer ones are dropped, status bit
 * 2), and an episode leaves the buffer once depth / 2 steps have passed since it finished (status bit
 * 1 if that happens before seq_cap newer episodes push it out), so every step a sample can reach is
 * still in its arena's ring. Size depth >= 2 x (the steps seq_cap episodes span + the longest
 * trajectory expected) and neither bit is ever set. */
/* Serve every arena, draw its first opponent, zero (h, c). */
int pm_rnn_selfplay_init(const pm_rnn_selfplay *sp, void *stream);
/* modelB's fold with fresh noise + both players' act (K5). */
int pm_rnn_selfplay_act(const pm_rnn_selfplay *sp, void *stream);
/* env tick + sequence store + counters; then, when d != NULL, sample d's batch and set *enable. */
int pm_rnn_selfplay_env(const pm_rnn_selfplay *sp, const pm_drqn *d, void *stream);
/* pm_rnn_selfplay_act then pm_rnn_selfplay_env. */
int pm_rnn_selfplay_rollout(const pm_rnn_selfplay *sp, const pm_drqn *d, void *stream);
/* rollout then pm_drqn_update(d) (d->enable should be sp->enable). */
int pm_rnn_selfplay_step(const pm_rnn_selfplay *sp, const pm_drqn *d, void *stream);
/* Replay ratio: the reference runs train_step_rnn once per env step (:776-777). Update u >= 1 of a
 * vector step samples its own batch (Philox counter (step, u); u = 0 is the env call's draw):
 * pm_rnn_selfplay_sample then pm_drqn_update. pm_rnn_selfplay_step_multi = rollout + update + (U - 1)
 * x [sample(u) + update]; U = 1 is pm_rnn_selfplay_step. */
int pm_rnn_selfplay_sample(const pm_rnn_selfplay *sp, const pm_drqn *d, int32_t u, void *stream);
int pm_rnn_selfplay_step_multi(const pm_rnn_selfplay *sp, const pm_drqn *d, int32_t updates, void *stream);
/* Overlapped act (ABI 10), as the DQN step's: part PM_ACT_ALL = pm_rnn_selfplay_act, PM_ACT_B = modelB's
 * fold + act only (select_action_for_model for B, :757-762), PM_ACT_A = the opponents' act only
 * (:753-755: modelA / pool nets, eval mode). pm_rnn_selfplay_step_overlap = act_part(B) + env + (fork to
 * side_stream: the NEXT step's act_part(A), on part of the chip) + `updates` DRQN updates + join. The
 * opponents' act depends on nothing the update writes, so the results are bit-identical to
 * pm_rnn_selfplay_step_multi. Contract: sp->aA holds the opponents' actions for the current
 * observations (act_part(A) once, then each overlapped step leaves them for the next). */
int pm_rnn_selfplay_act_part(const pm_rnn_selfplay *sp, int32_t part, void *stream);
int pm_rnn_selfplay_step_overlap(const pm_rnn_selfplay *sp, const pm_drqn *d, int32_t updates, void *side_stream,
                                 void *stream);
/* step_overlap without its act_part(B) (callers that time modelB's act on its own). */
int pm_rnn_selfplay_finish_overlap(const pm_rnn_selfplay *sp, const pm_drqn *d, int32_t updates, void *side_stream,
                                   void *stream);

/* ---------------------------------------------------------------- replay + PER (K4) */

/* Transition record, PM_TRANS_F floats per row (64 B): s [7] | r | s' [7] | bits(a | done << 8).
 * (memory.push((oB, aB, rB, nB, done)), scripts/train_iterative.py:243) */
#define PM_TRANS_F 16

/* PrioritizedReplay.sample (scripts/train_iterative.py:64-73): `bs` indices drawn from
 * prios[0:size]^alpha (proportional, with replacement) using the uniforms u[bs] (NULL -> Philox)
 * exactly as np.random.choice does (cdf, searchsorted right); writes idx [bs] and the IS weight
 * w [bs] = (size*P(i))^-beta / max. Scratch: `work` of pm_per_work_bytes(cap) bytes. */
int64_t pm_per_work_bytes(int64_t cap);
int pm_per_sample(const float* prios, int64_t size, float alpha, float beta, const double* u, uint64_t seed,
                  uint64_t counter, int64_t* idx, float* w, int32_t bs, void* work, void* stream);

/* update_priorities (train_iterative.py:74-76): prios[idx[j]] = |err[j]| + 1e-6, sequential order
 * (the last duplicate index wins). */
int pm_per_update(float* prios, const int64_t* idx, const float* err, int32_t bs, void* stream);
/* Full rebuild of a PER sum tree over prios[0, cap) (leaves prio^alpha, then both node levels) into
 * `work` (pm_per_work_bytes(cap)): the tree pm_rollout_push maintains, after the host changed
 * priorities by other means (ABI 18). */
int pm_per_build(const float* prios, int64_t cap, float alpha, void* work, void* stream);

/* ---------------------------------------------------------------- self-play learner (K1+K2+K3+K4) */

/* Device control block (one per shard): the loop counters of scripts/train_iterative.py:106-118,
 * kept on the device so a vector step never syncs the host. */
typedef struct pm_ctrl {
    uint64_t step;           /* vector steps done                                       */
    int64_t pos, size;       /* replay ring position / fill (memory.pos, len(buffer))     */
    int64_t train_steps;     /* train_step() calls that updated (Adam t, target sync)     */
    int64_t frame_idx;       /* beta annealing counter (:136-137)                        */
    int64_t episodes;        /* global_episode_count (:107,234)                          */
    double epsilon;          /* exploration rate of B (:106,261)                         */
    float max_prio;          /* PER max priority for the next push (:57)                 */
    float last_loss;         /* loss of the last update                                  */
    int64_t ep_step;         /* episodes finished during the current vector step          */
    int64_t win_A, ep_A, win_P, ep_P; /* wins / episodes of B vs modelA and vs pool (:247-248) */
    double reward_B;         /* sum of rB over finished episodes                          */
    int32_t status;          /* bit 0: the push-row hand-off inside k_learn timed out; the learner
                                computes those rows itself from then on (results unchanged);
                                bit 1: an update scattered a NaN priority (a diverged loss: its PER
                                leaf is 0, never sampled; the reference's np.random.choice raises);
                                bit 2: k_learn's tree-refresh block never received the learner's
                                priorities (bounded poll): the sum tree was left stale, until
                                pm_selfplay_repair_tree rebuilds it (bit 2 -> bit 3);
                                bit 3: a stale tree was repaired (informational: state consistent) */
    int32_t max_bits;        /* pm_selfplay_commit scratch: float bits of max(prios); 0 between steps */
} pm_ctrl;

/* One shard of the batched self-play learner: every buffer is a device pointer, [n] = per arena. */
typedef struct pm_selfplay {
    pm_env_params env;
    pm_env_state st;
    int32_t *opp;            /* [n] opponent of the running episode: 0 = modelA, 1..n_pool = pool  */
    float *ep_reward;        /* [n] ep_reward of B (:238,245)                                     */
    float *w_opp;            /* [1+n_pool][PM_QNET_NW] opponent effective weights                */
    float *paramsB;          /* [PM_QNET_NP] modelB parameter block (trained heads)              */
    float *paramsT;          /* [PM_QNET_NP] targetB parameter block (eval mode: mu only)         */
    float *w_B;              /* [PM_QNET_NW] modelB acting weights for the current step           */
    float *adam_m, *adam_v;  /* [PM_QNET_NHEAD] Adam state                                        */
    float *trans;            /* [cap][PM_TRANS_F] replay ring                                     */
    float *prios;            /* [cap] priorities                                                  */
    void *per_work;          /* pm_per_work_bytes(cap): PER sum tree (16-byte aligned, as prios)  */
    int64_t *idx;            /* [batch] sampled indices                                           */
    float *isw;              /* [batch] IS weights                                                */
    float *grad;             /* [PM_QNET_NHEAD + 8] grads + packed counters (all-reduced when sharded) */
    int64_t *partials;       /* [ceil(n/256)][8] per-block episode counters of the rollout          */
    float *obsA, *obsB;      /* [n][7] observations of the current step (written by the env kernel) */
    int8_t *aA, *aB;         /* [n] actions of the current step (written by the act kernel)        */
    float *hfeat;            /* [4 * batch + 8][80], zero-filled before the first step: batch forward
                                scratch: rows [0, batch) features of s, Q values at 64.. (stable rows);
                                rows [batch, 2 batch) the push rows k_learn's block 1 hands to the
                                learner; row 2 batch word 0 its flag, word 1 the tree-refresh epoch;
                                rows 2 batch + 1 .. the learner -> tree-refresh granules (ABI 21);
                                rows [2 batch + 8, 4 batch + 8) the push rows as tagged 8-byte
                                granules, [batch][76] (ABI 22) */
    float *learn_heads;      /* [3][264] next update's modelB heads (fresh noise) and targetB heads in
                                MFMA fragment order, and that noise (epsilon-buffer layout)        */
    pm_ctrl *ctrl;
    int32_t *opp_list;       /* [n] per 256-arena block: its arenas grouped by opponent net (ascending)  */
    int32_t *opp_cnt;        /* [ceil(n/256)][n_pool+1] (offset << 16 | count) of each net in the block;
                                written by the env kernel (and init) for the next act, n_pool < 64   */
    int32_t n, n_pool, batch, world;
    int32_t chunk_A, chunk_P;  /* act grouping: arenas per chunk for modelA / pool nets (multiples of
                                  256 use opp_list; others compact opp in the act kernel)        */
    int32_t fuse_apply;        /* world == 1: learn also applies (pm_selfplay_apply is then a no-op) */
    int32_t _pad0;
    int64_t cap;
    double gamma, alpha, lr, beta1, beta2, adam_eps;  /* train_iterative.py:33-37, torch.optim.Adam defaults */
    double min_epsilon, epsilon_decay, pool_ratio, beta_start;
    int64_t beta_frames, target_update_interval;
    uint64_t seed_env;       /* rank-specific: serves, opponents, epsilon draws */
    uint64_t seed_net;       /* rank-independent: NoisyNet noise, so replicas stay identical */
    float *featB;            /* nullable [ceil(n/32)][8][64][4]: modelB's hidden features of the current
                                observations (ABI 11), computed ahead by the side-A act work (the learner
                                launch's extra blocks, pm_selfplay_act_part A / ALL); pm_selfplay_actenv
                                then evaluates only the heads. NULL: actenv computes the features */
    float *frow;             /* nullable [cap][64] (ABI 16): ReLU(modelB's hidden features) of every replay
                                row's s, written at push time by pm_selfplay_actenv from featB (the features
                                are frozen: train_iterative.py:97). Needs featB. */
    int32_t frow_ready;      /* nonzero: every replay row with a nonzero priority was pushed through actenv
                                since modelB's feature layers last changed, so frow is current; then
                                pm_selfplay_step_multi runs updates 1..U-1 as ONE single-workgroup launch
                                (k_learn_multi) instead of 3 launches per update */
    int32_t _pad1;
} pm_selfplay;

/* Limits: 1 <= batch <= PM_MAX_BATCH (one learner workgroup), batch < n <= cap (every vector step
 * pushes n > batch transitions, which keeps the tracked max priority exact), n_pool <= 4096. */
#define PM_MAX_BATCH 256

/* One vector step of scripts/train_iterative.py:239-245 for all n arenas, as device work only:
 *   rollout: act (both players, :240-241; matrix-core kernel, which also draws this step's PER
 *            sample, :64-73, into sp->idx / sp->isw once the replay will hold >= batch) then env
 *            step (:242) + replay push (:243) + episode bookkeeping (:245-249, next opponent
 *            :235-236, env.reset :238);
 *   learn:   once the replay holds >= batch transitions: double-DQN loss/grads + priority update
 *            (train_step, :132-164) on the sampled batch, leaving grads and the finished-episode
 *            count in sp->grad; keeps the PER sum tree in sp->per_work current (incl. the next push);
 *   apply:   grads /= world, Adam on the 520 head parameters (:159-161), target sync every
 *            target_update_interval updates (:166-168), epsilon decay per finished episode
 *            (:261), replay/step counters, next step's acting noise (:125).
 * A sharded learner all-reduces sp->grad [PM_QNET_NHEAD + 8] (sum) between learn and apply.
 * pm_selfplay_step = rollout + learn + apply (unsharded). pm_selfplay_init serves every arena,
 * draws first opponents and folds the acting weights of step ctrl->step. */
int pm_selfplay_init(const pm_selfplay* sp, void* stream);
/* Re-derive everything the device keeps that follows from host-visible state: the weights that
 * follow from paramsB/paramsT (acting weights of step ctrl->step, the next update's noisy / target
 * heads) and a full rebuild of the PER sum tree from prios + ctrl. Call after the host changed
 * parameters, priorities or replay counters (checkpoint load, reset_B, promotion). Called by
 * pm_selfplay_init. */
int pm_selfplay_prepare(const pm_selfplay* sp, void* stream);
/* After ctrl.status bit 2 (a tree-refresh timeout): full rebuild of the PER sum tree from prios + ctrl,
 * then status bit 2 -> bit 3 (ABI 23). Test hook: PONGMI_TR_FORCE_TIMEOUT=1 makes the refresh block's
 * poll time out at once. */
int pm_selfplay_repair_tree(const pm_selfplay* sp, void* stream);
int pm_selfplay_rollout(const pm_selfplay* sp, void* stream); /* = pm_selfplay_act + pm_selfplay_env */
int pm_selfplay_act(const pm_selfplay* sp, void* stream);     /* actions -> sp->aA/aB; PER sample    */
int pm_selfplay_env(const pm_selfplay* sp, void* stream);     /* tick + push + bookkeeping + serves   */
int pm_selfplay_learn(const pm_selfplay* sp, void* stream);
int pm_selfplay_apply(const pm_selfplay* sp, void* stream);
int pm_selfplay_step(const pm_selfplay* sp, void* stream);

/* Overlapped stepping. The opponents' greedy actions (side A: modelA / pool nets, :240) depend only
 * on the observations and opponent ids k_env writes, not on anything the learner updates, and the
 * learner is a single workgroup, so the next vector step's side-A act rides in the learner's launch
 * on otherwise idle CUs.
 *   pm_selfplay_act_part: part PM_ACT_ALL = pm_selfplay_act; PM_ACT_B = PER sample + modelB's
 *     epsilon-greedy act (select_action_B, :124-130) only; PM_ACT_A = side A only.
 *   pm_selfplay_learn_act: pm_selfplay_learn, plus side-A actions for the observations the last
 *     pm_selfplay_env wrote (the next vector step's), into sp->aA.
 *   pm_selfplay_actenv: act_part(B) + env fused into one launch (k_actenv): every 256-arena block
 *     computes modelB's greedy actions for its arenas on the matrix cores and ticks them; the PER
 *     sampler blocks also compute the batch rows k_env's forward blocks would. Bit-identical to
 *     act_part(B) + env.
 *   pm_selfplay_step_overlap = actenv + learn_act + apply (unsharded).
 * Contract: before act_part(B) / actenv / step_overlap, sp->aA must hold side-A actions for the current
 * observations (pm_selfplay_act_part(A), or learn_act after the last env). Results are
 * bit-identical to pm_selfplay_step. */
#define PM_ACT_ALL 0
#define PM_ACT_B 1
#define PM_ACT_A 2
int pm_selfplay_act_part(const pm_selfplay* sp, int32_t part, void* stream);
int pm_selfplay_learn_act(const pm_selfplay* sp, void* stream);
int pm_selfplay_actenv(const pm_selfplay* sp, void* stream);
int pm_selfplay_step_overlap(const pm_selfplay* sp, void* stream);

/* Replay ratio: U >= 1 double-DQN updates per vector step. The reference trains once per env step
 * (train_iterative.py:243-244), i.e. once per pushed transition; U = n keeps that ratio for n arenas.
 *   update 0 (mode PM_UPD_FIRST) trains on the batch k_act_sp drew with this step's push pending, as
 *     the U = 1 step does, and carries the step's episode counters and epsilon decay (:245-261);
 *   updates 1..U-1 draw their batch with pm_selfplay_resample (PER sample + batch forward over the
 *     replay as this step's push left it; frame_idx, hence beta and the Philox draw, advance per
 *     update, :136-137) and run pm_selfplay_learn_ex / _apply_ex in mode 0;
 *   pm_selfplay_commit closes the step: max_prio = max(prios) over the replay (memory.push stores
 *     prios.max(), :57 — U * batch >= n scatters can lower the array maximum below the running
 *     maximum the U = 1 step tracks), the sum tree's nodes over the next push range, pos/size/step.
 * PM_UPD_FIRST | PM_UPD_LAST is the U = 1 update (pm_selfplay_learn / pm_selfplay_apply).
 * pm_selfplay_step_multi = actenv + learn_ex(FIRST, side-A act) + (U - 1) x [resample +
 * learn_ex(0)] + commit, unsharded, under step_overlap's contract (sp->aA holds side-A actions for
 * the current observations); U = 1 is pm_selfplay_step_overlap. Sharded callers run the same sequence
 * with an all-reduce of sp->grad and pm_selfplay_apply_ex after every learn_ex. */
#define PM_UPD_FIRST 1
#define PM_UPD_LAST 2
int pm_selfplay_learn_ex(const pm_selfplay* sp, int32_t mode, int32_t with_act, void* stream);
int pm_selfplay_apply_ex(const pm_selfplay* sp, int32_t mode, void* stream);
int pm_selfplay_resample(const pm_selfplay* sp, void* stream);
int pm_selfplay_commit(const pm_selfplay* sp, void* stream);
int pm_selfplay_step_multi(const pm_selfplay* sp, int32_t updates, void* stream);

/* ---------------------------------------------------------------- sharded steps (configs[3]) */

/* The learner's exchange step as a library-owned RCCL communicator. The reference is
 * single-process (scripts/train_iterative.py:80); the build shards arenas over one process per GPU
 * and sums the learner's gradient buffer once per update. Through torch.distributed that all-reduce
 * runs on the process group's own stream (an event hand-off each way) behind a Python call; the
 * *_step_sharded calls below issue a whole sharded vector step from C, with ncclAllReduce enqueued on
 * the caller's stream between the kernels (results identical to the Python sequence).
 *   rccl_path: the RCCL shared library to bind (dlopen at run time; pass the one the process already
 *     loaded, e.g. torch's bundled librccl.so, so a single RCCL instance serves both).
 *   pm_comm_unique_id: rank 0 creates the 128-byte id; the caller broadcasts it to every rank.
 *   pm_comm_init: collective over nranks processes (ncclCommInitRank on the current device).
 *   pm_comm_allreduce_f32: in-place SUM all-reduce of n floats on `stream`.
 *   pm_comm_info: the communicator's own view of the group, from RCCL itself (ncclCommCount,
 *     ncclCommUserRank, ncclCommCuDevice): a caller proves a sharded run really spans N ranks. */
#define PM_COMM_ID_BYTES 128
typedef struct pm_comm pm_comm;
int pm_comm_unique_id(const char* rccl_path, uint8_t* id);
int pm_comm_init(const char* rccl_path, const uint8_t* id, int32_t nranks, int32_t rank, pm_comm** out);
int pm_comm_allreduce_f32(pm_comm* comm, float* buf, int64_t n, void* stream);
int pm_comm_destroy(pm_comm* comm);
int pm_comm_info(const pm_comm* comm, int32_t* nranks, int32_t* rank, int32_t* device);
/* One sharded DQN vector step with `updates` updates (sp->world == comm ranks, fuse_apply 0):
 * actenv; per update u: [resample (u > 0)] + learn_ex (u = 0 with the next step's side-A act) +
 * all-reduce of sp->grad + apply_ex; commit when updates > 1. Same contract as step_overlap
 * (sp->aA holds the side-A actions for the current observations). */
int pm_selfplay_step_sharded(const pm_selfplay* sp, pm_comm* comm, int32_t updates, void* stream);
/* One sharded QNetRNN vector step: rollout; per update u: [sample(u) (u > 0)] + pm_drqn_grads +
 * all-reduce of d->grad (gradients + contributing-rank count) + pm_drqn_apply. */
int pm_rnn_selfplay_step_sharded(const pm_rnn_selfplay* sp, const pm_drqn* d, pm_comm* comm, int32_t updates,
                                 void* stream);
/* pm_rnn_selfplay_step_overlap (ABI 10) with every update's gradient all-reduced in stream order. */
int pm_rnn_selfplay_step_sharded_overlap(const pm_rnn_selfplay* sp, const pm_drqn* d, pm_comm* comm, int32_t updates,
                                         void* side_stream, void* stream);

/* ---------------------------------------------------------------- launch timing (benchmarks, diagnostics)
 * pm_timer_arm(kernel) queues one launch of that kernel, on the calling process's current device,
 * to be timed: the next untimed launch carries begin/end events in its own dispatch
 * (hipExtLaunchKernel), so no marker packet enters the stream and the kernel and its neighbours run
 * exactly as unarmed (a hipEventRecord marker between two launches costs several us of GPU time on
 * ROCm). Up to 64 launches per kernel may be armed or unread at once. pm_timer_read waits for the
 * oldest timed launch and returns its duration in ms (PM_E_ARG if none is left). Never arm while
 * capturing a hipGraph. */
#define PM_TIMER_ACTENV 0   /* k_actenv: modelB's act (heads) + env tick + replay push + PER sample */
#define PM_TIMER_LEARN 1    /* k_learn: the double-DQN update + side-A act + modelB's feature layers */
#define PM_TIMER_RNN_ACT 2  /* k_rnn_act */
#define PM_TIMER_ENV_STEP 3 /* k_env_step (K1, pm_env_step) */
#define PM_TIMER_ROLLOUT 4  /* k_rollout (K9, pm_rollout) */
#define PM_TIMER_DRQN 5     /* k_dq_recur (K6: the DRQN update's persistent recurrence, pm_drqn_grads) */
#define PM_TIMER_LEARN_MULTI 6 /* k_learn_multi: updates 1..U-1 of a vector step (pm_selfplay_step_multi, ABI 23) */
#define PM_TIMER_N 7
int pm_timer_arm(int32_t kernel);
int pm_timer_read(int32_t kernel, float* ms);

/* ---------------------------------------------------------------- misc */
const char* pm_last_error(void);
int pm_abi_version(void);
int32_t pm_sizeof(int32_t which); /* 0: pm_env_params 1: pm_env_state 2: pm_ctrl 3: pm_selfplay 4: pm_drqn
                                     5: pm_drqn_stats 6: pm_rnn_ctrl 7: pm_rnn_selfplay
                                     8: pm_roll_replay */

#ifdef __cplusplus
}
#endif
#endif /* PONGMI_H */
