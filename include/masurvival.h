/*
 * masurvival.h -- C-ABI of the MI355X-native batched MaSurvival env step.
 *
 * This is the drop-in boundary for the reference's hot path
 *   MaSurvival.step  (reference: masurvival/envs/masurvival_env.py:76-90)
 *   -> Simulation.step (reference: masurvival/simulation.py:233-242)
 * batched over N independent envs that live in HBM as struct-of-arrays.
 *
 * Plain C types only: every I/O pointer is a DEVICE pointer owned by the
 * caller unless stated otherwise; `stream` is a hipStream_t passed as void*.
 * Calls are stream-ordered and asynchronous (no implicit device sync) and are
 * not re-entrant per handle.  Errors: 0 = ok, negative = error code, with a
 * thread-local message from mas_last_error().  Nothing aborts or throws
 * across this ABI.
 */
#ifndef MASURVIVAL_H
#define MASURVIVAL_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MAS_ABI_VERSION 3  /* 2: mas_gae takes the caller's partial-sum scratch; 3: mas_adv_normalize */

#define MAS_OK 0
#define MAS_ERR_INVALID_ARG (-1)
#define MAS_ERR_UNSUPPORTED (-2)
#define MAS_ERR_HIP (-3)
#define MAS_ERR_OOM (-4)

#define MAS_MAX_ZONE_PHASES 8

/* Resolved env configuration: the POD lowering of onevsone_heals_config
 * (reference masurvival_env.py:140-238) after MaSurvival.__init__'s rewrites
 * (masurvival_env.py:293-389).  The Python front-end (masurvival.config)
 * builds it with the reference's one-level merge semantics. */
typedef struct mas_config {
    int32_t n_agents;          /* agents.n_agents                 (:166-169) */
    int32_t n_heals;           /* heals.reset_spawns.n_items      (:210-214) */
    int32_t n_boxes;           /* boxes.reset_spawns.n_boxes      (:191-195) */
    int32_t teams;             /* teams.twoteams -> TwoTeams       (:340-342) */
    int32_t ownership;         /* boxes.ownership -> OwnedObject*  (:196,345) */
    int32_t melee_cooldown;    /* >0: Melee(cooldown); 0: ContinuousMelee (:309-312) */
    int32_t omniscient;        /* observation.omniscent            (:141-143) */
    int32_t gameover_mode;     /* 0 = 'alldead', 1 = 'lastalive'   (:154-156) */
    float r_alive, r_dead, r_kill, r_death; /* reward_scheme      (:144-153) */
    int32_t grid_size;         /* spawn_grid.grid_size             (:158-161) */
    double floor_size;         /* spawn_grid.floor_size (= room size) */
    double agent_size;         /* agents.agent_size (diameter)     (:168) */
    float impulse[3];          /* motors.impulse                   (:177-180) */
    int32_t agent_health;      /* health.health                    (:181-183) */
    float melee_range;         /* melee.range                      (:184-190) */
    int32_t melee_damage;      /* melee.damage */
    double box_size;           /* boxes.reset_spawns.box_size */
    int32_t box_health;        /* boxes.health                     (:208) */
    int32_t randomized_boxes;  /* 'randomized_shape' in boxes      (:362-366) */
    double avg_w, std_w, avg_h, std_h, min_w, min_h; /* RandomizeBoxShapes (semantics.py:97-120) */
    double box_item_size;      /* boxes.item.item_size             (:204-207) */
    float box_item_offset;     /* boxes.item.offset */
    double heal_size;          /* heals.reset_spawns.item_size */
    int32_t healing;           /* heals.heal.healing               (:215-217) */
    int32_t slots;             /* inventory.slots                  (:219-221) */
    float pickup_radius;       /* auto_pickup.shape = circle(0.5)  (:222-224) */
    float give_radius;         /* give.shape = circle(2)           (:225-227) */
    float deathdrop_radius;    /* death_drop.radius                (:228-230) */
    int32_t zone_phases;       /* safe_zone.phases                 (:231-237) */
    int32_t zone_cooldown;
    int32_t zone_damage;
    int32_t zone_n_radii;      /* len(safe_zone.radiuses) (a 0 radius is appended) */
    double zone_radii[MAS_MAX_ZONE_PHASES];
    int32_t zone_random_centers; /* centers == 'random' */
    float zone_centers[MAS_MAX_ZONE_PHASES][2]; /* used when !zone_random_centers */
    float cam_depth;           /* cameras.depth                    (:173-176) */
    double cam_fov;            /* cameras.fov (radians, double as in Python) */
    double wall_aspect_ratio;  /* ThickRoomWalls default 100 (semantics.py:685) */
    /* Lidars(n_lasers, fov, depth) (simulation.py:357-392) as the last agents
     * module, observed as the 'lidars' key (the reference leaves
     * the module unwired, masurvival_env.py:392,857-858).  0 = off. */
    int32_t lidar_n_lasers;    /* lidars.n_lasers (0, or 2..MAS_MAX_LASERS) */
    float lidar_depth;         /* lidars.depth */
    double lidar_fov;          /* lidars.fov (radians, double as in Python) */
} mas_config;

#define MAS_MAX_LASERS 32

/* Observation layout: one flat float32 row of `obs_dim` per agent; the keys
 * are laid out in observation_space (gym Dict, sorted-key) order, each key's
 * per-agent sub-array flattened C-order (compute_obs_space :391-447). */
#define MAS_MAX_KEYS 16
typedef struct mas_obs_layout {
    int32_t n_agents;
    int32_t obs_dim;
    int32_t n_keys;
    char key_name[MAS_MAX_KEYS][24];
    int32_t key_offset[MAS_MAX_KEYS];   /* float offset inside the row */
    int32_t key_ndim[MAS_MAX_KEYS];     /* ndim of the per-agent sub-array */
    int32_t key_shape[MAS_MAX_KEYS][2]; /* per-agent sub-array shape */
} mas_obs_layout;

typedef struct mas_handle mas_handle;

/* replaces MaSurvival.__init__ (masurvival_env.py:293-389): validates the
 * config, allocates the SoA state of n_envs envs on `device` (HBM-resident,
 * no allocation afterwards). */
int mas_create(const mas_config* cfg, int64_t n_envs, int32_t device, mas_handle** out);
int mas_destroy(mas_handle* h);

/* replaces compute_obs_space (masurvival_env.py:391-447). */
int mas_get_obs_layout(const mas_handle* h, mas_obs_layout* out);
int64_t mas_num_envs(const mas_handle* h);

/* replaces the np_random assignment (masurvival_env.py:50,67,455-465):
 * per-env numpy PCG64 bit-generator state, HOST array [n_envs][6] of
 * {state_hi, state_lo, inc_hi, inc_lo, has_uint32, uinteger}
 * (numpy.random.PCG64().state).  One stream per env, shared by the spawn
 * shuffle, box shapes, zone centres and death drops as in the reference. */
int mas_seed(mas_handle* h, const uint64_t* host_rng_states, void* stream);

/* replaces BaseEnv.reset (masurvival_env.py:59-74) for every env whose
 * env_mask byte is non-zero (env_mask == NULL: all envs).  Writes the reset
 * observation rows of those envs into obs [n_envs][n_agents][obs_dim]. */
int mas_reset(mas_handle* h, const uint8_t* env_mask, float* obs, void* stream);

/* replaces BaseEnv.step (masurvival_env.py:76-90): actions int8
 * [n_envs][n_agents][6] (MultiDiscrete [3,3,3,2,2,2], dead agents ignored),
 * writes obs [n_envs][n_agents][obs_dim], rewards [n_envs][n_agents],
 * done [n_envs].  auto_reset != 0: an env that is done is reset in the same
 * launch and its obs rows hold the first observation of the new episode
 * (rewards/done still describe the finished step). */
int mas_step(mas_handle* h, const int8_t* actions, float* obs, float* rewards,
             uint8_t* done, int32_t auto_reset, void* stream);

/* mas_step with the observation rows written as the PPO consumer's bf16
 * policy input instead of fp32 obs: x_bf16 [n_envs * n_agents][x_stride]
 * (x_stride a multiple of 4 >= obs_dim, 8-B aligned), columns [0, obs_dim)
 * of each row = the fp32 row of mas_step rounded to bf16 (round to nearest
 * even, the conversion mas_policy_act applies to fp32 rows), the other
 * columns untouched (the caller's bias column and padding stay).  Rewards,
 * done and the env state are those of mas_step, bit for bit.  Not for the
 * lidars key or a config whose auto-reset runs in the separate reset launch
 * (MAS_ERR_UNSUPPORTED: use mas_step).  No reference equivalent (the rollout
 * side). */
int mas_step_x(mas_handle* h, const int8_t* actions, void* x_bf16, int64_t x_stride, float* rewards,
               uint8_t* done, int32_t auto_reset, void* stream);
/* 1 when mas_step_x can run this handle with this auto_reset, else 0. */
int mas_step_x_supported(const mas_handle* h, int32_t auto_reset);

/* Per-env episode statistics (flush_stats, masurvival_env.py:471-508):
 * device float [n_envs][MAS_STATS_WIDTH] laid out as
 * [0,8) reward0..reward{R-1}, [8,16) kills0..kills{R-1}, 16 steps,
 * 17 heals_used, 18 boxes_placed, with R = 2 (teams) or n_agents (unused
 * slots 0).  Accumulated since the last flush. */
#define MAS_STATS_WIDTH 19
int mas_flush_stats(mas_handle* h, float* stats, void* stream);

/* Raw SoA state image (checkpoint / parity state injection).  Byte size of
 * the image and copies to/from a caller DEVICE buffer of that size. */
int64_t mas_state_bytes(const mas_handle* h);
int mas_get_state(mas_handle* h, void* dst, void* stream);
int mas_set_state(mas_handle* h, const void* src, void* stream);

/* Rollout side (SURVEY.md 8(a) a24 -- new, the reference has no trainer):
 * GAE(gamma, lambda) over an on-device rollout buffer of T steps and
 * n_columns = n_envs * n_agents agent columns, all DEVICE pointers:
 *   rewards [T][n_columns], values [T+1][n_columns] (row T = bootstrap value
 *   of the observation after the last step), done [T][n_envs] (mas_step's
 *   done; an auto-reset env's next value is masked out),
 *   advantages/returns [T][n_columns] (out), adv_sums double[2] (out:
 *   sum and sum of squares of the advantages, for normalisation).
 *   delta_t = r_t + gamma * V_{t+1} * (1 - d_t) - V_t
 *   A_t     = delta_t + gamma * lambda * (1 - d_t) * A_{t+1}
 * scratch: DEVICE double[mas_gae_scratch_doubles(n_columns)], the call's
 * per-workgroup partial sums (no initialisation needed; the library keeps
 * no state between calls, so calls on different streams -- or handles,
 * trainers, threads -- may run concurrently as long as each has its own
 * scratch and outputs).  adv_sums is summed in a fixed order: the same
 * inputs give the same bits.
 * MAS_GAE_SCAN=1 (environment, read per call) selects the wavefront scan
 * over time instead of the per-column walk; same results within fp32
 * rounding.                                                            */
int64_t mas_gae_scratch_doubles(int64_t n_columns);
int mas_gae(int32_t T, int64_t n_columns, int32_t n_agents, const float* rewards, const float* values,
            const uint8_t* done, float gamma, float lam, float* advantages, float* returns, double* adv_sums,
            double* scratch, void* stream);
/* mas_adv_normalize: the n advantages (DEVICE float, 16-B aligned)
 * normalised in place from stats = DEVICE double[3] (sum, sum of squares,
 * count: mas_gae's adv_sums and the count, summed over ranks):
 *   mean = sum / count, var = max(sum_sq / count - mean^2, 0)   (double)
 *   adv  = (adv - (float)mean) / ((float)sqrt(var) + 1e-8f)     (float)
 * one launch, the roundings of the torch expression it replaces
 * (adv.sub_(mean.float()).div_(var.sqrt().float() + 1e-8)). */
int mas_adv_normalize(int64_t n, float* adv, const double* stats, void* stream);

/* Rollout side: sample the six action heads (MultiDiscrete [3,3,3,2,2,2]) of
 * n_rows agent rows from logits [n_rows][row_stride] (first 15 floats of a
 * row: the heads' logits in order), Gumbel-max with a counter-based RNG keyed
 * by (seed, step, row); writes actions int8 [n_rows][6] and the log-prob of
 * the drawn actions float [n_rows].  Batched form of the reference's policy
 * act() (demo.py:14-22).  DEVICE pointers. */
int mas_sample_actions(int64_t n_rows, const float* logits, int64_t row_stride, uint64_t seed, uint64_t step,
                       int8_t* actions, float* logp, void* stream);

/* Rollout / update side (SURVEY.md 8(a) a24 -- new): the shared-parameter
 * policy MLP obs_dim -> 256 -> 256 (tanh) -> 16 (the six heads' 15 logits,
 * then the value) as fused bf16-MFMA kernels with fp32 accumulation.  The
 * reference has no policy; its demo's act() (demo.py:14-22) is the random
 * policy this replaces.  All pointers are DEVICE pointers.
 *
 * mas_policy_pack fills a packed image of mas_policy_packed_bytes(obs_dim)
 * bytes from the fp32 parameters W1 [256][obs_dim], b1 [256], W2 [256][256],
 * b2 [256], W3 [16][256], b3 [16] (row-major, torch nn.Linear layout).
 *
 * mas_policy_act: forward of n_rows agent rows of obs [n_rows][obs_dim] fp32
 * plus Gumbel-max sampling of the six heads with the RNG of
 * mas_sample_actions; writes actions int8 [n_rows][6], logp and value
 * [n_rows], and, when x_bf16 != NULL, the bf16 copy of the rows
 * [n_rows][x_stride] (x_stride a multiple of 8 >= 16*ceil(obs_dim/16)) that
 * mas_policy_train reads: columns [0, 16*ceil(obs_dim/16)) are written, the
 * row's obs_dim values, then 1.0 in column obs_dim (a bias column for the
 * caller's dW1 GEMM) when it falls in that range, then zeros.
 * mas_policy_act_rows: the same for the rows [first_row, first_row + n_rows)
 * of a larger batch (obs, x_bf16, actions, logp, value point at that slice):
 * the sampling RNG is keyed by the row's index in the whole batch, so shards
 * launched on separate streams draw exactly what one launch over the batch
 * draws (mas_policy_act = first_row 0).
 *
 * mas_policy_train: forward of x_bf16 rows, the per-row gradient of the PPO
 * loss  mean(-min(r A, clip(r, 1-clip, 1+clip) A)) + vf_coef mean((v-ret)^2)
 * - ent_coef mean(entropy)  (r = exp(logp(actions) - old_logp); `scale` =
 * 1/rows of the minibatch), and the backward data path; writes feature-major
 * bf16 h1, h2, dA1, dA2 [256][n_rows] (dA = gradient at the pre-activation)
 * and dz [16][n_rows], from which the caller forms the weight gradients
 * (dW1 = dA1 x, dW2 = dA2 h1^T, dW3 = dz h2^T, db = row sums; a row of ones
 * appended to h1 / h2 and the bias column of x give the db's from the same
 * GEMMs), and
 * partials [mas_policy_blocks(n_rows)][4] = per-block sums of the clipped
 * surrogate loss, (v-ret)^2, entropy and the clipped-row count. */
/* mas_render_view: one env's bodies for rendering (debugging / GIF frames;
 * replaces what rendering.py:118-613 reads from the Box2D world).
 * Synchronous: waits for the device, then copies MAS_RENDER_VIEW_FLOATS
 * floats to host `out`:
 *   [0] n_agents  [1] n_boxes  [2] n_box_items  [3] n_heals
 *   [4..6] safe zone centre x, y, radius   [7..9] agent / box / heal slots
 *   (AM, BM, HM of the capacity class)   [10] floor size
 *   [12 + 5k] wall k = 0..3: centre x, y, angle, half extents x, y
 *   [32 ...] AM agents (x, y, angle, alive, health), BM boxes (x, y, hx, hy,
 *   health), BM box items (x, y, hx, hy), HM heals (x, y); entries past the
 *   counts are unused. */
#define MAS_RENDER_VIEW_FLOATS 320
int mas_render_view(mas_handle* h, int64_t env, float* out);

int64_t mas_policy_packed_bytes(int32_t obs_dim);
int64_t mas_policy_blocks(int64_t n_rows);
int mas_policy_pack(int32_t obs_dim, const float* w1, const float* b1, const float* w2, const float* b2,
                    const float* w3, const float* b3, void* packed, void* stream);
int mas_policy_act(const void* packed, int32_t obs_dim, int64_t n_rows, const float* obs, void* x_bf16,
                   int64_t x_stride, uint64_t seed, uint64_t step, int8_t* actions, float* logp, float* value,
                   void* stream);
int mas_policy_act_rows(const void* packed, int32_t obs_dim, int64_t n_rows, int64_t first_row, const float* obs,
                        void* x_bf16, int64_t x_stride, uint64_t seed, uint64_t step, int8_t* actions, float* logp,
                        float* value, void* stream);
/* mas_policy_act_x: mas_policy_act_rows over bf16 input rows x_bf16
 * [n_rows][x_stride] (mas_step_x's rows: columns past obs_dim are ignored --
 * W1 is zero there), which are not written; the same actions, log-probs and
 * values as mas_policy_act_rows on the fp32 rows they were rounded from. */
int mas_policy_act_x(const void* packed, int32_t obs_dim, int64_t n_rows, int64_t first_row, const void* x_bf16,
                     int64_t x_stride, uint64_t seed, uint64_t step, int8_t* actions, float* logp, float* value,
                     void* stream);
int mas_policy_train(const void* packed, int32_t obs_dim, int64_t n_rows, const void* x_bf16, int64_t x_stride,
                     const int8_t* actions, const float* old_logp, const float* adv, const float* ret, float clip,
                     float vf_coef, float ent_coef, float scale, void* h1, void* h2, void* da1, void* da2, void* dz,
                     float* partials, void* stream);
/* mas_policy_train_ld: mas_policy_train with the row stride `ld` >= n_rows
 * of h1, h2, dA1, dA2, dz ([256 | 16][ld]; mas_policy_train: ld = n_rows).
 * A power-of-two stride (the trainer's 4.2M-row minibatch) puts every
 * feature row on the same HBM channels; a padded one reads and writes them
 * about 30 % faster. */
int mas_policy_train_ld(const void* packed, int32_t obs_dim, int64_t n_rows, const void* x_bf16, int64_t x_stride,
                        const int8_t* actions, const float* old_logp, const float* adv, const float* ret, float clip,
                        float vf_coef, float ent_coef, float scale, void* h1, void* h2, void* da1, void* da2, void* dz,
                        int64_t ld, float* partials, void* stream);
/* mas_policy_train_rm: the same kernel writing the activations ROW-major,
 * each lane storing its own row as 16-B chunks (no lane exchange):
 * h1, h2 [n_rows][ld_h] (ld_h >= 257, a multiple of 8; the caller keeps
 * column 256 = 1, the bias column, the kernel writes columns 0..255),
 * dA1, dA2 [n_rows][256], dz [n_rows][16] (outputs in natural order).
 * Within every 32-column tile the 256 hidden columns are stored permuted:
 * column c holds hidden feature mas_policy_rm_feature(c).  The weight
 * gradients are then the row-sum GEMMs dW2 = dA2^T h1, dW3 = dz^T h2,
 * dW1 = dA1^T x with rows / columns mapped back through that permutation. */
int mas_policy_train_rm(const void* packed, int32_t obs_dim, int64_t n_rows, const void* x_bf16, int64_t x_stride,
                        const int8_t* actions, const float* old_logp, const float* adv, const float* ret, float clip,
                        float vf_coef, float ent_coef, float scale, void* h1, void* h2, int64_t ld_h, void* da1,
                        void* da2, void* dz, float* partials, void* stream);
int32_t mas_policy_rm_feature(int32_t col);

/* mas_policy_adam: one PPO optimizer step over flat fp32 buffers of n
 * parameters, replacing torch.nn.utils.clip_grad_norm_(params, max_norm)
 * followed by torch.optim.Adam.step() (no weight decay, no amsgrad):
 * g' = grad_scale * grads (1 / world size after a summing all-reduce),
 * scaled by min(1, max_norm / (|g'|_2 + 1e-6)) (max_norm <= 0: no clipping),
 * then exp_avg, exp_avg_sq and params updated in place with the bias
 * corrections of `step` (>= 1, the step being taken).  grads is not written.
 * scratch: mas_policy_adam_scratch() floats. */
int64_t mas_policy_adam_scratch(void);
int mas_policy_adam(int64_t n, float* params, const float* grads, float* exp_avg, float* exp_avg_sq, float grad_scale,
                    float max_norm, double lr, double beta1, double beta2, double eps, int64_t step, float* scratch,
                    void* stream);

/* mas_policy_dw: the weight and bias gradients of one policy layer from the
 * feature-major activations mas_policy_train writes, over the minibatch rows:
 * out[F*G + F] = (a [F][K] . b [G][K]^T, row sums of a) in fp32, a / b bf16
 * with K contiguous (row strides lda / ldb >= K, multiples of 8, 16-B aligned
 * rows); F = 256 (dW2 from dA2 and h1) or 16 (dW3 from dz and h2), G = 256,
 * K a multiple of 32.  scratch: mas_policy_dw_scratch(F, G, K) floats of
 * split-K partial sums.  Replaces the caller's GEMMs over the ones-row trick
 * for layers 2 and 3 (K % 64 == 0: the LDS-staged kernel); the dW1 GEMM
 * reads x row-major and stays a GEMM. */
int64_t mas_policy_dw_scratch(int32_t f, int32_t g, int64_t k);
int mas_policy_dw(int32_t f, int32_t g, int64_t k, const void* a, int64_t lda, const void* b, int64_t ldb, float* out,
                  float* scratch, void* stream);

/* Diagnostics (synchronises the device): host_out[0] = envs of the last
 * mas_step that left the contact-free physics fast path and ran the general
 * physics kernel (contacts, TOI events, box despawns). */
int mas_debug_counters(mas_handle* h, int64_t* host_out);

/* Diagnostics (synchronises the device): host_out[0] = appends to the
 * general-path env list (and the slow list) that their bounds refused since
 * mas_create.  The lists hold one entry per env and are emptied every step,
 * so this is 0 unless a kernel breaks that invariant; the tests assert it. */
int mas_debug_guards(mas_handle* h, int64_t* host_out);

/* Test diagnostics: bit 0 of `on` sends every env of every following
 * mas_step through the general physics path (the contact-free fast path
 * gives up for all envs); bit 1 runs the general path one lane per env
 * (k_gen_solve + k_gen_toi) instead of on lane groups (k_gen_solve_g) -- only
 * in the test library libmas_ab.so (`make ab`), MAS_ERR_UNSUPPORTED here;
 * bit 3 keeps mas_step on the caller's stream.  Default (MAS_SPLIT unset or
 * 2 in the environment at mas_create): the slow split, the envs whose last
 * general-path step had a SolveTOI at the sub-step cap (or >= MAS_SLOW_K,
 * default 4, TOI events) run their general path and post phases on the side
 * stream while the caller's stream runs the rest; it is on for 8 steps after
 * the general kernels last flagged such an env (a host-mapped signal), else
 * mas_step runs on one stream.  Bit 3 (or MAS_SPLIT=0): the caller's stream
 * alone -- the form a caller may capture into a graph and replay (the
 * general-path list is emptied on the device).  Bit 2 (the former
 * all-general split) is rejected with MAS_ERR_INVALID_ARG.  Results are
 * unchanged (every path is exact): A/B and parity tests only. */
int mas_debug_force_general(mas_handle* h, int32_t on);

/* Action validation.  The reference asserts action_space.contains(actions)
 * before every step (masurvival_env.py:80).  A kernel cannot raise, so
 * mas_step clamps each out-of-range entry into MultiDiscrete([3,3,3,2,2,2])
 * and counts the env-step; this returns that count since the handle was
 * created or last reset (synchronises; reset != 0 zeroes it).  The Python
 * facades check on the host before calling (MaSurvival.step always,
 * VecMaSurvival.step(validate=True)). */
int mas_invalid_actions(mas_handle* h, int64_t* host_count, int32_t reset);

/* Test diagnostics: copies the per-env "left the contact-free fast path in
 * the last mas_step" flags (uint8 [n_envs], device) into `flags`
 * (stream-ordered; no synchronisation). */
int mas_debug_gen_flags(mas_handle* h, uint8_t* flags, void* stream);

/* Test diagnostics: while `counts` (device int32 [n_envs], or NULL to stop)
 * is set, every mas_step adds per env the number of b2World::SolveTOI
 * events of its agents, plus 65536 for each agent whose SolveTOI reached
 * Box2D's sub-step cap (b2_maxSubSteps = 8 per contact). */
int mas_debug_set_toi_counter(mas_handle* h, int32_t* counts);

const char* mas_last_error(void);
int32_t mas_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* MASURVIVAL_H */
