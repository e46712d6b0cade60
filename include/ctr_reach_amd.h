/*
 * ctr_reach_amd.h -- C ABI of libctr_reach_amd.so, the MI355X (gfx950) batched
 * concentric-tube-robot reach environment.
 *
 * Every entry point is extern "C", takes plain pointers and sizes, and is asynchronous
 * and stream-ordered: it enqueues HIP kernels on `stream` and returns without a device
 * synchronisation.  All device buffers are allocated and owned by the caller (PyTorch);
 * the library allocates nothing on the hot path.  Pointers marked "device" must be
 * device memory; structs themselves are read from host memory at call time.
 *
 * Return codes: 0 = ok, CTR_EINVAL (-1) = bad argument, CTR_EHIP (-2) = HIP launch error.
 * ctr_last_error() returns a thread-local description of the last failure.
 * Per-environment numeric faults (ODE step-size underflow, sampler exhaustion) are
 * reported through per-lane `status` words, never by aborting.
 *
 * Reference interfaces each entry point replaces (reference = keshaviyengar/gym-ctr-reach,
 * paths relative to ctr_reach_envs/):
 *   ctr_fk              Model.forward_kinematics(joint, system)          envs/model.py:30-70
 *                       (+ Segment envs/CTR_Python/Segment.py:6-61, ode_eq model.py:72-117,
 *                        ctr_model model.py:119-174, scipy solve_ivp RK45)
 *   ctr_set_action      Obs.set_action(action, system) x n_substeps       envs/obs.py:166-183,
 *                                                                          envs/ctr_reach_env.py:134-135
 *   ctr_step            CtrReachEnv.step(action)                          envs/ctr_reach_env.py:124-158
 *   ctr_reset           CtrReachEnv.reset(goal=None, system=None)         envs/ctr_reach_env.py:70-114
 *                       (+ Obs.sample_goal envs/obs.py:185-207, get_obs obs.py:136-164)
 *   ctr_compute_reward  CtrReachEnv.compute_reward(ag, dg, info)          envs/ctr_reach_env.py:160-170
 *   ctr_fk_tables       Model.forward_kinematics with per-row tube tables  envs/model.py:30-70
 *   ctr_fk_shape        Model.forward_kinematics + Model.r / r1 / r2 / r3  envs/model.py:30-70,119-174
 *   ctr_jacobian        CTR_Model.jac (finite differences)             envs/CTR_Python/CTR_Model.py:251-262
 *   ctr_domain_params   Model.current_sys_parameters after randomize_parameters
 *                                                                          envs/model.py:20-28, model_utils.py:5-35
 *   ctr_her_open / ctr_her_record / ctr_her_sample
 *                       the replay side of the reference's training pipeline: stable-baselines 2
 *                       HER (HindsightExperienceReplayWrapper.add / _store_episode /
 *                       _sample_achieved_goal, ReplayBuffer.sample) with the reference's
 *                       settings goal_selection_strategy 'future', n_sampled_goal 4
 *                       (saved_policies/.../her/CTR-Generic-Reach-v0_1/CTR-Generic-Reach-v0/
 *                       config.yml), fed by CtrReachEnv.compute_reward (ctr_reach_env.py:160-170)
 */
#ifndef CTR_REACH_AMD_H
#define CTR_REACH_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CTR_ABI_VERSION 15
#define CTR_MAX_SYSTEMS 8
#define CTR_POOL_MAX 192          /* ctr_batch_t.pool_depth limit (reset slots per environment) */
#define CTR_EINVAL (-1)
#define CTR_EHIP (-2)

/* per-lane status bits */
#define CTR_STATUS_STEP_UNDERFLOW 1u   /* scipy "Required step size is less than spacing" */
#define CTR_STATUS_SAMPLER_STUCK  2u   /* obs.py:204 "Stuck sampling goals..." (>1000 tries) */
#define CTR_STATUS_NAN            4u   /* model.py:69 assert not any(isnan(r)) */
#define CTR_STATUS_TOO_LONG       8u   /* fixed-step RK4: a segment needs > 2^20 steps (joints far
                                           outside the action box); the tip is NaN          */
#define CTR_STATUS_POOL_MISS     16u   /* CTR_AUTORESET_POOLED step: a done env found no pooled
                                           reset (the caller's no-miss promise was broken); the
                                           env stays done and is reset on a later step       */

/* ctr_step / ctr_step_her autoreset argument */
#define CTR_AUTORESET_OFF    0   /* done environments are left as they are                          */
#define CTR_AUTORESET_SWEEP  1   /* done environments are reset in the same call: from the reset pool
                                    if it holds their next reset, else by a miss sweep (a second,
                                    small launch that computes the missing resets)                  */
#define CTR_AUTORESET_POOLED 2   /* as SWEEP, but the caller guarantees every done environment finds
                                    its reset in the pool, so no sweep is launched: true when at most
                                    pool_depth steps have run since the last ctr_pool_refill (each
                                    step takes at most one reset per environment, and a refill leaves
                                    every environment's next pool_depth resets precomputed)          */

/* One 3-tube system (index 0 = innermost tube), derived on the host from the
 * registration kwargs exactly as Tube.__init__ (envs/CTR_Python/Tube.py:7-19):
 * EI = E * pi (d_o^4 - d_i^4) / 64, GJ = G * pi (d_o^4 - d_i^4) / 32. */
typedef struct ctr_system_t {
    double L[3];       /* tube length                        (Tube.L)    */
    double Lc[3];      /* pre-curved length                  (Tube.L_c)  */
    double EI[3];      /* bending stiffness  E * I                       */
    double GJ[3];      /* torsional stiffness G * J                      */
    double Ux[3];      /* pre-curvature x    (Tube.U_x)                  */
    double Uy[3];      /* pre-curvature y    (Tube.U_y)                  */
} ctr_system_t;

/* Raw tube inputs of Tube.__init__ (envs/CTR_Python/Tube.py:7-19) for one system, needed only
 * by domain randomisation, which re-samples them every reset (envs/model_utils.py:5-35). */
typedef struct ctr_tube_raw_t {
    double Din[3];     /* diameter_inner                                 */
    double Dout[3];    /* diameter_outer                                 */
    double E[3];       /* stiffness                                      */
    double G[3];       /* torsional_stiffness                            */
} ctr_tube_raw_t;

/* Integrator selection */
#define CTR_INTEGRATOR_RK45_SCIPY 0    /* scipy solve_ivp RK45 emulation, rtol 1e-3 atol 1e-6 (parity) */
#define CTR_INTEGRATOR_RK4        1    /* fixed-step classical RK4 of the same ODE (throughput)       */

/* Mechanics model */
#define CTR_MODEL_COMPLIANT 0          /* torsionally compliant (the reference, model.py:72-117)        */
#define CTR_MODEL_RIGID     1          /* torsionally rigid: GJ -> infinity, tube angles constant       */

/* Environment configuration (registration kwargs, ctr_reach_envs/__init__.py:6-94). */
typedef struct ctr_env_config_t {
    int32_t n_systems;          /* len(select_systems), 1..CTR_MAX_SYSTEMS              */
    int32_t n_substeps;         /* n_substeps (10)                                       */
    int32_t max_steps;          /* max_steps_per_episode (150)                           */
    int32_t constrain_alpha;    /* constrain_alpha                                       */
    int32_t egocentric;         /* joint_representation == 'egocentric'                  */
    int32_t resample_joints;    /* resample_joints                                       */
    int32_t integrator;         /* CTR_INTEGRATOR_*                                      */
    int32_t rk4_steps_per_m;    /* RK4 only: steps per metre of arclength (> 0)          */
    int32_t model;              /* CTR_MODEL_*                                           */
    int32_t obs_f64;            /* observation buffers (ctr_step_out_t.obs / terminal_obs,
                                   ctr_reset's obs): 0 = float32 [n][obs_dim], 1 = float64
                                   [n][obs_dim], the reference's dtype (obs.py:153-156).
                                   The values are computed in float64 either way.        */
    double  tol;                /* goal_tolerance.get_tol()                              */
    uint64_t seed;              /* Philox key for resets                                 */
    ctr_system_t systems[CTR_MAX_SYSTEMS];
    /* Domain randomisation (domain_rand kwarg; Model.randomize_parameters, model.py:20-28, called
     * by reset, ctr_reach_env.py:80).  0 = off.  Otherwise every reset draws, per tube, d_in,
     * d_out, E, G and U_x uniformly in v * [1 - domain_rand, 1 + domain_rand] (L, L_c, U_y are
     * kept) from Philox stream 3 keyed (seed, global env id, reset number), and the episode's
     * FKs use the tube table derived from them.  raw[] holds the unrandomised inputs. */
    double domain_rand;
    double domain_pad;
    ctr_tube_raw_t raw[CTR_MAX_SYSTEMS];
} ctr_env_config_t;

/* Device-resident batch state, row-major per environment ([n][k]). */
/* One precomputed reset of the pool (ABI 15): 128 B, one cache line when the pool is 128-B
 * aligned, so a pooled auto-reset reads one line (the ABI-14 [P][n][k] arrays spread it over 7). */
typedef struct ctr_pool_slot_t {
    double   dg[3];              /* desired goal                   bytes   0 -  23 */
    double   ag[3];              /* start position (its FK tip)            24 -  47 */
    float    qd[6];              /* desired joints                         48 -  71 */
    float    q0[6];              /* start joints                           72 -  95 */
    int32_t  sys;                /* system index                           96      */
    uint32_t stat;               /* CTR_STATUS_* of the precomputation    100      */
    uint32_t r;                  /* reset number held (0 = empty)         104      */
    uint32_t pad[5];             /*                                       108 - 127 */
} ctr_pool_slot_t;

typedef struct ctr_batch_t {
    int64_t   n;                 /* environments in this shard                        */
    int64_t   env_base;          /* global id of environment 0 (RNG key; sharding)    */
    float    *joints;            /* [n][6] f32 [b0,b1,b2,a0,a1,a2] (Obs.joints)       */
    double   *desired_goal;      /* [n][3]                                            */
    double   *achieved_goal;     /* [n][3] tip after the last step / reset            */
    int32_t  *t;                 /* [n] steps taken in the episode                    */
    int32_t  *system;            /* [n] index into config.systems                     */
    uint32_t *epoch;             /* [n] resets taken so far (RNG counter)             */
    float    *desired_joints;    /* [n][6] or NULL (info q_desired)                   */
    float    *starting_joints;   /* [n][6] or NULL (info q_starting)                  */
    double   *starting_position; /* [n][3] or NULL                                    */
    int32_t  *work;              /* [n+2] auto-reset miss list: 2 counters, then ids  */
    int32_t   work_parity;       /* host toggles 0/1 every ctr_step: which counter   */
    int32_t   work_pad;
    /* Reset pool (optional, pool_depth 0 disables it).  Resets are a deterministic function of
     * (seed, global env id, reset number), so they can be computed ahead of time: slot (r mod P)
     * of env e holds reset number r (ctr_pool_slot_t.r), precomputed by ctr_pool_refill; an
     * auto-reset consumes it with a copy instead of two forward-kinematics solves.  A missing
     * slot falls back to computing the reset in the same ctr_step call.  Layout [P][n] of
     * 128-B slots (ABI 15; one cache line per reset, was [P][n][k] per field). */
    int32_t   pool_depth;        /* P (0 = no pool, at most CTR_POOL_MAX)             */
    int32_t   pool_pad;
    ctr_pool_slot_t *pool;       /* [P][n] slots, 128-B aligned, zero-initialised     */
    int32_t  *refill;            /* [2 + 2 refill_cap]: count, (env, reset number) pairs,
                                    then a completion ticket (zero-initialised)          */
    int64_t   refill_cap;
    /* Resumable refill (optional, carry NULL disables it; scipy RK45 on either model, and
     * fixed-step RK4 on the compliant model -- the rigid model's RK4 segment maps ignore it).
     * A reset at least
     * refill_lead resets ahead of its environment (r - epoch - 1 >= refill_lead at the time of
     * the refill) runs at most refill_budget iterations (segment start + RK45 attempt; one RK4
     * step) of each of its two FKs in one ctr_pool_refill; an unfinished one is suspended
     * into the carry list and resumed by the next ctr_pool_refill, which writes its pool slot
     * once both FKs are done.  The result is bit-identical; only the refill a reset lands in
     * changes.  With refill_lead >= the steps between refills, no reset is due before it lands
     * (after every refill, the resets fewer than refill_lead ahead are in the pool).  */
    void     *carry;             /* ctr_refill_carry_bytes(carry_cap) B, zero-initialised */
    int64_t   carry_cap;         /* resets each of its two lists holds                 */
    int32_t   refill_budget;     /* iterations (RK4 steps) per FK and refill (0 = none) */
    int32_t   refill_lead;
} ctr_batch_t;

typedef struct ctr_gather_push_t ctr_gather_push_t;   /* defined with the push gather below */

/* Per-step outputs (device). obs_dim = 13, or 14 when n_systems > 1 (obs.py:153-156). */
typedef struct ctr_step_out_t {
    void     *obs;               /* [n][obs_dim]   observation after the step (after auto-reset);
                                    float32, or float64 with cfg->obs_f64                         */
    float    *reward;            /* [n]            0 or -1                                       */
    uint8_t  *done;              /* [n]                                                          */
    uint8_t  *success;           /* [n]            info['is_success']                            */
    float    *error;             /* [n]            info['error'] = ||dg - ag||                   */
    void     *terminal_obs;      /* [n][obs_dim] or NULL: pre-reset observation of done envs
                                    (the dtype of obs)                                           */
    double   *terminal_achieved; /* [n][3] or NULL: achieved goal of the terminal step           */
    uint32_t *status;            /* [n] or NULL: CTR_STATUS_* bits                               */
    uint32_t *nfev;              /* [n] or NULL: RHS evaluations spent in the step's FK          */
    float    *packed;            /* [n][4] (16-B aligned) or NULL: the step's outputs packed for
                                    the optional all-gather of a single-process trainer: tip x, y,
                                    z (float32; the terminal achieved goal of a done env) and
                                    done | success << 1 | (reward == -1) << 2 as a float (the
                                    reward is -1 or 0).  Written by k_step itself, so gathering
                                    costs no packing launch.                                      */
    uint32_t  packed_seq;        /* != 0 (with packed): k_step also writes row n of packed as
                                    (packed_seq, 0, 0, 0) as uint32 bits, the step's sequence word
                                    that ctr_copy_list pushes after the rows (packed then holds
                                    n + 1 rows).  0: row n is not touched.                        */
    uint32_t  packed_pad;
    const ctr_gather_push_t *gather;      /* device or NULL: the fused push gather of step
                                             gather_seq (descriptor of its slot) -- k_step also
                                             stores each env's packed row (as in `packed`) into
                                             every rank's receive slot, gather->dst[p] + e for
                                             p < gather->world (IPC-mapped peer memory), after
                                             every rank has released that slot (flow control,
                                             see "Push all-gather"), as system-scope stores the
                                             storing wave waits for.  The first
                                             lanes also release this rank's slot of step
                                             gather_seq + 1 - depth to every producer          */
    const ctr_gather_push_t *gather_prev; /* device or NULL: the first lanes of k_step publish
                                             gather_prev_seq to every gather_prev->seqw[p]
                                             (system scope) -- the previous gathered
                                             step, whose launch has completed (so its row stores
                                             are performed at system scope) before this one
                                             starts                                              */
    uint32_t  gather_prev_seq;
    uint32_t  gather_seq;        /* the step pushed with `gather` (wraps modulo 2^32)            */
    int32_t   gather_wait_prev;  /* != 0 (with gather, depth >= 3): k_step also waits until every
                                    rank's rows of step gather_seq - 1 are published in this
                                    rank's ring (gather->wait_seqw), so after this launch the
                                    previous step's gathered slot is readable on the stream (the
                                    fused consumer wait; errors in gather->err)                  */
    int32_t   gather_pad;
} ctr_step_out_t;

/* ---------------------------------------------------------------------------------------
 * HER replay feed (device).  Episodes are recorded where the environments run and relabelled
 * with stable-baselines 2 HER semantics:
 *   - an episode enters the replay store when it ends (HindsightExperienceReplayWrapper.add
 *     stores on done); its L transitions become L real rows plus, per transition t, k relabelled
 *     rows (FUTURE: none for the last transition), in _store_episode's order;
 *   - a relabelled row of transition t takes the achieved goal of obs_sel, the observation
 *     before transition sel (_sample_achieved_goal returns selected_transition[0]'s
 *     achieved_goal): FUTURE sel ~ U{t+1 .. L-1}, FINAL sel = L-1, EPISODE sel ~ U{0 .. L-1};
 *     its reward is compute_reward(achieved goal of obs_{t+1}, goal) at the tolerance in force
 *     when the episode ended, its done is 0; only the desired_goal slots change (the
 *     'observation' part, which holds dg - ag, is kept, as the wrapper keeps it);
 *   - ctr_her_sample draws rows uniformly with replacement over all stored rows
 *     (ReplayBuffer.sample) and returns them in HERGoalEnvWrapper's flat layout
 *     [observation, achieved_goal, desired_goal].
 * Storage: each environment owns `slots` episode slots used round-robin (slot of episode r of
 * env e = e * slots + r mod slots), so the store keeps each env's last slots - 1 finished
 * episodes (first-in first-out per env; stable-baselines drops the globally oldest rows).
 * The sel draws are a pure function of (seed, global env id, reset number, t, j) (Philox
 * stream 4): they are fixed per row, as the wrapper fixes them when it stores the episode. */
#define CTR_HER_FUTURE  0
#define CTR_HER_FINAL   1
#define CTR_HER_EPISODE 2

typedef struct ctr_her_t {
    int32_t  obs_dim;          /* 13 or 14                                                  */
    int32_t  t_max;            /* longest episode (max_steps_per_episode), <= 65535          */
    int32_t  n_sampled_goal;   /* k (4), <= 255                                              */
    int32_t  strategy;         /* CTR_HER_*                                                  */
    int64_t  n;                /* environments                                               */
    int64_t  env_base;         /* global id of environment 0 (keys the relabel draws)       */
    int32_t  slots;            /* episode slots per environment (>= 2)                      */
    int32_t  pad;
    uint64_t seed;             /* Philox key of the relabel draws                            */
    /* episode store, E = n * slots slots (device) */
    /* slot id = env * slots + s.  Rows are env-minor ([slots][t][n]) so the lanes of a wave,
     * consecutive envs mostly at the same (slot, t), write one contiguous span, and 16-B
     * aligned so every row is whole dwordx4 stores; a sampled row is one or two cache lines. */
    float    *state;           /* [slots][t_max + 1][n][24], 96-B rows: floats 0 .. obs_dim-1 =
                                  obs_t (obs_0 .. obs_L), floats 16 .. 21 = its achieved goal
                                  as 3 doubles                                                */
    float    *step;            /* [slots][t_max][n][8], 32-B rows: action 0..5, reward 6      */
    double   *dg;              /* [E][3]                   the episode's desired goal         */
    double   *tol;             /* [E]                      tolerance when the episode ended   */
    int32_t  *len;             /* [E]   L of a stored episode; 0 = empty, -1 = being recorded */
    uint32_t *epoch;           /* [E]   reset number of the episode in the slot              */
    /* per environment (device) */
    int32_t  *cur_t;           /* [n]   transitions recorded in the open episode; -1 = none  */
    uint32_t *cur_epoch;       /* [n]   reset number of the open episode                     */
    /* sampler scratch (device), CTR_HER_CDF_LEN(n * slots) int64: every ctr_her_sample call
     * rebuilds the prefix sums of the stored rows per slot here, so a draw is one search */
    int64_t  *cdf;
} ctr_her_t;

#define CTR_HER_SCAN_TILE 1024     /* slots per scan tile of the sampler's prefix sums */
#define CTR_HER_CDF_LEN(E) ((E) + ((E) + CTR_HER_SCAN_TILE - 1) / CTR_HER_SCAN_TILE + 1)

/* Flat sampled batch (device), d = obs_dim + 6. */
typedef struct ctr_her_batch_t {
    float   *obs;              /* [B][d]  [observation_t, achieved_goal_t, desired_goal]      */
    float   *action;           /* [B][6]                                                      */
    float   *reward;           /* [B]                                                         */
    float   *next_obs;         /* [B][d]  [observation_t+1, achieved_goal_t+1, desired_goal]  */
    float   *done;             /* [B]     1 for the last real transition of an episode        */
    int32_t *index;            /* [B][3] or NULL: (slot, t, j), j = 0 real, 1..k relabelled;
                                  slot -1: the store holds no rows (the row is zeros)        */
} ctr_her_batch_t;

/* Opens an episode for the environments with mask[i] != 0 (NULL = all) from the batch's
 * current state (after ctr_reset): obs_0 = obs [n][obs_dim], its achieved goal, the desired
 * goal and the reset number.  An episode still open in that env is discarded. */
int ctr_her_open(const ctr_her_t *her, const ctr_batch_t *batch, const float *obs, const uint8_t *mask,
                 void *stream);

/* Records the step that ctr_step (autoreset on) just made: action [n][6], out's reward / done /
 * obs / terminal_obs / terminal_achieved (terminal_* required).  A done env's episode is closed
 * with the tolerance tol and stored; the env's next episode is opened from the post-reset
 * state. */
int ctr_her_record(const ctr_her_t *her, const ctr_batch_t *batch, const float *actions,
                   const ctr_step_out_t *out, double tol, void *stream);

/* ctr_step + ctr_her_record in one pass: k_step writes the step's transition into the store as
 * it finishes each env (no second launch, no re-read of the step outputs), and opens the next
 * episode of every env it auto-resets (the miss sweep does it for the envs it resets).  Same
 * arguments and outputs as ctr_step; terminal_obs / terminal_achieved may be NULL here. */
int ctr_step_her(const ctr_env_config_t *cfg, const ctr_batch_t *batch, const float *actions,
                 const ctr_step_out_t *out, int32_t autoreset, const ctr_her_t *her, void *stream);

/* Draws B rows uniformly with replacement over the stored rows: one uniform integer u per row
 * (keyed seed, counter, row) below the stored-row count, mapped to its (slot, row) through the
 * per-slot prefix sums this call rebuilds in her->cdf (exact inverse CDF: no retries, no
 * misses whatever the episode lengths). */
int ctr_her_sample(const ctr_her_t *her, int64_t batch_size, uint64_t seed, uint64_t counter,
                   const ctr_her_batch_t *out, void *stream);

int ctr_abi_version(void);
const char *ctr_last_error(void);

/* Batched Model.forward_kinematics: joints [n][6] f32 -> tip [n][3] f64.
 * sys_idx: [n] or NULL (all system 0).  stats: [n][4] or NULL = {RHS evaluations, accepted
 * RK steps, rejected RK attempts, integrated segments}.  Fixed-step RK4 never rejects; there
 * stats[1] counts the steps taken stage by stage and stats[2] the executed work of the segments
 * run as segment maps (matrix powers: every segment of the rigid model, the trailing segments of
 * the compliant model where tube 0 is alone): maps << 16 | square-and-multiply compositions.
 * stats[0] counts 4 RHS per RK4 step, mapped or not (the oracle's count).  status: [n] or NULL.
 * (device) */
int ctr_fk(const float *joints, const int32_t *sys_idx, int64_t n, const ctr_env_config_t *cfg,
           double *tip, uint32_t *stats, uint32_t *status, void *stream);

/* Model.forward_kinematics with one tube table per row: tables [n] (device), e.g. the
 * domain-randomised tables from ctr_domain_params (the reference integrates with
 * Model.current_sys_parameters, model.py:13,30).  cfg supplies the integrator and model. */
int ctr_fk_tables(const float *joints, const ctr_system_t *tables, int64_t n, const ctr_env_config_t *cfg,
                  double *tip, uint32_t *stats, uint32_t *status, void *stream);

/* Model.forward_kinematics with the backbone shape (Model.r, model.py:66-68 and ctr_model
 * model.py:119-174): besides the tip, r at the 30 sorted linspace points of every segment
 * (solve_ivp t_eval, RK45 dense output) and their arclengths s (ctr_model's Length), row-major
 * r [n][cap][3], s [n][cap]; npts [n] = 30 x segments (points past cap are not stored).
 * cap = 270 always suffices (<= 9 segments).  tables [n] or NULL: per-row tube tables as in
 * ctr_fk_tables (sys_idx is then ignored).  Needs integrator rk45_scipy.  (device) */
int ctr_fk_shape(const float *joints, const int32_t *sys_idx, const ctr_system_t *tables, int64_t n,
                 const ctr_env_config_t *cfg, int32_t cap, double *tip, double *r, double *s, int32_t *npts,
                 uint32_t *status, void *stream);

/* Forward-difference tip Jacobian d tip / d q over float64 joints [n][6] (device):
 * jac[n][3][6] = (tip(q + eps e_i) - tip(q)) / eps, the scheme of CTR_Model.jac
 * (envs/CTR_Python/CTR_Model.py:251-262, eps 1e-4 there) applied to Model.forward_kinematics;
 * the 7 FKs of an env run on 7 lanes.  tip [n][3] (the unperturbed FK) and status may be NULL;
 * status bits are OR-ed in. */
int ctr_jacobian(const double *joints, const int32_t *sys_idx, int64_t n, const ctr_env_config_t *cfg, double eps,
                 double *tip, double *jac, uint32_t *status, void *stream);

/* n_substeps x Obs.set_action, in place on joints [n][6] (device). */
int ctr_set_action(const ctr_env_config_t *cfg, float *joints, const int32_t *sys_idx,
                   const float *actions, int64_t n, void *stream);

/* One CtrReachEnv.step for every environment of the batch; actions [n][6] f32 (device).
 * autoreset (CTR_AUTORESET_*) != 0: done environments are reset in the same call (VecEnv
 * semantics) and their pre-reset observation goes to out->terminal_obs. */
int ctr_step(const ctr_env_config_t *cfg, const ctr_batch_t *batch, const float *actions,
             const ctr_step_out_t *out, int32_t autoreset, void *stream);

/* CtrReachEnv.reset for the environments with mask[i] != 0 (mask NULL = all).
 * goal [n][3] or NULL (sample a goal), system [n] or NULL (sample uniformly).
 * Writes the reset observation to obs [n][obs_dim]. */
int ctr_reset(const ctr_env_config_t *cfg, const ctr_batch_t *batch, const uint8_t *mask,
              const double *goal, const int32_t *system, void *obs, uint32_t *status, void *stream);

/* Precompute the resets queued in batch->refill (queued by ctr_step when a pooled reset is
 * consumed, and by ctr_reset for the P resets after the one it computes), then clear the
 * queue.  Call it every few steps; it is a no-op when the queue is empty. */
int ctr_pool_refill(const ctr_env_config_t *cfg, const ctr_batch_t *batch, void *stream);

/* Bytes of batch->carry for carry_cap resets per list (a header, then two lists of suspended
 * resets, each in 64 sub-lists); int32 counts[2][64] at byte 0 of the header give the resets each
 * sub-list holds (diagnostics). */
int64_t ctr_refill_carry_bytes(int64_t carry_cap);

/* Queue every environment's next pool_depth resets (epoch + 1 .. epoch + P) that its pool slots
 * do not hold, e.g. after the batch state was restored from a checkpoint or the seed changed;
 * the next ctr_pool_refill computes them.  Also empties both of the refill's suspended lists
 * (batch->carry: their resets are not in the pool, so they are queued again).  A suspended reset
 * the refill finds its environment has passed (a miss sweep computed it) or its slot already
 * holding is dropped, as a queued one is. */
int ctr_pool_requeue(const ctr_env_config_t *cfg, const ctr_batch_t *batch, void *stream);

/* The tube table each environment's current episode uses (Model.current_sys_parameters,
 * model.py:13,20-28): with domain randomisation the episode's re-sampled table, else the
 * environment's system row.  sys_out [n] (derived, as the FK uses it) and raw_out [n] (the
 * re-sampled Tube inputs; U_x is in sys_out) may each be NULL.  (device) */
int ctr_domain_params(const ctr_env_config_t *cfg, const ctr_batch_t *batch, ctr_system_t *sys_out,
                      ctr_tube_raw_t *raw_out, void *stream);

/* ---------------------------------------------------------------------------------------
 * Push all-gather of the packed step rows (BASELINE configs[3]: a single-process trainer that
 * wants every GPU's tip / reward / done; no reference counterpart -- the reference runs one env
 * per process).  Each rank pushes its [n][4] block of packed rows into every rank's receive ring
 * (IPC-mapped), then the block's sequence word into the receiver's sequence words (uncached device
 * memory).  Engines: the fused push (ctr_step_out_t.gather: k_step itself stores every env's row
 * into every rank's slot, and the next launch publishes the sequence words), ctr_gather_push (the
 * same stores as a standalone slim kernel), and ctr_copy_list, copy-engine copies (no CU at all,
 * but host-synchronous per copy in this runtime; the sequence word then comes from row n of the
 * packed rows, written by k_step: ctr_step_out_t.packed_seq).  RCCL's collective kernels, the
 * other option, cannot share a SIMD with k_step, so they hold CUs the next step needs.
 * A consumer waits for a step with ctr_gather_wait.  The host side
 * (ctr_reach_amd.distributed.PushGather) plans the destinations: receive ring
 * [depth][world][n][4] float32 (rank-major = global env id order within a slot), sequence words
 * [depth][world] uint32, release words [world] uint32.
 *
 * Ordering of the fused push (ABI 13).  Step t's rows are stored by the waves of k_step(t) with
 * system-scope stores (sc0 sc1: written through this GPU's L2) that each storing wave waits for
 * before it ends (performed at system scope), and k_step(t + 1), which the stream starts only
 * after k_step(t) has completed, publishes t's sequence words with system-scope stores.  A
 * consumer that acquires the words (system scope) therefore reads rows at least as new as step
 * t; the receive ring is uncached device memory, so the consumer's own L2 holds no stale line.
 * Flow control: slot t % depth is rewritten by step t + depth.  Consumer c releases its slot of
 * step s when it launches step s + depth - 1 (k_step's first lanes store s into every producer's
 * release word for c), so a gathered view of step s stays valid until this rank launches step
 * s + depth - 1; a producer's k_step(t) stores its rows only after every consumer has released
 * step t - depth (a bounded wait; on time-out the rows are stored anyway and err gets
 * CTR_GATHER_E_RELEASE_TIMEOUT).  ctr_gather_push and ctr_copy_list do not take part in the
 * flow control: their callers pace the ranks.
 * A time-out is also reported to the consumer it overran (ABI 14): before storing any row, the
 * producer stores the step into its poison word in the memory of every consumer that had not
 * released the slot (system scope, waited for), and every k_step with gather_wait_prev folds the
 * consumer's own poison words into its err (CTR_GATHER_E_RELEASE_TIMEOUT).  So err, read after a
 * view's readers have run (the next fused step, or PushGather.err_bits()), covers every overwrite
 * that reached the view -- no cross-rank reduction is needed to trust a local view.
 * Every bounded wait has a wall-clock budget (wait_us, s_memrealtime at 100 MHz), not a poll count.
 * ------------------------------------------------------------------------------------- */
#define CTR_IPC_HANDLE_BYTES 64
#define CTR_GATHER_MAX_RANKS 16
/* err bits of ctr_gather_wait and of the fused push (ctr_gather_push_t.err) */
#define CTR_GATHER_E_WAIT_TIMEOUT    1u   /* a consumer wait gave up after wait_us microseconds  */
#define CTR_GATHER_E_OVERWRITTEN     2u   /* a sequence word was already past the awaited step   */
#define CTR_GATHER_E_RELEASE_TIMEOUT 4u   /* a fused push stored into a slot not yet released
                                              (in the producer's err, and via the poison words in
                                              the err of the consumer it overran)                */
#define CTR_GATHER_E_PREV_TIMEOUT    8u   /* the fused consumer wait (gather_wait_prev) gave up  */

/* One rank's push of its block: the host struct of ctr_gather_push, and (in device memory) the
 * per-slot descriptor of the fused push (ctr_step_out_t.gather; src and ticket unused there). */
struct ctr_gather_push_t {
    const void *src;                          /* [n][4] float32 packed rows (16-B aligned)     */
    int64_t     n;
    int32_t     world;
    int32_t     pad;
    void       *dst[CTR_GATHER_MAX_RANKS];    /* rank p's copy of this block: its receive ring
                                                 slot + rank * n rows (IPC-mapped)           */
    uint32_t   *seqw[CTR_GATHER_MAX_RANKS];   /* this block's sequence word in rank p's memory  */
    uint32_t   *ticket;                       /* this rank's device word, zero-initialised (the
                                                 kernel leaves it zero)                      */
    /* fused push only (ABI 13): */
    uint32_t   *relw[CTR_GATHER_MAX_RANKS];   /* this rank's release word in rank p's memory   */
    const uint32_t *rel;                      /* [world] this rank's release words: rel[c] = the
                                                 last step whose slot consumer c released   */
    const uint32_t *wait_seqw;                /* [world] this rank's sequence words of the
                                                 previous slot (gather_wait_prev)           */
    uint32_t   *err;                          /* device word: CTR_GATHER_E_* bits             */
    int32_t     depth;                        /* ring slots (>= 2)                            */
    uint32_t    wait_us;                      /* wall-clock budget of every bounded wait, in
                                                 microseconds (ABI 14; was a poll count)     */
    /* ABI 14: */
    uint32_t   *poisonw[CTR_GATHER_MAX_RANKS];/* this rank's poison word in rank p's memory: on a
                                                 release time-out, step seq (1 if seq has
                                                 wrapped to 0) is stored into the words of the
                                                 consumers that had not released; a NULL entry
                                                 = not enabled for that consumer             */
    const uint32_t *poison;                   /* [world] this rank's poison words (producer p's
                                                 at [p]; zeroed, sticky): non-zero = a producer
                                                 overwrote a slot this rank had not released;
                                                 NULL = not enabled (only the producer's err
                                                 reports an overrun then)                    */
};

/* Enqueue the push kernel: the n rows to every dst[p] (p < world), then seq to every seqw[p]
 * (after all rows, release at system scope).  workgroups: grid size (e.g. 128); its waves use
 * ~20 VGPRs and no LDS, so they share SIMDs with k_step waves.  No flow control (see above). */
int ctr_gather_push(const ctr_gather_push_t *g, uint32_t seq, int32_t workgroups, void *stream);

/* Publish seq to every g_dev->seqw[p] (system scope) after the work already on
 * `stream`: the fused push's explicit publication of its last step (k_step publishes the previous
 * step itself, ctr_step_out_t.gather_prev).  g_dev: device descriptor.  One wave. */
int ctr_gather_publish(const ctr_gather_push_t *g_dev, uint32_t seq, void *stream);

/* hipIpcGetMemHandle of a device allocation (handle: CTR_IPC_HANDLE_BYTES bytes, host). */
int ctr_ipc_get_handle(const void *dev_ptr, void *handle);
/* Map another process's allocation (hipIpcOpenMemHandle, peer access enabled lazily). */
int ctr_ipc_open(const void *handle, void **dev_ptr);
int ctr_ipc_close(void *dev_ptr);

/* Uncached device memory for sequence words (zeroed; synchronous).  The only entry points that
 * allocate: the words are written by other GPUs' copy engines and polled by ctr_gather_wait,
 * so they must not sit in this GPU's L2. */
int ctr_seqw_alloc(int64_t bytes, void **dev_ptr);
int ctr_seqw_free(void *dev_ptr);

/* One copy of a copy list. */
typedef struct ctr_copy_t {
    void       *dst;
    const void *src;
    int64_t     bytes;
    int32_t     stream;      /* index into the streams of ctr_copy_list */
    int32_t     pad;
} ctr_copy_t;

/* Enqueue copy-engine copies (hipMemcpyDeviceToDeviceNoCU): every stream first waits for
 * ready_event (NULL: no wait), then runs its copies in list order, then records
 * done_events[s] (NULL array or entry: none).  Copies on one stream are ordered, so a sequence
 * word listed after its block lands after it. */
int ctr_copy_list(const ctr_copy_t *copies, int32_t n_copies, void *const *streams, int32_t n_streams,
                  void *ready_event, void *const *done_events);

/* Consumer side: enqueue on `stream` a one-wave kernel that waits until seqw[i] reaches seq for
 * every i < n (wrap-aware uint32 compare; seqw is uncached, polled at system scope), then
 * returns.  err (device, uint32) gets bit 1 if wait_us microseconds pass first (the kernel then
 * returns anyway: no unbounded wait) and bit 2 if a word is already past seq (the slot was
 * overwritten by a later step before it was consumed). */
int ctr_gather_wait(const uint32_t *seqw, int32_t n, uint32_t seq, uint32_t wait_us, uint32_t *err,
                    void *stream);

/* Batched compute_reward over leading dims: ag, dg [n][3] f64 -> reward [n] f32 in {-1, 0}. */
int ctr_compute_reward(const double *achieved, const double *desired, int64_t n, double tol,
                       float *reward, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* CTR_REACH_AMD_H */
