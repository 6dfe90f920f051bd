/*
 * hwy.h -- C ABI of libhwy.so, the MI355X-native vectorised highway-v0 step.
 *
 * This is the drop-in boundary for the hot path named in BASELINE.json:north_star.
 * Every entry point below replaces one reference interface (reference = DhruvDh/highway-rope-ppo,
 * paths relative to its repo root; highway-env 1.10.1 is the third-party package the reference
 * calls, pinned at uv.lock:163-178 and NOT vendored):
 *
 *   hwy_create / hwy_destroy  <- gym.make("highway-v0", config=cfg)      experiments/wrappers.py:80
 *                                env.close()                             experiments/runner.py:139-142
 *   hwy_reset                 <- env.reset(seed=exp_seed + episode_num)  training/routine.py:127
 *                                env.reset(seed=exp_seed + 1000 + ep)    training/routine.py:18
 *   hwy_step                  <- env.step(action)                        training/routine.py:24,134
 *                                (AbstractEnv.step/_simulate, HighwayEnv._reward/_is_terminated/
 *                                 _is_truncated, KinematicObservation.observe [highway-env 1.10.1])
 *                                + the PE wrapper's .observation() fused in (pe_kind != 0)
 *   hwy_set_pe_table          <- RankEmbedWrapper.__init__ table         experiments/rank_embed.py:21-22
 *                                DistanceEmbedWrapper freqs               experiments/dist_embed.py:48-52
 *                                RotaryEmbedWrapper inv_freq              experiments/rope_embed.py:36-39
 *   hwy_obs_pe                <- RotaryEmbedWrapper.observation          experiments/rope_embed.py:64-74
 *                                RotaryEmbedWrapper._apply_rope          experiments/rope_embed.py:44-62
 *                                DistanceEmbedWrapper.observation        experiments/dist_embed.py:76-96
 *                                RankEmbedWrapper.observation            experiments/rank_embed.py:45-51
 *   hwy_gae                   <- PPOMemory.compute_advantages            ppo/agent.py:126-138
 *   hwy_set_seed_groups       <- one gym.make per experiment of a sweep  experiments/runner.py:73-78
 *   hwy_step_group            <- env.step of every cell of a sweep batch (one launch)
 *                                (main.py:188-242 fans the seeds out as separate processes; here
 *                                 a cell's seeds share one handle, each with its own schedule)
 *
 * Conventions
 *   - Plain pointers and sizes only; device pointers are HIP device pointers (e.g. torch
 *     tensor.data_ptr()), `stream` is a hipStream_t passed as void* (NULL = default stream).
 *   - All compute calls are stream-ordered and asynchronous; none allocates or synchronises,
 *     so they can be captured into a hipGraph.
 *   - Return value: 0 on success, <0 on error; hwy_last_error() gives a thread-local message.
 *     HWY_EINVAL errors are configuration errors (the Python layer raises ValueError, as the
 *     reference's make_env / wrapper constructors do).
 *   - A handle is not thread-safe; use one handle per GPU rank.
 */
#ifndef HWY_H_
#define HWY_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HWY_ABI_VERSION 1

#define HWY_MAX_VEHICLES 64 /* simulated vehicles per env incl. ego (one wavefront lane each) */
#define HWY_MAX_FEATURES 8  /* observation features per row */
#define HWY_MAX_OBS_ROWS 64 /* observed rows N */
#define HWY_MAX_FOUT 64     /* features per row after the PE wrapper */
#define HWY_MAX_PE_TABLE 4096

#define HWY_OK 0
#define HWY_EINVAL (-1)
#define HWY_EDEVICE (-2)
#define HWY_ENOMEM (-3)

/* Kinematics observation features (KinematicObservation FEATURES / Vehicle.to_dict keys). */
enum hwy_feature {
  HWY_FEAT_PRESENCE = 0,
  HWY_FEAT_X = 1,
  HWY_FEAT_Y = 2,
  HWY_FEAT_VX = 3,
  HWY_FEAT_VY = 4,
  HWY_FEAT_COS_H = 5,
  HWY_FEAT_SIN_H = 6,
  HWY_FEAT_HEADING = 7
};

enum hwy_order { HWY_ORDER_SORTED = 0, HWY_ORDER_SHUFFLED = 1 };

/* Observation wrapper fused into the step (experiments/wrappers.py:91-104). */
enum hwy_pe_kind {
  HWY_PE_NONE = 0,
  HWY_PE_RANK = 1,  /* RankEmbedWrapper */
  HWY_PE_DIST = 2,  /* DistanceEmbedWrapper(use_euclidean=True) */
  HWY_PE_ROPE = 3,  /* RotaryEmbedWrapper */
  HWY_PE_DIST1 = 4  /* DistanceEmbedWrapper(use_euclidean=False): |x_i - x_ego| */
};

/* Mirrors HIGHWAY_CONFIG (config/base_config.py:5-39) after make_env's deep merge and
 * order resolution (experiments/wrappers.py:33-57). */
typedef struct hwy_config {
  int32_t num_envs;        /* E: envs owned by this handle */
  int32_t lanes_count;     /* "lanes_count" (4) */
  int32_t vehicles_count;  /* "vehicles_count" (50 traffic cars; +1 ego simulated) */
  int32_t obs_vehicles;    /* observation "vehicles_count" N (15) */
  int32_t n_features;      /* F */
  int32_t feature_ids[HWY_MAX_FEATURES];      /* enum hwy_feature, row order */
  int32_t has_range[HWY_MAX_FEATURES];        /* feature has a features_range entry */
  float features_range[HWY_MAX_FEATURES][2];  /* [lo, hi] per feature */
  int32_t order;           /* enum hwy_order */
  int32_t absolute;        /* "absolute" */
  int32_t normalize;       /* "normalize" */
  int32_t clip;            /* KinematicObservation clip (default True) */
  int32_t see_behind;      /* KinematicObservation see_behind (default False) */
  int32_t sim_freq;        /* "simulation_frequency" (15) */
  int32_t policy_freq;     /* "policy_frequency" (1) */
  int32_t max_steps;       /* truncation horizon in policy steps (horizon) */
  int32_t initial_lane_id; /* "initial_lane_id" (-1 = random) */
  float vehicles_density;  /* "vehicles_density" (2) */
  float ego_spacing;       /* "ego_spacing" (2) */
  float speed_limit;       /* straight_road_network speed_limit (30) */
  float collision_reward, right_lane_reward, high_speed_reward, lane_change_reward;
  float on_road_reward;    /* config.get("on_road_reward", 0) */
  float reward_speed_range[2];
  int32_t normalize_reward; /* "normalize_reward" (True) */
  int32_t offroad_terminal; /* "offroad_terminal" (False) */
  /* fused observation wrapper */
  int32_t pe_kind;          /* enum hwy_pe_kind */
  int32_t d_embed;          /* rank / dist: appended width d; rope: rotate_dim */
  int32_t ego_idx;          /* wrapper ego_idx (0) */
  float pe_max_dist;        /* utils/defaults.py:max_dist() (100) */
  /* episode schedule: seed(env e, episode k) = seed_base + env_offset + e + 1 + seed_stride*k,
   * i.e. training/routine.py:127's exp_seed + episode_num for E = 1. */
  int32_t autoreset;        /* reset finished envs inside hwy_step */
  int32_t env_offset;       /* global index of this handle's env 0 (rank * E) */
  int64_t seed_base;
  int64_t seed_stride;      /* global env count */
} hwy_config;

typedef struct hwy_handle hwy_handle;

/* Per-env state: uint32 words laid out [HWY_NFIELDS][num_envs][HWY_MAX_VEHICLES] (field-major
 * SoA; one wavefront reads 256 contiguous bytes per field). Lane v of an env is vehicle v in
 * road.vehicles order (v = 0 is the ego). Float fields hold IEEE binary32 bits. */
enum hwy_field {
  HWY_F_X = 0, HWY_F_Y, HWY_F_HEADING, HWY_F_SPEED,
  HWY_F_TSPEED,  /* IDM target_speed */
  HWY_F_DELTA,   /* IDM DELTA exponent (randomize_behavior) */
  HWY_F_TIMER,   /* MOBIL lane-change timer */
  HWY_F_IMPX, HWY_F_IMPY, /* pending collision impact */
  HWY_F_LANE,    /* int: closest lane id */
  HWY_F_TLANE,   /* int: target lane id */
  HWY_F_FLAGS,   /* int: bit0 crashed, bit1 impact pending, bit2 present, bits 8-13 the
                    vehicle's position in the road order (x ascending, index descending) of the
                    stored positions -- a hint the step validates before use */
  HWY_F_ENV,     /* per-env words, see enum hwy_env_word */
  HWY_NFIELDS
};
enum hwy_env_word {
  HWY_E_STEP = 0,    /* policy steps taken this episode */
  HWY_E_EPISODE,     /* per-env episode counter k */
  HWY_E_SEED_LO, HWY_E_SEED_HI, /* seed of the current episode */
  HWY_E_EGO_ACC, HWY_E_EGO_STEER, /* float: ego action dict (persists across frames) */
  HWY_E_RETURN,      /* float: running episode return */
  HWY_E_NWORDS
};
#define HWY_FLAG_CRASHED 1u
#define HWY_FLAG_IMPACT 2u
#define HWY_FLAG_PRESENT 4u
#define HWY_FLAG_ORDER_SHIFT 8u
#define HWY_FLAG_ORDER_MASK (63u << HWY_FLAG_ORDER_SHIFT)

int hwy_abi_version(void);
/* sizeof(hwy_config) as compiled into the library (binding layout check). */
int hwy_config_size(void);
const char* hwy_last_error(void);

/* Validates cfg and allocates the device state for cfg->num_envs envs on `device`. */
int hwy_create(const hwy_config* cfg, int device, hwy_handle** out);
void hwy_destroy(hwy_handle* h);
/* Feature count per observation row after the fused wrapper (F or F + d). */
int hwy_obs_features(const hwy_handle* h);

/* Host table for the fused wrapper: rank -> tanh(W) [N*d]; dist -> freqs [d/2];
 * rope -> inv_freq [rotate_dim/2]; with experiment groups (hwy_set_seed_groups) also
 * n_groups RankPE tables [n_groups*N*d], one per group. Synchronous (setup time only). */
int hwy_set_pe_table(hwy_handle* h, const float* table_host, int n);

/* Change the episode seed schedule (seed_base, env_offset, seed_stride) of an existing handle:
 * training/routine.py re-seeds every episode from exp_seed (routine.py:127) and every evaluation
 * from exp_seed + 1000 (routine.py:18).  Takes effect for the next reset / autoreset. */
int hwy_set_seed_schedule(hwy_handle* h, int64_t seed_base, int32_t env_offset, int64_t seed_stride);

/* Experiment groups (a sweep's seeds batched into one handle; experiments/sweep.py): the E envs
 * form E / envs_per_group groups of consecutive envs, group g an experiment of its own with
 * seed(env g*envs_per_group + l, episode k) = seed_bases[g] + env_offset + l + 1 + seed_stride*k
 * (set seed_stride = envs_per_group for the solo schedule of each group: the same seeds, so each
 * group's envs step bit for bit as a solo handle of envs_per_group envs would).  seed_bases
 * (host, [E / envs_per_group]) is copied; n_groups = 0 turns grouping off.  With a fused RankPE,
 * hwy_set_pe_table may then take n_groups tables back to back (group g reads table g).
 * Synchronous (setup time only). */
int hwy_set_seed_groups(hwy_handle* h, const int64_t* seed_bases, int n_groups, int envs_per_group);

/* Reset envs whose mask byte is nonzero (mask NULL = all) with the given per-env seeds
 * (seeds NULL = the autoreset schedule with k = 0). Writes obs [E, N, F_out] for reset envs. */
int hwy_reset(hwy_handle* h, const uint64_t* seeds, const uint8_t* mask, float* obs, void* stream);

/* One policy step (sim_freq/policy_freq frames) for all E envs.
 *   actions [E,2] f32 in; obs [E,N,F_out], reward [E] f32, terminated/truncated [E] u8 out.
 *   ep_return / ep_length (nullable) receive the finished episode's return / length where
 *   terminated|truncated (0 elsewhere). With cfg.autoreset, finished envs are reset and obs
 *   holds the first observation of the next episode. */
int hwy_step(hwy_handle* h, const float* actions, float* obs, float* reward, uint8_t* terminated,
             uint8_t* truncated, float* ep_return, int32_t* ep_length, void* stream);

/* ---- Grouped step: n handles (the cells of a sweep batch, each one experiment group's handle;
 * ppo/group.py GroupBatch) stepped in ONE launch instead of n.  Workgroup (x, y) runs hwy_step's
 * workgroup x for handle y, reading that handle's launch parameters from a device table; each
 * env computes exactly what hwy_step on its own handle computes (the same kernel body).  Handles
 * may differ in env count, observation width and fused wrapper; one launch takes the register
 * budget of the handles' total env count.  hwy_step_group_prepare builds the table from the
 * handles as they are now and the per-handle buffers io[i] (hwy_step's arguments); it is
 * synchronous (waits for `stream`) and must be redone after any handle's configuration changes
 * (seed schedule, groups, PE table).  hwy_step_group is asynchronous and hipGraph-capturable. */
typedef struct hwy_step_io {
  const float* actions;
  float* obs;
  float* reward;
  uint8_t* terminated;
  uint8_t* truncated;
  float* ep_return;  /* nullable */
  int32_t* ep_length; /* nullable */
} hwy_step_io;
typedef struct hwy_step_group_plan {
  int32_t n, blocks, big; /* handles; workgroups per handle (the largest); register budget */
} hwy_step_group_plan;
int64_t hwy_step_group_table_bytes(int n);
int hwy_step_group_prepare(hwy_handle* const* handles, const hwy_step_io* io, int n, void* table,
                           hwy_step_group_plan* plan, void* stream);
int hwy_step_group(const hwy_step_group_plan* plan, const void* table, void* stream);

/* Copy the packed state [HWY_NFIELDS][E][HWY_MAX_VEHICLES] u32 to / from device memory. */
int hwy_export_state(hwy_handle* h, uint32_t* dst, void* stream);
int hwy_import_state(hwy_handle* h, const uint32_t* src, void* stream);

/* Stand-alone observation wrapper on [E,N,F] f32 -> [E,N,F_out] f32 (foreign envs).
 *   kind = enum hwy_pe_kind, d = appended width (rank/dist) or rotate_dim (rope),
 *   table = device pointer as for hwy_set_pe_table. dist_override (nullable, [E,N]) replaces
 *   the computed normalised distance (RotaryEmbedWrapper._apply_rope(obs, dist_norm)). */
int hwy_obs_pe(const float* obs_in, float* obs_out, int E, int N, int F, int kind, int d,
               int ego_idx, float max_dist, const float* table, const float* dist_override,
               void* stream);

/* GAE over a [T,E] rollout (ppo/agent.py:126-138): float64 arithmetic, float32 storage,
 * done = terminated|truncated treated as terminal (training/routine.py:135). */
int hwy_gae(const float* rewards, const uint8_t* dones, const float* values,
            const float* last_values, double gamma, double lam, int T, int E, float* advantages,
            float* returns, void* stream);

/* Device self-test of the deterministic math library (tests only): out[i] = op(in[i], in2[i]). */
int hwy_math_selftest(int op, const float* in, const float* in2, float* out, int n, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* HWY_H_ */
