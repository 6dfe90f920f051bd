/*
 * hwy_ppo.h -- C ABI of the fused PPO minibatch step (libhwy.so).
 *
 * Replaces, for the batched path, the per-minibatch body of PPOAgent.update
 * (reference ppo/agent.py:216-252): ActorCritic.evaluate (:76-84) on the minibatch, the
 * ratio / KL / clipped surrogate / MSE / entropy loss (:226-245), loss.backward(),
 * clip_grad_norm_(0.5) (:249-251) and Adam.step() (:252, torch.optim.Adam defaults).
 *
 * Network (ppo/agent.py:23-42): shared = Lin(S,H)-ReLU-Lin(H,H)-ReLU; actor_mean =
 * Lin(H,H)-ReLU-Lin(H,A); log_std[A]; critic = Lin(H,H)-ReLU-Lin(H,1).  Parameters live in
 * one flat fp32 buffer in nn.Module.parameters() order:
 *   shared.0.{weight,bias} shared.2.{weight,bias} actor_mean.0.{weight,bias}
 *   actor_mean.2.{weight,bias} log_std critic.0.{weight,bias} critic.2.{weight,bias}
 * (weights [out, in] row-major, as nn.Linear stores them).
 *
 * All math is fp32; GEMMs use v_mfma_f32_16x16x4_f32 / v_mfma_f32_32x32x2_f32 (exact fp32
 * products, fp32 accumulate).
 * Calls are asynchronous, allocate nothing and are hipGraph-capturable.
 *
 * Weight tile image: on the fused path (S % 4 == 0, S <= 256, H <= 512) the row kernel streams
 * the weights from a tiled copy kept in the workspace.  hwy_ppo_optimizer rewrites it with every
 * Adam step; call hwy_ppo_sync_params once before the first hwy_ppo_forward_backward on a
 * workspace, and again whenever params were written by anything other than hwy_ppo_optimizer
 * (a checkpoint load, a torch optimizer step, a broadcast).
 */
#ifndef HWY_PPO_H_
#define HWY_PPO_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct hwy_ppo_dims {
  int32_t B; /* minibatch rows */
  int32_t S; /* state_dim */
  int32_t H; /* hidden_dim (multiple of 64) */
  int32_t A; /* action_dim (2) */
} hwy_ppo_dims;

/* Flat-parameter offsets (floats) for dims; numel returned. */
int hwy_ppo_param_layout(const hwy_ppo_dims* d, int64_t* offsets /*[13]*/, int64_t* numel);
/* Workspace bytes needed by hwy_ppo_forward_backward / hwy_ppo_optimizer for dims. */
int64_t hwy_ppo_workspace_bytes(const hwy_ppo_dims* d);

typedef struct hwy_ppo_args {
  hwy_ppo_dims dims;
  /* rollout sources (flattened [n, ...]) and this minibatch's row indices [B] (int64) */
  const float* states;    /* [n, S] */
  const float* pre_tanh;  /* [n, A] */
  const float* old_logp;  /* [n] */
  const float* adv;       /* [n] normalised advantages */
  const float* ret;       /* [n] returns */
  const int64_t* idx;     /* [B] */
  /* model / optimizer state (flat, hwy_ppo_param_layout order) */
  float* params;
  float* grads;
  float* adam_m;
  float* adam_v;
  int32_t* counters;      /* [0] Adam step t, [1] metrics row */
  float* metrics;         /* [rows, 6]: policy, value, entropy, loss, clip count, kl */
  void* workspace;        /* hwy_ppo_workspace_bytes(dims) bytes, owned by these calls */
  /* hyper-parameters (PPOAgent defaults: eps_clip .2, value_coef .5, entropy_coef .005) */
  float eps_clip, value_coef, entropy_coef, max_grad_norm;
  float lr, beta1, beta2, adam_eps;
  int32_t grads_modified; /* grads changed after forward_backward (e.g. all-reduced): the
                             optimizer recomputes the gradient norm from them */
} hwy_ppo_args;

/* Forward, loss, backward: writes grads (flat) and the metrics row. */
int hwy_ppo_forward_backward(const hwy_ppo_args* a, void* stream);
/* clip_grad_norm_(max_grad_norm) + Adam step on params (call after any gradient all-reduce). */
int hwy_ppo_optimizer(const hwy_ppo_args* a, void* stream);
/* Measurement aid (bench.py's per-kernel roofline): each kernel of the minibatch step
 * (ppo_rows, ppo_wgrad, ppo_wsum, ppo_adam) captured as a HIP graph of `reps` back-to-back
 * launches on a private stream and replayed between two events; writes the average microseconds
 * per launch to us[0..3], and to us[4] the same for an empty one-workgroup kernel (the launch
 * floor a kernel-trace duration leaves out).  The Adam launches update params / moments / the tile image as training
 * steps do; the Adam step count is restored and the metrics row index left at 0.  Waits for
 * `stream` first; synchronous, not graph-capturable; fused path, grads_modified == 0.
 * -1 bad args, -2 HIP error. */
int hwy_ppo_time_kernels(const hwy_ppo_args* a, void* stream, int reps, float* us);
/* Rebuild the workspace's weight tile image from params (uses dims, params, workspace). */
int hwy_ppo_sync_params(const hwy_ppo_args* a, void* stream);

/* Byte offset of the weight tile image inside a workspace for dims (-1 when the dims take
 * the general path, which keeps none).  The image depends on S and H only. */
int64_t hwy_ppo_tile_image_offset(const hwy_ppo_dims* d);

/* ActorCritic.act on a batch (replaces ppo/agent.py:86-95's forward + Normal sample + tanh +
 * squashed log-prob on the batched rollout path): dims.B rows of states [B][S] (contiguous);
 * noise [B][2] standard-normal draws (the caller's generator, as act() draws them) or NULL for
 * act(deterministic=True) (z = mean, log_prob = 0).  Needs S % 4 == 0, S <= 256,
 * H in {64, 128, ..., 512}.  tiles: NULL, or the tile image of a hwy_ppo workspace with the same
 * S and H that is in step with params (workspace + hwy_ppo_tile_image_offset; current after
 * hwy_ppo_optimizer / hwy_ppo_sync_params until params are written by anything else): the
 * forward then streams whole 1-KB operand tiles instead of 64-B pieces of params rows. */
typedef struct hwy_ppo_act_args {
  hwy_ppo_dims dims;
  const float* states;
  const float* params; /* flat, hwy_ppo_param_layout order */
  const float* noise;
  float* action;   /* [B][2] tanh(z) */
  float* pre_tanh; /* [B][2] z */
  float* logp;     /* [B] */
  float* value;    /* [B] */
  const float* tiles; /* optional weight tile image (see above), or NULL */
} hwy_ppo_act_args;
int hwy_ppo_act(const hwy_ppo_act_args* a, void* stream);

/* ---- Grouped learners: G independent learners (a sweep cell's seeds, or the cells of one
 * hidden width; ppo/group.py, ExperimentRunner.launch_group; the reference runs them as separate processes,
 * experiments/runner.py:46-155 under main.py:188-242's joblib / SLURM fan-out) stepped in ONE
 * launch per kernel.  Workgroup (x, y) runs the solo launch's workgroup x for learner y, whose
 * kernel arguments the kernels read from a device table; the kernel bodies and tile shapes are
 * the solo calls', so each learner's results are bit for bit its solo run's.  The *_prepare
 * calls build a table from G argument structs (synchronous: they wait for `stream`; not
 * capturable); the launch calls are asynchronous and hipGraph-capturable.
 *
 * hwy_ppo_group_step = hwy_ppo_forward_backward + hwy_ppo_optimizer for every learner (fused
 * path with 16-row tiles, i.e. minibatches below 64 x CUs rows; grads_modified == 0; 16-byte
 * aligned flat buffers).  The learners share B and H; their state dims S may differ (e.g. the
 * h256 cells of a sweep: no PE S = N*F, RankPE / DistPE S = N*(F+d)): each launch covers the
 * largest learner's grid (the plan prepare writes) and a learner's surplus workgroups exit.
 * hwy_ppo_group_table_bytes depends on B, H and G only.  -1 bad arguments / unsupported dims,
 * -2 HIP error. */
typedef struct hwy_ppo_group_plan {
  int32_t G, B, H;                                    /* learners; shared minibatch rows, hidden */
  int32_t grid_rows, grid_wgrad, grid_wsum, grid_adam; /* each launch's grid: the largest learner's */
} hwy_ppo_group_plan;
int64_t hwy_ppo_group_table_bytes(const hwy_ppo_dims* d, int G);
int hwy_ppo_group_prepare(const hwy_ppo_args* a /*[G]*/, int G, void* table,
                          hwy_ppo_group_plan* plan, void* stream);
int hwy_ppo_group_step(const hwy_ppo_group_plan* plan, const void* table, void* stream);
/* hwy_ppo_act for G learners (same B and H; S may differ); `tiles` = whether the learners' args
 * carry tile images (all or none), which picks the solo call's kernel. */
int64_t hwy_ppo_group_act_table_bytes(int G);
int hwy_ppo_group_act_prepare(const hwy_ppo_act_args* a /*[G]*/, int G, void* table, void* stream);
int hwy_ppo_group_act(const hwy_ppo_dims* d, int G, int tiles, const void* table, void* stream);

/* Build flags of this library: bit 0 = development knobs compiled in (HWY_DEV_KNOBS: the
 * HWY_WG_BAL / HWY_ROWS_RT / HWY_WG_FILL environment variables are read), bit 1 = section clocks
 * (HWY_SECTION_PROFILE).  A product build returns 0 and reads no environment variable. */
int hwy_ppo_build_flags(void);

#ifdef __cplusplus
}
#endif
#endif /* HWY_PPO_H_ */
