// hwy_api.cpp -- the C ABI of libhwy.so (include/hwy.h): handle management, validation and
// launches.  No allocation, copy or synchronisation happens inside the compute entry points
// (hwy_reset / hwy_step / hwy_obs_pe / hwy_gae), so callers may capture them in a hipGraph.
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <cstring>

#include "hwy.h"
#include "hwy_internal.h"

struct hwy_handle {
  hwy_config cfg;
  int device;
  int fout;
  uint32_t* state;  // [HWY_NFIELDS][E][64]
  float* pe_table;  // [HWY_MAX_PE_TABLE]
  int64_t* group_seed;  // [n_groups] (hwy_set_seed_groups), or null
  int n_groups, group_envs, pe_group_stride;
};

static thread_local char g_err[512];

static int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

static int hip_fail(hipError_t e, const char* what) {
  return fail(HWY_EDEVICE, "%s: %s", what, hipGetErrorString(e));
}

static int pe_extra(const hwy_config* c) {
  return (c->pe_kind == HWY_PE_RANK || c->pe_kind == HWY_PE_DIST || c->pe_kind == HWY_PE_DIST1)
             ? c->d_embed
             : 0;
}

static int validate(const hwy_config* c) {
  if (!c) return fail(HWY_EINVAL, "config is NULL");
  if (c->num_envs < 1) return fail(HWY_EINVAL, "num_envs must be >= 1, got %d", c->num_envs);
  if (c->num_envs > (1 << 26) - 1)  // state words of one field indexed with 32 bits on device
    return fail(HWY_EINVAL, "num_envs must be < 2^26 per handle, got %d", c->num_envs);
  if (c->lanes_count < 1 || c->lanes_count > 64)
    return fail(HWY_EINVAL, "lanes_count must be in [1, 64], got %d", c->lanes_count);
  if (c->vehicles_count < 0 || c->vehicles_count + 1 > HWY_MAX_VEHICLES)
    return fail(HWY_EINVAL, "vehicles_count must be in [0, %d], got %d", HWY_MAX_VEHICLES - 1,
                c->vehicles_count);
  if (c->obs_vehicles < 1 || c->obs_vehicles > HWY_MAX_OBS_ROWS)
    return fail(HWY_EINVAL, "observation vehicles_count must be in [1, %d], got %d",
                HWY_MAX_OBS_ROWS, c->obs_vehicles);
  if (c->n_features < 1 || c->n_features > HWY_MAX_FEATURES)
    return fail(HWY_EINVAL, "feature count must be in [1, %d], got %d", HWY_MAX_FEATURES,
                c->n_features);
  for (int f = 0; f < c->n_features; ++f)
    if (c->feature_ids[f] < 0 || c->feature_ids[f] > HWY_FEAT_HEADING)
      return fail(HWY_EINVAL, "unsupported feature id %d", c->feature_ids[f]);
  if (c->order != HWY_ORDER_SORTED && c->order != HWY_ORDER_SHUFFLED)
    return fail(HWY_EINVAL, "order must be sorted or shuffled");
  if (c->sim_freq < 1 || c->policy_freq < 1 || c->sim_freq < c->policy_freq)
    return fail(HWY_EINVAL, "simulation_frequency (%d) must be >= policy_frequency (%d) >= 1",
                c->sim_freq, c->policy_freq);
  if (c->max_steps < 1) return fail(HWY_EINVAL, "max_steps must be >= 1");
  if (c->initial_lane_id >= c->lanes_count)
    return fail(HWY_EINVAL, "initial_lane_id %d out of range", c->initial_lane_id);
  if (!(c->vehicles_density > 0.0f)) return fail(HWY_EINVAL, "vehicles_density must be > 0");
  switch (c->pe_kind) {
    case HWY_PE_NONE: break;
    case HWY_PE_RANK:
      if (c->d_embed < 1) return fail(HWY_EINVAL, "d_embed must be >= 1 for RankPE");
      break;
    case HWY_PE_DIST:
      if (c->d_embed < 2 || c->d_embed % 2)
        return fail(HWY_EINVAL, "DistanceEmbedWrapper requires even d_embed; got %d", c->d_embed);
      if (c->n_features < 2) return fail(HWY_EINVAL, "DistPE needs at least 2 features");
      break;
    case HWY_PE_DIST1:
      if (c->d_embed < 2 || c->d_embed % 2)
        return fail(HWY_EINVAL, "DistanceEmbedWrapper requires even d_embed; got %d", c->d_embed);
      break;
    case HWY_PE_ROPE:
      if (c->d_embed % 2 || c->d_embed > c->n_features || c->d_embed < 0)
        return fail(HWY_EINVAL, "rotate_dim must be even and <= %d; got %d", c->n_features,
                    c->d_embed);
      if (c->n_features < 2) return fail(HWY_EINVAL, "RoPE needs at least 2 features");
      break;
    default: return fail(HWY_EINVAL, "unknown pe_kind %d", c->pe_kind);
  }
  if (c->n_features + pe_extra(c) > HWY_MAX_FOUT)
    return fail(HWY_EINVAL, "F + d_embed exceeds %d", HWY_MAX_FOUT);
  if (c->ego_idx < 0 || c->ego_idx >= c->obs_vehicles)
    return fail(HWY_EINVAL, "ego_idx %d out of range", c->ego_idx);
  if (!(c->pe_max_dist > 0.0f)) return fail(HWY_EINVAL, "max_dist must be > 0");
  return HWY_OK;
}

extern "C" {

int hwy_abi_version(void) { return HWY_ABI_VERSION; }

int hwy_config_size(void) { return (int)sizeof(hwy_config); }

const char* hwy_last_error(void) { return g_err; }

int hwy_create(const hwy_config* cfg, int device, hwy_handle** out) {
  if (!out) return fail(HWY_EINVAL, "out is NULL");
  *out = nullptr;
  int rc = validate(cfg);
  if (rc) return rc;
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
  hwy_handle* h = new hwy_handle();
  h->cfg = *cfg;
  h->device = device;
  h->fout = cfg->n_features + pe_extra(cfg);
  size_t words = (size_t)HWY_NFIELDS * (size_t)cfg->num_envs * HWY_MAX_VEHICLES;
  e = hipMalloc(&h->state, words * sizeof(uint32_t));
  if (e != hipSuccess) {
    delete h;
    return hip_fail(e, "hipMalloc(state)");
  }
  e = hipMalloc(&h->pe_table, HWY_MAX_PE_TABLE * sizeof(float));
  if (e != hipSuccess) {
    (void)hipFree(h->state);
    delete h;
    return hip_fail(e, "hipMalloc(pe_table)");
  }
  (void)hipMemset(h->state, 0, words * sizeof(uint32_t));
  (void)hipMemset(h->pe_table, 0, HWY_MAX_PE_TABLE * sizeof(float));
  e = hipDeviceSynchronize();
  if (e != hipSuccess) {
    (void)hipFree(h->state);
    (void)hipFree(h->pe_table);
    delete h;
    return hip_fail(e, "hipMemset");
  }
  *out = h;
  return HWY_OK;
}

void hwy_destroy(hwy_handle* h) {
  if (!h) return;
  (void)hipSetDevice(h->device);
  (void)hipDeviceSynchronize();
  (void)hipFree(h->state);
  (void)hipFree(h->pe_table);
  if (h->group_seed) (void)hipFree(h->group_seed);
  delete h;
}

int hwy_obs_features(const hwy_handle* h) { return h ? h->fout : HWY_EINVAL; }

int hwy_set_pe_table(hwy_handle* h, const float* table_host, int n) {
  if (!h) return fail(HWY_EINVAL, "handle is NULL");
  const hwy_config& c = h->cfg;
  int need = 0;
  if (c.pe_kind == HWY_PE_RANK) need = c.obs_vehicles * c.d_embed;
  if (c.pe_kind == HWY_PE_DIST || c.pe_kind == HWY_PE_DIST1) need = c.d_embed / 2;
  if (c.pe_kind == HWY_PE_ROPE) need = c.d_embed / 2;
  int stride = 0;
  if (c.pe_kind == HWY_PE_RANK && h->n_groups > 0 && n == need * h->n_groups && n != need) {
    stride = need;  // one RankPE table per experiment group
    need = n;
  }
  if (n != need) return fail(HWY_EINVAL, "pe table needs %d floats, got %d", need, n);
  if (n > HWY_MAX_PE_TABLE) return fail(HWY_EINVAL, "pe table too large (%d)", n);
  if (n == 0) return HWY_OK;
  (void)hipSetDevice(h->device);
  hipError_t e = hipMemcpy(h->pe_table, table_host, (size_t)n * sizeof(float), hipMemcpyHostToDevice);
  if (e != hipSuccess) return hip_fail(e, "hipMemcpy(pe_table)");
  h->pe_group_stride = stride;
  return HWY_OK;
}

int hwy_set_seed_groups(hwy_handle* h, const int64_t* seed_bases, int n_groups, int envs_per_group) {
  if (!h) return fail(HWY_EINVAL, "handle is NULL");
  (void)hipSetDevice(h->device);
  if (n_groups == 0) {
    if (h->group_seed) (void)hipFree(h->group_seed);
    h->group_seed = nullptr;
    h->n_groups = h->group_envs = h->pe_group_stride = 0;
    return HWY_OK;
  }
  if (!seed_bases || n_groups < 0 || envs_per_group < 1 ||
      (int64_t)n_groups * envs_per_group != h->cfg.num_envs)
    return fail(HWY_EINVAL, "seed groups: %d groups x %d envs must cover num_envs %d", n_groups,
                envs_per_group, h->cfg.num_envs);
  int64_t* dev = nullptr;
  hipError_t e = hipMalloc(&dev, (size_t)n_groups * sizeof(int64_t));
  if (e != hipSuccess) return hip_fail(e, "hipMalloc(group_seed)");
  e = hipMemcpy(dev, seed_bases, (size_t)n_groups * sizeof(int64_t), hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    (void)hipFree(dev);
    return hip_fail(e, "hipMemcpy(group_seed)");
  }
  if (h->group_seed) (void)hipFree(h->group_seed);
  h->group_seed = dev;
  h->n_groups = n_groups;
  h->group_envs = envs_per_group;
  h->pe_group_stride = 0;  // a grouped RankPE table is set after the groups
  return HWY_OK;
}

int hwy_set_seed_schedule(hwy_handle* h, int64_t seed_base, int32_t env_offset, int64_t seed_stride) {
  if (!h) return fail(HWY_EINVAL, "handle is NULL");
  if (seed_stride < 0) return fail(HWY_EINVAL, "seed_stride must be >= 0");
  h->cfg.seed_base = seed_base;
  h->cfg.env_offset = env_offset;
  h->cfg.seed_stride = seed_stride;
  return HWY_OK;
}

static StepParams params_of(hwy_handle* h) {
  StepParams p;
  memset(&p, 0, sizeof(p));
  p.cfg = h->cfg;
  p.state = h->state;
  p.pe_table = h->pe_table;
  p.fout = h->fout;
  p.group_seed = h->group_seed;
  p.group_envs = h->group_envs;
  p.pe_group_stride = h->pe_group_stride;
  return p;
}

int hwy_reset(hwy_handle* h, const uint64_t* seeds, const uint8_t* mask, float* obs, void* stream) {
  if (!h) return fail(HWY_EINVAL, "handle is NULL");
  StepParams p = params_of(h);
  p.seeds = seeds;
  p.mask = mask;
  p.obs = obs;
  if (hwy_launch_reset(&p, (hipStream_t)stream)) return hip_fail(hipGetLastError(), "hwy_reset_kernel");
  return HWY_OK;
}

int hwy_step(hwy_handle* h, const float* actions, float* obs, float* reward, uint8_t* terminated,
             uint8_t* truncated, float* ep_return, int32_t* ep_length, void* stream) {
  if (!h) return fail(HWY_EINVAL, "handle is NULL");
  if (!actions || !obs || !reward || !terminated || !truncated)
    return fail(HWY_EINVAL, "hwy_step: actions/obs/reward/terminated/truncated must be non-NULL");
  StepParams p = params_of(h);
  p.actions = actions;
  p.obs = obs;
  p.reward = reward;
  p.term = terminated;
  p.trunc = truncated;
  p.ep_ret = ep_return;
  p.ep_len = ep_length;
  if (hwy_launch_step(&p, (hipStream_t)stream)) return hip_fail(hipGetLastError(), "hwy_step_kernel");
  return HWY_OK;
}

int64_t hwy_step_group_table_bytes(int n) {
  return n < 1 ? -1 : (int64_t)n * (int64_t)sizeof(StepParams);
}

int hwy_step_group_prepare(hwy_handle* const* handles, const hwy_step_io* io, int n, void* table,
                           hwy_step_group_plan* plan, void* stream) {
  if (!handles || !io || n < 1 || !table || !plan)
    return fail(HWY_EINVAL, "hwy_step_group_prepare: handles/io/table/plan NULL or n < 1");
  StepParams* tab = new StepParams[n];
  int blocks = 0, dev = -1;
  int64_t total = 0;
  for (int i = 0; i < n; ++i) {
    hwy_handle* h = handles[i];
    const hwy_step_io& a = io[i];
    if (!h || !a.actions || !a.obs || !a.reward || !a.terminated || !a.truncated) {
      delete[] tab;
      return fail(HWY_EINVAL, "hwy_step_group_prepare: handle %d or its actions/obs/reward/"
                              "terminated/truncated is NULL", i);
    }
    if (dev >= 0 && h->device != dev) {
      delete[] tab;
      return fail(HWY_EINVAL, "hwy_step_group_prepare: handles on devices %d and %d", dev,
                  h->device);
    }
    dev = h->device;
    StepParams p = params_of(h);
    p.actions = a.actions;
    p.obs = a.obs;
    p.reward = a.reward;
    p.term = a.terminated;
    p.trunc = a.truncated;
    p.ep_ret = a.ep_return;
    p.ep_len = a.ep_length;
    tab[i] = p;
    const int b = hwy_step_blocks(h->cfg.num_envs);
    blocks = b > blocks ? b : blocks;
    total += h->cfg.num_envs;
  }
  hipStream_t s = (hipStream_t)stream;
  hipError_t e = hipStreamSynchronize(s);
  if (e == hipSuccess)
    e = hipMemcpyAsync(table, tab, (size_t)n * sizeof(StepParams), hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  delete[] tab;
  if (e != hipSuccess) return hip_fail(e, "hwy_step_group_prepare");
  plan->n = n;
  plan->blocks = blocks;
  plan->big = hwy_step_big(total);
  return HWY_OK;
}

int hwy_step_group(const hwy_step_group_plan* plan, const void* table, void* stream) {
  if (!plan || !table || plan->n < 1 || plan->blocks < 1)
    return fail(HWY_EINVAL, "hwy_step_group: empty plan or NULL table");
  if (hwy_launch_step_group((const StepParams*)table, plan->n, plan->blocks, plan->big,
                            (hipStream_t)stream))
    return hip_fail(hipGetLastError(), "hwy_step_grp_kernel");
  return HWY_OK;
}

int hwy_export_state(hwy_handle* h, uint32_t* dst, void* stream) {
  if (!h || !dst) return fail(HWY_EINVAL, "handle/dst is NULL");
  size_t bytes = (size_t)HWY_NFIELDS * h->cfg.num_envs * HWY_MAX_VEHICLES * sizeof(uint32_t);
  hipError_t e = hipMemcpyAsync(dst, h->state, bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream);
  return e == hipSuccess ? HWY_OK : hip_fail(e, "hwy_export_state");
}

int hwy_import_state(hwy_handle* h, const uint32_t* src, void* stream) {
  if (!h || !src) return fail(HWY_EINVAL, "handle/src is NULL");
  size_t bytes = (size_t)HWY_NFIELDS * h->cfg.num_envs * HWY_MAX_VEHICLES * sizeof(uint32_t);
  hipError_t e = hipMemcpyAsync(h->state, src, bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream);
  return e == hipSuccess ? HWY_OK : hip_fail(e, "hwy_import_state");
}

int hwy_obs_pe(const float* obs_in, float* obs_out, int E, int N, int F, int kind, int d,
               int ego_idx, float max_dist, const float* table, const float* dist_override,
               void* stream) {
  if (E < 0 || N < 1 || F < 1 || F > HWY_MAX_FEATURES)
    return fail(HWY_EINVAL, "hwy_obs_pe: bad shape E=%d N=%d F=%d", E, N, F);
  if (kind == HWY_PE_ROPE && (d % 2 || d > F || d < 0))
    return fail(HWY_EINVAL, "rotate_dim must be even and <= %d; got %d", F, d);
  if ((kind == HWY_PE_DIST || kind == HWY_PE_DIST1) && (d % 2 || d < 2))
    return fail(HWY_EINVAL, "DistanceEmbedWrapper requires even d_embed; got %d", d);
  if ((kind == HWY_PE_DIST || kind == HWY_PE_ROPE) && F < 2)
    return fail(HWY_EINVAL, "distance wrappers need at least 2 features");
  if (kind < HWY_PE_NONE || kind > HWY_PE_DIST1) return fail(HWY_EINVAL, "unknown pe kind %d", kind);
  if (ego_idx < 0 || ego_idx >= N) return fail(HWY_EINVAL, "ego_idx %d out of range", ego_idx);
  if (kind != HWY_PE_NONE && !table && !(kind == HWY_PE_ROPE && d == 0))
    return fail(HWY_EINVAL, "pe table is NULL");
  if (hwy_launch_obs_pe(obs_in, obs_out, E, N, F, kind, d, ego_idx, max_dist, table, dist_override,
                        (hipStream_t)stream))
    return hip_fail(hipGetLastError(), "hwy_obs_pe_kernel");
  return HWY_OK;
}

int hwy_gae(const float* rewards, const uint8_t* dones, const float* values,
            const float* last_values, double gamma, double lam, int T, int E, float* advantages,
            float* returns, void* stream) {
  if (T < 0 || E < 0) return fail(HWY_EINVAL, "hwy_gae: bad shape T=%d E=%d", T, E);
  if (T == 0 || E == 0) return HWY_OK;
  if (hwy_launch_gae(rewards, dones, values, last_values, gamma, lam, T, E, advantages, returns,
                     (hipStream_t)stream))
    return hip_fail(hipGetLastError(), "hwy_gae_kernel");
  return HWY_OK;
}

int hwy_math_selftest(int op, const float* in, const float* in2, float* out, int n, void* stream) {
  if (op < 0 || op > 16 || n < 0) return fail(HWY_EINVAL, "bad selftest op %d", op);
  if (hwy_launch_math(op, in, in2, out, n, (hipStream_t)stream))
    return hip_fail(hipGetLastError(), "hwy_math_kernel");
  return HWY_OK;
}

}  // extern "C"
