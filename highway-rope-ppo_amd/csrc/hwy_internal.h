// hwy_internal.h -- launch parameters shared by hwy_api.cpp (host) and hwy_kernels.hip.
#ifndef HWY_INTERNAL_H_
#define HWY_INTERNAL_H_
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hwy.h"

struct StepParams {
  hwy_config cfg;
  uint32_t* state;
  const float* actions;
  float* obs;
  float* reward;
  uint8_t* term;
  uint8_t* trunc;
  float* ep_ret;
  int32_t* ep_len;
  const float* pe_table;
  const uint64_t* seeds;
  const uint8_t* mask;
  int fout;
  // experiment groups (hwy_set_seed_groups): per-group seed bases, envs per group, and the
  // floats between consecutive groups' PE tables (0: one table for all)
  const int64_t* group_seed;
  int group_envs;
  int pe_group_stride;
};

extern "C" {
int hwy_launch_step(const StepParams* p, hipStream_t s);
// n handles' steps in one launch: dtab = n StepParams in device memory, blocks = the largest
// handle's hwy_step_blocks, big = hwy_step_big(total envs) (the register budget of the launch)
int hwy_launch_step_group(const StepParams* dtab, int n, int blocks, int big, hipStream_t s);
int hwy_step_blocks(int num_envs);
int hwy_step_big(int64_t total_envs);
int hwy_launch_reset(const StepParams* p, hipStream_t s);
int hwy_launch_obs_pe(const float* in, float* out, int E, int N, int F, int kind, int d, int ego,
                      float max_dist, const float* table, const float* dov, hipStream_t s);
int hwy_launch_gae(const float* rew, const uint8_t* done, const float* val, const float* last_val,
                   double gamma, double lam, int T, int E, float* adv, float* ret, hipStream_t s);
int hwy_launch_math(int op, const float* in, const float* in2, float* out, int n, hipStream_t s);
}
#endif
