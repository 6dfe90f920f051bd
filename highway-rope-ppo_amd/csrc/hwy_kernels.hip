// hwy_kernels.hip -- gfx950 kernels of the vectorised highway-v0 hot path.
//
// Layout: one 64-lane wavefront per env, lane v = vehicle v of road.vehicles (v = 0 ego,
// 1..vehicles_count IDM traffic).  A 256-thread workgroup advances 4 envs.  The per-env state is
// field-major SoA in HBM ([field][env][64] u32, include/hwy.h) so each wave loads 256
// contiguous bytes per field once, runs all sim_freq/policy_freq frames in registers, and
// stores once.  Cross-vehicle reads use v_readlane (uniform index, SGPR broadcast) or
// ds_bpermute (per-lane index); nothing else touches LDS except the observation row maps.
//
// Semantics follow upstream highway-env 1.10.1 as restated in oracle/hwy_oracle.c, which runs
// every vehicle sequentially; the parallel formulation below is arranged to give the same bits:
//   * Road.act order dependence: MOBIL decisions do not read other vehicles' target lanes, so
//     they run in parallel; the "abort ongoing lane change" check (which does) runs afterwards
//     over the mid-change vehicles in ascending index, each seeing the already-final targets of
//     lower-index vehicles and the frame-start targets of higher-index ones.
//   * Road.step collisions: lane k evaluates every pair {k, j} (always as a = lower index, so
//     both lanes of a pair compute identical bits) in ascending j, which is exactly the order
//     in which upstream's i<j double loop last writes k's impact.
// All floating point goes through hwy_math.h and is compiled with -ffp-contract=off.
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "hwy.h"
#include "hwy_math.h"
#include "hwy_internal.h"

#define WAVE 64
// envs (one wave each) per workgroup: 1, 2 and 4 measured the same (round 4)
constexpr int ENVS_PER_BLOCK = 4;

// upstream constants (same literals as oracle/hwy_oracle.c)
#define LANE_WIDTH 4.0f
#define LANE_VEH_LEN 5.0f
#define ROAD_LENGTH 10000.0f
#define VEH_LENGTH 5.0f
#define VEH_WIDTH 2.0f
#define MAX_SPEED 40.0f
#define MIN_SPEED (-40.0f)
#define KP_HEADING (1.0f / 0.2f)
#define KP_LATERAL (1.0f / 0.6f)
#define MAX_STEERING (HM_PI_F / 3.0f)
#define TAN_MAX_STEERING 1.7320509f  // tan(MAX_STEERING), correctly rounded
#define ACC_MAX 6.0f
#define COMFORT_ACC_MAX 3.0f
#define DISTANCE_WANTED 10.0f
#define TIME_WANTED 1.5f
#define LANE_CHANGE_MIN_ACC_GAIN 0.2f
#define LANE_CHANGE_MAX_BRAKING_IMPOSED 2.0f
#define LANE_CHANGE_DELAY 1.0f
#define PERCEPTION_DISTANCE 200.0f
#define TWO_SQRT_AB 7.745966692414834f
#define INV_TWO_SQRT_AB 0.12909944487358056f  // 1 / (2 sqrt(15)), correctly rounded
#define VEH_DIAGONAL 5.385164807134504f

// ------------------------------------------------------------------------- wave primitives
__device__ __forceinline__ float rdlf(float v, int k) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), k));
}
__device__ __forceinline__ int rdli(int v, int k) { return __builtin_amdgcn_readlane(v, k); }
// per-lane gather; must run with all 64 lanes active
__device__ __forceinline__ float shf(float v, int src) {
  return __int_as_float(__builtin_amdgcn_ds_bpermute(src << 2, __float_as_int(v)));
}
__device__ __forceinline__ int shi(int v, int src) { return __builtin_amdgcn_ds_bpermute(src << 2, v); }
// DPP forms (VALU-local, no LDS round trip); all 64 lanes active.  GFX9 DPP controls:
// wave_shr:1 0x138, row_shr:k 0x110+k, row_bcast:15 0x142, row_bcast:31 0x143,
// quad_perm 0x00-0xFF, row_mirror 0x140, row_half_mirror 0x141.
// lane i <- lane i-1; lane 0 keeps its own value
__device__ __forceinline__ float shr1f(float v) {
  const int b = __float_as_int(v);
  return __int_as_float(__builtin_amdgcn_update_dpp(b, b, 0x138, 0xf, 0xf, false));
}
// lane i <- lane i+1; lane 63 keeps its own value
__device__ __forceinline__ int shl1i(int v) {
  return __builtin_amdgcn_update_dpp(v, v, 0x130, 0xf, 0xf, false);
}
__device__ __forceinline__ int shr1i(int v) {
  return __builtin_amdgcn_update_dpp(v, v, 0x138, 0xf, 0xf, false);
}
// lane i <- lane i^1
__device__ __forceinline__ int swp1i(int v) {
  return __builtin_amdgcn_update_dpp(v, v, 0xb1, 0xf, 0xf, false);
}
// inclusive prefix sum over the 64 lanes
__device__ __forceinline__ int wave_incl_scan(int x) {
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, true);
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, true);
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, true);
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, true);
  x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);
  x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);
  return x;
}
// max over the 64 lanes (exact: no NaN reaches it), uniform result
__device__ __forceinline__ float wave_max_f(float v) {
  int b = __float_as_int(v);
  b = __float_as_int(hm_maxf(__int_as_float(b), __int_as_float(
      __builtin_amdgcn_update_dpp(b, b, 0xb1, 0xf, 0xf, false))));
  b = __float_as_int(hm_maxf(__int_as_float(b), __int_as_float(
      __builtin_amdgcn_update_dpp(b, b, 0x4e, 0xf, 0xf, false))));
  b = __float_as_int(hm_maxf(__int_as_float(b), __int_as_float(
      __builtin_amdgcn_update_dpp(b, b, 0x141, 0xf, 0xf, false))));
  b = __float_as_int(hm_maxf(__int_as_float(b), __int_as_float(
      __builtin_amdgcn_update_dpp(b, b, 0x140, 0xf, 0xf, false))));
  b = __float_as_int(hm_maxf(__int_as_float(b), __int_as_float(
      __builtin_amdgcn_update_dpp(b, b, 0x142, 0xa, 0xf, false))));
  b = __float_as_int(hm_maxf(__int_as_float(b), __int_as_float(
      __builtin_amdgcn_update_dpp(b, b, 0x143, 0xc, 0xf, false))));
  return __int_as_float(__builtin_amdgcn_readlane(b, 63));
}
// the lane mask of p straight from the compare (HIP's __ballot(int) re-materialises p as an
// int and compares it again: two VALU per ballot)
__device__ __forceinline__ uint64_t ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }
__device__ __forceinline__ bool wave_any(bool p) { return ballot(p) != 0ull; }
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ------------------------------------------------------------------------- section clocks
// Development build only (make prof -> libhwy_prof.so): per-section shader-clock totals of the
// step kernel, accumulated per env (plain loads and stores by the env's own wave: one device
// atomic per section and wave on shared counters serialised the launch's tail and inflated the
// last sections several-fold) and summed over envs by hwy_debug_sections().
#define HWY_NSEC 18
#define HWY_NSEC_ENVS 32768  // the largest profiled workload (configs[4]: 32,768 envs per GPU)
#ifdef HWY_SECTION_PROFILE
__device__ unsigned long long g_hwy_sections[HWY_NSEC_ENVS][HWY_NSEC];
struct SecProf {
  uint64_t t;
  uint64_t acc[HWY_NSEC];
};
#define SEC_START(sp)                                      \
  do {                                                     \
    (sp).t = __builtin_amdgcn_s_memtime();                 \
    for (int _i = 0; _i < HWY_NSEC; ++_i) (sp).acc[_i] = 0; \
  } while (0)
#define SEC(sp, id)                                      \
  do {                                                   \
    const uint64_t _n = __builtin_amdgcn_s_memtime();    \
    (sp).acc[id] += _n - (sp).t;                         \
    (sp).t = _n;                                         \
  } while (0)
#define SEC_FLUSH(sp, lane, e)                                                \
  do {                                                                        \
    if ((lane) == 0) /* envs past the cap fold onto env mod cap: none is dropped */ \
      for (int _i = 0; _i < HWY_NSEC; ++_i)                                   \
        g_hwy_sections[(e) % HWY_NSEC_ENVS][_i] += (sp).acc[_i];             \
  } while (0)
#else
struct SecProf {};
#define SEC_START(sp) \
  do {                \
  } while (0)
#define SEC(sp, id) \
  do {              \
  } while (0)
#define SEC_FLUSH(sp, lane, e) \
  do {                         \
  } while (0)
#endif
// Development builds (make prof / make waves -> libhwy_waves.so, tools/probe_waves.py):
#if defined(HWY_SECTION_PROFILE) || defined(HWY_WAVE_TIMES)
// per-env (start, end, done | HW_ID << 8 | XCC_ID << 40) of the last step launch, first
// HWY_NWT envs
#define HWY_NWT 16384
__device__ unsigned long long g_hwy_wave_t[5 * HWY_NWT];
#define WAVE_T(e, lane, k, val)                                          \
  do {                                                                   \
    if ((lane) == 0 && (e) < HWY_NWT) g_hwy_wave_t[5 * (e) + (k)] = (val); \
  } while (0)
#define WAVE_HWID()                                                                  \
  (((unsigned long long)(uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 4) << 8) |  \
   ((unsigned long long)(__builtin_amdgcn_s_getreg((31 << 11) | 20) & 0xff) << 40))
#else
#define WAVE_T(e, lane, k, val) \
  do {                          \
  } while (0)
#define WAVE_HWID() 0ull
#endif

// Development pricing builds only (hwy_dev_knobs.h, a make variant with -DHWY_DEV_KNOBS and the
// mask; WRONG results, never the product): kSkip skips parts of the frame to price their
// instruction count.  The product build compiles every such site away (kSkip = 0).
#ifdef HWY_DEV_KNOBS
#include "hwy_dev_knobs.h"
#else
constexpr int kSkip = 0;
#endif

// ------------------------------------------------------------------------- vehicle state
struct Veh {
  float x, y, h, spd, tsp, dlt, tmr, ix, iy;
  // Vehicle.action.  asteer: lane 0 the ego's steering angle (persists across frames); the
  // traffic lanes hold the TANGENT of their clipped steering angle (what kinematics uses)
  float aacc, asteer;
  int ln, tl;
  bool crashed, imp, present;
};

__device__ __forceinline__ float lane_lat(float y, int c) { return y - (float)c * LANE_WIDTH; }

__device__ __forceinline__ bool on_lane_m(float x, float y, int c, float margin) {
  float lat = lane_lat(y, c);
  return hm_absf(lat) <= LANE_WIDTH / 2.0f + margin && -LANE_VEH_LEN <= x &&
         x < ROAD_LENGTH + LANE_VEH_LEN;
}

// the loop form: the first lane of least |lateral offset| (upstream's argmin over the lanes)
__device__ __forceinline__ int closest_lane_scan(float y, int lanes) {
  int best = 0;
  float bd = hm_absf(lane_lat(y, 0));
  for (int c = 1; c < lanes; ++c) {
    float d = hm_absf(lane_lat(y, c));
    if (d < bd) {
      bd = d;
      best = c;
    }
  }
  return best;
}

// closest_lane_scan's answer from two candidates: for |y| < 2^20 (lane offsets exact to 1/8) the
// first least offset is c0 = floor(y / 4) clamped to the lanes, or c0 + 1 if its offset is
// strictly smaller.  Below c0 the offsets are >= 4 > |offset(c0)| (y - 4 c0 is exact, Sterbenz),
// above c0 + 1 likewise; outside the road the offsets are strictly monotone in c.  Any other y
// (and NaN) takes the scan.
__device__ __forceinline__ int closest_lane(float y, int lanes) {
  if (!(hm_absf(y) < 1048576.0f)) return closest_lane_scan(y, lanes);
  const float q = hm_floorf(y * (1.0f / LANE_WIDTH));
  const int c0 = q >= (float)(lanes - 1) ? lanes - 1 : (q > 0.0f ? (int)q : 0);
  const bool up = c0 + 1 < lanes && hm_absf(lane_lat(y, c0 + 1)) < hm_absf(lane_lat(y, c0));
  return up ? c0 + 1 : c0;
}

// IDMVehicle.desired_gap(ego=a, front=b), from the velocity vectors (speed * (cos h, sin h),
// formed once per vehicle and frame: the same products upstream's velocity property forms)
__device__ __forceinline__ float desired_gap_v(float a_spd, float a_c, float a_s, float avx,
                                               float avy, float bvx, float bvy) {
  float dv = hm_fma(avx - bvx, a_c, (avy - bvy) * a_s);
  return hm_fma(a_spd, TIME_WANTED, DISTANCE_WANTED) + (a_spd * dv) * INV_TWO_SQRT_AB;
}

// IDMVehicle.acceleration, free-road term: the ego vehicle's base speed / target speed ...
__device__ __forceinline__ float idm_base(float ev_spd, float ev_tsp, float limit) {
  float tsp = hm_clipf(ev_tsp, 0.0f, limit);
  return hm_maxf(ev_spd, 0.0f) / hm_absf(hm_not_zero(tsp));
}

// ... raised to the deciding vehicle's DELTA, from the base and its log (hm_logf_idm):
// np.power(base, DELTA) in hm_powf's arithmetic, branch-free (bit-identical, hwy_math.h)
__device__ __forceinline__ float idm_free_from(float base, float lg, float delta) {
  if (kSkip & 32) return hm_fma(-COMFORT_ACC_MAX, base * base, COMFORT_ACC_MAX);
  return hm_fma(-COMFORT_ACC_MAX, hm_expf_idm(lg, delta, base), COMFORT_ACC_MAX);
}

// IDMVehicle.acceleration given its free-road term `acc` (interaction with the front vehicle)
// (ev_vx, ev_vy, fv_vx, fv_vy: the two velocity vectors)
__device__ __forceinline__ float idm_with_front(float acc, float ev_spd, float ev_x, float ev_c,
                                                float ev_s, float ev_vx, float ev_vy,
                                                bool has_front, float fv_x, float fv_vx,
                                                float fv_vy) {
  if (has_front) {
    float d = fv_x - ev_x;
    float g = desired_gap_v(ev_spd, ev_c, ev_s, ev_vx, ev_vy, fv_vx, fv_vy) / hm_not_zero(d);
    acc = hm_fma(-COMFORT_ACC_MAX, g * g, acc);
  }
  return acc;
}

// ControlledVehicle.steering_control(target lane c) clipped to +-MAX_STEERING, returned as its
// tangent.  Closed form (DESIGN.md deviations; oracle steering_tan): with z the clipped sine of
// the slip angle, tan(clip(atan(2 tan(asin z)))) = clip(2 z / sqrt((1 - z)(1 + z)), +-tan MAX).
__device__ __forceinline__ float steering_tan(float y, float h, float spd, int c) {
  float lat = lane_lat(y, c);
  float lane_future_heading = 0.0f;
  float lateral_speed_command = -KP_LATERAL * lat;
  const float inv_spd = 1.0f / hm_not_zero(spd);  // both of upstream's divisions by not_zero(speed)
  float heading_command = hm_asinf(hm_clipf(lateral_speed_command * inv_spd, -1.0f, 1.0f));
  float heading_ref = lane_future_heading + hm_clipf(heading_command, -HM_PIO4_F, HM_PIO4_F);
  float heading_rate_command = KP_HEADING * hm_wrap_to_pi(heading_ref - h);
  const float z =
      hm_clipf(((VEH_LENGTH / 2.0f) * inv_spd) * heading_rate_command, -1.0f, 1.0f);
  const float t = 2.0f * (z / __builtin_sqrtf((1.0f - z) * (1.0f + z)));
  return hm_clipf(t, -TAN_MAX_STEERING, TAN_MAX_STEERING);
}

// utils.are_polygons_intersecting on the two 5x2 m rectangles (a = lower road index), in the
// closed form of oracle/hwy_oracle.c rect_sat (same operations in the same order): intervals
// centre.n -/+ (L/2 |u.n| + W/2 |v.n|) on upstream's eight edge normals
// -u_a, v_a, u_a, -v_a, -u_b, v_b, u_b, -v_b, the opposite ones by exact negation.
__device__ __forceinline__ void rect_interval(float x, float y, float c, float s, float nx,
                                              float ny, float& mn, float& mx) {
  const float p = hm_fma(x, nx, y * ny);
  const float r = hm_fma(VEH_LENGTH / 2.0f, hm_absf(hm_fma(c, nx, s * ny)),
                         (VEH_WIDTH / 2.0f) * hm_absf(hm_fma(c, ny, -(s * nx))));
  mn = p - r;
  mx = p + r;
}

__device__ __forceinline__ float interval_distance(float min_a, float max_a, float min_b,
                                                   float max_b) {
  return min_a < min_b ? min_b - max_a : min_a - max_b;
}

// `activem`: the lanes holding a pair.  The wave stops once every active lane has broken out
// (nothing changes for a lane after its break), which after a's own two normals is the usual
// case: cars in adjacent lanes separate on v_a, cars in one lane on u_a.  Each edge runs on every
// lane: a lane already out has inter = will = false, which the edge's updates keep (the same
// values upstream's break leaves); the break test reads wave masks kept from the compares.
__device__ __forceinline__ void sat_collide(uint64_t activem, float xa, float ya, float ca, float sa,
                                            float dax, float day, float xb, float yb, float cb,
                                            float sb, float dbx, float dby, bool* inter_out,
                                            bool* will_out, float* tx, float* ty) {
  const float cdx = xa - xb, cdy = ya - yb;
  const float ddx = dax - dbx, ddy = day - dby;
  bool inter = true, will = true;
  uint64_t interm = activem, willm = activem;  // ballot(active && inter), ballot(active && will)
  float min_distance = __builtin_huge_valf(), axx = 0.0f, axy = 0.0f;
  float pa0[2], pa1[2], pb0[2], pb1[2], vpk[2], cdk[2], nxk[2], nyk[2];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int k = e & 1;
    float min_a, max_a, min_b, max_b, vp, cd, sx, sy;
    if (!(e & 2)) {  // -u (k = 0) or v (k = 1) of rectangle e / 4
      const float c = e < 4 ? ca : cb, s = e < 4 ? sa : sb;
      nxk[k] = k ? -s : -c;
      nyk[k] = k ? c : -s;
      rect_interval(xa, ya, ca, sa, nxk[k], nyk[k], pa0[k], pa1[k]);
      rect_interval(xb, yb, cb, sb, nxk[k], nyk[k], pb0[k], pb1[k]);
      vpk[k] = hm_fma(nxk[k], ddx, nyk[k] * ddy);
      cdk[k] = hm_fma(cdx, nxk[k], cdy * nyk[k]);
      min_a = pa0[k], max_a = pa1[k], min_b = pb0[k], max_b = pb1[k];
      vp = vpk[k], cd = cdk[k], sx = nxk[k], sy = nyk[k];
    } else {  // the opposite edge: n -> -n
      min_a = -pa1[k], max_a = -pa0[k], min_b = -pb1[k], max_b = -pb0[k];
      vp = -vpk[k], cd = -cdk[k], sx = -nxk[k], sy = -nyk[k];
    }
    {  // upstream breaks out once both are false (a lane past that keeps both false here)
      const bool s0 = interval_distance(min_a, max_a, min_b, max_b) > 0.0f;
      inter = inter && !s0;
      if (vp < 0.0f)
        min_a = min_a + vp;
      else
        max_a = max_a + vp;
      const float distance = interval_distance(min_a, max_a, min_b, max_b);
      const bool s1 = distance > 0.0f;
      will = will && !s1;
      interm &= ~ballot(s0);
      willm &= ~ballot(s1);
      if ((inter || will) && hm_absf(distance) < min_distance) {
        min_distance = hm_absf(distance);
        axx = cd > 0.0f ? sx : -sx;
        axy = cd > 0.0f ? sy : -sy;
      }
    }
    if ((e & 1) && e < 7 && !(interm | willm)) break;
  }
  *inter_out = inter;
  *will_out = will;
  *tx = will ? min_distance * axx : 0.0f;
  *ty = will ? min_distance * axy : 0.0f;
}

// ------------------------------------------------------------------------- reset
__device__ __forceinline__ uint64_t schedule_seed(const hwy_config& C, int e, int episode) {
  return (uint64_t)(C.seed_base + (int64_t)C.env_offset + (int64_t)e + 1 +
                    C.seed_stride * (int64_t)episode);
}

// the seed of (env e, episode k): the handle's schedule, or its experiment group's
// (hwy_set_seed_groups: group g = e / group_envs, l = e - g * group_envs)
__device__ __forceinline__ uint64_t episode_seed(const StepParams& P, int e, int episode) {
  const hwy_config& C = P.cfg;
  if (!P.group_seed) return schedule_seed(C, e, episode);
  const int g = e / P.group_envs, l = e - g * P.group_envs;
  return (uint64_t)(P.group_seed[g] + (int64_t)C.env_offset + (int64_t)l + 1 +
                    C.seed_stride * (int64_t)episode);
}

__device__ __forceinline__ const float* group_pe_table(const StepParams& P, int e) {
  return P.pe_group_stride ? P.pe_table + (size_t)(e / P.group_envs) * P.pe_group_stride
                           : P.pe_table;
}

// HighwayEnv._create_vehicles via Vehicle.create_random / IDMVehicle.randomize_behavior
__device__ void reset_wave(const hwy_config& C, int lane, uint64_t seed, Veh& v) {
  const int V = C.vehicles_count + 1;
  const int lanes = C.lanes_count;
  uint32_t k0 = (uint32_t)(seed & 0xffffffffu), k1 = (uint32_t)(seed >> 32);
  hm_u32x4 u = hm_philox4x32_10((uint32_t)lane, 0u, 0u, 0x52535431u, k0, k1);
  float fac = hm_expf((-5.0f / 40.0f) * (float)lanes);
  int ln;
  float speed, spacing;
  if (lane == 0) {
    ln = C.initial_lane_id >= 0 ? C.initial_lane_id : hm_choice(u.v[0], lanes);
    speed = 25.0f;
    spacing = C.ego_spacing;
  } else {
    ln = hm_choice(u.v[0], lanes);
    speed = hm_uniform(u.v[1], 0.7f * C.speed_limit, 0.8f * C.speed_limit);
    spacing = 1.0f / C.vehicles_density;
  }
  float default_spacing = 12.0f + 1.0f * speed;
  float offset = spacing * default_spacing * fac;
  float inc = offset * hm_uniform(u.v[2], 0.9f, 1.1f);
  // x0 = max(x of vehicles already on the road) + inc: a sequential chain in road order
  float mx = 3.0f * rdlf(offset, 0) + rdlf(inc, 0);
  float x = mx;
  for (int k = 1; k < V; ++k) {
    float xk = mx + rdlf(inc, k);
    if (lane == k) x = xk;
    if (xk > mx) mx = xk;
  }
  v.x = x;
  v.y = (float)ln * LANE_WIDTH;
  v.h = 0.0f;
  v.spd = speed;
  v.ln = ln;
  v.tl = ln;
  v.tsp = speed;
  v.present = lane < V;
  v.crashed = false;
  v.imp = false;
  v.ix = 0.0f;
  v.iy = 0.0f;
  v.aacc = 0.0f;
  v.asteer = 0.0f;
  if (lane == 0) {
    v.dlt = 0.0f;
    v.tmr = 0.0f;
  } else {
    float t = (v.x + v.y) * HM_PI_F;
    v.tmr = t - hm_floorf(t);
    v.dlt = hm_uniform(u.v[3], 3.5f, 4.5f);
  }
  if (!v.present) {
    v.x = v.y = v.spd = v.tsp = v.dlt = v.tmr = 0.0f;
    v.ln = v.tl = 0;
  }
}

// road-order position of every vehicle after a reset: create_random places each car ahead of all
// previous ones (x strictly increasing with the index), so the order is the index order
__device__ __forceinline__ int reset_order_pos(int lane, int V) {
  return lane < V ? lane : V + (WAVE - 1 - lane);
}

// ------------------------------------------------------------------------- observation
__device__ __forceinline__ float feature_value(int fid, float x, float y, float spd, float h,
                                               float c, float s) {
  switch (fid) {
    case HWY_FEAT_PRESENCE: return 1.0f;
    case HWY_FEAT_X: return x;
    case HWY_FEAT_Y: return y;
    case HWY_FEAT_VX: return spd * c;
    case HWY_FEAT_VY: return spd * s;
    case HWY_FEAT_COS_H: return c;
    case HWY_FEAT_SIN_H: return s;
    case HWY_FEAT_HEADING: return h;
  }
  return 0.0f;
}
__device__ __forceinline__ bool is_relative_feature(int fid) {
  return fid == HWY_FEAT_X || fid == HWY_FEAT_Y || fid == HWY_FEAT_VX || fid == HWY_FEAT_VY;
}

// One wrapped observation row: in[F] (row values), exy = ego row's first two values.
// Writes F_out values to out (global).  rope_embed.py:44-74 / dist_embed.py:76-96 /
// rank_embed.py:45-51.
__device__ __forceinline__ void write_pe_row(const float* vals, int F, int kind, int d, int row,
                                             float ex0, float ex1, float max_dist,
                                             const float* table, bool have_override,
                                             float override_nd, float* out) {
  if (kind == HWY_PE_ROPE) {
    float rx = vals[0] - ex0, ry = vals[1] - ex1;
    float nd = have_override ? override_nd
                             : hm_clipf(__builtin_sqrtf(rx * rx + ry * ry) / max_dist, 0.0f, 1.0f);
#pragma unroll
    for (int f = 0; f < HWY_MAX_FEATURES; ++f)
      if (f < F) {
        if (f < (d & ~1)) {
          const int p = f >> 1;
          float th = (HM_TWO_PI_F * nd) * table[p];
          float s = hm_sinf(th), c = hm_cosf(th);
          float xx = vals[2 * p], yy = vals[2 * p + 1];
          out[f] = (f & 1) ? (xx * s + yy * c) : (xx * c - yy * s);
        } else {
          out[f] = vals[f];
        }
      }
    return;
  }
#pragma unroll
  for (int f = 0; f < HWY_MAX_FEATURES; ++f)
    if (f < F) out[f] = vals[f];
  if (kind == HWY_PE_RANK) {
    for (int k = 0; k < d; ++k) out[F + k] = table[row * d + k];
  } else if (kind == HWY_PE_DIST || kind == HWY_PE_DIST1) {
    float rx = vals[0] - ex0, ry = vals[1] - ex1;
    float dist = kind == HWY_PE_DIST ? __builtin_sqrtf(rx * rx + ry * ry) : hm_absf(rx);
    float nd = have_override ? override_nd : hm_clipf(dist / max_dist, 0.0f, 1.0f);
    const int hd = d / 2;
    for (int k = 0; k < hd; ++k) {
      float ang = (HM_TWO_PI_F * nd) * table[k];
      out[F + k] = hm_sinf(ang);
      out[F + hd + k] = hm_cosf(ang);
    }
  }
}

// KinematicObservation.observe + fused wrapper for the env of this wave.
// ch / sh: hm_cosf / hm_sinf of v.h (the step carries them from the last frame)
// lds_key: WAVE 64-bit words of per-wave LDS scratch (the distance ranking)
__device__ void observe_wave(const hwy_config& C, int lane, const Veh& v, float ch, float sh,
                             int step, uint64_t seed, const float* pe_table, float* obs_env,
                             int fout, int* lds_vor, int* lds_inv, unsigned long long* lds_key) {
  const int V = C.vehicles_count + 1;
  const int N = C.obs_vehicles, F = C.n_features;
  const float ex = rdlf(v.x, 0), ey = rdlf(v.y, 0), eh = rdlf(v.h, 0), espd = rdlf(v.spd, 0);
  const float ec = rdlf(ch, 0), es = rdlf(sh, 0);
  // Road.close_objects_to(ego, PERCEPTION_DISTANCE, count=N-1, see_behind, sort)
  float dx = v.x - ex, dy = v.y - ey;
  bool elig = v.present && lane >= 1 && lane < V &&
              (__builtin_sqrtf(hm_fma(dx, dx, dy * dy)) < PERCEPTION_DISTANCE) &&
              (C.see_behind || -2.0f * VEH_LENGTH < v.x - ex);
  const uint64_t em = ballot(elig);
  int rank;
  if (C.order == HWY_ORDER_SORTED && (kSkip & 64)) {
    rank = __popcll(em & ((1ull << lane) - 1ull));
  } else if (C.order == HWY_ORDER_SORTED) {
    // rank = #{eligible k : |dx_k| < |dx| or (|dx_k| == |dx| and k < lane)}: the bits of |dx|
    // (non-negative: their order is the value order) above the vehicle index make one 64-bit
    // key per vehicle, so a single compare orders by distance and breaks ties by index; an
    // ineligible vehicle holds ~0 and is never below an eligible one.  The keys go through LDS
    // and every lane reads them at the same address (broadcast): two VALU per vehicle
    const unsigned long long ck =
        elig ? ((unsigned long long)hm_f2bits(hm_absf(v.x - ex)) << 32) | (uint32_t)lane : ~0ull;
    lds_key[lane] = ck;
    wave_lds_sync();
    rank = 0;
    for (int k0 = 0; k0 < V; k0 += 2) {
      const unsigned long long k_a = lds_key[k0], k_b = lds_key[k0 + 1];
      rank += k_a < ck ? 1 : 0;
      rank += k_b < ck ? 1 : 0;  // lane k0 + 1 >= V is not present: ~0
    }
    wave_lds_sync();
  } else {
    rank = __popcll(em & ((1ull << lane) - 1ull));
  }
  int nvis = __popcll(em);
  if (nvis > N - 1) nvis = N - 1;
  if (elig && rank < N - 1) lds_vor[rank] = lane;
  // np_random.shuffle(obs[1:]) -> Philox keyed permutation of the N-1 rows
  const bool shuffle = C.order == HWY_ORDER_SHUFFLED && N > 2;
  if (shuffle) {
    uint32_t key = 0u;
    if (lane < N - 1)
      key = hm_philox4x32_10((uint32_t)lane, (uint32_t)step, 0u, 0x53485546u,
                             (uint32_t)(seed & 0xffffffffu), (uint32_t)(seed >> 32))
                .v[0];
    int dest = 0;
    for (int p0 = 0; p0 < N - 1; p0 += 4) {
      uint32_t kp[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) kp[u] = (uint32_t)rdli((int)key, min(p0 + u, WAVE - 1));
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int p = p0 + u;
        dest += (p < N - 1 && (kp[u] < key || (kp[u] == key && p < lane))) ? 1 : 0;
      }
    }
    if (lane < N - 1) lds_inv[dest] = lane;
  }
  wave_lds_sync();
  // output row r = lane
  int kind = 0;  // 0 zero row, 1 ego, 2 other
  int src = 0;
  if (lane == 0) {
    kind = 1;
  } else if (lane < N) {
    int q = shuffle ? lds_inv[lane - 1] : lane - 1;
    if (q < nvis) {
      kind = 2;
      src = lds_vor[q];
    }
  }
  wave_lds_sync();
  const float sx = shf(v.x, src), sy = shf(v.y, src), sspd = shf(v.spd, src), shh = shf(v.h, src);
  const float sc = shf(ch, src), ss = shf(sh, src);
  float vals[HWY_MAX_FEATURES];
#pragma unroll
  for (int f = 0; f < HWY_MAX_FEATURES; ++f) {
    float val = 0.0f;
    if (f < F && kind != 0) {
      int fid = C.feature_ids[f];
      val = feature_value(fid, sx, sy, sspd, shh, sc, ss);
      if (kind == 2 && !C.absolute && is_relative_feature(fid))
        val = val - feature_value(fid, ex, ey, espd, eh, ec, es);
      if (C.normalize && C.has_range[f]) {
        val = hm_lmap(val, C.features_range[f][0], C.features_range[f][1], -1.0f, 1.0f);
        if (C.clip) val = hm_clipf(val, -1.0f, 1.0f);
      }
    }
    vals[f] = val;
  }
  const int eg = C.ego_idx;
  const float ex0 = rdlf(vals[0], eg), ex1 = rdlf(vals[1], eg);
  if (lane < N)
    write_pe_row(vals, F, C.pe_kind, C.d_embed, lane, ex0, ex1, C.pe_max_dist, pe_table, false,
                 0.0f, obs_env + (size_t)lane * fout);
}

// ------------------------------------------------------------------------- state I/O

__device__ __forceinline__ void load_veh(const uint32_t* st, size_t fstride, uint32_t idx, int lane,
                                         int V, Veh& v, int& order_pos) {
  v.x = hm_bits2f((st + HWY_F_X * fstride)[idx]);
  v.y = hm_bits2f((st + HWY_F_Y * fstride)[idx]);
  v.h = hm_bits2f((st + HWY_F_HEADING * fstride)[idx]);
  v.spd = hm_bits2f((st + HWY_F_SPEED * fstride)[idx]);
  v.tsp = hm_bits2f((st + HWY_F_TSPEED * fstride)[idx]);
  v.dlt = hm_bits2f((st + HWY_F_DELTA * fstride)[idx]);
  v.tmr = hm_bits2f((st + HWY_F_TIMER * fstride)[idx]);
  v.ix = hm_bits2f((st + HWY_F_IMPX * fstride)[idx]);
  v.iy = hm_bits2f((st + HWY_F_IMPY * fstride)[idx]);
  v.ln = (int)(st + HWY_F_LANE * fstride)[idx];
  v.tl = (int)(st + HWY_F_TLANE * fstride)[idx];
  uint32_t fl = (st + HWY_F_FLAGS * fstride)[idx];
  v.crashed = (fl & HWY_FLAG_CRASHED) != 0u;
  v.imp = (fl & HWY_FLAG_IMPACT) != 0u;
  v.present = ((fl & HWY_FLAG_PRESENT) != 0u) && lane < V;
  order_pos = (int)((fl & HWY_FLAG_ORDER_MASK) >> HWY_FLAG_ORDER_SHIFT);
  v.aacc = 0.0f;
  v.asteer = 0.0f;
}

__device__ __forceinline__ void store_veh(uint32_t* st, size_t fstride, uint32_t idx, int lane, int V,
                                          const Veh& v, int order_pos) {
  // opaque copies of the offset, the base and the field stride: the 13 field addresses are
  // rebuilt here instead of being kept live from load_veh across the whole step (26 VGPRs for the
  // lane addresses, 26 SGPRs for the field bases, which otherwise spill the frame loop's scalars)
  asm volatile("" : "+v"(idx));
  asm volatile("" : "+s"(st));
  asm volatile("" : "+s"(fstride));
  const bool live = lane < V;
  (st + HWY_F_X * fstride)[idx] = live ? hm_f2bits(v.x) : 0u;
  (st + HWY_F_Y * fstride)[idx] = live ? hm_f2bits(v.y) : 0u;
  (st + HWY_F_HEADING * fstride)[idx] = live ? hm_f2bits(v.h) : 0u;
  (st + HWY_F_SPEED * fstride)[idx] = live ? hm_f2bits(v.spd) : 0u;
  (st + HWY_F_TSPEED * fstride)[idx] = live ? hm_f2bits(v.tsp) : 0u;
  (st + HWY_F_DELTA * fstride)[idx] = live ? hm_f2bits(v.dlt) : 0u;
  (st + HWY_F_TIMER * fstride)[idx] = live ? hm_f2bits(v.tmr) : 0u;
  (st + HWY_F_IMPX * fstride)[idx] = (live && v.imp) ? hm_f2bits(v.ix) : 0u;
  (st + HWY_F_IMPY * fstride)[idx] = (live && v.imp) ? hm_f2bits(v.iy) : 0u;
  (st + HWY_F_LANE * fstride)[idx] = live ? (uint32_t)v.ln : 0u;
  (st + HWY_F_TLANE * fstride)[idx] = live ? (uint32_t)v.tl : 0u;
  (st + HWY_F_FLAGS * fstride)[idx] =
      live ? ((v.crashed ? HWY_FLAG_CRASHED : 0u) | (v.imp ? HWY_FLAG_IMPACT : 0u) |
              (v.present ? HWY_FLAG_PRESENT : 0u) |
              ((uint32_t)order_pos << HWY_FLAG_ORDER_SHIFT))
           : 0u;
}

__device__ __forceinline__ void store_env_words(uint32_t* st, size_t fstride, uint32_t idx, int lane,
                                                int step, int episode, uint64_t seed, float ego_acc,
                                                float ego_steer, float ep_return) {
  asm volatile("" : "+v"(idx));
  asm volatile("" : "+s"(st));
  asm volatile("" : "+s"(fstride));
  uint32_t w = 0u;
  if (lane == HWY_E_STEP) w = (uint32_t)step;
  if (lane == HWY_E_EPISODE) w = (uint32_t)episode;
  if (lane == HWY_E_SEED_LO) w = (uint32_t)(seed & 0xffffffffu);
  if (lane == HWY_E_SEED_HI) w = (uint32_t)(seed >> 32);
  if (lane == HWY_E_EGO_ACC) w = hm_f2bits(ego_acc);
  if (lane == HWY_E_EGO_STEER) w = hm_f2bits(ego_steer);
  if (lane == HWY_E_RETURN) w = hm_f2bits(ep_return);
  (st + HWY_F_ENV * fstride)[idx] = w;
}

// ------------------------------------------------------------------------- road order
// The vehicles of a wave sorted by (x ascending, index descending), kept across the frames of
// a step: lane p of `ord` holds the vehicle at position p, `rk` is this lane's position.
// Absent lanes sort after every present vehicle, so the positions form a permutation of 0..63.
struct RoadOrder {
  int rk, ord;
  bool valid;
};

__device__ __forceinline__ uint64_t shf64(uint64_t v, int src) {
  const uint32_t lo = (uint32_t)shi((int)(uint32_t)v, src);
  const uint32_t hi = (uint32_t)shi((int)(uint32_t)(v >> 32), src);
  return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t shl1_64(uint64_t v) {
  return ((uint64_t)(uint32_t)shl1i((int)(uint32_t)(v >> 32)) << 32) |
         (uint32_t)shl1i((int)(uint32_t)v);
}
__device__ __forceinline__ uint64_t shr1_64(uint64_t v) {
  return ((uint64_t)(uint32_t)shr1i((int)(uint32_t)(v >> 32)) << 32) |
         (uint32_t)shr1i((int)(uint32_t)v);
}
__device__ __forceinline__ uint64_t swp1_64(uint64_t v) {
  return ((uint64_t)(uint32_t)swp1i((int)(uint32_t)(v >> 32)) << 32) |
         (uint32_t)swp1i((int)(uint32_t)v);
}

// order-preserving u32 image of x (+0 and -0 map together); absent -> above every float
__device__ __forceinline__ uint64_t road_key(float x, bool present, int lane) {
  const uint32_t u = hm_f2bits(x + 0.0f);
  uint32_t s = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
  if (!present) s = 0xffffffffu;
  return ((uint64_t)s << 32) | (uint32_t)(WAVE - 1 - lane);
}

// Re-validates (or rebuilds) the order for the current positions.
__device__ void road_order(int lane, const Veh& v, uint64_t pres, RoadOrder& o) {
  const uint64_t key = road_key(v.x, v.present, lane);
  bool sorted = false;
  if (o.valid) {
    uint64_t kp = shf64(key, o.ord);
    uint64_t kn = shl1_64(kp);  // the next position's key (DPP)
    sorted = (~ballot(kp < kn) & (~0ull >> 1)) == 0ull;  // every position but the last ascends
    // a few overtakes since the last frame: odd-even transposition rounds on (key, vehicle)
    // in position space usually restore the order without a full re-rank; the partner is
    // lane ^ 1 in the even phase and lane + 1 / lane - 1 (odd / even lane) in the odd one
    int ordp = o.ord;
    for (int round = 0; round < 3 && !sorted; ++round) {
#pragma unroll
      for (int ph = 0; ph < 2; ++ph) {
        const bool left = (lane & 1) == ph;
        int partner = left ? lane + 1 : lane - 1;
        if (partner < 0 || partner >= WAVE) partner = lane;
        uint64_t pk;
        int po;
        if (ph == 0) {
          pk = swp1_64(kp);
          po = swp1i(ordp);
        } else {
          const uint64_t up = shl1_64(kp), dn = shr1_64(kp);
          const int uo = shl1i(ordp), dno = shr1i(ordp);
          pk = left ? up : dn;
          po = left ? uo : dno;
        }
        const bool swap = partner != lane && (left ? (pk < kp) : (kp < pk));
        kp = swap ? pk : kp;
        ordp = swap ? po : ordp;
      }
      kn = shl1_64(kp);
      sorted = (~ballot(kp < kn) & (~0ull >> 1)) == 0ull;
    }
    if (sorted) {
      o.ord = ordp;
      o.rk = __builtin_amdgcn_ds_permute(ordp << 2, lane);  // vehicle ordp sits at position lane
    }
  }
  if (!sorted) {
    int r = 0;
    if (v.present) {
      for (int k = 0; k < WAVE; ++k) {
        if (!((pres >> k) & 1ull)) continue;
        const uint64_t kk = ((uint64_t)(uint32_t)rdli((int)(key >> 32), k) << 32) |
                            (uint32_t)(WAVE - 1 - k);
        r += kk < key ? 1 : 0;
      }
    } else {  // absent lanes: after all present ones, by descending lane index
      const uint64_t above = lane >= WAVE - 1 ? 0ull : (~0ull << (lane + 1));
      r = __popcll(pres) + __popcll(~pres & above);
    }
    o.rk = r;
    o.ord = __builtin_amdgcn_ds_permute(r << 2, lane);
    o.valid = true;
  }
}

// Road.neighbour_vehicles(self, lane c) for c = ln-1, ln, ln+1 (slot s <-> c = ln-1+s) from the
// road order: for each lane c a 64-bit mask over positions of the vehicles with
// on_lane(c, margin 1).  Upstream scans the list in index order with `s <= s_v and s_v <=
// s_front` (front: nearest x ahead or level, the LAST such vehicle on a tie) and `s_v < s and
// s_v > s_rear` (rear: nearest x strictly behind, the FIRST on a tie).  Equal x sit together in
// the order by descending index, so with g = the first position of this vehicle's x group the
// front is the lowest set position >= g other than its own, the rear the highest below g.  NaN
// positions fail on_lane; a vehicle at NaN itself finds nothing (every comparison is false).
struct LaneScan {
  float yp;      // y of the vehicle at position `lane`
  bool okp;      // that vehicle is present and inside the road's x range
  uint64_t okm;  // ballot(okp)
  uint64_t ahead, behind;  // candidate positions for the front / the rear of this vehicle
};

// xp: x of the vehicle at position `lane` (shf(v.x, o.ord), when the caller has it)
__device__ __forceinline__ LaneScan lane_scan(int lane, const Veh& v, uint64_t pres,
                                              const RoadOrder& o, float xp) {
  LaneScan L;
  const int npres = __popcll(pres);
  L.yp = shf(v.y, o.ord);
  L.okp = lane < npres && -LANE_VEH_LEN <= xp && xp < ROAD_LENGTH + LANE_VEH_LEN;
  L.okm = ballot(lane < npres) & ballot(-LANE_VEH_LEN <= xp) & ballot(xp < ROAD_LENGTH + LANE_VEH_LEN);
  const float xprev = shr1f(xp);
  const uint64_t starts = ballot(xprev != xp) | 1ull;  // x-group starts (bit 0 set)
  const int g = 63 - __builtin_clzll(starts & ((2ull << o.rk) - 1ull));  // rk = 63: all ones
  const bool selfok = v.x == v.x;
  L.ahead = selfok ? (~0ull << g) & ~(1ull << o.rk) : 0ull;
  L.behind = selfok ? (1ull << g) - 1ull : 0ull;
  return L;
}

__device__ __forceinline__ uint64_t on_lane_mask(const LaneScan& L, int c) {
  // (the compare's own mask, then a scalar AND: a ballot of p && q costs two VALU more)
  return ballot(hm_absf(lane_lat(L.yp, c)) <= LANE_WIDTH / 2.0f + 1.0f) & L.okm;
}

// Also returns qf[s], the road-order position of front s (this vehicle's own position when
// there is none), for gathers from position-space copies one bpermute level earlier.
__device__ __forceinline__ void neighbours_ordered(const hwy_config& C, int lane, const Veh& v,
                                                   uint64_t pres, const RoadOrder& o, float xq,
                                                   int fi[3], int ri[3], int qfp[3]) {
  const LaneScan L = lane_scan(lane, v, pres, o, xq);
  uint64_t m[3] = {0ull, 0ull, 0ull};
  if (C.lanes_count <= WAVE - 2) {
    // lane c's position mask (wave-uniform) goes to lane c + 1 of a VGPR pair (lanes 0 and
    // lanes_count + 1 .. 63 hold no lane: 0), and each vehicle reads its slots ln .. ln + 2
    int tlo = 0, thi = 0;
    for (int c = 0; c < C.lanes_count; ++c) {
      const uint64_t mc = on_lane_mask(L, c);
      const bool mine = lane == c + 1;
      tlo = mine ? (int)(uint32_t)mc : tlo;
      thi = mine ? (int)(uint32_t)(mc >> 32) : thi;
    }
#pragma unroll
    for (int s = 0; s < 3; ++s) {
      const int src = v.ln + s;  // slot of lane ln - 1 + s
      const bool in = src >= 0 && src < WAVE;
      const int q = in ? src : 0;
      const uint64_t mq = ((uint64_t)(uint32_t)shi(thi, q) << 32) | (uint32_t)shi(tlo, q);
      m[s] = in ? mq : 0ull;
    }
  } else {
    for (int c = 0; c < C.lanes_count; ++c) {
      const uint64_t mc = on_lane_mask(L, c);
#pragma unroll
      for (int s = 0; s < 3; ++s)
        if (c == v.ln - 1 + s) m[s] = mc;
    }
  }
#pragma unroll
  for (int s = 0; s < 3; ++s) {
    const uint64_t fa = m[s] & L.ahead, rb = m[s] & L.behind;
    const int qf = fa ? __builtin_ctzll(fa) : 0;
    const int qr = rb ? 63 - __builtin_clzll(rb) : 0;
    const int vf = shi(o.ord, qf), vr = shi(o.ord, qr);
    fi[s] = fa ? vf : -1;
    ri[s] = rb ? vr : -1;
    qfp[s] = fa ? qf : o.rk;
  }
}

// the front vehicle on an arbitrary lane c of each vehicle (same rule as neighbours_ordered)
__device__ __forceinline__ int front_on_lane(const hwy_config& C, int lane, const Veh& v,
                                             uint64_t pres, const RoadOrder& o, int c_own) {
  const LaneScan L = lane_scan(lane, v, pres, o, shf(v.x, o.ord));
  uint64_t m = 0ull;
  for (int c = 0; c < C.lanes_count; ++c) {
    const uint64_t mc = on_lane_mask(L, c);
    if (c == c_own) m = mc;
  }
  const uint64_t fa = m & L.ahead;
  const int vf = shi(o.ord, fa ? __builtin_ctzll(fa) : 0);
  return fa ? vf : -1;
}

// per-wave LDS of the collision pass (5.4 KB)
struct CollLds {
  unsigned long long imx[WAVE], imy[WAVE];  // (partner + 1) << 32 | impact bits, max-reduced
  int crash[WAVE];
  int pord[WAVE];                         // vehicle at each road-order position
  uint16_t plist[WAVE * (WAVE - 1) / 2];  // candidate pairs (a << 8 | b), a < b
};

// ------------------------------------------------------------------------- one frame
// Road.act() then Road.step(dt) for the env of this wave (lane = vehicle).
// pres: ballot(v.present), fixed for the step (presence changes only at a reset)
__device__ void frame_wave(const hwy_config& C, int lane, Veh& v, float dt, float tan_ego, RoadOrder& ro,
                           float& cos_h, float& sin_h, CollLds& cl, SecProf& sp, uint64_t pres) {
  const int lanes = C.lanes_count;
  const float limit = C.speed_limit;
  const float ch = cos_h, sh = sin_h;  // cos / sin of v.h (carried from the previous frame)

  // ---------------- Road.act: IDMVehicle.act for every non-crashed traffic car
  const bool actor = v.present && lane >= 1 && !v.crashed;
  const int tl_old = v.tl;
  const bool mid = v.ln != v.tl;
  const bool fire = actor && !mid && (LANE_CHANGE_DELAY < v.tmr);  // utils.do_every
  // (wave masks from the compares' own masks: a ballot of a compound bool costs two VALU)
  const uint64_t actm = pres & ~1ull & ~ballot(v.crashed);  // ballot(actor)
  const uint64_t firem = actm & ~ballot(v.ln != v.tl) & ballot(LANE_CHANGE_DELAY < v.tmr);
  if (fire) v.tmr = 0.0f;

  // Road.neighbour_vehicles on lanes ln-1, ln, ln+1 (slot s <-> lane ln-1+s)
  int fi[3], ri[3];
  SEC(sp, 0);
  if (!ro.valid) road_order(lane, v, pres, ro);  // later frames: validated after the last move
  SEC(sp, 9);
  // position-space copies of the fronts' state (vehicle at position p on lane p), gathered
  // alongside the order so the fronts' values are one bpermute from their positions
  // this vehicle's velocity vector (Vehicle.velocity), shared by every desired_gap of the frame
  const float vvx = v.spd * ch, vvy = v.spd * sh;
  const float xq = shf(v.x, ro.ord), vxq = shf(vvx, ro.ord), vyq = shf(vvy, ro.ord);
  int qfp[3];
  neighbours_ordered(C, lane, v, pres, ro, xq, fi, ri, qfp);
  SEC(sp, 1);

  // gathers (all lanes active); a missing front reads this vehicle's own values (unused)
  const int sop = qfp[1];
  const float op_x = shf(xq, sop), op_vx = shf(vxq, sop), op_vy = shf(vyq, sop);
  float np_x[2], np_vx[2], np_vy[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int a = qfp[2 * q];  // slot 0 (left, ln-1) and slot 2 (right, ln+1)
    np_x[q] = shf(xq, a);
    np_vx[q] = shf(vxq, a);
    np_vy[q] = shf(vyq, a);
  }

  // acceleration(self, front on own lane): IDM term and MOBIL's self_a
  float self_a = 0.0f;
  // (the free-road term is shared by every acceleration(self, .) evaluated this frame)
  // every lane's free-road base and its log (the ego as a plain Vehicle: target speed 0), also
  // read by mobil for a new follower (same base, the deciding vehicle's DELTA)
  const float fbase = idm_base(v.spd, lane == 0 ? 0.0f : v.tsp, limit);
  const float flog = hm_logf_idm(fbase);
  float a_free = 0.0f;
  if (actor) {
    a_free = idm_free_from(fbase, flog, v.dlt);
    self_a = idm_with_front(a_free, v.spd, v.x, ch, sh, vvx, vvy, fi[1] >= 0, op_x, op_vx, op_vy);
  }

  // IDMVehicle.change_lane_policy -> mobil, side lanes left then right (POLITENESS = 0, so the
  // followers' unchanged-lane terms multiply by zero and are not evaluated).  mobil's two tests
  // are pure and both must hold, so the cheap one (own acceleration gain, free-road term shared)
  // runs first, and the new followers' data and IDM (a pow) only for the candidates that would
  // gain -- rarely any in a frame; the decision is upstream's.
  SEC(sp, 2);
  int ntl = v.tl;
  // (every lane evaluates both sides when any lane fires -- a lane without a front on a side,
  // or outside the lanes, reads a_free -- and the lane's own tests mask the result)
  bool gain[2] = {false, false};
  uint64_t gainm = 0ull;
  // the side-independent tests, once (a ballot of a compare used again under another branch
  // re-materialises too)
  const uint64_t basem = firem & ballot(0.0f <= v.x) & ballot(v.x < ROAD_LENGTH + LANE_VEH_LEN) &
                         ~ballot(hm_absf(v.spd) < 1.0f);
  if (basem && !(kSkip & 1)) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int c = v.ln - 1 + 2 * q;
      const int s = 2 * q;
      const float spa = idm_with_front(a_free, v.spd, v.x, ch, sh, vvx, vvy, fi[s] >= 0, np_x[q],
                                       np_vx[q], np_vy[q]);
      const bool in_lanes = c >= 0 && c < lanes;
      const bool reach = hm_absf(lane_lat(v.y, c)) <= 2.0f * LANE_WIDTH && 0.0f <= v.x &&
                         v.x < ROAD_LENGTH + LANE_VEH_LEN;  // is_reachable_from
      const bool slow = hm_absf(v.spd) < 1.0f;
      const bool loss = (spa - self_a) < LANE_CHANGE_MIN_ACC_GAIN;
      gain[q] = fire && in_lanes && reach && !slow && !loss;
      gainm |= basem & ballot(c >= 0) & ballot(c < lanes) &
               ballot(hm_absf(lane_lat(v.y, c)) <= 2.0f * LANE_WIDTH) & ~ballot(loss);
    }
  }
  if (gainm) {
    // upstream tries left, then right, and a passing right side overrides the left: so each
    // lane first evaluates the side that decides if it passes -- the right where it gains, else
    // the left -- in one pass over the lanes (one new-follower IDM, a pow, instead of two), and
    // only lanes whose right side gained but failed the braking test evaluate their left side
    // after it (rare).  The same arithmetic per side as the sequential order, so the same bits.
    auto new_follower_ok = [&](int q) {
      const int rq = q ? ri[2] : ri[0];
      const int b = rq >= 0 ? rq : lane;  // all lanes active: ds_bpermute
      const float nf_x = shf(v.x, b), nf_spd = shf(v.spd, b), nf_c = shf(ch, b), nf_s = shf(sh, b);
      const float nf_base = shf(fbase, b), nf_log = shf(flog, b);
      float nfp = 0.0f;
      if (rq >= 0)  // acceleration(ego_vehicle=new follower, front_vehicle=self), self's DELTA
        nfp = idm_with_front(idm_free_from(nf_base, nf_log, v.dlt), nf_spd, nf_x, nf_c, nf_s,
                             nf_spd * nf_c, nf_spd * nf_s, true, v.x, vvx, vvy);
      return !(nfp < -LANE_CHANGE_MAX_BRAKING_IMPOSED);
    };
    const int q1 = gain[1] ? 1 : 0;
    const bool nok = new_follower_ok(q1);  // every lane (the gathers need all 64 active)
    const bool ok1 = (gain[0] || gain[1]) && nok;
    if (ok1) ntl = v.ln - 1 + 2 * q1;
    const bool retry = gain[1] && !ok1 && gain[0];
    if (wave_any(retry)) {
      const bool ok0 = new_follower_ok(0);
      if (retry && ok0) ntl = v.ln - 1;
    }
  }

  SEC(sp, 3);
  // abort an ongoing lane change if another car targets the same lane within its desired gap,
  // in road order (lower indices already final, higher ones at their frame-start target)
  int tl_cur = ntl;
  uint64_t cm = (kSkip & 8) ? 0ull : actm & ballot(v.ln != v.tl);  // actor && mid
  // a lane can trigger an abort only while its visible target is not its own lane (vis == tj
  // and ln != tj), under either visibility; aborts only ever clear that, so this superset holds
  // for the whole loop
  const uint64_t canm = pres & ~1ull & (ballot(tl_cur != v.ln) | ballot(tl_old != v.ln));
  while (cm) {
    const int j = __builtin_ctzll(cm);
    cm &= cm - 1ull;
    const int tj = rdli(tl_cur, j);
    const int vis = (lane < j) ? tl_cur : tl_old;
    // the target-lane part of upstream's test first: most vehicles find no other car targeting
    // their lane, and then the gap test (four broadcasts and a desired_gap) is skipped
    const uint64_t cheapm = canm & ~(1ull << j) & ballot(v.ln != tj) & ballot(vis == tj);
    if (!cheapm) continue;
    const float xj = rdlf(v.x, j), vj = rdlf(v.spd, j), cj = rdlf(ch, j), sj = rdlf(sh, j);
    const float d = v.x - xj;
    const float d_star = desired_gap_v(vj, cj, sj, vj * cj, vj * sj, vvx, vvy);
    const uint64_t condm = cheapm & ballot(0.0f < d) & ballot(d < d_star);
    if (condm && lane == j) tl_cur = v.ln;
  }
  v.tl = tl_cur;

  SEC(sp, 4);
  // IDM on the target lane while changing lanes
  const bool need_t = actor && v.ln != v.tl;
  int ft = -1;
  if (v.tl == v.ln - 1) ft = fi[0];
  if (v.tl == v.ln + 1) ft = fi[2];
  const bool extra = need_t && !(v.tl == v.ln - 1 || v.tl == v.ln + 1);
  if (actm & ballot(v.ln != v.tl) & ~ballot(v.tl == v.ln - 1) & ~ballot(v.tl == v.ln + 1)) {  // target lane not adjacent (rare): its own lane mask
    const int fx = front_on_lane(C, lane, v, pres, ro, v.tl);
    if (extra) ft = fx;
  }
  const int st_ = ft >= 0 ? ft : lane;
  const float ft_x = shf(v.x, st_), ft_vx = shf(vvx, st_), ft_vy = shf(vvy, st_);
  if (actor) {
    const float steer = (kSkip & 16) ? 0.0f : steering_tan(v.y, v.h, v.spd, v.tl);
    float acc = self_a;
    if (need_t) {
      const float acc_t =
          idm_with_front(a_free, v.spd, v.x, ch, sh, vvx, vvy, ft >= 0, ft_x, ft_vx, ft_vy);
      acc = hm_minf(acc, acc_t);
    }
    acc = hm_clipf(acc, -ACC_MAX, ACC_MAX);
    v.asteer = steer;
    v.aacc = acc;
  }

  SEC(sp, 5);
  // ---------------- Road.step: Vehicle.step for every vehicle
  if (v.present) {
    if (lane != 0) v.tmr = v.tmr + dt;  // IDMVehicle.step
    if (v.crashed) {                    // clip_actions
      v.asteer = 0.0f;
      v.aacc = -1.0f * v.spd;
    }
    if (v.spd > MAX_SPEED) {
      v.aacc = hm_minf(v.aacc, 1.0f * (MAX_SPEED - v.spd));
    } else if (v.spd < MIN_SPEED) {
      v.aacc = hm_maxf(v.aacc, 1.0f * (MIN_SPEED - v.spd));
    }
    // beta = atan(tan(steering) / 2) in closed form (oracle vehicle_step): cos and sin of beta
    // from u = tan(beta), cos / sin of h + beta by angle addition from the carried cos / sin h
    const float u = 0.5f * ((lane == 0 && !v.crashed) ? tan_ego : v.asteer);
    const float cb = 1.0f / __builtin_sqrtf(hm_fma(u, u, 1.0f));
    const float sb = u * cb;
    const float cdir = hm_fma(ch, cb, -(sh * sb));
    const float sdir = hm_fma(sh, cb, ch * sb);
    const float vx = v.spd * cdir;
    const float vy = v.spd * sdir;
    v.x = hm_fma(vx, dt, v.x);
    v.y = hm_fma(vy, dt, v.y);
    if (v.imp) {
      v.x = v.x + v.ix;
      v.y = v.y + v.iy;
      v.crashed = true;
      v.imp = false;
    }
    v.h = hm_fma(v.spd * sb, dt * (2.0f / VEH_LENGTH), v.h);  // speed sin(beta) / (L/2) dt
    v.spd = hm_fma(v.aacc, dt, v.spd);
    v.ln = closest_lane(v.y, lanes);  // on_state_update
  }

  SEC(sp, 6);
  // ---------------- Road.step: handle_collisions for every pair, a = lower index
  float c2, s2;
  hm_sincosf(v.h, &s2, &c2);
  cos_h = c2;
  sin_h = s2;
  road_order(lane, v, pres, ro);  // new positions; also serves the next frame's neighbours
  SEC(sp, 7);
  // Candidates first: a pair can pass the centre-distance pre-check only if |dx| is within
  // that bound, taken here with the wave's largest speed (and widened past any rounding; a
  // non-finite speed or position disables the filter).
  float vabs = v.present ? hm_absf(v.spd) : 0.0f;
  // any present vehicle with a non-finite x, y or speed (the compares' own masks)
  const uint64_t nonfinite = pres & (ballot(!(hm_absf(v.x) <= 3.0e38f)) |
                                     ballot(!(hm_absf(v.y) <= 3.0e38f)) |
                                     ballot(!(hm_absf(v.spd) <= 3.0e38f)));
  vabs = wave_max_f(vabs);
  const float xbound = nonfinite ? __builtin_huge_valf()
                                 : (VEH_DIAGONAL + vabs * dt) * 1.001f + 1.0e-3f;
  // x-sorted road order, in position space (lane = position p, holding vehicle ord[p]): the
  // candidates are the pairs (p, p+o) whose |dx| is within the bound.  x is monotone along the
  // order, so the run from p upwards is contiguous and every pair is found once, from its lower
  // position; x at p+o comes from a one-lane DPP shift per step (equal x sit together; a NaN x,
  // or any non-finite value, makes the bound infinite: every pair of present vehicles).
  int run = 0;  // the candidates of position p: (p, p + o) for o = 1 .. run
  {
    const int npres = __popcll(pres);
    const float xs = shf(v.x, ro.ord);  // x at position `lane`
    float xu = xs;
    // the loop runs on the wave mask U = ballot(up), kept from the compares' own masks (a
    // ballot of a compound or loop-carried bool re-materialises it: two VALU), and counts each
    // position's run; its candidates are o = 1 .. run
    bool up = lane < npres;
    uint64_t U = (kSkip & 4) ? 0ull : ballot(lane < npres);
    for (int o = 1; U; ++o) {
      xu = __int_as_float(shl1i(__float_as_int(xu)));  // x at position lane + o
      const bool inr = lane < npres - o;
      const bool far = hm_absf(xu - xs) > xbound;
      up = up && inr && !far;
      U &= ballot(inr) & ~ballot(far);
      run += up ? 1 : 0;
    }
  }
  SEC(sp, 10);
  // Each candidate pair once, spread over the lanes: position p lists its pairs (as vehicle
  // indices a < b) at its exclusive prefix offset, then lane t takes pair t (64 per round).
  // Per vehicle, upstream keeps the impact of its highest-index partner (the last
  // handle_collisions call that writes it) and ORs the crash flag; the translation therefore
  // goes through a 64-bit LDS max keyed by (partner + 1) in the high word.
  const int cnt = run;
  int off = wave_incl_scan(cnt);
  const int total = rdli(off, WAVE - 1);
  off -= cnt;
  cl.imx[lane] = 0ull;
  cl.imy[lane] = 0ull;
  cl.crash[lane] = 0;
  cl.pord[lane] = ro.ord;
  wave_lds_sync();
  // (a loop over o = 1 .. run measured the same time with more VALU, round 5)
  uint64_t om = (2ull << run) - 2ull;  // bits 1 .. run (run <= 63)
  while (om) {
    const int o = __builtin_ctzll(om);
    om &= om - 1ull;
    const int q = cl.pord[lane + o];
    const int lo = ro.ord < q ? ro.ord : q, hi = ro.ord < q ? q : ro.ord;
    cl.plist[off++] = (uint16_t)((lo << 8) | hi);
  }
  wave_lds_sync();
  for (int base = 0; base < ((kSkip & 2) ? 0 : total); base += WAVE) {
    const bool has = base + lane < total;
    const int pr = has ? cl.plist[base + lane] : 0;
    const int a = pr >> 8, b = pr & 0xff;  // a < b
    const float xa = shf(v.x, a), ya = shf(v.y, a), ca = shf(c2, a), sa = shf(s2, a),
                va = shf(v.spd, a);
    const float xb = shf(v.x, b), yb = shf(v.y, b), cb = shf(c2, b), sb = shf(s2, b),
                vb = shf(v.spd, b);
    // exact pre-check (are_polygons_intersecting is only called inside it), then the SAT test
    const float dx = xb - xa, dy = yb - ya;
    // upstream's sqrt(dx^2 + dy^2) > B, decided from the squares where they are 2^-19 apart (a
    // margin far above the roundings of B^2 and of the thresholds: the correctly rounded root
    // lies on the same side of B); a lane near the boundary, with B outside [1e-10, 2^60) or a
    // non-finite square, takes the root itself
    const float q2 = hm_fma(dx, dx, dy * dy);
    const float bb = (VEH_DIAGONAL + VEH_DIAGONAL) / 2.0f + va * dt;
    const float b2 = bb * bb;
    const uint64_t bokm = ballot(bb >= 1.0e-10f) & ballot(bb < 0x1p60f);
    const bool gt = q2 > b2 * (1.0f + 0x1p-19f), lt = q2 < b2 * (1.0f - 0x1p-19f);
    bool far = gt;
    uint64_t farm = ballot(gt);  // ballot(far), from the compare's own mask on the usual path
    if (~(bokm & (farm | ballot(lt)))) {  // some lane undecided (rare): its root
      const bool sure = (bb >= 1.0e-10f && bb < 0x1p60f) && (gt || lt);
      far = sure ? gt : __builtin_sqrtf(q2) > bb;
      farm = ballot(far);
    }
    bool pass = has && !far;
    uint64_t passm = ballot(lane < total - base) & ~farm;  // ballot(pass)
    if (!passm) continue;
    const float dax = (va * ca) * dt, day = (va * sa) * dt, dbx = (vb * cb) * dt, dby = (vb * sb) * dt;
    // a's v axis (the SAT's second edge normal) first: a pair separated on it both as it stands
    // and swept by the velocities ends with intersecting = will_intersect = false and no
    // translation whatever the other axes give (the SAT only ever clears the two flags), so it
    // leaves the round; rounds whose pairs all leave skip the SAT (cars side by side in adjacent
    // lanes).  The same operations as sat_collide's edge 1, so the decision is exact.
    {
      float a0, a1, b0, b1;
      rect_interval(xa, ya, ca, sa, -sa, ca, a0, a1);
      rect_interval(xb, yb, cb, sb, -sa, ca, b0, b1);
      const float vp = hm_fma(-sa, dax - dbx, ca * (day - dby));
      const bool sep0 = interval_distance(a0, a1, b0, b1) > 0.0f;
      const bool sep1 = interval_distance(vp < 0.0f ? a0 + vp : a0, vp < 0.0f ? a1 : a1 + vp, b0,
                                          b1) > 0.0f;
      pass = pass && !(sep0 && sep1);
      passm &= ~(ballot(sep0) & ballot(sep1));
      if (!passm) continue;
    }
    bool inter, will;
    float tx, ty;
    sat_collide(passm, xa, ya, ca, sa, dax, day, xb, yb, cb, sb, dbx, dby, &inter, &will, &tx, &ty);
    if (pass && will) {
      atomicMax(&cl.imx[a], ((uint64_t)(b + 1) << 32) | hm_f2bits(tx / 2.0f));
      atomicMax(&cl.imy[a], ((uint64_t)(b + 1) << 32) | hm_f2bits(ty / 2.0f));
      atomicMax(&cl.imx[b], ((uint64_t)(a + 1) << 32) | hm_f2bits(-tx / 2.0f));
      atomicMax(&cl.imy[b], ((uint64_t)(a + 1) << 32) | hm_f2bits(-ty / 2.0f));
    }
    if (pass && inter) {
      cl.crash[a] = 1;
      cl.crash[b] = 1;
    }
  }
  wave_lds_sync();
  const uint64_t mx = cl.imx[lane], my = cl.imy[lane];
  if (mx != 0ull) {
    v.ix = hm_bits2f((uint32_t)mx);
    v.iy = hm_bits2f((uint32_t)my);
    v.imp = true;
  }
  if (cl.crash[lane]) v.crashed = true;
  wave_lds_sync();  // the lists are rewritten next frame
  SEC(sp, 8);
}

// ------------------------------------------------------------------------- kernels
// W: waves per SIMD the registers are sized for.  4 (106 VGPRs) when the envs fit one wave per
// env on 4 waves per SIMD (4,096 envs on 256 CUs: 0.160 ms); 6 (80 VGPRs, 14 spilled to scratch
// outside the hot loop) when more envs queue behind them: 16,384 envs 0.412 -> 0.365 ms,
// 32,768 0.775 -> 0.670 (5 waves: 0.381 / 0.702), 8,192 0.228 -> 0.220; at 4,096 envs the 6-wave
// build takes 0.164 ms, so hwy_launch_step picks by env count (round 6, launch parameters from a
// table: the 4-wave build also wins at 8,192 envs, so the 6-wave one starts above 32 envs per CU)
// The step of one handle's envs; the kernels below run it for one handle (hwy_step) or for
// handle blockIdx.y of a table (hwy_step_group: a sweep's cells in one launch).  It reads no
// gridDim and no blockIdx.y, so a grouped launch computes every env exactly as its handle's own.
template <int W>
__device__ __forceinline__ void step_body(const StepParams& P) {
  __shared__ int lds_vor[ENVS_PER_BLOCK][WAVE];
  __shared__ int lds_inv[ENVS_PER_BLOCK][WAVE];
  __shared__ CollLds lds_coll[ENVS_PER_BLOCK];
  const hwy_config& C = P.cfg;
  const int lane = threadIdx.x & (WAVE - 1);
  const int w = threadIdx.x / WAVE;
  const int e = blockIdx.x * ENVS_PER_BLOCK + w;
  if (e >= C.num_envs) return;  // whole wave
  const int V = C.vehicles_count + 1;
  const size_t fstride = (size_t)C.num_envs * WAVE;
  const uint32_t idx = (uint32_t)e * WAVE + lane;  // < 2^32: hwy_create bounds num_envs
  uint32_t* st = P.state;

  SecProf sp;
  SEC_START(sp);
  WAVE_T(e, lane, 0, __builtin_amdgcn_s_memtime());
  WAVE_T(e, lane, 3, __builtin_amdgcn_s_memrealtime());
  Veh v;
  int order_pos;
  load_veh(st, fstride, idx, lane, V, v, order_pos);
  const uint32_t ew = (st + HWY_F_ENV * fstride)[idx];
  int step = rdli((int)ew, HWY_E_STEP);
  int episode = rdli((int)ew, HWY_E_EPISODE);
  uint64_t seed = (uint64_t)(uint32_t)rdli((int)ew, HWY_E_SEED_LO) |
                  ((uint64_t)(uint32_t)rdli((int)ew, HWY_E_SEED_HI) << 32);
  float ep_return = hm_bits2f((uint32_t)rdli((int)ew, HWY_E_RETURN));
  if (lane == 0) {
    v.aacc = hm_bits2f((uint32_t)rdli((int)ew, HWY_E_EGO_ACC));
    v.asteer = hm_bits2f((uint32_t)rdli((int)ew, HWY_E_EGO_STEER));
  }

  const float dt = 1.0f / (float)C.sim_freq;
  const int frames = C.sim_freq / C.policy_freq;
  const float a0 = P.actions[2 * (size_t)e], a1 = P.actions[2 * (size_t)e + 1];
  // the road order of the stored positions, kept from the previous step (flags bits 8-13; the
  // absent lanes follow the present ones by descending index), validated -- and repaired or
  // rebuilt when the state was written by someone else -- before frame 0 uses it
  RoadOrder ro;
  ro.rk = lane < V ? order_pos : V + (WAVE - 1 - lane);
  ro.ord = __builtin_amdgcn_ds_permute(ro.rk << 2, lane);
  ro.valid = true;
  const uint64_t pres = ballot(v.present);
  road_order(lane, v, pres, ro);
  float cos_h, sin_h;
  hm_sincosf(v.h, &sin_h, &cos_h);
  SEC(sp, 15);
  if (frames > 0 && lane == 0) {  // ContinuousAction.act (first frame)
    v.aacc = hm_lmap(hm_clipf(a0, -1.0f, 1.0f), -1.0f, 1.0f, -5.0f, 5.0f);
    v.asteer = hm_lmap(hm_clipf(a1, -1.0f, 1.0f), -1.0f, 1.0f, -HM_PIO4_F, HM_PIO4_F);
  }
  // the ego's steering changes only here and to 0 on a crash (handled in frame_wave)
  const float tan_ego = rdlf(lane == 0 ? hm_tanf_sc(v.asteer) : 0.0f, 0);
  // Issue priority falls with progress through the frames (s_setprio 3, 2, 1, 0 from 6/15, 10/15
  // and 13/15 of them): the SIMD's arbiter otherwise prefers its oldest wave, so a SIMD's four
  // waves finished one after another and the last ran its final frames alone, with no other
  // wave to hide its latency.  Lagging waves now catch up and the four finish together (the
  // launch ends with the slowest SIMD).  Scheduling only: the same instructions and results.
  for (int frame = 0; frame < frames; ++frame) {
    const int f15 = 15 * frame;
    if (f15 < 6 * frames) __builtin_amdgcn_s_setprio(3);
    else if (f15 < 10 * frames) __builtin_amdgcn_s_setprio(2);
    else if (f15 < 13 * frames) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
    frame_wave(C, lane, v, dt, tan_ego, ro, cos_h, sin_h, lds_coll[w], sp, pres);
  }
  __builtin_amdgcn_s_setprio(0);  // the reward, observation and stores at the lowest priority
  step += 1;
  SEC(sp, 16);

  // HighwayEnv._reward / _is_terminated / _is_truncated on the ego (lane 0)
  float rew = 0.0f;
  int terminated = 0;
  if (lane == 0) {
    const float forward_speed = v.spd * cos_h;  // hm_cosf(v.h), carried from the last frame
    const float scaled_speed = hm_lmap(forward_speed, C.reward_speed_range[0],
                                       C.reward_speed_range[1], 0.0f, 1.0f);
    const float collision = v.crashed ? 1.0f : 0.0f;
    const int nl = C.lanes_count - 1;
    const float right_lane = (float)v.ln / (float)(nl > 1 ? nl : 1);
    const float high_speed = hm_clipf(scaled_speed, 0.0f, 1.0f);
    const bool on_road = on_lane_m(v.x, v.y, v.ln, 0.0f);
    const float on_road_f = on_road ? 1.0f : 0.0f;
    rew = 0.0f;
    rew = rew + C.collision_reward * collision;
    rew = rew + C.right_lane_reward * right_lane;
    rew = rew + C.high_speed_reward * high_speed;
    rew = rew + C.on_road_reward * on_road_f;
    if (C.normalize_reward)
      rew = hm_lmap(rew, C.collision_reward, C.high_speed_reward + C.right_lane_reward, 0.0f, 1.0f);
    rew = rew * on_road_f;
    terminated = v.crashed || (C.offroad_terminal && !on_road);
  }
  rew = rdlf(rew, 0);
  terminated = rdli(terminated, 0);
  const int truncated = step >= C.max_steps;
  ep_return = ep_return + rew;
  const bool done = terminated || truncated;
  if (lane == 0) {
    P.reward[e] = rew;
    P.term[e] = (uint8_t)terminated;
    P.trunc[e] = (uint8_t)truncated;
    if (P.ep_ret) P.ep_ret[e] = done ? ep_return : 0.0f;
    if (P.ep_len) P.ep_len[e] = done ? step : 0;
  }
  SEC(sp, 11);
  if (done && C.autoreset) {
    episode += 1;
    seed = episode_seed(P, e, episode);
    reset_wave(C, lane, seed, v);
    step = 0;
    ep_return = 0.0f;
    ro.rk = reset_order_pos(lane, V);
    cos_h = 1.0f;  // hm_cosf / hm_sinf of the reset heading 0, exactly
    sin_h = 0.0f;
  }
  SEC(sp, 12);
  observe_wave(C, lane, v, cos_h, sin_h, step, seed, group_pe_table(P, e),
               P.obs + (size_t)e * C.obs_vehicles * P.fout, P.fout, lds_vor[w], lds_inv[w],
               lds_coll[w].imx);  // the collision pass's scratch is free after the frames
  SEC(sp, 13);
  store_veh(st, fstride, idx, lane, V, v, ro.rk);
  SEC(sp, 17);
  store_env_words(st, fstride, idx, lane, step, episode, seed, rdlf(v.aacc, 0), rdlf(v.asteer, 0),
                  ep_return);
  SEC(sp, 14);
  WAVE_T(e, lane, 1, __builtin_amdgcn_s_memtime());
  WAVE_T(e, lane, 4, __builtin_amdgcn_s_memrealtime());
  WAVE_T(e, lane, 2, (unsigned long long)done | WAVE_HWID());
  SEC_FLUSH(sp, lane, e);
}

template <int W>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(W, 8)))
hwy_step_kernel(StepParams P) {
  step_body<W>(P);
}

// handle blockIdx.y of tab; blocks past a handle's envs exit in step_body (whole waves).  The
// profiling builds' per-env clocks and section counters index by env within the handle.
template <int W>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(W, 8)))
hwy_step_grp_kernel(const StepParams* __restrict__ tab) {
  step_body<W>(tab[blockIdx.y]);
}

__global__ void __launch_bounds__(256) hwy_reset_kernel(StepParams P) {
  __shared__ int lds_vor[ENVS_PER_BLOCK][WAVE];
  __shared__ int lds_inv[ENVS_PER_BLOCK][WAVE];
  __shared__ unsigned long long lds_key[ENVS_PER_BLOCK][WAVE];
  const hwy_config& C = P.cfg;
  const int lane = threadIdx.x & (WAVE - 1);
  const int w = threadIdx.x / WAVE;
  const int e = blockIdx.x * ENVS_PER_BLOCK + w;
  if (e >= C.num_envs) return;
  if (P.mask && !P.mask[e]) return;
  const int V = C.vehicles_count + 1;
  const size_t fstride = (size_t)C.num_envs * WAVE;
  const uint32_t idx = (uint32_t)e * WAVE + lane;  // < 2^32: hwy_create bounds num_envs
  const uint64_t seed = P.seeds ? P.seeds[e] : episode_seed(P, e, 0);
  Veh v;
  reset_wave(C, lane, seed, v);
  if (P.obs)
    observe_wave(C, lane, v, 1.0f, 0.0f, 0, seed, group_pe_table(P, e),
                 P.obs + (size_t)e * C.obs_vehicles * P.fout, P.fout, lds_vor[w], lds_inv[w],
                 lds_key[w]);
  store_veh(P.state, fstride, idx, lane, V, v, reset_order_pos(lane, V));
  store_env_words(P.state, fstride, idx, lane, 0, 0, seed, 0.0f, 0.0f, 0.0f);
}

// Stand-alone wrapper on [E,N,F]: one thread per (env, row).
__global__ void __launch_bounds__(256) hwy_obs_pe_kernel(const float* __restrict__ in,
                                                         float* __restrict__ out, int E, int N,
                                                         int F, int kind, int d, int ego_idx,
                                                         float max_dist, const float* table,
                                                         const float* dist_override) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long)E * N) return;
  const long e = t / N;
  const int r = (int)(t - e * N);
  const int Fo = F + ((kind == HWY_PE_RANK || kind == HWY_PE_DIST || kind == HWY_PE_DIST1) ? d : 0);
  float vals[HWY_MAX_FEATURES];
#pragma unroll
  for (int f = 0; f < HWY_MAX_FEATURES; ++f) vals[f] = f < F ? in[t * F + f] : 0.0f;
  const float* eg = in + (e * N + ego_idx) * F;
  const float ex0 = eg[0], ex1 = F > 1 ? eg[1] : 0.0f;
  write_pe_row(vals, F, kind, d, r, ex0, ex1, max_dist, table, dist_override != nullptr,
               dist_override ? dist_override[t] : 0.0f, out + t * Fo);
}

// PPOMemory.compute_advantages on [T,E]: one thread per env, reversed scan over t.
__global__ void __launch_bounds__(64) hwy_gae_kernel(const float* __restrict__ rew,
                                                      const uint8_t* __restrict__ done,
                                                      const float* __restrict__ val,
                                                      const float* __restrict__ last_val,
                                                      double gamma, double lam, int T, int E,
                                                      float* __restrict__ adv,
                                                      float* __restrict__ ret) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  const double gl = gamma * lam;
  float last_adv = 0.0f;
  double v1 = (double)last_val[e];
  // the recurrence is sequential per env (each step rounds to float, as the reference's float
  // tensors do), but its inputs are not: kGaeAhead steps' rewards, values and dones are loaded
  // before they are used, so one memory round trip serves kGaeAhead steps instead of one
  constexpr int kGaeAhead = 8;
  for (int t1 = T; t1 > 0; t1 -= kGaeAhead) {
    float rv[kGaeAhead], vv[kGaeAhead];
    uint8_t dv[kGaeAhead];
#pragma unroll
    for (int j = 0; j < kGaeAhead; ++j) {
      const int t = t1 - 1 - j;
      const size_t i = (size_t)(t < 0 ? 0 : t) * E + e;
      rv[j] = rew[i], vv[j] = val[i], dv[j] = done[i];
    }
#pragma unroll
    for (int j = 0; j < kGaeAhead; ++j) {
      const int t = t1 - 1 - j;
      if (t < 0) break;
      const size_t i = (size_t)t * E + e;
      const float v0f = vv[j];
      const double nd = dv[j] ? 0.0 : 1.0;
      const double delta = ((double)rv[j] + (gamma * v1) * nd) - (double)v0f;
      const float a = (float)(delta + (gl * nd) * (double)last_adv);
      adv[i] = a;
      ret[i] = a + v0f;
      last_adv = a;
      v1 = (double)v0f;
    }
  }
}

__global__ void hwy_math_kernel(int op, const float* in, const float* in2, float* out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float x = in[i], y = in2 ? in2[i] : 0.0f;
  float r = 0.0f;
  switch (op) {
    case 0: r = hm_sinf(x); break;
    case 1: r = hm_cosf(x); break;
    case 2: r = hm_tanf(x); break;
    case 3: r = hm_atanf(x); break;
    case 4: r = hm_asinf(x); break;
    case 5: r = hm_expf(x); break;
    case 6: r = hm_logf(x); break;
    case 7: r = hm_powf(x, y); break;
    case 8: r = hm_wrap_to_pi(x); break;
    case 9: r = __builtin_sqrtf(x); break;
    case 10: r = x / y; break;
    case 11: r = hm_floorf(x); break;
    case 12: { float c_; hm_sincosf(x, &r, &c_); } break;
    case 13: { float s_; hm_sincosf(x, &s_, &r); } break;
    case 14: r = hm_tanf_sc(x); break;
    case 15: r = hm_powf_idm(x, y); break;
    case 16: r = (float)closest_lane(x, (int)y); break;  // y: lanes_count
  }
  out[i] = r;
}

// ------------------------------------------------------------------------- launch helpers
extern "C" {
// compute units of the current device (cached per device; 256 without one)
// waves per SIMD the step kernel's registers are sized for at large E (5 and 8 measured slower)
#ifndef HWY_STEP_BIG_W
#define HWY_STEP_BIG_W 6
#endif
// envs per CU above which the big build runs: at 8,192 envs (32 per CU) the 4-wave build is
// 6-7 % faster than the 6-wave one (0.205 vs 0.219-0.245 ms per step), at 16,384 the 6-wave build
// wins (0.295 vs 0.324) and at 32,768 ties the 5-wave one (profiles/r6/micro/ab_bigw.log)
#ifndef HWY_STEP_BIG_WAVES
#define HWY_STEP_BIG_WAVES 32
#endif
constexpr int kStepBigW = HWY_STEP_BIG_W;
static int device_cus() {
  static int cache[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) {
    (void)hipGetLastError();
    return 256;
  }
  if (!cache[dev]) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus < 1)
      cus = 256;
    (void)hipGetLastError();
    cache[dev] = cus;
  }
  return cache[dev];
}

int hwy_launch_step(const StepParams* p, hipStream_t s) {
  const int blocks = (p->cfg.num_envs + ENVS_PER_BLOCK - 1) / ENVS_PER_BLOCK;
  // one wave per env: more than 4 waves per SIMD of envs queue behind the first four
  if (hwy_step_big(p->cfg.num_envs))
    hipLaunchKernelGGL(hwy_step_kernel<kStepBigW>, dim3(blocks), dim3(ENVS_PER_BLOCK * WAVE), 0, s, *p);
  else
    hipLaunchKernelGGL(hwy_step_kernel<4>, dim3(blocks), dim3(ENVS_PER_BLOCK * WAVE), 0, s, *p);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
int hwy_launch_step_group(const StepParams* dtab, int n, int blocks, int big, hipStream_t s) {
  if (big)
    hipLaunchKernelGGL(hwy_step_grp_kernel<kStepBigW>, dim3(blocks, n), dim3(ENVS_PER_BLOCK * WAVE),
                       0, s, dtab);
  else
    hipLaunchKernelGGL(hwy_step_grp_kernel<4>, dim3(blocks, n), dim3(ENVS_PER_BLOCK * WAVE), 0, s,
                       dtab);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
int hwy_step_blocks(int num_envs) { return (num_envs + ENVS_PER_BLOCK - 1) / ENVS_PER_BLOCK; }
int hwy_step_big(int64_t total_envs) {
  return total_envs > (int64_t)HWY_STEP_BIG_WAVES * device_cus() ? 1 : 0;
}
int hwy_launch_reset(const StepParams* p, hipStream_t s) {
  const int blocks = (p->cfg.num_envs + ENVS_PER_BLOCK - 1) / ENVS_PER_BLOCK;
  hipLaunchKernelGGL(hwy_reset_kernel, dim3(blocks), dim3(ENVS_PER_BLOCK * WAVE), 0, s, *p);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
int hwy_launch_obs_pe(const float* in, float* out, int E, int N, int F, int kind, int d, int ego,
                      float max_dist, const float* table, const float* dov, hipStream_t s) {
  const long n = (long)E * N;
  if (n == 0) return 0;
  const int blocks = (int)((n + 255) / 256);
  hipLaunchKernelGGL(hwy_obs_pe_kernel, dim3(blocks), dim3(256), 0, s, in, out, E, N, F, kind, d,
                     ego, max_dist, table, dov);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
int hwy_launch_gae(const float* rew, const uint8_t* done, const float* val, const float* last_val,
                   double gamma, double lam, int T, int E, float* adv, float* ret, hipStream_t s) {
  if (E == 0) return 0;
  // one wave per workgroup: 4,096 envs spread over 64 CUs instead of 16
  const int blocks = (E + 63) / 64;
  hipLaunchKernelGGL(hwy_gae_kernel, dim3(blocks), dim3(64), 0, s, rew, done, val, last_val,
                     gamma, lam, T, E, adv, ret);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
int hwy_launch_math(int op, const float* in, const float* in2, float* out, int n, hipStream_t s) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(hwy_math_kernel, dim3((n + 255) / 256), dim3(256), 0, s, op, in, in2, out, n);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
}

#if defined(HWY_SECTION_PROFILE) || defined(HWY_WAVE_TIMES)
extern "C" int hwy_debug_wave_times(unsigned long long* out, int n) {
  if (n > 5 * HWY_NWT) n = 5 * HWY_NWT;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_hwy_wave_t), sizeof(unsigned long long) * n) ==
                 hipSuccess ? 0 : -2;
}
#endif
#ifdef HWY_SECTION_PROFILE
// development build only: copy out (and optionally clear) the section clock totals
// development build only: the per-env totals themselves ([n][HWY_NSEC], n <= HWY_NSEC_ENVS)
extern "C" int hwy_debug_sections_env(unsigned long long* out, int n) {
  if (!out || n < 0) return -1;
  if (n > HWY_NSEC_ENVS) n = HWY_NSEC_ENVS;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_hwy_sections),
                             sizeof(unsigned long long) * HWY_NSEC * n) == hipSuccess ? 0 : -2;
}
extern "C" int hwy_debug_sections(unsigned long long* out, int reset) {
  static unsigned long long h[HWY_NSEC_ENVS][HWY_NSEC];
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_hwy_sections), sizeof(h)) != hipSuccess) return -2;
  for (int i = 0; i < HWY_NSEC; ++i) out[i] = 0;
  for (int e = 0; e < HWY_NSEC_ENVS; ++e)
    for (int i = 0; i < HWY_NSEC; ++i) out[i] += h[e][i];
  if (reset) {
    void* p = nullptr;
    if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_hwy_sections)) != hipSuccess) return -2;
    if (hipMemset(p, 0, sizeof(h)) != hipSuccess || hipDeviceSynchronize() != hipSuccess) return -2;
  }
  return 0;
}
#endif
