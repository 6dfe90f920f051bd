/*
 * hwy_math.h -- deterministic binary32 math shared by the gfx950 kernels and the host.
 *
 * Why: the highway step is chaotic (MOBIL thresholds, collision tests), so GPU/CPU parity is
 * only meaningful if both sides round identically. libm (glibc) and the device library (ocml)
 * differ in the last ulp of sin/atan/pow, so both sides use these routines instead. They use
 * only IEEE-754 correctly rounded operations (+ - * / sqrt, fma, floor, int<->float), so with
 * -ffp-contract=off they produce the same bits on x86-64 (SSE) and on gfx950.  Fused
 * multiply-adds are explicit (hm_fma: v_fma_f32 on gfx950, the correctly rounded fmaf on the
 * host), never left to the compiler's contraction, so both sides fuse the same operations.
 * Polynomials are the classic Cephes single-precision ones (S. Moshier, public domain),
 * accurate to ~1-3 ulp on the ranges used; tests/test_math.py checks them against libm double.
 *
 * Usable from C (gcc) and HIP C++ (hipcc): HWY_HD expands to __host__ __device__ under HIP.
 */
#ifndef HWY_MATH_H_
#define HWY_MATH_H_

#include <stdint.h>

#if defined(__HIPCC__)
#define HWY_HD __host__ __device__ static inline
#else
#define HWY_HD static inline
#endif

#define HM_PI_F 3.14159265358979323846f
#define HM_PIO2_F 1.5707963267948966192f
#define HM_PIO4_F 0.7853981633974483096f
#define HM_TWO_PI_F 6.28318530717958647692f

HWY_HD float hm_bits2f(uint32_t u) {
  union { uint32_t u; float f; } c;
  c.u = u;
  return c.f;
}
HWY_HD uint32_t hm_f2bits(float f) {
  union { uint32_t u; float f; } c;
  c.f = f;
  return c.u;
}

HWY_HD float hm_absf(float x) { return hm_bits2f(hm_f2bits(x) & 0x7fffffffu); }
/* a * b + c with one rounding (IEEE fusedMultiplyAdd) */
HWY_HD float hm_fma(float a, float b, float c) { return __builtin_fmaf(a, b, c); }
HWY_HD int hm_isnan(float x) { return x != x; }

/* numpy.clip semantics for scalars: NaN propagates. */
HWY_HD float hm_clipf(float x, float lo, float hi) { return x < lo ? lo : (x > hi ? hi : x); }
HWY_HD float hm_minf(float a, float b) { return (b < a) ? b : a; } /* min(a,b) python */
HWY_HD float hm_maxf(float a, float b) { return (b > a) ? b : a; } /* max(a,b) python */

/* floor for |x| < 2^31 without libm (exact) */
HWY_HD float hm_floorf(float x) {
  if (!(hm_absf(x) < 8388608.0f)) return x; /* already integral, inf or nan */
  float t = (float)(int32_t)x;              /* truncation, exact */
  return (t > x) ? t - 1.0f : t;
}

/* x * 2^n, n in [-300, 300] */
HWY_HD float hm_ldexpf(float x, int n) {
  if (n > 127) {
    x *= hm_bits2f(0x7f000000u); /* 2^127 */
    n -= 127;
    if (n > 127) n = 127;
  }
  if (n < -126) {
    x *= hm_bits2f(0x00800000u); /* 2^-126 */
    n += 126;
    if (n < -126) {
      x *= hm_bits2f(0x00800000u);
      n += 126;
      if (n < -126) n = -126;
    }
  }
  return x * hm_bits2f((uint32_t)(n + 127) << 23);
}

/* x = m * 2^e with m in [0.5, 1); x finite > 0 */
HWY_HD float hm_frexpf(float x, int* e) {
  uint32_t u = hm_f2bits(x);
  int ex = (int)((u >> 23) & 0xffu);
  int adj = 0;
  if (ex == 0) { /* subnormal: scale by 2^25 */
    x *= 33554432.0f;
    u = hm_f2bits(x);
    ex = (int)((u >> 23) & 0xffu);
    adj = -25;
  }
  *e = ex - 126 + adj;
  return hm_bits2f((u & 0x807fffffu) | 0x3f000000u);
}

/* Cephes sinf/cosf core: returns sin (want_cos = 0) or cos (want_cos = 1). */
HWY_HD float hm_sincos_core(float xx, int want_cos) {
  const float FOPI = 1.27323954473516f;
  const float DP1 = 0.78515625f;
  const float DP2 = 2.4187564849853515625e-4f;
  const float DP3 = 3.77489497744594108e-8f;
  float x = xx;
  int sign = 1;
  if (x < 0.0f) {
    x = -x;
    if (!want_cos) sign = -1;
  }
  /* |x| >= 2^24: total loss of precision, Cephes returns 0; x - x keeps that for finite x and
   * gives NaN for inf and NaN, as libm / numpy do */
  if (!(x <= 16777215.0f)) return x - x;
  uint32_t j = (uint32_t)(FOPI * x);
  float y = (float)j;
  if (j & 1u) {
    j += 1u;
    y += 1.0f;
  }
  j &= 7u;
  if (j > 3u) {
    sign = -sign;
    j -= 4u;
  }
  if (want_cos && j > 1u) sign = -sign;
  x = hm_fma(-y, DP3, hm_fma(-y, DP2, hm_fma(-y, DP1, x)));
  float z = x * x;
  int use_cos_poly = want_cos ? !(j == 1u || j == 2u) : (j == 1u || j == 2u);
  float r;
  if (use_cos_poly) {
    r = hm_fma(hm_fma(2.443315711809948E-005f, z, -1.388731625493765E-003f), z,
               4.166664568298827E-002f);
    r = hm_fma(r, z * z, hm_fma(-0.5f, z, 1.0f));
  } else {
    r = hm_fma(hm_fma(-1.9515295891E-4f, z, 8.3321608736E-3f), z, -1.6666654611E-1f);
    r = hm_fma(r, z * x, x);
  }
  return sign < 0 ? -r : r;
}
HWY_HD float hm_sinf(float x) { return hm_sincos_core(x, 0); }
HWY_HD float hm_cosf(float x) { return hm_sincos_core(x, 1); }
HWY_HD float hm_tanf(float x) { return hm_sinf(x) / hm_cosf(x); }

/* hm_sinf(x) and hm_cosf(x) from one range reduction (bit-identical to the two calls). */
HWY_HD void hm_sincosf(float xx, float* s_out, float* c_out) {
  const float FOPI = 1.27323954473516f;
  const float DP1 = 0.78515625f;
  const float DP2 = 2.4187564849853515625e-4f;
  const float DP3 = 3.77489497744594108e-8f;
  float x = xx;
  int sign_s = 1, sign_c = 1;
  if (x < 0.0f) {
    x = -x;
    sign_s = -1;
  }
  if (!(x <= 16777215.0f)) {
    const float r = x - x; /* as hm_sincos_core */
    *s_out = r;
    *c_out = r;
    return;
  }
  uint32_t j = (uint32_t)(FOPI * x);
  float y = (float)j;
  if (j & 1u) {
    j += 1u;
    y += 1.0f;
  }
  j &= 7u;
  if (j > 3u) {
    sign_s = -sign_s;
    sign_c = -sign_c;
    j -= 4u;
  }
  if (j > 1u) sign_c = -sign_c;
  x = hm_fma(-y, DP3, hm_fma(-y, DP2, hm_fma(-y, DP1, x)));
  const float z = x * x;
  float rc = hm_fma(hm_fma(2.443315711809948E-005f, z, -1.388731625493765E-003f), z,
                    4.166664568298827E-002f);
  rc = hm_fma(rc, z * z, hm_fma(-0.5f, z, 1.0f));
  float rs = hm_fma(hm_fma(-1.9515295891E-4f, z, 8.3321608736E-3f), z, -1.6666654611E-1f);
  rs = hm_fma(rs, z * x, x);
  const int swap = (j == 1u || j == 2u);
  const float s = swap ? rc : rs, c = swap ? rs : rc;
  *s_out = sign_s < 0 ? -s : s;
  *c_out = sign_c < 0 ? -c : c;
}
HWY_HD float hm_tanf_sc(float x) {
  float s, c;
  hm_sincosf(x, &s, &c);
  return s / c;
}

/* Cephes atanf */
HWY_HD float hm_atanf(float xx) {
  float x = xx, y;
  int sign = 1;
  if (xx < 0.0f) {
    sign = -1;
    x = -xx;
  }
  if (x > 2.414213562373095f) {
    y = HM_PIO2_F;
    x = -(1.0f / x);
  } else if (x > 0.4142135623730950f) {
    y = HM_PIO4_F;
    x = (x - 1.0f) / (x + 1.0f);
  } else {
    y = 0.0f;
  }
  float z = x * x;
  float p = hm_fma(hm_fma(hm_fma(8.05374449538e-2f, z, -1.38776856032E-1f), z,
                          1.99777106478E-1f), z, -3.33329491539E-1f);
  y = y + hm_fma(p * z, x, x);
  return sign < 0 ? -y : y;
}

/* Cephes asinf; caller clips to [-1, 1] (np.arcsin(np.clip(...)) in the reference). */
HWY_HD float hm_asinf(float xx) {
  float a, x = xx, z;
  int sign, flag;
  if (x > 0.0f) {
    sign = 1;
    a = x;
  } else {
    sign = -1;
    a = -x;
  }
  if (a > 1.0f) return 0.0f / 0.0f;
  if (a < 1.0e-4f) {
    z = a;
  } else {
    if (a > 0.5f) {
      z = 0.5f * (1.0f - a);
      x = __builtin_sqrtf(z);
      flag = 1;
    } else {
      x = a;
      z = x * x;
      flag = 0;
    }
    float p = hm_fma(hm_fma(hm_fma(hm_fma(4.2163199048E-2f, z, 2.4181311049E-2f), z,
                                      4.5470025998E-2f), z, 7.4953002686E-2f), z,
                     1.6666752422E-1f);
    z = hm_fma(p * z, x, x);
    if (flag) {
      z = z + z;
      z = HM_PIO2_F - z;
    }
  }
  return sign < 0 ? -z : z;
}

/* Cephes expf */
HWY_HD float hm_expf(float xx) {
  float x = xx;
  if (hm_isnan(x)) return x;
  if (x > 88.72283905206835f) return hm_bits2f(0x7f800000u);
  if (x < -103.278929903431851103f) return 0.0f;
  float z = hm_floorf(hm_fma(1.44269504088896341f, x, 0.5f));
  x = hm_fma(-z, 0.693359375f, x);
  x = hm_fma(z, 2.12194440e-4f, x);
  int n = (int)z;
  z = x * x;
  float p = hm_fma(hm_fma(1.9875691500E-4f, x, 1.3981999507E-3f), x, 8.3334519073E-3f);
  p = hm_fma(hm_fma(hm_fma(p, x, 4.1665795894E-2f), x, 1.6666665459E-1f), x,
             5.0000001201E-1f);
  p = hm_fma(p, z, x) + 1.0f;
  return hm_ldexpf(p, n);
}

/* Cephes logf (x > 0 finite; 0 -> -inf; <0 -> nan) */
HWY_HD float hm_logf(float xx) {
  float x = xx;
  if (hm_isnan(x)) return x;
  if (x <= 0.0f) return x == 0.0f ? hm_bits2f(0xff800000u) : 0.0f / 0.0f;
  if (x == hm_bits2f(0x7f800000u)) return x;
  int e;
  x = hm_frexpf(x, &e);
  if (x < 0.707106781186547524f) {
    e -= 1;
    x = (x + x) - 1.0f;
  } else {
    x = x - 1.0f;
  }
  float z = x * x;
  float y = hm_fma(hm_fma(hm_fma(7.0376836292E-2f, x, -1.1514610310E-1f), x, 1.1676998740E-1f),
                   x, -1.2420140846E-1f);
  y = hm_fma(hm_fma(hm_fma(y, x, 1.4249322787E-1f), x, -1.6668057665E-1f), x, 2.0000714765E-1f);
  y = hm_fma(hm_fma(y, x, -2.4999993993E-1f), x, 3.3333331174E-1f);
  y = y * x * z;
  float fe = (float)e;
  if (e) y = hm_fma(-2.12194440e-4f, fe, y);
  y = hm_fma(-0.5f, z, y);
  z = x + y;
  if (e) z = hm_fma(0.693359375f, fe, z);
  return z;
}

/* np.power(b, p) for b >= 0 (IDM: max(v,0)/|v0| ** DELTA) */
HWY_HD float hm_powf(float b, float p) {
  if (b == 0.0f) return p > 0.0f ? 0.0f : (p == 0.0f ? 1.0f : hm_bits2f(0x7f800000u));
  if (b == 1.0f || p == 0.0f) return 1.0f;
  return hm_expf(p * hm_logf(b));
}

/* np.power(b, p) for the IDM free-road term -- b = max(v, 0) / |target speed| (>= 0, or NaN),
 * p = DELTA in [3.5, 4.5] -- as one short branch-free sequence (the general
 * hm_powf costs ~100 VALU and 10 exec-mask branches per call on gfx950, once per vehicle and
 * frame).  exp(p * log b) with Cephes' logf / expf polynomials, but: the mantissa taken in
 * [sqrt(1/2), sqrt(2)) straight from the bits (no frexp, no subnormal path: a subnormal b gives
 * a result below 2^-400, i.e. 0), 2^n built from its bits for n in [-126, 127], and the special
 * cases as selects: b = 0 -> 0, NaN -> NaN, +inf -> +inf, exp overflow (p log b > 88) -> +inf,
 * underflow (< -87) -> 0.  Inside that range every operation is hm_powf's, in its order, so the
 * result is hm_powf's bit for bit for every normal b (tests/test_oracle_golden.py); the IDM's
 * bases (<= 4,000) never reach the ends, where hm_powf would return a subnormal or a finite
 * value above e^88 (3 (1 - b^p) rounds the same either way).  The same operations on the host and
 * on gfx950 (correctly rounded primitives, explicit fma): the oracle and the kernel agree bit for
 * bit. */
/* hm_powf_idm's two halves: log b, then exp(p log b) with its special-case selects on b.  One
 * log serves every exponent applied to the same base (mobil's new follower: its own free-road
 * base under the deciding vehicle's DELTA), and the composition is hm_powf_idm's arithmetic. */
HWY_HD float hm_logf_idm(float b) {
  const uint32_t u = hm_f2bits(b);
  int e = (int)(u >> 23) - 127;
  float m = hm_bits2f((u & 0x007fffffu) | 0x3f800000u); /* [1, 2) */
  const int up = m >= 2.0f * 0.707106781186547524f; /* frexp's mantissa >= hm_logf's threshold */
  m = up ? 0.5f * m : m; /* exact */
  e += up;
  const float x = m - 1.0f; /* exact (Sterbenz), in [-0.293, 0.415) */
  const float z = x * x;
  float y = hm_fma(hm_fma(hm_fma(7.0376836292E-2f, x, -1.1514610310E-1f), x, 1.1676998740E-1f),
                   x, -1.2420140846E-1f);
  y = hm_fma(hm_fma(hm_fma(y, x, 1.4249322787E-1f), x, -1.6668057665E-1f), x, 2.0000714765E-1f);
  y = hm_fma(hm_fma(y, x, -2.4999993993E-1f), x, 3.3333331174E-1f);
  y = y * x * z;
  const float fe = (float)e;
  y = hm_fma(-2.12194440e-4f, fe, y);
  y = hm_fma(-0.5f, z, y);
  return hm_fma(0.693359375f, fe, x + y); /* log b (b > 0 normal) */
}

HWY_HD float hm_expf_idm(float lg, float p, float b) {
  const float t = p * lg;
  const float tc = hm_minf(hm_maxf(t, -87.0f), 88.0f);
  const float w = hm_fma(1.44269504088896341f, tc, 0.5f);
  const float wt = (float)(int32_t)w;
  const float n = (wt > w) ? wt - 1.0f : wt; /* hm_floorf(w), |w| < 2^23: in [-125, 127] */
  float r = hm_fma(-n, 0.693359375f, tc);
  r = hm_fma(n, 2.12194440e-4f, r);
  const float r2 = r * r;
  float q = hm_fma(hm_fma(1.9875691500E-4f, r, 1.3981999507E-3f), r, 8.3334519073E-3f);
  q = hm_fma(hm_fma(hm_fma(q, r, 4.1665795894E-2f), r, 1.6666665459E-1f), r, 5.0000001201E-1f);
  q = hm_fma(q, r2, r) + 1.0f;
  float res = q * hm_bits2f((uint32_t)((int)n + 127) << 23);
  res = t > 88.0f ? hm_bits2f(0x7f800000u) : res;
  res = t < -87.0f ? 0.0f : res;
  res = b == hm_bits2f(0x7f800000u) ? b : res;
  res = b != b ? b : res;
  return b > 0.0f ? res : (b == 0.0f ? 0.0f : res);
}

HWY_HD float hm_powf_idm(float b, float p) { return hm_expf_idm(hm_logf_idm(b), p, b); }

/* utils.wrap_to_pi: ((x + pi) % (2 pi)) - pi with Python's floored modulo.  The quotient is
 * taken with the reciprocal (a possible off-by-one next to a multiple of 2 pi is corrected
 * below). */
HWY_HD float hm_wrap_to_pi(float x) {
  float t = x + HM_PI_F;
  float n = hm_floorf(t * 0.15915494309189535f);
  float r = hm_fma(-n, HM_TWO_PI_F, t);
  if (r < 0.0f) r = r + HM_TWO_PI_F;
  if (r >= HM_TWO_PI_F) r = r - HM_TWO_PI_F;
  return r - HM_PI_F;
}

/* utils.not_zero(x, eps=1e-2) */
HWY_HD float hm_not_zero(float x) {
  if (hm_absf(x) > 1e-2f) return x;
  return x >= 0.0f ? 1e-2f : -1e-2f;
}

/* utils.lmap(v, [x0, x1], [y0, y1]) = y0 + (v - x0) * (y1 - y0) / (x1 - x0) */
HWY_HD float hm_lmap(float v, float x0, float x1, float y0, float y1) {
  return y0 + (v - x0) * (y1 - y0) / (x1 - x0);
}

/* ---------------------------------------------------------------------------------------
 * Philox4x32-10 (Salmon et al., SC'11), counter-based RNG for traffic generation and the
 * "shuffled" row permutation. Verified against the Random123 known-answer vectors.
 * ------------------------------------------------------------------------------------- */
typedef struct hm_u32x4 {
  uint32_t v[4];
} hm_u32x4;

HWY_HD hm_u32x4 hm_philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0,
                                 uint32_t k1) {
  for (int r = 0; r < 10; ++r) {
    if (r > 0) {
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    uint64_t p0 = (uint64_t)0xD2511F53u * (uint64_t)c0;
    uint64_t p1 = (uint64_t)0xCD9E8D57u * (uint64_t)c2;
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    uint32_t n0 = hi1 ^ c1 ^ k0;
    uint32_t n2 = hi0 ^ c3 ^ k1;
    c0 = n0;
    c1 = lo1;
    c2 = n2;
    c3 = lo0;
  }
  hm_u32x4 o;
  o.v[0] = c0;
  o.v[1] = c1;
  o.v[2] = c2;
  o.v[3] = c3;
  return o;
}

/* uniform [0, 1) with 24 random bits (exact in binary32) */
HWY_HD float hm_u01(uint32_t u) { return (float)(u >> 8) * 5.9604644775390625e-8f; }
/* np_random.uniform(lo, hi) */
HWY_HD float hm_uniform(uint32_t u, float lo, float hi) { return lo + (hi - lo) * hm_u01(u); }
/* np_random.choice(n): multiply-shift bounded integer */
HWY_HD int hm_choice(uint32_t u, int n) { return (int)(((uint64_t)u * (uint64_t)n) >> 32); }

#endif /* HWY_MATH_H_ */
