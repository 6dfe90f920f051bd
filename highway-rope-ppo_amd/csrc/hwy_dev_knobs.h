/*
 * hwy_dev_knobs.h -- development-only switches of the env-step kernel (included by
 * hwy_kernels.hip only under -DHWY_DEV_KNOBS; the product library never sees this file).
 *
 * kSkip: timing-only pricing builds (WRONG results) that skip one part of the frame to price its
 * instruction count and time (tools/ab.sh MODE=pmc / MODE=step):
 *   1 MOBIL, 2 the SAT pair loop, 4 collision candidates + SAT, 8 the abort loop, 16 steering,
 *   32 the IDM pow, 64 the observation's rank count.
 */
#ifndef HWY_DEV_KNOBS_H_
#define HWY_DEV_KNOBS_H_
#ifndef HWY_SKIP
#define HWY_SKIP 0
#endif
constexpr int kSkip = HWY_SKIP;
#endif /* HWY_DEV_KNOBS_H_ */
