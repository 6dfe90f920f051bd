// ppo_kernels.hip -- PPO minibatch step and batched acting for gfx950 (include/hwy_ppo.h).
//
// One minibatch step of the reference's PPOAgent.update (ppo/agent.py:216-252).
//
// Fused path (S % 4 == 0, S <= 256, H a multiple of 64 up to 512): four launches, captured per
// epoch in one HIP graph:
//   ppo_rows   16 or 32 minibatch rows per workgroup (rows_tile): forward (h1, h2, [a1|c1]),
//              the loss head (ratio, clipped surrogate, MSE, entropy, their gradients,
//              head-parameter partials), backward data gradients (dh2, dh1); weights streamed
//              from a tile image
//   ppo_wgrad  dW = (output gradient)^T (input) as 128x64 tiles over 8 row slices (one per XCD)
//              plus bias column sums, the head-parameter sums and the metrics row
//   ppo_wsum   the 8 slice partials summed in slice order, sum-of-squares partials
//   ppo_adam   clip_grad_norm_ + Adam (torch.optim.Adam formula), the tile image rewritten
// ppo_act is ppo_rows' forward + a sampling head (ActorCritic.act on a batch).
//
// General path (other shapes): 11 launches of a 64x64-tile GEMM (gemm64 / gemm64v), the loss
// head kernel (ppo_head), split-K partial slabs and one deterministic reduction (ppo_reduce).
// All GEMMs use v_mfma_f32_*_f32: exact fp32 products, fp32 accumulation.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <type_traits>

#include "hwy_ppo.h"

typedef float f32x16 __attribute__((ext_vector_type(16)));

// Development build only (make prof): shader-clock totals per phase of ppo_rows / ppo_wgrad,
// summed over workgroups (wave 0), read back with hwy_ppo_debug_sections().
#if defined(HWY_SECTION_PROFILE) || defined(HWY_CLOCK_PROBE)
__device__ unsigned long long g_ppo_sections[16];
#endif
// Development build only (HWY_CLOCK_PROBE): the in-kernel shader clock of ppo_rows* / ppo_wgrad,
// as s_memtime (shader cycles) and s_memrealtime (100 MHz) deltas of thread 0 of every
// workgroup, summed into g_ppo_sections[2k], [2k + 1] (k = 0 rows, 1 wgrad)
#ifdef HWY_CLOCK_PROBE
// also every workgroup's (start, end) s_memrealtime and HW_ID | XCC_ID << 32 of the last
// launch of each kernel: g_ppo_wgt[k][blockIdx.x][3] (read with hwy_ppo_debug_wgtimes)
__device__ unsigned long long g_ppo_wgt[2][1024][3];
#define CLK_BEGIN                                         \
  const uint64_t _c0 = __builtin_amdgcn_s_memtime();      \
  const uint64_t _r0 = __builtin_amdgcn_s_memrealtime();
#define CLK_END(k)                                                                   \
  do {                                                                               \
    if (threadIdx.x == 0) {                                                          \
      const uint64_t _r1 = __builtin_amdgcn_s_memrealtime();                         \
      atomicAdd(&g_ppo_sections[2 * (k)], __builtin_amdgcn_s_memtime() - _c0);       \
      atomicAdd(&g_ppo_sections[2 * (k) + 1], _r1 - _r0);                            \
      if (blockIdx.x < 1024) {                                                       \
        g_ppo_wgt[k][blockIdx.x][0] = _r0;                                           \
        g_ppo_wgt[k][blockIdx.x][1] = _r1;                                           \
        g_ppo_wgt[k][blockIdx.x][2] =                                                \
            (unsigned long long)(uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 4) |  \
            ((unsigned long long)(__builtin_amdgcn_s_getreg((31 << 11) | 20) & 0xff) << 32); \
      }                                                                              \
    }                                                                                \
  } while (0)
#else
#define CLK_BEGIN
#define CLK_END(k) \
  do {             \
  } while (0)
#endif
#ifdef HWY_SECTION_PROFILE
#define PSEC_DECL                                \
  uint64_t _pt = __builtin_amdgcn_s_memtime();   \
  uint64_t _pacc[16];                            \
  for (int _i = 0; _i < 16; ++_i) _pacc[_i] = 0;
#define PSEC(id)                                       \
  do {                                                 \
    const uint64_t _n = __builtin_amdgcn_s_memtime();  \
    _pacc[id] += _n - _pt;                             \
    _pt = _n;                                          \
  } while (0)
#define PSEC_FLUSH                                                             \
  do {                                                                         \
    if (threadIdx.x == 0)                                                      \
      for (int _i = 0; _i < 16; ++_i)                                          \
        if (_pacc[_i]) atomicAdd(&g_ppo_sections[_i], _pacc[_i]);              \
  } while (0)
#define PSEC_PARAMS , uint64_t &_pt, uint64_t *_pacc
#define PSEC_ARGS , _pt, _pacc
#else
#define PSEC_PARAMS
#define PSEC_ARGS
#define PSEC_DECL
#define PSEC(id) \
  do {           \
  } while (0)
#define PSEC_FLUSH \
  do {             \
  } while (0)
#endif

namespace {

constexpr int kTile = 64;
constexpr int kKStep = 32;
constexpr int kHeadRows = 16;  // minibatch rows per head workgroup (4 per wave)
constexpr int kRowTile = 16;   // minibatch rows per ppo_rows workgroup
constexpr int kMaxRowS = 256;  // states dim bound of the fused path (LDS)
// Product constants, each measured against its alternatives (the rejected
// alternatives are in git history, round 4 and earlier):
//  - ppo_rows at H = 256, 16-row tiles: 8 waves (2 per SIMD, two 16-column tiles each);
//  - 32-row tiles at H = 256: the compact-LDS ppo_rows_c (two workgroups per CU), 8 waves;
//  - 64-row tiles at H = 256 once every CU gets one (ppo_rows_c64, one workgroup per CU);
//  - the row kernels issue their states gather before the weight ring's prime (vector memory
//    completes in issue order) and pin their activation reads one block ahead of the MFMAs;
//  - ppo_wgrad stages its chunks by LDS-DMA, the next chunk's pieces spread between the MFMA
//    groups of the current one;
//  - kRingDC weight blocks in flight per wave in the compact-LDS row kernels.
constexpr int kRingDC = 2;
constexpr int kWgTM = 128, kWgTN = 64;          // ppo_wgrad output tile
constexpr int kWgWaves = 8;                     // ppo_wgrad waves (2 per SIMD)
constexpr int kWgPart = kWgTM * kWgTN + kWgTM;  // floats per partial tile (+ bias sums)

struct GemmArgs {
  int M, N, K;
  const float* A;
  int lda;
  const int64_t* a_gather;
  const float* B;
  const float* B2;
  int ldb;
  int split;
  const int64_t* b_gather;
  float* C;
  int ldc;
  const float* bias;
  const float* bias2;
  const float* mask;
  int ldm;
  float* bias_part;
  int kchunk;
  long slab;
};

enum { A_ROW = 0, A_TRANS = 1 };
enum { B_NT = 0, B_NN = 1 };
enum { EPI_BIAS_RELU = 0, EPI_MASK = 1, EPI_SPLITK = 2 };

template <int AM>
__device__ __forceinline__ float load_a(const GemmArgs& g, int m, int k, int kend) {
  if (m >= g.M || k >= kend) return 0.0f;
  if (AM == A_ROW) {
    const long row = g.a_gather ? (long)g.a_gather[m] : (long)m;
    return g.A[row * g.lda + k];
  }
  return g.A[(long)k * g.lda + m];
}

template <int BM>
__device__ __forceinline__ float load_b(const GemmArgs& g, int k, int n, int kend) {
  if (n >= g.N || k >= kend) return 0.0f;
  if (BM == B_NT) {
    return n < g.split ? g.B[(long)n * g.ldb + k] : g.B2[(long)(n - g.split) * g.ldb + k];
  }
  if (k >= g.split) return g.B2[(long)(k - g.split) * g.ldb + n];
  const long row = g.b_gather ? (long)g.b_gather[k] : (long)k;
  return g.B[row * g.ldb + n];
}

template <int AM, int BM, int EPI>
__global__ void __launch_bounds__(256) gemm64(GemmArgs g) {
  __shared__ float As[kKStep][kTile + 1];
  __shared__ float Bs[kKStep][kTile + 1];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int m0 = blockIdx.x * kTile, n0 = blockIdx.y * kTile;
  int kbeg = 0, kend = g.K;
  if (EPI == EPI_SPLITK) {
    kbeg = blockIdx.z * g.kchunk;
    kend = min(g.K, kbeg + g.kchunk);
  }
  const int wm = (w & 1) * 32, wn = (w >> 1) * 32;
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
  float ra[8], rb[8];
  float colsum = 0.0f;
  const bool do_colsum = EPI == EPI_SPLITK && g.bias_part && blockIdx.y == 0 && t < kTile;

  auto fetch = [&](int k0) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int e = t + 256 * i;
      const int am = AM == A_ROW ? (e >> 5) : (e & 63), ak = AM == A_ROW ? (e & 31) : (e >> 6);
      ra[i] = load_a<AM>(g, m0 + am, k0 + ak, kend);
      const int bn = BM == B_NT ? (e >> 5) : (e & 63), bk = BM == B_NT ? (e & 31) : (e >> 6);
      rb[i] = load_b<BM>(g, k0 + bk, n0 + bn, kend);
    }
  };
  if (kbeg < kend) fetch(kbeg);
  for (int k0 = kbeg; k0 < kend; k0 += kKStep) {
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int e = t + 256 * i;
      const int am = AM == A_ROW ? (e >> 5) : (e & 63), ak = AM == A_ROW ? (e & 31) : (e >> 6);
      As[ak][am] = ra[i];
      const int bn = BM == B_NT ? (e >> 5) : (e & 63), bk = BM == B_NT ? (e & 31) : (e >> 6);
      Bs[bk][bn] = rb[i];
    }
    __syncthreads();
    if (k0 + kKStep < kend) fetch(k0 + kKStep);  // prefetch next tile during the MFMAs
#pragma unroll
    for (int s = 0; s < kKStep / 2; ++s) {
      const float a = As[2 * s + (lane >> 5)][wm + (lane & 31)];
      const float b = Bs[2 * s + (lane >> 5)][wn + (lane & 31)];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
    }
    if (do_colsum) {
#pragma unroll
      for (int k = 0; k < kKStep; ++k) colsum += As[k][t];
    }
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int i = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
    const int gm = m0 + wm + i, gn = n0 + wn + (lane & 31);
    if (gm >= g.M || gn >= g.N) continue;
    float v = acc[r];
    if (EPI == EPI_BIAS_RELU) {
      v = v + (gn < g.split ? g.bias[gn] : g.bias2[gn - g.split]);
      v = v > 0.0f ? v : 0.0f;
      g.C[(long)gm * g.ldc + gn] = v;
    } else if (EPI == EPI_MASK) {
      g.C[(long)gm * g.ldc + gn] = g.mask[(long)gm * g.ldm + gn] > 0.0f ? v : 0.0f;
    } else {
      g.C[blockIdx.z * g.slab + (long)gm * g.ldc + gn] = v;
    }
  }
  if (do_colsum && m0 + t < g.M) g.bias_part[(long)blockIdx.z * g.M + m0 + t] = colsum;
}

// ----------------------------------------------------------------------------- vector GEMM
// Same contract as gemm64, 16-byte global loads and LDS images in each operand's natural
// layout.  Operands whose k index is contiguous in memory (A row-major, B NT) are kept as
// [row][k] images with a 36-float pitch and read with ds_read_b128 (16 k-values per lane per
// K-tile: MFMA step s uses k = 16*(lane>>5) + s, a permutation of the K-tile the sum does not
// see); k-major operands (A transposed, B NN) are kept as [k][row] images (68-float pitch) and
// read one k per MFMA.  Needs K % 4 == 0 for [row][k] operands and M, N % 4 == 0 otherwise.
typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int kVK = 64;        // K-tile of the vector kernel: 8 16-byte loads per thread in flight
constexpr int kPitchRK = 68;   // [row][k] image: 272-B rows, conflict-free ds_read_b128
constexpr int kPitchKR = 68;   // [k][row] image
constexpr int kV4 = kTile * kVK / 4 / 256;  // float4 per thread per operand per K-tile (4)

template <int AM>
__device__ __forceinline__ f32x4 load_a4(const GemmArgs& g, int e4, int m0, int k0, int kend) {
  f32x4 z = {0.0f, 0.0f, 0.0f, 0.0f};
  if (AM == A_ROW) {  // [row][k]: 16 float4 per 64-k row
    const int r = e4 >> 4, k = k0 + (e4 & 15) * 4, m = m0 + r;
    if (m >= g.M || k >= kend) return z;
    const long row = g.a_gather ? (long)g.a_gather[m] : (long)m;
    return *reinterpret_cast<const f32x4*>(g.A + row * g.lda + k);
  }
  const int k = k0 + (e4 >> 4), m = m0 + (e4 & 15) * 4;  // [k][row]: 16 float4 per 64-m row
  if (m >= g.M || k >= kend) return z;
  return *reinterpret_cast<const f32x4*>(g.A + (long)k * g.lda + m);
}

template <int BM>
__device__ __forceinline__ f32x4 load_b4(const GemmArgs& g, int e4, int n0, int k0, int kend) {
  f32x4 z = {0.0f, 0.0f, 0.0f, 0.0f};
  if (BM == B_NT) {
    const int r = e4 >> 4, k = k0 + (e4 & 15) * 4, n = n0 + r;
    if (n >= g.N || k >= kend) return z;
    const float* p = n < g.split ? g.B + (long)n * g.ldb : g.B2 + (long)(n - g.split) * g.ldb;
    return *reinterpret_cast<const f32x4*>(p + k);
  }
  const int k = k0 + (e4 >> 4), n = n0 + (e4 & 15) * 4;
  if (n >= g.N || k >= kend) return z;
  const float* p;
  if (k >= g.split) {
    p = g.B2 + (long)(k - g.split) * g.ldb;
  } else {
    const long row = g.b_gather ? (long)g.b_gather[k] : (long)k;
    p = g.B + row * g.ldb;
  }
  return *reinterpret_cast<const f32x4*>(p + n);
}

// Same contract as gemm64 with 16-byte global loads, a 64-deep K-tile and LDS images in each
// operand's natural layout.  Operands with k contiguous in memory (A row-major, B NT) become
// [row][k] images read with ds_read_b128 (MFMA step s of lane half h uses k = 32h + s, a
// permutation of the K-tile that the sum does not see); k-major operands (A transposed, B NN)
// become [k][row] images read one k per MFMA.  Needs K % 4 == 0 for [row][k] operands and
// M, N % 4 == 0 for [k][row] ones (launch_gemm falls back to gemm64 otherwise).
template <int AM, int BM, int EPI>
__global__ void __launch_bounds__(256) gemm64v(GemmArgs g) {
  __shared__ __attribute__((aligned(16))) float As[64 * kPitchRK];
  __shared__ __attribute__((aligned(16))) float Bs[64 * kPitchRK];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, h = lane >> 5, l32 = lane & 31;
  const int m0 = blockIdx.x * kTile, n0 = blockIdx.y * kTile;
  int kbeg = 0, kend = g.K;
  if (EPI == EPI_SPLITK) {
    kbeg = blockIdx.z * g.kchunk;
    kend = min(g.K, kbeg + g.kchunk);
  }
  const int wm = (w & 1) * 32, wn = (w >> 1) * 32;
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
  f32x4 ra[kV4], rb[kV4];
  float colsum = 0.0f;
  const bool do_colsum = EPI == EPI_SPLITK && g.bias_part && blockIdx.y == 0 && t < kTile;
  auto fetch = [&](int k0) {
#pragma unroll
    for (int i = 0; i < kV4; ++i) {
      ra[i] = load_a4<AM>(g, t + 256 * i, m0, k0, kend);
      rb[i] = load_b4<BM>(g, t + 256 * i, n0, k0, kend);
    }
  };
  if (kbeg < kend) fetch(kbeg);
  for (int k0 = kbeg; k0 < kend; k0 += kVK) {
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kV4; ++i) {
      const int e4 = t + 256 * i;
      // both layouts: image row = e4 >> 4, column = (e4 & 15) * 4
      const int off = (e4 >> 4) * kPitchRK + (e4 & 15) * 4;
      *reinterpret_cast<f32x4*>(&As[off]) = ra[i];
      *reinterpret_cast<f32x4*>(&Bs[off]) = rb[i];
    }
    __syncthreads();
    if (k0 + kVK < kend) fetch(k0 + kVK);  // next K-tile in flight during the MFMAs
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      float a[16], b[16];
      if (AM == A_ROW) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const f32x4 v = *reinterpret_cast<const f32x4*>(
              &As[(wm + l32) * kPitchRK + h * 32 + half * 16 + 4 * q]);
          a[4 * q] = v[0], a[4 * q + 1] = v[1], a[4 * q + 2] = v[2], a[4 * q + 3] = v[3];
        }
      } else {
#pragma unroll
        for (int s = 0; s < 16; ++s) a[s] = As[(h * 32 + half * 16 + s) * kPitchKR + wm + l32];
      }
      if (BM == B_NT) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const f32x4 v = *reinterpret_cast<const f32x4*>(
              &Bs[(wn + l32) * kPitchRK + h * 32 + half * 16 + 4 * q]);
          b[4 * q] = v[0], b[4 * q + 1] = v[1], b[4 * q + 2] = v[2], b[4 * q + 3] = v[3];
        }
      } else {
#pragma unroll
        for (int s = 0; s < 16; ++s) b[s] = Bs[(h * 32 + half * 16 + s) * kPitchKR + wn + l32];
      }
#pragma unroll
      for (int s = 0; s < 16; ++s)
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s], b[s], acc, 0, 0, 0);
    }
    if (do_colsum) {
#pragma unroll 8
      for (int k = 0; k < kVK; ++k) colsum += As[k * kPitchKR + t];
    }
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int i = (r & 3) + 8 * (r >> 2) + 4 * h;
    const int gm = m0 + wm + i, gn = n0 + wn + l32;
    if (gm >= g.M || gn >= g.N) continue;
    float v = acc[r];
    if (EPI == EPI_BIAS_RELU) {
      v = v + (gn < g.split ? g.bias[gn] : g.bias2[gn - g.split]);
      v = v > 0.0f ? v : 0.0f;
      g.C[(long)gm * g.ldc + gn] = v;
    } else if (EPI == EPI_MASK) {
      g.C[(long)gm * g.ldc + gn] = g.mask[(long)gm * g.ldm + gn] > 0.0f ? v : 0.0f;
    } else {
      g.C[blockIdx.z * g.slab + (long)gm * g.ldc + gn] = v;
    }
  }
  if (do_colsum && m0 + t < g.M) g.bias_part[(long)blockIdx.z * g.M + m0 + t] = colsum;
}

// Tile image of the row kernels' weights (in the workspace): for a matrix read as B[k][n] in
// 16-deep k blocks, tile (G, b) is the 1-KB MFMA operand of columns 16G..16G+15 and block b:
// float 4*(16g + c) + j = B[16b + 4g + j][16G + c] (0 past K), tiles ordered G-major.  Forward
// images (f*) hold B = W^T of W1, W2, Wa1, Wc1; backward images (b*) B = W of Wa1, Wc1, W2.
struct TileGeom {
  int64_t f1, f2, fa, fc, ba, bc, b2, total;  // float offsets
};
__host__ __device__ inline TileGeom tile_geom(int S, int H, int sb, int hb) {
  TileGeom T;
  const int64_t g = H / 16, big = g * hb * 256;
  T.f1 = 0;
  T.f2 = g * sb * 256;
  T.fa = T.f2 + big;
  T.fc = T.fa + big;
  T.ba = T.fc + big;
  T.bc = T.ba + big;
  T.b2 = T.bc + big;
  T.total = T.b2 + big;
  return T;
}
// ring depth of the row kernels for H (ppo_rows<H/64, NW>: 16-column tiles per wave TW)
__host__ __device__ inline int rows_ring_depth(int H) {
  const int qh = H / 64, nw = (qh % 2 == 0) ? 8 : 4, tw = H / nw / 16;
  return tw <= 4 ? 4 : 2;  // weight blocks in flight per wave (8 at H 256: slower, round 5)
}
__host__ __device__ inline void rows_blocks(int S, int H, int* sb, int* hb) {
  const int D = rows_ring_depth(H);
  *hb = (H / 16 + D - 1) / D * D;
  *sb = ((S + 15) / 16 + D - 1) / D * D;
}

// ----------------------------------------------------------------------------- layout
struct Layout {
  int64_t off[13];
  int64_t numel;
};

__host__ __device__ inline Layout make_layout(const hwy_ppo_dims& d) {
  Layout L;
  const int64_t S = d.S, H = d.H, A = d.A;
  const int64_t sizes[13] = {H * S, H, H * H, H, H * H, H, A * H, A, A, H * H, H, H, 1};
  int64_t o = 0;
  for (int i = 0; i < 13; ++i) {
    L.off[i] = o;
    o += sizes[i];
  }
  L.numel = o;
  return L;
}
enum { P_W1, P_B1, P_W2, P_B2, P_WA1, P_BA1, P_WA2, P_BA2, P_LOGSTD, P_WC1, P_BC1, P_WC2, P_BC2 };

inline int split_for(int tiles, int K) {
  int s = 256 / (tiles > 0 ? tiles : 1);
  if (s < 1) s = 1;
  int maxs = (K + kKStep - 1) / kKStep;
  return s > maxs ? maxs : s;
}
inline int chunk_for(int K, int split) {
  int c = (K + split - 1) / split;
  return (c + kKStep - 1) / kKStep * kKStep;
}

struct Work {
  float *h1, *h2, *ac, *dac, *dh2, *dh1;
  float *head_part;   // [max(nhead, 4 * n1)][HP]
  float *slab_ac, *bias_ac;  // [sa][2H][H], [sa][2H]   (split-K path only)
  float *slab_2, *bias_2;    // [s2][H][H], [s2][H]
  float *slab_1, *bias_1;    // [s1][H][S], [s1][H]
  float *norm_part;          // [max(nred, nred2)]
  float *wg_slab;            // fused: [ntile][split][kWgPart] partial tiles
  float *xg;                 // fused: [B][S] gathered states
  float *wtile;              // fused: weight tile image (TileGeom)
  int nhead, HP, sa, s2, s1, ca, c2, c1, nred;
  // fused path (ppo_rows + ppo_wgrad)
  bool fused;
  int rt, n1, tac, t2, t1, nh, split, grid2, nred2;  // rt: rows per ppo_rows workgroup
  int bal, wm, tpe, nslot;                            // ppo_wgrad's balanced partition
  int sb, hb;  // ring blocks of the row kernels (rows_blocks)
};

// The chip the partitions are sized for: compute units and XCDs of the current device
// (hipDeviceAttributeNumberOfXccs; a compute-partitioned MI355X reports its own share).  Without
// a device (the CPU-side workspace queries of the tests) the full MI355X: 256 CUs, 8 XCDs.
struct ChipGeom {
  int cus, xcds;
};
inline ChipGeom chip_geom() {
  static ChipGeom cache[64];
  static bool have[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) {
    (void)hipGetLastError();
    return {256, 8};
  }
  if (!have[dev]) {
    int cus = 0, xcds = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus < 1)
      cus = 256;
    if (hipDeviceGetAttribute(&xcds, hipDeviceAttributeNumberOfXccs, dev) != hipSuccess ||
        xcds < 1 || xcds > cus)
      xcds = 1;
    (void)hipGetLastError();
    cache[dev] = {cus, xcds};
    have[dev] = true;
  }
  return cache[dev];
}

// Development knobs (make dev builds only, -DHWY_DEV_KNOBS): HWY_WG_BAL=0 keeps one ppo_wgrad
// workgroup per (tile, slice), HWY_ROWS_RT=16|32 forces the ppo_rows tile, HWY_WG_FILL prices an
// extra's pipeline fill.  The product library reads no environment: the partitions, and with
// them the summation order of every gradient, depend only on the shapes and the chip.
#ifdef HWY_DEV_KNOBS
inline int dev_knob_int(const char* name, int dflt) {
  const char* e = getenv(name);
  return e ? atoi(e) : dflt;
}
inline double dev_knob_double(const char* name, double dflt) {
  const char* e = getenv(name);
  return e ? atof(e) : dflt;
}
#else
inline int dev_knob_int(const char*, int dflt) { return dflt; }
inline double dev_knob_double(const char*, double dflt) { return dflt; }
#endif

// ppo_wgrad's balanced partition (see ppo_wgrad)
inline bool wg_balance_on() { return dev_knob_int("HWY_WG_BAL", 1) != 0; }

// minibatch rows per ppo_rows workgroup: 32 (two 16-row blocks sharing every weight register
// block: half the weight stream per row) when the grid still covers the chip and the LDS images
// fit (H <= 256), else 16.
inline int rows_tile(int B, int H) {
  if (H > 256) return kRowTile;
  // 64-row tiles (ppo_rows_c64, one workgroup per CU) once every CU gets one: each weight
  // fragment then feeds 4 row blocks, half the weight loads per MFMA of the 32-row tiles
  const int force = dev_knob_int("HWY_ROWS_RT", 0);  // development builds only
  if (force == 16 || force == 32) return force;
  if (H == 256 && B >= 64 * chip_geom().cus) return 4 * kRowTile;
  return B >= 32 * chip_geom().cus ? 2 * kRowTile : kRowTile;
}

// the fused row path covers the reference's shapes: float4 state rows, H a multiple of 64
inline bool fused_ok(const hwy_ppo_dims& d) {
  return d.S % 4 == 0 && d.S <= kMaxRowS && d.H % 64 == 0 && d.H >= 64 && d.H <= 512;
}

inline int head_stride(int H) { return 3 * H + 16; }

constexpr int kRedThreads = 256;

inline Work carve(const hwy_ppo_dims& d, void* ws, int64_t* bytes_out) {
  Work w;
  const int B = d.B, S = d.S, H = d.H;
  w.nhead = (B + kHeadRows - 1) / kHeadRows;
  w.HP = head_stride(H);
  const int tiles_ac = ((2 * H + 63) / 64) * ((H + 63) / 64);
  const int tiles_2 = ((H + 63) / 64) * ((H + 63) / 64);
  const int tiles_1 = ((H + 63) / 64) * ((S + 63) / 64);
  w.sa = split_for(tiles_ac, B);
  w.ca = chunk_for(B, w.sa);
  w.sa = (B + w.ca - 1) / w.ca;
  w.s2 = split_for(tiles_2, B);
  w.c2 = chunk_for(B, w.s2);
  w.s2 = (B + w.c2 - 1) / w.c2;
  w.s1 = split_for(tiles_1, B);
  w.c1 = chunk_for(B, w.s1);
  w.s1 = (B + w.c1 - 1) / w.c1;
  const Layout L = make_layout(d);
  w.nred = (int)((L.numel + kRedThreads - 1) / kRedThreads);
  w.fused = fused_ok(d);
  w.rt = rows_tile(B, H);
  w.n1 = (B + w.rt - 1) / w.rt;
  const int tmh = (H + kWgTM - 1) / kWgTM, tnh = (H + kWgTN - 1) / kWgTN;
  w.tac = ((2 * H + kWgTM - 1) / kWgTM) * tnh;
  w.t2 = tmh * tnh;
  w.t1 = tmh * ((S + kWgTN - 1) / kWgTN);
  w.nh = (3 * H + 9 + 63) / 64;
  const int ntile = w.tac + w.t2 + w.t1;
  // Row slices per tile (split) and the balanced partition (ppo_wgrad).  Balanced: cus / split
  // workgroups per slice when the tiles leave at least two CUs of each slice's share idle and
  // the slices are long enough; the first wm chunks of every tile run on its own workgroup and
  // the "extras" take the rest, tpe tiles each, paying ~1.5 chunks of pipeline fill per tile.
  // The split is the largest divisor of the XCD count that gives every tile a workgroup (slice
  // z = workgroup id % split then lands on the XCDs x with x % split == z under round-robin
  // placement: each XCD's L2 serves one slice), unless another split's balanced partition
  // shortens the critical path (64-row chunks per workgroup) by 15 % or more: 66 tiles at 32,768
  // rows (H 384, S 240) run 3 slices at 138 chunks (332 us) instead of 2 at 172 (400 us; with
  // tpe 2 half of the extras were idle).  (A 4-slice balanced partition of 32 tiles, H 256 /
  // S 240, measured slower than 8 unbalanced slices: 186 against 164 us.)
  const ChipGeom chip = chip_geom();
  const double fill = dev_knob_double("HWY_WG_FILL", 1.5);
  struct Plan {
    int split, bal, wm, tpe, cost;
  };
  auto plan = [&](int sp) {
    Plan q = {sp, 0, 0, 0, 0};
    const int P = chip.cus / sp;                          // workgroups per slice
    const int nck = ((B + sp - 1) / sp + 63) / 64;        // chunks of the longest slice
    q.cost = nck;
    if (wg_balance_on() && ntile >= 16 && P - ntile >= 2 && nck >= 16) {
      const int E = P - ntile, tpe = (ntile + E - 1) / E;
      const int m = (int)std::ceil(tpe * (nck + fill) / (1.0 + tpe));
      if (m < nck) q.bal = 1, q.wm = m, q.tpe = tpe, q.cost = m;
    }
    return q;
  };
  const int cap = std::max(1, std::min({chip.xcds, 8, chip.cus / ntile, (B + 63) / 64}));
  Plan best = plan(1);
  for (int sp = cap; sp >= 1; --sp)
    if (chip.xcds % sp == 0) {
      best = plan(sp);
      break;
    }
  for (int sp = 2; sp <= std::min(8, std::max(1, (B + 63) / 64)); ++sp) {
    if (chip.xcds % sp == 0) continue;
    const Plan q = plan(sp);
    if (q.bal && q.cost < 0.85 * best.cost && (!best.bal || q.cost < best.cost)) best = q;
  }
  w.split = best.split;
  w.bal = best.bal, w.wm = best.wm, w.tpe = best.tpe, w.nslot = best.bal ? 2 : 1;
  w.grid2 = best.bal ? w.split * (chip.cus / w.split) : ntile * w.split + w.nh;
  w.nred2 = w.nh + ntile * (kWgTM * kWgTN / 1024);
  const int64_t head_rows = w.fused ? std::max<int64_t>(w.nhead, w.n1) : w.nhead;
  const int64_t norm_n = w.fused ? std::max(w.nred, w.nred2) : w.nred;
  // the fused path needs no split-K slabs of full weight size, only the per-split tiles
  const int64_t sa = w.fused ? 0 : w.sa, s2 = w.fused ? 0 : w.s2, s1 = w.fused ? 0 : w.s1;
  const int64_t wg_slab_n = w.fused ? (int64_t)ntile * w.split * w.nslot * kWgPart : 0;
  const int64_t xg_n = w.fused ? (int64_t)B * S : 0;
  rows_blocks(S, H, &w.sb, &w.hb);
  const int64_t tile_n = w.fused ? tile_geom(S, H, w.sb, w.hb).total : 0;
  int64_t sizes[17] = {
      (int64_t)B * H, (int64_t)B * H, (int64_t)B * 2 * H, (int64_t)B * 2 * H, (int64_t)B * H,
      (int64_t)B * H, head_rows * w.HP, sa * 2 * H * H, sa * 2 * H,
      s2 * H * H, s2 * H, s1 * H * S, s1 * H,
      norm_n, wg_slab_n, xg_n, tile_n};
  float* p = (float*)ws;
  float** dst[17] = {&w.h1, &w.h2, &w.ac, &w.dac, &w.dh2, &w.dh1, &w.head_part, &w.slab_ac,
                     &w.bias_ac, &w.slab_2, &w.bias_2, &w.slab_1, &w.bias_1, &w.norm_part,
                     &w.wg_slab, &w.xg, &w.wtile};
  int64_t total = 0;
  for (int i = 0; i < 17; ++i) {
    int64_t n = (sizes[i] + 63) / 64 * 64;  // 256-B aligned sub-buffers
    if (p) *dst[i] = p + total;
    total += n;
  }
  if (bytes_out) *bytes_out = total * (int64_t)sizeof(float);
  return w;
}

// ----------------------------------------------------------------------------- head + loss
// One wave per minibatch row at a time (kHeadRows rows per workgroup, 4 waves); lane owns the
// hidden columns lane + 64q.  Per row: mean = a1 Wa2^T + ba2, v = c1 Wc2^T + bc2 (wave
// butterfly sums, fixed order), then the reference's loss (ppo/agent.py:226-245) and its
// gradient w.r.t. mean, v and log_std; dL/d[a1|c1] (through the ReLU) goes to dac and the head
// weight / bias / log_std gradients accumulate per lane, combined per workgroup at the end.
struct HeadArgs {
  int B, H, A;
  const float* ac;  // [B, 2H]
  float* dac;       // [B, 2H]
  const float* params;
  const float* pre_tanh;
  const float* old_logp;
  const float* adv;
  const float* ret;
  const int64_t* idx;
  float* part;  // [nhead][HP]
  int HP;
  int64_t off_wa2, off_ba2, off_ls, off_wc2, off_bc2;
  float eps_clip, value_coef, entropy_coef;
  int32_t* counters;
};

constexpr int kHeadMaxQ = 8;  // H <= 512

// v + DPP-moved copy of v (lanes outside row_mask add 0)
template <int CTRL, int ROWS>
__device__ __forceinline__ float dpp_add(float v) {
  const int m = __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, ROWS, 0xf, false);
  return v + __builtin_bit_cast(float, m);
}
// wave sum with DPP steps (pairs, quads, 8, 16 lanes, then rows by broadcast), total read from
// lane 63 as a wave-uniform value
__device__ __forceinline__ float wave_sum_dpp(float v) {
  v = dpp_add<0xB1, 0xf>(v);   // quad_perm(1,0,3,2)
  v = dpp_add<0x4E, 0xf>(v);   // quad_perm(2,3,0,1)
  v = dpp_add<0x141, 0xf>(v);  // row_half_mirror
  v = dpp_add<0x140, 0xf>(v);  // row_mirror
  v = dpp_add<0x142, 0xa>(v);  // row_bcast:15 -> rows 1, 3
  v = dpp_add<0x143, 0xc>(v);  // row_bcast:31 -> rows 2, 3
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 63));
}

__global__ void __launch_bounds__(256) ppo_head(HeadArgs h) {
  __shared__ float wpart[4][3 * 512 + 16];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int H = h.H, Q = H / 64;
  float wa0[kHeadMaxQ], wa1[kHeadMaxQ], wc[kHeadMaxQ];
  float ga0[kHeadMaxQ], ga1[kHeadMaxQ], gc[kHeadMaxQ];
#pragma unroll
  for (int q = 0; q < kHeadMaxQ; ++q) {
    const int col = lane + 64 * q;
    const bool ok = q < Q;
    wa0[q] = ok ? h.params[h.off_wa2 + col] : 0.0f;
    wa1[q] = ok ? h.params[h.off_wa2 + H + col] : 0.0f;
    wc[q] = ok ? h.params[h.off_wc2 + col] : 0.0f;
    ga0[q] = ga1[q] = gc[q] = 0.0f;
  }
  const float ba0 = h.params[h.off_ba2], ba1 = h.params[h.off_ba2 + 1];
  const float bcv = h.params[h.off_bc2];
  const float ls0 = h.params[h.off_ls], ls1 = h.params[h.off_ls + 1];
  // torch Normal: scale = exp(log_std); var = scale**2; log_scale = log(scale)
  const float sc0 = expf(ls0), sc1 = expf(ls1);
  const float var0 = sc0 * sc0, var1 = sc1 * sc1;
  const float lsc0 = logf(sc0), lsc1 = logf(sc1);
  const float LOG_SQRT_2PI = 0.91893853320467274178f;
  const float invB = 1.0f / (float)h.B;
  const float lo = 1.0f - h.eps_clip, hi = 1.0f + h.eps_clip;
  float s_dba0 = 0, s_dba1 = 0, s_dbc = 0, s_dls0 = 0, s_dls1 = 0;
  float s_pg = 0, s_vf = 0, s_clip = 0, s_kl = 0;
  const int rows_per_wave = kHeadRows / 4;
  const int r0 = blockIdx.x * kHeadRows + w * rows_per_wave;
  for (int rr = 0; rr < rows_per_wave; ++rr) {
    const int b = r0 + rr;
    if (b >= h.B) break;
    const float* arow = h.ac + (long)b * 2 * H;
    float a[kHeadMaxQ], c[kHeadMaxQ];
    float p0 = 0.0f, p1 = 0.0f, pv = 0.0f;
#pragma unroll
    for (int q = 0; q < kHeadMaxQ; ++q) {
      const int col = lane + 64 * q;
      a[q] = q < Q ? arow[col] : 0.0f;
      c[q] = q < Q ? arow[H + col] : 0.0f;
      p0 += a[q] * wa0[q];
      p1 += a[q] * wa1[q];
      pv += c[q] * wc[q];
    }
    const long src = (long)h.idx[b];
    const float z0 = h.pre_tanh[src * 2], z1 = h.pre_tanh[src * 2 + 1];
    const float old = h.old_logp[src], ad = h.adv[src], rt = h.ret[src];
    const float mu0 = wave_sum_dpp(p0) + ba0, mu1 = wave_sum_dpp(p1) + ba1,
                val = wave_sum_dpp(pv) + bcv;
    const float d0 = z0 - mu0, d1 = z1 - mu1;
    const float t0 = tanhf(z0), t1 = tanhf(z1);
    const float lp0 = -(d0 * d0) / (2.0f * var0) - lsc0 - LOG_SQRT_2PI;
    const float lp1 = -(d1 * d1) / (2.0f * var1) - lsc1 - LOG_SQRT_2PI;
    const float logp = (lp0 - log1pf(-(t0 * t0) + 1e-6f)) + (lp1 - log1pf(-(t1 * t1) + 1e-6f));
    const float log_ratio = logp - old;
    const float ratio = expf(log_ratio);
    const float cr = fminf(fmaxf(ratio, lo), hi);
    const float s1 = ratio * ad, s2 = cr * ad;
    const float inr = (ratio >= lo && ratio <= hi) ? 1.0f : 0.0f;
    // torch.min / clamp backward: ties split the gradient evenly
    const float wsel = s1 < s2 ? 1.0f : (s1 > s2 ? inr : 0.5f * (1.0f + inr));
    const float dlogp = -invB * ad * wsel * ratio;  // d(actor_loss)/d(logp)
    const float dmu0 = dlogp * d0 / var0, dmu1 = dlogp * d1 / var1;
    const float dv = h.value_coef * 2.0f * (val - rt) * invB;
    float* drow = h.dac + (long)b * 2 * H;
#pragma unroll
    for (int q = 0; q < kHeadMaxQ; ++q) {
      if (q < Q) {
        const int col = lane + 64 * q;
        drow[col] = a[q] > 0.0f ? (dmu0 * wa0[q] + dmu1 * wa1[q]) : 0.0f;
        drow[H + col] = c[q] > 0.0f ? dv * wc[q] : 0.0f;
        ga0[q] += dmu0 * a[q];
        ga1[q] += dmu1 * a[q];
        gc[q] += dv * c[q];
      }
    }
    s_dba0 += dmu0;
    s_dba1 += dmu1;
    s_dbc += dv;
    s_dls0 += dlogp * ((d0 * d0) / var0 - 1.0f);
    s_dls1 += dlogp * ((d1 * d1) / var1 - 1.0f);
    s_pg += -fminf(s1, s2);
    s_vf += (val - rt) * (val - rt);
    s_clip += fabsf(ratio - 1.0f) > h.eps_clip ? 1.0f : 0.0f;
    s_kl += (ratio - 1.0f) - log_ratio;
  }
  // combine the 4 waves in a fixed order
  float* mine = wpart[w];
#pragma unroll
  for (int q = 0; q < kHeadMaxQ; ++q) {
    if (q < Q) {
      const int col = lane + 64 * q;
      mine[col] = ga0[q];
      mine[H + col] = ga1[q];
      mine[2 * H + col] = gc[q];
    }
  }
  if (lane == 0) {
    float* tl = mine + 3 * H;
    tl[0] = s_dba0, tl[1] = s_dba1, tl[2] = s_dbc, tl[3] = s_dls0, tl[4] = s_dls1;
    tl[5] = s_pg, tl[6] = s_vf, tl[7] = s_clip, tl[8] = s_kl;
  }
  __syncthreads();
  float* out = h.part + (long)blockIdx.x * h.HP;
  for (int j = t; j < 3 * H + 9; j += 256)
    out[j] = ((wpart[0][j] + wpart[1][j]) + wpart[2][j]) + wpart[3][j];
  if (blockIdx.x == 0 && t == 0) {
    h.counters[0] += 1;  // Adam step t for this minibatch
    h.counters[1] += 1;  // metrics row (this step writes row counters[1]-1)
  }
}

// ----------------------------------------------------------------------------- fused row kernel
// ppo_rows: one workgroup per 16 minibatch rows runs the whole row-local part of the step --
// forward (3 layers), the loss head and the backward data gradients (dh2, dh1) -- with the
// activations of its rows in LDS.  The weights stream from L2 (every workgroup reads them once
// per layer; 1-2 MB per step, L2-resident).  v_mfma_f32_16x16x4_f32: C[16 rows][16 cols] per
// accumulator, wave w owns output columns [w*N/4, (w+1)*N/4); A (activations) from LDS with
// ds_read_b128, B (weights) from global -- float4 along k for [N][K] weights (forward), one
// float per k for [K][N] weights (backward); within each 16-deep k block, sub-step j of lane
// group g = lane>>4 uses k = kb + 4g + j (a permutation of the block the sum does not see).
// Outputs for ppo_wgrad: h1, h2, dac, dh2, dh1 ([B][.] row-major) and per-wave head partials.
struct RowArgs {
  int B, S;
  const float* states;
  const int64_t* idx;
  const float* pre_tanh;
  const float* old_logp;
  const float* adv;
  const float* ret;
  const float* params;
  int64_t off[13];
  float *h1, *h2, *dac, *dh2, *dh1;
  float* xg;         // [B][S] gathered states (ppo_wgrad's dW1 operand)
  const float* tiles;  // weight tile image (TileGeom), in sync with params
  float* head_part;  // [gridDim.x][HP], one row per row tile
  int HP;
  float eps_clip, value_coef, entropy_coef;
  int32_t* counters;
};

// Row pitch (floats) of the row kernels' LDS images for n columns (n % 16 == 0): n + 8, i.e. a
// quad pitch = 2 mod 4.  The MFMA operand reads (ds_read_b128, lane (g, c) reads quad
// c * pitch/4 + g + kb/4) are serviced in the lane groups {0-3,12-15,20-27}, {4-11,16-19,28-31}
// (+32): with a quad pitch = 1 mod 16 (n + 4) two lanes of every group land on the same four
// banks (SQ_LDS_BANK_CONFLICT: 3.3 M cycles per 16,384-row launch); with 2 mod 4 none do.  The
// epilogues' ds_write_b32 then meet 2-way, which costs a store nothing.
constexpr int lds_pitch(int n) { return n + 8; }
__device__ __forceinline__ int row_pitch(int n) { return lds_pitch(n); }

// The weights of every layer a ppo_rows / ppo_act wave touches, as one stream of 16-deep k
// blocks (segments = layers, in execution order).  D blocks stay in flight in registers and the
// stream runs on across layer boundaries, barriers and the loss head, so a layer's first
// weights are already loaded when its activations are ready.  Segment lengths are multiples of
// D blocks (K is zero-padded: weights past K load as 0 and the activation images are zero-padded
// to the padded K).
#define H_TW(QH, NW) ((64 * (QH)) / (NW) / 16)

struct WSeg {
  const float* W;
  int ldw, K, nblk, nn;  // nn: 0 W is [N][K], 1 W is [K][N] (k-major), 2 W is a tile image
};

// UNI: the tile-image block address is made wave-uniform (scalar base + one 32-bit lane offset);
// it frees the VGPRs the compact ppo_rows needs to fit two workgroups per CU (141 -> 134 us at
// 16,384 rows) but costs the 16-row kernels at H 384 (648 -> 686 us at 32,768 rows, S 240)
template <int TW, int D, int NSEG, bool TL, bool UNI = false>
struct WRing {
  f32x4 buf[D][TW];
  WSeg sg[NSEG];
  int n_base, g, c;

  // Branch-free loads (so the compiler can count them): element (k, n) of segment s sits at
  // W + n*sn + k*sk with (sn, sk) = (ldw, 1) for [N][K] and (1, ldw) for [K][N]; k past K is
  // clamped into range here and zeroed when the block is consumed.
  __device__ __forceinline__ void load_blk(const float* W, int ldw, int nn, int kb,
                                           f32x4 (&dst)[TW]) {
    if constexpr (TL) {  // tile image (TileGeom): one contiguous KB per 16 columns and block
      if constexpr (UNI) {
        // wave-uniform tile address (scalar registers) + the lane's float4 (16 g + c = lane)
        const int tile0 = __builtin_amdgcn_readfirstlane((n_base / 16) * ldw + (kb >> 4));
        const float* p = W + (long)tile0 * 256;
        const int lo = 4 * (16 * g + c);
#pragma unroll
        for (int t = 0; t < TW; ++t)
          dst[t] = *reinterpret_cast<const f32x4*>(p + (long)t * ldw * 256 + lo);
      } else {
        const float* p = W + ((long)(n_base / 16) * ldw + (kb >> 4)) * 256 + (16 * g + c) * 4;
#pragma unroll
        for (int t = 0; t < TW; ++t)
          dst[t] = *reinterpret_cast<const f32x4*>(p + (long)t * ldw * 256);
      }
      return;
    }
    const int k = kb + 4 * g;
    const long sn = nn ? 1 : ldw, sk = nn ? ldw : 1;
#pragma unroll
    for (int t = 0; t < TW; ++t) {
      const float* p = W + (long)(n_base + 16 * t + c) * sn + (long)k * sk;
      dst[t] = f32x4{p[0], p[sk], p[2 * sk], p[3 * sk]};
    }
  }
  // load local block b of segment SEG, or (past its end) of the next segment; past the last
  // segment a harmless in-range block (never consumed)
  template <int SEG>
  __device__ __forceinline__ void load_ahead(int b, f32x4 (&dst)[TW]) {
    constexpr int NX = SEG + 1 < NSEG ? SEG + 1 : SEG;
    const bool nxt = b >= sg[SEG].nblk;
    const WSeg& s0 = sg[SEG];
    const WSeg& s1 = sg[NX];
    const float* W = nxt ? s1.W : s0.W;
    const int ldw = nxt ? s1.ldw : s0.ldw, nn = nxt ? s1.nn : s0.nn, K = nxt ? s1.K : s0.K;
    int kb = nxt ? 16 * (b - s0.nblk) : 16 * b;
    if (SEG + 1 >= NSEG && nxt) kb = 0;
    // k + 3 < K for every lane (K % 4 == 0); a tile image holds whole (zero-padded) blocks, so
    // its block index stays wave-uniform
    if constexpr (!TL) kb = min(kb, K - 4 - 4 * g);
    load_blk(W, ldw, nn, kb, dst);
  }
  __device__ __forceinline__ void prime() {
#pragma unroll
    for (int d = 0; d < D; ++d) load_ahead<0>(d, buf[d]);
    __builtin_amdgcn_sched_barrier(0);
  }
  // acc += act[16 RB][16*nblk] (LDS, pitch pa) x segment SEG's weights for this wave's columns;
  // the RB 16-row blocks share every weight register block (RB = 2 halves the weight stream
  // per row)
  template <int SEG, int RB>
  __device__ __forceinline__ void run(const float* act, int pa, f32x4 (&acc)[RB][TW]) {
    const int nblk = sg[SEG].nblk;
    const float* arow = act + c * pa + 4 * g;
    f32x4 a_nxt[RB];
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
      a_nxt[rb] = *reinterpret_cast<const f32x4*>(arow + 16 * rb * pa);
    for (int b0 = 0; b0 < nblk; b0 += D) {
#pragma unroll
      for (int d = 0; d < D; ++d) {
        const int kb = 16 * (b0 + d);
        f32x4 a[RB];  // activations of this block, read one block ahead
        const int kn = min(kb + 16, 16 * (nblk - 1));
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) {
          a[rb] = a_nxt[rb];
          a_nxt[rb] = *reinterpret_cast<const f32x4*>(arow + 16 * rb * pa + kn);
        }
        // pinned: the next block's activation reads go out before this block's MFMAs (the
        // scheduler otherwise sinks them to the block's end, right before their use)
        __builtin_amdgcn_sched_barrier(0);
        const bool kin = kb + 4 * g < sg[SEG].K;  // else the block was clamped: weights are 0
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int t = 0; t < TW; ++t) {
            const float bw = kin ? buf[d][t][j] : 0.0f;
#pragma unroll
            for (int rb = 0; rb < RB; ++rb)
              acc[rb][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[rb][j], bw, acc[rb][t], 0, 0, 0);
          }
        // issue the refill here: the scheduler would otherwise sink it next to its use
        __builtin_amdgcn_sched_barrier(0);
        load_ahead<SEG>(b0 + d + D, buf[d]);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
};

template <int RB, int TW>
__device__ __forceinline__ void zero_acc(f32x4 (&acc)[RB][TW]) {
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int t = 0; t < TW; ++t) acc[rb][t] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
}

template <int TW>
constexpr int ring_depth() { return TW <= 4 ? 4 : 2; }

// segment table of the row kernels: forward W1, W2, Wa1, Wc1 ([N][K]); backward Wa1, Wc1, W2
// read k-major for dh2 = dac [Wa1; Wc1] and dh1 = dh2 W2.  With a tile image (TileGeom; kept by
// hwy_ppo_sync_params / ppo_adam) every segment streams whole 1-KB tiles instead.
template <int TW, int D, int NSEG, bool TL, bool UNI>
__device__ __forceinline__ void ring_setup(WRing<TW, D, NSEG, TL, UNI>& R, const float* P,
                                           const int64_t* off, int S, int H, int n_base,
                                           const float* tiles) {
  const int lane = threadIdx.x & 63;
  R.g = lane >> 4;
  R.c = lane & 15;
  R.n_base = n_base;
  // the blocks of the tile image (rows_blocks: multiples of the default ring depth, which every
  // ring depth used here divides)
  int sb, hb;
  rows_blocks(S, H, &sb, &hb);
  if constexpr (TL) {
    const TileGeom T = tile_geom(S, H, sb, hb);
    const WSeg all[7] = {{tiles + T.f1, sb, 16 * sb, sb, 2},  {tiles + T.f2, hb, H, hb, 2},
                         {tiles + T.fa, hb, H, hb, 2},        {tiles + T.fc, hb, H, hb, 2},
                         {tiles + T.ba, hb, H, hb, 2},        {tiles + T.bc, hb, H, hb, 2},
                         {tiles + T.b2, hb, H, hb, 2}};
#pragma unroll
    for (int i = 0; i < NSEG; ++i) R.sg[i] = all[i];
    return;
  }
  const WSeg all[7] = {{P + off[P_W1], S, S, sb, 0},   {P + off[P_W2], H, H, hb, 0},
                       {P + off[P_WA1], H, H, hb, 0},  {P + off[P_WC1], H, H, hb, 0},
                       {P + off[P_WA1], H, H, hb, 1},  {P + off[P_WC1], H, H, hb, 1},
                       {P + off[P_W2], H, H, hb, 1}};
#pragma unroll
  for (int i = 0; i < NSEG; ++i) R.sg[i] = all[i];
}

// C element (rb, t, r) of lane: row 16 rb + 4*(lane>>4) + r, column n_base + 16 t + (lane & 15)
template <int RB, int TW>
__device__ __forceinline__ void row_epi_bias_relu(const f32x4 (&acc)[RB][TW],
                                                  const float (&bias)[TW], float* out, int po,
                                                  int n_base) {
  const int lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int t = 0; t < TW; ++t) {
      const int n = n_base + 16 * t + c;
      const float bn = bias[t];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 16 * rb + 4 * g + r;
        float v = acc[rb][t][r] + bn;
        v = v > 0.0f ? v : 0.0f;
        out[row * po + n] = v;
      }
    }
}

// row_epi_bias_relu that also returns the ReLU decisions of the lane's C elements as bits
// (bit (rb TW + t) 4 + r: the output is > 0), for the backward's masks
template <int RB, int TW>
__device__ __forceinline__ uint32_t row_epi_bias_relu_bits(const f32x4 (&acc)[RB][TW],
                                                           const float (&bias)[TW], float* out,
                                                           int po, int n_base) {
  static_assert(RB * TW * 4 <= 32, "mask bits: one 32-bit word per lane");
  const int lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
  uint32_t m = 0u;
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int t = 0; t < TW; ++t) {
      const int n = n_base + 16 * t + c;
      const float bn = bias[t];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 16 * rb + 4 * g + r;
        float v = acc[rb][t][r] + bn;
        v = v > 0.0f ? v : 0.0f;
        out[row * po + n] = v;
        m |= (v > 0.0f ? 1u : 0u) << ((rb * TW + t) * 4 + r);
      }
    }
  return m;
}

// the layer's output gradient through the ReLU decisions kept as bits (row_epi_bias_relu_bits)
// into the LDS image `out`: the same value row_epi_mask writes
template <int RB, int TW>
__device__ __forceinline__ void row_epi_maskbits(const f32x4 (&acc)[RB][TW], uint32_t m, float* out,
                                                 int po, int n_base) {
  const int lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int t = 0; t < TW; ++t) {
      const int n = n_base + 16 * t + c;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 16 * rb + 4 * g + r;
        out[row * po + n] = ((m >> ((rb * TW + t) * 4 + r)) & 1u) ? acc[rb][t][r] : 0.0f;
      }
    }
}

// bias + ReLU on the accumulators, kept in registers
template <int RB, int TW>
__device__ __forceinline__ void bias_relu_regs(f32x4 (&acc)[RB][TW], const float (&bias)[TW]) {
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int t = 0; t < TW; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v = acc[rb][t][r] + bias[t];
        acc[rb][t][r] = v > 0.0f ? v : 0.0f;
      }
}

// sum over the 16 lanes of each DPP row (every lane of the row gets the same total)
__device__ __forceinline__ float row16_sum(float v) {
  v = dpp_add<0xB1, 0xf>(v);   // quad_perm(1,0,3,2)
  v = dpp_add<0x4E, 0xf>(v);   // quad_perm(2,3,0,1)
  v = dpp_add<0x141, 0xf>(v);  // row_half_mirror
  v = dpp_add<0x140, 0xf>(v);  // row_mirror
  return v;
}

// the layer's output gradient through the ReLU mask of its forward activation, in place
template <int RB, int TW>
__device__ __forceinline__ void row_epi_mask(const f32x4 (&acc)[RB][TW], float* mask_inout, int pm,
                                             int n_base) {
  const int lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int t = 0; t < TW; ++t) {
      const int n = n_base + 16 * t + c;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 16 * rb + 4 * g + r;
        const float v = mask_inout[row * pm + n] > 0.0f ? acc[rb][t][r] : 0.0f;
        mask_inout[row * pm + n] = v;
      }
    }
}

// 16-B store of a row-kernel output (write-through sc1 stores measured no faster here)
__device__ __forceinline__ void st_f4(float* p, f32x4 v) { *reinterpret_cast<f32x4*>(p) = v; }

// rows 0 .. nrows-1 of an LDS image (pitch floats, ncols % 4 == 0) to HBM rows of ldg floats:
// whole 16-B segments, consecutive lanes on consecutive segments of a row
template <int NT, int RT>
__device__ __forceinline__ void rows_out(const float* img, int pitch, float* g, int ldg, int ncols,
                                         int nrows) {
  const int per_row = ncols / 4;
  for (int e = threadIdx.x; e < RT * per_row; e += NT) {
    const int row = e / per_row, c4 = (e - row * per_row) * 4;
    if (row < nrows)
      st_f4(g + (long)row * ldg + c4, *reinterpret_cast<const f32x4*>(&img[row * pitch + c4]));
  }
}

// The states gather of rows_forward, issued before the weight ring's first loads: vector memory
// completes in issue order, so a gather issued after the ring's prime waited for the prime's loads
// too.  Thread t holds elements t + i NT (row e / (Sp/4), float4 e % (Sp/4)) of the zero-padded
// RT x Sp image; rows_forward stores them.
template <int RT, int NT>
struct Gathered {
  static constexpr int N = RT * (kMaxRowS / 4) / NT;  // elements per thread at the widest S
  f32x4 v[N];
};
template <int RT, int NT>
__device__ __forceinline__ void gather_issue(const float* states, const int64_t* idx, int S,
                                             int nrows, int row0, int H, Gathered<RT, NT>& x) {
  int sbk, hbk;
  rows_blocks(S, H, &sbk, &hbk);
  const int q4 = 4 * sbk;  // Sp / 4
  const int t = threadIdx.x;
#pragma unroll
  for (int i = 0; i < Gathered<RT, NT>::N; ++i) {
    const int e = t + i * NT;
    f32x4 v = {0.0f, 0.0f, 0.0f, 0.0f};
    if (e < RT * q4) {
      const int row = e / q4, k = 4 * (e - row * q4);
      if (row < nrows && k < S) {
        const long src = idx ? (long)idx[row0 + row] : (long)(row0 + row);
        v = *reinterpret_cast<const f32x4*>(states + src * S + k);
      }
    }
    x.v[i] = v;
  }
}

// Forward of the RT rows starting at row0 (rows idx[row0 + i], or row0 + i without idx) into
// the LDS images X, H1, H2, AC = [a1 | c1]; optionally also to HBM (xg, h1, h2; null = no).
// X may alias AC (it is dead once h1 is computed).  Ends with a workgroup barrier.
// KEEP: [a1 | c1] stays in the layer-3 accumulators (a1 -> av, c1 -> cv, after bias and ReLU)
// instead of going to AC, and the function ends without the barrier.
// MSK: the ReLU decisions of h1 and h2 (this lane's C elements) also go to mb[0], mb[1] as bits
// (row_epi_bias_relu_bits), so the backward needs neither image for its masks.
template <int QH, int NW, int RT, bool KEEP, int D, int NSEG, bool TL, bool MSK = false,
          bool UNI = false>
__device__ __forceinline__ void rows_forward(WRing<H_TW(QH, NW), D, NSEG, TL, UNI>& R,
                                             const float* states,
                                             const int64_t* idx, int S, int nrows, int row0,
                                             const float* P, const int64_t* off, float* X,
                                             float* H1, float* H2, float* AC, float* xg,
                                             float* h1g, float* h2g, uint32_t (&mb)[2],
                                             f32x4 (&av)[RT / 16][H_TW(QH, NW)],
                                             f32x4 (&cv)[RT / 16][H_TW(QH, NW)] PSEC_PARAMS,
                                             const Gathered<RT, 64 * NW>* pre = nullptr) {
  constexpr int H = 64 * QH;
  constexpr int TW = H_TW(QH, NW);
  constexpr int NT = 64 * NW;
  constexpr int RB = RT / 16;
  constexpr int PH = lds_pitch(H), PA = lds_pitch(2 * H);
  const int t = threadIdx.x;
  // this wave's bias values of the four layers, loaded ahead of their epilogues
  float bias[4][TW];
  {
    const int c = t & 15;
    const int64_t bo[4] = {off[P_B1], off[P_B2], off[P_BA1], off[P_BC1]};
#pragma unroll
    for (int l = 0; l < 4; ++l)
#pragma unroll
      for (int u = 0; u < TW; ++u) bias[l][u] = P[bo[l] + R.n_base + 16 * u + c];
  }
  // zero-padded to whole ring groups of 16-deep blocks (the ring's layer-1 segment, rows_blocks)
  int sbk, hbk;
  rows_blocks(S, H, &sbk, &hbk);
  const int Sp = 16 * sbk, px = row_pitch(Sp);
  // states rows, zero-padded to Sp columns and RT rows (pre: gathered by gather_issue)
  if (pre) {
#pragma unroll
    for (int i = 0; i < Gathered<RT, NT>::N; ++i) {
      const int e = t + i * NT;
      if (e < RT * (Sp / 4)) {
        const int row = e / (Sp / 4), k = 4 * (e - row * (Sp / 4));
        const f32x4 v = pre->v[i];
        if (xg && row < nrows && k < S)
          *reinterpret_cast<f32x4*>(xg + (long)(row0 + row) * S + k) = v;
        *reinterpret_cast<f32x4*>(&X[row * px + k]) = v;
      }
    }
  } else {
    for (int e = t; e < RT * (Sp / 4); e += NT) {
      const int row = e / (Sp / 4), k = 4 * (e % (Sp / 4));
      f32x4 v = {0.0f, 0.0f, 0.0f, 0.0f};
      if (row < nrows && k < S) {
        const long src = idx ? (long)idx[row0 + row] : (long)(row0 + row);
        v = *reinterpret_cast<const f32x4*>(states + src * S + k);
        if (xg) *reinterpret_cast<f32x4*>(xg + (long)(row0 + row) * S + k) = v;
      }
      *reinterpret_cast<f32x4*>(&X[row * px + k]) = v;
    }
  }
  __syncthreads();
  PSEC(0);
  const int nb = R.n_base;  // this wave's output columns of an H-wide layer
  f32x4 acc[RB][TW];
  // h1 = relu(x W1^T + b1)
  zero_acc(acc);
  R.template run<0>(X, px, acc);
  if constexpr (MSK)
    mb[0] = row_epi_bias_relu_bits(acc, bias[0], H1, PH, nb);
  else
    row_epi_bias_relu(acc, bias[0], H1, PH, nb);
  __syncthreads();
  if (h1g) rows_out<NT, RT>(H1, PH, h1g + (long)row0 * H, H, H, nrows);
  PSEC(1);
  // h2 = relu(h1 W2^T + b2)
  zero_acc(acc);
  R.template run<1>(H1, PH, acc);
  if constexpr (MSK)  // H2 may alias X: every wave is past layer 1's reads (the barrier above)
    mb[1] = row_epi_bias_relu_bits(acc, bias[1], H2, PH, nb);
  else
    row_epi_bias_relu(acc, bias[1], H2, PH, nb);
  __syncthreads();
  if (h2g) rows_out<NT, RT>(H2, PH, h2g + (long)row0 * H, H, H, nrows);
  PSEC(2);
  // [a1 | c1] = relu(h2 [Wa1; Wc1]^T + [ba1; bc1])  (X may alias AC: X is dead since layer 1)
  if constexpr (KEEP) {
    zero_acc(av);
    R.template run<2>(H2, PH, av);
    bias_relu_regs(av, bias[2]);
    zero_acc(cv);
    R.template run<3>(H2, PH, cv);
    bias_relu_regs(cv, bias[3]);
    return;
  }
  zero_acc(acc);
  R.template run<2>(H2, PH, acc);
  row_epi_bias_relu(acc, bias[2], AC, PA, nb);
  zero_acc(acc);
  R.template run<3>(H2, PH, acc);
  row_epi_bias_relu(acc, bias[3], AC + H, PA, nb);
  __syncthreads();
}

// log1p(-tanh(z)^2 + 1e-6): the tanh-squash correction of the stored pre-tanh action z
// (ppo/agent.py squashed_log_prob), as the row kernels and the pre-gather compute it
__device__ __forceinline__ float squash_corr(float z) {
  return log1pf(-(tanhf(z) * tanhf(z)) + 1e-6f);
}

// CMP (compact LDS, H 256 at 32-row tiles): one region of two H-wide row images P0 | P1 holds,
// in turn, the states (P1), h1 (P0), h2 (P1), dac (across both, pitch PA), dh2 (P0) and dh1 (P1);
// the ReLU decisions of h1 / h2 stay in registers as bits.  72.6 KB instead of 139 KB, so two
// workgroups share a CU (4 waves per SIMD, <= 128 VGPRs) and one's phase boundaries, gather and
// loss head overlap the other's MFMAs.  One extra barrier: dh2 overwrites dac's image only after
// every wave has finished reading it.
template <int QH, int NW, int RT, bool CMP>
__device__ __forceinline__ void rows_body(const RowArgs& r) {
  constexpr int H = 64 * QH;
  constexpr int TW = H / NW / 16;        // 16-column output tiles per wave
  constexpr int RB = RT / 16;            // 16-row blocks per workgroup
  constexpr int RPW = RT / NW;           // loss-head rows per wave
  constexpr int NT = 64 * NW;            // threads
  static_assert(TW * 16 * NW == H, "H must split into 16-column tiles per wave");
  static_assert(RT % 16 == 0 && RPW >= 1 && RPW <= 16, "RT: whole 16-row blocks, <= 16 head rows per wave");
  constexpr int PH = lds_pitch(H), PA = lds_pitch(2 * H), PXMAX = lds_pitch(kMaxRowS);
  // the states image lives in [a1|c1] when its rows fit (it is dead before dac is written there)
  constexpr bool kOwnX = !CMP && PXMAX > PA;
  static_assert(!CMP || (PA <= 2 * PH && PXMAX <= PH), "CMP: dac spans P0 | P1, the states fit P1");
  __shared__ __attribute__((aligned(16))) float XX[kOwnX ? RT * PXMAX : 4];
  __shared__ __attribute__((aligned(16))) float H1[CMP ? 2 * RT * PH : RT * PH];  // CMP: P0 | P1
  __shared__ __attribute__((aligned(16))) float H2[CMP ? 4 : RT * PH];
  __shared__ __attribute__((aligned(16))) float ACI[CMP ? 4 : RT * PA];
  float* const P1 = CMP ? H1 + RT * PH : H2;  // h2 (and, CMP, the states, then dh1)
  float* const AC = CMP ? H1 : ACI;            // [a1 | c1] / dac image
  // the loss head works from the layer-3 accumulators: per-wave partial dot products of every
  // row, the per-row output scalars, the per-wave metric / bias / log_std sums
  __shared__ __attribute__((aligned(16))) f32x4 HDOT[NW][RT];
  __shared__ __attribute__((aligned(16))) f32x4 HROW[RT];
  __shared__ float HTAIL[NW][12];
  float* X = CMP ? P1 : (kOwnX ? XX : AC);
  PSEC_DECL
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int S = r.S;
  const int tile = blockIdx.x;
  const int row0 = tile * RT;
  const int nrows = min(RT, r.B - row0);
  const float* P = r.params;
  constexpr int D = CMP ? kRingDC : ring_depth<TW>();  // CMP: 4 waves per SIMD hide more
  WRing<TW, D, 7, true, CMP> R;
  ring_setup(R, P, r.off, S, H, w * (H / NW), r.tiles);
  // the loss head's inputs and weights, loaded now so that their latency hides behind the
  // forward: lane l < RPW of wave w holds row RPW*w + l; the head weights of this wave's
  // output columns nb + 16t + (lane & 15).  The row indices of the head and of
  // the states gather go out first, then the rows they name, then the weight ring's prime
  // (vector memory completes in issue order: a gather behind the prime waited for it)
  const int hl = min(RPW * w + min(lane, RPW - 1), nrows - 1);
  float hz0, hz1, hold, hadv, hret, hq0, hq1;
  Gathered<RT, NT> xpre;
  const long hsrc = (long)r.idx[row0 + hl];
  gather_issue<RT, NT>(r.states, r.idx, S, nrows, row0, H, xpre);
  hz0 = r.pre_tanh[hsrc * 2];
  hz1 = r.pre_tanh[hsrc * 2 + 1];
  hold = r.old_logp[hsrc];
  hadv = r.adv[hsrc];
  hret = r.ret[hsrc];
  R.prime();
  const int nb = w * (H / NW);  // this wave's output columns of an H-wide layer
  f32x4 acc[RB][TW];
  // the squash correction depends on the stored pre-tanh actions only: computed here, its
  // latency hides behind the forward instead of lengthening the loss head's dependent chain
  hq0 = squash_corr(hz0);
  hq1 = squash_corr(hz1);
  float wa0[TW], wa1[TW], wc[TW];
#pragma unroll
  for (int u = 0; u < TW; ++u) {
    const int col = w * (H / NW) + 16 * u + (lane & 15);
    wa0[u] = P[r.off[P_WA2] + col];
    wa1[u] = P[r.off[P_WA2] + H + col];
    wc[u] = P[r.off[P_WC2] + col];
  }
  const float ba0 = P[r.off[P_BA2]], ba1 = P[r.off[P_BA2] + 1], bcv = P[r.off[P_BC2]];
  const float ls0 = P[r.off[P_LOGSTD]], ls1 = P[r.off[P_LOGSTD] + 1];
  // torch Normal: scale = exp(log_std); var = scale**2; log_scale = log(scale) -- parameters
  // only, so computed here, off the loss head's dependent chain (same bits)
  const float sc0 = expf(ls0), sc1 = expf(ls1);
  const float var0 = sc0 * sc0, var1 = sc1 * sc1;
  const float lsc0 = logf(sc0), lsc1 = logf(sc1);
  f32x4 av[RB][TW], cv[RB][TW];  // a1, c1 of this wave's columns (C layout)
  uint32_t mb[2] = {0u, 0u};      // CMP: ReLU decisions of h1, h2 (this lane's C elements)
  rows_forward<QH, NW, RT, true, D, 7, true, CMP>(R, r.states, r.idx, S, nrows, row0, P, r.off, X,
                                                  H1, P1, AC, r.xg, r.h1,
                                                  r.h2, mb, av,
                                                  cv PSEC_ARGS, &xpre);
  PSEC(3);
  const int g4 = lane >> 4, c16 = lane & 15;

  // ---- loss head (ppo/agent.py:226-245).  (1) each wave's partial dot products a1 . wa2 and
  // c1 . wc2 of every row over its columns, from the layer-3 accumulators (16-lane DPP sums);
  // (2) the per-row scalar part, RPW rows per wave (lane = row), the partials summed in wave
  // order; (3) dL/d[a1|c1] of this wave's columns into the [a1|c1] image for dh2 and ppo_wgrad,
  // and the head-parameter gradients of its columns summed over the rows
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float p0 = 0.0f, p1 = 0.0f, pv = 0.0f;
#pragma unroll
      for (int u = 0; u < TW; ++u) {
        p0 += av[rb][u][q] * wa0[u];
        p1 += av[rb][u][q] * wa1[u];
        pv += cv[rb][u][q] * wc[u];
      }
      p0 = row16_sum(p0), p1 = row16_sum(p1), pv = row16_sum(pv);
      if (c16 == 0) HDOT[w][16 * rb + 4 * g4 + q] = f32x4{p0, p1, pv, 0.0f};
    }
  __syncthreads();
  PSEC(7);
  {
    const float LOG_SQRT_2PI = 0.91893853320467274178f;
    const float invB = 1.0f / (float)r.B;
    const float lo = 1.0f - r.eps_clip, hi = 1.0f + r.eps_clip;
    const int hr = RPW * w + min(lane, RPW - 1);  // this lane's row (lanes >= RPW: a copy)
    f32x4 dsum = HDOT[0][hr];
#pragma unroll
    for (int ww = 1; ww < NW; ++ww) dsum += HDOT[ww][hr];
    const float mu0 = dsum[0] + ba0, mu1 = dsum[1] + ba1, val = dsum[2] + bcv;
    const float d0 = hz0 - mu0, d1 = hz1 - mu1;
    const float lp0 = -(d0 * d0) / (2.0f * var0) - lsc0 - LOG_SQRT_2PI;
    const float lp1 = -(d1 * d1) / (2.0f * var1) - lsc1 - LOG_SQRT_2PI;
    const float logp = (lp0 - hq0) + (lp1 - hq1);
    const float log_ratio = logp - hold;
    const float ratio = expf(log_ratio);
    const float cr = fminf(fmaxf(ratio, lo), hi);
    const float s1 = ratio * hadv, s2 = cr * hadv;
    const float inr = (ratio >= lo && ratio <= hi) ? 1.0f : 0.0f;
    // torch.min / clamp backward: ties split the gradient evenly
    const float wsel = s1 < s2 ? 1.0f : (s1 > s2 ? inr : 0.5f * (1.0f + inr));
    const float dlogp = -invB * hadv * wsel * ratio;  // d(actor_loss)/d(logp)
    // rows past nrows (and lanes past RPW) contribute nothing
    const bool live = lane < RPW && hr < nrows;
    const float dmu0 = live ? dlogp * d0 / var0 : 0.0f;
    const float dmu1 = live ? dlogp * d1 / var1 : 0.0f;
    const float dv = live ? r.value_coef * 2.0f * (val - hret) * invB : 0.0f;
    if (lane < RPW) HROW[hr] = f32x4{dmu0, dmu1, dv, 0.0f};
    // this wave's rows' bias / log_std gradient terms and metrics, summed over its lanes in
    // lane order (the quad / half-row / row DPP tree over RPW <= 16 lanes)
    float tl[9] = {dmu0, dmu1, dv,
                   live ? dlogp * ((d0 * d0) / var0 - 1.0f) : 0.0f,
                   live ? dlogp * ((d1 * d1) / var1 - 1.0f) : 0.0f,
                   live ? -fminf(s1, s2) : 0.0f,
                   live ? (val - hret) * (val - hret) : 0.0f,
                   live ? (fabsf(ratio - 1.0f) > r.eps_clip ? 1.0f : 0.0f) : 0.0f,
                   live ? (ratio - 1.0f) - log_ratio : 0.0f};
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      const float v = row16_sum(lane < 16 ? tl[k] : 0.0f);
      if (lane == 0) HTAIL[w][k] = v;
    }
    if (blockIdx.x == 0 && t == 0) {
      r.counters[0] += 1;  // Adam step t for this minibatch
      r.counters[1] += 1;  // metrics row (this step writes row counters[1]-1)
    }
  }
  __syncthreads();
  PSEC(11);
  {
    // dac of this wave's columns (the reference's expression per element), and the head
    // weight gradients sum_rows dmu * a1 / dv * c1 of its columns: per lane over its rows, then
    // over the four 16-lane groups
    float ga0[TW], ga1[TW], gc[TW];
#pragma unroll
    for (int u = 0; u < TW; ++u) ga0[u] = ga1[u] = gc[u] = 0.0f;
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = 16 * rb + 4 * g4 + q;
        const f32x4 sc = HROW[row];
        const float dmu0 = sc[0], dmu1 = sc[1], dv = sc[2];
        float* arow = AC + row * PA;
#pragma unroll
        for (int u = 0; u < TW; ++u) {
          const int col = nb + 16 * u + c16;
          const float a = av[rb][u][q], cc = cv[rb][u][q];
          arow[col] = a > 0.0f ? (dmu0 * wa0[u] + dmu1 * wa1[u]) : 0.0f;
          arow[H + col] = cc > 0.0f ? dv * wc[u] : 0.0f;
          ga0[u] += dmu0 * a;
          ga1[u] += dmu1 * a;
          gc[u] += dv * cc;
        }
      }
    float* out = r.head_part + (long)tile * r.HP;
#pragma unroll
    for (int u = 0; u < TW; ++u) {
      // lanes c, c+16, c+32, c+48 hold the same column: (g0 + g1) + (g2 + g3)
      ga0[u] += __shfl_xor(ga0[u], 16);
      ga1[u] += __shfl_xor(ga1[u], 16);
      gc[u] += __shfl_xor(gc[u], 16);
      ga0[u] += __shfl_xor(ga0[u], 32);
      ga1[u] += __shfl_xor(ga1[u], 32);
      gc[u] += __shfl_xor(gc[u], 32);
      if (g4 == 0) {
        const int col = nb + 16 * u + c16;
        out[col] = ga0[u];
        out[H + col] = ga1[u];
        out[2 * H + col] = gc[u];
      }
    }
    if (w == 0 && lane < 9) {  // the waves' tail sums in wave order
      float v = HTAIL[0][lane];
#pragma unroll
      for (int ww = 1; ww < NW; ++ww) v += HTAIL[ww][lane];
      out[3 * H + lane] = v;
    }
  }
  __syncthreads();
  rows_out<NT, RT>(AC, PA, r.dac + (long)row0 * 2 * H, 2 * H, 2 * H, nrows);
  PSEC(4);
  // dh2 = (dac [Wa1; Wc1]) * (h2 > 0)   ([Wa1; Wc1] is [2H][H]: k-major); the two halves of
  // K = 2H (Wa1 rows, Wc1 rows) are summed at the end
  zero_acc(acc);
  R.template run<4>(AC, PA, acc);
  R.template run<5>(AC + H, PA, acc);
  float* const DH2 = CMP ? H1 : H2;  // CMP: P0
  float* const DH1 = CMP ? P1 : H1;
  if constexpr (CMP) {
    __syncthreads();  // every wave has read dac (P0 | P1)
    row_epi_maskbits(acc, mb[1], DH2, PH, nb);
  } else {
    row_epi_mask(acc, H2, PH, nb);
  }
  __syncthreads();
  if (r.dh2) rows_out<NT, RT>(DH2, PH, r.dh2 + (long)row0 * H, H, H, nrows);
  PSEC(5);
  // dh1 = (dh2 W2) * (h1 > 0)
  zero_acc(acc);
  R.template run<6>(DH2, PH, acc);
  if constexpr (CMP)
    row_epi_maskbits(acc, mb[0], DH1, PH, nb);  // P1: dac is dead, dh2 is in P0
  else
    row_epi_mask(acc, H1, PH, nb);  // dh1 over h1 (same thread)
  __syncthreads();
  if (r.dh1) rows_out<NT, RT>(DH1, PH, r.dh1 + (long)row0 * H, H, H, nrows);
  PSEC(6);
  PSEC_FLUSH;
}

template <int QH, int NW, int RT>
__global__ void __launch_bounds__(64 * NW, 1) ppo_rows(RowArgs r) {
  rows_body<QH, NW, RT, false>(r);
}

// the compact-LDS variant: two workgroups per CU, so at most 128 VGPRs (4 waves per SIMD)
template <int QH, int NW, int RT>
__global__ void __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(2 * NW / 4, 8)))
ppo_rows_c(RowArgs r) {
  CLK_BEGIN
  rows_body<QH, NW, RT, true>(r);
  CLK_END(0);
}

// the compact layout at 64-row tiles: 145 KB of LDS, one workgroup per CU (2 waves per SIMD,
// up to 256 VGPRs).  An fp32 MFMA fed by global_load_dwordx4 weight fragments sustains ~75 % of
// the matrix pipe at 8 MFMAs per fragment load (RB 2) and ~90 % at 16 (RB 4), 2 waves per SIMD
// (tools/micro/mfma_f32_rate.hip); the 64-row tile buys the second ratio
template <int QH, int NW>
__global__ void __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(NW / 4, 8)))
ppo_rows_c64(RowArgs r) {
  CLK_BEGIN
  rows_body<QH, NW, 64, true>(r);
  CLK_END(0);
}

// ----------------------------------------------------------------------------- acting
// ppo_act: ActorCritic.act for a batch of states (ppo/agent.py act(): forward, z = mean +
// exp(log_std) * eps, action = tanh(z), squashed Normal log-prob, value) -- the forward of
// ppo_rows followed by a per-row sampling head; noise = null is act(deterministic=True).
struct ActArgs {
  int B, S;
  const float* states;  // [B][S]
  const float* params;
  int64_t off[13];
  const float* noise;  // [B][2] standard normal, or null
  float *action, *pre_tanh, *logp, *value;
  const float* tiles;  // weight tile image in step with params (TL), else null
};

template <int QH, int NW, bool TL>
__device__ __forceinline__ void act_body(ActArgs r) {
  constexpr int H = 64 * QH;
  constexpr int RPW = kRowTile / NW;
  constexpr int PH = lds_pitch(H), PA = lds_pitch(2 * H), PXMAX = lds_pitch(kMaxRowS);
  __shared__ __attribute__((aligned(16))) float X[kRowTile * PXMAX];
  __shared__ __attribute__((aligned(16))) float H1[kRowTile * PH];
  __shared__ __attribute__((aligned(16))) float H2[kRowTile * PH];
  __shared__ __attribute__((aligned(16))) float AC[kRowTile * PA];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int row0 = blockIdx.x * kRowTile;
  const int nrows = min(kRowTile, r.B - row0);
  const float* P = r.params;
  constexpr int TW = H_TW(QH, NW);
  constexpr int D = ring_depth<TW>();
  WRing<TW, D, 4, TL> R;
  ring_setup(R, P, r.off, r.S, H, w * (H / NW), r.tiles);
  R.prime();
#ifdef HWY_SECTION_PROFILE
  uint64_t _pt = 0, _pacc[16];
#endif
  f32x4 unused_a[kRowTile / 16][TW], unused_c[kRowTile / 16][TW];
  uint32_t unused_m[2];
  rows_forward<QH, NW, kRowTile, false>(R, r.states, nullptr, r.S, nrows, row0, P, r.off, X, H1,
                                        H2, AC, nullptr, nullptr, nullptr, unused_m, unused_a,
                                        unused_c PSEC_ARGS);
  float wa0[QH], wa1[QH], wc[QH];
#pragma unroll
  for (int q = 0; q < QH; ++q) {
    const int col = lane + 64 * q;
    wa0[q] = P[r.off[P_WA2] + col];
    wa1[q] = P[r.off[P_WA2] + H + col];
    wc[q] = P[r.off[P_WC2] + col];
  }
  const float ba0 = P[r.off[P_BA2]], ba1 = P[r.off[P_BA2] + 1], bcv = P[r.off[P_BC2]];
  const float ls0 = P[r.off[P_LOGSTD]], ls1 = P[r.off[P_LOGSTD] + 1];
  const float sc0 = expf(ls0), sc1 = expf(ls1);
  const float var0 = sc0 * sc0, var1 = sc1 * sc1;
  const float lsc0 = logf(sc0), lsc1 = logf(sc1);
  const float LOG_SQRT_2PI = 0.91893853320467274178f;
  for (int rr = 0; rr < RPW; ++rr) {
    const int lr = RPW * w + rr;
    if (lr >= nrows) break;
    const int b = row0 + lr;
    const float* arow = AC + lr * PA;
    float p0 = 0.0f, p1 = 0.0f, pv = 0.0f;
#pragma unroll
    for (int q = 0; q < QH; ++q) {
      const int col = lane + 64 * q;
      const float a = arow[col], c = arow[H + col];
      p0 += a * wa0[q];
      p1 += a * wa1[q];
      pv += c * wc[q];
    }
    const float mu0 = wave_sum_dpp(p0) + ba0, mu1 = wave_sum_dpp(p1) + ba1,
                val = wave_sum_dpp(pv) + bcv;
    if (lane == 0) {
      float z0 = mu0, z1 = mu1, lp = 0.0f;
      if (r.noise) {
        z0 = mu0 + sc0 * r.noise[2 * (long)b];
        z1 = mu1 + sc1 * r.noise[2 * (long)b + 1];
        const float d0 = z0 - mu0, d1 = z1 - mu1;
        const float t0 = tanhf(z0), t1 = tanhf(z1);
        const float lp0 = -(d0 * d0) / (2.0f * var0) - lsc0 - LOG_SQRT_2PI;
        const float lp1 = -(d1 * d1) / (2.0f * var1) - lsc1 - LOG_SQRT_2PI;
        lp = (lp0 - log1pf(-(t0 * t0) + 1e-6f)) + (lp1 - log1pf(-(t1 * t1) + 1e-6f));
      }
      r.action[2 * (long)b] = tanhf(z0);
      r.action[2 * (long)b + 1] = tanhf(z1);
      r.pre_tanh[2 * (long)b] = z0;
      r.pre_tanh[2 * (long)b + 1] = z1;
      r.logp[b] = lp;
      r.value[b] = val;
    }
  }
}

template <int QH, int NW, bool TL>
__global__ void __launch_bounds__(64 * NW, 1) ppo_act(ActArgs r) {
  act_body<QH, NW, TL>(r);
}

// ppo_act_c: ppo_act at H = 256 in the compact layout of ppo_rows_c -- the states / h1 / h2
// images in two H-wide regions (P0 | P1: 71 KB with the head partials at 32-row tiles, 36 KB at
// 16), [a1 | c1] kept in the layer-3 accumulators, <= 128 VGPRs: two workgroups per CU.
// The head is ppo_rows_c's: per-wave partial dot products of every row over the wave's columns,
// summed in wave order, so mean / value are the bits the minibatch step recomputes.
// (A 4-deep ring with the one-workgroup-per-CU register budget at 4,096 rows measured 22.4 against
// 21.9 us, round 5.)
template <int QH, int NW, int RT>
__device__ __forceinline__ void act_c_body(ActArgs r) {
  constexpr int H = 64 * QH;
  constexpr int TW = H / NW / 16;
  constexpr int RB = RT / 16;
  constexpr int RPW = RT / NW;
  constexpr int PH = lds_pitch(H), PXMAX = lds_pitch(kMaxRowS);
  static_assert(TW * 16 * NW == H && PXMAX <= PH && RPW >= 1 && RPW <= 16, "ppo_act_c geometry");
  __shared__ __attribute__((aligned(16))) float P01[2 * RT * PH];
  __shared__ __attribute__((aligned(16))) f32x4 HDOT[NW][RT];
  float* const H1 = P01;            // P0
  float* const P1 = P01 + RT * PH;  // the states, then h2
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int row0 = blockIdx.x * RT;
  const int nrows = min(RT, r.B - row0);
  const float* P = r.params;
  constexpr int D = kRingDC;
  WRing<TW, D, 4, true, true> R;
  ring_setup(R, P, r.off, r.S, H, w * (H / NW), r.tiles);
  Gathered<RT, 64 * NW> xpre;  // the states rows, issued before the ring's prime (rows_body)
  gather_issue<RT, 64 * NW>(r.states, nullptr, r.S, nrows, row0, H, xpre);
  R.prime();
#ifdef HWY_SECTION_PROFILE
  uint64_t _pt = 0, _pacc[16];
#endif
  float wa0[TW], wa1[TW], wc[TW];
#pragma unroll
  for (int u = 0; u < TW; ++u) {
    const int col = w * (H / NW) + 16 * u + (lane & 15);
    wa0[u] = P[r.off[P_WA2] + col];
    wa1[u] = P[r.off[P_WA2] + H + col];
    wc[u] = P[r.off[P_WC2] + col];
  }
  const float ba0 = P[r.off[P_BA2]], ba1 = P[r.off[P_BA2] + 1], bcv = P[r.off[P_BC2]];
  const float ls0 = P[r.off[P_LOGSTD]], ls1 = P[r.off[P_LOGSTD] + 1];
  // this lane's head row (lanes < RPW of wave w: row RPW w + lane) and its noise
  const int hr = RPW * w + min(lane, RPW - 1);
  const bool live = lane < RPW && hr < nrows;
  const long b = row0 + min(hr, nrows - 1);
  float n0 = 0.0f, n1 = 0.0f;
  if (r.noise) n0 = r.noise[2 * b], n1 = r.noise[2 * b + 1];
  f32x4 av[RB][TW], cv[RB][TW];
  uint32_t mb[2] = {0u, 0u};
  rows_forward<QH, NW, RT, true, D, 4, true, false>(R, r.states, nullptr, r.S, nrows, row0, P,
                                                     r.off, P1, H1, P1, nullptr, nullptr,
                                                     nullptr, nullptr, mb, av, cv PSEC_ARGS,
                                                     &xpre);
  const int g4 = lane >> 4, c16 = lane & 15;
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float p0 = 0.0f, p1 = 0.0f, pv = 0.0f;
#pragma unroll
      for (int u = 0; u < TW; ++u) {
        p0 += av[rb][u][q] * wa0[u];
        p1 += av[rb][u][q] * wa1[u];
        pv += cv[rb][u][q] * wc[u];
      }
      p0 = row16_sum(p0), p1 = row16_sum(p1), pv = row16_sum(pv);
      if (c16 == 0) HDOT[w][16 * rb + 4 * g4 + q] = f32x4{p0, p1, pv, 0.0f};
    }
  __syncthreads();
  if (!live) return;
  f32x4 dsum = HDOT[0][hr];
#pragma unroll
  for (int ww = 1; ww < NW; ++ww) dsum += HDOT[ww][hr];
  const float mu0 = dsum[0] + ba0, mu1 = dsum[1] + ba1, val = dsum[2] + bcv;
  float z0 = mu0, z1 = mu1, lp = 0.0f;
  if (r.noise) {
    // torch Normal: scale = exp(log_std); var = scale**2; log_scale = log(scale)
    const float sc0 = expf(ls0), sc1 = expf(ls1);
    const float var0 = sc0 * sc0, var1 = sc1 * sc1;
    const float lsc0 = logf(sc0), lsc1 = logf(sc1);
    const float LOG_SQRT_2PI = 0.91893853320467274178f;
    z0 = mu0 + sc0 * n0;
    z1 = mu1 + sc1 * n1;
    const float d0 = z0 - mu0, d1 = z1 - mu1;
    const float t0 = tanhf(z0), t1 = tanhf(z1);
    const float lp0 = -(d0 * d0) / (2.0f * var0) - lsc0 - LOG_SQRT_2PI;
    const float lp1 = -(d1 * d1) / (2.0f * var1) - lsc1 - LOG_SQRT_2PI;
    lp = (lp0 - log1pf(-(t0 * t0) + 1e-6f)) + (lp1 - log1pf(-(t1 * t1) + 1e-6f));
  }
  r.action[2 * b] = tanhf(z0);
  r.action[2 * b + 1] = tanhf(z1);
  r.pre_tanh[2 * b] = z0;
  r.pre_tanh[2 * b + 1] = z1;
  r.logp[b] = lp;
  r.value[b] = val;
}

template <int QH, int NW, int RT>
__global__ void __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(2 * NW / 4, 8)))
ppo_act_c(ActArgs r) {
  act_c_body<QH, NW, RT>(r);
}

// ----------------------------------------------------------------------------- weight grads
// ppo_wgrad: every weight gradient of the minibatch step (the autograd of ppo/agent.py:241-248
// for the four hidden layers), the bias column sums, the head-parameter sums over the ppo_rows
// partials, the metrics row and the sum-of-squares partials of clip_grad_norm_ (:249-251).
//
// Output tiles are 128 x 64 (dWac = dac^T h2: rows < H -> Wa1, >= H -> Wc1; dW2 = dh2^T h1;
// dW1 = dh1^T gather(states)).  Workgroup id = tile * split + z: slice z of the minibatch rows
// (B / split rows, split = 8 at the bench shapes) goes to workgroup id % 8 = the XCD the
// dispatcher places it on, so each XCD reads one 1/8 row slice (~3 MB at B = 4096, H = 256) and
// keeps it in its own L2 across all the tiles.  One 512-thread workgroup per CU (8 waves, 2 per
// SIMD); the two waves of a SIMD own the same 64 x 32 output block as two 32x32
// v_mfma_f32_32x32x2_f32 accumulators sharing the B operand, over the two row halves of every
// 64-row chunk (summed through LDS at the end).  The chunks are staged by LDS-DMA
// (wgrad_tile_dma: three buffers, two chunks in flight).
//
// The split partial tiles go to a slab that ppo_wsum sums in split order (the kernel
// boundary is the one L2 writeback that makes the other XCDs' partials visible; a last-arriver
// reduction inside this kernel paid an agent-scope L2 writeback per workgroup, ~20 us).
struct WgArgs {
  int B, S, H;
  const float *dac, *h2, *dh2, *h1, *dh1, *xg;
  float* grads;
  int64_t off[13];
  const float* head_part;
  int nhp, HP;
  float* norm_part;     // [nh] head-sum partials, then [ntile] tile partials
  int tac, t2, t1, nh;  // 128x64 tiles per region, head-sum workgroups
  int split;            // minibatch-row slices per tile (one per XCD at the bench shapes)
  int bal, wm, tpe, nslot;  // balanced partition (ppo_wgrad): main chunks, tail tiles per extra
  float* slab;          // [tiles][split][nslot][128*64 + 128] partial tiles + bias partials
  float entropy_coef, value_coef, ent_const;
  const float* params;
  float* metrics;
  int32_t* counters;
};

template <int NW = 4>
__device__ __forceinline__ float block_sum4(float v, float* red) {
  const int t = threadIdx.x;
  v = wave_sum_dpp(v);
  __syncthreads();
  if ((t & 63) == 0) red[t >> 6] = v;
  __syncthreads();
  float s = red[0];
#pragma unroll
  for (int i = 1; i < NW; ++i) s += red[i];
  return s;
}

// head parameters (the ppo_rows partials summed in row-block order) + the metrics row
__device__ void wgrad_head(const WgArgs& a, int hid, float* lds, float* red) {
  float(*tile)[64] = reinterpret_cast<float(*)[64]>(lds);
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, H = a.H;
  const int e = hid * 64 + lane;
  const int ne = 3 * H + 9;
  const int per = (a.nhp + kWgWaves - 1) / kWgWaves, p0 = w * per, p1 = min(a.nhp, p0 + per);
  float s = 0.0f, sq = 0.0f;
  if (e < ne) {
    for (int pb = p0; pb < p1; pb += 16) {  // 16 loads in flight, summed in row order
      float pv[16];
#pragma unroll
      for (int u = 0; u < 16; ++u)
        pv[u] = pb + u < p1 ? a.head_part[(long)(pb + u) * a.HP + e] : 0.0f;
#pragma unroll
      for (int u = 0; u < 16; ++u) s += pv[u];
    }
  }
  tile[w][lane] = s;
  __syncthreads();
  if (t < 64 && e < ne) {
    float g = tile[0][t];
#pragma unroll
    for (int i = 1; i < kWgWaves; ++i) g += tile[i][t];
    long dst = -1;
    float gv = g;
    if (e < 2 * H) {
      dst = a.off[P_WA2] + e;
    } else if (e < 3 * H) {
      dst = a.off[P_WC2] + (e - 2 * H);
    } else {
      const int k = e - 3 * H;
      if (k < 2) dst = a.off[P_BA2] + k;
      else if (k == 2) dst = a.off[P_BC2];
      else if (k < 5) dst = a.off[P_LOGSTD] + (k - 3), gv = g - a.entropy_coef;
    }
    if (dst >= 0) {
      a.grads[dst] = gv;
      sq = gv * gv;
    }
    tile[0][t] = g;  // keep the totals for the metrics row
  }
  const float tot = block_sum4<kWgWaves>(sq, red);
  if (t == 0) a.norm_part[hid] = tot;
  if (3 * H >= e - lane && 3 * H < e - lane + 64 && t == 0) {
    // metrics row (ppo/agent.py:255-262): policy, value, entropy, loss, clip count, kl
    const int k0 = 3 * H - (e - lane);
    const float pg = tile[0][k0 + 5], vf = tile[0][k0 + 6], clip = tile[0][k0 + 7],
                kl = tile[0][k0 + 8];
    const float invB = 1.0f / (float)a.B;
    const float ls0 = a.params[a.off[P_LOGSTD]], ls1 = a.params[a.off[P_LOGSTD] + 1];
    const float ent = (a.ent_const + logf(expf(ls0))) + (a.ent_const + logf(expf(ls1)));
    float* m = a.metrics + (int64_t)(a.counters[1] - 1) * 6;
    m[0] = pg * invB;
    m[1] = vf * invB;
    m[2] = ent;
    m[3] = (pg * invB + a.value_coef * (vf * invB)) - a.entropy_coef * ent;
    m[4] = clip;
    m[5] = kl * invB;
  }
}

#define WG_ST(p, v) (*(p) = (v))  // (nontemporal partial stores measured slower in ppo_wsum)

typedef __attribute__((address_space(3))) void lds_void_t;

// ppo_wgrad's chunk loop with LDS-DMA staging.  Chunks of 64 rows go
// global -> LDS by global_load_lds_dwordx4 (1 KB per wave instruction, no VGPRs, no VALU) into
// row-major images: A = 64 rows x 128 features (32 pieces of 2 rows), B = 64 rows x 64 features
// (16 pieces of 4 rows); each wave issues 4 A and 2 B pieces per chunk.  Odd rows are stored
// rotated by 32 floats (the rotation goes on the per-lane SOURCE address: the DMA destination is
// lane-linear), so the MFMA operand reads -- one ds_read_b32 per operand and k-step, lanes 0-31
// row 2s, lanes 32-63 row 2s + 1 of the same 32 features -- hit 64 distinct banks.  Three
// buffers: chunk c + 2 is issued right after the barrier that opens chunk c (every wave has
// finished reading chunk c - 1, whose buffer it reuses), and stays in flight across the next
// barrier (counted vmcnt, raw s_barrier).  The register-staged loop spent 14 us of a 75 us
// launch in its transposing staging (timing-only build without it: 61 us).
// The A column sums (bias gradients) come from the A operand values in registers.
__device__ __forceinline__ void wgrad_tile_dma(const WgArgs& a, int tile_id, int kb0, int kb1,
                                               float* part, float* wg_lds PSEC_PARAMS) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, h = lane >> 5, l32 = lane & 31;
  const int H = a.H;
  if (kb1 <= kb0) {
    for (int i = t; i < kWgPart; i += 64 * kWgWaves) part[i] = 0.0f;
    return;
  }
  int id = tile_id;
  const float *A, *Bm;
  int lda, ldb, M, N, ntj;
  if (id < a.tac) {  // dWac = dac^T h2
    A = a.dac, lda = 2 * H, Bm = a.h2, ldb = H, M = 2 * H, N = H;
  } else if (id < a.tac + a.t2) {  // dW2 = dh2^T h1
    id -= a.tac;
    A = a.dh2, lda = H, Bm = a.h1, ldb = H, M = H, N = H;
  } else {  // dW1 = dh1^T x (gathered states rows written by ppo_rows)
    id -= a.tac + a.t2;
    A = a.dh1, lda = H, Bm = a.xg, ldb = a.S, M = H, N = a.S;
  }
  ntj = (N + kWgTN - 1) / kWgTN;
  const int ti = id / ntj, tj = id % ntj;
  const int i0 = ti * kWgTM, j0 = tj * kWgTN;
  const int nchunk = (kb1 - kb0 + 63) / 64;  // >= 1
  constexpr int BUF = (kWgTM + kWgTN) * 64;  // floats per chunk buffer (48 KB)

  // DMA sources (element offsets from the wave-uniform bases; 32 bits suffice).  A piece 4w + i:
  // rows 2(4w + i) + h, lanes l32 -> feature quad l32 (even row) / (l32 - 8) & 31 (odd row);
  // B piece 2w + i: rows 4(2w + i) + (lane >> 4), quad lane & 15 / (lane - 8) & 15 (odd row).
  // Rows past the range load the last row (zeroed in the operands below); features past M / N
  // load in-range duplicates whose outputs are never stored.
  const int rb = lane >> 4, qb = lane & 15;
  const uint32_t a_col = (uint32_t)min(i0 + 4 * (h ? ((l32 - 8) & 31) : l32), M - 4);
  const uint32_t b_col = (uint32_t)min(j0 + 4 * ((rb & 1) ? ((qb - 8) & 15) : qb), N - 4);
  // part 0: A pieces 0-1, part 1: A pieces 2-3, part 2: the two B pieces; -1: all three
  auto dma = [&](int c, float* buf, int part = -1) {
    const int k0 = kb0 + 64 * c;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (part >= 0 && part != i / 2) continue;
      const uint32_t row = (uint32_t)min(k0 + 2 * (4 * w + i) + h, kb1 - 1);
      __builtin_amdgcn_global_load_lds((const void*)(A + (row * (uint32_t)lda + a_col)),
                                       (lds_void_t*)(buf + (4 * w + i) * 256), 16, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      if (part >= 0 && part != 2) continue;
      const uint32_t row = (uint32_t)min(k0 + 4 * (2 * w + i) + rb, kb1 - 1);
      __builtin_amdgcn_global_load_lds((const void*)(Bm + (row * (uint32_t)ldb + b_col)),
                                       (lds_void_t*)(buf + kWgTM * 64 + (2 * w + i) * 256), 16,
                                       0, 0);
    }
  };
  // MFMA: waves w and w + 4 (one SIMD) own the same 64 x 32 output block (two 32x32
  // accumulators sharing the B operand), over rows 0-31 / 32-63 of every chunk.
  const int kh = w >> 2, wq = w & 3;
  const int wm = (wq & 1) * 64, wn = (wq >> 1) * 32;
  // per-lane operand offsets within a chunk image (row 2s + h, rotated odd rows)
  const int offa0 = h * 128 + ((wm + l32 + 32 * h) & 127);
  const int offa1 = h * 128 + ((wm + 32 + l32 + 32 * h) & 127);
  const int offb = kWgTM * 64 + h * 64 + ((wn + l32 + 32 * h) & 63);
  f32x16 acc0, acc1;
#pragma unroll
  for (int q = 0; q < 16; ++q) acc0[q] = acc1[q] = 0.0f;
  float bs0 = 0.0f, bs1 = 0.0f;  // A column sums of this lane's features over its rows
  // dc / dbuf: the chunk whose DMAs go out between this chunk's MFMA groups (dc < 0: none);
  // issued all at once after the barrier, both waves of a SIMD issued them together (round 4:
  // 203.4 -> 201.5 us per 16,384-row step with the activation reads pinned, same weights)
  auto compute = [&](const float* buf, int lim, auto mask_tag, int dc, float* dbuf) {
    constexpr bool MASK = decltype(mask_tag)::value;  // rows >= lim (of the chunk) are zero
    const float* pa0 = buf + offa0 + 32 * kh * 128;
    const float* pa1 = buf + offa1 + 32 * kh * 128;
    const float* pb = buf + offb + 32 * kh * 64;
    float x0[2][4], x1[2][4], y[2][4];
    auto rd = [&](int g, int b) {  // k-steps 4g .. 4g + 3 of this wave's 16
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int st = 4 * g + j;
        x0[b][j] = pa0[st * 256];
        x1[b][j] = pa1[st * 256];
        y[b][j] = pb[st * 128];
      }
    };
    rd(0, 0);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int b = g & 1;
      // the next group's reads go out before this group's MFMAs (pinned: the scheduler would
      // otherwise sink them to their use and wait for them there)
      if (g + 1 < 4) rd(g + 1, b ^ 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float u0 = x0[b][j], u1 = x1[b][j];
        if constexpr (MASK) {
          const bool live = 32 * kh + 2 * (4 * g + j) + h < lim;
          u0 = live ? u0 : 0.0f;
          u1 = live ? u1 : 0.0f;
        }
        bs0 += u0;
        bs1 += u1;
        acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(u0, y[b][j], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(u1, y[b][j], acc1, 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
      if (g < 3 && dc >= 0) {
        dma(dc, dbuf, g);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };
  const std::integral_constant<bool, true> masked;
  const std::integral_constant<bool, false> unmasked;
  float* b0 = wg_lds;
  float* b1 = wg_lds + BUF;
  float* b2 = wg_lds + 2 * BUF;
  // earlier stores of this wave (a previous tile's partial) drained: the vmcnt counts are exact
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  dma(0, b0);
  if (nchunk > 1) dma(1, b1);
  auto step = [&](int c, auto mask_tag) {
    // this wave's pieces of chunk c landed (chunk c + 1's 6 may still be in flight) and its
    // reads of chunk c - 1 returned; after the barrier, every wave's
    if (c + 1 < nchunk)
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    // chunk c + 2 into chunk c - 1's buffer, spread between this chunk's MFMA groups
    compute(b0, kb1 - (kb0 + 64 * c), mask_tag, c + 2 < nchunk ? c + 2 : -1, b2);
    float* tb = b0;
    b0 = b1, b1 = b2, b2 = tb;
  };
  // whole chunks, then (ragged minibatches only) the last, partial one with its rows masked
  const int nfull = (kb1 - kb0) / 64;
  for (int c = 0; c < nfull; ++c) step(c, unmasked);
  if (nfull < nchunk) step(nfull, masked);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  PSEC(8);
  // bias sums over the wave's two row halves (lanes l, l + 32), then the two waves of a SIMD
  bs0 += __shfl_xor(bs0, 32);
  bs1 += __shfl_xor(bs1, 32);
  // waves 4-7 hand their accumulators (and bias sums) to waves 0-3 through LDS
  float* xch = wg_lds;                    // [4 waves][32 floats][64 lanes]
  float* bx = wg_lds + 4 * 32 * 64;       // [4 waves][2][32]
  if (kh == 1) {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      xch[(wq * 32 + q) * 64 + lane] = acc0[q];
      xch[(wq * 32 + 16 + q) * 64 + lane] = acc1[q];
    }
    if (h == 0) {
      bx[(wq * 2) * 32 + l32] = bs0;
      bx[(wq * 2 + 1) * 32 + l32] = bs1;
    }
  }
  __syncthreads();
  if (kh == 0) {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int ri = wm + (q & 3) + 8 * (q >> 2) + 4 * h;
      WG_ST(&part[ri * kWgTN + wn + l32], acc0[q] + xch[(wq * 32 + q) * 64 + lane]);
      WG_ST(&part[(ri + 32) * kWgTN + wn + l32], acc1[q] + xch[(wq * 32 + 16 + q) * 64 + lane]);
    }
    if (tj == 0 && wn == 0 && h == 0) {  // waves 0, 1: features wm .. wm + 63
      WG_ST(&part[kWgTM * kWgTN + wm + l32], bs0 + bx[(wq * 2) * 32 + l32]);
      WG_ST(&part[kWgTM * kWgTN + wm + 32 + l32], bs1 + bx[(wq * 2 + 1) * 32 + l32]);
    }
  }
  PSEC(9);
}

#define WGRAD_TILE wgrad_tile_dma

// Workgroups.  Default: tile * split + z -> tile `tile`, row slice z (rows [z ceil(B / split),
// ...)), then the head-sum workgroups.  Slice z goes to workgroups with id % 8 = z, i.e. to one
// XCD (the dispatcher deals workgroups to the 8 XCDs round-robin), so each XCD reads one slice
// of the activations and serves all its tiles from its own L2.
// Balanced (a.bal; e.g. 26 tiles x 8 slices would leave 48 of 256 CUs idle): 256 / split
// workgroups per slice.  Workgroup j < ntile takes tile j over the slice's first wm chunks, in
// lockstep with the other tiles (the XCD's L2 holds the chunks they share); the remaining
// 256 / split - ntile "extras" take the other chunks of tpe tiles each (those chunks stay
// L2-resident while an extra walks its tiles), into a second partial slot; the last extra of
// each slice also runs the head sums.
__device__ __forceinline__ void ppo_wgrad_body(const WgArgs& a) {
  PSEC_DECL
  // one LDS array (a second __shared__ object beside the LDS-DMA images can make the compiler
  // drain every DMA before the first operand read of a chunk): the chunk buffers, then the
  // reduction slots
  constexpr int kWgBufs = 3;
  __shared__ __attribute__((aligned(16))) float wg_lds[kWgBufs * (kWgTM + kWgTN) * 64 + kWgWaves + 2];
  float* red = wg_lds + kWgBufs * (kWgTM + kWgTN) * 64;
  const int ntile = a.tac + a.t2 + a.t1;
  const int id = blockIdx.x;
  const int rows = (a.B + a.split - 1) / a.split;
  if (!a.bal) {
    if (id >= ntile * a.split) {  // ---- head parameters + metrics
      wgrad_head(a, id - ntile * a.split, wg_lds, red);
      PSEC(10);
      PSEC_FLUSH;
      return;
    }
    const int z = id % a.split, tile = id / a.split;
    const int kb0 = z * rows, kb1 = min(a.B, kb0 + rows);
    WGRAD_TILE(a, tile, kb0, kb1, a.slab + ((long)tile * a.split + z) * kWgPart,
               wg_lds PSEC_ARGS);
    PSEC_FLUSH;
    return;
  }
  const int z = id % a.split, j = id / a.split;
  const int kz = min(a.B, z * rows), kz1 = min(a.B, kz + rows), km = min(kz1, kz + 64 * a.wm);
  auto slot = [&](int tile, int sl) {
    return a.slab + (((long)tile * a.split + z) * a.nslot + sl) * kWgPart;
  };
  if (j < ntile) {
    WGRAD_TILE(a, j, kz, km, slot(j, 0), wg_lds PSEC_ARGS);
  } else {
    const int e = j - ntile, nextra = (int)gridDim.x / a.split - ntile;
    const int t0 = min(ntile, e * a.tpe), t1 = min(ntile, t0 + a.tpe);
    for (int tile = t0; tile < t1; ++tile) {
      if (tile > t0) __syncthreads();  // the last segment's accumulator exchange used the LDS
      WGRAD_TILE(a, tile, km, kz1, slot(tile, 1), wg_lds PSEC_ARGS);
    }
    if (e == nextra - 1) {
      for (int hid = z; hid < a.nh; hid += a.split) {
        __syncthreads();
        wgrad_head(a, hid, wg_lds, red);
      }
      PSEC(10);
    }
  }
  PSEC_FLUSH;
}

__global__ void __launch_bounds__(512) ppo_wgrad(WgArgs a) {
  CLK_BEGIN
  ppo_wgrad_body(a);
  CLK_END(1);
}

// One ppo_wsum work item (1024 elements of a weight-gradient tile, 16 tile rows): the split
// partial tiles summed in split order (deterministic) into the flat gradient, with all splits'
// float4s in flight per thread, and the bias sums of the tile's rows (work item 0 of the tile's
// first column).  Returns this thread's sum of squares of what it wrote.
__device__ __forceinline__ float wsum_item(const WgArgs& a, int item) {
  const int t = threadIdx.x, H = a.H;
  constexpr int kParts = kWgTM * kWgTN / 1024;
  const int tile_id = item / kParts, part = item % kParts;
  int id = tile_id, M, N, region;
  if (id < a.tac) {
    M = 2 * H, N = H, region = 0;
  } else if (id < a.tac + a.t2) {
    id -= a.tac, M = H, N = H, region = 1;
  } else {
    id -= a.tac + a.t2, M = H, N = a.S, region = 2;
  }
  const int ntj = (N + kWgTN - 1) / kWgTN;
  const int ti = id / ntj, tj = id % ntj, i0 = ti * kWgTM, j0 = tj * kWgTN;
  auto grad_row = [&](int i) -> long {  // flat index of row i (of M) of this region's weight
    if (region == 0) return i < H ? a.off[P_WA1] + (long)i * H : a.off[P_WC1] + (long)(i - H) * H;
    if (region == 1) return a.off[P_W2] + (long)i * H;
    return a.off[P_W1] + (long)i * a.S;
  };
  const float* sl = a.slab + (long)tile_id * a.split * a.nslot * kWgPart;
  const int e = part * 1024 + 4 * t, ri = e / kWgTN, cj = e % kWgTN;
  constexpr int kMaxParts = 16;  // 8 slices x 2 slots
  const int np = a.split * a.nslot;
  f32x4 pv[kMaxParts];
#pragma unroll
  for (int q = 0; q < kMaxParts; ++q)
    if (q < np) pv[q] = *reinterpret_cast<const f32x4*>(sl + (long)q * kWgPart + e);
  // the bias partials of output row i0 + t load in the same round trip as the tile's
  const bool bias_t = part == 0 && tj == 0 && t < kWgTM && i0 + t < M;
  float bp[kMaxParts];
#pragma unroll
  for (int q = 0; q < kMaxParts; ++q)
    bp[q] = (bias_t && q < np) ? sl[(long)q * kWgPart + kWgTM * kWgTN + t] : 0.0f;
  // summed in (slice, slot) order
  f32x4 v = pv[0];
#pragma unroll
  for (int q = 1; q < kMaxParts; ++q)
    if (q < np) v += pv[q];
  float sq = 0.0f;
  if (i0 + ri < M) {
    const long row = grad_row(i0 + ri) + j0 + cj;
    float* dst = a.grads + row;
#pragma unroll
    for (int c4 = 0; c4 < 4; ++c4)
      if (j0 + cj + c4 < N) {
        dst[c4] = v[c4];
        sq += v[c4] * v[c4];
      }
  }
  if (bias_t) {  // bias of output row i0 + t
    float b = 0.0f;
#pragma unroll
    for (int q = 0; q < kMaxParts; ++q)
      if (q < np) b += bp[q];
    const int i = i0 + t;
    long bo;
    if (region == 0) bo = i < H ? a.off[P_BA1] + i : a.off[P_BC1] + (i - H);
    else if (region == 1) bo = a.off[P_B2] + i;
    else bo = a.off[P_B1] + i;
    a.grads[bo] = b;
    sq += b * b;
  }
  return sq;
}

// ppo_wsum: every work item of every weight-gradient tile, one sum-of-squares partial each
__device__ __forceinline__ void wsum_body(const WgArgs& a) {
  __shared__ float red[4];
  const float tot = block_sum4(wsum_item(a, blockIdx.x), red);
  if (threadIdx.x == 0) a.norm_part[a.nh + blockIdx.x] = tot;
}

__global__ void __launch_bounds__(256) ppo_wsum(WgArgs a) { wsum_body(a); }

// ----------------------------------------------------------------------------- reduce
struct RedDesc {
  const float* src;
  int64_t stride;  // floats between consecutive partials
  int32_t nsplit;
  int64_t numel;
  int64_t dst;
};
struct RedArgs {
  RedDesc d[13];
  float* grads;
  float* norm_part;
  int64_t numel;
  // metrics
  const float* head_tail;  // head_part + 3H
  int HP, nhead, B;
  float value_coef, entropy_coef, ent_const;
  const float* params;
  int64_t off_ls;
  float* metrics;
  int32_t* counters;
};

__global__ void __launch_bounds__(kRedThreads) ppo_reduce(RedArgs r) {
  __shared__ float red[kRedThreads / 64];
  const int64_t i = (int64_t)blockIdx.x * kRedThreads + threadIdx.x;
  float sq = 0.0f;
  if (i < r.numel) {
    int p = 0;
#pragma unroll 1
    for (int q = 1; q < 13; ++q)
      if (i >= r.d[q].dst) p = q;
    const RedDesc& D = r.d[p];
    const int64_t j = i - D.dst;
    float s = 0.0f;
#pragma unroll 8
    for (int z = 0; z < D.nsplit; ++z) s += D.src[z * D.stride + j];
    if (p == P_LOGSTD) s = s - r.entropy_coef;  // d(-ec * mean entropy)/d log_std
    r.grads[i] = s;
    sq = s * s;
  }
  sq = wave_sum_dpp(sq);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = sq;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.0f;
    for (int k = 0; k < kRedThreads / 64; ++k) s += red[k];
    r.norm_part[blockIdx.x] = s;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    // metrics row (ppo/agent.py:255-262): policy, value, entropy, loss, clip count, kl
    float pg = 0.0f, vf = 0.0f, clip = 0.0f, kl = 0.0f;
#pragma unroll 8
    for (int z = 0; z < r.nhead; ++z) {
      const float* tl = r.head_tail + (int64_t)z * r.HP;
      pg += tl[5];
      vf += tl[6];
      clip += tl[7];
      kl += tl[8];
    }
    const float invB = 1.0f / (float)r.B;
    const float ls0 = r.params[r.off_ls], ls1 = r.params[r.off_ls + 1];
    const float ent = (r.ent_const + logf(expf(ls0))) + (r.ent_const + logf(expf(ls1)));
    float* m = r.metrics + (int64_t)(r.counters[1] - 1) * 6;
    m[0] = pg * invB;
    m[1] = vf * invB;
    m[2] = ent;
    m[3] = (pg * invB + r.value_coef * (vf * invB)) - r.entropy_coef * ent;
    m[4] = clip;
    m[5] = kl * invB;
  }
}

// entropy & total loss need the actor/critic means: second tiny pass by the optimizer kernel
struct OptArgs {
  float* params;
  const float* grads;
  float* m;
  float* v;
  const float* norm_part;
  int nred;
  int64_t numel;
  const int32_t* counters;
  float lr, beta1, beta2, eps, max_norm;
  float* tiles;  // fused path: the weight tile image, rewritten with the new weights
  int64_t o_w1, o_w2, o_wa1, o_wc1;
  int S, H, sb, hb;
  int skip;  // dev builds' pricing (HWY_PPO_SKIP, WRONG results): 1 no tile writes, 2 empty; 0
  // ppo_adam_tiles: workgroups per weight matrix (W1, W2, Wa1, Wc1) and the small parameters'
  // contiguous runs [b1], [b2], [ba1 wa2 ba2 log_std], [bc1 wc2 bc2] (flat offsets, prefix counts)
  int nwg1, nwgh, nkg1;
  int64_t run_off[4], run_pre[5];
};

// float index of B[k][n] in a tile image region with nblk blocks per 16 columns
__device__ __forceinline__ int64_t tile_index(int k, int n, int nblk) {
  return ((int64_t)(n >> 4) * nblk + (k >> 4)) * 256 + ((((k & 15) >> 2) << 4) + (n & 15)) * 4 +
         (k & 3);
}

// the tile image entries of flat parameter i (new value v)
__device__ __forceinline__ void write_tiles(const OptArgs& o, int64_t i, float v) {
  const TileGeom T = tile_geom(o.S, o.H, o.sb, o.hb);
  const int64_t H = o.H;
  int64_t j = i - o.o_w1;
  if (j >= 0 && j < H * o.S) {  // W1 [H][S]: forward only, B[k][n] = W1[n][k]
    // j / S in float: (j + 1/2) / S stays >= 1/(2S) away from an integer, far above rounding
    const int n = (int)(((float)j + 0.5f) * (1.0f / (float)o.S));
    const int k = (int)(j - (int64_t)n * o.S);
    o.tiles[T.f1 + tile_index(k, n, o.sb)] = v;
    return;
  }
  const int64_t offs[3] = {o.o_w2, o.o_wa1, o.o_wc1};
  const int64_t fwd[3] = {T.f2, T.fa, T.fc}, bwd[3] = {T.b2, T.ba, T.bc};
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    j = i - offs[q];
    if (j >= 0 && j < H * H) {  // [H][H]: forward B = W^T, backward B = W
      const int n = (int)(((float)j + 0.5f) * (1.0f / (float)o.H));
      const int k = (int)(j - (int64_t)n * H);
      o.tiles[fwd[q] + tile_index(k, n, o.hb)] = v;
      o.tiles[bwd[q] + tile_index(n, k, o.hb)] = v;
      return;
    }
  }
}

struct TileArgs {
  const float* P;
  int64_t o_w1, o_w2, o_wa1, o_wc1;
  int S, H, sb, hb;
  float* tiles;
};

// the whole tile image from params (hwy_ppo_sync_params): one float per thread
__global__ void __launch_bounds__(256) ppo_retile(TileArgs a) {
  const TileGeom T = tile_geom(a.S, a.H, a.sb, a.hb);
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= T.total) return;
  const float* W;
  int64_t base;
  int K, nblk;
  bool fwd;
  if (i < T.f2) W = a.P + a.o_w1, base = T.f1, K = a.S, nblk = a.sb, fwd = true;
  else if (i < T.fa) W = a.P + a.o_w2, base = T.f2, K = a.H, nblk = a.hb, fwd = true;
  else if (i < T.fc) W = a.P + a.o_wa1, base = T.fa, K = a.H, nblk = a.hb, fwd = true;
  else if (i < T.ba) W = a.P + a.o_wc1, base = T.fc, K = a.H, nblk = a.hb, fwd = true;
  else if (i < T.bc) W = a.P + a.o_wa1, base = T.ba, K = a.H, nblk = a.hb, fwd = false;
  else if (i < T.b2) W = a.P + a.o_wc1, base = T.bc, K = a.H, nblk = a.hb, fwd = false;
  else W = a.P + a.o_w2, base = T.b2, K = a.H, nblk = a.hb, fwd = false;
  const int64_t r = i - base;
  const int tile = (int)(r >> 8), e = (int)(r & 255);
  const int G = tile / nblk, b = tile - G * nblk;
  const int l = e >> 2, jj = e & 3;
  const int k = 16 * b + 4 * (l >> 4) + jj, n = 16 * G + (l & 15);
  float v = 0.0f;
  if (fwd) {
    if (k < K) v = W[(int64_t)n * K + k];  // B[k][n] = W[n][k], W [H][K]
  } else {
    if (k < a.H) v = W[(int64_t)k * a.H + n];  // B[k][n] = W[k][n], W [H][H]
  }
  a.tiles[i] = v;
}

// sum of squares of the (all-reduced) gradient, same partition as ppo_reduce
__global__ void __launch_bounds__(kRedThreads) ppo_sumsq(const float* g, int64_t n, float* part) {
  __shared__ float red[kRedThreads / 64];
  const int64_t i = (int64_t)blockIdx.x * kRedThreads + threadIdx.x;
  float sq = i < n ? g[i] * g[i] : 0.0f;
  sq = wave_sum_dpp(sq);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = sq;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.0f;
    for (int k = 0; k < kRedThreads / 64; ++k) s += red[k];
    part[blockIdx.x] = s;
  }
}

constexpr int kAdamEPT = 2;  // elements per thread (same box: 1 5.9 µs, 2 5.5, 4 5.7, 8 7.4)

// clip_grad_norm_'s coefficient from the norm partials and Adam's bias corrections, into
// sh[0] (coef), sh[1] (lr / bc1), sh[2] (sqrt bc2); every thread of the workgroup calls it
// first / t: this thread's first norm partial (norm_part[threadIdx.x], 0 past nred) and the Adam
// step, loaded by the caller ahead of its other loads (vector memory completes in issue order)
__device__ __forceinline__ void adam_scalars(const OptArgs& o, float* red, float* sh, float first,
                                             int t) {
  float s = 0.0f;
  if ((int)threadIdx.x < o.nred) s += first;
  for (int k = threadIdx.x + 256; k < o.nred; k += 256) s += o.norm_part[k];
  s = wave_sum_dpp(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  if (threadIdx.x == 64) {  // wave 1, while the norm partials combine
    // torch.optim.Adam (foreach, non-capturable): bias corrections in double on the host side
    // (beta ** t by binary powering: a few dependent multiplies instead of a double pow())
    double p1 = 1.0, p2 = 1.0, b1 = (double)o.beta1, b2 = (double)o.beta2;
    for (int e = t; e > 0; e >>= 1) {
      if (e & 1) p1 *= b1, p2 *= b2;
      b1 *= b1, b2 *= b2;
    }
    const double bc1 = 1.0 - p1;
    const double bc2 = 1.0 - p2;
    sh[1] = (float)((double)o.lr / bc1);
    sh[2] = (float)sqrt(bc2);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const float total = sqrtf(((red[0] + red[1]) + red[2]) + red[3]);
    const float c = o.max_norm / (total + 1e-6f);
    sh[0] = c < 1.0f ? c : 1.0f;
  }
  __syncthreads();
}

// torch.optim.Adam on one element after the clip: the raw gradient and the old state in, the new
// moments and parameter out
__device__ __forceinline__ void adam_math(const OptArgs& o, float g_raw, float& mm, float& vv,
                                          float& p, const float* sh) {
  const float coef = sh[0], step_size = sh[1], bc2_sqrt = sh[2];
  const float g = g_raw * coef;
  mm = mm + (1.0f - o.beta1) * (g - mm);  // exp_avg.lerp_(grad, 1 - beta1)
  vv = vv * o.beta2 + (1.0f - o.beta2) * g * g;
  const float denom = sqrtf(vv) / bc2_sqrt + o.eps;
  p = p - step_size * (mm / denom);
}

// one element of torch.optim.Adam after the clip (parameter i, its raw gradient and old state)
__device__ __forceinline__ void adam_elem(const OptArgs& o, int64_t i, float g_raw, float m_old,
                                          float v_old, float p_old, const float* sh) {
  float mm = m_old, vv = v_old, pn = p_old;
  adam_math(o, g_raw, mm, vv, pn, sh);
  o.m[i] = mm;
  o.v[i] = vv;
  o.params[i] = pn;
  if (o.tiles) write_tiles(o, i, pn);
}

__global__ void __launch_bounds__(256) ppo_adam(OptArgs o) {
  if (o.skip & 2) return;
  if (o.skip & 1) o.tiles = nullptr;
  __shared__ float red[4];
  __shared__ float sh[3];
  // the norm partial and the step count first (the clip coefficient's chain waits on them), then
  // this thread's elements (256 apart, coalesced), whose loads overlap the norm reduction
  const float first = (int)threadIdx.x < o.nred ? o.norm_part[threadIdx.x] : 0.0f;
  const int step = o.counters[0];
  float g_raw[kAdamEPT], m_old[kAdamEPT], v_old[kAdamEPT], p_old[kAdamEPT];
#pragma unroll
  for (int q = 0; q < kAdamEPT; ++q) {
    const int64_t i = ((int64_t)blockIdx.x * kAdamEPT + q) * 256 + threadIdx.x;
    const int64_t ii = i < o.numel ? i : 0;
    g_raw[q] = o.grads[ii], m_old[q] = o.m[ii], v_old[q] = o.v[ii], p_old[q] = o.params[ii];
  }
  adam_scalars(o, red, sh, first, step);
#pragma unroll
  for (int q = 0; q < kAdamEPT; ++q) {
    const int64_t i = ((int64_t)blockIdx.x * kAdamEPT + q) * 256 + threadIdx.x;
    if (i >= o.numel) break;
    adam_elem(o, i, g_raw[q], m_old[q], v_old[q], p_old[q], sh);
  }
}

// ppo_adam over the fused path's weight tile image, tile-major: a weight workgroup takes 16 rows x
// 64 columns of one of W1, W2, Wa1, Wc1 (wave w: the 16 x 16 block of columns 16w..16w+15; lane
// l: row l & 15, columns 4 (l >> 4) .. + 3 as one float4), so each wave rewrites whole 1-KB image
// blocks: the forward block (B = W^T) straight from its float4s (lane-linear), the backward block
// (B = W) after a 4 x 4 transpose through LDS.  The small parameters (biases, heads, log_std)
// follow in flat workgroups of 1,024.  Same Adam arithmetic per element as ppo_adam, so the same
// bits; ppo_adam's one-element mapping scatters 4-byte image writes over 16 blocks per wave.
__device__ __forceinline__ void adam_tiles_body(const OptArgs& o) {
  __shared__ float red[4];
  __shared__ float sh[3];
  __shared__ __attribute__((aligned(16))) f32x4 tr[4][64];  // per wave: its block, [row][col]
  const float first = (int)threadIdx.x < o.nred ? o.norm_part[threadIdx.x] : 0.0f;
  const int step = o.counters[0];
  const int t = threadIdx.x, wv = t >> 6, lane = t & 63;
  const int H = o.H;
  if ((int)blockIdx.x < o.nwg1 + 3 * o.nwgh) {
    int b = blockIdx.x, q, kg;
    if (b < o.nwg1) {
      q = 0, kg = o.nkg1;
    } else {
      b -= o.nwg1;
      q = 1 + b / o.nwgh, b -= (q - 1) * o.nwgh, kg = H / 64;
    }
    const int n0 = 16 * (b / kg), k0 = 64 * (b % kg) + 16 * wv;  // this wave's block
    const int K = q == 0 ? o.S : H;
    const int64_t off = q == 0 ? o.o_w1 : (q == 1 ? o.o_w2 : (q == 2 ? o.o_wa1 : o.o_wc1));
    const int nn = lane & 15, kq = lane >> 4;
    const int k = k0 + 4 * kq;
    const bool live = k < K;  // S % 4 == 0 (host check): a float4 is all live or all padding
    const int64_t i = off + (int64_t)(n0 + nn) * K + k;
    f32x4 g4 = {}, m4 = {}, v4 = {}, p4 = {};
    if (live) {
      g4 = *reinterpret_cast<const f32x4*>(o.grads + i);
      m4 = *reinterpret_cast<const f32x4*>(o.m + i);
      v4 = *reinterpret_cast<const f32x4*>(o.v + i);
      p4 = *reinterpret_cast<const f32x4*>(o.params + i);
    }
    adam_scalars(o, red, sh, first, step);
    if (o.skip & 2) return;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float mm = m4[j], vv = v4[j], pp = p4[j];
      adam_math(o, g4[j], mm, vv, pp, sh);
      m4[j] = mm, v4[j] = vv, p4[j] = pp;
    }
    if (live) {
      *reinterpret_cast<f32x4*>(o.m + i) = m4;
      *reinterpret_cast<f32x4*>(o.v + i) = v4;
      *reinterpret_cast<f32x4*>(o.params + i) = p4;
    } else {
      p4 = f32x4{0.0f, 0.0f, 0.0f, 0.0f};  // the image's zero padding past K
    }
    if ((o.skip & 1) || k0 >= K) return;  // a W1 block wholly past S: padding, already zero
    const TileGeom T = tile_geom(o.S, H, o.sb, o.hb);
    const int64_t fb = q == 0 ? T.f1 : (q == 1 ? T.f2 : (q == 2 ? T.fa : T.fc));
    const int nblk = q == 0 ? o.sb : o.hb;
    // forward image B[k][n] = W[n][k]: float 4 (16 kq + nn) + j of block (n0 / 16, k0 / 16)
    *reinterpret_cast<f32x4*>(o.tiles + fb + ((int64_t)(n0 >> 4) * nblk + (k0 >> 4)) * 256 +
                              4 * lane) = p4;
    if (q == 0) return;  // W1 has no backward image (uniform per workgroup: no barrier below)
    // backward image B[k'][n'] = W[k'][n'] (k' = row, n' = column): float
    // 4 (16 (row >> 2) + col) + (row & 3) of block (k0 / 16, n0 / 16); lane 16 kq + 4 a + c takes
    // rows 4a..4a+3 of column 4 kq + c from the block staged in LDS
    tr[wv][nn * 4 + kq] = p4;
    __syncthreads();
    const float* blk = reinterpret_cast<const float*>(tr[wv]);
    const int a = (lane >> 2) & 3, col = 4 * kq + (lane & 3);
    const f32x4 o4 = {blk[(4 * a) * 16 + col], blk[(4 * a + 1) * 16 + col],
                      blk[(4 * a + 2) * 16 + col], blk[(4 * a + 3) * 16 + col]};
    const int64_t bb = q == 1 ? T.b2 : (q == 2 ? T.ba : T.bc);
    *reinterpret_cast<f32x4*>(o.tiles + bb + ((int64_t)(k0 >> 4) * o.hb + (n0 >> 4)) * 256 +
                              4 * (16 * a + col)) = o4;
    return;
  }
  // the small parameters: four contiguous runs, 4 elements per thread 256 apart
  const int64_t e0 = (int64_t)(blockIdx.x - o.nwg1 - 3 * o.nwgh) * 1024 + t;
  float g_raw[4], m_old[4], v_old[4], p_old[4];
  int64_t ii[4];
#pragma unroll
  for (int qq = 0; qq < 4; ++qq) {
    const int64_t e = e0 + 256 * qq;
    int r = 0;
#pragma unroll
    for (int z = 1; z < 4; ++z)
      if (e >= o.run_pre[z]) r = z;
    ii[qq] = e < o.run_pre[4] ? o.run_off[r] + (e - o.run_pre[r]) : -1;
    const int64_t src = ii[qq] >= 0 ? ii[qq] : 0;
    g_raw[qq] = o.grads[src], m_old[qq] = o.m[src], v_old[qq] = o.v[src], p_old[qq] = o.params[src];
  }
  adam_scalars(o, red, sh, first, step);
  if (o.skip & 2) return;
#pragma unroll
  for (int qq = 0; qq < 4; ++qq) {
    if (ii[qq] < 0) break;
    float mm = m_old[qq], vv = v_old[qq], pp = p_old[qq];
    adam_math(o, g_raw[qq], mm, vv, pp, sh);
    o.m[ii[qq]] = mm, o.v[ii[qq]] = vv, o.params[ii[qq]] = pp;
  }
}

__global__ void __launch_bounds__(256) ppo_adam_tiles(OptArgs o) { adam_tiles_body(o); }

// ----------------------------------------------------------------------------- grouped
// G independent learners of the same dims in one launch per kernel (experiments/sweep.py: a
// sweep's seeds of one condition).  Workgroup (x, y) runs the solo kernel's workgroup x for
// learner y, whose arguments the kernel reads from a device table (hwy_ppo_group_prepare): the
// same bodies and tile shapes as the solo launches, so each learner's bits are its solo run's.
// a learner's own grid of each grouped launch (the launch covers the largest learner's)
struct GroupLim {
  int rows, wgrad, wsum, adam;
};

template <int QH, int NW, int RT>
__global__ void __launch_bounds__(64 * NW, 1) ppo_rows_grp(const RowArgs* __restrict__ tab,
                                                           const GroupLim* __restrict__ lim) {
  if ((int)blockIdx.x >= lim[blockIdx.y].rows) return;  // whole workgroup
  rows_body<QH, NW, RT, false>(tab[blockIdx.y]);
}

__global__ void __launch_bounds__(512) ppo_wgrad_grp(const WgArgs* __restrict__ tab,
                                                     const GroupLim* __restrict__ lim) {
  if ((int)blockIdx.x >= lim[blockIdx.y].wgrad) return;
  ppo_wgrad_body(tab[blockIdx.y]);
}

__global__ void __launch_bounds__(256) ppo_wsum_grp(const WgArgs* __restrict__ tab,
                                                    const GroupLim* __restrict__ lim) {
  if ((int)blockIdx.x >= lim[blockIdx.y].wsum) return;
  wsum_body(tab[blockIdx.y]);
}

__global__ void __launch_bounds__(256) ppo_adam_tiles_grp(const OptArgs* __restrict__ tab,
                                                          const GroupLim* __restrict__ lim) {
  if ((int)blockIdx.x >= lim[blockIdx.y].adam) return;
  adam_tiles_body(tab[blockIdx.y]);
}

template <int QH, int NW, bool TL>
__global__ void __launch_bounds__(64 * NW, 1) ppo_act_grp(const ActArgs* __restrict__ tab) {
  act_body<QH, NW, TL>(tab[blockIdx.y]);
}

template <int QH, int NW, int RT>
__global__ void __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(2 * NW / 4, 8)))
ppo_act_c_grp(const ActArgs* __restrict__ tab) {
  act_c_body<QH, NW, RT>(tab[blockIdx.y]);
}

template <int AM, int BM, int EPI>
int launch_gemm(const GemmArgs& g, int splits, hipStream_t s) {
  dim3 grid((g.M + kTile - 1) / kTile, (g.N + kTile - 1) / kTile, splits);
  // 16-byte path when every vector access is aligned and in-bounds-or-fully-out
  auto al = [](const void* p) { return ((uintptr_t)p & 15u) == 0; };
  bool vec = al(g.A) && al(g.B) && (!g.B2 || al(g.B2));
  vec = vec && (AM == A_ROW ? (g.K % 4 == 0 && g.lda % 4 == 0) : (g.M % 4 == 0 && g.lda % 4 == 0));
  vec = vec && (BM == B_NT ? (g.K % 4 == 0 && g.ldb % 4 == 0) : (g.N % 4 == 0 && g.ldb % 4 == 0));
  if (vec)
    hipLaunchKernelGGL((gemm64v<AM, BM, EPI>), grid, dim3(256), 0, s, g);
  else
    hipLaunchKernelGGL((gemm64<AM, BM, EPI>), grid, dim3(256), 0, s, g);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

GemmArgs gemm_args() {
  GemmArgs g = {};
  g.split = 1 << 30;
  return g;
}

}  // namespace

extern "C" {

int hwy_ppo_param_layout(const hwy_ppo_dims* d, int64_t* offsets, int64_t* numel) {
  if (!d || d->A != 2 || d->H < 64 || d->H % 64 || d->S < 1 || d->B < 1) return -1;
  Layout L = make_layout(*d);
  if (offsets)
    for (int i = 0; i < 13; ++i) offsets[i] = L.off[i];
  if (numel) *numel = L.numel;
  return 0;
}

int64_t hwy_ppo_workspace_bytes(const hwy_ppo_dims* d) {
  if (!d || d->A != 2 || d->H < 64 || d->H % 64 || d->H > 512 || d->S < 1 || d->B < 1) return -1;
  int64_t bytes = 0;
  carve(*d, nullptr, &bytes);
  return bytes;
}

int64_t hwy_ppo_tile_image_offset(const hwy_ppo_dims* d) {
  if (hwy_ppo_workspace_bytes(d) < 0 || !fused_ok(*d)) return -1;
  char* base = reinterpret_cast<char*>(uintptr_t(1) << 20);  // carve only adds offsets to it
  const Work w = carve(*d, base, nullptr);
  return (int64_t)(reinterpret_cast<char*>(w.wtile) - base);
}

// The fused path's per-kernel arguments for one learner's minibatch step (shared by the solo
// launches and the grouped table of hwy_ppo_group_prepare).
static RowArgs row_args(const hwy_ppo_args& a0, const Layout& L, const Work& w) {
  const hwy_ppo_args* a = &a0;
  const float* P = a->params;
  const int B = a->dims.B, S = a->dims.S;
  RowArgs r = {};
  r.B = B, r.S = S;
  r.states = a->states, r.idx = a->idx, r.pre_tanh = a->pre_tanh, r.old_logp = a->old_logp;
  r.adv = a->adv, r.ret = a->ret, r.params = P;
  for (int i = 0; i < 13; ++i) r.off[i] = L.off[i];
  r.h1 = w.h1, r.h2 = w.h2, r.dac = w.dac, r.dh2 = w.dh2, r.dh1 = w.dh1, r.xg = w.xg;
  r.tiles = w.wtile;
  r.head_part = w.head_part, r.HP = w.HP;
  r.eps_clip = a->eps_clip, r.value_coef = a->value_coef, r.entropy_coef = a->entropy_coef;
  r.counters = a->counters;
  return r;
}

static WgArgs wg_args(const hwy_ppo_args& a0, const Layout& L, const Work& w) {
  const hwy_ppo_args* a = &a0;
  const float* P = a->params;
  const int B = a->dims.B, S = a->dims.S, H = a->dims.H;
  WgArgs g = {};
  g.B = B, g.S = S, g.H = H;
  g.dac = w.dac, g.h2 = w.h2, g.dh2 = w.dh2, g.h1 = w.h1, g.dh1 = w.dh1, g.xg = w.xg;
  g.grads = a->grads;
  for (int i = 0; i < 13; ++i) g.off[i] = L.off[i];
  g.head_part = w.head_part, g.nhp = w.n1, g.HP = w.HP, g.norm_part = w.norm_part;
  g.tac = w.tac, g.t2 = w.t2, g.t1 = w.t1, g.nh = w.nh;
  g.split = w.split, g.slab = w.wg_slab;
  g.bal = w.bal, g.wm = w.wm, g.tpe = w.tpe, g.nslot = w.nslot;
  g.entropy_coef = a->entropy_coef, g.value_coef = a->value_coef;
  g.ent_const = 0.5f + 0.91893853320467274178f;
  g.params = P, g.metrics = a->metrics, g.counters = a->counters;
  return g;
}

// clip_grad_norm_ + Adam's arguments for one learner (solo launches and the grouped table)
static OptArgs opt_args(const hwy_ppo_args& a0, const Layout& L, const Work& w) {
  const hwy_ppo_args* a = &a0;
  const hwy_ppo_dims& d = a->dims;
  OptArgs o = {};
  o.params = a->params, o.grads = a->grads, o.m = a->adam_m, o.v = a->adam_v;
  // norm partials: ppo_sumsq / ppo_reduce write nred of them, ppo_wgrad grid2
  o.norm_part = w.norm_part, o.numel = L.numel, o.counters = a->counters;
  o.nred = (w.fused && !a->grads_modified) ? w.nred2 : w.nred;
  o.lr = a->lr, o.beta1 = a->beta1, o.beta2 = a->beta2, o.eps = a->adam_eps;
  o.max_norm = a->max_grad_norm;
  if (w.fused) {
    o.tiles = w.wtile;
    o.o_w1 = L.off[P_W1], o.o_w2 = L.off[P_W2], o.o_wa1 = L.off[P_WA1], o.o_wc1 = L.off[P_WC1];
    o.S = d.S, o.H = d.H, o.sb = w.sb, o.hb = w.hb;
  }
  o.skip = dev_knob_int("HWY_PPO_SKIP", 0) & 3;
  if (w.fused) {  // ppo_adam_tiles' geometry (used when adam_tiles_ok)
    const int kb1 = (d.S + 15) / 16;  // W1's live 16-column blocks
    o.nkg1 = (kb1 + 3) / 4;
    o.nwg1 = (d.H / 16) * o.nkg1;
    o.nwgh = (d.H / 16) * (d.H / 64);
    const int64_t r0[4] = {L.off[P_B1], L.off[P_B2], L.off[P_BA1], L.off[P_BC1]};
    const int64_t r1[4] = {L.off[P_W2], L.off[P_WA1], L.off[P_WC1], L.numel};
    o.run_pre[0] = 0;
    for (int z = 0; z < 4; ++z) {
      o.run_off[z] = r0[z];
      o.run_pre[z + 1] = o.run_pre[z] + (r1[z] - r0[z]);
    }
  }
  return o;
}

// the tile-major kernel wherever its float4s are aligned: S % 4 == 0 and 16-byte aligned bases
static bool adam_tiles_ok(const hwy_ppo_args& a, const OptArgs& o, const Work& w) {
  auto al16 = [](const void* p) { return ((uintptr_t)p & 15u) == 0; };
  return w.fused && a.dims.S % 4 == 0 && al16(o.params) && al16(o.grads) && al16(o.m) &&
         al16(o.v) && dev_knob_int("HWY_ADAM_FLAT", 0) == 0;
}

static int adam_tiles_grid(const OptArgs& o) {
  const int nsmall = (int)((o.run_pre[4] + 1023) / 1024);
  return o.nwg1 + 3 * o.nwgh + nsmall;
}

// mask (fused path; hwy_ppo_time_kernels launches them one at a time): bit 0 ppo_rows, bit 1
// ppo_wgrad, bit 2 ppo_wsum
static int forward_backward_k(const hwy_ppo_args* a, void* stream, int mask) {
  if (!a) return -1;
  const hwy_ppo_dims& d = a->dims;
  if (hwy_ppo_workspace_bytes(&d) < 0) return -1;
  hipStream_t s = (hipStream_t)stream;
  const int B = d.B, S = d.S, H = d.H;
  const Layout L = make_layout(d);
  Work w = carve(d, a->workspace, nullptr);
  const float* P = a->params;
  int rc = 0;
  if (w.fused) {
    const RowArgs r = row_args(*a, L, w);
    // 8 waves (2 per SIMD) when the columns split into 16-wide tiles, else 4
    const dim3 g1(w.n1), b4(256), b8(512), blk(256);
    if (!(mask & 1)) {
    } else if (w.rt == 4 * kRowTile) {
      hipLaunchKernelGGL((ppo_rows_c64<4, 8>), g1, b8, 0, s, r);
    } else if (w.rt == 2 * kRowTile) {
      switch (H / 64) {
        case 1: hipLaunchKernelGGL((ppo_rows<1, 4, 32>), g1, b4, 0, s, r); break;
        case 2: hipLaunchKernelGGL((ppo_rows<2, 8, 32>), g1, b8, 0, s, r); break;
        case 3: hipLaunchKernelGGL((ppo_rows<3, 4, 32>), g1, b4, 0, s, r); break;
        default:
          hipLaunchKernelGGL((ppo_rows_c<4, 8, 32>), g1, b8, 0, s, r);
          break;
      }
    } else {
      switch (H / 64) {
        case 1: hipLaunchKernelGGL((ppo_rows<1, 4, 16>), g1, b4, 0, s, r); break;
        case 2: hipLaunchKernelGGL((ppo_rows<2, 8, 16>), g1, b8, 0, s, r); break;
        case 3: hipLaunchKernelGGL((ppo_rows<3, 4, 16>), g1, b4, 0, s, r); break;
        // (16 waves, one 16-column tile each, measured 73.2-73.6 vs 72.0-72.6 us per 4,096-row
        // step, round 5; its head sums would also leave ppo_act_c's order)
        case 4: hipLaunchKernelGGL((ppo_rows<4, 8, 16>), g1, b8, 0, s, r); break;
        case 5: hipLaunchKernelGGL((ppo_rows<5, 4, 16>), g1, b4, 0, s, r); break;
        case 6: hipLaunchKernelGGL((ppo_rows<6, 8, 16>), g1, b8, 0, s, r); break;
        case 7: hipLaunchKernelGGL((ppo_rows<7, 4, 16>), g1, b4, 0, s, r); break;
        default: hipLaunchKernelGGL((ppo_rows<8, 8, 16>), g1, b8, 0, s, r); break;
      }
    }
    rc |= hipGetLastError() == hipSuccess ? 0 : -1;
    const WgArgs g = wg_args(*a, L, w);
    if (mask & 2) hipLaunchKernelGGL(ppo_wgrad, dim3(w.grid2), dim3(64 * kWgWaves), 0, s, g);
    rc |= hipGetLastError() == hipSuccess ? 0 : -1;
    if (mask & 4)
      hipLaunchKernelGGL(ppo_wsum, dim3((w.tac + w.t2 + w.t1) * (kWgTM * kWgTN / 1024)), blk, 0, s, g);
    rc |= hipGetLastError() == hipSuccess ? 0 : -1;
    return rc;
  }
  if (mask != 7) return -1;  // the per-kernel timing covers the fused path only
  // ---- forward (general path: separate GEMMs, split-K weight gradients)
  {
    GemmArgs g = gemm_args();
    g.M = B, g.N = H, g.K = S;
    g.A = a->states, g.lda = S, g.a_gather = a->idx;
    g.B = P + L.off[P_W1], g.ldb = S;
    g.C = w.h1, g.ldc = H, g.bias = P + L.off[P_B1];
    rc |= launch_gemm<A_ROW, B_NT, EPI_BIAS_RELU>(g, 1, s);
  }
  {
    GemmArgs g = gemm_args();
    g.M = B, g.N = H, g.K = H;
    g.A = w.h1, g.lda = H;
    g.B = P + L.off[P_W2], g.ldb = H;
    g.C = w.h2, g.ldc = H, g.bias = P + L.off[P_B2];
    rc |= launch_gemm<A_ROW, B_NT, EPI_BIAS_RELU>(g, 1, s);
  }
  {
    GemmArgs g = gemm_args();
    g.M = B, g.N = 2 * H, g.K = H;
    g.A = w.h2, g.lda = H;
    g.B = P + L.off[P_WA1], g.B2 = P + L.off[P_WC1], g.ldb = H, g.split = H;
    g.C = w.ac, g.ldc = 2 * H, g.bias = P + L.off[P_BA1], g.bias2 = P + L.off[P_BC1];
    rc |= launch_gemm<A_ROW, B_NT, EPI_BIAS_RELU>(g, 1, s);
  }
  // ---- loss head
  {
    HeadArgs h = {};
    h.B = B, h.H = H, h.A = 2;
    h.ac = w.ac, h.dac = w.dac, h.params = P;
    h.pre_tanh = a->pre_tanh, h.old_logp = a->old_logp, h.adv = a->adv, h.ret = a->ret;
    h.idx = a->idx, h.part = w.head_part, h.HP = w.HP;
    h.off_wa2 = L.off[P_WA2], h.off_ba2 = L.off[P_BA2], h.off_ls = L.off[P_LOGSTD];
    h.off_wc2 = L.off[P_WC2], h.off_bc2 = L.off[P_BC2];
    h.eps_clip = a->eps_clip, h.value_coef = a->value_coef, h.entropy_coef = a->entropy_coef;
    h.counters = a->counters;
    hipLaunchKernelGGL(ppo_head, dim3(w.nhead), dim3(256), 0, s, h);
    rc |= hipGetLastError() == hipSuccess ? 0 : -1;
  }
  // ---- backward
  {
    GemmArgs g = gemm_args();  // dh2 = dac [Wa1;Wc1] * (h2 > 0)
    g.M = B, g.N = H, g.K = 2 * H;
    g.A = w.dac, g.lda = 2 * H;
    g.B = P + L.off[P_WA1], g.B2 = P + L.off[P_WC1], g.ldb = H, g.split = H;
    g.C = w.dh2, g.ldc = H, g.mask = w.h2, g.ldm = H;
    rc |= launch_gemm<A_ROW, B_NN, EPI_MASK>(g, 1, s);
  }
  {
    GemmArgs g = gemm_args();  // d[Wa1;Wc1] = dac^T h2 (+ bias column sums)
    g.M = 2 * H, g.N = H, g.K = B;
    g.A = w.dac, g.lda = 2 * H;
    g.B = w.h2, g.ldb = H;
    g.C = w.slab_ac, g.ldc = H, g.slab = (long)2 * H * H, g.bias_part = w.bias_ac, g.kchunk = w.ca;
    rc |= launch_gemm<A_TRANS, B_NN, EPI_SPLITK>(g, w.sa, s);
  }
  {
    GemmArgs g = gemm_args();  // dh1 = dh2 W2 * (h1 > 0)
    g.M = B, g.N = H, g.K = H;
    g.A = w.dh2, g.lda = H;
    g.B = P + L.off[P_W2], g.ldb = H;
    g.C = w.dh1, g.ldc = H, g.mask = w.h1, g.ldm = H;
    rc |= launch_gemm<A_ROW, B_NN, EPI_MASK>(g, 1, s);
  }
  {
    GemmArgs g = gemm_args();  // dW2 = dh2^T h1
    g.M = H, g.N = H, g.K = B;
    g.A = w.dh2, g.lda = H;
    g.B = w.h1, g.ldb = H;
    g.C = w.slab_2, g.ldc = H, g.slab = (long)H * H, g.bias_part = w.bias_2, g.kchunk = w.c2;
    rc |= launch_gemm<A_TRANS, B_NN, EPI_SPLITK>(g, w.s2, s);
  }
  {
    GemmArgs g = gemm_args();  // dW1 = dh1^T gather(states)
    g.M = H, g.N = S, g.K = B;
    g.A = w.dh1, g.lda = H;
    g.B = a->states, g.ldb = S, g.b_gather = a->idx;
    g.C = w.slab_1, g.ldc = S, g.slab = (long)H * S, g.bias_part = w.bias_1, g.kchunk = w.c1;
    rc |= launch_gemm<A_TRANS, B_NN, EPI_SPLITK>(g, w.s1, s);
  }
  // ---- reduce partials into the flat gradient
  {
    RedArgs r = {};
    const int64_t HH = (int64_t)H * H;
    auto set = [&](int p, const float* src, int64_t stride, int nsplit) {
      r.d[p].src = src;
      r.d[p].stride = stride;
      r.d[p].nsplit = nsplit;
      r.d[p].dst = L.off[p];
    };
    set(P_W1, w.slab_1, (int64_t)H * S, w.s1);
    set(P_B1, w.bias_1, H, w.s1);
    set(P_W2, w.slab_2, HH, w.s2);
    set(P_B2, w.bias_2, H, w.s2);
    set(P_WA1, w.slab_ac, 2 * HH, w.sa);
    set(P_BA1, w.bias_ac, 2 * H, w.sa);
    set(P_WA2, w.head_part, w.HP, w.nhead);  // [gwa0 | gwa1] = rows 0,1 of dWa2
    set(P_BA2, w.head_part + 3 * H, w.HP, w.nhead);
    set(P_LOGSTD, w.head_part + 3 * H + 3, w.HP, w.nhead);
    set(P_WC1, w.slab_ac + HH, 2 * HH, w.sa);
    set(P_BC1, w.bias_ac + H, 2 * H, w.sa);
    set(P_WC2, w.head_part + 2 * H, w.HP, w.nhead);
    set(P_BC2, w.head_part + 3 * H + 2, w.HP, w.nhead);
    r.grads = a->grads, r.norm_part = w.norm_part, r.numel = L.numel;
    r.head_tail = w.head_part + 3 * H, r.HP = w.HP, r.nhead = w.nhead, r.B = B;
    r.value_coef = a->value_coef, r.entropy_coef = a->entropy_coef;
    r.ent_const = 0.5f + 0.91893853320467274178f;
    r.params = P, r.off_ls = L.off[P_LOGSTD];
    r.metrics = a->metrics, r.counters = a->counters;
    hipLaunchKernelGGL(ppo_reduce, dim3(w.nred), dim3(kRedThreads), 0, s, r);
    rc |= hipGetLastError() == hipSuccess ? 0 : -1;
  }
  return rc;
}

int hwy_ppo_forward_backward(const hwy_ppo_args* a, void* stream) {
  return forward_backward_k(a, stream, 7);
}

int hwy_ppo_optimizer(const hwy_ppo_args* a, void* stream) {
  if (!a) return -1;
  const hwy_ppo_dims& d = a->dims;
  if (hwy_ppo_workspace_bytes(&d) < 0) return -1;
  const Layout L = make_layout(d);
  Work w = carve(d, a->workspace, nullptr);
  hipStream_t s = (hipStream_t)stream;
  if (a->grads_modified) {  // e.g. after the RCCL gradient all-reduce
    hipLaunchKernelGGL(ppo_sumsq, dim3(w.nred), dim3(kRedThreads), 0, s, a->grads, L.numel,
                       w.norm_part);
    if (hipGetLastError() != hipSuccess) return -1;
  }
  OptArgs o = opt_args(*a, L, w);
  if (adam_tiles_ok(*a, o, w)) {
    hipLaunchKernelGGL(ppo_adam_tiles, dim3(adam_tiles_grid(o)), dim3(256), 0, s, o);
    return hipGetLastError() == hipSuccess ? 0 : -1;
  }
  const int nadam = (int)((L.numel + 256 * kAdamEPT - 1) / (256 * kAdamEPT));
  hipLaunchKernelGGL(ppo_adam, dim3(nadam), dim3(256), 0, s, o);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// an empty workgroup: hwy_ppo_time_kernels' launch floor (a graph of dependent empty launches)
__global__ void __launch_bounds__(64) ppo_nop() {}

int hwy_ppo_time_kernels(const hwy_ppo_args* a, void* stream, int reps, float* us) {
  if (!a || !us || reps < 1 || a->grads_modified || !a->counters) return -1;
  if (hwy_ppo_workspace_bytes(&a->dims) < 0 || !fused_ok(a->dims)) return -1;
  // Each kernel as its own HIP graph of `reps` back-to-back launches on a private stream,
  // replayed once to warm up and once between two events: the average launch of a kernel in the
  // same position it has in the epoch graph (graph-issued, dependent on its predecessor), without
  // host launch costs; us[4]: the same for an empty one-workgroup kernel, the per-launch floor
  // (dispatch and completion of a dependent launch) that a kernel-trace duration leaves out.  The caller's Adam step count is restored afterwards; the metrics row
  // index is reset before each replay so ppo_wgrad always writes metrics row 0.
  if (hipStreamSynchronize((hipStream_t)stream) != hipSuccess) return -2;
  int32_t saved[2];
  if (hipMemcpy(saved, a->counters, sizeof(saved), hipMemcpyDeviceToHost) != hipSuccess) return -2;
  hipStream_t s = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  int rc = 0;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess)
    rc = -2;
  const int32_t one = 1;
  for (int k = 0; k < 5 && rc == 0; ++k) {
    hipGraph_t g = nullptr;
    hipGraphExec_t x = nullptr;
    if (hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal) != hipSuccess) {
      rc = -2;
      break;
    }
    for (int i = 0; i < reps; ++i) {
      if (k < 3) {
        rc |= forward_backward_k(a, s, 1 << k);
      } else if (k == 3) {
        rc |= hwy_ppo_optimizer(a, s);
      } else {
        hipLaunchKernelGGL(ppo_nop, dim3(1), dim3(64), 0, s);
        rc |= hipGetLastError() == hipSuccess ? 0 : -2;
      }
    }
    rc |= hipStreamEndCapture(s, &g) == hipSuccess ? 0 : -2;
    if (rc == 0) rc = hipGraphInstantiate(&x, g, nullptr, nullptr, 0) == hipSuccess ? 0 : -2;
    for (int rep = 0; rep < 2 && rc == 0; ++rep) {
      rc |= hipMemcpyAsync(a->counters + 1, &one, sizeof(one), hipMemcpyHostToDevice, s) ==
                    hipSuccess ? 0 : -2;
      if (rep) rc |= hipEventRecord(e0, s) == hipSuccess ? 0 : -2;
      rc |= hipGraphLaunch(x, s) == hipSuccess ? 0 : -2;
      if (rep) rc |= hipEventRecord(e1, s) == hipSuccess ? 0 : -2;
      rc |= hipStreamSynchronize(s) == hipSuccess ? 0 : -2;
    }
    float ms = 0.0f;
    if (rc == 0) rc = hipEventElapsedTime(&ms, e0, e1) == hipSuccess ? 0 : -2;
    us[k] = ms * 1e3f / (float)reps;
    if (x) (void)hipGraphExecDestroy(x);
    if (g) (void)hipGraphDestroy(g);
  }
  if (e0) (void)hipEventDestroy(e0);
  if (e1) (void)hipEventDestroy(e1);
  if (s) {
    (void)hipStreamSynchronize(s);
    (void)hipStreamDestroy(s);
  }
  saved[1] = 0;
  if (hipMemcpy(a->counters, saved, sizeof(saved), hipMemcpyHostToDevice) != hipSuccess) rc = -2;
  (void)hipGetLastError();
  return rc;
}

int hwy_ppo_sync_params(const hwy_ppo_args* a, void* stream) {
  if (!a || !a->params || !a->workspace) return -1;
  const hwy_ppo_dims& d = a->dims;
  if (hwy_ppo_workspace_bytes(&d) < 0) return -1;
  Work w = carve(d, a->workspace, nullptr);
  if (!w.fused) return 0;  // the general path reads params directly
  const Layout L = make_layout(d);
  TileArgs t = {};
  t.P = a->params;
  t.o_w1 = L.off[P_W1], t.o_w2 = L.off[P_W2], t.o_wa1 = L.off[P_WA1], t.o_wc1 = L.off[P_WC1];
  t.S = d.S, t.H = d.H, t.sb = w.sb, t.hb = w.hb;
  t.tiles = w.wtile;
  const int64_t n = tile_geom(d.S, d.H, w.sb, w.hb).total;
  hipLaunchKernelGGL(ppo_retile, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, t);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int hwy_ppo_act(const hwy_ppo_act_args* a, void* stream) {
  if (!a || !a->states || !a->params || !a->action || !a->pre_tanh || !a->logp || !a->value)
    return -1;
  const hwy_ppo_dims& d = a->dims;
  if (!fused_ok(d) || d.A != 2 || d.B < 1) return -1;
  hipStream_t s = (hipStream_t)stream;
  const Layout L = make_layout(d);
  ActArgs r = {};
  r.B = d.B, r.S = d.S, r.states = a->states, r.params = a->params, r.noise = a->noise;
  for (int i = 0; i < 13; ++i) r.off[i] = L.off[i];
  r.action = a->action, r.pre_tanh = a->pre_tanh, r.logp = a->logp, r.value = a->value;
  r.tiles = a->tiles;
  const dim3 g((d.B + kRowTile - 1) / kRowTile), b4(256), b8(512);
  auto launch = [&](auto tl) {
    constexpr bool TL = decltype(tl)::value;
    switch (d.H / 64) {
      case 1: hipLaunchKernelGGL((ppo_act<1, 4, TL>), g, b4, 0, s, r); break;
      case 2: hipLaunchKernelGGL((ppo_act<2, 8, TL>), g, b8, 0, s, r); break;
      case 3: hipLaunchKernelGGL((ppo_act<3, 4, TL>), g, b4, 0, s, r); break;
      case 4: hipLaunchKernelGGL((ppo_act<4, 8, TL>), g, b8, 0, s, r); break;
      case 5: hipLaunchKernelGGL((ppo_act<5, 4, TL>), g, b4, 0, s, r); break;
      case 6: hipLaunchKernelGGL((ppo_act<6, 8, TL>), g, b8, 0, s, r); break;
      case 7: hipLaunchKernelGGL((ppo_act<7, 4, TL>), g, b4, 0, s, r); break;
      default: hipLaunchKernelGGL((ppo_act<8, 8, TL>), g, b8, 0, s, r); break;
    }
  };
  // H = 256 from the tile image: the compact kernel, 32-row tiles once there are two per CU
  // (16,384 rows on MI355X: 91.3 -> 69.4 us), else 16-row tiles (4,096 rows: 25.1 -> 22.0 us)
  if (r.tiles && d.H == 256) {
    if (d.B >= 64 * chip_geom().cus)
      hipLaunchKernelGGL((ppo_act_c<4, 8, 32>), dim3((d.B + 31) / 32), b8, 0, s, r);
    else
      hipLaunchKernelGGL((ppo_act_c<4, 8, 16>), dim3((d.B + 15) / 16), b8, 0, s, r);
  } else if (r.tiles)
    launch(std::integral_constant<bool, true>());
  else
    launch(std::integral_constant<bool, false>());
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ---- grouped learners (include/hwy_ppo.h): the device table of one minibatch step is
// [G RowArgs | G WgArgs | G OptArgs | G GroupLim], each section 256-byte aligned.  The learners
// share B and H (so every learner takes the 16-row tiles and the same row-kernel grid); their
// state dims may differ, which changes the weight-gradient tile count and Adam's W1 blocks, so
// each launch covers the largest learner's grid and a learner's surplus workgroups exit.
static int64_t align256(int64_t x) { return (x + 255) & ~int64_t(255); }
static int64_t grp_row_off(int) { return 0; }
static int64_t grp_wg_off(int G) { return align256((int64_t)G * sizeof(RowArgs)); }
static int64_t grp_opt_off(int G) { return grp_wg_off(G) + align256((int64_t)G * sizeof(WgArgs)); }
static int64_t grp_lim_off(int G) { return grp_opt_off(G) + align256((int64_t)G * sizeof(OptArgs)); }

static bool group_dims_ok(const hwy_ppo_dims& d) {
  if (hwy_ppo_workspace_bytes(&d) < 0 || !fused_ok(d) || d.A != 2 || d.B < 1) return false;
  char* base = reinterpret_cast<char*>(uintptr_t(1) << 20);  // carve only adds offsets to it
  const Work w = carve(d, base, nullptr);
  // 16-row tiles (minibatches below the 32-row threshold) and one workgroup per (tile, slice):
  // the balanced weight-gradient partition reads gridDim.x, which the grouped launch widens
  return w.fused && w.rt == kRowTile && !w.bal;
}

// one learner's grids (the solo launches'): rows, ppo_wgrad, ppo_wsum, ppo_adam_tiles
static GroupLim group_lim(const hwy_ppo_dims& d) {
  char* base = reinterpret_cast<char*>(uintptr_t(1) << 20);
  const Work w = carve(d, base, nullptr);
  hwy_ppo_args geom = {};
  geom.dims = d;
  const OptArgs og = opt_args(geom, make_layout(d), w);
  GroupLim l;
  l.rows = w.n1, l.wgrad = w.grid2, l.wsum = (w.tac + w.t2 + w.t1) * (kWgTM * kWgTN / 1024);
  l.adam = adam_tiles_grid(og);
  return l;
}

int64_t hwy_ppo_group_table_bytes(const hwy_ppo_dims* d, int G) {
  if (!d || G < 1 || !group_dims_ok(*d)) return -1;
  return grp_lim_off(G) + align256((int64_t)G * sizeof(GroupLim));
}

int hwy_ppo_group_prepare(const hwy_ppo_args* a, int G, void* table, hwy_ppo_group_plan* plan,
                          void* stream) {
  if (!a || G < 1 || !table || !plan) return -1;
  const hwy_ppo_dims& d0 = a[0].dims;
  if (!group_dims_ok(d0)) return -1;
  const int64_t bytes = hwy_ppo_group_table_bytes(&d0, G);
  char* host = static_cast<char*>(calloc((size_t)bytes, 1));
  if (!host) return -2;
  hwy_ppo_group_plan p = {};
  p.G = G, p.B = d0.B, p.H = d0.H;
  int rc = 0;
  for (int g = 0; g < G && rc == 0; ++g) {
    const hwy_ppo_args& ag = a[g];
    const hwy_ppo_dims& d = ag.dims;
    if (d.B != d0.B || d.H != d0.H || d.A != d0.A || !group_dims_ok(d) || ag.grads_modified ||
        !ag.workspace || !ag.counters || !ag.params || !ag.grads || !ag.adam_m || !ag.adam_v) {
      rc = -1;
      break;
    }
    const Layout L = make_layout(d);
    const Work w = carve(d, ag.workspace, nullptr);
    const OptArgs o = opt_args(ag, L, w);
    if (!adam_tiles_ok(ag, o, w)) {
      rc = -1;
      break;
    }
    reinterpret_cast<RowArgs*>(host + grp_row_off(G))[g] = row_args(ag, L, w);
    reinterpret_cast<WgArgs*>(host + grp_wg_off(G))[g] = wg_args(ag, L, w);
    reinterpret_cast<OptArgs*>(host + grp_opt_off(G))[g] = o;
    const GroupLim l = group_lim(d);
    reinterpret_cast<GroupLim*>(host + grp_lim_off(G))[g] = l;
    p.grid_rows = std::max(p.grid_rows, l.rows), p.grid_wgrad = std::max(p.grid_wgrad, l.wgrad);
    p.grid_wsum = std::max(p.grid_wsum, l.wsum), p.grid_adam = std::max(p.grid_adam, l.adam);
  }
  hipStream_t s = (hipStream_t)stream;
  if (rc == 0 && (hipMemcpyAsync(table, host, (size_t)bytes, hipMemcpyHostToDevice, s) != hipSuccess ||
                  hipStreamSynchronize(s) != hipSuccess))
    rc = -2;
  free(host);
  if (rc == 0) *plan = p;
  return rc;
}

int hwy_ppo_group_step(const hwy_ppo_group_plan* plan, const void* table, void* stream) {
  if (!plan || !table || plan->G < 1 || plan->H < 64 || plan->H > 512 || plan->H % 64 ||
      plan->grid_rows < 1 || plan->grid_wgrad < 1 || plan->grid_wsum < 1 || plan->grid_adam < 1)
    return -1;
  const int G = plan->G;
  const char* t = static_cast<const char*>(table);
  const RowArgs* tr = reinterpret_cast<const RowArgs*>(t + grp_row_off(G));
  const WgArgs* tw = reinterpret_cast<const WgArgs*>(t + grp_wg_off(G));
  const OptArgs* to = reinterpret_cast<const OptArgs*>(t + grp_opt_off(G));
  const GroupLim* tl = reinterpret_cast<const GroupLim*>(t + grp_lim_off(G));
  hipStream_t s = (hipStream_t)stream;
  const dim3 g1(plan->grid_rows, G), b4(256), b8(512);
  switch (plan->H / 64) {
    case 1: hipLaunchKernelGGL((ppo_rows_grp<1, 4, 16>), g1, b4, 0, s, tr, tl); break;
    case 2: hipLaunchKernelGGL((ppo_rows_grp<2, 8, 16>), g1, b8, 0, s, tr, tl); break;
    case 3: hipLaunchKernelGGL((ppo_rows_grp<3, 4, 16>), g1, b4, 0, s, tr, tl); break;
    case 4: hipLaunchKernelGGL((ppo_rows_grp<4, 8, 16>), g1, b8, 0, s, tr, tl); break;
    case 5: hipLaunchKernelGGL((ppo_rows_grp<5, 4, 16>), g1, b4, 0, s, tr, tl); break;
    case 6: hipLaunchKernelGGL((ppo_rows_grp<6, 8, 16>), g1, b8, 0, s, tr, tl); break;
    case 7: hipLaunchKernelGGL((ppo_rows_grp<7, 4, 16>), g1, b4, 0, s, tr, tl); break;
    default: hipLaunchKernelGGL((ppo_rows_grp<8, 8, 16>), g1, b8, 0, s, tr, tl); break;
  }
  int rc = hipGetLastError() == hipSuccess ? 0 : -1;
  hipLaunchKernelGGL(ppo_wgrad_grp, dim3(plan->grid_wgrad, G), dim3(64 * kWgWaves), 0, s, tw, tl);
  rc |= hipGetLastError() == hipSuccess ? 0 : -1;
  hipLaunchKernelGGL(ppo_wsum_grp, dim3(plan->grid_wsum, G), dim3(256), 0, s, tw, tl);
  rc |= hipGetLastError() == hipSuccess ? 0 : -1;
  hipLaunchKernelGGL(ppo_adam_tiles_grp, dim3(plan->grid_adam, G), dim3(256), 0, s, to, tl);
  rc |= hipGetLastError() == hipSuccess ? 0 : -1;
  return rc;
}

int64_t hwy_ppo_group_act_table_bytes(int G) {
  return G < 1 ? -1 : align256((int64_t)G * sizeof(ActArgs));
}

int hwy_ppo_group_act_prepare(const hwy_ppo_act_args* a, int G, void* table, void* stream) {
  if (!a || G < 1 || !table) return -1;
  const hwy_ppo_dims& d = a[0].dims;
  if (!fused_ok(d) || d.A != 2 || d.B < 1) return -1;
  const int64_t bytes = hwy_ppo_group_act_table_bytes(G);
  char* host = static_cast<char*>(calloc((size_t)bytes, 1));
  if (!host) return -2;
  int rc = 0;
  for (int g = 0; g < G; ++g) {
    const hwy_ppo_act_args& ag = a[g];
    // the learners share B and H (the kernel and its grid); S may differ per learner
    if (ag.dims.B != d.B || ag.dims.H != d.H || ag.dims.A != d.A || !fused_ok(ag.dims) ||
        !ag.states || !ag.params || !ag.action || !ag.pre_tanh || !ag.logp || !ag.value ||
        (!ag.tiles) != (!a[0].tiles) || (!ag.noise) != (!a[0].noise)) {
      rc = -1;
      break;
    }
    const Layout Lg = make_layout(ag.dims);
    ActArgs r = {};
    r.B = d.B, r.S = ag.dims.S, r.states = ag.states, r.params = ag.params, r.noise = ag.noise;
    for (int i = 0; i < 13; ++i) r.off[i] = Lg.off[i];
    r.action = ag.action, r.pre_tanh = ag.pre_tanh, r.logp = ag.logp, r.value = ag.value;
    r.tiles = ag.tiles;
    reinterpret_cast<ActArgs*>(host)[g] = r;
  }
  hipStream_t s = (hipStream_t)stream;
  if (rc == 0 && (hipMemcpyAsync(table, host, (size_t)bytes, hipMemcpyHostToDevice, s) != hipSuccess ||
                  hipStreamSynchronize(s) != hipSuccess))
    rc = -2;
  free(host);
  return rc;
}

int hwy_ppo_group_act(const hwy_ppo_dims* d, int G, int tiles, const void* table, void* stream) {
  if (!d || G < 1 || !table || !fused_ok(*d) || d->A != 2 || d->B < 1) return -1;
  const ActArgs* ta = static_cast<const ActArgs*>(table);
  hipStream_t s = (hipStream_t)stream;
  const dim3 g((d->B + kRowTile - 1) / kRowTile, G), b4(256), b8(512);
  auto launch = [&](auto tl) {
    constexpr bool TL = decltype(tl)::value;
    switch (d->H / 64) {
      case 1: hipLaunchKernelGGL((ppo_act_grp<1, 4, TL>), g, b4, 0, s, ta); break;
      case 2: hipLaunchKernelGGL((ppo_act_grp<2, 8, TL>), g, b8, 0, s, ta); break;
      case 3: hipLaunchKernelGGL((ppo_act_grp<3, 4, TL>), g, b4, 0, s, ta); break;
      case 4: hipLaunchKernelGGL((ppo_act_grp<4, 8, TL>), g, b8, 0, s, ta); break;
      case 5: hipLaunchKernelGGL((ppo_act_grp<5, 4, TL>), g, b4, 0, s, ta); break;
      case 6: hipLaunchKernelGGL((ppo_act_grp<6, 8, TL>), g, b8, 0, s, ta); break;
      case 7: hipLaunchKernelGGL((ppo_act_grp<7, 4, TL>), g, b4, 0, s, ta); break;
      default: hipLaunchKernelGGL((ppo_act_grp<8, 8, TL>), g, b8, 0, s, ta); break;
    }
  };
  // the solo hwy_ppo_act's kernel choice, per learner's B (so each learner's bits are its solo's)
  if (tiles && d->H == 256) {
    if (d->B >= 64 * chip_geom().cus)
      hipLaunchKernelGGL((ppo_act_c_grp<4, 8, 32>), dim3((d->B + 31) / 32, G), b8, 0, s, ta);
    else
      hipLaunchKernelGGL((ppo_act_c_grp<4, 8, 16>), dim3((d->B + 15) / 16, G), b8, 0, s, ta);
  } else if (tiles)
    launch(std::integral_constant<bool, true>());
  else
    launch(std::integral_constant<bool, false>());
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int hwy_ppo_build_flags(void) {
  int f = 0;
#ifdef HWY_DEV_KNOBS
  f |= 1;
#endif
#ifdef HWY_SECTION_PROFILE
  f |= 2;
#endif
  return f;
}

#ifdef HWY_CLOCK_PROBE
int hwy_ppo_debug_wgtimes(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ppo_wgt), sizeof(g_ppo_wgt)) == hipSuccess ? 0 : -2;
}
#endif
#if defined(HWY_SECTION_PROFILE) || defined(HWY_CLOCK_PROBE)
int hwy_ppo_debug_sections(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ppo_sections), sizeof(g_ppo_sections)) != hipSuccess)
    return -2;
  if (reset) {
    unsigned long long z[16] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_ppo_sections), z, sizeof(z)) != hipSuccess) return -2;
  }
  return 0;
}
#endif

}  // extern "C"
