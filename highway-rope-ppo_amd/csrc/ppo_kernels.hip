// ppo_kernels.hip -- fused PPO minibatch step for gfx950 (include/hwy_ppo.h).
//
// One minibatch step of the reference's PPOAgent.update (ppo/agent.py:216-252) as 11 launches:
//   fwd:  h1 = relu(gather(states) W1^T + b1)            gemm64<A row-major+gather, B NT, bias+relu>
//         h2 = relu(h1 W2^T + b2)
//         ac = relu(h2 [Wa1;Wc1]^T + [ba1;bc1])          actor/critic first layers as one GEMM
//   head: mean, value, log-prob, entropy, ratio, clipped surrogate, MSE, their gradients, the
//         head weight/bias/log_std partials and the metrics, one row per thread-group pass
//   bwd:  dh2 = (dac [Wa1;Wc1]) * (h2 > 0)               gemm64<.., B NN, relu mask>
//         d[Wa1;Wc1] = dac^T h2, d[ba1;bc1] = colsum(dac)   split-K partial slabs
//         dh1 = (dh2 W2) * (h1 > 0); dW2 = dh2^T h1; dW1 = dh1^T gather(states)
//   reduce: partial slabs -> flat grads (fixed order, deterministic) + sum-of-squares partials
//   opt:  clip_grad_norm_ + Adam (torch.optim.Adam formula) over the flat parameter buffer
// GEMM core: 64x64 output tile per 256-thread workgroup, each wave a 32x32 tile accumulated
// with v_mfma_f32_32x32x2_f32 (exact fp32 products), K staged 32 at a time through LDS with
// the next tile prefetched into registers during the MFMAs.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hwy_ppo.h"

typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace {

constexpr int kTile = 64;
constexpr int kKStep = 32;
constexpr int kHeadRows = 16;  // minibatch rows per head workgroup (4 per wave)

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
  float *head_part;   // [nhead][HP]
  float *slab_ac, *bias_ac;  // [sa][2H][H], [sa][2H]
  float *slab_2, *bias_2;    // [s2][H][H], [s2][H]
  float *slab_1, *bias_1;    // [s1][H][S], [s1][H]
  float *norm_part;          // [nred]
  int nhead, HP, sa, s2, s1, ca, c2, c1, nred;
};

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
  int64_t sizes[14] = {
      (int64_t)B * H, (int64_t)B * H, (int64_t)B * 2 * H, (int64_t)B * 2 * H, (int64_t)B * H,
      (int64_t)B * H, (int64_t)w.nhead * w.HP, (int64_t)w.sa * 2 * H * H, (int64_t)w.sa * 2 * H,
      (int64_t)w.s2 * H * H, (int64_t)w.s2 * H, (int64_t)w.s1 * H * S, (int64_t)w.s1 * H,
      (int64_t)w.nred};
  float* p = (float*)ws;
  float** dst[14] = {&w.h1, &w.h2, &w.ac, &w.dac, &w.dh2, &w.dh1, &w.head_part, &w.slab_ac,
                     &w.bias_ac, &w.slab_2, &w.bias_2, &w.slab_1, &w.bias_1, &w.norm_part};
  int64_t total = 0;
  for (int i = 0; i < 14; ++i) {
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

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  return v;
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
    const float mu0 = wave_sum(p0) + ba0, mu1 = wave_sum(p1) + ba1, val = wave_sum(pv) + bcv;
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
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) sq += __shfl_xor(sq, o);
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
};

// sum of squares of the (all-reduced) gradient, same partition as ppo_reduce
__global__ void __launch_bounds__(kRedThreads) ppo_sumsq(const float* g, int64_t n, float* part) {
  __shared__ float red[kRedThreads / 64];
  const int64_t i = (int64_t)blockIdx.x * kRedThreads + threadIdx.x;
  float sq = i < n ? g[i] * g[i] : 0.0f;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) sq += __shfl_xor(sq, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = sq;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.0f;
    for (int k = 0; k < kRedThreads / 64; ++k) s += red[k];
    part[blockIdx.x] = s;
  }
}

__global__ void __launch_bounds__(256) ppo_adam(OptArgs o) {
  __shared__ float red[4];
  __shared__ float coef_s;
  float s = 0.0f;
  for (int k = threadIdx.x; k < o.nred; k += 256) s += o.norm_part[k];
#pragma unroll
  for (int q = 32; q >= 1; q >>= 1) s += __shfl_xor(s, q);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float total = sqrtf(((red[0] + red[1]) + red[2]) + red[3]);
    const float c = o.max_norm / (total + 1e-6f);
    coef_s = c < 1.0f ? c : 1.0f;
  }
  __syncthreads();
  const float coef = coef_s;
  const int t = o.counters[0];
  // torch.optim.Adam (foreach, non-capturable): bias corrections in double on the host side
  const double bc1 = 1.0 - pow((double)o.beta1, (double)t);
  const double bc2 = 1.0 - pow((double)o.beta2, (double)t);
  const float step_size = (float)((double)o.lr / bc1);
  const float bc2_sqrt = (float)sqrt(bc2);
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= o.numel) return;
  const float g = o.grads[i] * coef;
  float mm = o.m[i], vv = o.v[i];
  mm = mm + (1.0f - o.beta1) * (g - mm);  // exp_avg.lerp_(grad, 1 - beta1)
  vv = vv * o.beta2 + (1.0f - o.beta2) * g * g;
  o.m[i] = mm;
  o.v[i] = vv;
  const float denom = sqrtf(vv) / bc2_sqrt + o.eps;
  o.params[i] = o.params[i] - step_size * (mm / denom);
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

int hwy_ppo_forward_backward(const hwy_ppo_args* a, void* stream) {
  if (!a) return -1;
  const hwy_ppo_dims& d = a->dims;
  if (hwy_ppo_workspace_bytes(&d) < 0) return -1;
  hipStream_t s = (hipStream_t)stream;
  const int B = d.B, S = d.S, H = d.H;
  const Layout L = make_layout(d);
  Work w = carve(d, a->workspace, nullptr);
  const float* P = a->params;
  int rc = 0;
  // ---- forward
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
  OptArgs o = {};
  o.params = a->params, o.grads = a->grads, o.m = a->adam_m, o.v = a->adam_v;
  o.norm_part = w.norm_part, o.nred = w.nred, o.numel = L.numel, o.counters = a->counters;
  o.lr = a->lr, o.beta1 = a->beta1, o.beta2 = a->beta2, o.eps = a->adam_eps;
  o.max_norm = a->max_grad_norm;
  hipLaunchKernelGGL(ppo_adam, dim3(w.nred), dim3(256), 0, s, o);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // extern "C"
