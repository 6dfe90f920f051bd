// Micro-benchmark (development aid): sustained rate of v_mfma_f32_16x16x4_f32 on MI355X for the
// ppo_rows inner-loop shape -- per wave RB x TW = 2 x 2 accumulators, 16 MFMAs per 16-deep block
// -- at 1, 2 and 4 waves per SIMD, with operands (a) in registers, (b) A from LDS (ds_read_b128
// one block ahead) and B from a global ring (global_load_dwordx4, 2 blocks ahead) as ppo_rows_c
// streams them.  Prints TFLOP/s and the fraction of the 157.3 TF/s fp32 MFMA peak.
// Build: hipcc --offload-arch=gfx950 -O3 tools/micro/mfma_f32_rate.hip -o tools/micro/mfma_f32_rate
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int MODE, int RB = 2, int TW = 2>
__global__ void __launch_bounds__(1024) mfma_loop(const float* __restrict__ w, float* out, int nblk) {
  __shared__ __attribute__((aligned(16))) float act[16 * RB * 264];
  const int lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
  for (int i = threadIdx.x; i < 16 * RB * 264; i += blockDim.x) act[i] = 0.001f * (i % 97);
  __syncthreads();
  f32x4 acc[RB][TW] = {};
  f32x4 a_nxt[RB], buf[2][TW];
  const float* arow = act + c * 264 + 4 * g;
  // MODE & 4: every workgroup streams its own copy of the weights (no L2 line shared by CUs)
  const f32x4* wp = reinterpret_cast<const f32x4*>(w) + ((threadIdx.x >> 6) & 3) * 64 * 2 + lane +
                    ((MODE & 4) ? (size_t)(blockIdx.x % 64) * 65536 : 0);
  for (int rb = 0; rb < RB; ++rb)
    a_nxt[rb] = (MODE & 1) ? *reinterpret_cast<const f32x4*>(arow + 16 * rb * 264)
                           : f32x4{1.0f, 2.0f, 3.0f, 4.0f} * (float)(lane + rb);
  for (int d = 0; d < 2; ++d)
    for (int t = 0; t < TW; ++t)
      buf[d][t] = (MODE & 2) ? wp[(d * 2 + t) * 64 * 8] : f32x4{0.5f, 0.25f, 0.125f, 1.0f} * (float)(t + d);
  for (int b0 = 0; b0 < nblk; b0 += 2) {
#pragma unroll
    for (int d = 0; d < 2; ++d) {
      f32x4 a[RB];
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) {
        a[rb] = a_nxt[rb];
        if (MODE & 1)
          a_nxt[rb] = *reinterpret_cast<const f32x4*>(arow + 16 * rb * 264 + (((b0 + d + 1) & 15) * 16));
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int t = 0; t < TW; ++t)
#pragma unroll
          for (int rb = 0; rb < RB; ++rb) {
            if (MODE & 8)  // accumulator in AGPRs (timing only: no hazard padding)
              asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, %0"
                           : "+a"(acc[rb][t]) : "v"(a[rb][j]), "v"(buf[d][t][j]));
            else
              acc[rb][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[rb][j], buf[d][t][j], acc[rb][t], 0, 0, 0);
          }
      __builtin_amdgcn_sched_barrier(0);
      if (MODE & 2) {
#pragma unroll
        for (int t = 0; t < TW; ++t) buf[d][t] = wp[(((b0 + d + 2) & 63) * 2 + t) * 64 * 8];
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  float s = 0.0f;
  for (int rb = 0; rb < RB; ++rb)
    for (int t = 0; t < TW; ++t) s += acc[rb][t][0] + acc[rb][t][1] + acc[rb][t][2] + acc[rb][t][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// the ppo_wgrad chunk loop's shape: v_mfma_f32_32x32x2_f32, two accumulators per wave sharing
// the B operand, operands read from LDS per k-step (one float per lane per operand)
typedef __attribute__((address_space(3))) void lds_void_t;
template <int NDMA>
__global__ void __launch_bounds__(512) wg_loop(const float* __restrict__ src, float* out, int nchunk) {
  __shared__ __attribute__((aligned(16))) float lds[64 * 192 + (NDMA ? 8 * 6 * 256 : 4)];
  const int lane = threadIdx.x & 63, h = lane >> 5, l32 = lane & 31;
  for (int i = threadIdx.x; i < 64 * 192; i += blockDim.x) lds[i] = 0.001f * (i % 89);
  __syncthreads();
  typedef float f32x16 __attribute__((ext_vector_type(16)));
  f32x16 acc0 = {}, acc1 = {};
  for (int c = 0; c < nchunk; ++c) {
    const float* buf = lds + (c & 1) * 0;
    const float* pa0 = buf + h * 128 + l32;
    const float* pa1 = pa0 + 32 * (1 + 0);
    const float* pb = buf + 128 * 64 + h * 64 + l32;
    float x0[2][4], x1[2][4], y[2][4];
    auto rd = [&](int g, int b) {
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
      if (g + 1 < 4) rd(g + 1, b ^ 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(x0[b][j], y[b][j], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(x1[b][j], y[b][j], acc1, 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
      // NDMA LDS-DMA pieces (1 KB each) per chunk per wave, spread over the first groups, into a
      // scratch region nobody reads (issue cost only), as ppo_wgrad's staging issues them
      if (NDMA && g < 3) {
        const int w = threadIdx.x >> 6;
#pragma unroll
        for (int i = 0; i < NDMA / 3; ++i)
          __builtin_amdgcn_global_load_lds(
              (const void*)(src + ((size_t)((blockIdx.x * 8 + w) & 63) * 64 + (c & 63)) * 256 + 4 * lane),
              (lds_void_t*)(lds + 64 * 192 + (w * 6 + g * (NDMA / 3) + i) * 256), 16, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
  float s = 0.0f;
  for (int q = 0; q < 16; ++q) s += acc0[q] + acc1[q];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  std::vector<float> hw((size_t)65 * 65536 * 4, 0.01f);
  float *w, *out;
  hipMalloc(&w, hw.size() * 4);
  hipMemcpy(w, hw.data(), hw.size() * 4, hipMemcpyHostToDevice);
  hipMalloc(&out, (size_t)cus * 4 * 512 * 4);
  const int nblk = 4096;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int mode : {0})
    for (int wps : {1, 2, 4}) {  // waves per SIMD: workgroups of 4 waves x wps per CU
      const int threads = 256, grid = cus * wps;
      for (int rep = 0; rep < 2; ++rep) {
        hipEventRecord(e0);
        if (mode == 0)
          hipLaunchKernelGGL(mfma_loop<0>, dim3(grid), dim3(threads), 0, 0, w, out, nblk);
        else if (mode == 1)
          hipLaunchKernelGGL(mfma_loop<1>, dim3(grid), dim3(threads), 0, 0, w, out, nblk);
        else if (mode == 2)
          hipLaunchKernelGGL(mfma_loop<2>, dim3(grid), dim3(threads), 0, 0, w, out, nblk);
        else if (mode == 3)
          hipLaunchKernelGGL(mfma_loop<3>, dim3(grid), dim3(threads), 0, 0, w, out, nblk);
        else
          hipLaunchKernelGGL(mfma_loop<6>, dim3(grid), dim3(threads), 0, 0, w, out, nblk);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
      }
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      const double flop = (double)grid * 4 * nblk * 16 * 2048.0;
      const double tfs = flop / (ms * 1e-3) / 1e12;
      const char* names[7] = {"registers", "A lds", "B global", "A lds + B global", "", "",
                              "B global, private per workgroup"};
      printf("mode %s waves/SIMD %d: %.3f ms  %.1f TFLOP/s  frac %.3f\n", names[mode], wps, ms,
             tfs, tfs / 157.3);
    }
  // rows per weight load: RB = 4 (64-row tiles) against RB = 2, A from LDS and B from global
  for (int cfg = 0; cfg < 5; ++cfg)
    for (int wps : {1, 2}) {  // 256-thread workgroups (1 wave per SIMD each), wps per CU
      const int grid = cus * wps;
      for (int rep = 0; rep < 2; ++rep) {
        hipEventRecord(e0);
        if (cfg == 0)
          hipLaunchKernelGGL((mfma_loop<3, 2, 2>), dim3(grid), dim3(256), 0, 0, w, out, nblk);
        else if (cfg == 1)
          hipLaunchKernelGGL((mfma_loop<3, 4, 2>), dim3(grid), dim3(256), 0, 0, w, out, nblk);
        else if (cfg == 2)
          hipLaunchKernelGGL((mfma_loop<3, 4, 1>), dim3(grid), dim3(256), 0, 0, w, out, nblk);
        else if (cfg == 3)
          hipLaunchKernelGGL((mfma_loop<11, 2, 2>), dim3(grid), dim3(256), 0, 0, w, out, nblk);
        else
          hipLaunchKernelGGL((mfma_loop<11, 4, 2>), dim3(grid), dim3(256), 0, 0, w, out, nblk);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
      }
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      const int RBv[5] = {2, 4, 4, 2, 4}, TWv[5] = {2, 2, 1, 2, 2};
      const double flop = (double)grid * 4 * nblk * 4 * RBv[cfg] * TWv[cfg] * 2048.0;
      const double tfs = flop / (ms * 1e-3) / 1e12;
      printf("A lds + B global, RB %d TW %d (MFMAs per weight load %d)%s, waves/SIMD %d: %.1f TFLOP/s  frac %.3f\n",
             RBv[cfg], TWv[cfg], 4 * RBv[cfg], cfg >= 3 ? ", AGPR acc" : "", wps, tfs, tfs / 157.3);
    }
  for (int ndma : {0, 6})
  for (int wps : {1, 2}) {  // 512-thread workgroups: 2 waves per SIMD each; 1 or 2 per CU
    const int grid = cus * wps, nchunk = 2048;
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(e0);
      if (ndma)
        hipLaunchKernelGGL(wg_loop<6>, dim3(grid), dim3(512), 0, 0, w, out, nchunk);
      else
        hipLaunchKernelGGL(wg_loop<0>, dim3(grid), dim3(512), 0, 0, w, out, nchunk);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
    }
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double flop = (double)grid * 8 * nchunk * 32 * 4096.0;
    const double tfs = flop / (ms * 1e-3) / 1e12;
    printf("wgrad-shape 32x32x2 lds operands, %d LDS-DMA per chunk and wave, waves/SIMD %d: %.3f ms  %.1f TFLOP/s  frac %.3f\n",
           ndma, 2 * wps, ms, tfs, tfs / 157.3);
  }
  hipFree(w);
  hipFree(out);
  return 0;
}
