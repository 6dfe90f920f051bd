// Micro-benchmark (development aid): the 16-row ppo_rows inner loop (RB = 1: every weight
// fragment feeds 4 MFMAs) at 2 and 4 waves per SIMD, one workgroup per CU, with the weights
// streamed (a) into VGPRs by global_load_dwordx4 (the product ring), (b) into a per-wave LDS ring
// by LDS-DMA (global_load_lds_dwordx4: the tile image's 1-KB blocks are lane-linear, so the DMA
// destination needs no swizzle) and read back with ds_read_b128 one block later.  Every wave
// streams its own columns of a 1.6 MB image shared by all CUs (L2-resident), as the row kernel
// does at 4,096-row minibatches.  Prints TFLOP/s, the fraction of the 157.3 TF/s fp32 MFMA peak
// and the weight bytes per CU per microsecond.
// Build: hipcc --offload-arch=gfx950 -O3 tools/micro/rows16_stream.hip -o tools/micro/rows16_stream
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void_t;

constexpr int kImgBlocks = 2048;  // 1-KB blocks in the weight image (2 MB, L2-resident)

// MODE 0: global -> VGPR ring (D blocks in flight); MODE 1: LDS-DMA ring (D slots per wave)
template <int MODE, int TW, int D, int NW, int ROT = 0>
__global__ void __launch_bounds__(64 * NW) rows16(const float* __restrict__ w, float* out,
                                                   int nblk) {
  constexpr int PA = 264;
  __shared__ __attribute__((aligned(16))) float lds[16 * PA + (MODE == 1 ? NW * D * TW * 256 : 4)];
  const int lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15, wv = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < 16 * PA; i += 64 * NW) lds[i] = 0.001f * (i % 97);
  __syncthreads();
  f32x4 acc[TW] = {};
  const float* arow = lds + c * PA + 4 * g;
  // block b of tile t of this wave: image block ((wv * TW + t) * 97 + b) mod kImgBlocks
  // ROT: every workgroup starts at another image offset (a per-CU rotation of which columns a
  // wave streams, so the CUs of an XCD do not all hit the same L2 lines at the same moment)
  const int rot = ROT ? (int)blockIdx.x * ROT : 0;
  auto src = [&](int b, int t) {
    return w + (size_t)((((wv * TW + t) * 97 + b + rot) & (kImgBlocks - 1)) * 256) + 4 * lane;
  };
  f32x4 a_nxt = *reinterpret_cast<const f32x4*>(arow);
  if constexpr (MODE == 0) {
    f32x4 buf[D][TW];
#pragma unroll
    for (int d = 0; d < D; ++d)
#pragma unroll
      for (int t = 0; t < TW; ++t) buf[d][t] = *reinterpret_cast<const f32x4*>(src(d, t));
    __builtin_amdgcn_sched_barrier(0);
    for (int b0 = 0; b0 < nblk; b0 += D) {
#pragma unroll
      for (int d = 0; d < D; ++d) {
        const f32x4 a = a_nxt;
        a_nxt = *reinterpret_cast<const f32x4*>(arow + (((b0 + d + 1) & 15) * 16));
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int t = 0; t < TW; ++t)
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j], buf[d][t][j], acc[t], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int t = 0; t < TW; ++t) buf[d][t] = *reinterpret_cast<const f32x4*>(src(b0 + d + D, t));
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  } else {
    float* ring = lds + 16 * PA + wv * D * TW * 256;
    auto dma = [&](int b, int d) {
#pragma unroll
      for (int t = 0; t < TW; ++t)
        __builtin_amdgcn_global_load_lds((const void*)src(b, t),
                                         (lds_void_t*)(ring + (d * TW + t) * 256), 16, 0, 0);
    };
#pragma unroll
    for (int d = 0; d < D; ++d) dma(d, d);
    for (int b0 = 0; b0 < nblk; b0 += D) {
#pragma unroll
      for (int d = 0; d < D; ++d) {
        // this block's DMAs landed (the D - 1 younger blocks' may still be in flight)
        if constexpr (D == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(1 * TW) : "memory");
        else if constexpr (D == 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * TW) : "memory");
        else if constexpr (D == 4) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * TW) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(5 * TW) : "memory");
        f32x4 bb[TW];
#pragma unroll
        for (int t = 0; t < TW; ++t)
          bb[t] = *reinterpret_cast<const f32x4*>(ring + (d * TW + t) * 256 + 4 * lane);
        const f32x4 a = *reinterpret_cast<const f32x4*>(arow + (((b0 + d) & 15) * 16));
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int t = 0; t < TW; ++t)
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j], bb[t][j], acc[t], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        dma(b0 + d + D, d);  // the slot was read (its values fed the MFMAs): refill it
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  float s = 0.0f;
#pragma unroll
  for (int t = 0; t < TW; ++t) s += acc[t][0] + acc[t][1] + acc[t][2] + acc[t][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int MODE, int TW, int D, int NW, int ROT = 0>
void run(const char* name, int cus, const float* w, float* out) {
  const int nblk = 2048;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  float ms = 0;
  for (int rep = 0; rep < 3; ++rep) {
    hipEventRecord(e0);
    hipLaunchKernelGGL((rows16<MODE, TW, D, NW, ROT>), dim3(cus), dim3(64 * NW), 0, 0, w, out, nblk);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
  }
  const double flop = (double)cus * NW * nblk * 4 * TW * 2048.0;
  const double tfs = flop / (ms * 1e-3) / 1e12;
  const double bytes_cu = (double)NW * nblk * TW * 1024.0;  // weight bytes per CU
  printf("%-34s ROT %d TW %d D %d waves/SIMD %d: %.3f ms  %.1f TFLOP/s  frac %.3f  weights %.1f GB/s/CU\n",
         name, ROT, TW, D, NW / 4, ms, tfs, tfs / 157.3, bytes_cu / (ms * 1e-3) / 1e9);
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  std::vector<float> hw((size_t)kImgBlocks * 256, 0.01f);
  for (size_t i = 0; i < hw.size(); ++i) hw[i] = 0.001f * (float)(i % 89);
  float *w, *out;
  hipMalloc(&w, hw.size() * 4);
  hipMemcpy(w, hw.data(), hw.size() * 4, hipMemcpyHostToDevice);
  hipMalloc(&out, (size_t)cus * 1024 * 4);
  for (int rep = 0; rep < 2; ++rep) {
    run<0, 2, 4, 8, 0>("global->VGPR ring (product)", cus, w, out);
    run<0, 2, 4, 8, 16>("global->VGPR ring, rotated", cus, w, out);
    run<0, 2, 4, 8, 61>("global->VGPR ring, rotated", cus, w, out);
    run<1, 2, 4, 8, 61>("LDS-DMA ring, rotated", cus, w, out);
    run<1, 2, 6, 8, 61>("LDS-DMA ring, rotated", cus, w, out);
    run<1, 2, 6, 8, 0>("LDS-DMA ring", cus, w, out);
    run<0, 2, 4, 8, 0>("global->VGPR ring (product)", cus, w, out);
    run<0, 1, 4, 16>("global->VGPR ring", cus, w, out);
    run<1, 2, 2, 8>("LDS-DMA ring", cus, w, out);
    run<1, 2, 3, 8>("LDS-DMA ring", cus, w, out);
    run<1, 2, 4, 8>("LDS-DMA ring", cus, w, out);
    run<1, 1, 4, 16>("LDS-DMA ring", cus, w, out);
    run<1, 4, 4, 4>("LDS-DMA ring", cus, w, out);
  }
  hipFree(w);
  hipFree(out);
  return 0;
}
