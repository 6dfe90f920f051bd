// Micro-benchmark (development aid): the cross-CU hand-offs a weight-stationary cluster split of
// ppo_rows would add (DESIGN.md §3 "Round 6: the weight-stationary cluster
// split").  The split: k = 4 CUs of one XCD share a 64-row tile, each owning 64 of the 256 output
// columns of every layer, so each CU streams 1/4 of the weight image.  Every layer boundary then
// becomes a hand-off inside the launch -- h1, h2, the loss head's partial dot products, dac,
// dh2: five per tile -- in which each CU publishes its 64 x 64 fp32 slice (16 KB) and reads the
// other three (48 KB).
//
// One launch = 256 workgroups of 8 waves (one per CU, as ppo_rows), 64 clusters of 4 with equal
// blockIdx % 8 (one XCD under round-robin placement: speed only).  Per tile, six phases: a work
// phase (each wave streams W 1-KB weight blocks from an L2-resident 1.6 MB image, every block
// feeding 16 MFMAs 16x16x4 f32 -- the cluster split's 64 rows per fragment) followed, except
// after the last, by a seam:
//   publish: every thread stores its 32 B of the slice with write-through (sc1) dwordx4 stores,
//            every wave waits for its stores (s_waitcnt vmcnt(0)), workgroup barrier, one lane
//            adds 1 to the cluster's counter (agent-scope atomic);
//   wait:    one lane polls the counter with sc1 loads (s_sleep between polls, bounded) until
//            all four members have published this seam; workgroup barrier;
//   read:    every thread loads its 96 B of the three peer slices with sc1 dwordx4 loads
//            (the guide's hand-off form R1: sc1 stores + drained flag + sc1 loads).
// Every word read is checked against the value its producer wrote; mismatches and poll
// timeouts are counted (a wrong protocol shows up as errors, a stuck one as timeouts, never as a
// hang).  Variants: work only (no seams), seams only (W = 0), work + seams.  The seam cost is
// (work + seams) - (work only), per launch; the split pays off only if five seams cost less than
// the ~13 us of weight stream it removes at 4,096 rows.
// Build: hipcc --offload-arch=gfx950 -O3 tools/micro/cluster_seams.hip -o tools/micro/cluster_seams
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kImgBlocks = 1664;  // 1.6 MB weight image (L2-resident)
constexpr int kNW = 8;            // waves per workgroup
constexpr int kK = 4;             // CUs per cluster
constexpr int kSlice = 64 * 64;   // floats per published slice (16 KB)
constexpr int kPhases = 6;        // work phases per tile; kPhases - 1 seams
constexpr int kPollCap = 400000;

// The s_nop: a VALU write to the data registers of a store wider than 8 bytes needs one wait
// state after the store, and the compiler's hazard recognizer does not look inside this asm (the
// first build overwrote v[34:37] right after the store: 12.5 % of the words arrived corrupted).
__device__ __forceinline__ void store_wt(float* p, f32x4 v) {
  asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}
// six write-through loads in flight, then one wait: a single asm statement, so the compiler cannot
// touch a destination register before the loads have landed
__device__ __forceinline__ void load6_wt(f32x4 (&v)[6], const float* const (&p)[6]) {
  asm volatile(
      "global_load_dwordx4 %0, %6, off sc1\n"
      "global_load_dwordx4 %1, %7, off sc1\n"
      "global_load_dwordx4 %2, %8, off sc1\n"
      "global_load_dwordx4 %3, %9, off sc1\n"
      "global_load_dwordx4 %4, %10, off sc1\n"
      "global_load_dwordx4 %5, %11, off sc1\n"
      "s_waitcnt vmcnt(0)"
      : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4]), "=&v"(v[5])
      : "v"(p[0]), "v"(p[1]), "v"(p[2]), "v"(p[3]), "v"(p[4]), "v"(p[5])
      : "memory");
}
__device__ __forceinline__ float tagval(int cluster, int member, int seam, int launch, int i) {
  return (float)(((cluster * 7 + member * 3 + seam * 11 + launch * 13) & 1023) * 4096 + (i & 4095));
}

template <int SEAMS>
__global__ void __launch_bounds__(64 * kNW) cluster_tile(const float* __restrict__ w,
                                                         float* slab, int* counters, int* err,
                                                         float* out, int W, int launch,
                                                         int* wg_xcc, int* wg_bad) {
  const int b = blockIdx.x, lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int cluster = (b & 7) + 8 * ((b >> 3) / kK), member = (b >> 3) % kK;
  const int nclusters = gridDim.x / kK;
  __shared__ int s_timeout;
  if (threadIdx.x == 0) s_timeout = 0;
  __syncthreads();
  f32x4 acc[4] = {};
  f32x4 a = {0.001f, 0.002f, 0.003f, 0.004f};
  float check = 0.0f;
  int bad = 0;
  // slab: [seam][cluster][member][kSlice]
  for (int ph = 0; ph < kPhases; ++ph) {
    // work: this wave's W weight blocks, 16 MFMAs each (64 rows x 16 columns x k 4 per block)
    const int base = ((b * kNW + wv) * 37 + ph * 101) % kImgBlocks;
    f32x4 buf[4];
#pragma unroll
    for (int d = 0; d < 4; ++d)
      buf[d] = *reinterpret_cast<const f32x4*>(w + (size_t)((base + d) % kImgBlocks) * 256 + 4 * lane);
    for (int i = 0; i < W; i += 4) {
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const f32x4 bb = buf[d];
        buf[d] = *reinterpret_cast<const f32x4*>(w + (size_t)((base + i + d + 4) % kImgBlocks) * 256 + 4 * lane);
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            acc[r] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j], bb[j], acc[r], 0, 0, 0);
      }
    }
    if (!SEAMS || ph == kPhases - 1) continue;
    const int seam = ph;
    // publish this member's slice: 32 B per thread, write-through
    float* mine = slab + ((size_t)(seam * nclusters + cluster) * kK + member) * kSlice;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int i = (q * 64 * kNW + threadIdx.x) * 4;
      f32x4 v;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = tagval(cluster, member, seam, launch, i + e) + acc[0][0] * 0.0f;
      store_wt(mine + i, v);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const int target = (launch * (kPhases - 1) + seam + 1) * kK;
    if (threadIdx.x == 0) {
      __hip_atomic_fetch_add(counters + cluster, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      int it = 0;
      if (!s_timeout) {
        while (__hip_atomic_load(counters + cluster, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
          __builtin_amdgcn_s_sleep(1);
          if (++it == kPollCap) {
            s_timeout = 1;
            atomicAdd(err + 1, 1);
            break;
          }
        }
      }
    }
    __syncthreads();
    // read the three peer slices: 96 B per thread, write-through loads
    f32x4 v[6];
    const float* p[6];
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      const int peer = (member + 1 + q / 2) % kK;
      const int i = ((q & 1) * 64 * kNW + threadIdx.x) * 4;
      p[q] = slab + ((size_t)(seam * nclusters + cluster) * kK + peer) * kSlice + i;
    }
    load6_wt(v, p);
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      const int peer = (member + 1 + q / 2) % kK;
      const int i = ((q & 1) * 64 * kNW + threadIdx.x) * 4;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        bad += v[q][e] != tagval(cluster, peer, seam, launch, i + e);
        check += v[q][e];
      }
    }
    a[0] += check * 1e-30f;
  }
  if (bad && !s_timeout) atomicAdd(err, bad);
  if (threadIdx.x == 0) wg_xcc[b] = __builtin_amdgcn_s_getreg((3 << 11) | 20);  // HW_REG_XCC_ID[3:0]
  if (bad) atomicAdd(wg_bad + b, bad);
  float s = check;
#pragma unroll
  for (int r = 0; r < 4; ++r) s += acc[r][0] + acc[r][1] + acc[r][2] + acc[r][3];
  out[b * blockDim.x + threadIdx.x] = s;
}

int *g_xcc, *g_bad;

template <int SEAMS>
float run(const char* name, int W, const float* w, float* slab, int* counters, int* err,
          float* out, int& launch, int reps) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipMemset(counters, 0, 64 * sizeof(int) * 4);
  hipMemset(err, 0, 2 * sizeof(int));
  hipMemset(g_bad, 0, 256 * sizeof(int));
  launch = 0;
  for (int i = 0; i < 3; ++i, ++launch)  // warm-up
    hipLaunchKernelGGL(cluster_tile<SEAMS>, dim3(256), dim3(64 * kNW), 0, 0, w, slab, counters, err,
                       out, W, launch, g_xcc, g_bad);
  hipEventRecord(e0);
  for (int i = 0; i < reps; ++i, ++launch)
    hipLaunchKernelGGL(cluster_tile<SEAMS>, dim3(256), dim3(64 * kNW), 0, 0, w, slab, counters, err,
                       out, W, launch, g_xcc, g_bad);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  int herr[2];
  hipMemcpy(herr, err, sizeof(herr), hipMemcpyDeviceToHost);
  const float us = ms * 1e3f / reps;
  if (herr[0]) {  // which workgroups read stale words: by XCC of the cluster's members
    int xcc[256], bad[256];
    hipMemcpy(xcc, g_xcc, sizeof(xcc), hipMemcpyDeviceToHost);
    hipMemcpy(bad, g_bad, sizeof(bad), hipMemcpyDeviceToHost);
    int split = 0, split_bad = 0, same_bad = 0, nbad = 0;
    for (int c = 0; c < 64; ++c) {
      int m[4], any = 0;
      for (int j = 0; j < 4; ++j) m[j] = (c & 7) + 8 * (4 * (c >> 3) + j);
      const bool same = xcc[m[0]] == xcc[m[1]] && xcc[m[0]] == xcc[m[2]] && xcc[m[0]] == xcc[m[3]];
      for (int j = 0; j < 4; ++j) any += bad[m[j]], nbad += bad[m[j]] > 0;
      split += !same;
      if (same) same_bad += any; else split_bad += any;
    }
    printf("    clusters spanning XCCs %d/64; stale words in them %d, in single-XCC clusters %d; workgroups with stale reads %d/256\n",
           split, split_bad, same_bad, nbad);
    printf("    xcc of blocks 0..15:");
    for (int i = 0; i < 16; ++i) printf(" %d", xcc[i]);
    printf("\n");
  }
  printf("%-22s W %3d blocks/wave/phase: %8.2f us per launch  (mismatched words %d, poll timeouts %d)\n",
         name, W, us, herr[0], herr[1]);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  return us;
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  printf("CUs %d; 256 workgroups x %d waves, clusters of %d, %d seams per launch, %d KB published / %d KB read per seam per CU\n",
         cus, kNW, kK, kPhases - 1, kSlice * 4 / 1024, 3 * kSlice * 4 / 1024);
  std::vector<float> hw((size_t)kImgBlocks * 256);
  for (size_t i = 0; i < hw.size(); ++i) hw[i] = 0.001f * (float)(i % 89);
  float *w, *slab, *out;
  int *counters, *err;
  hipMalloc(&w, hw.size() * 4);
  hipMemcpy(w, hw.data(), hw.size() * 4, hipMemcpyHostToDevice);
  hipMalloc(&slab, (size_t)(kPhases - 1) * 64 * kK * kSlice * 4);
  hipMalloc(&counters, 64 * sizeof(int) * 4);
  hipMalloc(&err, 2 * sizeof(int));
  hipMalloc(&g_xcc, 256 * sizeof(int));
  hipMalloc(&g_bad, 256 * sizeof(int));
  hipMalloc(&out, 256 * 64 * kNW * 4);
  int launch = 0;
  const int reps = 200;
  // the cluster split's per-CU weight stream at 4,096 rows: 1.6 MB / 4 = 400 KB = 400 blocks per
  // CU = 50 per wave over the tile, ~8 per phase
  for (int round = 0; round < 2; ++round) {
    run<0>("empty phases", 0, w, slab, counters, err, out, launch, reps);
    const float s0 = run<1>("seams only", 0, w, slab, counters, err, out, launch, reps);
    for (int W : {8, 16}) {
      const float a = run<0>("work only", W, w, slab, counters, err, out, launch, reps);
      const float b = run<1>("work + seams", W, w, slab, counters, err, out, launch, reps);
      printf("  -> seams beside work W %d: +%.2f us per launch (%.2f us per seam); seams alone %.2f\n",
             W, b - a, (b - a) / (kPhases - 1), s0);
    }
  }
  hipFree(w);
  hipFree(slab);
  hipFree(counters);
  hipFree(err);
  hipFree(out);
  return 0;
}
