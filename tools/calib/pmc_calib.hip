// pmc_calib.hip -- known-byte-count kernels for calibrating rocprofv3 FETCH_SIZE / WRITE_SIZE on
// the access pattern of hwy_step_kernel (4-byte lanes, one 256-B row per wave per field,
// field-major [field][env][64]).  Measurement tooling only (tools/pmc_step.sh).
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ void __launch_bounds__(256) calib_read(const uint32_t* __restrict__ src, int nfields,
                                                  long fstride, uint32_t* __restrict__ sink) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  uint32_t acc = 0;
  for (int f = 0; f < nfields; ++f) acc ^= src[f * fstride + idx];
  if (acc == 0x9e3779b9u) sink[0] = acc;  // practically never: keeps the loads alive
}

__global__ void __launch_bounds__(256) calib_write(uint32_t* __restrict__ dst, int nfields,
                                                   long fstride) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  for (int f = 0; f < nfields; ++f) dst[f * fstride + idx] = (uint32_t)(idx + f);
}

extern "C" int calib_run(void* buf, void* sink, int nfields, long fstride, void* stream) {
  const int blocks = (int)(fstride / 256);
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(calib_read, dim3(blocks), dim3(256), 0, s, (const uint32_t*)buf, nfields,
                     fstride, (uint32_t*)sink);
  hipLaunchKernelGGL(calib_write, dim3(blocks), dim3(256), 0, s, (uint32_t*)buf, nfields, fstride);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
