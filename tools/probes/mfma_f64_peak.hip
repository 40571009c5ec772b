// Achievable v_mfma_f64_16x16x4_f64 (and v_fma_f64) rate on this MI355X: every wave issues back-to-back MFMAs
// into 8 independent accumulators (no memory traffic), grid = 256 CUs x 4 SIMDs x WPS waves.
// Build: hipcc --offload-arch=gfx950 -O3 tools/probes/mfma_f64_peak.hip -o build/mfma_f64_peak
#include <hip/hip_runtime.h>

#include <cstdio>

typedef double f64x4 __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(256) peak(double* out, int iters, double a, double b) {
  f64x4 acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = f64x4{0, 0, 0, 0};
  const double x = a + threadIdx.x * 1e-9, y = b - threadIdx.x * 1e-9;
  for (int it = 0; it < iters; ++it)
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, acc[i], 0, 0, 0);
  double s = 0;
  for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  if (s == 12345.678) out[0] = s;  // keep the chain alive
}

__global__ void __launch_bounds__(256) valu_peak(double* out, int iters, double a, double b) {
  double acc[16];
  for (int i = 0; i < 16; ++i) acc[i] = a + i * 1e-3 + threadIdx.x * 1e-9;
  const double y = b - threadIdx.x * 1e-9;
  for (int it = 0; it < iters; ++it)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = fma(acc[i], y, a);
  double s = 0;
  for (int i = 0; i < 16; ++i) s += acc[i];
  if (s == 12345.678) out[0] = s;
}

int main() {
  double* out;
  hipMalloc(&out, 8);
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int iters = 2000;
  for (int wps : {1, 2, 4}) {  // waves per SIMD
    const int blocks = cus * wps;  // 256-thread blocks = 4 waves = one per SIMD
    hipLaunchKernelGGL(peak, dim3(blocks), dim3(256), 0, 0, out, 10, 1.0, 2.0);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(peak, dim3(blocks), dim3(256), 0, 0, out, iters, 1.0, 2.0);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double flop = 2.0 * 16 * 16 * 4 * 8.0 * iters * blocks * 4;
    printf("{\"waves_per_simd\": %d, \"ms\": %.4f, \"TFLOPs\": %.2f, \"cus\": %d}\n", wps, ms, flop / ms / 1e9, cus);
  }
  for (int wps : {1, 2, 4}) {
    const int blocks = cus * wps;
    hipLaunchKernelGGL(valu_peak, dim3(blocks), dim3(256), 0, 0, out, 10, 1.0, 0.999);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(valu_peak, dim3(blocks), dim3(256), 0, 0, out, iters * 8, 1.0, 0.999);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double flop = 2.0 * 16 * iters * 8.0 * blocks * 256;
    printf("{\"valu_fma_f64_waves_per_simd\": %d, \"ms\": %.4f, \"TFLOPs\": %.2f}\n", wps, ms, flop / ms / 1e9);
  }
  return 0;
}
