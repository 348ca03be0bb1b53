// Peak of v_mfma_f64_16x16x4f64 on gfx950: 16 independent accumulators per wave, back-to-back issue.
// hipcc --offload-arch=gfx950 -O3 tools/mb/f64_mfma_mb.hip -o tools/mb/f64_mfma_mb
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double f64x4 __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(256) mfma_loop(double* out, int iters, double a0) {
  f64x4 acc[16];
  for (int i = 0; i < 16; ++i) acc[i] = f64x4{0, 0, 0, 0};
  double a = a0 + threadIdx.x, b = a0 * 0.5;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  }
  double s = 0;
  for (int i = 0; i < 16; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  double* out;
  const int per_cu[] = {1, 2, 4};
  hipMalloc(&out, sizeof(double) * 256 * cus * 8);
  const int iters = 4096;
  for (int w : per_cu) {
    const int blocks = cus * w;
    hipLaunchKernelGGL(mfma_loop, dim3(blocks), dim3(256), 0, 0, out, 16, 1.0);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(mfma_loop, dim3(blocks), dim3(256), 0, 0, out, iters, 1.0);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double flop = 2.0 * 16 * 16 * 4 * 16.0 * iters * (blocks * 4.0);
    printf("{\"blocks_per_cu\": %d, \"waves_per_simd\": %d, \"ms\": %.3f, \"tflops_f64\": %.1f}\n", w, w, ms,
           flop / ms / 1e9);
  }
  return 0;
}
