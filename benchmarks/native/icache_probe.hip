// Instruction-fetch cost of a small launch: one 64-thread block executes N dependent v_add_f32, either as N
// straight-line instructions (N * 8 bytes of code, fetched once each) or as a 64-instruction loop body run N / 64
// times (512 bytes of code).  Same VALU work, different code footprint; kernel durations come from
// `rocprofv3 --kernel-trace --stats`.  Build: hipcc --offload-arch=gfx950 -O3 icache_probe.hip -o icache_probe
#include <hip/hip_runtime.h>
#include <cstdio>

#define ADD1 "v_add_f32 %0, %0, %1\n"
#define ADD8 ADD1 ADD1 ADD1 ADD1 ADD1 ADD1 ADD1 ADD1
#define ADD64 ADD8 ADD8 ADD8 ADD8 ADD8 ADD8 ADD8 ADD8

template <int N>
__global__ void __launch_bounds__(64) straight_kernel(float* out, float b) {
  float a = threadIdx.x;
#pragma unroll
  for (int i = 0; i < N / 64; ++i) asm volatile(ADD64 : "+v"(a) : "v"(b));
  out[threadIdx.x] = a;
}

template <int N>
__global__ void __launch_bounds__(64) loop_kernel(float* out, float b) {
  float a = threadIdx.x;
#pragma unroll 1
  for (int i = 0; i < N / 64; ++i) asm volatile(ADD64 : "+v"(a) : "v"(b));
  out[threadIdx.x] = a;
}

template <int N>
void run(float* d, int reps) {
  for (int r = 0; r < reps; ++r) {
    hipLaunchKernelGGL(straight_kernel<N>, dim3(1), dim3(64), 0, 0, d, 1.0f);
    hipLaunchKernelGGL(loop_kernel<N>, dim3(1), dim3(64), 0, 0, d, 1.0f);
  }
}

int main() {
  float* d;
  if (hipMalloc(&d, 256 * sizeof(float)) != hipSuccess) return 1;
  const int reps = 200;
  run<64>(d, reps);
  run<512>(d, reps);
  run<2048>(d, reps);
  run<8192>(d, reps);
  run<16384>(d, reps);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  std::printf("icache_probe done\n");
  hipFree(d);
  return 0;
}
