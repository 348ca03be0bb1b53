// The headline's timed region with no Python in the way: a 406 MB bf16 ring (26 x 8192 x 1000), W = 5 warm-up
// launches, a 4-byte device->host read (compute()'s validation word), a memset (reset), a device sync, then 4 regions
// of [20 launches (host timestamp after each) + 4-byte read + hipDeviceSynchronize].  One JSON line per process: run it
// under different HIP runtime environments to see which part of the first region is the runtime's.
// Kernel: one row per wave, 2 x 16 B per lane, order-key max + int64 atomic into a 1000 x 1000 matrix (the shape of
// mc_argmax_ord16_kernel).  Build: hipcc -O3 --offload-arch=gfx950 region_mb.hip -o region_mb
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::printf("{\"error\": \"%s\", \"line\": %d}\n", hipGetErrorString(e_), __LINE__); \
      std::exit(1);                                                            \
    }                                                                          \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(512) row_max_kernel(const uint16_t* __restrict__ preds, const int64_t* __restrict__ target,
                                                      int N, int C, unsigned long long* __restrict__ cm) {
  const int lane = threadIdx.x & 63;
  const int row = (blockIdx.x * blockDim.x + threadIdx.x) / 64;
  if (row >= N) return;
  const u32x4* rp = reinterpret_cast<const u32x4*>(preds + (long long)row * C);
  const int nch = C / 8;
  uint32_t best = 0, bi = 0;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int ci = lane + 64 * j;
    if (ci < nch) {
      const u32x4 v = __builtin_nontemporal_load(rp + ci);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t lo = v[k] & 0xffffu, hi = v[k] >> 16;
        if (lo > best) { best = lo; bi = ci * 8 + 2 * k; }
        if (hi > best) { best = hi; bi = ci * 8 + 2 * k + 1; }
      }
    }
  }
  uint32_t key = (best << 16) | (0xffffu - bi);
  for (int off = 32; off > 0; off >>= 1) {
    const uint32_t o = __shfl_xor(key, off, 64);
    key = o > key ? o : key;
  }
  if (lane == 0) {
    const long long t = target[row];
    if (t >= 0 && t < C) atomicAdd(cm + t * C + (0xffffu - (key & 0xffffu)) % C, 1ull);
  }
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const int C = 1000, B = 8192, K = 26, W = 5, STEPS = 20, REPS = 4;
  const char* label = argc > 1 ? argv[1] : "default";
  // compute()'s completion check: memcpy (a 4-byte device->host read, as .item()), streamsync (hipStreamSynchronize
  // then a host-memory read), eventsync (record + hipEventSynchronize), none (only the final device sync)
  const char* cmode = argc > 2 ? argv[2] : "memcpy";
  hipEvent_t ev_done;
  CK(hipEventCreateWithFlags(&ev_done, hipEventDisableTiming));
  uint16_t* ring;
  int64_t* tgt;
  unsigned long long* cm;
  int* word;
  CK(hipMalloc(&ring, (size_t)K * B * C * 2));
  CK(hipMalloc(&tgt, (size_t)K * B * 8));
  CK(hipMalloc(&cm, (size_t)C * C * 8));
  CK(hipMalloc(&word, 4));
  CK(hipMemset(ring, 0x3c, (size_t)K * B * C * 2));
  std::vector<int64_t> ht((size_t)K * B);
  for (size_t i = 0; i < ht.size(); ++i) ht[i] = (i * 2654435761u) % C;
  CK(hipMemcpy(tgt, ht.data(), ht.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemset(cm, 0, (size_t)C * C * 8));
  CK(hipMemset(word, 0, 4));
  CK(hipDeviceSynchronize());
  const dim3 grid(B / 8), block(512);
  auto launch = [&](int slot) {
    hipLaunchKernelGGL(row_max_kernel, grid, block, 0, 0, ring + (size_t)slot * B * C, tgt + (size_t)slot * B, B, C, cm);
  };
  int host_word = 0;
  for (int i = 0; i < W; ++i) launch(i % K);
  CK(hipMemcpy(&host_word, word, 4, hipMemcpyDeviceToHost));
  CK(hipMemsetAsync(cm, 0, (size_t)C * C * 8, 0));
  CK(hipDeviceSynchronize());
  std::printf("{\"case\": \"%s\", \"compute_mode\": \"%s\"", label, cmode);
  for (int rep = 0; rep < REPS; ++rep) {
    double ts[STEPS + 1];
    const double t0 = now_us();
    ts[0] = t0;
    for (int i = 0; i < STEPS; ++i) {
      launch((W + rep * STEPS + i) % K);
      ts[i + 1] = now_us();
    }
    if (cmode[0] == 'm') {
      CK(hipMemcpy(&host_word, word, 4, hipMemcpyDeviceToHost));
    } else if (cmode[0] == 's') {
      CK(hipStreamSynchronize(0));
    } else if (cmode[0] == 'e') {
      CK(hipEventRecord(ev_done, 0));
      CK(hipEventSynchronize(ev_done));
    }
    const double t2 = now_us();
    CK(hipDeviceSynchronize());
    const double t3 = now_us();
    std::printf(", \"rep%d\": [%.1f, %.1f, %.1f, %.1f], \"launch%d\": [", rep, t3 - t0, ts[STEPS] - t0, t2 - ts[STEPS],
                t3 - t2, rep);
    for (int i = 0; i < STEPS; ++i) std::printf("%s%.1f", i ? ", " : "", ts[i + 1] - ts[i]);
    std::printf("]");
    CK(hipMemsetAsync(cm, 0, (size_t)C * C * 8, 0));
    CK(hipDeviceSynchronize());
  }
  // steady device time per launch: 200 back-to-back launches between two events
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int i = 0; i < 20; ++i) launch(i % K);
  CK(hipEventRecord(e0, 0));
  for (int i = 0; i < 200; ++i) launch(i % K);
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, e0, e1));
  std::printf(", \"steady_us_per_launch\": %.3f", ms * 1000.f / 200.f);
  std::printf("}\n");
  return 0;
}
