// Standalone microbenchmark for the headline confusion-matrix update (8192 x 1000 bf16 logits -> 1000x1000 int64).
// Variants of the per-row argmax + histogram kernel, timed with HIP events over back-to-back launches with the
// inputs cycling through 4 buffers (as bench.py does).  Build: hipcc -O3 --offload-arch=gfx950 confmat_mb.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e = (x);                                                         \
    if (e != hipSuccess) {                                                      \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);     \
      std::exit(1);                                                             \
    }                                                                           \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr int kWave = 64;

__device__ __forceinline__ bool better(float va, int ia, float vb, int ib) {
  const bool na = va != va, nb = vb != vb;
  if (na != nb) return na;
  if (na && nb) return ia < ib;
  if (va != vb) return va > vb;
  return ia < ib;
}

// orderable 32-bit key for a bf16 value at column idx: larger key = larger value, ties -> smaller index; NaN max.
__device__ __forceinline__ uint32_t bf16_key(uint32_t h, uint32_t idx) {
  uint32_t ord = (h & 0x8000u) ? (~h & 0xffffu) : (h | 0x8000u);
  const bool nan = (h & 0x7fffu) > 0x7f80u;
  ord = nan ? 0xffffu : ord;
  return (ord << 16) | (0xffffu - idx);
}

// V0: current production design (one row per wave, next row prefetched, float compare, shfl reduce)
template <int kPer>
__global__ void __launch_bounds__(256) v0(const uint16_t* __restrict__ preds, const int64_t* __restrict__ target,
                                          int N, int C, unsigned long long* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int nwaves = gridDim.x * 4;
  const int wave = (blockIdx.x * 256 + threadIdx.x) / 64;
  const int nchunks = C / 8;
  for (int row = wave; row < N; row += nwaves) {
    const u32x4* rp = reinterpret_cast<const u32x4*>(preds + (long long)row * C);
    u32x4 buf[kPer];
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const int ci = lane + j * 64;
      if (ci < nchunks) buf[j] = __builtin_nontemporal_load(rp + ci);
    }
    float best = -INFINITY;
    int bidx = 0x7fffffff;
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const int ci = lane + j * 64;
      if (ci < nchunks) {
        const uint16_t* e = reinterpret_cast<const uint16_t*>(&buf[j]);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float v = __uint_as_float((uint32_t)e[k] << 16);
          if (better(v, ci * 8 + k, best, bidx)) {
            best = v;
            bidx = ci * 8 + k;
          }
        }
      }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const float ov = __shfl_xor(best, off, 64);
      const int oi = __shfl_xor(bidx, off, 64);
      if (better(ov, oi, best, bidx)) {
        best = ov;
        bidx = oi;
      }
    }
    if (lane == 0) atomicAdd(out + target[row] * C + bidx, 1ull);
  }
}

// V1: packed-key argmax (one u32 max per element, DPP-friendly reduce)
template <int kPer, bool kAtomic>
__global__ void __launch_bounds__(256) v1(const uint16_t* __restrict__ preds, const int64_t* __restrict__ target,
                                          int N, int C, unsigned long long* __restrict__ out, int* __restrict__ lab) {
  const int lane = threadIdx.x & 63;
  const int nwaves = gridDim.x * (blockDim.x / 64);
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) / 64;
  const int nchunks = C / 8;
  for (int row = wave; row < N; row += nwaves) {
    const u32x4* rp = reinterpret_cast<const u32x4*>(preds + (long long)row * C);
    u32x4 buf[kPer];
    long long t = 0;
    if (kAtomic && lane == 0) t = target[row];
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const int ci = lane + j * 64;
      if (ci < nchunks) buf[j] = __builtin_nontemporal_load(rp + ci);
    }
    uint32_t key = 0;
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const int ci = lane + j * 64;
      if (ci < nchunks) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const uint32_t w = buf[j][k];
          const uint32_t i0 = ci * 8 + 2 * k;
          const uint32_t k0 = bf16_key(w & 0xffffu, i0), k1 = bf16_key(w >> 16, i0 + 1);
          key = max(key, max(k0, k1));
        }
      }
    }
    key = __reduce_max_sync(~0ull, (int)(key ^ 0x80000000u)) ^ 0x80000000u;
    const int bidx = 0xffff - (int)(key & 0xffffu);
    if (lane == 0) {
      if (kAtomic) atomicAdd(out + t * C + bidx, 1ull);
      else lab[row] = bidx;
    }
  }
}

// V2: pure streaming read floor (xor of all words, written once per row)
template <int kPer>
__global__ void __launch_bounds__(256) vread(const uint16_t* __restrict__ preds, int N, int C, int* __restrict__ lab) {
  const int lane = threadIdx.x & 63;
  const int nwaves = gridDim.x * (blockDim.x / 64);
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) / 64;
  const int nchunks = C / 8;
  for (int row = wave; row < N; row += nwaves) {
    const u32x4* rp = reinterpret_cast<const u32x4*>(preds + (long long)row * C);
    uint32_t x = 0;
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const int ci = lane + j * 64;
      if (ci < nchunks) {
        u32x4 v = __builtin_nontemporal_load(rp + ci);
        x ^= v[0] ^ v[1] ^ v[2] ^ v[3];
      }
    }
    if (x == 0x12345678u) lab[row] = x;
  }
}

// V3: row-block layout -- a workgroup of 256 threads takes 4 consecutive rows, each lane loads 16B chunks spread
// over the 4 rows' contiguous 8000 B (fully coalesced 1 KiB per wave-instruction), argmax via LDS.
__global__ void __launch_bounds__(256) v3(const uint16_t* __restrict__ preds, const int64_t* __restrict__ target,
                                          int N, int C, unsigned long long* __restrict__ out) {
  // assumes C == 1000 -> 125 chunks per row, 500 chunks per 4 rows; 256 threads x 2 chunks = 512 >= 500
  __shared__ uint32_t red[4][4];
  const int tid = threadIdx.x;
  const int row0 = blockIdx.x * 4;
  const u32x4* base = reinterpret_cast<const u32x4*>(preds + (long long)row0 * C);
  const int nch = 125;
  uint32_t key[2] = {0, 0};
  int r[2];
  u32x4 buf[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int c = tid + j * 256;
    r[j] = c / nch;
    if (c < 4 * nch && row0 + r[j] < N) buf[j] = __builtin_nontemporal_load(base + c);
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int c = tid + j * 256;
    if (c < 4 * nch && row0 + r[j] < N) {
      const int ci = c - r[j] * nch;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t w = buf[j][k];
        const uint32_t i0 = ci * 8 + 2 * k;
        key[j] = max(key[j], max(bf16_key(w & 0xffffu, i0), bf16_key(w >> 16, i0 + 1)));
      }
    }
  }
  // per-wave: each lane's chunks may belong to 2 rows; reduce per row with masked max
  const int wave = tid / 64;
  for (int rr = 0; rr < 4; ++rr) {
    uint32_t k = 0;
#pragma unroll
    for (int j = 0; j < 2; ++j) k = max(k, r[j] == rr ? key[j] : 0u);
    k = __reduce_max_sync(~0ull, (int)(k ^ 0x80000000u)) ^ 0x80000000u;
    if ((tid & 63) == 0) red[wave][rr] = k;
  }
  __syncthreads();
  if (tid < 4 && row0 + tid < N) {
    uint32_t k = max(max(red[0][tid], red[1][tid]), max(red[2][tid], red[3][tid]));
    const int bidx = 0xffff - (int)(k & 0xffffu);
    atomicAdd(out + target[row0 + tid] * C + bidx, 1ull);
  }
}


typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
typedef short s16x2 __attribute__((ext_vector_type(2)));

// V4: two-step argmax on packed 16-bit ordinals: per word (2 bf16) ord = w ^ ((w >>a 15) | 0x8000) with packed
// 16-bit ops, lane max/min with v_pk_max_u16/v_pk_min_u16, then a reverse scan for the lane's first index of its max
// and ONE wave max over (ord << 16 | 0xffff - idx).  NaN rows (max ordinal > +inf or min ordinal < -inf) fall back
// to the float compare.  R rows per wave in flight.
template <int R, bool kAtomic>
__global__ void __launch_bounds__(256) v4(const uint16_t* __restrict__ preds, const int64_t* __restrict__ target,
                                          int N, int C, unsigned long long* __restrict__ out, int* __restrict__ lab) {
  constexpr int kPer = 2;
  const int lane = threadIdx.x & 63;
  const int nwaves = gridDim.x * (blockDim.x / 64);
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) / 64;
  const int nchunks = C / 8;
  for (int row0 = wave; row0 < N; row0 += nwaves * R) {
    u32x4 buf[R][kPer];
    long long t[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int row = row0 + r * nwaves;
      t[r] = 0;
      if (row < N) {
        if (kAtomic && lane == 0) t[r] = target[row];
        const u32x4* rp = reinterpret_cast<const u32x4*>(preds + (long long)row * C);
#pragma unroll
        for (int j = 0; j < kPer; ++j) {
          const int ci = lane + j * 64;
          if (ci < nchunks) buf[r][j] = __builtin_nontemporal_load(rp + ci);
        }
      }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int row = row0 + r * nwaves;
      if (row >= N) break;  // wave-uniform
      u16x2 mx = {0, 0}, mn = {0xffff, 0xffff};
      uint32_t ordw[kPer][4];
#pragma unroll
      for (int j = 0; j < kPer; ++j) {
        const int ci = lane + j * 64;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const uint32_t w = buf[r][j][k];
          const s16x2 sw = __builtin_bit_cast(s16x2, w);
          const uint32_t sgn = __builtin_bit_cast(uint32_t, (s16x2)(sw >> (s16x2){15, 15}));
          const uint32_t o = w ^ (sgn | 0x80008000u);
          ordw[j][k] = o;
          if (ci < nchunks) {
            const u16x2 ov = __builtin_bit_cast(u16x2, o);
            mx = __builtin_elementwise_max(mx, ov);
            mn = __builtin_elementwise_min(mn, ov);
          }
        }
      }
      const uint32_t lmax = max(mx.x, mx.y), lmin = min(mn.x, mn.y);
      // lane's first index holding lmax (reverse scan: last hit wins)
      uint32_t first = 0xffffu;
#pragma unroll
      for (int j = kPer - 1; j >= 0; --j) {
        const int ci = lane + j * 64;
        if (ci < nchunks) {
#pragma unroll
          for (int k = 3; k >= 0; --k) {
            const uint32_t o = ordw[j][k];
            if ((o >> 16) == lmax) first = ci * 8 + 2 * k + 1;
            if ((o & 0xffffu) == lmax) first = ci * 8 + 2 * k;
          }
        }
      }
      uint32_t key = (lmax << 16) | (0xffffu - first);
      key = __reduce_max_sync(~0ull, (int)(key ^ 0x80000000u)) ^ 0x80000000u;
      const bool nan_row = (key >> 16) > 0xff80u || __any(lmin < 0x007fu);
      int bidx = 0xffff - (int)(key & 0xffffu);
      if (nan_row) {  // rare: exact torch.argmax semantics with the float compare
        float best = -INFINITY;
        int bi = 0x7fffffff;
#pragma unroll
        for (int j = 0; j < kPer; ++j) {
          const int ci = lane + j * 64;
          if (ci < nchunks) {
            const uint16_t* e = reinterpret_cast<const uint16_t*>(&buf[r][j]);
#pragma unroll
            for (int k = 0; k < 8; ++k) {
              const float v = __uint_as_float((uint32_t)e[k] << 16);
              if (better(v, ci * 8 + k, best, bi)) {
                best = v;
                bi = ci * 8 + k;
              }
            }
          }
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
          const float ov = __shfl_xor(best, off, 64);
          const int oi = __shfl_xor(bi, off, 64);
          if (better(ov, oi, best, bi)) {
            best = ov;
            bi = oi;
          }
        }
        bidx = bi;
      }
      if (lane == 0) {
        if (kAtomic) atomicAdd(out + t[r] * C + bidx, 1ull);
        else lab[row] = bidx;
      }
    }
  }
}

int main(int argc, char** argv) {
  const int N = 8192, C = 1000, NB = 4;
  int cus = 256;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  std::vector<uint16_t> h(static_cast<size_t>(N) * C);
  std::vector<int64_t> ht(N);
  uint32_t s = 12345;
  auto rnd = [&] { s = s * 1664525u + 1013904223u; return s; };
  uint16_t *dp[NB];
  int64_t* dt[NB];
  for (int b = 0; b < NB; ++b) {
    for (auto& x : h) {
      float f = ((rnd() >> 8) / 16777216.0f - 0.5f) * 6.f;
      uint32_t u;
      std::memcpy(&u, &f, 4);
      x = (uint16_t)(u >> 16);
    }
    for (auto& t : ht) t = rnd() % C;
    CK(hipMalloc(&dp[b], h.size() * 2));
    CK(hipMalloc(&dt[b], N * 8));
    CK(hipMemcpy(dp[b], h.data(), h.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(dt[b], ht.data(), N * 8, hipMemcpyHostToDevice));
  }
  unsigned long long *o0, *o1;
  int* lab;
  CK(hipMalloc(&o0, (size_t)C * C * 8));
  CK(hipMalloc(&o1, (size_t)C * C * 8));
  CK(hipMalloc(&lab, N * 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int reps = 400;
  auto timeit = [&](const char* name, auto launch) {
    for (int i = 0; i < 20; ++i) launch(i % NB);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) launch(i % NB);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::printf("{\"variant\": \"%s\", \"us\": %.2f, \"GBps\": %.0f}\n", name, ms * 1e3 / reps,
                (double)N * C * 2 / (ms * 1e-3 / reps) / 1e9);
  };
  // correctness: v0 vs v1 vs v3 on one batch
  CK(hipMemset(o0, 0, (size_t)C * C * 8));
  CK(hipMemset(o1, 0, (size_t)C * C * 8));
  hipLaunchKernelGGL((v0<2>), dim3(cus * 8), dim3(256), 0, 0, dp[0], dt[0], N, C, o0);
  hipLaunchKernelGGL((v1<2, true>), dim3(cus * 8), dim3(256), 0, 0, dp[0], dt[0], N, C, o1, lab);
  CK(hipDeviceSynchronize());
  std::vector<unsigned long long> a((size_t)C * C), b((size_t)C * C);
  CK(hipMemcpy(a.data(), o0, a.size() * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(b.data(), o1, b.size() * 8, hipMemcpyDeviceToHost));
  std::printf("{\"check_v1\": %s}\n", a == b ? "true" : "false");
  CK(hipMemset(o1, 0, (size_t)C * C * 8));
  hipLaunchKernelGGL(v3, dim3(N / 4), dim3(256), 0, 0, dp[0], dt[0], N, C, o1);
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(b.data(), o1, b.size() * 8, hipMemcpyDeviceToHost));
  std::printf("{\"check_v3\": %s}\n", a == b ? "true" : "false");
  for (int R : {1, 2}) {
    CK(hipMemset(o1, 0, (size_t)C * C * 8));
    if (R == 1) hipLaunchKernelGGL((v4<1, true>), dim3(cus * 8), dim3(256), 0, 0, dp[0], dt[0], N, C, o1, lab);
    else hipLaunchKernelGGL((v4<2, true>), dim3(cus * 4), dim3(256), 0, 0, dp[0], dt[0], N, C, o1, lab);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(b.data(), o1, b.size() * 8, hipMemcpyDeviceToHost));
    std::printf("{\"check_v4_R%d\": %s}\n", R, a == b ? "true" : "false");
  }
  // NaN rows: plant +NaN / -NaN / ties into buffer 1 and compare v0 vs v4
  {
    std::vector<uint16_t> hh((size_t)N * C);
    CK(hipMemcpy(hh.data(), dp[1], hh.size() * 2, hipMemcpyDeviceToHost));
    for (int r = 0; r < 64; ++r) {
      hh[(size_t)r * C + (r * 37) % C] = (r & 1) ? 0x7fc1 : 0xffc1;
      hh[(size_t)r * C + (r * 11) % C] = (r & 2) ? 0x7fc3 : 0xffc0;
    }
    for (int r = 64; r < 128; ++r) { hh[(size_t)r * C + 3] = 0x7f80; hh[(size_t)r * C + 900] = 0x7f80; }
    for (int r = 128; r < 160; ++r) for (int c = 0; c < C; ++c) hh[(size_t)r * C + c] = 0x3f80;
    CK(hipMemcpy(dp[1], hh.data(), hh.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemset(o0, 0, (size_t)C * C * 8));
    CK(hipMemset(o1, 0, (size_t)C * C * 8));
    hipLaunchKernelGGL((v0<2>), dim3(cus * 8), dim3(256), 0, 0, dp[1], dt[1], N, C, o0);
    hipLaunchKernelGGL((v4<1, true>), dim3(cus * 8), dim3(256), 0, 0, dp[1], dt[1], N, C, o1, lab);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(a.data(), o0, a.size() * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), o1, b.size() * 8, hipMemcpyDeviceToHost));
    std::printf("{\"check_v4_nan_ties\": %s}\n", a == b ? "true" : "false");
  }

  for (int bpc : {4, 8}) {
    char nm[64];
    std::snprintf(nm, 64, "v0 pipe %d/CU", bpc);
    timeit(nm, [&](int i) { hipLaunchKernelGGL((v0<2>), dim3(cus * bpc), dim3(256), 0, 0, dp[i], dt[i], N, C, o0); });
    std::snprintf(nm, 64, "v1 key atomics %d/CU", bpc);
    timeit(nm, [&](int i) { hipLaunchKernelGGL((v1<2, true>), dim3(cus * bpc), dim3(256), 0, 0, dp[i], dt[i], N, C, o0, lab); });
    std::snprintf(nm, 64, "v1 key noatomic %d/CU", bpc);
    timeit(nm, [&](int i) { hipLaunchKernelGGL((v1<2, false>), dim3(cus * bpc), dim3(256), 0, 0, dp[i], dt[i], N, C, o0, lab); });
    std::snprintf(nm, 64, "read floor %d/CU", bpc);
    timeit(nm, [&](int i) { hipLaunchKernelGGL((vread<2>), dim3(cus * bpc), dim3(256), 0, 0, dp[i], N, C, lab); });
  }
  timeit("v4 R1 8/CU", [&](int i) { hipLaunchKernelGGL((v4<1, true>), dim3(cus * 8), dim3(256), 0, 0, dp[i], dt[i], N, C, o0, lab); });
  timeit("v4 R2 4/CU", [&](int i) { hipLaunchKernelGGL((v4<2, true>), dim3(cus * 4), dim3(256), 0, 0, dp[i], dt[i], N, C, o0, lab); });
  timeit("v4 R1 noatomic 8/CU", [&](int i) { hipLaunchKernelGGL((v4<1, false>), dim3(cus * 8), dim3(256), 0, 0, dp[i], dt[i], N, C, o0, lab); });
  timeit("v4 R1 4/CU", [&](int i) { hipLaunchKernelGGL((v4<1, true>), dim3(cus * 4), dim3(256), 0, 0, dp[i], dt[i], N, C, o0, lab); });
  timeit("v4 R2 2/CU", [&](int i) { hipLaunchKernelGGL((v4<2, true>), dim3(cus * 2), dim3(256), 0, 0, dp[i], dt[i], N, C, o0, lab); });
      timeit("v3 rowblock", [&](int i) { hipLaunchKernelGGL(v3, dim3(N / 4), dim3(256), 0, 0, dp[i], dt[i], N, C, o0); });
  timeit("empty-ish launch", [&](int i) { hipLaunchKernelGGL((vread<2>), dim3(1), dim3(64), 0, 0, dp[i], 1, C, lab); });
  return 0;
}
