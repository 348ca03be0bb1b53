// Shared pieces of the sort / scan kernel family (csrc/sort/*.hip).
//
// * order-preserving radix keys: ascending key order == DESCENDING score order, NaN first (torch.sort(descending)
//   puts NaN first), -0.0 == +0.0 (so they form one tie run, as ``preds[1:] != preds[:-1]`` sees them);
// * rocPRIM radix sort entry points whose temporary storage comes from the PyTorch caching allocator;
// * wave/block inclusive scans over any trivially-copyable struct with an associative combine (64-lane waves:
//   6 shuffle steps, then one LDS slot per wave).
#pragma once

#include <rocprim/device/device_radix_sort.hpp>

#include "common/tm_common.h"

namespace tm_amd {
namespace sortscan {

__device__ __forceinline__ uint32_t desc_key32(float f) {
  uint32_t u = __float_as_uint(f);
  if (f != f) u = 0x7fc00000u;
  else if (f == 0.0f) u = 0u;
  const uint32_t asc = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
  return ~asc;
}

__device__ __forceinline__ float desc_key32_decode(uint32_t k) {
  const uint32_t asc = ~k;
  const uint32_t u = (asc & 0x80000000u) ? (asc & 0x7fffffffu) : ~asc;
  return __uint_as_float(u);
}

__device__ __forceinline__ uint64_t desc_key64(double d) {
  uint64_t u = static_cast<uint64_t>(__double_as_longlong(d));
  if (d != d) u = 0x7ff8000000000000ULL;
  else if (d == 0.0) u = 0ULL;
  const uint64_t asc = (u & 0x8000000000000000ULL) ? ~u : (u | 0x8000000000000000ULL);
  return ~asc;
}

// n / d for 0 <= n, d < 2^31 with one mul-hi (no 64-bit division in the hot loops)
struct FastDiv {
  uint32_t d, m, sh;
  FastDiv() = default;
  explicit FastDiv(uint32_t div) : d(div) {
    sh = 0;
    while ((1ULL << sh) < div) ++sh;
    m = static_cast<uint32_t>(((1ULL << 32) * ((1ULL << sh) - div)) / div + 1);
  }
  __device__ __forceinline__ uint32_t div(uint32_t n) const { return (__umulhi(n, m) + n) >> sh; }
};

inline int ceil_log2(int64_t v) {
  int b = 0;
  while ((int64_t(1) << b) < v) ++b;
  return b;
}

// ------------------------------------------------------------------------------------------------ radix sorts
template <typename K, typename V>
void sort_pairs(const K* kin, K* kout, const V* vin, V* vout, int64_t n, int begin_bit, int end_bit,
                const at::Device& dev, hipStream_t s) {
  if (n <= 0) return;
  size_t bytes = 0;
  TORCH_CHECK(rocprim::radix_sort_pairs(nullptr, bytes, kin, kout, vin, vout, static_cast<unsigned int>(n),
                                        begin_bit, end_bit, s) == hipSuccess, "radix_sort_pairs: size query failed");
  auto tmp = at::empty({static_cast<int64_t>(bytes) + 16}, at::TensorOptions().dtype(at::kByte).device(dev));
  TORCH_CHECK(rocprim::radix_sort_pairs(tmp.data_ptr(), bytes, kin, kout, vin, vout, static_cast<unsigned int>(n),
                                        begin_bit, end_bit, s) == hipSuccess, "radix_sort_pairs failed");
}

template <typename K>
void sort_keys(const K* kin, K* kout, int64_t n, int begin_bit, int end_bit, const at::Device& dev, hipStream_t s) {
  if (n <= 0) return;
  size_t bytes = 0;
  TORCH_CHECK(rocprim::radix_sort_keys(nullptr, bytes, kin, kout, static_cast<unsigned int>(n), begin_bit, end_bit,
                                       s) == hipSuccess, "radix_sort_keys: size query failed");
  auto tmp = at::empty({static_cast<int64_t>(bytes) + 16}, at::TensorOptions().dtype(at::kByte).device(dev));
  TORCH_CHECK(rocprim::radix_sort_keys(tmp.data_ptr(), bytes, kin, kout, static_cast<unsigned int>(n), begin_bit,
                                       end_bit, s) == hipSuccess, "radix_sort_keys failed");
}

// ------------------------------------------------------------------------------------------------------ scans
template <typename T>
__device__ __forceinline__ T shfl_up_any(const T& v, int d) {
  static_assert(sizeof(T) % 4 == 0, "shfl_up_any: size must be a multiple of 4 bytes");
  constexpr int W = sizeof(T) / 4;
  T r;
  const int* src = reinterpret_cast<const int*>(&v);
  int* dst = reinterpret_cast<int*>(&r);
#pragma unroll
  for (int w = 0; w < W; ++w) dst[w] = __shfl_up(src[w], d, kWave);
  return r;
}

template <typename T, typename Op>
__device__ __forceinline__ T wave_inclusive_scan(T v, Op op) {
  const int lane = threadIdx.x & (kWave - 1);
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    const T o = shfl_up_any(v, d);
    if (lane >= d) v = op(o, v);
  }
  return v;
}

// Block-wide inclusive scan of one value per thread. ``lds`` holds NW = blockDim.x / 64 slots. Returns the
// inclusive value; ``excl`` gets the exclusive one (identity for thread 0) and ``total`` the block aggregate.
template <int NW, typename T, typename Op>
__device__ __forceinline__ T block_inclusive_scan(T v, Op op, const T& identity, T* lds, T& excl, T& total) {
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = threadIdx.x / kWave;
  T inc = wave_inclusive_scan(v, op);
  if (lane == kWave - 1) lds[wave] = inc;
  __syncthreads();
  T wave_prefix = identity;
  for (int w = 0; w < wave; ++w) wave_prefix = op(wave_prefix, lds[w]);
  total = identity;
#pragma unroll
  for (int w = 0; w < NW; ++w) total = op(total, lds[w]);
  T lane_excl = shfl_up_any(inc, 1);
  if (lane == 0) lane_excl = identity;
  excl = op(wave_prefix, lane_excl);
  inc = op(wave_prefix, inc);
  __syncthreads();  // lds may be reused by the caller
  return inc;
}

}  // namespace sortscan
}  // namespace tm_amd
