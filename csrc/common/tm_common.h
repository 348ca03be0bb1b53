// Shared device helpers for the torchmetrics_amd HIP kernels (gfx950 / CDNA4, wave64).
//
// Conventions used by every kernel in csrc/:
//   * wave = 64 lanes; blocks are multiples of 64 threads; lane = threadIdx.x & 63.
//   * validation failures are OR-ed into a per-metric int32 flag word (bits in validation.h); the host reads it
//     lazily at compute() instead of synchronising on every update.
//   * integer state accumulation uses 64-bit global atomics (order independent -> deterministic results).
#pragma once

#include <ATen/ATen.h>
#include <ATen/hip/HIPContext.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <c10/util/BFloat16.h>
#include <c10/util/Half.h>
#include <hip/hip_runtime.h>
#include <torch/library.h>

#include <cstdint>

namespace tm_amd {

constexpr int kWave = 64;

// native 16-byte vector (usable with __builtin_nontemporal_load, unlike HIP's uint4 class)
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// --------------------------------------------------------------------------------------------- validation bits
// keep in sync with torchmetrics_amd/utils/validation.py
constexpr int kErrTargetOutOfRange = 1 << 0;
constexpr int kErrPredsOutOfRange = 1 << 1;
constexpr int kErrTargetNotBinary = 1 << 2;
constexpr int kErrPredsNotBinary = 1 << 3;
constexpr int kErrPredsNan = 1 << 4;
constexpr int kErrValueNan = 1 << 5;
constexpr int kErrNegValue = 1 << 6;
constexpr int kErrValueNanWarn = 1 << 7;  // not an error: compute() emits the 'warn' nan_strategy UserWarning
constexpr int kErrOneshot = 1 << 8;        // a one-shot all-reduce of this metric's states failed (comm/oneshot)

// ------------------------------------------------------------------------------------------------ type helpers
template <typename T>
__device__ __forceinline__ float to_f32(T v) {
  return static_cast<float>(v);
}
template <>
__device__ __forceinline__ float to_f32<c10::BFloat16>(c10::BFloat16 v) {
  return __uint_as_float(static_cast<uint32_t>(v.x) << 16);
}
template <>
__device__ __forceinline__ float to_f32<c10::Half>(c10::Half v) {
  return __half2float(*reinterpret_cast<const __half*>(&v));
}

// round an fp32 value to storage type T and back (emulates ATen computing in fp32 and storing in T)
template <typename T>
__device__ __forceinline__ float round_to(float v) {
  return v;
}
template <>
__device__ __forceinline__ float round_to<c10::BFloat16>(float v) {
  // round-to-nearest-even, NaN preserved (same as c10::BFloat16 conversion)
  uint32_t u = __float_as_uint(v);
  if ((u & 0x7fffffffu) > 0x7f800000u) return v;
  uint32_t lsb = (u >> 16) & 1u;
  u += 0x7fffu + lsb;
  return __uint_as_float(u & 0xffff0000u);
}
template <>
__device__ __forceinline__ float round_to<c10::Half>(float v) {
  return __half2float(__float2half(v));
}
template <>
__device__ __forceinline__ float round_to<double>(float v) {
  return v;
}

template <typename T>
struct IsFloating {
  static constexpr bool value = false;
};
template <>
struct IsFloating<float> {
  static constexpr bool value = true;
};
template <>
struct IsFloating<double> {
  static constexpr bool value = true;
};
template <>
struct IsFloating<c10::Half> {
  static constexpr bool value = true;
};
template <>
struct IsFloating<c10::BFloat16> {
  static constexpr bool value = true;
};

// ------------------------------------------------------------------------------------------ wave reductions
// Whole-wave sums through the device library's wave reductions (DPP row shifts + readlane, inactive lanes count as
// zero, the result is wave-uniform): VALU work.  A __shfl_xor tree is six dependent ds_bpermutes (twice for 64-bit
// values) through the LDS pipe -- ~100 cycles each in a latency-bound tail and ~8 clk of LDS issue per wave.
extern "C" __device__ __attribute__((const)) float __ockl_wfred_add_f32(float);
extern "C" __device__ __attribute__((const)) double __ockl_wfred_add_f64(double);
extern "C" __device__ __attribute__((const)) int __ockl_wfred_add_i32(int);
extern "C" __device__ __attribute__((const)) unsigned int __ockl_wfred_add_u32(unsigned int);
extern "C" __device__ __attribute__((const)) long long __ockl_wfred_add_i64(long long);
extern "C" __device__ __attribute__((const)) unsigned long long __ockl_wfred_add_u64(unsigned long long);

__device__ __forceinline__ float wave_sum_impl(float v) { return __ockl_wfred_add_f32(v); }
__device__ __forceinline__ double wave_sum_impl(double v) { return __ockl_wfred_add_f64(v); }
__device__ __forceinline__ int wave_sum_impl(int v) { return __ockl_wfred_add_i32(v); }
__device__ __forceinline__ unsigned int wave_sum_impl(unsigned int v) { return __ockl_wfred_add_u32(v); }
__device__ __forceinline__ long long wave_sum_impl(long long v) { return __ockl_wfred_add_i64(v); }
__device__ __forceinline__ long wave_sum_impl(long v) { return __ockl_wfred_add_i64(v); }
__device__ __forceinline__ unsigned long long wave_sum_impl(unsigned long long v) { return __ockl_wfred_add_u64(v); }

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
  return wave_sum_impl(v);
}

__device__ __forceinline__ long long wave_sum_ll(long long v) { return __ockl_wfred_add_i64(v); }

// ---------------------------------------------------------------------- VALU-only f64 column sums in a wave
// v[s] summed over the lanes of this wave that share (lane mod k), k a power of two dividing 64 (k = 1: the whole
// wave): row_ror DPP moves for offsets 1..8, the gfx950 permlane16 / permlane32 swaps for 16 / 32 -- no LDS.  Every
// lane ends with its residue class's sum (so lane c < k holds column c).  ds_bpermute shuffles cost the LDS pipe
// ~8 clk each: 19 sums x 6 offsets x 2 halves x 8 waves of them were ~6 us of a 512-thread moments launch.
template <typename T>
__device__ __forceinline__ long long bits64(T x) {
  static_assert(sizeof(T) == 8, "64-bit values");
  return __builtin_bit_cast(long long, x);
}

template <int CTRL, typename T>
__device__ __forceinline__ T dpp64(T x) {
  const long long b = bits64(x);
  const int lo = __builtin_amdgcn_update_dpp(0, static_cast<int>(b), CTRL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, static_cast<int>(b >> 32), CTRL, 0xf, 0xf, false);
  return __builtin_bit_cast(T, (static_cast<long long>(hi) << 32) | static_cast<unsigned>(lo));
}

template <typename T>
__device__ __forceinline__ T join64(unsigned lo, unsigned hi) {
  return __builtin_bit_cast(T, static_cast<long long>((static_cast<unsigned long long>(hi) << 32) | lo));
}

// x[lane] + x[lane ^ 16] (the same sum, in the same order, in both lanes)
template <typename T>
__device__ __forceinline__ T xor16_sum64(T x) {
  const long long b = bits64(x);
  const unsigned lo = static_cast<unsigned>(b), hi = static_cast<unsigned>(b >> 32);
  const auto l = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);  // [0]: even rows' values, [1]: odd rows'
  const auto h = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  return join64<T>(l[0], h[0]) + join64<T>(l[1], h[1]);
}

// x[lane] + x[lane ^ 32]
template <typename T>
__device__ __forceinline__ T xor32_sum64(T x) {
  const long long b = bits64(x);
  const unsigned lo = static_cast<unsigned>(b), hi = static_cast<unsigned>(b >> 32);
  const auto l = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);  // [0]: lanes 0-31's values, [1]: 32-63's
  const auto h = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
  return join64<T>(l[0], h[0]) + join64<T>(l[1], h[1]);
}

// T = double or long long; call with every lane of the wave active
template <typename T, int NS>
__device__ __forceinline__ void wave_colsum64(T (&v)[NS], int k) {
  // offsets below k would mix columns; the branches are uniform (and fold away for a constant k)
  if (k <= 1) {
#pragma unroll
    for (int s = 0; s < NS; ++s) v[s] += dpp64<0x121>(v[s]);  // row_ror:1
  }
  if (k <= 2) {
#pragma unroll
    for (int s = 0; s < NS; ++s) v[s] += dpp64<0x122>(v[s]);  // row_ror:2
  }
  if (k <= 4) {
#pragma unroll
    for (int s = 0; s < NS; ++s) v[s] += dpp64<0x124>(v[s]);  // row_ror:4
  }
  if (k <= 8) {
#pragma unroll
    for (int s = 0; s < NS; ++s) v[s] += dpp64<0x128>(v[s]);  // row_ror:8
  }
  if (k <= 16) {
#pragma unroll
    for (int s = 0; s < NS; ++s) v[s] = xor16_sum64(v[s]);
  }
  if (k <= 32) {
#pragma unroll
    for (int s = 0; s < NS; ++s) v[s] = xor32_sum64(v[s]);
  }
}

template <int NS>
__device__ __forceinline__ void wave_colsum_f64(double (&v)[NS], int k) {
  wave_colsum64(v, k);
}

// the same over the sums whose bit is set in `use` only (a wave-uniform mask: unused sums skip their 6 exchange steps)
template <int NS>
__device__ __forceinline__ void wave_colsum_f64_masked(double (&v)[NS], int k, int use) {
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    if (!((use >> s) & 1)) continue;
    double one[1] = {v[s]};
    wave_colsum64(one, k);
    v[s] = one[0];
  }
}

// argmax combine with torch.argmax semantics: NaN wins, then larger value, then smaller index
__device__ __forceinline__ bool argmax_better(float va, int ia, float vb, int ib) {
  const bool na = va != va, nb = vb != vb;
  if (na != nb) return na;
  if (na && nb) return ia < ib;
  if (va != vb) return va > vb;
  return ia < ib;
}

__device__ __forceinline__ void wave_argmax(float& v, int& i) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const float ov = __shfl_xor(v, off, kWave);
    const int oi = __shfl_xor(i, off, kWave);
    if (argmax_better(ov, oi, v, i)) {
      v = ov;
      i = oi;
    }
  }
}

__device__ __forceinline__ void atomic_add_i64(int64_t* p, long long v) {
  atomicAdd(reinterpret_cast<unsigned long long*>(p), static_cast<unsigned long long>(v));
}

__device__ __forceinline__ void raise_flag(int* flag, int bit) { atomicOr(flag, bit); }

inline int grid_cap(long long blocks, int cap = 256 * 16) {
  return static_cast<int>(blocks < cap ? (blocks < 1 ? 1 : blocks) : cap);
}

inline hipStream_t stream() { return at::hip::getCurrentHIPStream().stream(); }

// True while `s` is being captured into a hipGraph.  The double-buffered "scores are not probabilities" words pick
// their slot from a host-side update parity, which a captured graph would freeze at the capture-time value (one slot
// read and never re-armed on replay): under capture the launchers use slot 0 and re-arm it inside the captured work.
inline bool stream_capturing(hipStream_t s) {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  return hipStreamIsCapturing(s, &st) == hipSuccess && st == hipStreamCaptureStatusActive;
}

// which word of a binary / multilabel "not probabilities" pair a reader uses, and whether the pair is double-buffered
// (stat_scores.hip notprob_view)
struct NpView {
  int slot;
  bool two;
};

// zero n (<= 64) int words: the captured-mode re-arm of a decision word buffer (one copy per translation unit)
namespace {
__global__ void zero_words_kernel(int* __restrict__ p, int n) {
  if (static_cast<int>(threadIdx.x) < n) p[threadIdx.x] = 0;
}
}  // namespace
inline void launch_zero_words(int* p, int n, hipStream_t s) {
  hipLaunchKernelGGL(zero_words_kernel, dim3(1), dim3(64), 0, s, p, n);
}

// kStreamTickets zeroed uint32 words per (device, stream), kept for the process (csrc/regression/moments.hip): the
// last-block hand-offs count finished blocks in them and every kernel re-arms (zeroes) the words it used before it
// ends, so consecutive launches on a stream -- which never overlap -- share them.  Word 0: the moments kernels;
// words 1..127: the few-class tile kernel's hand-off groups (stat_scores.hip).
constexpr int kStreamTickets = 128;
unsigned int* stream_ticket(int device, hipStream_t s);

// CU count of a device, queried once per device (hipDeviceGetAttribute costs host time on every call).
inline int cu_count(int device) {
  static int cache[64] = {0};
  if (device < 0 || device >= 64) device = 0;
  int v = cache[device];
  if (v == 0) {
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || v <= 0) v = 256;
    cache[device] = v;
  }
  return v;
}

// Every launcher starts with TM_CHECK_CUDA(<first tensor>): it checks the tensor is on a ROCm device and makes that
// device current for the rest of the launcher (kernels, stream() and allocations then all target the tensor's device,
// whatever device the calling thread had selected).  TM_SAME_DEVICE checks the remaining tensor arguments.
#define TM_CONCAT_(a, b) a##b
#define TM_CONCAT(a, b) TM_CONCAT_(a, b)
#define TM_CHECK_CUDA(x)                                                  \
  TORCH_CHECK((x).is_cuda(), #x " must be a ROCm (cuda) tensor");          \
  const c10::hip::HIPGuardMasqueradingAsCUDA TM_CONCAT(tm_device_guard_, __LINE__)((x).device())
#define TM_SAME_DEVICE(a, b) \
  TORCH_CHECK((a).device() == (b).device(), #b " is on ", (b).device(), " but " #a " is on ", (a).device())
#define TM_CHECK_CONTIG(x) TORCH_CHECK((x).is_contiguous(), #x " must be contiguous")

// Dispatch over the element types a metric input can have (floating: f32/f16/bf16/f64; integral: i64/i32/u8/bool)
#define TM_DISPATCH_PREDS(dtype, NAME, ...)                                     \
  [&] {                                                                          \
    switch (dtype) {                                                             \
      case at::kFloat: { using scalar_t = float; return __VA_ARGS__(); }         \
      case at::kHalf: { using scalar_t = c10::Half; return __VA_ARGS__(); }      \
      case at::kBFloat16: { using scalar_t = c10::BFloat16; return __VA_ARGS__(); } \
      case at::kDouble: { using scalar_t = double; return __VA_ARGS__(); }       \
      case at::kLong: { using scalar_t = int64_t; return __VA_ARGS__(); }        \
      case at::kInt: { using scalar_t = int32_t; return __VA_ARGS__(); }         \
      case at::kByte: { using scalar_t = uint8_t; return __VA_ARGS__(); }        \
      case at::kBool: { using scalar_t = uint8_t; return __VA_ARGS__(); }        \
      default: TORCH_CHECK(false, NAME ": unsupported preds dtype ", dtype);     \
    }                                                                            \
  }()

#define TM_DISPATCH_TARGET(dtype, NAME, ...)                                    \
  [&] {                                                                          \
    switch (dtype) {                                                             \
      case at::kLong: { using target_t = int64_t; return __VA_ARGS__(); }        \
      case at::kInt: { using target_t = int32_t; return __VA_ARGS__(); }         \
      case at::kByte: { using target_t = uint8_t; return __VA_ARGS__(); }        \
      case at::kBool: { using target_t = uint8_t; return __VA_ARGS__(); }        \
      default: TORCH_CHECK(false, NAME ": unsupported target dtype ", dtype);    \
    }                                                                            \
  }()

#define TM_DISPATCH_FLOAT(dtype, NAME, ...)                                     \
  [&] {                                                                          \
    switch (dtype) {                                                             \
      case at::kFloat: { using scalar_t = float; return __VA_ARGS__(); }         \
      case at::kHalf: { using scalar_t = c10::Half; return __VA_ARGS__(); }      \
      case at::kBFloat16: { using scalar_t = c10::BFloat16; return __VA_ARGS__(); } \
      case at::kDouble: { using scalar_t = double; return __VA_ARGS__(); }       \
      default: TORCH_CHECK(false, NAME ": unsupported float dtype ", dtype);     \
    }                                                                            \
  }()

}  // namespace tm_amd
