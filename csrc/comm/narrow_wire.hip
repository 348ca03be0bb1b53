// Optimistic narrow wire for integer SUM buckets (parallel/sync.py ``_narrow_bucket``).
//
// Count states (a 1000-class confusion matrix: 8 MB of int64 whose cells are small) cross xGMI far narrower than
// their dtype: a ring all-reduce is per-link bandwidth-bound, so an int64 bucket sent as uint8 moves 1/8 of the
// bytes.  The width must be agreed by every rank before the collective.  Instead of a range all-reduce (one extra
// collective + a host read per bucket), every rank encodes at the width the previous syncs settled on and appends two
// check slots: each rank sets "too big" when one of its values exceeds (wire max) / world (then no partial sum of
// the ring can leave the exact range) and "negative" on a negative value.  The slots are summed by the same
// all-reduce, so every rank sees the same verdict; the decode folds it into the metric's validation word, which
// compute() reads anyway, and only a rare overflow costs a wider re-send.
//
//   narrow_encode(src int64 | int32 [n], code, world) -> wire [n + 2] of uint8 (code 0) / fp16 (1) / int32 (2)
//   narrow_decode(wire, n, out_dtype, word?, bit)     -> [n] out_dtype; word |= bit when a check slot is non-zero
#include <hip/hip_fp16.h>

#include "../common/tm_common.h"

namespace tm_amd {
namespace {

constexpr int kThreads = 256;
constexpr int kPer = 4;  // elements per thread and step

template <typename W>
struct Wire;
template <>
struct Wire<uint8_t> {
  static constexpr long long kMax = 255;
  __device__ static uint8_t enc(long long v) { return static_cast<uint8_t>(v); }
  __device__ static long long dec(uint8_t w) { return w; }
  __device__ static uint8_t one() { return 1; }
  __device__ static bool nonzero(uint8_t w) { return w != 0; }
};
template <>
struct Wire<__half> {
  static constexpr long long kMax = 2048;  // every integer <= 2^11 is exact in fp16
  __device__ static __half enc(long long v) { return __float2half_rn(static_cast<float>(v)); }
  __device__ static long long dec(__half w) { return static_cast<long long>(__half2float(w)); }
  __device__ static __half one() { return __float2half_rn(1.0f); }
  __device__ static bool nonzero(__half w) { return __half2float(w) != 0.0f; }
};
template <>
struct Wire<int32_t> {
  static constexpr long long kMax = 2147483647LL;
  __device__ static int32_t enc(long long v) { return static_cast<int32_t>(v); }
  __device__ static long long dec(int32_t w) { return w; }
  __device__ static int32_t one() { return 1; }
  __device__ static bool nonzero(int32_t w) { return w != 0; }
};

template <typename S, typename W>
__global__ void __launch_bounds__(kThreads) narrow_encode_kernel(const S* __restrict__ src, W* __restrict__ wire,
                                                                long long n, long long cap) {
  bool big = false, neg = false;
  const long long stride = static_cast<long long>(gridDim.x) * kThreads * kPer;
  for (long long base = static_cast<long long>(blockIdx.x) * kThreads * kPer + threadIdx.x; base < n;
       base += stride) {
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const long long i = base + static_cast<long long>(k) * kThreads;  // coalesced per unrolled load
      if (i < n) {
        const long long v = static_cast<long long>(src[i]);
        big |= v > cap;
        neg |= v < 0;
        wire[i] = Wire<W>::enc(v);
      }
    }
  }
  // one store per wave that saw a failure (every writer stores the same value; the slots were zeroed in stream order)
  if (__ballot(big) != 0 && (threadIdx.x & (kWave - 1)) == 0) wire[n] = Wire<W>::one();
  if (__ballot(neg) != 0 && (threadIdx.x & (kWave - 1)) == 0) wire[n + 1] = Wire<W>::one();
}

template <typename W, typename O>
__global__ void __launch_bounds__(kThreads) narrow_decode_kernel(const W* __restrict__ wire, O* __restrict__ out,
                                                                long long n, int* __restrict__ word, int bit) {
  if (word != nullptr && blockIdx.x == 0 && threadIdx.x == 0 &&
      (Wire<W>::nonzero(wire[n]) || Wire<W>::nonzero(wire[n + 1])))
    raise_flag(word, bit);
  const long long stride = static_cast<long long>(gridDim.x) * kThreads * kPer;
  for (long long base = static_cast<long long>(blockIdx.x) * kThreads * kPer + threadIdx.x; base < n;
       base += stride) {
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const long long i = base + static_cast<long long>(k) * kThreads;  // coalesced per unrolled load
      if (i < n) out[i] = static_cast<O>(Wire<W>::dec(wire[i]));
    }
  }
}

int blocks_for(long long n) { return grid_cap((n + kThreads * kPer - 1) / (kThreads * kPer), 256 * 8); }

at::ScalarType wire_dtype(int64_t code) {
  TORCH_CHECK(code >= 0 && code <= 2, "narrow wire: code must be 0 (uint8), 1 (fp16) or 2 (int32)");
  return code == 0 ? at::kByte : (code == 1 ? at::kHalf : at::kInt);
}

template <typename W>
long long wire_max() {
  return Wire<W>::kMax;
}

}  // namespace

at::Tensor narrow_encode(const at::Tensor& src, int64_t code, int64_t world) {
  TM_CHECK_CUDA(src);
  TM_CHECK_CONTIG(src);
  TORCH_CHECK(src.scalar_type() == at::kLong || src.scalar_type() == at::kInt, "narrow_encode: int64 / int32 source");
  TORCH_CHECK(world >= 1, "narrow_encode: world must be positive");
  const long long n = src.numel();
  at::Tensor wire = at::empty({n + 2}, src.options().dtype(wire_dtype(code)));
  C10_HIP_CHECK(hipMemsetAsync(static_cast<char*>(wire.data_ptr()) + n * wire.element_size(), 0,
                               2 * wire.element_size(), stream()));
  if (n == 0) return wire;
  AT_DISPATCH_SWITCH(src.scalar_type(), "narrow_encode", AT_DISPATCH_CASE(at::kLong, [&] {
    using S = scalar_t;
    auto launch = [&](auto* w) {
      using W = std::remove_pointer_t<decltype(w)>;
      hipLaunchKernelGGL((narrow_encode_kernel<S, W>), dim3(blocks_for(n)), dim3(kThreads), 0, stream(),
                         src.data_ptr<S>(), w, n, wire_max<W>() / world);
    };
    if (code == 0) launch(wire.data_ptr<uint8_t>());
    else if (code == 1) launch(reinterpret_cast<__half*>(wire.data_ptr<at::Half>()));
    else launch(wire.data_ptr<int32_t>());
  }) AT_DISPATCH_CASE(at::kInt, [&] {
    using S = scalar_t;
    TORCH_CHECK(code != 2, "narrow_encode: an int32 source is not narrowed to int32");
    auto launch = [&](auto* w) {
      using W = std::remove_pointer_t<decltype(w)>;
      hipLaunchKernelGGL((narrow_encode_kernel<S, W>), dim3(blocks_for(n)), dim3(kThreads), 0, stream(),
                         src.data_ptr<S>(), w, n, wire_max<W>() / world);
    };
    if (code == 0) launch(wire.data_ptr<uint8_t>());
    else launch(reinterpret_cast<__half*>(wire.data_ptr<at::Half>()));
  }));
  C10_HIP_KERNEL_LAUNCH_CHECK();
  return wire;
}

at::Tensor narrow_decode(const at::Tensor& wire, int64_t n, at::ScalarType out_dtype, const c10::optional<at::Tensor>& word,
                         int64_t bit) {
  TM_CHECK_CUDA(wire);
  TM_CHECK_CONTIG(wire);
  TORCH_CHECK(wire.dim() == 1 && wire.numel() == n + 2, "narrow_decode: wire must be [n + 2]");
  TORCH_CHECK(out_dtype == at::kLong || out_dtype == at::kInt, "narrow_decode: int64 / int32 output");
  int* wp = nullptr;
  if (word.has_value() && word->defined()) {
    TM_SAME_DEVICE(wire, (*word));
    TORCH_CHECK(word->scalar_type() == at::kInt && word->numel() >= 1, "narrow_decode: word must be int32");
    wp = word->data_ptr<int>();
  }
  at::Tensor out = at::empty({n}, wire.options().dtype(out_dtype));
  auto launch = [&](auto* w, auto* o) {
    using W = std::remove_const_t<std::remove_pointer_t<decltype(w)>>;
    using O = std::remove_pointer_t<decltype(o)>;
    hipLaunchKernelGGL((narrow_decode_kernel<W, O>), dim3(std::max(blocks_for(n), 1)), dim3(kThreads), 0, stream(),
                       w, o, n, wp, static_cast<int>(bit));
  };
  auto with_out = [&](auto* w) {
    if (out_dtype == at::kLong) launch(w, out.data_ptr<int64_t>());
    else launch(w, out.data_ptr<int32_t>());
  };
  switch (wire.scalar_type()) {
    case at::kByte: with_out(wire.data_ptr<uint8_t>()); break;
    case at::kHalf: with_out(reinterpret_cast<const __half*>(wire.data_ptr<at::Half>())); break;
    case at::kInt: with_out(wire.data_ptr<int32_t>()); break;
    default: TORCH_CHECK(false, "narrow_decode: wire must be uint8 / fp16 / int32");
  }
  C10_HIP_KERNEL_LAUNCH_CHECK();
  return out;
}

// Optimistic static-shape gather (parallel/sync.py ``_gather_static``): every rank sends its fixed-shape
// ``None`` / callable-reduction states at their configured shapes plus one signature element (1 = every state had
// that shape and dtype, 0 = not) in ONE all_gather with no shape header.  This one-thread-per-rank check ORs `bit`
// into the caller's validation word when any rank's signature (the last column of the gathered [W, L + 1] buffer) is
// not 1; compute() reads the word anyway and re-syncs with the header in that (rare) case.
namespace {
template <typename T>
__global__ void static_sig_check_kernel(const T* __restrict__ g, int world, long long row, int* __restrict__ word,
                                        int bit) {
  const int r = threadIdx.x;
  const bool bad = r < world && static_cast<double>(g[static_cast<long long>(r) * row + row - 1]) != 1.0;
  if (__any(bad) && (threadIdx.x & (kWave - 1)) == 0) atomicOr(word, bit);
}
}  // namespace

void static_gather_check(const at::Tensor& gathered, at::Tensor word, int64_t bit) {
  TM_CHECK_CUDA(gathered);
  TM_SAME_DEVICE(gathered, word);
  TM_CHECK_CONTIG(gathered);
  TORCH_CHECK(gathered.dim() == 2 && gathered.size(1) >= 1, "static_gather_check: gathered must be [W, L + 1]");
  TORCH_CHECK(word.scalar_type() == at::kInt && word.numel() >= 1, "static_gather_check: word must be int32");
  const int world = static_cast<int>(gathered.size(0));
  TORCH_CHECK(world >= 1 && world <= 1024, "static_gather_check: 1 <= W <= 1024");
  const long long row = gathered.size(1);
  const int threads = (world + kWave - 1) / kWave * kWave;
  AT_DISPATCH_ALL_TYPES_AND2(at::kHalf, at::kBFloat16, gathered.scalar_type(), "static_gather_check", [&] {
    hipLaunchKernelGGL((static_sig_check_kernel<scalar_t>), dim3(1), dim3(threads), 0, stream(),
                       gathered.data_ptr<scalar_t>(), world, row, word.data_ptr<int>(), static_cast<int>(bit));
  });
  C10_HIP_KERNEL_LAUNCH_CHECK();
}

TORCH_LIBRARY_FRAGMENT(tm_amd, m) {
  m.def("narrow_encode(Tensor src, int code, int world) -> Tensor");
  m.def("narrow_decode(Tensor wire, int n, ScalarType out_dtype, Tensor? word, int bit) -> Tensor");
  m.def("static_gather_check(Tensor gathered, Tensor(a!) word, int bit) -> ()");
}
TORCH_LIBRARY_IMPL(tm_amd, CUDA, m) {
  m.impl("narrow_encode", &narrow_encode);
  m.impl("narrow_decode", &narrow_decode);
  m.impl("static_gather_check", &static_gather_check);
}

}  // namespace tm_amd
