// Deterministic integer histogram (bincount) used by _bincount and the clustering / nominal contingency paths.
// LDS-privatised when the bin count fits (one int32 sub-histogram per block, flushed with 64-bit atomics),
// global 64-bit atomics otherwise.  Integer atomics are order-independent, so the result is deterministic
// (the reference needs an O(N*C) fallback under torch.use_deterministic_algorithms, S/utilities/data.py:203-205).
#include "tm_common.h"

namespace tm_amd {
namespace {
constexpr int kBlock = 256;
constexpr int kLdsBins = 12288;

template <typename idx_t>
__global__ void __launch_bounds__(kBlock) histogram_kernel(const idx_t* __restrict__ x, long long n, long long nbins,
                                                           int64_t* __restrict__ out, int* __restrict__ flag,
                                                           bool use_lds) {
  extern __shared__ __attribute__((aligned(16))) int lds[];
  if (use_lds) {
    for (long long b = threadIdx.x; b < nbins; b += blockDim.x) lds[b] = 0;
    __syncthreads();
  }
  for (long long i = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += static_cast<long long>(gridDim.x) * blockDim.x) {
    const long long v = static_cast<long long>(x[i]);
    if (v < 0 || v >= nbins) {
      raise_flag(flag, kErrValueNan);
      continue;
    }
    if (use_lds)
      atomicAdd(&lds[v], 1);
    else
      atomic_add_i64(out + v, 1);
  }
  if (use_lds) {
    __syncthreads();
    for (long long b = threadIdx.x; b < nbins; b += blockDim.x) {
      const int c = lds[b];
      if (c) atomic_add_i64(out + b, c);
    }
  }
}
}  // namespace

void histogram(const at::Tensor& x, at::Tensor out, at::Tensor flag) {
  TM_CHECK_CUDA(x);
  TM_CHECK_CONTIG(x);
  TORCH_CHECK(out.scalar_type() == at::kLong && out.is_contiguous(), "histogram: out must be contiguous int64");
  const long long n = x.numel();
  if (n == 0) return;
  const long long nbins = out.numel();
  const int grid = grid_cap((n + kBlock * 8 - 1) / (kBlock * 8), 256 * 8);
  const bool use_lds = nbins <= kLdsBins && static_cast<long long>(grid) * kBlock * 2 <= n;
  const size_t lds = use_lds ? nbins * sizeof(int) : 0;
  TM_DISPATCH_TARGET(x.scalar_type(), "histogram", [&] {
    hipLaunchKernelGGL((histogram_kernel<target_t>), dim3(grid), dim3(kBlock), lds, stream(),
                       reinterpret_cast<const target_t*>(x.data_ptr()), n, nbins, out.data_ptr<int64_t>(),
                       flag.data_ptr<int>(), use_lds);
  });
  C10_HIP_KERNEL_LAUNCH_CHECK();
}

}  // namespace tm_amd

TORCH_LIBRARY_FRAGMENT(tm_amd, m) { m.def("histogram(Tensor x, Tensor(a!) out, Tensor(b!) flag) -> ()"); }

TORCH_LIBRARY_IMPL(tm_amd, CUDA, m) { m.impl("histogram", &tm_amd::histogram); }
