// Measurement probes (benchmarks/bench_atomics.py): the cost of the flush patterns the histogram kernels use.
//
// atomic_probe: `blocks` blocks of 64 threads; thread t < bins of every block adds 1 to out[t * spread] (int64 when
// out is int64, else int32).  bins = 31, spread = 1 is a few-bin kernel's per-block flush onto one shared histogram:
// every bin address receives `blocks` device-scope atomics.
#include "../common/tm_common.h"

namespace tm_amd {
namespace {

template <typename T>
__global__ void __launch_bounds__(64) atomic_probe_kernel(T* __restrict__ out, int bins, int spread) {
  if (static_cast<int>(threadIdx.x) < bins) atomicAdd(out + static_cast<long long>(threadIdx.x) * spread, T(1));
}

}  // namespace

void atomic_probe(at::Tensor out, int64_t blocks, int64_t bins, int64_t spread) {
  TM_CHECK_CUDA(out);
  TORCH_CHECK(bins >= 1 && bins <= 64 && spread >= 1 && blocks >= 1 && blocks < (1 << 20), "atomic_probe: bad shape");
  TORCH_CHECK(out.is_contiguous() && out.numel() >= (bins - 1) * spread + 1, "atomic_probe: out too small");
  if (out.scalar_type() == at::kLong) {
    hipLaunchKernelGGL(atomic_probe_kernel<unsigned long long>, dim3(blocks), dim3(64), 0, stream(),
                       reinterpret_cast<unsigned long long*>(out.data_ptr<int64_t>()), static_cast<int>(bins),
                       static_cast<int>(spread));
  } else {
    TORCH_CHECK(out.scalar_type() == at::kInt, "atomic_probe: int32 / int64 out");
    hipLaunchKernelGGL(atomic_probe_kernel<int>, dim3(blocks), dim3(64), 0, stream(), out.data_ptr<int>(),
                       static_cast<int>(bins), static_cast<int>(spread));
  }
  C10_HIP_KERNEL_LAUNCH_CHECK();
}

TORCH_LIBRARY_FRAGMENT(tm_amd, m) { m.def("atomic_probe(Tensor(a!) out, int blocks, int bins, int spread) -> ()"); }
TORCH_LIBRARY_IMPL(tm_amd, CUDA, m) { m.impl("atomic_probe", &atomic_probe); }

}  // namespace tm_amd
