// Macro-averaged curves (multiclass / multilabel ROC and precision-recall with average="macro"): the mean over the C
// per-class curves of their piecewise-linear interpolation at every point of the merged grid, in ONE launch.
//
// The reference (F/classification/roc.py:189-200, precision_recall_curve.py:566-580, utilities/compute.py:134-157)
// loops over the classes in Python: per class one `interp` = slope / intercept / searchsorted / gather / mul / add
// chain (~10 launches), C x 10 launches per compute().  Here one thread owns one grid point x[j] and walks the C curves
// in class order, doing exactly what `interp` does for it:
//   idx   = upper_bound(xp_c, x[j]) - 1, clamped to [0, n_c - 2]   (torch.searchsorted(right=True)'s binary search --
//           the same probe sequence, so curves whose xp is not monotone, e.g. per-class precision, give the same idx)
//   slope = (fp[idx+1] - fp[idx]) / (xp[idx+1] - xp[idx], or 1 if that is 0)         (`_safe_divide`)
//   value = slope * x + (fp[idx] - slope * xp[idx])
// and accumulates `mean += value` in class order, then divides by C: every operation is rounded as the reference's
// separate ATen kernels round it (explicit _rn intrinsics: no fma contraction), so the result is bit-identical.
// Curves are ragged: xp / fp flat [T] with offsets [C + 1] (n_c = offsets[c+1] - offsets[c] >= 2; n_c == 1 gives the
// reference's empty-slope behaviour, handled as a constant).
#include "../common/tm_common.h"

#include <ATen/Parallel.h>

// The fp64 ops below are written as operators under this pragma: the HIP math header's __dmul_rn / __dadd_rn are plain
// operators compiled with contraction allowed, so the device compiler fused slope * v + intercept into one FMA (one
// rounding short of the reference's separate mul and add kernels; measured: 28 of 64 grid points 1 ulp off)
#pragma clang fp contract(off)

namespace tm_amd {
namespace {

// Rounding policies: the device one pins every operation to its own correctly rounded instruction (no fma
// contraction, matching the reference's one-op-per-kernel ATen chain); the host one is plain C++ (built without fma
// contraction for the x86-64 baseline).
struct DevRn {
  static __device__ __forceinline__ float mul(float a, float b) { return __fmul_rn(a, b); }
  static __device__ __forceinline__ float add(float a, float b) { return __fadd_rn(a, b); }
  static __device__ __forceinline__ float sub(float a, float b) { return __fsub_rn(a, b); }
  static __device__ __forceinline__ float div(float a, float b) { return __fdiv_rn(a, b); }
  static __device__ __forceinline__ double mul(double a, double b) { return a * b; }
  static __device__ __forceinline__ double add(double a, double b) { return a + b; }
  static __device__ __forceinline__ double sub(double a, double b) { return a - b; }
  static __device__ __forceinline__ double div(double a, double b) { return a / b; }
};
struct HostRn {
  template <typename T>
  static T mul(T a, T b) { return a * b; }
  template <typename T>
  static T add(T a, T b) { return a + b; }
  template <typename T>
  static T sub(T a, T b) { return a - b; }
  template <typename T>
  static T div(T a, T b) { return a / b; }
};

// interp of one curve at v (see the file header)
template <typename Rn, typename T>
__device__ __host__ __forceinline__ T interp_one(const T* __restrict__ xp, const T* __restrict__ fp, long long n, T v) {
  if (n < 2) return T(0);  // no segment: the reference's empty slope tensor -> nothing to gather (caller skips)
  long long lo = 0, hi = n;  // upper_bound with torch's probe sequence
  while (lo < hi) {
    const long long mid = lo + ((hi - lo) >> 1);
    if (!(xp[mid] > v)) lo = mid + 1;
    else hi = mid;
  }
  long long k = lo - 1;
  if (k < 0) k = 0;
  if (k > n - 2) k = n - 2;
  T den = Rn::sub(xp[k + 1], xp[k]);
  if (den == T(0)) den = T(1);
  const T slope = Rn::div(Rn::sub(fp[k + 1], fp[k]), den);
  const T icpt = Rn::sub(fp[k], Rn::mul(slope, xp[k]));
  return Rn::add(Rn::mul(slope, v), icpt);
}

template <typename T>
__global__ void __launch_bounds__(256) interp_mean_kernel(const T* __restrict__ x, long long M,
                                                          const T* __restrict__ xp, const T* __restrict__ fp,
                                                          const int64_t* __restrict__ off, int C, T* __restrict__ out) {
  for (long long j = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x; j < M;
       j += static_cast<long long>(gridDim.x) * blockDim.x) {
    const T v = x[j];
    T acc = T(0);
    for (int c = 0; c < C; ++c) {
      const long long b = off[c], n = off[c + 1] - b;
      if (n >= 2) acc = DevRn::add(acc, interp_one<DevRn>(xp + b, fp + b, n, v));
    }
    out[j] = DevRn::div(acc, static_cast<T>(C));
  }
}

void check_args(const at::Tensor& x, const at::Tensor& xp, const at::Tensor& fp, const at::Tensor& off) {
  TORCH_CHECK(x.dim() == 1 && xp.dim() == 1 && fp.dim() == 1 && off.dim() == 1, "interp_mean: 1-D inputs");
  TORCH_CHECK(x.scalar_type() == xp.scalar_type() && xp.scalar_type() == fp.scalar_type() &&
                  (x.scalar_type() == at::kFloat || x.scalar_type() == at::kDouble),
              "interp_mean: x / xp / fp must share one float32 / float64 dtype");
  TORCH_CHECK(off.scalar_type() == at::kLong && off.numel() >= 2, "interp_mean: offsets int64 [C + 1]");
  TORCH_CHECK(xp.numel() == fp.numel(), "interp_mean: xp / fp lengths differ");
  TM_CHECK_CONTIG(x);
  TM_CHECK_CONTIG(xp);
  TM_CHECK_CONTIG(fp);
  TM_CHECK_CONTIG(off);
}

}  // namespace

// mean over the C curves (xp, fp)[off[c] : off[c+1]] of interp(x, xp_c, fp_c); x [M] -> [M]
at::Tensor interp_mean(const at::Tensor& x, const at::Tensor& xp, const at::Tensor& fp, const at::Tensor& off) {
  TM_CHECK_CUDA(x);
  TM_SAME_DEVICE(x, xp);
  TM_SAME_DEVICE(x, fp);
  TM_SAME_DEVICE(x, off);
  check_args(x, xp, fp, off);
  auto out = at::empty_like(x);
  const long long M = x.numel();
  const int C = static_cast<int>(off.numel() - 1);
  if (M == 0) return out;
  const int grid = grid_cap((M + 255) / 256);
  AT_DISPATCH_FLOATING_TYPES(x.scalar_type(), "interp_mean", [&] {
    hipLaunchKernelGGL(interp_mean_kernel<scalar_t>, dim3(grid), dim3(256), 0, stream(), x.data_ptr<scalar_t>(), M,
                       xp.data_ptr<scalar_t>(), fp.data_ptr<scalar_t>(), off.data_ptr<int64_t>(), C,
                       out.data_ptr<scalar_t>());
  });
  C10_HIP_KERNEL_LAUNCH_CHECK();
  return out;
}

// host twin (CPU tensors): the same per-point walk
at::Tensor interp_mean_cpu(const at::Tensor& x, const at::Tensor& xp, const at::Tensor& fp, const at::Tensor& off) {
  check_args(x, xp, fp, off);
  auto out = at::empty_like(x);
  const long long M = x.numel();
  const int C = static_cast<int>(off.numel() - 1);
  const int64_t* o = off.data_ptr<int64_t>();
  AT_DISPATCH_FLOATING_TYPES(x.scalar_type(), "interp_mean_cpu", [&] {
    const scalar_t* xv = x.data_ptr<scalar_t>();
    const scalar_t* xpv = xp.data_ptr<scalar_t>();
    const scalar_t* fpv = fp.data_ptr<scalar_t>();
    scalar_t* ov = out.data_ptr<scalar_t>();
    at::parallel_for(0, M, 2048, [&](int64_t beg, int64_t end) {
      for (int64_t j = beg; j < end; ++j) {
        scalar_t acc = 0;
        for (int c = 0; c < C; ++c) {
          const long long b = o[c], n = o[c + 1] - b;
          if (n >= 2) acc = acc + interp_one<HostRn>(xpv + b, fpv + b, n, xv[j]);
        }
        ov[j] = acc / static_cast<scalar_t>(C);
      }
    });
  });
  return out;
}

TORCH_LIBRARY_FRAGMENT(tm_amd, m) { m.def("interp_mean(Tensor x, Tensor xp, Tensor fp, Tensor offsets) -> Tensor"); }
TORCH_LIBRARY_IMPL(tm_amd, CUDA, m) { m.impl("interp_mean", &interp_mean); }
TORCH_LIBRARY_IMPL(tm_amd, CPU, m) { m.impl("interp_mean", &interp_mean_cpu); }

}  // namespace tm_amd
