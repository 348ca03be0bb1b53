// Macro-averaged curves (multiclass / multilabel ROC and precision-recall with average="macro"): the mean over the C
// per-class curves of their piecewise-linear interpolation at every point of the merged grid, in ONE launch.
//
// The reference (F/classification/roc.py:189-200, precision_recall_curve.py:566-580, utilities/compute.py:134-157)
// loops over the classes in Python: per class one `interp` = slope / intercept / searchsorted / gather / mul / add
// chain (~10 launches), C x 10 launches per compute().  Here one thread owns one grid point x[j] and walks the C curves
// in class order, doing exactly what `interp` does for it:
//   idx   = #{i : x[j] >= xp_c[i]} - 1, clamped to [0, n_c - 2]   (the reference's `sum(ge(x[:, None], xp[None]), 1) - 1`,
//           utilities/compute.py:154: a COUNT over the whole curve, not a search, so it is also the reference's segment
//           for curves whose xp is not monotone -- per-class precision).  The count is order-free, so it is an
//           upper_bound over a per-class SORTED copy of xp (one segmented radix sort of order-preserving keys, NaN
//           last: `v >= NaN` is false, as in the reference); the slope / intercept use the curve in its own order.
//   slope = (fp[idx+1] - fp[idx]) / (xp[idx+1] - xp[idx], or 1 if that is 0)         (`_safe_divide`)
//   value = slope * x + (fp[idx] - slope * xp[idx])
// and accumulates `mean += value` in class order, then divides by C: every operation is rounded as the reference's
// separate ATen kernels round it (explicit _rn intrinsics: no fma contraction), so the result is bit-identical.
// Curves are ragged: xp / fp flat [T] with offsets [C + 1] (n_c = offsets[c+1] - offsets[c] >= 2; n_c == 1 gives the
// reference's empty-slope behaviour, handled as a constant).
#include "../common/tm_common.h"
#include "../sort/sortscan.h"

#include <ATen/Parallel.h>

#include <algorithm>
#include <cstring>
#include <vector>

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

// ascending order-preserving radix key (NaN canonical and last, -0.0 == +0.0): a >= b <=> key(a) >= key(b) for
// non-NaN a, b; a NaN xp sorts after every number, so `v >= xp` is false for it as for the reference's ge
template <typename T>
struct AscKey;
template <>
struct AscKey<float> {
  using K = uint32_t;
  static __device__ __host__ __forceinline__ K of(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    if (f != f) u = 0x7fc00000u;
    else if (f == 0.0f) u = 0u;
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
  }
};
template <>
struct AscKey<double> {
  using K = uint64_t;
  static __device__ __host__ __forceinline__ K of(double d) {
    uint64_t u;
    memcpy(&u, &d, 8);
    if (d != d) u = 0x7ff8000000000000ULL;
    else if (d == 0.0) u = 0ULL;
    return (u & 0x8000000000000000ULL) ? ~u : (u | 0x8000000000000000ULL);
  }
};

// interp of one curve at v (see the file header); ``xs`` = the curve's xp keys in ascending order
template <typename Rn, typename T>
__device__ __host__ __forceinline__ T interp_one(const T* __restrict__ xp, const T* __restrict__ fp,
                                                 const typename AscKey<T>::K* __restrict__ xs, long long n, T v) {
  if (n < 2) return T(0);  // no segment: the reference's empty slope tensor -> nothing to gather (caller skips)
  long long lo = 0;
  if (v == v) {  // count of xp <= v (a NaN v is >= nothing: count 0)
    const auto kv = AscKey<T>::of(v);
    long long hi = n;
    while (lo < hi) {
      const long long mid = lo + ((hi - lo) >> 1);
      if (kv >= xs[mid]) lo = mid + 1;
      else hi = mid;
    }
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

// per element: its ascending key and its class (segment) id
template <typename T>
__global__ void __launch_bounds__(256) interp_keys_kernel(const T* __restrict__ xp, long long n,
                                                          const int64_t* __restrict__ off, int C,
                                                          typename AscKey<T>::K* __restrict__ key,
                                                          int32_t* __restrict__ seg) {
  for (long long i = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += static_cast<long long>(gridDim.x) * blockDim.x) {
    int lo = 0, hi = C;  // last c with off[c] <= i
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (off[mid] <= i) lo = mid;
      else hi = mid;
    }
    key[i] = AscKey<T>::of(xp[i]);
    seg[i] = lo;
  }
}

template <typename T>
__global__ void __launch_bounds__(256) interp_mean_kernel(const T* __restrict__ x, long long M,
                                                          const T* __restrict__ xp, const T* __restrict__ fp,
                                                          const typename AscKey<T>::K* __restrict__ xs,
                                                          const int64_t* __restrict__ off, int C, T* __restrict__ out) {
  for (long long j = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x; j < M;
       j += static_cast<long long>(gridDim.x) * blockDim.x) {
    const T v = x[j];
    T acc = T(0);
    for (int c = 0; c < C; ++c) {
      const long long b = off[c], n = off[c + 1] - b;
      if (n >= 2) acc = DevRn::add(acc, interp_one<DevRn>(xp + b, fp + b, xs + b, n, v));
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
  const long long T_ = xp.numel();
  const auto dev = x.device();
  AT_DISPATCH_FLOATING_TYPES(x.scalar_type(), "interp_mean", [&] {
    using K = typename AscKey<scalar_t>::K;
    constexpr auto kdt = sizeof(K) == 4 ? at::kInt : at::kLong;
    // per-class sorted xp keys: sort by key, then (stable) by class id
    auto key = at::empty({T_}, x.options().dtype(kdt));
    auto key2 = at::empty_like(key);
    auto seg = at::empty({T_}, x.options().dtype(at::kInt));
    auto seg2 = at::empty_like(seg);
    if (T_ > 0) {
      hipLaunchKernelGGL(interp_keys_kernel<scalar_t>, dim3(grid_cap((T_ + 255) / 256)), dim3(256), 0, stream(),
                         xp.data_ptr<scalar_t>(), T_, off.data_ptr<int64_t>(), C,
                         reinterpret_cast<K*>(key.data_ptr()), seg.data_ptr<int32_t>());
      sortscan::sort_pairs(reinterpret_cast<const K*>(key.data_ptr()), reinterpret_cast<K*>(key2.data_ptr()),
                           seg.data_ptr<int32_t>(), seg2.data_ptr<int32_t>(), T_, 0, 8 * int(sizeof(K)), dev,
                           stream());
      if (C > 1)
        sortscan::sort_pairs(reinterpret_cast<const uint32_t*>(seg2.data_ptr()),
                             reinterpret_cast<uint32_t*>(seg.data_ptr()), reinterpret_cast<const K*>(key2.data_ptr()),
                             reinterpret_cast<K*>(key.data_ptr()), T_, 0, sortscan::ceil_log2(C), dev, stream());
      else
        key.copy_(key2);
    }
    hipLaunchKernelGGL(interp_mean_kernel<scalar_t>, dim3(grid_cap((M + 255) / 256)), dim3(256), 0, stream(),
                       x.data_ptr<scalar_t>(), M, xp.data_ptr<scalar_t>(), fp.data_ptr<scalar_t>(),
                       reinterpret_cast<const K*>(key.data_ptr()), off.data_ptr<int64_t>(), C,
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
    using K = typename AscKey<scalar_t>::K;
    std::vector<K> xs(static_cast<size_t>(xp.numel()));
    for (int c = 0; c < C; ++c) {
      for (int64_t i = o[c]; i < o[c + 1]; ++i) xs[i] = AscKey<scalar_t>::of(xpv[i]);
      std::sort(xs.begin() + o[c], xs.begin() + o[c + 1]);
    }
    at::parallel_for(0, M, 2048, [&](int64_t beg, int64_t end) {
      for (int64_t j = beg; j < end; ++j) {
        scalar_t acc = 0;
        for (int c = 0; c < C; ++c) {
          const long long b = o[c], n = o[c + 1] - b;
          if (n >= 2) acc = acc + interp_one<HostRn>(xpv + b, fpv + b, xs.data() + b, n, xv[j]);
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
