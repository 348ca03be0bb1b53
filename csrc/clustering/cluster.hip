// Clustering / nominal-association kernels.
//
// Reference sites: F/clustering/utils.py:119-173 (`calculate_contingency_matrix`: two `torch.unique` sorts, a sparse
// COO tensor densified), F/clustering/davies_bouldin_score.py:46-57 / dunn_index.py / calinski_harabasz_score.py
// (per-cluster Python loops over `data[labels == k]`), F/nominal/utils.py:35-110 (confusion-matrix based tables).
//
// * label_minmax: one pass -> [min, max] of an integer label tensor (per-block partials, fixed-order final reduce).
//   The host reads the two numbers once and sizes a DENSE contingency over the label ranges, instead of sorting both
//   label tensors (`unique(return_inverse)`), which is what dominates the reference path at 10^7 labels.
// * contingency_dense: 2-D histogram of (target - tmin, preds - pmin) into an int64 [Rt, Rp] table with the key
//   computed in registers (no key tensor); LDS-privatised int32 sub-tables when Rt * Rp fits, 64-bit global atomics
//   otherwise.  Integer atomics are order-independent: bitwise deterministic.  Empty rows / columns (label values
//   that never occur) are dropped on the host side by their marginals, which reproduces the sorted-unique order.
// * cluster_sums: per-cluster feature sums (fp64) and sizes for dense cluster ids -- LDS-privatised [K, D] fp64
//   partials when K * D <= 4096, fp64 global atomics otherwise.
// * cluster_dispersion: one pass over the samples with the centroids in LDS: per sample the Minkowski-p distance to
//   its centroid and the squared L2 distance; per cluster Σ d_p and max d_p (Davies-Bouldin intra, Dunn radius), and
//   the total Σ d2 (Calinski-Harabasz within-dispersion).
#include <climits>

#include "../common/tm_common.h"

namespace tm_amd {
namespace {

constexpr int kBlock = 256;
constexpr int kLdsBins = 8192;     // int32 contingency bins per block in LDS (32 KiB)
constexpr int kLdsSums = 4096;     // fp64 [K, D] partial sums per block in LDS (32 KiB)
constexpr long long kMaxLdsBytes = 64 * 1024;

template <typename T>
__global__ void __launch_bounds__(kBlock) minmax_partial_kernel(const T* __restrict__ x, long long n,
                                                                int64_t* __restrict__ part) {
  long long mn = LLONG_MAX, mx = LLONG_MIN;
  for (long long i = static_cast<long long>(blockIdx.x) * kBlock + threadIdx.x; i < n;
       i += static_cast<long long>(gridDim.x) * kBlock) {
    const long long v = static_cast<long long>(x[i]);
    mn = v < mn ? v : mn;
    mx = v > mx ? v : mx;
  }
  __shared__ long long smn[kBlock / kWave], smx[kBlock / kWave];
#pragma unroll
  for (int off = kWave / 2; off > 0; off >>= 1) {
    const long long a = __shfl_xor(mn, off, kWave), b = __shfl_xor(mx, off, kWave);
    mn = a < mn ? a : mn;
    mx = b > mx ? b : mx;
  }
  const int wave = threadIdx.x / kWave;
  if ((threadIdx.x & (kWave - 1)) == 0) {
    smn[wave] = mn;
    smx[wave] = mx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < kBlock / kWave; ++w) {
      mn = smn[w] < mn ? smn[w] : mn;
      mx = smx[w] > mx ? smx[w] : mx;
    }
    part[2 * blockIdx.x] = mn;
    part[2 * blockIdx.x + 1] = mx;
  }
}

// one wave over the block partials (min / max are exact in any order; the first version walked them with one thread:
// ~107 us for 2048 partials of dependent loads)
__global__ void minmax_final_kernel(const int64_t* __restrict__ part, int nb, int64_t* __restrict__ out) {
  long long mn = LLONG_MAX, mx = LLONG_MIN;
  for (int b = threadIdx.x; b < nb; b += kWave) {
    mn = part[2 * b] < mn ? part[2 * b] : mn;
    mx = part[2 * b + 1] > mx ? part[2 * b + 1] : mx;
  }
#pragma unroll
  for (int off = kWave / 2; off > 0; off >>= 1) {
    const long long a = __shfl_xor(mn, off, kWave), b = __shfl_xor(mx, off, kWave);
    mn = a < mn ? a : mn;
    mx = b > mx ? b : mx;
  }
  if (threadIdx.x == 0) {
    out[0] = mn;
    out[1] = mx;
  }
}

template <typename TT, typename TP>
__global__ void __launch_bounds__(kBlock) contingency_kernel(const TT* __restrict__ t, const TP* __restrict__ p,
                                                             long long n, long long tmin, long long pmin, long long rt,
                                                             long long rp, int64_t* __restrict__ out, bool use_lds) {
  extern __shared__ __attribute__((aligned(16))) int lds[];
  const long long nbins = rt * rp;
  if (use_lds) {
    for (long long b = threadIdx.x; b < nbins; b += kBlock) lds[b] = 0;
    __syncthreads();
  }
  for (long long i = static_cast<long long>(blockIdx.x) * kBlock + threadIdx.x; i < n;
       i += static_cast<long long>(gridDim.x) * kBlock) {
    const long long r = static_cast<long long>(t[i]) - tmin, c = static_cast<long long>(p[i]) - pmin;
    if (r < 0 || r >= rt || c < 0 || c >= rp) continue;  // cannot happen for the ranges label_minmax reported
    const long long key = r * rp + c;
    if (use_lds)
      atomicAdd(&lds[key], 1);
    else
      atomic_add_i64(out + key, 1);
  }
  if (use_lds) {
    __syncthreads();
    for (long long b = threadIdx.x; b < nbins; b += kBlock) {
      const int v = lds[b];
      if (v) atomic_add_i64(out + b, v);
    }
  }
}

template <typename T>
__device__ __forceinline__ double to_f64(T v) {
  return static_cast<double>(to_f32(v));
}
template <>
__device__ __forceinline__ double to_f64<double>(double v) {
  return v;
}

template <typename T, typename I>
__global__ void __launch_bounds__(kBlock) cluster_sums_kernel(const T* __restrict__ x, const I* __restrict__ ids,
                                                              long long n, int d, int k, double* __restrict__ sums,
                                                              int64_t* __restrict__ sizes, bool use_lds) {
  extern __shared__ __attribute__((aligned(16))) double sl[];  // [k * d] sums, then [k] sizes as int
  int* cnt = reinterpret_cast<int*>(sl + static_cast<long long>(k) * d);
  if (use_lds) {
    for (int b = threadIdx.x; b < k * d; b += kBlock) sl[b] = 0.0;
    for (int b = threadIdx.x; b < k; b += kBlock) cnt[b] = 0;
    __syncthreads();
  }
  // one thread per (sample, feature) element: consecutive threads read consecutive features (coalesced)
  const long long total = n * d;
  for (long long e = static_cast<long long>(blockIdx.x) * kBlock + threadIdx.x; e < total;
       e += static_cast<long long>(gridDim.x) * kBlock) {
    const long long s = e / d;
    const int f = static_cast<int>(e - s * d);
    const long long c = static_cast<long long>(ids[s]);
    if (c < 0 || c >= k) continue;
    const double v = to_f64(x[e]);
    if (use_lds) {
      atomicAdd(&sl[c * d + f], v);
      if (f == 0) atomicAdd(&cnt[c], 1);
    } else {
      atomicAdd(&sums[c * d + f], v);
      if (f == 0) atomic_add_i64(sizes + c, 1);
    }
  }
  if (use_lds) {
    __syncthreads();
    for (int b = threadIdx.x; b < k * d; b += kBlock)
      if (sl[b] != 0.0) atomicAdd(&sums[b], sl[b]);
    for (int b = threadIdx.x; b < k; b += kBlock)
      if (cnt[b]) atomic_add_i64(sizes + b, cnt[b]);
  }
}

// ordered-int encoding of a non-negative double for atomicMax on its bits
__device__ __forceinline__ unsigned long long dbl_key(double v) { return __double_as_longlong(v); }

template <typename T, typename I>
__global__ void __launch_bounds__(kBlock) cluster_dispersion_kernel(const T* __restrict__ x,
                                                                    const I* __restrict__ ids, long long n, int d,
                                                                    int k, const double* __restrict__ cent, double p,
                                                                    double* __restrict__ dsum,
                                                                    unsigned long long* __restrict__ dmax,
                                                                    double* __restrict__ sq_total) {
  // LDS: centroids [k * d], per-cluster Σ d_p [k], per-cluster max d_p bits [k] (block-private, flushed once)
  extern __shared__ __attribute__((aligned(16))) double cl[];
  double* lsum = cl + static_cast<long long>(k) * d;
  unsigned long long* lmax = reinterpret_cast<unsigned long long*>(lsum + k);
  for (int b = threadIdx.x; b < k * d; b += kBlock) cl[b] = cent[b];
  for (int b = threadIdx.x; b < k; b += kBlock) {
    lsum[b] = 0.0;
    lmax[b] = 0ull;
  }
  __syncthreads();
  const bool pinf = isinf(p);
  double sq_acc = 0.0;
  for (long long s = static_cast<long long>(blockIdx.x) * kBlock + threadIdx.x; s < n;
       s += static_cast<long long>(gridDim.x) * kBlock) {
    const long long c = static_cast<long long>(ids[s]);
    if (c < 0 || c >= k) continue;
    const T* row = x + s * d;
    double acc_p = 0.0, acc2 = 0.0, accmax = 0.0;
    for (int f = 0; f < d; ++f) {
      const double diff = to_f64(row[f]) - cl[c * d + f];
      const double a = fabs(diff);
      acc2 += diff * diff;
      if (pinf) accmax = a > accmax ? a : accmax;
      else acc_p += p == 2.0 ? a * a : pow(a, p);
    }
    const double dist = pinf ? accmax : (p == 2.0 ? sqrt(acc_p) : pow(acc_p, 1.0 / p));
    sq_acc += acc2;
    atomicAdd(&lsum[c], dist);
    atomicMax(&lmax[c], dbl_key(dist));
  }
#pragma unroll
  for (int off = kWave / 2; off > 0; off >>= 1) sq_acc += __shfl_xor(sq_acc, off, kWave);
  if ((threadIdx.x & (kWave - 1)) == 0) atomicAdd(sq_total, sq_acc);
  __syncthreads();
  for (int b = threadIdx.x; b < k; b += kBlock) {
    if (lsum[b] != 0.0) atomicAdd(&dsum[b], lsum[b]);
    if (lmax[b] != 0ull) atomicMax(&dmax[b], lmax[b]);
  }
}

int grid_for(long long work) { return grid_cap((work + kBlock * 8 - 1) / (kBlock * 8), 256 * 8); }

}  // namespace

at::Tensor label_minmax(const at::Tensor& x) {
  TM_CHECK_CUDA(x);
  TM_CHECK_CONTIG(x);
  at::Tensor out = at::empty({2}, x.options().dtype(at::kLong));
  const long long n = x.numel();
  TORCH_CHECK(n > 0, "label_minmax: empty input");
  const int nb = grid_cap((n + kBlock * 16 - 1) / (kBlock * 16), 1024);
  at::Tensor part = at::empty({2 * nb}, x.options().dtype(at::kLong));
  TM_DISPATCH_TARGET(x.scalar_type(), "label_minmax", [&] {
    hipLaunchKernelGGL((minmax_partial_kernel<target_t>), dim3(nb), dim3(kBlock), 0, stream(),
                       reinterpret_cast<const target_t*>(x.data_ptr()), n, part.data_ptr<int64_t>());
  });
  hipLaunchKernelGGL(minmax_final_kernel, dim3(1), dim3(64), 0, stream(), part.data_ptr<int64_t>(), nb,
                     out.data_ptr<int64_t>());
  C10_HIP_KERNEL_LAUNCH_CHECK();
  return out;
}

void contingency_dense(const at::Tensor& target, const at::Tensor& preds, int64_t tmin, int64_t pmin, at::Tensor out) {
  TM_CHECK_CUDA(target);
  TM_SAME_DEVICE(target, preds);
  TM_SAME_DEVICE(target, out);
  TM_CHECK_CONTIG(target);
  TM_CHECK_CONTIG(preds);
  TORCH_CHECK(out.scalar_type() == at::kLong && out.dim() == 2 && out.is_contiguous(),
              "contingency_dense: out must be contiguous int64 [Rt, Rp]");
  TORCH_CHECK(target.numel() == preds.numel(), "contingency_dense: size mismatch");
  const long long n = target.numel();
  if (n == 0) return;
  const long long rt = out.size(0), rp = out.size(1);
  const int grid = grid_for(n);
  const bool use_lds = rt * rp <= kLdsBins && static_cast<long long>(grid) * kBlock * 2 <= n;
  const size_t lds = use_lds ? rt * rp * sizeof(int) : 0;
  TM_DISPATCH_TARGET(target.scalar_type(), "contingency_dense", [&] {
    using tt = target_t;
    const tt* tp = reinterpret_cast<const tt*>(target.data_ptr());
    TM_DISPATCH_TARGET(preds.scalar_type(), "contingency_dense", [&] {
      hipLaunchKernelGGL((contingency_kernel<tt, target_t>), dim3(grid), dim3(kBlock), lds, stream(), tp,
                         reinterpret_cast<const target_t*>(preds.data_ptr()), n, tmin, pmin, rt, rp,
                         out.data_ptr<int64_t>(), use_lds);
    });
  });
  C10_HIP_KERNEL_LAUNCH_CHECK();
}

#define TM_DISPATCH_FEATURES(TYPE, NAME, ...)                                                       \
  [&] {                                                                                            \
    switch (TYPE) {                                                                                \
      case at::kFloat: { using feat_t = float; return __VA_ARGS__(); }                             \
      case at::kDouble: { using feat_t = double; return __VA_ARGS__(); }                           \
      case at::kHalf: { using feat_t = c10::Half; return __VA_ARGS__(); }                          \
      case at::kBFloat16: { using feat_t = c10::BFloat16; return __VA_ARGS__(); }                  \
      default: TORCH_CHECK(false, NAME, ": unsupported feature dtype ", TYPE);                     \
    }                                                                                              \
  }()

void cluster_sums(const at::Tensor& x, const at::Tensor& ids, int64_t k, at::Tensor sums, at::Tensor sizes) {
  TM_CHECK_CUDA(x);
  TM_SAME_DEVICE(x, ids);
  TM_SAME_DEVICE(x, sums);
  TM_SAME_DEVICE(x, sizes);
  TM_CHECK_CONTIG(x);
  TM_CHECK_CONTIG(ids);
  TORCH_CHECK(x.dim() == 2 && ids.dim() == 1 && ids.size(0) == x.size(0), "cluster_sums: x [N, D], ids [N]");
  const long long n = x.size(0);
  const int d = static_cast<int>(x.size(1));
  TORCH_CHECK(sums.scalar_type() == at::kDouble && sums.is_contiguous() && sums.numel() == k * d,
              "cluster_sums: sums must be contiguous f64 [K, D]");
  TORCH_CHECK(sizes.scalar_type() == at::kLong && sizes.is_contiguous() && sizes.numel() == k,
              "cluster_sums: sizes must be int64 [K]");
  if (n == 0 || d == 0) return;
  const int grid = grid_for(n * d);
  const bool use_lds = k * d <= kLdsSums && static_cast<long long>(grid) * kBlock * 4 <= n * d;
  const size_t lds = use_lds ? k * d * sizeof(double) + k * sizeof(int) : 0;
  TM_DISPATCH_FEATURES(x.scalar_type(), "cluster_sums", [&] {
    TM_DISPATCH_TARGET(ids.scalar_type(), "cluster_sums", [&] {
      hipLaunchKernelGGL((cluster_sums_kernel<feat_t, target_t>), dim3(grid), dim3(kBlock), lds, stream(),
                         reinterpret_cast<const feat_t*>(x.data_ptr()),
                         reinterpret_cast<const target_t*>(ids.data_ptr()), n, d, static_cast<int>(k),
                         sums.data_ptr<double>(), sizes.data_ptr<int64_t>(), use_lds);
    });
  });
  C10_HIP_KERNEL_LAUNCH_CHECK();
}

// dsum f64 [K], dmax f64 [K] (non-negative distances; max via the ordered bits), sq_total f64 [1]
void cluster_dispersion(const at::Tensor& x, const at::Tensor& ids, const at::Tensor& cent, double p, at::Tensor dsum,
                        at::Tensor dmax, at::Tensor sq_total) {
  TM_CHECK_CUDA(x);
  for (const at::Tensor* t : {&ids, &cent}) TM_SAME_DEVICE(x, *t);
  TM_CHECK_CONTIG(x);
  TM_CHECK_CONTIG(ids);
  TM_CHECK_CONTIG(cent);
  const long long n = x.size(0);
  const int d = static_cast<int>(x.size(1));
  const int k = static_cast<int>(cent.size(0));
  TORCH_CHECK(cent.scalar_type() == at::kDouble && cent.dim() == 2 && cent.size(1) == d,
              "cluster_dispersion: centroids must be f64 [K, D]");
  TORCH_CHECK((static_cast<long long>(k) * d + 2LL * k) * 8 <= kMaxLdsBytes,
              "cluster_dispersion: K * D too large for LDS-resident centroids");
  TORCH_CHECK(dsum.scalar_type() == at::kDouble && dsum.numel() == k && dmax.scalar_type() == at::kDouble &&
                  dmax.numel() == k && sq_total.scalar_type() == at::kDouble && sq_total.numel() == 1,
              "cluster_dispersion: bad outputs");
  if (n == 0) return;
  const int grid = grid_for(n);
  const size_t lds = (static_cast<size_t>(k) * d + 2 * static_cast<size_t>(k)) * sizeof(double);
  TM_DISPATCH_FEATURES(x.scalar_type(), "cluster_dispersion", [&] {
    TM_DISPATCH_TARGET(ids.scalar_type(), "cluster_dispersion", [&] {
      hipLaunchKernelGGL((cluster_dispersion_kernel<feat_t, target_t>), dim3(grid), dim3(kBlock), lds, stream(),
                         reinterpret_cast<const feat_t*>(x.data_ptr()),
                         reinterpret_cast<const target_t*>(ids.data_ptr()), n, d, k, cent.data_ptr<double>(), p,
                         dsum.data_ptr<double>(), reinterpret_cast<unsigned long long*>(dmax.data_ptr<double>()),
                         sq_total.data_ptr<double>());
    });
  });
  C10_HIP_KERNEL_LAUNCH_CHECK();
}

TORCH_LIBRARY_FRAGMENT(tm_amd, m) {
  m.def("label_minmax(Tensor x) -> Tensor");
  m.def("contingency_dense(Tensor target, Tensor preds, int tmin, int pmin, Tensor(a!) out) -> ()");
  m.def("cluster_sums(Tensor x, Tensor ids, int k, Tensor(a!) sums, Tensor(b!) sizes) -> ()");
  m.def(
      "cluster_dispersion(Tensor x, Tensor ids, Tensor cent, float p, Tensor(a!) dsum, Tensor(b!) dmax, "
      "Tensor(c!) sq_total) -> ()");
}
TORCH_LIBRARY_IMPL(tm_amd, CUDA, m) {
  m.impl("label_minmax", &label_minmax);
  m.impl("contingency_dense", &contingency_dense);
  m.impl("cluster_sums", &cluster_sums);
  m.impl("cluster_dispersion", &cluster_dispersion);
}

}  // namespace tm_amd
