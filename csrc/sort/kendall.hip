// Kendall rank correlation statistics in O(n log n) per column (gfx950): radix sorts + merge-path inversion count.
//
// Reference behaviour: F/regression/kendall.py:61-85 compares all pairs (a Python loop over i building n x n sign
// products) and counts ties with torch.unique per column.  Knight's algorithm instead:
//   1. rocPRIM radix sort of the order-preserving y keys, then a stable radix sort of the x keys carrying y:
//      the y sequence is now ordered lexicographically by (x, y);
//   2. discordant pairs = strict inversions of that y sequence, counted by a bottom-up merge sort: one launch per
//      level, each element finds its merged position by binary search in the sibling run (merge path), elements of
//      the right run add the number of strictly greater left elements; 64-bit integer atomics (order independent);
//   3. tie statistics (sum of t(t-1)/2, t(t-1)(t-2), t(t-1)(2t+5) over tie groups of x, of y, and of (x, y) pairs,
//      plus the distinct counts for tau-c) from one binary-search pass over the sorted keys: the first element of
//      every tie group contributes its group's terms exactly, in integer arithmetic.
// Output per column (fp64): [discordant, tx, tx1, tx2, ty, ty1, ty2, txy, ux, uy].
#include "sort/sortscan.h"

namespace tm_amd {
namespace {

using sortscan::desc_key32;
using sortscan::desc_key64;

template <typename scalar_t>
__global__ void asc_keys_kernel(const scalar_t* __restrict__ x, int64_t n, int64_t stride, uint64_t* __restrict__ kx,
                                int32_t* __restrict__ idx) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    if constexpr (std::is_same<scalar_t, double>::value) kx[i] = ~desc_key64(x[i * stride]);
    else kx[i] = ~desc_key64(static_cast<double>(to_f32(x[i * stride])));
    if (idx) idx[i] = static_cast<int32_t>(i);
  }
}

__global__ void gather_u64_kernel(const uint64_t* __restrict__ src, const int32_t* __restrict__ idx, int64_t n,
                                  uint64_t* __restrict__ dst) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = src[idx[i]];
}

__device__ __forceinline__ int64_t lower_bound_u64(const uint64_t* a, int64_t len, uint64_t v) {
  int64_t lo = 0, hi = len;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (a[mid] < v) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

__device__ __forceinline__ int64_t upper_bound_u64(const uint64_t* a, int64_t len, uint64_t v) {
  int64_t lo = 0, hi = len;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (a[mid] <= v) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

__device__ __forceinline__ void block_add_u64(unsigned long long v, unsigned long long* dst) {
  __shared__ unsigned long long red[256 / kWave];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
  const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
  if (lane == 0) red[wave] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long t = 0;
    for (int w = 0; w < static_cast<int>(blockDim.x) / kWave; ++w) t += red[w];
    if (t) atomicAdd(dst, t);
  }
  __syncthreads();  // red is reused by the next call
}

// one merge level of width w: runs [base, base + w) and [base + w, base + 2w) -> out
__global__ __launch_bounds__(256) void merge_level_kernel(const uint64_t* __restrict__ in, uint64_t* __restrict__ out,
                                                          int64_t n, int64_t w, unsigned long long* __restrict__ disc) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  unsigned long long cnt = 0;
  if (i < n) {
    const int64_t base = (i / (2 * w)) * (2 * w);
    const int64_t lo_len = min(w, n - base);
    const int64_t hi_start = base + w;
    const int64_t hi_len = hi_start < n ? min(w, n - hi_start) : 0;
    const uint64_t v = in[i];
    if (i < hi_start) {
      const int64_t r = hi_len ? lower_bound_u64(in + hi_start, hi_len, v) : 0;
      out[base + (i - base) + r] = v;
    } else {
      const int64_t r = upper_bound_u64(in + base, lo_len, v);
      out[base + (i - hi_start) + r] = v;
      cnt = static_cast<unsigned long long>(lo_len - r);
    }
  }
  block_add_u64(cnt, disc);
}

// tie terms: the first element of every tie group adds t(t-1)/2, t(t-1)(t-2), t(t-1)(2t+5) and 1 (distinct count)
// acc layout (u64): [t2, t3, t5, distinct]
__global__ __launch_bounds__(256) void tie_terms_kernel(const uint64_t* __restrict__ s, int64_t n,
                                                        unsigned long long* __restrict__ acc) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  unsigned long long a = 0, b = 0, c = 0, d = 0;
  if (i < n && (i == 0 || s[i - 1] != s[i])) {
    const unsigned long long t = static_cast<unsigned long long>(upper_bound_u64(s, n, s[i]) - i);
    a = t * (t - 1) / 2;
    b = t * (t - 1) * (t >= 2 ? t - 2 : 0);
    c = t * (t - 1) * (2 * t + 5);
    d = 1;
  }
  block_add_u64(a, acc + 0);
  block_add_u64(b, acc + 1);
  block_add_u64(c, acc + 2);
  block_add_u64(d, acc + 3);
}

// joint (x, y) ties: with both sequences in (x, y) order, groups of equal pairs are contiguous
__global__ __launch_bounds__(256) void joint_ties_kernel(const uint64_t* __restrict__ xs, const uint64_t* __restrict__ ys,
                                                         int64_t n, unsigned long long* __restrict__ acc) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  unsigned long long a = 0;
  if (i < n && (i == 0 || xs[i - 1] != xs[i] || ys[i - 1] != ys[i])) {
    // inside the x group [i, xend) the y keys ascend: the pair group ends at the first larger y
    const int64_t xend = upper_bound_u64(xs, n, xs[i]);
    const int64_t yend = i + upper_bound_u64(ys + i, xend - i, ys[i]);
    const unsigned long long t = static_cast<unsigned long long>(yend - i);
    a = t * (t - 1) / 2;
  }
  block_add_u64(a, acc);
}

}  // namespace

// x, y: [n, k] (any strides); returns fp64 [k, 10] = [disc, tx, tx1, tx2, ty, ty1, ty2, txy, ux, uy]
at::Tensor kendall_stats(const at::Tensor& x, const at::Tensor& y) {
  TM_CHECK_CUDA(x);
  TM_SAME_DEVICE(x, y);
  TORCH_CHECK(x.dim() == 2 && x.sizes() == y.sizes(), "kendall_stats: x, y must be [n, k] of equal shape");
  const int64_t n = x.size(0), k = x.size(1);
  TORCH_CHECK(n < (1LL << 31), "kendall_stats: n < 2^31");
  const auto dev = x.device();
  auto st = stream();
  auto i64 = at::TensorOptions().dtype(at::kLong).device(dev);
  auto i32 = at::TensorOptions().dtype(at::kInt).device(dev);
  auto acc = at::zeros({k, 16}, i64);
  auto* accp = reinterpret_cast<unsigned long long*>(acc.data_ptr());
  if (n == 0) return at::zeros({k, 10}, at::TensorOptions().dtype(at::kDouble).device(dev));
  auto kx = at::empty({n}, i64), ky = at::empty({n}, i64), t1 = at::empty({n}, i64), t2 = at::empty({n}, i64),
       t3 = at::empty({n}, i64);
  auto ia = at::empty({n}, i32), ib = at::empty({n}, i32);
  auto u = [](const at::Tensor& t) { return reinterpret_cast<uint64_t*>(t.data_ptr()); };
  const int grid = grid_cap((n + 255) / 256);
  const int full = static_cast<int>((n + 255) / 256);
  for (int64_t c = 0; c < k; ++c) {
    unsigned long long* a = accp + c * 16;
    TM_DISPATCH_FLOAT(x.scalar_type(), "kendall_stats", [&] {
      hipLaunchKernelGGL((asc_keys_kernel<scalar_t>), dim3(grid), dim3(256), 0, st, x.data_ptr<scalar_t>() + c * x.stride(1), n,
                         x.stride(0), u(kx), static_cast<int32_t*>(nullptr));
      hipLaunchKernelGGL((asc_keys_kernel<scalar_t>), dim3(grid), dim3(256), 0, st, y.data_ptr<scalar_t>() + c * y.stride(1), n,
                         y.stride(0), u(ky), ia.data_ptr<int32_t>());
    });
    // y order: t1 = sorted y keys, ib = permutation
    sortscan::sort_pairs<uint64_t, int32_t>(u(ky), u(t1), ia.data_ptr<int32_t>(), ib.data_ptr<int32_t>(), n, 0, 64,
                                            dev, st);
    hipLaunchKernelGGL(tie_terms_kernel, dim3(full), dim3(256), 0, st, u(t1), n, a + 4);  // ty, ty1, ty2, uy
    // x keys in y order (ky reused), then stable sort by x carrying y: t2 = xs, t3 = ys in (x, y) order
    hipLaunchKernelGGL(gather_u64_kernel, dim3(grid), dim3(256), 0, st, u(kx), ib.data_ptr<int32_t>(), n, u(ky));
    sortscan::sort_pairs<uint64_t, uint64_t>(u(ky), u(t2), u(t1), u(t3), n, 0, 64, dev, st);
    hipLaunchKernelGGL(tie_terms_kernel, dim3(full), dim3(256), 0, st, u(t2), n, a + 0);  // tx, tx1, tx2, ux
    hipLaunchKernelGGL(joint_ties_kernel, dim3(full), dim3(256), 0, st, u(t2), u(t3), n, a + 8);
    // inversions of t3 (ping-pong t3 <-> t1)
    uint64_t* src = u(t3);
    uint64_t* dst = u(t1);
    for (int64_t w = 1; w < n; w <<= 1) {
      hipLaunchKernelGGL(merge_level_kernel, dim3(full), dim3(256), 0, st, src, dst, n, w, a + 9);
      std::swap(src, dst);
    }
  }
  C10_HIP_KERNEL_LAUNCH_CHECK();
  auto d = acc.to(at::kDouble);
  // [disc, tx, tx1, tx2, ty, ty1, ty2, txy, ux, uy]
  return at::stack({d.select(1, 9), d.select(1, 0), d.select(1, 1), d.select(1, 2), d.select(1, 4), d.select(1, 5),
                    d.select(1, 6), d.select(1, 8), d.select(1, 3), d.select(1, 7)}, 1);
}

}  // namespace tm_amd

TORCH_LIBRARY_FRAGMENT(tm_amd, m) { m.def("kendall_stats(Tensor x, Tensor y) -> Tensor"); }
TORCH_LIBRARY_IMPL(tm_amd, CUDA, m) { m.impl("kendall_stats", &tm_amd::kendall_stats); }
