// Exact 1-D distance transforms along the last dim of a [L, n] cost array -- the separable building block of
// `functional.segmentation.distance_transform` (reference F/segmentation/utils.py:177-283: scipy ndimage EDT / CDT,
// or an all-pairs torch engine).  out[l, j] = min_k combine(|j - k| * spacing, cost[l, k]) with combine:
//
//   metric 0 (squared euclidean)  d^2 + f : Felzenszwalb-Huttenlocher lower envelope of parabolas, O(n) per line
//   metric 1 (taxicab)            d + f   : forward + backward min-plus scan, O(n) per line
//   metric 2 (chessboard)         max(d,f): monotone-deque min-max pass per direction, O(n) per line
//
// Costs are 0 on sites and +inf elsewhere on the first axis; later axes take the previous pass's output.  One thread
// per line (lines are independent, a [L, n] problem has L >> #CUs threads for images); envelope / deque scratch
// (site index, boundary) lives in global memory, read back by the same thread (L1/L2 resident).
// The same routines run on the host for CPU tensors (CPU dispatch key, at::parallel_for over lines).
#include <ATen/Parallel.h>

#include <limits>
#include <vector>

#include "../common/tm_common.h"

namespace tm_amd {
namespace {

constexpr int kEuclid = 0, kTaxicab = 1, kChessboard = 2;

template <typename T>
__host__ __device__ inline void envelope_line(const T* f, T* out, int n, T sp, int* v, T* z) {
  const T inf = std::numeric_limits<T>::infinity();
  int k = -1;
  for (int q = 0; q < n; ++q) {
    const T fq = f[q];
    if (!(fq < inf)) continue;  // not a site (inf; NaN never occurs for 0/inf masks)
    const T pq = static_cast<T>(q) * sp;
    if (k < 0) {
      k = 0;
      v[0] = q;
      z[0] = -inf;
      z[1] = inf;
      continue;
    }
    T s;
    while (true) {
      const T pv = static_cast<T>(v[k]) * sp;
      s = ((fq + pq * pq) - (f[v[k]] + pv * pv)) / (T(2) * (pq - pv));
      if (s <= z[k] && k > 0) {
        --k;
        continue;
      }
      break;
    }
    if (s <= z[k]) {  // k == 0 and the new parabola dominates the first one everywhere
      v[0] = q;
      z[0] = -inf;
      z[1] = inf;
      continue;
    }
    ++k;
    v[k] = q;
    z[k] = s;
    z[k + 1] = inf;
  }
  if (k < 0) {
    for (int q = 0; q < n; ++q) out[q] = inf;
    return;
  }
  int j = 0;
  for (int q = 0; q < n; ++q) {
    const T pq = static_cast<T>(q) * sp;
    while (z[j + 1] < pq) ++j;
    const T d = pq - static_cast<T>(v[j]) * sp;
    out[q] = d * d + f[v[j]];
  }
}

template <typename T>
__host__ __device__ inline void taxicab_line(const T* f, T* out, int n, T sp) {
  T run = std::numeric_limits<T>::infinity();
  for (int q = 0; q < n; ++q) {
    run = run + sp < f[q] ? run + sp : f[q];
    out[q] = run;
  }
  run = std::numeric_limits<T>::infinity();
  for (int q = n - 1; q >= 0; --q) {
    run = run + sp < out[q] ? run + sp : out[q];
    out[q] = run;
  }
}

// min-max transform g(j) = min_k max(|j - k| * sp, f(k)), O(n): one pass per direction over a monotone deque of
// candidate sites (front = oldest / farthest, f strictly increasing towards the back).  A new site evicts the back
// entries it dominates (f >= its f: farther and no lower); the front is popped once the next entry is no worse --
// permanently, since every distance grows by sp per step.  The costs along the deque are max(decreasing distance,
// increasing f), i.e. unimodal, so the surviving front is the minimum.  g = min(left pass, right pass).
template <typename T>
__host__ __device__ inline void chessboard_line(const T* f, T* out, int n, T sp, int* dq) {
  const T inf = std::numeric_limits<T>::infinity();
  for (int dir = 0; dir < 2; ++dir) {
    int head = 0, tail = 0;  // deque dq[head, tail)
    for (int step = 0; step < n; ++step) {
      const int j = dir == 0 ? step : n - 1 - step;
      const T fj = f[j];
      if (fj < inf) {
        while (tail > head && f[dq[tail - 1]] >= fj) --tail;
        dq[tail++] = j;
      }
      auto cost = [&](int k) {
        const T d = static_cast<T>(j > k ? j - k : k - j) * sp;
        return d > f[k] ? d : f[k];
      };
      while (tail - head >= 2 && cost(dq[head]) >= cost(dq[head + 1])) ++head;
      const T c = tail > head ? cost(dq[head]) : inf;
      out[j] = dir == 0 ? c : (c < out[j] ? c : out[j]);
    }
  }
}

template <typename T>
__global__ void __launch_bounds__(256) line_kernel(const T* __restrict__ cost, T* __restrict__ out, long long lines,
                                                  int n, T sp, int metric, int* __restrict__ vbuf,
                                                  T* __restrict__ zbuf) {
  const long long l = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x;
  if (l >= lines) return;
  const T* f = cost + l * n;
  T* o = out + l * n;
  if (metric == kEuclid) envelope_line(f, o, n, sp, vbuf + l * n, zbuf + l * (n + 1));
  else if (metric == kChessboard) chessboard_line(f, o, n, sp, vbuf + l * n);
  else taxicab_line(f, o, n, sp);
}

void check_args(const at::Tensor& cost, int64_t metric) {
  TORCH_CHECK(cost.dim() == 2 && cost.is_contiguous(), "line_distance_transform: cost must be a contiguous [L, n]");
  TORCH_CHECK(cost.scalar_type() == at::kFloat || cost.scalar_type() == at::kDouble,
              "line_distance_transform: f32 / f64 cost");
  TORCH_CHECK(metric >= 0 && metric <= 2, "line_distance_transform: metric 0 euclidean^2, 1 taxicab, 2 chessboard");
  TORCH_CHECK(cost.size(1) < (1LL << 30), "line_distance_transform: line too long");
}

}  // namespace

at::Tensor line_distance_transform(const at::Tensor& cost, double spacing, int64_t metric) {
  TM_CHECK_CUDA(cost);
  check_args(cost, metric);
  at::Tensor out = at::empty_like(cost);
  const long long lines = cost.size(0);
  const int n = static_cast<int>(cost.size(1));
  if (lines == 0 || n == 0) return out;
  auto s = stream();
  AT_DISPATCH_FLOATING_TYPES(cost.scalar_type(), "line_distance_transform", [&] {
    const scalar_t sp = static_cast<scalar_t>(spacing);
    at::Tensor vbuf, zbuf;
    if (metric != kTaxicab) vbuf = at::empty({lines * n}, cost.options().dtype(at::kInt));
    if (metric == kEuclid) zbuf = at::empty({lines * (n + 1)}, cost.options());
    hipLaunchKernelGGL((line_kernel<scalar_t>), dim3((lines + 255) / 256), dim3(256), 0, s, cost.data_ptr<scalar_t>(),
                       out.data_ptr<scalar_t>(), lines, n, sp, static_cast<int>(metric),
                       metric != kTaxicab ? vbuf.data_ptr<int>() : nullptr,
                       metric == kEuclid ? zbuf.data_ptr<scalar_t>() : nullptr);
  });
  C10_HIP_KERNEL_LAUNCH_CHECK();
  return out;
}

at::Tensor line_distance_transform_cpu(const at::Tensor& cost, double spacing, int64_t metric) {
  check_args(cost, metric);
  at::Tensor out = at::empty_like(cost);
  const int64_t lines = cost.size(0);
  const int n = static_cast<int>(cost.size(1));
  if (lines == 0 || n == 0) return out;
  AT_DISPATCH_FLOATING_TYPES(cost.scalar_type(), "line_distance_transform_cpu", [&] {
    const scalar_t sp = static_cast<scalar_t>(spacing);
    const scalar_t* c = cost.data_ptr<scalar_t>();
    scalar_t* o = out.data_ptr<scalar_t>();
    at::parallel_for(0, lines, 16, [&](int64_t lo, int64_t hi) {
      std::vector<int> v(metric != kTaxicab ? n : 0);
      std::vector<scalar_t> z(metric == kEuclid ? n + 1 : 0);
      for (int64_t l = lo; l < hi; ++l) {
        const scalar_t* f = c + l * n;
        scalar_t* ol = o + l * n;
        if (metric == kEuclid) envelope_line(f, ol, n, sp, v.data(), z.data());
        else if (metric == kTaxicab) taxicab_line(f, ol, n, sp);
        else chessboard_line(f, ol, n, sp, v.data());
      }
    });
  });
  return out;
}

}  // namespace tm_amd

TORCH_LIBRARY_FRAGMENT(tm_amd, m) {
  m.def("line_distance_transform(Tensor cost, float spacing, int metric) -> Tensor");
}
TORCH_LIBRARY_IMPL(tm_amd, CUDA, m) { m.impl("line_distance_transform", &tm_amd::line_distance_transform); }
TORCH_LIBRARY_IMPL(tm_amd, CPU, m) { m.impl("line_distance_transform", &tm_amd::line_distance_transform_cpu); }
