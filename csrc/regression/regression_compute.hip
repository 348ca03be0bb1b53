// Fused compute() of the streaming regression scores that are ratios of running sums: explained variance, R^2 and
// Pearson / concordance correlation.
//
// The reference reductions (regression/{explained_variance,r2,pearson,concordance}.py `_*_compute`) are 10-20 tiny
// ATen launches on [num_outputs]-sized tensors each (0.1-0.25 ms of host time per compute() on the MI355X host);
// here one block evaluates the per-output formulas, their zero-variance rules and the raw / uniform /
// variance-weighted averaging in one launch.  Arithmetic stays in the states' dtype (as the reference's eager ops),
// so the exact-zero tests (`numerator != 0`, `isclose(x, 0, atol=1e-4)`) see the same values.
#include "common/compute_bodies.h"

namespace tm_amd {
namespace {

constexpr int kThreads = cbody::kThreads;
using cbody::kExplainedVariance;
using cbody::kNDouble;
using cbody::kNFloat;
using cbody::kNLong;
using cbody::kNScalar;
using cbody::kR2;
using cbody::kRaw;
using cbody::kVarianceWeighted;

// s0..s4: per-kind state pointers (see the host function)
template <typename T>
__global__ void __launch_bounds__(kThreads)
    regression_compute_kernel(int kind, int k, const T* __restrict__ s0, const T* __restrict__ s1,
                              const T* __restrict__ s2, const T* __restrict__ s3, const T* __restrict__ s4,
                              const void* __restrict__ n_ptr, int n_kind, int n_per_col, double n_scalar,
                              int multioutput, T bound, T* __restrict__ out) {
  __shared__ T red[kThreads / kWave];
  cbody::regression_compute_block<T>(kind, k, s0, s1, s2, s3, s4, n_ptr, n_kind, n_per_col, n_scalar, multioutput,
                                     bound, out, red);
}


// Per-rank merge of the Pearson / concordance running states (reference S/regression/pearson.py:28-71, a Python loop
// over the W ranks of ~25 elementwise ops each): one thread per output column folds the W stacked rows in rank order
// with Chan et al.'s pairwise update, in fp64 (rounded once to the states' dtype at the end).
// in: [6][W][k] = mean_x, mean_y, var_x, var_y, corr_xy, n (one dtype); out: [6][k].
template <typename T>
__host__ __device__ __forceinline__ void corr_merge_col(const T* __restrict__ in, int W, long long k, long long j,
                                                        T* __restrict__ out) {
  const long long plane = static_cast<long long>(W) * k;
  double mx = in[j], my = in[plane + j], vx = in[2 * plane + j], vy = in[3 * plane + j], cxy = in[4 * plane + j],
         n = in[5 * plane + j];
  for (int w = 1; w < W; ++w) {
    const long long o = static_cast<long long>(w) * k + j;
    const double mx2 = in[o], my2 = in[plane + o], n2 = in[5 * plane + o];
    const double tot = n + n2;
    const double dx = mx2 - mx, dy = my2 - my;
    const double wt = tot != 0.0 ? n * n2 / tot : 0.0;
    vx += in[2 * plane + o] + dx * dx * wt;
    vy += in[3 * plane + o] + dy * dy * wt;
    cxy += in[4 * plane + o] + dx * dy * wt;
    if (tot != 0.0) {
      mx += dx * n2 / tot;
      my += dy * n2 / tot;
    }
    n = tot;
  }
  out[j] = static_cast<T>(mx);
  out[k + j] = static_cast<T>(my);
  out[2 * k + j] = static_cast<T>(vx);
  out[3 * k + j] = static_cast<T>(vy);
  out[4 * k + j] = static_cast<T>(cxy);
  out[5 * k + j] = static_cast<T>(n);
}

template <typename T>
__global__ void __launch_bounds__(256) corr_merge_kernel(const T* __restrict__ in, int W, long long k,
                                                         T* __restrict__ out) {
  for (long long j = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x; j < k;
       j += static_cast<long long>(gridDim.x) * blockDim.x)
    corr_merge_col(in, W, k, j, out);
}

}  // namespace

// kind 0 EV (s0..s3), 1 R2 (s0..s2), 2 Pearson / 3 concordance (s0..s4); every state is [k] in ONE dtype (f32/f64).
// n: the observation count as a tensor ([1] or [k]; f32 / f64 / i64) or, without one, the number `n_value`.
// out: [k + 2] in the states' dtype: per-output scores, the multioutput average (unset for raw), then 1 / 0 when a
// Pearson variance is / is not below `bound`.
void regression_compute(int64_t kind, at::TensorList states, const c10::optional<at::Tensor>& n, double n_value,
                        int64_t multioutput, double bound, at::Tensor out) {
  const size_t need = kind == kExplainedVariance ? 4 : kind == kR2 ? 3 : 5;
  TORCH_CHECK(kind >= 0 && kind <= 3 && states.size() == need, "regression_compute: kind ", kind, " takes ", need,
              " states");
  const at::Tensor& s0 = states[0];
  TM_CHECK_CUDA(s0);
  const int64_t k = s0.numel();
  TORCH_CHECK(k >= 1 && k <= (1 << 20), "regression_compute: 1..2^20 outputs");
  const auto dt = s0.scalar_type();
  TORCH_CHECK(dt == at::kFloat || dt == at::kDouble, "regression_compute: f32 / f64 states");
  for (const auto& s : states)
    TORCH_CHECK(s.is_cuda() && s.get_device() == s0.get_device() && s.scalar_type() == dt && s.is_contiguous() &&
                    s.numel() == k,
                "regression_compute: states must be contiguous [k] tensors of one dtype on one device");
  int n_kind = kNScalar, n_per_col = 0;
  const void* n_ptr = nullptr;
  if (n.has_value()) {
    const at::Tensor& nt = *n;
    TORCH_CHECK(nt.is_cuda() && nt.get_device() == s0.get_device() && nt.is_contiguous() &&
                    (nt.numel() == 1 || nt.numel() == k),
                "regression_compute: n must be a contiguous [1] or [k] tensor on the states' device");
    switch (nt.scalar_type()) {
      case at::kFloat: n_kind = kNFloat; break;
      case at::kDouble: n_kind = kNDouble; break;
      case at::kLong: n_kind = kNLong; break;
      default: TORCH_CHECK(false, "regression_compute: n dtype ", nt.scalar_type());
    }
    n_per_col = nt.numel() == k && k > 1 ? 1 : 0;
    n_ptr = nt.data_ptr();
  }
  TORCH_CHECK(out.is_cuda() && out.get_device() == s0.get_device() && out.scalar_type() == dt &&
                  out.numel() == k + 2 && out.is_contiguous(),
              "regression_compute: out must be a contiguous [k + 2] tensor of the states' dtype");
  const int mo = static_cast<int>(multioutput);
  TORCH_CHECK(mo >= kRaw && mo <= kVarianceWeighted, "regression_compute: multioutput");
  if (dt == at::kFloat) {
    hipLaunchKernelGGL((regression_compute_kernel<float>), dim3(1), dim3(kThreads), 0, stream(),
                       static_cast<int>(kind), static_cast<int>(k), s0.data_ptr<float>(), states[1].data_ptr<float>(),
                       states[need > 2 ? 2 : 0].data_ptr<float>(), states[need > 3 ? 3 : 0].data_ptr<float>(),
                       states[need > 4 ? 4 : 0].data_ptr<float>(), n_ptr, n_kind, n_per_col, n_value, mo,
                       static_cast<float>(bound), out.data_ptr<float>());
  } else {
    hipLaunchKernelGGL((regression_compute_kernel<double>), dim3(1), dim3(kThreads), 0, stream(),
                       static_cast<int>(kind), static_cast<int>(k), s0.data_ptr<double>(),
                       states[1].data_ptr<double>(), states[need > 2 ? 2 : 0].data_ptr<double>(),
                       states[need > 3 ? 3 : 0].data_ptr<double>(), states[need > 4 ? 4 : 0].data_ptr<double>(), n_ptr,
                       n_kind, n_per_col, n_value, mo, bound, out.data_ptr<double>());
  }
  C10_HIP_KERNEL_LAUNCH_CHECK();
}


// stacked [6, W, k] per-rank Pearson states -> merged [6, k] (ROCm: one launch; CPU: the same fold on the host)
at::Tensor corr_merge(const at::Tensor& stacked) {
  TORCH_CHECK(stacked.dim() == 3 && stacked.size(0) == 6 && stacked.is_contiguous(), "corr_merge: contiguous [6, W, k]");
  const auto dt = stacked.scalar_type();
  TORCH_CHECK(dt == at::kFloat || dt == at::kDouble, "corr_merge: f32 / f64 states");
  const int W = static_cast<int>(stacked.size(1));
  const long long k = stacked.size(2);
  TORCH_CHECK(W >= 1, "corr_merge: at least one rank");
  auto out = at::empty({6, k}, stacked.options());
  if (k == 0) return out;
  AT_DISPATCH_FLOATING_TYPES(dt, "corr_merge", [&] {
    if (stacked.is_cuda()) {
      hipLaunchKernelGGL(corr_merge_kernel<scalar_t>, dim3(grid_cap((k + 255) / 256)), dim3(256), 0, stream(),
                         stacked.data_ptr<scalar_t>(), W, k, out.data_ptr<scalar_t>());
    } else {
      for (long long j = 0; j < k; ++j) corr_merge_col(stacked.data_ptr<scalar_t>(), W, k, j, out.data_ptr<scalar_t>());
    }
  });
  if (stacked.is_cuda()) C10_HIP_KERNEL_LAUNCH_CHECK();
  return out;
}

}  // namespace tm_amd

TORCH_LIBRARY_FRAGMENT(tm_amd, m) {
  m.def("regression_compute(int kind, Tensor[] states, Tensor? n, float n_value, int multioutput, float bound, "
        "Tensor(a!) out) -> ()");
  m.def("corr_merge(Tensor stacked) -> Tensor");
}
TORCH_LIBRARY_IMPL(tm_amd, CUDA, m) {
  m.impl("regression_compute", &tm_amd::regression_compute);
  m.impl("corr_merge", &tm_amd::corr_merge);
}
TORCH_LIBRARY_IMPL(tm_amd, CPU, m) { m.impl("corr_merge", &tm_amd::corr_merge); }
