// Fused compute() of the streaming regression scores that are ratios of running sums: explained variance, R^2 and
// Pearson / concordance correlation.
//
// The reference reductions (regression/{explained_variance,r2,pearson,concordance}.py `_*_compute`) are 10-20 tiny
// ATen launches on [num_outputs]-sized tensors each (0.1-0.25 ms of host time per compute() on the MI355X host);
// here one block evaluates the per-output formulas, their zero-variance rules and the raw / uniform /
// variance-weighted averaging in one launch.  Arithmetic stays in the states' dtype (as the reference's eager ops),
// so the exact-zero tests (`numerator != 0`, `isclose(x, 0, atol=1e-4)`) see the same values.
#include "../common/tm_common.h"

namespace tm_amd {
namespace {

constexpr int kThreads = 256;
enum Kind : int { kExplainedVariance = 0, kR2 = 1, kPearson = 2, kConcordance = 3 };
enum MultiOut : int { kRaw = 0, kUniform = 1, kVarianceWeighted = 2 };
enum NKind : int { kNScalar = 0, kNFloat = 1, kNDouble = 2, kNLong = 3 };

template <typename T>
__device__ __forceinline__ T load_n(const void* p, int kind, int idx, double scalar) {
  switch (kind) {
    case kNFloat: return static_cast<T>(static_cast<const float*>(p)[idx]);
    case kNDouble: return static_cast<T>(static_cast<const double*>(p)[idx]);
    case kNLong: return static_cast<T>(static_cast<const int64_t*>(p)[idx]);
    default: return static_cast<T>(scalar);
  }
}

template <typename T>
__device__ __forceinline__ T block_sum(T v, T* red) {
  v = wave_sum(v);
  const int wave = threadIdx.x / kWave, lane = threadIdx.x & (kWave - 1);
  __syncthreads();
  if (lane == 0) red[wave] = v;
  __syncthreads();
  T s = 0;
  for (int w = 0; w < kThreads / kWave; ++w) s += red[w];
  return s;
}

// s0..s4: per-kind state pointers (see the host function)
template <typename T>
__global__ void __launch_bounds__(kThreads)
    regression_compute_kernel(int kind, int k, const T* __restrict__ s0, const T* __restrict__ s1,
                              const T* __restrict__ s2, const T* __restrict__ s3, const T* __restrict__ s4,
                              const void* __restrict__ n_ptr, int n_kind, int n_per_col, double n_scalar,
                              int multioutput, T bound, T* __restrict__ out) {
  __shared__ T red[kThreads / kWave];
  T num_sum = 0, w_sum = 0, wscore = 0;
  int low_var = 0;
  for (int c = threadIdx.x; c < k; c += kThreads) {
    const T n = load_n<T>(n_ptr, n_kind, n_per_col ? c : 0, n_scalar);
    T score = 0, weight = 0;
    if (kind == kExplainedVariance) {
      // s0 = sum_error, s1 = sum_squared_error, s2 = sum_target, s3 = sum_squared_target
      const T diff_avg = s0[c] / n;
      const T numer = s1[c] / n - diff_avg * diff_avg;
      const T tavg = s2[c] / n;
      const T denom = s3[c] / n - tavg * tavg;
      score = (numer != T(0) && denom != T(0)) ? T(1) - numer / denom : (numer != T(0) ? T(0) : T(1));
      weight = denom;
    } else if (kind == kR2) {
      // s0 = sum_squared_obs, s1 = sum_obs, s2 = rss; nonzero = !isclose(x, 0, atol=1e-4) (NaN counts as nonzero)
      const T mean = s1[c] / n;
      const T tss = s0[c] - s1[c] * mean;
      const T rss = s2[c];
      const bool nz_rss = !(fabs(rss) <= T(1e-4)), nz_tss = !(fabs(tss) <= T(1e-4));
      score = (nz_rss && nz_tss) ? T(1) - rss / tss : (nz_rss ? T(0) : T(1));
      weight = tss;
    } else {
      // s0 = mean_x, s1 = mean_y, s2 = m2_x, s3 = m2_y, s4 = c_xy (sums of squared deviations)
      const T vx = s2[c] / (n - T(1)), vy = s3[c] / (n - T(1)), cxy = s4[c] / (n - T(1));
      low_var |= (vx < bound || vy < bound) ? 1 : 0;
      T corr = cxy / sqrt(vx * vy);
      corr = corr != corr ? corr : fmin(fmax(corr, T(-1)), T(1));
      if (kind == kPearson) {
        score = corr;
      } else {
        const T dm = s0[c] - s1[c];
        score = T(2) * corr * sqrt(vx) * sqrt(vy) / (vx + vy + dm * dm);
      }
    }
    out[c] = score;
    num_sum += score;
    w_sum += weight;
    wscore += weight * score;
  }
  if (multioutput != kRaw) {
    num_sum = block_sum(num_sum, red);
    w_sum = block_sum(w_sum, red);
    wscore = block_sum(wscore, red);
  }
  low_var = __syncthreads_or(low_var);
  if (threadIdx.x == 0) {
    out[k + 1] = low_var ? T(1) : T(0);
    if (multioutput == kUniform) out[k] = num_sum / static_cast<T>(k);
    else if (multioutput == kVarianceWeighted) out[k] = wscore / w_sum;
  }
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

}  // namespace tm_amd

TORCH_LIBRARY_FRAGMENT(tm_amd, m) {
  m.def("regression_compute(int kind, Tensor[] states, Tensor? n, float n_value, int multioutput, float bound, "
        "Tensor(a!) out) -> ()");
}
TORCH_LIBRARY_IMPL(tm_amd, CUDA, m) { m.impl("regression_compute", &tm_amd::regression_compute); }
