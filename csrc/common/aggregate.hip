// Aggregator updates (Sum / Mean / Max / Min metrics) in ONE launch (K35 in SURVEY.md §2.5).
//
// Reference (S/aggregation.py:75-105 + the update bodies at :170-560): isnan(x), isnan(w), `nans.any()` (a host
// sync on every update), a boolean-mask compaction `x[~nans]` / `w[~nans]` (a second sync for the output size),
// ones_like(x) for the weights, then `(x * w).sum()` / `w.sum()` / `max()` / `min()` and the state add: ~8-10
// launches and two host round trips per update, for what is usually a single loss scalar.
// Here one grid-stride pass applies the nan strategy per element (error: validation bit; ignore / warn: the element
// drops out, and 'warn' raises a warning bit that compute() turns into the reference's UserWarning -- no per-update
// host sync; float: x and w imputed, as the reference does) and reduces sum(x*w), sum(w), max and min in fp64; the
// per-block partials are folded in a fixed order -- deterministic whatever the block completion order -- and added
// into the metric's state tensors in place: by the single block itself up to 64 Ki elements (one launch), else by a
// one-block fold launch (a last-block ticket with a grid-wide fence per block ran at ~1 TB/s).  A python-number weight
// is a kernel argument (no H2D copy of a ones tensor); a tensor weight may be one element (broadcast) or N.
#include "common/tm_common.h"

namespace tm_amd {
namespace {

constexpr int kBlock = 256;
constexpr int kMaxBlocks = 2048;
enum Kind : int { kSum = 0, kMean = 1, kMax = 2, kMin = 3 };
enum NanMode : int { kNanError = 0, kNanIgnore = 1, kNanImpute = 2, kNanWarn = 3 };

template <typename T>
__device__ __forceinline__ double to_f64(T v) {
  return static_cast<double>(to_f32(v));
}
template <>
__device__ __forceinline__ double to_f64<double>(double v) {
  return v;
}

__device__ __forceinline__ double nan_max(double a, double b) { return (a != a || a > b) ? a : b; }
__device__ __forceinline__ double nan_min(double a, double b) { return (a != a || a < b) ? a : b; }

// validation bits + the in-place state fold of one call's totals (one thread)
template <typename out_t>
__device__ void apply_fold(double sxw, double sw, double mx, double mn, int nan_total, long long N, int kind,
                           int nan_mode, int* __restrict__ ctl, out_t* __restrict__ s0, out_t* __restrict__ s1,
                           int* __restrict__ flag) {
  if (nan_mode == kNanError && nan_total) raise_flag(flag, kErrValueNan);
  if (nan_mode == kNanWarn && nan_total) raise_flag(flag, kErrValueNanWarn);  // warned at compute(), no sync here
  const bool any_kept = N - (nan_mode == kNanImpute ? 0 : nan_total) > 0;
  switch (kind) {
    case kSum:
      *s0 = static_cast<out_t>(static_cast<double>(*s0) + sxw);
      break;
    case kMean:
      *s0 = static_cast<out_t>(static_cast<double>(*s0) + sxw);
      *s1 = static_cast<out_t>(static_cast<double>(*s1) + sw);
      break;
    case kMax:
      if (any_kept) *s0 = static_cast<out_t>(nan_max(static_cast<double>(*s0), mx));
      break;
    default:
      if (any_kept) *s0 = static_cast<out_t>(nan_min(static_cast<double>(*s0), mn));
      break;
  }
  ctl[1] = nan_total;  // this call's NaN count
}

// part: f64 [kMaxBlocks][5] (sum x*w, sum w, max, min, NaN count); ctl: i32 [2] = {unused, NaN count of the last call}
// WMODE: 0 python-number weight (wconst), 1 one-element weight tensor, 2 one weight per element -- a template
// parameter so the unrolled loop below issues its loads back to back (a runtime select split them with waits)
template <typename x_t, typename w_t, typename out_t, int WMODE>
__global__ void __launch_bounds__(kBlock) agg_update_kernel(const x_t* __restrict__ x, const w_t* __restrict__ w,
                                                            long long N, long long w_n, double wconst, bool vec, int kind,
                                                            int nan_mode, double impute, double* __restrict__ part,
                                                            int* __restrict__ ctl, out_t* __restrict__ s0,
                                                            out_t* __restrict__ s1, int* __restrict__ flag) {
  __shared__ double red[4][kBlock / kWave];
  __shared__ int red_nan[kBlock / kWave];
  double s = 0.0, sw = 0.0, mx = -INFINITY, mn = INFINITY;
  int nan = 0;
  const bool impute_nan = nan_mode == kNanImpute;
  // branch-free element step: ignore / warn / error drop a NaN element (error only raises the bit), impute replaces
  auto step = [&](double xv, double wv) {
    const bool isn = xv != xv || wv != wv;
    nan += isn;
    if (impute_nan) {
      xv = isn ? impute : xv;
      wv = isn ? impute : wv;
    }
    const bool keep = impute_nan || !isn;
    s += keep ? xv * wv : 0.0;
    sw += keep ? wv : 0.0;
    mx = keep ? nan_max(mx, xv) : mx;
    mn = keep ? nan_min(mn, xv) : mn;
  };
  const long long stride = static_cast<long long>(gridDim.x) * kBlock;
  const long long tid = static_cast<long long>(blockIdx.x) * kBlock + threadIdx.x;
  const double wfix = WMODE == 0 ? wconst : (WMODE == 1 ? to_f64(w[0]) : 0.0);
  long long i = tid;
  if constexpr (std::is_same<x_t, float>::value && WMODE != 2) {
    if (vec) {
      // f32 values with a shared weight: 16-byte loads, 4 in flight per lane (64 B) -- 4-byte loads left HBM idle
      const u32x4* x4 = reinterpret_cast<const u32x4*>(x);
      const long long n4 = N / 4;
      long long j = tid;
      for (; j + 3 * stride < n4; j += 4 * stride) {
        u32x4 b[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) b[k] = __builtin_nontemporal_load(x4 + j + k * stride);
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
          for (int e = 0; e < 4; ++e) step(static_cast<double>(__uint_as_float(b[k][e])), wfix);
      }
      for (; j < n4; j += stride) {
        const u32x4 b = __builtin_nontemporal_load(x4 + j);
#pragma unroll
        for (int e = 0; e < 4; ++e) step(static_cast<double>(__uint_as_float(b[e])), wfix);
      }
      i = 4 * n4 + tid;  // the < 4 element tail
    }
  }
  // 4 independent loads in flight per thread before any use (the loop is latency-bound, not ALU-bound)
  for (; i + 3 * stride < N; i += 4 * stride) {
    double xv[4], wv[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) xv[k] = to_f64(x[i + k * stride]);
    if constexpr (WMODE == 2) {
#pragma unroll
      for (int k = 0; k < 4; ++k) wv[k] = to_f64(w[i + k * stride]);
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) wv[k] = wfix;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) step(xv[k], wv[k]);
  }
  for (; i < N; i += stride) step(to_f64(x[i]), WMODE == 2 ? to_f64(w[i]) : wfix);
  s = wave_sum(s);
  sw = wave_sum(sw);
  nan = static_cast<int>(wave_sum_ll(nan));
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    mx = nan_max(mx, __shfl_xor(mx, off, kWave));
    mn = nan_min(mn, __shfl_xor(mn, off, kWave));
  }
  const int wv_id = threadIdx.x / kWave;
  if ((threadIdx.x & (kWave - 1)) == 0) {
    red[0][wv_id] = s;
    red[1][wv_id] = sw;
    red[2][wv_id] = mx;
    red[3][wv_id] = mn;
    red_nan[wv_id] = nan;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double a = 0.0, b = 0.0, c = -INFINITY, d = INFINITY;
    int n = 0;
    for (int k = 0; k < kBlock / kWave; ++k) {
      a += red[0][k];
      b += red[1][k];
      c = nan_max(c, red[2][k]);
      d = nan_min(d, red[3][k]);
      n += red_nan[k];
    }
    if (gridDim.x == 1) {  // small inputs: one block, folded right here (one launch per update)
      apply_fold<out_t>(a, b, c, d, n, N, kind, nan_mode, ctl, s0, s1, flag);
      return;
    }
    double* p = part + 5 * blockIdx.x;
    p[0] = a;
    p[1] = b;
    p[2] = c;
    p[3] = d;
    p[4] = static_cast<double>(n);
  }
}

// multi-block inputs: one block folds the G partials in a fixed order (thread t takes blocks t, t + 256, ...; wave
// trees; LDS) -- deterministic, and no grid-wide fence / ticket in the streaming kernel
template <typename out_t>
__global__ void __launch_bounds__(kBlock) agg_fold_kernel(const double* __restrict__ part, int G, long long N,
                                                          int kind, int nan_mode, int* __restrict__ ctl,
                                                          out_t* __restrict__ s0, out_t* __restrict__ s1,
                                                          int* __restrict__ flag) {
  __shared__ double red[4][kBlock / kWave];
  __shared__ double red_nan[kBlock / kWave];
  double a = 0.0, b = 0.0, c = -INFINITY, d = INFINITY, e = 0.0;
  for (int k = threadIdx.x; k < G; k += kBlock) {
    const double* p = part + 5 * k;
    a += p[0];
    b += p[1];
    c = nan_max(c, p[2]);
    d = nan_min(d, p[3]);
    e += p[4];
  }
  a = wave_sum(a);
  b = wave_sum(b);
  e = wave_sum(e);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    c = nan_max(c, __shfl_xor(c, off, kWave));
    d = nan_min(d, __shfl_xor(d, off, kWave));
  }
  const int w = threadIdx.x / kWave;
  if ((threadIdx.x & (kWave - 1)) == 0) {
    red[0][w] = a;
    red[1][w] = b;
    red[2][w] = c;
    red[3][w] = d;
    red_nan[w] = e;
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  for (int k = 1; k < kBlock / kWave; ++k) {
    red[0][0] += red[0][k];
    red[1][0] += red[1][k];
    red[2][0] = nan_max(red[2][0], red[2][k]);
    red[3][0] = nan_min(red[3][0], red[3][k]);
    red_nan[0] += red_nan[k];
  }
  apply_fold<out_t>(red[0][0], red[1][0], red[2][0], red[3][0], static_cast<int>(red_nan[0]), N, kind, nan_mode, ctl,
                    s0, s1, flag);
}

}  // namespace

// x: ROCm float tensor [N] (contiguous); w: empty (use wconst), [1] or [N] float; kind 0 sum / 1 mean / 2 max /
// 3 min; nan_mode 0 error / 1 ignore / 2 impute / 3 warn (ignore + warning bit); part: f64 [>= 5 * 2048]; ctl: i32 [2] (ctl[0] == 0 on
// entry); s0 (and s1 for mean): f32 / f64 0-d state tensors updated in place; flag: i32 validation word.
void agg_update(const at::Tensor& x, const at::Tensor& w, double wconst, int64_t kind, int64_t nan_mode,
                double impute, at::Tensor part, at::Tensor ctl, at::Tensor s0, at::Tensor s1, at::Tensor flag) {
  TM_CHECK_CUDA(x);
  for (const at::Tensor* t : std::initializer_list<const at::Tensor*>{&part, &ctl, &s0, &s1, &flag})
    TM_SAME_DEVICE(x, (*t));
  TM_CHECK_CONTIG(x);
  TORCH_CHECK(kind >= 0 && kind <= 3, "agg_update: bad kind");
  TORCH_CHECK(nan_mode >= 0 && nan_mode <= 3, "agg_update: bad nan_mode");
  const long long N = x.numel();
  const long long w_n = w.numel();
  TORCH_CHECK(w_n == 0 || w_n == 1 || w_n == N, "agg_update: weight must have 0, 1 or N elements");
  if (w_n) {
    TM_SAME_DEVICE(x, w);
    TM_CHECK_CONTIG(w);
  }
  TORCH_CHECK(part.scalar_type() == at::kDouble && part.numel() >= 5 * kMaxBlocks && part.is_contiguous(),
              "agg_update: part workspace");
  TORCH_CHECK(ctl.scalar_type() == at::kInt && ctl.numel() >= 2, "agg_update: ctl workspace");
  TORCH_CHECK(s0.scalar_type() == at::kFloat || s0.scalar_type() == at::kDouble, "agg_update: state dtype");
  TORCH_CHECK(s0.numel() == 1 && s1.numel() == 1 && s1.scalar_type() == s0.scalar_type(), "agg_update: states");
  TORCH_CHECK(flag.scalar_type() == at::kInt && flag.numel() >= 1, "agg_update: flag");
  auto s = stream();
  if (N == 0) return;
  const bool vec = reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0;
  // one block (folded in the same launch) up to 64 Ki elements; above, up to 4 blocks (16 waves) per CU and one
  // 1-block fold launch
  const int blocks = N <= 65536 ? 1
                                : grid_cap((N + 4 * kBlock - 1) / (4 * kBlock),
                                           std::min(kMaxBlocks, 4 * cu_count(x.get_device())));
  TM_DISPATCH_FLOAT(x.scalar_type(), "agg_update", [&] {
    using x_t = scalar_t;
    const at::ScalarType wt = w_n ? w.scalar_type() : x.scalar_type();
    TM_DISPATCH_FLOAT(wt, "agg_update", [&] {
      using w_t = scalar_t;
      const w_t* wp = w_n ? reinterpret_cast<const w_t*>(w.data_ptr()) : nullptr;
      const x_t* xp = reinterpret_cast<const x_t*>(x.data_ptr());
      auto launch = [&](auto out_tag, auto wmode) {
        using out_t = decltype(out_tag);
        hipLaunchKernelGGL((agg_update_kernel<x_t, w_t, out_t, decltype(wmode)::value>), dim3(blocks), dim3(kBlock), 0,
                           s, xp, wp, N, w_n, wconst, vec, static_cast<int>(kind), static_cast<int>(nan_mode), impute,
                           part.data_ptr<double>(), ctl.data_ptr<int>(), reinterpret_cast<out_t*>(s0.data_ptr()),
                           reinterpret_cast<out_t*>(s1.data_ptr()), flag.data_ptr<int>());
      };
      auto by_w = [&](auto out_tag) {
        if (w_n == 0)
          launch(out_tag, std::integral_constant<int, 0>{});
        else if (w_n == 1)
          launch(out_tag, std::integral_constant<int, 1>{});
        else
          launch(out_tag, std::integral_constant<int, 2>{});
      };
      if (s0.scalar_type() == at::kFloat)
        by_w(float{});
      else
        by_w(double{});
      if (blocks > 1) {
        if (s0.scalar_type() == at::kFloat)
          hipLaunchKernelGGL(agg_fold_kernel<float>, dim3(1), dim3(kBlock), 0, s, part.data_ptr<double>(), blocks, N,
                             static_cast<int>(kind), static_cast<int>(nan_mode), ctl.data_ptr<int>(),
                             s0.data_ptr<float>(), s1.data_ptr<float>(), flag.data_ptr<int>());
        else
          hipLaunchKernelGGL(agg_fold_kernel<double>, dim3(1), dim3(kBlock), 0, s, part.data_ptr<double>(), blocks,
                             N, static_cast<int>(kind), static_cast<int>(nan_mode), ctl.data_ptr<int>(),
                             s0.data_ptr<double>(), s1.data_ptr<double>(), flag.data_ptr<int>());
      }
    });
  });
  C10_HIP_KERNEL_LAUNCH_CHECK();
}

TORCH_LIBRARY_FRAGMENT(tm_amd, m) {
  m.def(
      "agg_update(Tensor x, Tensor w, float wconst, int kind, int nan_mode, float impute, Tensor(a!) part, "
      "Tensor(b!) ctl, Tensor(c!) s0, Tensor(d!) s1, Tensor(e!) flag) -> ()");
}
TORCH_LIBRARY_IMPL(tm_amd, CUDA, m) { m.impl("agg_update", &agg_update); }

}  // namespace tm_amd
