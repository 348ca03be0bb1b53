// Fused compute() of the confusion-matrix family on a multiclass [C, C] int64 state: Jaccard index, Cohen's kappa
// and Matthews' correlation coefficient, plus the calibration-error bin statistics.
//
// Reference reductions (F/classification/{jaccard,cohen_kappa,matthews_corrcoef}.py `_*_reduce`) are ~10-25 ATen
// launches each, and MCC branches on `denom == 0` / degenerate 2x2 cases with host syncs: ~0.12-0.17 ms of host time
// per compute() at C = 10.  Here one block reads the matrix once (row sums, column sums, diagonal in LDS, fp64),
// evaluates the reduction including the data-dependent branches on the device, and writes [C] per-class values
// (Jaccard) plus the scalar result: one launch, no sync.
//
// Calibration (F/classification/calibration_error.py `_binning_bucketize`): bucketize + stack + index_add over
// every accumulated confidence is replaced by one pass with an LDS-privatised (count, Σconf, Σacc) histogram
// (SURVEY K7); the per-bin divisions stay a handful of [n_bins]-sized ops.
#include "common/compute_bodies.h"

namespace tm_amd {
namespace {

constexpr int kThreads = cbody::kThreads;
using cbody::kJaccard;

__global__ void __launch_bounds__(kThreads) confmat_reduce_kernel(const int64_t* __restrict__ cm, int C, int kind,
                                                                  int average, int ignore, int kw,
                                                                  float* __restrict__ out) {
  extern __shared__ double sm[];  // rows [C], cols [C], diag [C]
  __shared__ double red[kThreads / kWave];
  cbody::confmat_reduce_block(cm, C, kind, average, ignore, kw, out, sm, red);
}

// (count, Σconf, Σacc) per bin; bin = #{boundaries <= conf} - 1 (torch.bucketize(right=True) - 1); nb <= 4096
__global__ void __launch_bounds__(kThreads) calib_bins_kernel(const float* __restrict__ conf,
                                                              const float* __restrict__ acc, long long n,
                                                              const float* __restrict__ bounds, int nb,
                                                              float* __restrict__ sums, int* __restrict__ bad) {
  extern __shared__ float hs[];  // [nb][3] histogram, then [nb] boundaries
  float* bs = hs + 3 * nb;
  for (int i = threadIdx.x; i < 3 * nb; i += blockDim.x) hs[i] = 0.f;
  for (int i = threadIdx.x; i < nb; i += blockDim.x) bs[i] = bounds[i];
  __syncthreads();
  bool oob = false;
  for (long long e = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x; e < n;
       e += static_cast<long long>(gridDim.x) * blockDim.x) {
    const float x = conf[e];
    int lo = 0, hi = nb;  // first index with bounds[idx] > x
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (bs[mid] <= x) lo = mid + 1;
      else hi = mid;
    }
    const int b = x != x ? nb - 1 : lo - 1;  // NaN: past every bound, as torch.bucketize(right=True) sorts it
    if (b < 0) {  // below the first boundary: index -1, which index_add rejects in the reference
      oob = true;
      continue;
    }
    atomicAdd(&hs[3 * b], 1.f);
    atomicAdd(&hs[3 * b + 1], x);
    atomicAdd(&hs[3 * b + 2], acc[e]);
  }
  if (oob) atomicOr(bad, 1);
  __syncthreads();
  for (int i = threadIdx.x; i < 3 * nb; i += blockDim.x)
    if (hs[i] != 0.f) atomicAdd(&sums[i], hs[i]);
}

// Few-bin variant (nb <= 16, the default 15 bins): every thread owns a private (count, Σconf, Σacc) column in LDS
// (layout [3 * nb][256]: a lane's updates never collide with another lane's, no atomics), so the per-element cost is
// three plain LDS read-modify-writes instead of three same-address LDS atomics contended by the whole wave.  At the
// end each wave reduces whole rows (256 values -> 1) and adds them to the global sums with one atomic per row.
constexpr int kPrivBins = 16;

__global__ void __launch_bounds__(kThreads) calib_bins_private_kernel(const float* __restrict__ conf,
                                                                      const float* __restrict__ acc, long long n,
                                                                      const float* __restrict__ bounds, int nb,
                                                                      float* __restrict__ sums,
                                                                      int* __restrict__ bad) {
  __shared__ float hist[3 * kPrivBins * kThreads];
  __shared__ float bs[kPrivBins];
  for (int i = threadIdx.x; i < 3 * nb * kThreads; i += kThreads) hist[i] = 0.f;
  if (threadIdx.x < nb) bs[threadIdx.x] = bounds[threadIdx.x];
  __syncthreads();
  bool oob = false;
  const int t = threadIdx.x;
  for (long long e = static_cast<long long>(blockIdx.x) * kThreads + t; e < n;
       e += static_cast<long long>(gridDim.x) * kThreads) {
    const float x = conf[e];
    int b = -1;
    for (int k = 0; k < nb; ++k) b += (bs[k] <= x) ? 1 : 0;  // #{bounds <= x} - 1 (ascending bounds)
    if (x != x) b = nb - 1;  // NaN: torch.bucketize(right=True) sorts it past every bound (the reference's last bin)
    if (b < 0) {
      oob = true;
      continue;
    }
    hist[(3 * b) * kThreads + t] += 1.f;
    hist[(3 * b + 1) * kThreads + t] += x;
    hist[(3 * b + 2) * kThreads + t] += acc[e];
  }
  if (oob) atomicOr(bad, 1);
  __syncthreads();
  const int lane = t & (kWave - 1), wave = t / kWave;
  for (int row = wave; row < 3 * nb; row += kThreads / kWave) {
    const float* r = hist + row * kThreads;
    float v = r[lane] + r[lane + 64] + r[lane + 128] + r[lane + 192];
    v = wave_sum(v);
    if (lane == 0 && v != 0.f) atomicAdd(&sums[row], v);
  }
}

}  // namespace

// confmat: int64 [C, C]; kind 0 Jaccard (average 0 micro / 1 macro / 2 weighted / 3 none, ignore: class to drop or -1),
// 1 Cohen kappa (kw 0 none / 1 linear / 2 quadratic), 2 MCC.  out: f32 [C + 1] (Jaccard: per class + scalar) or [1].
void confmat_reduce(const at::Tensor& confmat, int64_t kind, int64_t average, int64_t ignore, int64_t kw,
                    at::Tensor out) {
  TM_CHECK_CUDA(confmat);
  TORCH_CHECK(confmat.scalar_type() == at::kLong && confmat.is_contiguous() && confmat.dim() == 2 &&
                  confmat.size(0) == confmat.size(1), "confmat_reduce: int64 [C, C] contiguous");
  const int C = static_cast<int>(confmat.size(0));
  TORCH_CHECK(C >= 2 && C <= 4096, "confmat_reduce: 2 <= C <= 4096");
  TORCH_CHECK(out.scalar_type() == at::kFloat && out.is_contiguous() && out.numel() >= (kind == kJaccard ? C + 1 : 1),
              "confmat_reduce: out");
  hipLaunchKernelGGL(confmat_reduce_kernel, dim3(1), dim3(kThreads), 3 * C * sizeof(double), stream(),
                     confmat.data_ptr<int64_t>(), C, static_cast<int>(kind), static_cast<int>(average),
                     static_cast<int>(ignore), static_cast<int>(kw), out.data_ptr<float>());
  C10_HIP_KERNEL_LAUNCH_CHECK();
}

// conf/acc: f32 [N]; bounds: f32 [nb] ascending; sums: f32 [nb, 3] zeroed (accumulated); bad: i32 [1] (conf below
// bounds[0]).
void calibration_bins(const at::Tensor& conf, const at::Tensor& acc, const at::Tensor& bounds, at::Tensor sums,
                      at::Tensor bad) {
  TM_CHECK_CUDA(conf);
  TORCH_CHECK(conf.scalar_type() == at::kFloat && acc.scalar_type() == at::kFloat && conf.is_contiguous() &&
                  acc.is_contiguous() && conf.numel() == acc.numel(), "calibration_bins: f32 conf / acc");
  TORCH_CHECK(bounds.scalar_type() == at::kFloat && bounds.is_contiguous(), "calibration_bins: f32 bounds");
  const int nb = static_cast<int>(bounds.numel());
  TORCH_CHECK(nb >= 1 && nb <= 4096, "calibration_bins: 1 <= bins <= 4096");
  TORCH_CHECK(sums.scalar_type() == at::kFloat && sums.numel() == 3 * nb && sums.is_contiguous(),
              "calibration_bins: sums f32 [nb, 3]");
  const long long n = conf.numel();
  if (n == 0) return;
  if (nb <= kPrivBins) {
    // ~32 elements per thread amortise the 3*nb*256-float LDS clear and row reduction per block on large inputs;
    // small ones (a per-update batch) spread over more blocks instead: one block walking 8k elements is ~26 us of
    // latency, eight blocks of 4 elements per thread finish in a few us
    const long long per = n >= (1LL << 20) ? 32 : 4;
    const int grid = grid_cap((n + kThreads * per - 1) / (kThreads * per), 1024);
    hipLaunchKernelGGL(calib_bins_private_kernel, dim3(grid), dim3(kThreads), 0, stream(), conf.data_ptr<float>(),
                       acc.data_ptr<float>(), n, bounds.data_ptr<float>(), nb, sums.data_ptr<float>(),
                       bad.data_ptr<int>());
    C10_HIP_KERNEL_LAUNCH_CHECK();
    return;
  }
  const int grid = grid_cap((n + kThreads - 1) / kThreads, 256 * 4);
  hipLaunchKernelGGL(calib_bins_kernel, dim3(grid), dim3(kThreads), 4 * nb * sizeof(float), stream(),
                     conf.data_ptr<float>(), acc.data_ptr<float>(), n, bounds.data_ptr<float>(), nb,
                     sums.data_ptr<float>(), bad.data_ptr<int>());
  C10_HIP_KERNEL_LAUNCH_CHECK();
}

// Calibration error from the [nb, 3] (count, Σconf, Σacc) bins in one block: per bin acc / conf means (0 for empty
// bins, the reference's nan_to_num), proportion = count / Σcount, then l1 = Σ |acc - conf| * prop or
// max = max |acc - conf| (reference F/classification/calibration_error.py `_ce_compute`, ~10 ATen launches).
namespace {
__global__ void __launch_bounds__(kThreads) calib_reduce_kernel(float* __restrict__ sums, int nb, int norm,
                                                                float* __restrict__ out, int clear) {
  __shared__ float red[kThreads / kWave];
  float tot = 0.f;
  for (int b = threadIdx.x; b < nb; b += blockDim.x) tot += sums[3 * b];
  tot = wave_sum(tot);
  const int wave = threadIdx.x / kWave, lane = threadIdx.x & (kWave - 1);
  if (lane == 0) red[wave] = tot;
  __syncthreads();
  tot = 0.f;
  for (int w = 0; w < kThreads / kWave; ++w) tot += red[w];
  __syncthreads();
  float v = 0.f;
  for (int b = threadIdx.x; b < nb; b += blockDim.x) {
    const float cnt = sums[3 * b];
    float conf = sums[3 * b + 1] / cnt, acc = sums[3 * b + 2] / cnt;
    conf = conf != conf ? 0.f : conf;
    acc = acc != acc ? 0.f : acc;
    const float gap = fabsf(acc - conf);
    v = norm == 0 ? v + gap * (cnt / tot) : fmaxf(v, gap);
  }
  if (norm == 0) {
    v = wave_sum(v);
  } else {
#pragma unroll
    for (int off = kWave / 2; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, kWave));
  }
  if (lane == 0) red[wave] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    float r = red[0];
    for (int w = 1; w < kThreads / kWave; ++w) r = norm == 0 ? r + red[w] : fmaxf(r, red[w]);
    out[0] = r;
  }
  if (clear) {  // self-cleaning workspace: the next calibration_bins accumulates into zeros
    __syncthreads();
    for (int i = threadIdx.x; i < 3 * nb; i += blockDim.x) sums[i] = 0.f;
  }
}
}  // namespace

// sums: f32 [nb, 3] from calibration_bins; norm 0 = l1, 1 = max; out: f32 [1]
void calibration_reduce(const at::Tensor& sums, int64_t norm, at::Tensor out) {
  TM_CHECK_CUDA(sums);
  TORCH_CHECK(sums.scalar_type() == at::kFloat && sums.is_contiguous() && sums.dim() == 2 && sums.size(1) == 3,
              "calibration_reduce: sums must be contiguous f32 [nb, 3]");
  TORCH_CHECK(norm == 0 || norm == 1, "calibration_reduce: norm 0 (l1) or 1 (max)");
  TORCH_CHECK(out.scalar_type() == at::kFloat && out.numel() >= 1, "calibration_reduce: out f32 [1]");
  hipLaunchKernelGGL(calib_reduce_kernel, dim3(1), dim3(kThreads), 0, stream(), sums.data_ptr<float>(),
                     static_cast<int>(sums.size(0)), static_cast<int>(norm), out.data_ptr<float>(), 0);
  C10_HIP_KERNEL_LAUNCH_CHECK();
}

// as calibration_reduce, then zeroes `sums` (a persistent workspace reused by the next compute())
void calibration_reduce_clear(at::Tensor sums, int64_t norm, at::Tensor out) {
  TM_CHECK_CUDA(sums);
  TORCH_CHECK(sums.scalar_type() == at::kFloat && sums.is_contiguous() && sums.dim() == 2 && sums.size(1) == 3,
              "calibration_reduce_clear: sums must be contiguous f32 [nb, 3]");
  TORCH_CHECK(norm == 0 || norm == 1, "calibration_reduce_clear: norm 0 (l1) or 1 (max)");
  TORCH_CHECK(out.scalar_type() == at::kFloat && out.numel() >= 1, "calibration_reduce_clear: out f32 [1]");
  hipLaunchKernelGGL(calib_reduce_kernel, dim3(1), dim3(kThreads), 0, stream(), sums.data_ptr<float>(),
                     static_cast<int>(sums.size(0)), static_cast<int>(norm), out.data_ptr<float>(), 1);
  C10_HIP_KERNEL_LAUNCH_CHECK();
}

}  // namespace tm_amd

TORCH_LIBRARY_FRAGMENT(tm_amd, m) {
  m.def("calibration_reduce(Tensor sums, int norm, Tensor(a!) out) -> ()");
  m.def("calibration_reduce_clear(Tensor(a!) sums, int norm, Tensor(b!) out) -> ()");
  m.def("confmat_reduce(Tensor confmat, int kind, int average, int ignore, int kw, Tensor(a!) out) -> ()");
  m.def("calibration_bins(Tensor conf, Tensor acc, Tensor bounds, Tensor(a!) sums, Tensor(b!) bad) -> ()");
}
TORCH_LIBRARY_IMPL(tm_amd, CUDA, m) {
  m.impl("confmat_reduce", &tm_amd::confmat_reduce);
  m.impl("calibration_bins", &tm_amd::calibration_bins);
  m.impl("calibration_reduce", &tm_amd::calibration_reduce);
  m.impl("calibration_reduce_clear", &tm_amd::calibration_reduce_clear);
}
