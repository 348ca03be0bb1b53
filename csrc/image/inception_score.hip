// Inception Score from the accumulated logits in three launches (K18 in SURVEY.md §2.5).
//
// Reference (S/image/inception.py:152-170): permute the [N, C] logits, full softmax and log_softmax copies
// ([N, C] each), then per split a column mean, a log, an elementwise product and two reductions, exp, stack, mean/std
// -- ~6 launches per split plus two [N, C] temporaries.  Here:
//   1. one wave per (permuted) row: logsumexp, then the row's probabilities added to its split's column sums (fp64);
//   2. one wave per row: KL(p_i || m_split) = sum_j p_ij (log p_ij - log m_j), summed per split (fp64);
//   3. one block: exp(mean KL) per split, their mean and unbiased std.
// The permutation is applied by indexing (no permuted copy); split s = rows [s*chunk, (s+1)*chunk) of the permuted
// order, as torch.chunk does.
#include "common/tm_common.h"

namespace tm_amd {
namespace {

constexpr int kBlock = 256;

template <typename T>
__device__ __forceinline__ float lse_row(const T* r, int C) {
  const int lane = threadIdx.x & (kWave - 1);
  float m = -INFINITY;
  for (int j = lane; j < C; j += kWave) m = fmaxf(m, to_f32(r[j]));
#pragma unroll
  for (int off = kWave / 2; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off, kWave));
  float s = 0.f;
  for (int j = lane; j < C; j += kWave) s += expf(to_f32(r[j]) - m);
  s = wave_sum(s);
  return m + logf(s);
}

template <typename T>
__global__ void __launch_bounds__(kBlock) is_colsum_kernel(const T* __restrict__ x, const int64_t* __restrict__ perm,
                                                           long long N, int C, long long chunk,
                                                           float* __restrict__ lse, double* __restrict__ colsum) {
  const long long nw = static_cast<long long>(gridDim.x) * (kBlock / kWave);
  const int lane = threadIdx.x & (kWave - 1);
  for (long long k = (static_cast<long long>(blockIdx.x) * kBlock + threadIdx.x) / kWave; k < N; k += nw) {
    const T* r = x + perm[k] * static_cast<long long>(C);
    const float l = lse_row(r, C);
    if (lane == 0) lse[k] = l;
    double* cs = colsum + (k / chunk) * static_cast<long long>(C);
    for (int j = lane; j < C; j += kWave) atomicAdd(cs + j, static_cast<double>(expf(to_f32(r[j]) - l)));
  }
}

template <typename T>
__global__ void __launch_bounds__(kBlock) is_kl_kernel(const T* __restrict__ x, const int64_t* __restrict__ perm,
                                                       long long N, int C, long long chunk,
                                                       const float* __restrict__ lse,
                                                       const double* __restrict__ colsum,
                                                       double* __restrict__ kl_sum) {
  const long long nw = static_cast<long long>(gridDim.x) * (kBlock / kWave);
  const int lane = threadIdx.x & (kWave - 1);
  for (long long k = (static_cast<long long>(blockIdx.x) * kBlock + threadIdx.x) / kWave; k < N; k += nw) {
    const T* r = x + perm[k] * static_cast<long long>(C);
    const long long s = k / chunk;
    const long long n_s = (s + 1) * chunk < N ? chunk : N - s * chunk;
    const double* cs = colsum + s * static_cast<long long>(C);
    const float l = lse[k];
    double acc = 0.0;
    for (int j = lane; j < C; j += kWave) {
      const float lp = to_f32(r[j]) - l;
      const double m = cs[j] / static_cast<double>(n_s);
      acc += static_cast<double>(expf(lp)) * (static_cast<double>(lp) - log(m));
    }
    acc = wave_sum(acc);
    if (lane == 0) atomicAdd(kl_sum + s, acc);
  }
}

__global__ void is_finalize_kernel(const double* __restrict__ kl_sum, long long N, long long chunk, int nsplit,
                                   float* __restrict__ out) {
  if (threadIdx.x != 0) return;
  double sum = 0.0, sq = 0.0;
  for (int s = 0; s < nsplit; ++s) {
    const long long n_s = (s + 1) * chunk < N ? chunk : N - s * chunk;
    const double v = exp(kl_sum[s] / static_cast<double>(n_s));
    sum += v;
    sq += v * v;
  }
  const double mean = sum / nsplit;
  const double var = nsplit > 1 ? (sq - nsplit * mean * mean) / (nsplit - 1) : NAN;
  out[0] = static_cast<float>(mean);
  out[1] = static_cast<float>(var > 0.0 ? sqrt(var) : (var == var ? 0.0 : NAN));
}

}  // namespace

// logits: [N, C] (f32/f16/bf16/f64), perm: int64 [N] on the device, splits as torch.chunk; out: f32 [2] (mean, std).
void inception_score(const at::Tensor& logits, const at::Tensor& perm, int64_t splits, at::Tensor out) {
  TM_CHECK_CUDA(logits);
  TM_SAME_DEVICE(logits, perm);
  TM_SAME_DEVICE(logits, out);
  TM_CHECK_CONTIG(logits);
  TM_CHECK_CONTIG(perm);
  TORCH_CHECK(logits.dim() == 2 && perm.scalar_type() == at::kLong && perm.numel() == logits.size(0),
              "inception_score: logits [N, C] and an int64 [N] permutation");
  TORCH_CHECK(out.scalar_type() == at::kFloat && out.numel() == 2, "inception_score: out f32 [2]");
  const long long N = logits.size(0);
  const int C = static_cast<int>(logits.size(1));
  TORCH_CHECK(N >= 1 && C >= 1 && splits >= 1, "inception_score: empty input");
  const long long chunk = (N + splits - 1) / splits;
  const int nsplit = static_cast<int>((N + chunk - 1) / chunk);
  auto dopt = logits.options().dtype(at::kDouble);
  at::Tensor colsum = at::zeros({nsplit, C}, dopt);
  at::Tensor kl = at::zeros({nsplit}, dopt);
  at::Tensor lse = at::empty({N}, logits.options().dtype(at::kFloat));
  const int grid = grid_cap((N + (kBlock / kWave) - 1) / (kBlock / kWave), 256 * 8);
  TM_DISPATCH_FLOAT(logits.scalar_type(), "inception_score", [&] {
    const scalar_t* x = reinterpret_cast<const scalar_t*>(logits.data_ptr());
    hipLaunchKernelGGL((is_colsum_kernel<scalar_t>), dim3(grid), dim3(kBlock), 0, stream(), x,
                       perm.data_ptr<int64_t>(), N, C, chunk, lse.data_ptr<float>(), colsum.data_ptr<double>());
    hipLaunchKernelGGL((is_kl_kernel<scalar_t>), dim3(grid), dim3(kBlock), 0, stream(), x, perm.data_ptr<int64_t>(),
                       N, C, chunk, lse.data_ptr<float>(), colsum.data_ptr<double>(), kl.data_ptr<double>());
  });
  hipLaunchKernelGGL(is_finalize_kernel, dim3(1), dim3(64), 0, stream(), kl.data_ptr<double>(), N, chunk, nsplit,
                     out.data_ptr<float>());
  C10_HIP_KERNEL_LAUNCH_CHECK();
}

TORCH_LIBRARY_FRAGMENT(tm_amd, m) {
  m.def("inception_score(Tensor logits, Tensor perm, int splits, Tensor(a!) out) -> ()");
}
TORCH_LIBRARY_IMPL(tm_amd, CUDA, m) { m.impl("inception_score", &inception_score); }

}  // namespace tm_amd
