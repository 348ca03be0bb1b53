// Fused LPIPS layer distance.
//
// For one backbone layer with features f0, f1 [N, C, P] (P = H*W) and linear weights w [C] the reference evaluates
//   mean_p sum_c w_c (f0 / (||f0||_c + eps) - f1 / (||f1||_c + eps))^2
// as normalise (2 reductions + 2 divides), subtract, square, 1x1 conv and spatial mean (F/image/lpips.py:215-366):
// ~6 full passes over the feature maps.  Here one thread owns one pixel and streams its C channels once (adjacent
// threads = adjacent pixels, so every channel step is a coalesced 1 KB row), accumulating the five moments
//   S_aa, S_bb, S_waa, S_wbb, S_wab   (fp64, so the expanded form has no cancellation trouble)
// and evaluates  S_waa / na^2 - 2 S_wab / (na nb) + S_wbb / nb^2  with na = sqrt(S_aa) + eps.  Each block reduces its
// 256 pixels and writes one partial per (image, block) -> deterministic host-side sum.
#include "common/tm_common.h"

namespace tm_amd {
namespace {

constexpr int kThreads = 256;

template <typename T>
__global__ void __launch_bounds__(kThreads) lpips_layer_kernel(const T* __restrict__ f0, const T* __restrict__ f1,
                                                               const float* __restrict__ w, int channels, int pixels,
                                                               double eps, double* __restrict__ partial) {
  const int n = blockIdx.y;
  const int p = blockIdx.x * kThreads + threadIdx.x;
  double val = 0.0;
  if (p < pixels) {
    const long long base = static_cast<long long>(n) * channels * pixels + p;
    double saa = 0.0, sbb = 0.0, swaa = 0.0, swbb = 0.0, swab = 0.0;
    for (int c = 0; c < channels; ++c) {
      const double a = to_f32<T>(f0[base + static_cast<long long>(c) * pixels]);
      const double b = to_f32<T>(f1[base + static_cast<long long>(c) * pixels]);
      const double wc = w[c];
      saa = fma(a, a, saa);
      sbb = fma(b, b, sbb);
      swaa = fma(wc * a, a, swaa);
      swbb = fma(wc * b, b, swbb);
      swab = fma(wc * a, b, swab);
    }
    const double na = sqrt(saa) + eps, nb = sqrt(sbb) + eps;
    val = swaa / (na * na) - 2.0 * swab / (na * nb) + swbb / (nb * nb);
  }
  val = wave_sum(val);
  __shared__ double red[kThreads / kWave];
  const int wave = threadIdx.x / kWave, lane = threadIdx.x & (kWave - 1);
  if (lane == 0) red[wave] = val;
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = 0.0;
    for (int i = 0; i < kThreads / kWave; ++i) s += red[i];
    partial[static_cast<long long>(n) * gridDim.x + blockIdx.x] = s;
  }
}

}  // namespace

// partial[n, b] = sum over the pixels of block b of the weighted normalised squared feature difference.
void lpips_layer(const at::Tensor& f0, const at::Tensor& f1, const at::Tensor& w, at::Tensor partial, double eps) {
  TM_CHECK_CUDA(f0);
  TM_CHECK_CONTIG(f0);
  TM_CHECK_CONTIG(f1);
  TM_CHECK_CONTIG(w);
  TM_CHECK_CONTIG(partial);
  TORCH_CHECK(f0.dim() == 3 && f0.sizes() == f1.sizes(), "lpips_layer: features must be [N, C, P] of equal shape");
  TORCH_CHECK(f0.scalar_type() == f1.scalar_type(), "lpips_layer: dtype mismatch");
  TORCH_CHECK(w.scalar_type() == at::kFloat && w.numel() == f0.size(1), "lpips_layer: weights must be fp32 [C]");
  const int n = static_cast<int>(f0.size(0)), c = static_cast<int>(f0.size(1)), p = static_cast<int>(f0.size(2));
  const int blocks = (p + kThreads - 1) / kThreads;
  TORCH_CHECK(partial.scalar_type() == at::kDouble && partial.numel() == static_cast<long long>(n) * blocks,
              "lpips_layer: partial must be fp64 [N, ceil(P / 256)]");
  if (n == 0 || p == 0) return;
  TM_DISPATCH_FLOAT(f0.scalar_type(), "lpips_layer", [&] {
    hipLaunchKernelGGL((lpips_layer_kernel<scalar_t>), dim3(blocks, n), dim3(kThreads), 0, stream(),
                       f0.data_ptr<scalar_t>(), f1.data_ptr<scalar_t>(), w.data_ptr<float>(), c, p, eps,
                       partial.data_ptr<double>());
  });
}

TORCH_LIBRARY_FRAGMENT(tm_amd, m) { m.def("lpips_layer(Tensor f0, Tensor f1, Tensor w, Tensor(a!) partial, float eps) -> ()"); }
TORCH_LIBRARY_IMPL(tm_amd, CUDA, m) { m.impl("lpips_layer", &lpips_layer); }

}  // namespace tm_amd
