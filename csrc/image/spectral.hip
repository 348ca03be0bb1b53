// Spectral image metrics: SAM and ERGAS in one pass over the images each.
//
// sam_angles -- reference F/image/sam.py:56-83: `(preds * target).sum(1)`, two `norm(dim=1)`, divide, clamp, acos,
// then a reduction: five full-size temporaries and six launches.  Here one thread per pixel walks the C channels
// (stride H*W, so a wave's loads of one channel are 64 consecutive pixels: coalesced), accumulates the dot product and
// both squared norms in registers, writes the angle (reduction 'none') and/or folds it into an fp64 per-block partial
// (reductions 'sum' / 'elementwise_mean'; the partials are summed in a fixed order on the host side of the op).
// The clamp keeps NaN (zero vectors give 0/0 -> NaN, like the reference).
//
// band_stats -- reference F/image/ergas.py:57-71: per (image, band) RMSE over the pixels and the band's mean target,
// via a [B, C, H*W] difference tensor and three reductions.  Here per row (image, band) the sums sum (p - t)^2 and
// sum t in fp64, with several blocks per row for large bands (fp64 partials, folded by the caller's sum).
#include <type_traits>

#include "../common/tm_common.h"

namespace tm_amd {
namespace {

constexpr int kThreads = 256;

template <typename T>
__device__ __forceinline__ float to_acc(T v) {
  return to_f32(v);
}
__device__ __forceinline__ double to_acc(double v) { return v; }

template <typename T>
__device__ __forceinline__ T from_acc(double v) {
  return static_cast<T>(static_cast<float>(v));
}
template <>
__device__ __forceinline__ double from_acc<double>(double v) {
  return v;
}

template <typename T>
__global__ void __launch_bounds__(kThreads) sam_kernel(const T* __restrict__ p, const T* __restrict__ t, long long npix,
                                                       int C, long long hw, T* __restrict__ angle_map,
                                                       double* __restrict__ part) {
  using acc_t = typename std::conditional<std::is_same<T, double>::value, double, float>::type;
  double local = 0.0;
  const long long stride = static_cast<long long>(gridDim.x) * kThreads;
  for (long long i = static_cast<long long>(blockIdx.x) * kThreads + threadIdx.x; i < npix; i += stride) {
    const long long b = i / hw, s = i - b * hw;
    const long long base = b * C * hw + s;
    acc_t dot = 0, pp = 0, tt = 0;
    for (int c = 0; c < C; ++c) {
      const acc_t x = to_acc(p[base + c * hw]), y = to_acc(t[base + c * hw]);
      dot += x * y;
      pp += x * x;
      tt += y * y;
    }
    acc_t cosv = dot / (sqrt(pp) * sqrt(tt));
    cosv = cosv < acc_t(-1) ? acc_t(-1) : (cosv > acc_t(1) ? acc_t(1) : cosv);  // NaN stays NaN
    const acc_t a = acos(cosv);
    if (angle_map != nullptr) angle_map[i] = from_acc<T>(static_cast<double>(a));
    local += static_cast<double>(a);
  }
  if (part == nullptr) return;
  __shared__ double red[kThreads / 64];
  local = wave_sum(local);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = local;
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = 0.0;
    for (int w = 0; w < kThreads / 64; ++w) s += red[w];
    part[blockIdx.x] = s;
  }
}

template <typename T>
__global__ void __launch_bounds__(kThreads) band_stats_kernel(const T* __restrict__ p, const T* __restrict__ t,
                                                              long long len, int bpr, double* __restrict__ part) {
  const int row = blockIdx.x / bpr, sub = blockIdx.x % bpr;
  const T* pr = p + static_cast<long long>(row) * len;
  const T* tr = t + static_cast<long long>(row) * len;
  double sse = 0.0, st = 0.0;
  for (long long j = static_cast<long long>(sub) * kThreads + threadIdx.x; j < len;
       j += static_cast<long long>(bpr) * kThreads) {
    const double x = static_cast<double>(to_acc(pr[j])), y = static_cast<double>(to_acc(tr[j]));
    sse += (x - y) * (x - y);
    st += y;
  }
  __shared__ double red[2][kThreads / 64];
  sse = wave_sum(sse);
  st = wave_sum(st);
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = sse;
    red[1][threadIdx.x >> 6] = st;
  }
  __syncthreads();
  if (threadIdx.x < 2) {
    double s = 0.0;
    for (int w = 0; w < kThreads / 64; ++w) s += red[threadIdx.x][w];
    part[(static_cast<long long>(row) * bpr + sub) * 2 + threadIdx.x] = s;
  }
}

}  // namespace

// preds / target [B, C, H, W] contiguous, same dtype.  angle_map: [B, H, W] of the input dtype or empty; part: fp64
// [blocks] (blocks = part.numel(), >= 1) or empty.  At least one of them must be given.
void sam_angles(const at::Tensor& preds, const at::Tensor& target, at::Tensor angle_map, at::Tensor part) {
  TM_CHECK_CUDA(preds);
  TM_SAME_DEVICE(preds, target);
  TM_CHECK_CONTIG(preds);
  TM_CHECK_CONTIG(target);
  TORCH_CHECK(preds.dim() == 4 && preds.sizes() == target.sizes() && preds.scalar_type() == target.scalar_type(),
              "sam_angles: preds / target must be [B, C, H, W] of one dtype");
  const long long B = preds.size(0), C = preds.size(1), hw = preds.size(2) * preds.size(3);
  const long long npix = B * hw;
  const bool want_map = angle_map.numel() > 0, want_sum = part.numel() > 0;
  TORCH_CHECK(want_map || want_sum, "sam_angles: nothing to write");
  if (want_map) {
    TM_SAME_DEVICE(preds, angle_map);
    TORCH_CHECK(angle_map.is_contiguous() && angle_map.numel() == npix && angle_map.scalar_type() == preds.scalar_type(),
                "sam_angles: angle_map must be [B, H, W] of the input dtype");
  }
  if (want_sum) {
    TM_SAME_DEVICE(preds, part);
    TORCH_CHECK(part.is_contiguous() && part.scalar_type() == at::kDouble, "sam_angles: part must be fp64");
  }
  TORCH_CHECK(C >= 1 && C < (1LL << 31), "sam_angles: channel count");
  const long long need = (npix + kThreads - 1) / kThreads;
  const int blocks = want_sum ? static_cast<int>(part.numel())
                              : static_cast<int>(std::max<long long>(1, std::min<long long>(need, 8192)));
  if (want_sum) part.zero_();
  if (npix == 0) return;
  TM_DISPATCH_FLOAT(preds.scalar_type(), "sam_angles", [&] {
    hipLaunchKernelGGL((sam_kernel<scalar_t>), dim3(blocks), dim3(kThreads), 0, stream(), preds.data_ptr<scalar_t>(),
                       target.data_ptr<scalar_t>(), npix, static_cast<int>(C), hw,
                       want_map ? angle_map.data_ptr<scalar_t>() : nullptr,
                       want_sum ? part.data_ptr<double>() : nullptr);
  });
  C10_HIP_KERNEL_LAUNCH_CHECK();
}

// preds / target [R, L] contiguous (R = images * bands), same dtype -> part fp64 [R, bpr, 2] (sum (p - t)^2, sum t)
void band_stats(const at::Tensor& preds, const at::Tensor& target, at::Tensor part) {
  TM_CHECK_CUDA(preds);
  TM_SAME_DEVICE(preds, target);
  TM_SAME_DEVICE(preds, part);
  TM_CHECK_CONTIG(preds);
  TM_CHECK_CONTIG(target);
  TORCH_CHECK(preds.dim() == 2 && preds.sizes() == target.sizes() && preds.scalar_type() == target.scalar_type(),
              "band_stats: preds / target must be [rows, len] of one dtype");
  TORCH_CHECK(part.dim() == 3 && part.size(0) == preds.size(0) && part.size(2) == 2 && part.is_contiguous() &&
                  part.scalar_type() == at::kDouble && part.size(1) >= 1,
              "band_stats: part must be fp64 [rows, blocks_per_row, 2]");
  const long long R = preds.size(0), L = preds.size(1);
  const int bpr = static_cast<int>(part.size(1));
  TORCH_CHECK(R * bpr < (1LL << 31), "band_stats: too many blocks");
  if (R == 0) return;
  TM_DISPATCH_FLOAT(preds.scalar_type(), "band_stats", [&] {
    hipLaunchKernelGGL((band_stats_kernel<scalar_t>), dim3(static_cast<unsigned>(R * bpr)), dim3(kThreads), 0, stream(),
                       preds.data_ptr<scalar_t>(), target.data_ptr<scalar_t>(), L, bpr, part.data_ptr<double>());
  });
  C10_HIP_KERNEL_LAUNCH_CHECK();
}

TORCH_LIBRARY_FRAGMENT(tm_amd, m) {
  m.def("sam_angles(Tensor preds, Tensor target, Tensor(a!) angle_map, Tensor(b!) part) -> ()");
  m.def("band_stats(Tensor preds, Tensor target, Tensor(a!) part) -> ()");
}
TORCH_LIBRARY_IMPL(tm_amd, CUDA, m) {
  m.impl("sam_angles", &sam_angles);
  m.impl("band_stats", &band_stats);
}

}  // namespace tm_amd
