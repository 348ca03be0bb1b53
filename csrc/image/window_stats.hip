// Box-window and neighbour-difference image statistics: RMSE-SW, RASE, PSNR-B, total variation.
//
// box_rmse_maps -- reference F/image/rmse_sw.py + helper.py:112-132: per channel a Python loop of conv2d over the
// edge-mirrored ("symmetric") padded (target - preds)^2, sqrt, then a sum over the batch; RASE additionally filters
// the target.  Here ONE launch: a block owns a 16 x 64 output tile of one channel, stages the haloed tile of
// (t - p)^2 (and t) for each image of the batch in LDS with the reference's padding rule (w/2 mirrored rows/cols
// before, w/2 + w%2 - 1 after, edge included), runs the separable box sums (horizontal pass to LDS, vertical pass in
// registers), and accumulates sqrt(mean) over the batch in registers -- so the batch-summed maps are written once,
// with no atomics (deterministic), no padded copies and no per-channel launches.
//
// neighbour_diff_stats -- reference F/image/psnrb.py:21-100 (`_compute_bef`: index lists of block boundaries, four
// masked sums) and F/image/tv.py:20 (two shifted-difference reductions): one pass over the pixels; per image b
//   [0] sum (x - y)^2              (PSNR-B's SSE, when y is given)
//   [1] sum d_h over block-boundary columns      [2] sum d_h elsewhere
//   [3] sum d_v over block-boundary rows         [4] sum d_v elsewhere
// with d = squared (PSNR-B) or absolute (TV) neighbour differences.  fp64 per-block partials, reduced in a fixed
// order by a second tiny kernel (bitwise reproducible).
#include <type_traits>

#include "../common/tm_common.h"

namespace tm_amd {
namespace {

constexpr int kTH = 16, kTW = 64, kThreads = 256, kMaxWin = 32;

template <typename T>
__device__ __forceinline__ float to_acc(T v) {
  return to_f32(v);
}
__device__ __forceinline__ double to_acc(double v) { return v; }

__device__ __forceinline__ int mirror(int i, int n) {
  // edge-inclusive mirror: -1 -> 0, -2 -> 1, n -> n-1, n+1 -> n-2 (the reference's padding; its windows are shorter
  // than the image).  Halo rows / cols staged for output positions past the image edge (the last tile) can lie
  // further out: those feed no output, and the clamp keeps every load in bounds.
  if (i < 0) i = -i - 1;
  if (i >= n) i = 2 * n - i - 1;
  return i < 0 ? 0 : (i >= n ? n - 1 : i);
}

template <typename T>
__global__ void __launch_bounds__(kThreads) box_rmse_kernel(const T* __restrict__ p, const T* __restrict__ t, int B,
                                                            int C, int H, int W, int win, bool want_t,
                                                            T* __restrict__ rmse_map, T* __restrict__ t_map) {
  using acc_t = typename std::conditional<std::is_same<T, double>::value, double, float>::type;
  constexpr int kMaxRows = kTH + kMaxWin - 1, kMaxCols = kTW + kMaxWin - 1;
  __shared__ acc_t sd[kMaxRows][kMaxCols + 1];   // (t - p)^2 tile with halo
  __shared__ acc_t st[kMaxRows][kMaxCols + 1];   // t tile with halo (RASE)
  __shared__ acc_t hd[kMaxRows][kTW + 1];        // horizontal window sums
  __shared__ acc_t ht[kMaxRows][kTW + 1];
  const int tiles_w = (W + kTW - 1) / kTW;
  const int tile = blockIdx.x % (tiles_w * ((H + kTH - 1) / kTH));
  const int c = blockIdx.x / (tiles_w * ((H + kTH - 1) / kTH));
  const int i0 = (tile / tiles_w) * kTH, j0 = (tile % tiles_w) * kTW;
  const int before = win / 2;
  const int rows = kTH + win - 1, cols = kTW + win - 1;
  const acc_t inv = acc_t(1) / (acc_t(win) * acc_t(win));
  // per-thread outputs: thread -> (row r = tid / 16, cols q*16 + tid%16 for q < 4)
  const int orow = threadIdx.x / 16, ocol = threadIdx.x % 16;
  acc_t accd[4] = {0, 0, 0, 0}, acct[4] = {0, 0, 0, 0};
  for (int b = 0; b < B; ++b) {
    const long long plane = (static_cast<long long>(b) * C + c) * H * W;
    for (int e = threadIdx.x; e < rows * cols; e += kThreads) {
      const int r = e / cols, q = e % cols;
      const int gi = mirror(i0 + r - before, H), gj = mirror(j0 + q - before, W);
      const long long off = plane + static_cast<long long>(gi) * W + gj;
      const acc_t tv = static_cast<acc_t>(to_acc(t[off])), d = tv - static_cast<acc_t>(to_acc(p[off]));
      sd[r][q] = d * d;
      if (want_t) st[r][q] = tv;
    }
    __syncthreads();
    for (int e = threadIdx.x; e < rows * kTW; e += kThreads) {
      const int r = e / kTW, q = e % kTW;
      acc_t s0 = 0, s1 = 0;
      for (int k = 0; k < win; ++k) {
        s0 += sd[r][q + k];
        if (want_t) s1 += st[r][q + k];
      }
      hd[r][q] = s0;
      if (want_t) ht[r][q] = s1;
    }
    __syncthreads();
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) {
      const int q = qq * 16 + ocol;
      acc_t s0 = 0, s1 = 0;
      for (int k = 0; k < win; ++k) {
        s0 += hd[orow + k][q];
        if (want_t) s1 += ht[orow + k][q];
      }
      accd[qq] += sqrt(s0 * inv);
      if (want_t) acct[qq] += s1 * inv * inv;  // reference: uniform_filter(t) / w^2 (the filter already averages)
    }
    __syncthreads();  // the tiles are restaged for the next image
  }
  const int gi = i0 + orow;
  if (gi < H) {
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) {
      const int gj = j0 + qq * 16 + ocol;
      if (gj < W) {
        const long long off = (static_cast<long long>(c) * H + gi) * W + gj;
        rmse_map[off] = static_cast<T>(accd[qq]);
        if (want_t) t_map[off] = static_cast<T>(acct[qq]);
      }
    }
  }
}

template <typename T>
__global__ void __launch_bounds__(kThreads) neighbour_diff_kernel(const T* __restrict__ x, const T* __restrict__ y,
                                                                  int B, int C, int H, int W, int bs, bool squared,
                                                                  int blocks_per_image, double* __restrict__ part) {
  const int b = blockIdx.x / blocks_per_image, sub = blockIdx.x % blocks_per_image;
  const long long plane = static_cast<long long>(C) * H * W;
  const T* xb = x + b * plane;
  const T* yb = y != nullptr ? y + b * plane : nullptr;
  double s[5] = {0, 0, 0, 0, 0};
  for (long long e = static_cast<long long>(sub) * kThreads + threadIdx.x; e < plane;
       e += static_cast<long long>(blocks_per_image) * kThreads) {
    const int j = static_cast<int>(e % W);
    const int i = static_cast<int>((e / W) % H);
    const double v = static_cast<double>(to_acc(xb[e]));
    if (yb != nullptr) {
      const double d = v - static_cast<double>(to_acc(yb[e]));
      s[0] += d * d;
    }
    if (j + 1 < W) {
      const double d = static_cast<double>(to_acc(xb[e + 1])) - v;
      const double m = squared ? d * d : fabs(d);
      if (j % bs == bs - 1) s[1] += m;
      else s[2] += m;
    }
    if (i + 1 < H) {
      const double d = static_cast<double>(to_acc(xb[e + W])) - v;
      const double m = squared ? d * d : fabs(d);
      if (i % bs == bs - 1) s[3] += m;
      else s[4] += m;
    }
  }
  __shared__ double red[kThreads / kWave][5];
#pragma unroll
  for (int k = 0; k < 5; ++k) {
#pragma unroll
    for (int off = kWave / 2; off > 0; off >>= 1) s[k] += __shfl_xor(s[k], off, kWave);
  }
  if ((threadIdx.x & (kWave - 1)) == 0) {
#pragma unroll
    for (int k = 0; k < 5; ++k) red[threadIdx.x / kWave][k] = s[k];
  }
  __syncthreads();
  if (threadIdx.x < 5) {
    double v = 0;
    for (int w = 0; w < kThreads / kWave; ++w) v += red[w][threadIdx.x];
    part[static_cast<long long>(blockIdx.x) * 5 + threadIdx.x] = v;
  }
}

__global__ void neighbour_diff_final_kernel(const double* __restrict__ part, int B, int blocks_per_image,
                                            double* __restrict__ out) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= B * 5) return;
  const int b = e / 5, k = e % 5;
  double v = 0;
  for (int s = 0; s < blocks_per_image; ++s) v += part[(static_cast<long long>(b) * blocks_per_image + s) * 5 + k];
  out[e] = v;
}

}  // namespace

// rmse_map / t_map: [C, H, W] in the input dtype (t_map may be empty); returns nothing.
void box_rmse_maps(const at::Tensor& preds, const at::Tensor& target, int64_t window, at::Tensor rmse_map,
                   at::Tensor t_map) {
  TM_CHECK_CUDA(preds);
  TM_SAME_DEVICE(preds, target);
  TM_SAME_DEVICE(preds, rmse_map);
  TM_CHECK_CONTIG(preds);
  TM_CHECK_CONTIG(target);
  TORCH_CHECK(preds.dim() == 4 && preds.sizes() == target.sizes(), "box_rmse_maps: preds / target must be [B,C,H,W]");
  const int B = preds.size(0), C = preds.size(1), H = preds.size(2), W = preds.size(3);
  TORCH_CHECK(window >= 1 && window <= kMaxWin && window <= H && window <= W, "box_rmse_maps: window out of range");
  TORCH_CHECK(rmse_map.is_contiguous() && rmse_map.numel() == static_cast<long long>(C) * H * W &&
                  rmse_map.scalar_type() == preds.scalar_type(),
              "box_rmse_maps: rmse_map must be [C, H, W] of the input dtype");
  const bool want_t = t_map.numel() > 0;
  if (want_t) {
    TM_SAME_DEVICE(preds, t_map);
    TORCH_CHECK(t_map.is_contiguous() && t_map.numel() == rmse_map.numel() &&
                    t_map.scalar_type() == preds.scalar_type(),
                "box_rmse_maps: t_map must be [C, H, W] of the input dtype");
  }
  if (B == 0) return;
  const int tiles = ((H + kTH - 1) / kTH) * ((W + kTW - 1) / kTW) * C;
  TM_DISPATCH_FLOAT(preds.scalar_type(), "box_rmse_maps", [&] {
    hipLaunchKernelGGL((box_rmse_kernel<scalar_t>), dim3(tiles), dim3(kThreads), 0, stream(),
                       preds.data_ptr<scalar_t>(), target.data_ptr<scalar_t>(), B, C, H, W, static_cast<int>(window),
                       want_t, rmse_map.data_ptr<scalar_t>(), want_t ? t_map.data_ptr<scalar_t>() : nullptr);
  });
  C10_HIP_KERNEL_LAUNCH_CHECK();
}

// out: f64 [B, 5] (see the header); y may be empty.
void neighbour_diff_stats(const at::Tensor& x, const at::Tensor& y, int64_t block_size, bool squared, at::Tensor out) {
  TM_CHECK_CUDA(x);
  TM_CHECK_CONTIG(x);
  TORCH_CHECK(x.dim() == 4, "neighbour_diff_stats: x must be [B, C, H, W]");
  const bool has_y = y.numel() > 0;
  if (has_y) {
    TM_SAME_DEVICE(x, y);
    TM_CHECK_CONTIG(y);
    TORCH_CHECK(y.sizes() == x.sizes() && y.scalar_type() == x.scalar_type(), "neighbour_diff_stats: y mismatch");
  }
  const int B = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  TORCH_CHECK(out.scalar_type() == at::kDouble && out.is_contiguous() && out.numel() == 5LL * B,
              "neighbour_diff_stats: out must be f64 [B, 5]");
  TORCH_CHECK(block_size >= 1, "neighbour_diff_stats: block_size must be positive");
  if (B == 0) return;
  const long long plane = static_cast<long long>(C) * H * W;
  const int bpi = static_cast<int>(std::max<long long>(1, std::min<long long>(64, plane / (kThreads * 16))));
  at::Tensor part = at::empty({static_cast<long long>(B) * bpi * 5}, out.options());
  TM_DISPATCH_FLOAT(x.scalar_type(), "neighbour_diff_stats", [&] {
    hipLaunchKernelGGL((neighbour_diff_kernel<scalar_t>), dim3(B * bpi), dim3(kThreads), 0, stream(),
                       x.data_ptr<scalar_t>(), has_y ? y.data_ptr<scalar_t>() : nullptr, B, C, H, W,
                       static_cast<int>(block_size), squared, bpi, part.data_ptr<double>());
  });
  hipLaunchKernelGGL(neighbour_diff_final_kernel, dim3((B * 5 + 255) / 256), dim3(256), 0, stream(),
                     part.data_ptr<double>(), B, bpi, out.data_ptr<double>());
  C10_HIP_KERNEL_LAUNCH_CHECK();
}

TORCH_LIBRARY_FRAGMENT(tm_amd, m) {
  m.def("box_rmse_maps(Tensor preds, Tensor target, int window, Tensor(a!) rmse_map, Tensor(b!) t_map) -> ()");
  m.def("neighbour_diff_stats(Tensor x, Tensor y, int block_size, bool squared, Tensor(a!) out) -> ()");
}
TORCH_LIBRARY_IMPL(tm_amd, CUDA, m) {
  m.impl("box_rmse_maps", &box_rmse_maps);
  m.impl("neighbour_diff_stats", &neighbour_diff_stats);
}

}  // namespace tm_amd
