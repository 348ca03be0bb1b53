// Fused SSIM / contrast-sensitivity kernel (2-D, Gaussian or uniform window); also UQI, SCC and one VIF scale.
//
// Reference (F/image/ssim.py:45-186) reflect-pads both images, stacks 5 maps (x, y, x*x, y*y, x*y) into a 5B-batch,
// runs a grouped 11x11 conv2d, then forms the SSIM map and crops the padded border before the per-image mean.  The
// crop keeps exactly the windows that lie fully inside the image, so the padding never reaches the result.  This
// kernel therefore evaluates only those valid windows, straight from the unpadded images:
//
//   block = 16 x 64 output tile of one (image, channel) plane, 256 threads (4 wave64)
//   1. stage the (16+kh-1) x (64+kw-1) input tile of x and y in LDS (fp32)
//   2. horizontal separable pass: 5 running moments per (row, out-col) -> LDS
//   3. vertical pass per output pixel -> mu_x, mu_y, E[x^2], E[y^2], E[xy] -> SSIM and CS
//   4. block reduction of sum(SSIM), sum(CS) -> one partial per block (fixed order, deterministic)
//
// One read of each input pixel, no 5x stacked temporaries, no padded copies, one launch.  c1/c2 come from a device
// tensor, so the data_range=None path (max - min of the batch) never synchronises with the host.
#include "../common/tm_common.h"

namespace tm_amd {
namespace {

constexpr int kTH = 16;       // output rows per block
constexpr int kTW = 64;       // output cols per block (one wave across)
constexpr int kMaxK = 33;     // largest window edge supported by the fused path
constexpr int kThreads = 256;

template <typename T>
struct Acc {
  using type = float;
};
template <>
struct Acc<double> {
  using type = double;
};

template <typename scalar_t>
__global__ void __launch_bounds__(kThreads) ssim2d_kernel(const scalar_t* __restrict__ x,
                                                          const scalar_t* __restrict__ y, int H, int W, int kh,
                                                          int kw, const typename Acc<scalar_t>::type* __restrict__ wh,
                                                          const typename Acc<scalar_t>::type* __restrict__ ww,
                                                          const typename Acc<scalar_t>::type* __restrict__ c12,
                                                          int tiles_w, int mode,
                                                          typename Acc<scalar_t>::type* __restrict__ part) {
  using acc_t = typename Acc<scalar_t>::type;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int in_h = kTH + kh - 1, in_w = kTW + kw - 1;
  acc_t* sx = reinterpret_cast<acc_t*>(smem);
  acc_t* sy = sx + in_h * in_w;
  acc_t* hm = sy + in_h * in_w;  // 5 x [in_h][kTW]
  __shared__ acc_t swh[kMaxK], sww[kMaxK];
  __shared__ acc_t red[2][kThreads / kWave];

  const long long plane = blockIdx.y;
  const int tile = blockIdx.x;
  const int r0 = (tile / tiles_w) * kTH, c0 = (tile % tiles_w) * kTW;
  const scalar_t* px = x + plane * H * W;
  const scalar_t* py = y + plane * H * W;
  const int tid = threadIdx.x;
  if (tid < kh) swh[tid] = wh[tid];
  if (tid < kw) sww[tid] = ww[tid];
  for (int i = tid; i < in_h * in_w; i += kThreads) {
    const int r = i / in_w, c = i % in_w;
    const int gr = r0 + r, gc = c0 + c;
    const bool ok = gr < H && gc < W;
    sx[i] = ok ? static_cast<acc_t>(to_f32(px[static_cast<long long>(gr) * W + gc])) : acc_t(0);
    sy[i] = ok ? static_cast<acc_t>(to_f32(py[static_cast<long long>(gr) * W + gc])) : acc_t(0);
  }
  __syncthreads();
  const int plane_sz = in_h * kTW;
  for (int i = tid; i < plane_sz; i += kThreads) {
    const int r = i / kTW, c = i % kTW;
    const acc_t* rx = sx + r * in_w + c;
    const acc_t* ry = sy + r * in_w + c;
    acc_t m1 = 0, m2 = 0, m3 = 0, m4 = 0, m5 = 0;
    for (int j = 0; j < kw; ++j) {
      const acc_t w = sww[j], a = rx[j], b = ry[j];
      m1 += w * a;
      m2 += w * b;
      m3 += w * a * a;
      m4 += w * b * b;
      m5 += w * a * b;
    }
    hm[i] = m1;
    hm[plane_sz + i] = m2;
    hm[2 * plane_sz + i] = m3;
    hm[3 * plane_sz + i] = m4;
    hm[4 * plane_sz + i] = m5;
  }
  __syncthreads();
  const acc_t c1 = c12[0], c2 = c12[1], eps = c12[2];
  const int out_h = H - kh + 1, out_w = W - kw + 1;
  acc_t s_ssim = 0, s_cs = 0;
  for (int i = tid; i < kTH * kTW; i += kThreads) {
    const int r = i / kTW, c = i % kTW;
    if (r0 + r >= out_h || c0 + c >= out_w) continue;
    acc_t mx = 0, my = 0, exx = 0, eyy = 0, exy = 0;
    for (int k = 0; k < kh; ++k) {
      const int o = (r + k) * kTW + c;
      const acc_t w = swh[k];
      mx += w * hm[o];
      my += w * hm[plane_sz + o];
      exx += w * hm[2 * plane_sz + o];
      eyy += w * hm[3 * plane_sz + o];
      exy += w * hm[4 * plane_sz + o];
    }
    const acc_t mxx = mx * mx, myy = my * my, mxy = mx * my;
    const acc_t sxx = exx - mxx > 0 ? exx - mxx : acc_t(0);
    const acc_t syy = eyy - myy > 0 ? eyy - myy : acc_t(0);
    const acc_t sxy = exy - mxy;
    if (mode == 0) {  // SSIM (+ contrast sensitivity)
      const acc_t upper = 2 * sxy + c2;
      const acc_t lower = sxx + syy + c2;
      s_ssim += ((2 * mxy + c1) * upper) / ((mxx + myy + c1) * lower);
      s_cs += upper / lower;
    } else if (mode == 1) {  // universal image quality index (F/image/uqi.py): no stabilisers, eps in the denominator
      const acc_t upper = 2 * sxy;
      const acc_t lower = sxx + syy;
      s_ssim += ((2 * mxy) * upper) / ((mxx + myy) * lower + eps);
    } else if (mode == 3) {  // spatial correlation coefficient (F/image/scc.py): cov / (sd_x sd_y), 0 where undefined
      const acc_t den = sqrt(sxx) * sqrt(syy);
      s_ssim += den == acc_t(0) ? acc_t(0) : sxy / den;
    } else {  // VIF at one scale (F/image/vif.py): x = reference, y = distorted; c1 = sigma_n^2, eps = 1e-10
      acc_t stt = sxx, g = sxy / (sxx + eps), sv = syy - g * sxy;
      if (stt < eps) {
        g = 0;
        sv = syy;
        stt = 0;
      }
      if (syy < eps) {
        g = 0;
        sv = 0;
      }
      if (g < 0) {
        sv = syy;
        g = 0;
      }
      sv = sv > eps ? sv : eps;
      s_ssim += log10(acc_t(1) + g * g * stt / (sv + c1));
      s_cs += log10(acc_t(1) + stt / c1);
    }
  }
  s_ssim = wave_sum(s_ssim);
  s_cs = wave_sum(s_cs);
  const int wave = tid / kWave;
  if ((tid & (kWave - 1)) == 0) {
    red[0][wave] = s_ssim;
    red[1][wave] = s_cs;
  }
  __syncthreads();
  if (tid == 0) {
    acc_t a = 0, b = 0;
    for (int w = 0; w < kThreads / kWave; ++w) {
      a += red[0][w];
      b += red[1][w];
    }
    const long long slot = plane * gridDim.x + tile;
    part[slot * 2] = a;
    part[slot * 2 + 1] = b;
  }
}

}  // namespace

// x, y: [P, H, W] planes (contiguous, same dtype); wh [kh], ww [kw] window weights; c12 [3] (c1, c2, eps) in the
// accumulation dtype (f32, or f64 for f64 inputs); mode 0 = SSIM, 1 = UQI, 2 = VIF (x reference, y distorted;
// c12 = (sigma_n^2, -, eps)), 3 = SCC (x, y high-passed, uniform window;
// c12 unused).  Returns part [P, tiles, 2] of per-tile (sum SSIM|UQI|VIF numerator, sum CS|VIF
// denominator) over the valid windows.
at::Tensor ssim2d_partials(const at::Tensor& x, const at::Tensor& y, const at::Tensor& wh, const at::Tensor& ww,
                           const at::Tensor& c12, int64_t mode) {
  TM_CHECK_CUDA(x);
  TM_CHECK_CONTIG(x);
  TM_CHECK_CONTIG(y);
  TORCH_CHECK(x.sizes() == y.sizes() && x.scalar_type() == y.scalar_type(), "ssim2d: x / y mismatch");
  TORCH_CHECK(x.dim() == 3, "ssim2d: expects [planes, H, W]");
  const int kh = static_cast<int>(wh.numel()), kw = static_cast<int>(ww.numel());
  TORCH_CHECK(kh >= 1 && kw >= 1 && kh <= kMaxK && kw <= kMaxK, "ssim2d: window must be 1..", kMaxK);
  const long long planes = x.size(0);
  const int H = static_cast<int>(x.size(1)), W = static_cast<int>(x.size(2));
  TORCH_CHECK(H >= kh && W >= kw, "ssim2d: image smaller than the window");
  TORCH_CHECK(planes <= 65535, "ssim2d: too many planes for one launch");
  const bool dbl = x.scalar_type() == at::kDouble;
  const auto acc_type = dbl ? at::kDouble : at::kFloat;
  TORCH_CHECK(c12.numel() >= 3, "ssim2d: c12 must hold (c1, c2, eps)");
  TORCH_CHECK(wh.scalar_type() == acc_type && ww.scalar_type() == acc_type && c12.scalar_type() == acc_type,
              "ssim2d: window / constants must be in the accumulation dtype");
  const int out_h = H - kh + 1, out_w = W - kw + 1;
  const int tiles_w = (out_w + kTW - 1) / kTW, tiles_h = (out_h + kTH - 1) / kTH;
  const int tiles = tiles_w * tiles_h;
  at::Tensor part = at::empty({planes, tiles, 2}, x.options().dtype(acc_type));
  if (planes == 0) return part;
  const int in_h = kTH + kh - 1, in_w = kTW + kw - 1;
  const size_t esz = dbl ? sizeof(double) : sizeof(float);
  const size_t lds = esz * (2 * static_cast<size_t>(in_h) * in_w + 5 * static_cast<size_t>(in_h) * kTW);
  TORCH_CHECK(lds <= 150 * 1024, "ssim2d: window too large for the LDS tile (use a smaller kernel / fp32 inputs)");
  auto s = stream();
  TM_DISPATCH_FLOAT(x.scalar_type(), "ssim2d", [&] {
    using acc_t = typename Acc<scalar_t>::type;
    if (lds > 64 * 1024) {
      TORCH_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&ssim2d_kernel<scalar_t>),
                                      hipFuncAttributeMaxDynamicSharedMemorySize,
                                      static_cast<int>(lds)) == hipSuccess,
                  "ssim2d: could not raise the dynamic LDS limit");
    }
    hipLaunchKernelGGL((ssim2d_kernel<scalar_t>), dim3(tiles, static_cast<unsigned>(planes)), dim3(kThreads), lds, s,
                       reinterpret_cast<const scalar_t*>(x.data_ptr()), reinterpret_cast<const scalar_t*>(y.data_ptr()),
                       H, W, kh, kw, wh.data_ptr<acc_t>(), ww.data_ptr<acc_t>(), c12.data_ptr<acc_t>(), tiles_w,
                       static_cast<int>(mode), part.data_ptr<acc_t>());
  });
  C10_HIP_KERNEL_LAUNCH_CHECK();
  return part;
}

}  // namespace tm_amd

TORCH_LIBRARY_FRAGMENT(tm_amd, m) {
  m.def("ssim2d_partials(Tensor x, Tensor y, Tensor wh, Tensor ww, Tensor c12, int mode) -> Tensor");
}

TORCH_LIBRARY_IMPL(tm_amd, CUDA, m) { m.impl("ssim2d_partials", &tm_amd::ssim2d_partials); }
